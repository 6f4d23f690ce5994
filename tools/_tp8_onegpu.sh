# Llama-3-70B TP=8 end to end with 8 ranks sharing ONE MI355X (RCCL refuses two ranks
# on one device, so the group runs over gloo, eager).  Functional rehearsal of the
# 8-GPU node's TP phase (BASELINE config 4), not a performance number.  The custom
# all-reduce is off here: its kernels spin on peer flags, and with 8 eager processes
# time-sliced on one GPU a spinning rank starves the peers it waits for (a first
# attempt with it on completed no document in 730 s); on the node each rank owns a GPU.
set -e
export RFQ_DIST_BACKEND=gloo RFQ_TILED_WEIGHTS=0 RFQ_TUNE_GEMM=0 RFQ_CUSTOM_AR=0
start=$(date +%s)
timeout -k 20 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --model llama3-70b --tp 8 \
  --steps 1 --warmup 0 --docs-per-step 4 --max-num-seqs 8 --latency-runs 0 --no-graphs \
  --kv-fraction 0.02 --phases none --tp-latency-model none \
  > gpurun_out/tp8_onegpu.json 2> gpurun_out/tp8_onegpu.err
echo "wall_s=$(( $(date +%s) - start ))" > gpurun_out/tp8_onegpu.wall
