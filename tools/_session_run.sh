set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
P=replisense_rfq_amd
cp $P/_C_hack.so $P/_C.so
echo hack; timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/attn_hack.log 2>&1; grep '^{' gpurun_out/attn_hack.log
cp $P/_C_orig.so $P/_C.so
echo orig; timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/attn_orig.log 2>&1; grep '^{' gpurun_out/attn_orig.log
