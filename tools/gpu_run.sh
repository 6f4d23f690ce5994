#!/bin/bash
# One entry point for the GPU-box runs of a session (replaces the one-off round-3
# wrappers).  Usage, on the box (gpurun -- 'bash tools/gpu_run.sh TASK [TASK ...]'):
#
#   tests        pytest -m gpu (one process, per-test timeout), then smoke()
#   kernels      tests/kernels only
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py $BENCH_ARGS            (default: the driver's flags)
#   tp8          tools/tp8_rank_emulation.py             (70B TP=8 rank 0 on one GPU)
#   tp8prof      rocprofv3 kernel window of the tp8 emulation -> gpurun_out/tp8_window.md
#   lat8b        latency-path kernel window of the 8B single stream
#   tput         kernel window of a short throughput bench
#   gemv         tools/bench_decode_gemv.py  (8B and TP=8 shard shapes)
#   rows         tools/bench_gemv_rows.py    (row-streaming GEMV vs the split-K / skinny GEMVs)
#   gemm         tools/bench_gemm_dense.py   (hand-written large-M GEMM vs hipBLASLt)
#   attn         tools/bench_attn.py         (decode attention)
#   prefill      tools/bench_prefill.py
#   car          tools/bench_car_norm.py     (custom all-reduce, 2 processes, one GPU)
#
# Every GPU step has its own time limit; the script stops at the first failing step
# (set -e) so nothing runs on a GPU after a fault, abort or timeout.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"

prof() {   # prof <out dir> <timeout s> <cmd...>: kernel trace + stats, trace csv removed
  local out=$1 t=$2; shift 2
  mkdir -p "$out"
  (cd /tmp && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$out" -o run -- "$@") > "$out.log" 2>&1
}

for task in "$@"; do
  echo "[gpu_run] $task $(date +%T)"
  case $task in
    tests)
      timeout -k 10 1200 $PYT tests -m gpu > gpurun_out/gpu_tests.log 2>&1
      tail -3 gpurun_out/gpu_tests.log
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/smoke.log 2>&1 ;;
    kernels)
      timeout -k 10 900 $PYT tests/kernels ${PYTEST_K:+-k "$PYTEST_K"} \
        > gpurun_out/kernel_tests.log 2>&1
      tail -3 gpurun_out/kernel_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-900} python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} \
        > gpurun_out/bench.json 2> gpurun_out/bench.err
      tail -c 600 gpurun_out/bench.json ;;
    tp8)
      timeout -k 10 400 python -u tools/tp8_rank_emulation.py ${TP8_ARGS:-} \
        --md gpurun_out/tp8_proj.md > gpurun_out/tp8.json 2> gpurun_out/tp8.err
      tail -c 400 gpurun_out/tp8.json ;;
    tp8prof)
      prof gpurun_out/prof_tp8 400 python3 "$R/tools/tp8_rank_emulation.py" --runs 3 \
        --decode-tokens 100
      python3 tools/trace_window_stats.py gpurun_out/prof_tp8 1.5 > gpurun_out/tp8_window.md
      find gpurun_out/prof_tp8 -name '*_trace.csv' -delete ;;
    lat8b)
      prof gpurun_out/prof_lat 400 python3 "$R/bench.py" --steps 1 --warmup 0 \
        --docs-per-step 1 --max-num-seqs 64 --latency-runs 8 --phases none
      python3 tools/prof_gaps.py gpurun_out/prof_lat 3 > gpurun_out/lat8b_window.md
      find gpurun_out/prof_lat -name '*_trace.csv' -delete ;;
    tput)
      prof gpurun_out/prof_tput 600 python3 "$R/bench.py" --steps 4 --warmup 2 \
        --latency-runs 0 --phases none
      python3 tools/trace_window_stats.py gpurun_out/prof_tput 6 > gpurun_out/tput_window.md
      find gpurun_out/prof_tput -name '*_trace.csv' -delete ;;
    gemv)
      timeout -k 10 400 python -u tools/bench_decode_gemv.py ${GEMV_ARGS:-} \
        > gpurun_out/gemv.jsonl 2> gpurun_out/gemv.err ;;
    gemm)
      timeout -k 10 600 python -u tools/bench_gemm_dense.py ${GEMM_ARGS:---ms 2048,4096,7168} \
        > gpurun_out/gemm.log 2>&1
      tail -20 gpurun_out/gemm.log ;;
    rows)
      timeout -k 10 400 python -u tools/bench_gemv_rows.py ${ROWS_ARGS:-} \
        > gpurun_out/gemv_rows.jsonl 2> gpurun_out/gemv_rows.err ;;
    attn)
      timeout -k 10 300 python -u tools/bench_attn.py ${ATTN_ARGS:-} > gpurun_out/attn.log 2>&1 ;;
    prefill)
      timeout -k 10 300 python -u tools/bench_prefill.py ${PREFILL_ARGS:-} \
        > gpurun_out/prefill.log 2>&1 ;;
    car)
      timeout -k 10 300 python -u tools/bench_car_norm.py ${CAR_ARGS:-} > gpurun_out/car.log 2>&1 ;;
    *)
      echo "unknown task $task" >&2; exit 2 ;;
  esac
done
