#!/bin/bash
# GPU CI step used with gpurun: tests, then the 1-GPU bench.  Stops at the first
# crash-class exit (abort/segfault/timeout); plain test failures (rc=1) continue.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests crashed rc=$rc"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-900} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
brc=$?
tail -3 gpurun_out/bench.log
exit $brc
