set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
A="--steps 8 --warmup 3 --latency-runs 0 --phases none"
val() { python -c "import json,sys;print(sys.argv[1], json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value'])" "$1"; }
for r in 1 2; do
  timeout -k 10 420 python -u bench.py $A > gpurun_out/ab_off_$r.json 2> gpurun_out/ab_off_$r.err
  val gpurun_out/ab_off_$r.json
  RFQ_SHARED_PREFIX_MIN_ROWS=64 timeout -k 10 420 python -u bench.py $A > gpurun_out/ab_on_$r.json 2> gpurun_out/ab_on_$r.err
  val gpurun_out/ab_on_$r.json
done
