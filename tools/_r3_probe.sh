set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/probe_mall.py > gpurun_out/mall.json 2> gpurun_out/mall.err
timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/bench_host.json 2> gpurun_out/bench_host.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tput -o run -- python3 $R/bench.py --steps 4 --warmup 2 --latency-runs 0 --phases none > $R/gpurun_out/prof_tput.log 2>&1
cd $R
python3 tools/prof_gaps.py gpurun_out/prof_tput 6 > gpurun_out/tput_gaps.md
find gpurun_out/prof_tput -name '*_trace.csv' -delete
