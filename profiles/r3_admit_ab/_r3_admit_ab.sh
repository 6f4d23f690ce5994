set -e
for v in 1 0 1; do
RFQ_BENCH_OVERLAP_ADMIT=$v timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/admit_$v.$RANDOM.json 2> gpurun_out/admit_$v.err
done
