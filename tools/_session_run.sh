set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/distributed/test_custom_ar_gpu.py -k "2" > gpurun_out/t_car.log 2>&1 || { tail -40 gpurun_out/t_car.log; exit 1; }
tail -1 gpurun_out/t_car.log
for wld in 1 2; do
timeout -k 10 300 python -u tools/bench_car_norm.py $wld gemv > gpurun_out/car_gemv_w$wld.md 2> gpurun_out/car_gemv_w$wld.err
grep -v "^\[\|amdgpu.ids\|Gloo\|socket" gpurun_out/car_gemv_w$wld.md
done
