set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_model.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/dp1.log 2>&1 || { tail -30 gpurun_out/dp1.log; exit 1; }
grep -E "passed|failed|rel-L2|segments" gpurun_out/dp1.log
