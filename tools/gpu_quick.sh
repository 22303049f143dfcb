set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_nnops.py tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_hourglass.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s4d_pytest.log 2>&1 || { tail -30 gpurun_out/s4d_pytest.log; exit 1; }
tail -3 gpurun_out/s4d_pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/s4d_bench.json 2> gpurun_out/s4d_bench.err || { tail -30 gpurun_out/s4d_bench.err; exit 1; }
cat gpurun_out/s4d_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/s4d_prof -o prof -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/s4d_prof_bench.json 2> gpurun_out/s4d_prof.err || { tail -30 gpurun_out/s4d_prof.err; exit 1; }
cat gpurun_out/s4d_prof_bench.json
