set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_production.py tests/test_gpu_model.py tests/test_gpu_fcos_step.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p1_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/p1_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/p1_pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/conv_table.py --out gpurun_out/p1_conv_table.md > gpurun_out/p1_conv_table.log 2>&1 || exit 1
grep "1x1\|Total" gpurun_out/p1_conv_table.md | head -40
