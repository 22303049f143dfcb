set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_conv_production.py tests/test_gpu_nnops.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/p2_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/p2_pytest.log | head -30; exit $rc; fi
timeout -k 10 200 python3 tools/p_probe.py "" CVL_P_ABLATE=1 CVL_P_ABLATE=2 CVL_CONV_NO_P=1 CVL_CONV_P_BN=128 CVL_CONV_P_BN=256
