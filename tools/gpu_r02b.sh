set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u tools/tower_ab.py 5 > gpurun_out/r02b_ab.log 2>&1; rc=$?; cat gpurun_out/r02b_ab.log | tail -20
[ $rc -ne 0 ] && exit $rc
NOBENCH=0 bash tools/gpu_tests.sh r02b tests/test_gpu_conv.py tests/test_gpu_conv_production.py tests/test_gpu_fullsize.py tests/test_gpu_model.py
