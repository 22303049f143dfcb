set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u tools/tower_ab.py 5 > gpurun_out/r02g_ab.log 2>&1; rc=$?; tail -14 gpurun_out/r02g_ab.log
[ $rc -ne 0 ] && exit $rc
NOBENCH=0 bash tools/gpu_tests.sh r02g tests/test_gpu_conv.py tests/test_gpu_conv_production.py
