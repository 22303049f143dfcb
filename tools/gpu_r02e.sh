set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u tools/tower_ab.py 5 > gpurun_out/r02e_ab.log 2>&1; rc=$?; tail -8 gpurun_out/r02e_ab.log
[ $rc -ne 0 ] && exit $rc
(cd tools && timeout -k 10 200 python -u x_ablate.py 3 0,4,32,64,96,100) > gpurun_out/r02e_abl.log 2>&1; rc=$?; tail -7 gpurun_out/r02e_abl.log
[ $rc -ne 0 ] && exit $rc
NOBENCH=0 bash tools/gpu_tests.sh r02e tests/test_gpu_conv.py tests/test_gpu_conv_production.py tests/test_gpu_fullsize.py
