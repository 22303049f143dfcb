set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
(cd tools && timeout -k 10 200 python -u x_ablate.py 3) > gpurun_out/r02d_abl.log 2>&1; rc=$?; tail -12 gpurun_out/r02d_abl.log
[ $rc -ne 0 ] && exit $rc
NOBENCH=1 bash tools/gpu_tests.sh r02d tests/test_gpu_torch_ops.py tests/test_gpu_train_api.py tests/test_gpu_model.py
