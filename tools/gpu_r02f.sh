set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u tools/tower_ab.py 5 > gpurun_out/r02f_ab.log 2>&1; rc=$?; tail -6 gpurun_out/r02f_ab.log
[ $rc -ne 0 ] && exit $rc
bash tools/pmc_x.sh r02f
