#!/bin/bash
# quick GPU pass over the given test selection: usage tools/gpu_t.sh <tag> <pytest args...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest "$@" -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pytest.log | tail -40
[ $rc -ne 0 ] && grep -E "^E " gpurun_out/${TAG}_pytest.log | head -30
exit $rc
