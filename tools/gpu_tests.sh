#!/bin/bash
# GPU-box pass: the given -m gpu test files (all of tests/ if none), then (unless NOBENCH=1) one
# bench line.  A test FAILURE (pytest exit 1) still runs the bench; a crash / timeout stops.
# usage: bash tools/gpu_tests.sh <tag> [test files...]
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FILES=${@:-tests}
timeout -k 10 900 python -u -m pytest $FILES -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_pytest.log | grep -v "^E " | tail -60
tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ "${NOBENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
exit $rc
