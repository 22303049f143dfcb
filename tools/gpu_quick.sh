#!/bin/bash
# quick GPU check: named test files (-m gpu) then the backbone 3x3 probe.  usage: gpu_quick.sh <tag> <tests...>
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 200 python3 -u tools/bb3_probe.py "" ${PROBE_ARGS}
