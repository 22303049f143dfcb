#!/bin/bash
# full GPU test suite + CenterNet bench profile: tools/gpu_cn_prof.sh <tag>
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_cnprof -o prof -- python3 bench.py --model centernet --steps 10 --warmup 3 > gpurun_out/${TAG}_cn.json 2> gpurun_out/${TAG}_cn.err || { tail -20 gpurun_out/${TAG}_cn.err; exit 1; }
cat gpurun_out/${TAG}_cn.json
exit $rc
