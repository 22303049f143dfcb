#!/bin/bash
# round-end evidence: full -m gpu suite, the default bench line (with the CPU baseline), the
# rocprofv3 kernel-stats profile of the bench, side benches: tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
timeout -k 10 300 python3 bench.py --model centernet --steps 20 --warmup 5 > gpurun_out/${TAG}_cn.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --model retinanet --steps 20 --warmup 5 > gpurun_out/${TAG}_rn.json 2>/dev/null || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
exit $rc
