#!/bin/bash
# One GPU-box pass: gpu parity tests, a bench line, and a rocprofv3 kernel-stats profile.
# usage: bash tools/gpu_round.sh <tag> [tests|notests]
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest.log
fi
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -30 gpurun_out/${TAG}_prof.err; exit 1; }
cat gpurun_out/${TAG}_prof_bench.json
timeout -k 10 300 python3 bench.py --model centernet --steps 10 --warmup 3 > gpurun_out/${TAG}_cn.json 2> gpurun_out/${TAG}_cn.err || { tail -30 gpurun_out/${TAG}_cn.err; exit 1; }
cat gpurun_out/${TAG}_cn.json
timeout -k 10 300 python3 bench.py --model retinanet --steps 10 --warmup 3 > gpurun_out/${TAG}_rn.json 2> gpurun_out/${TAG}_rn.err || { tail -30 gpurun_out/${TAG}_rn.err; exit 1; }
cat gpurun_out/${TAG}_rn.json
