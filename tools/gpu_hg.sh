#!/bin/bash
# CenterNet hourglass GPU pass: its parity tests and a bench line.
set -o pipefail
TAG=${1:-hg}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hourglass.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
grep -E "passed|failed|rel-L2|oracle" gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --model centernet --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
