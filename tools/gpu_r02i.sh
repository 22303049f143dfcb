#!/bin/bash
# r02i: wgrad X kernel parity (conv + model tests), per-shape conv table, bench line.
set -o pipefail
TAG=${1:-r02i}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -q -x -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_wg.log 2>&1
rc=$?; tail -15 gpurun_out/${TAG}_wg.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 240 python -u tools/conv_table.py --out gpurun_out/${TAG}_table.md > gpurun_out/${TAG}_table.log 2>&1 || { tail -20 gpurun_out/${TAG}_table.log; exit 1; }
head -40 gpurun_out/${TAG}_table.md
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
exit $rc
