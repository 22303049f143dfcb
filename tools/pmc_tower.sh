#!/bin/bash
# HBM traffic of the bench's dominant kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE and
# WRITE_SIZE do not fit one pass on gfx950), written under gpurun_out/pmc_{fetch,write}/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -o pmc -- python3 tools/tower_conv.py 10 > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -o pmc -- python3 tools/tower_conv.py 10 > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
tail -2 gpurun_out/pmc_fetch.log
