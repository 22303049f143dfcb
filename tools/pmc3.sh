#!/bin/bash
# Three separate rocprofv3 --pmc passes (MFMA busy + wave-state cycles + GRBM | FETCH_SIZE |
# WRITE_SIZE) over a python program, reduced per (kernel, grid) by tools/pmc_bb3_json.py.
# usage: bash tools/pmc3.sh <tag> <python script> [args...]
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for P in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -f csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -1 gpurun_out/${TAG}_p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_bb3_json.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 gpurun_out/${TAG}_p3 gpurun_out/${TAG}_pmc.json
