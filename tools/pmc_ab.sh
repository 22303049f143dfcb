#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) of the paired tower conv for the X and L256 kernels.
# usage: bash tools/pmc_ab.sh <tag>
set -o pipefail
TAG=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
for v in X L256; do
  if [ $v = L256 ]; then export CVL_CONV_NO_X=1; else unset CVL_CONV_NO_X; fi
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -f csv -d gpurun_out/${TAG}_${v}_p$i -o pmc -- python3 tools/tower_one.py 6 fwd > gpurun_out/${TAG}_${v}_p$i.log 2>&1
    rc=$?
    echo "$v pass $i rc=$rc"; tail -2 gpurun_out/${TAG}_${v}_p$i.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
