#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) of the paired tower conv forward on the current
# default kernel.  usage: bash tools/pmc_x.sh <tag>
set -o pipefail
TAG=${1:-pmcx}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P1="SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
P3="FETCH_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -f csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 tools/tower_one.py 6 fwd > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -1 gpurun_out/${TAG}_p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
