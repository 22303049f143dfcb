#!/bin/bash
# X32 vs X32H (halo) on the paired tower layer: event timing + one SQ/GRBM PMC pass each.
# usage: bash tools/pmc_halo.sh <tag>
set -o pipefail
TAG=${1:-pmch}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P1="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for H in 0 1; do
  for M in fwd dgrad; do
    CVL_CONV_HALO=$H timeout -k 10 60 python3 tools/tower_one.py 20 $M 2>&1 | grep done || exit 1
  done
  CVL_CONV_HALO=$H timeout -s KILL 90 rocprofv3 --pmc $P1 -f csv -d gpurun_out/${TAG}_h$H -o pmc -- python3 tools/tower_one.py 6 fwd > gpurun_out/${TAG}_h$H.log 2>&1
  rc=$?; echo "pmc halo=$H rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary2.py "conv_igemm_x32" gpurun_out/${TAG}_h0/pmc_counter_collection.csv gpurun_out/${TAG}_h1/pmc_counter_collection.csv
