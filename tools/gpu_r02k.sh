#!/bin/bash
# r02k: PMC of the current dominant kernel (tower conv fwd, default kernel selection): FETCH_SIZE,
# WRITE_SIZE and MFMA-busy passes (one rocprofv3 --pmc run each); the non-conv op table (GB/s);
# a kernel-stats profile of the bench.  usage: bash tools/gpu_r02k.sh <tag>
set -o pipefail
TAG=${1:-r02k}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -f csv -d gpurun_out/${TAG}_p$i -o pmc -- python3 tools/tower_one.py 8 fwd > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc"; tail -1 gpurun_out/${TAG}_p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 240 python3 -u tools/op_table.py --out gpurun_out/${TAG}_ops.md > gpurun_out/${TAG}_ops.log 2>&1 || { tail -20 gpurun_out/${TAG}_ops.log; exit 1; }
head -30 gpurun_out/${TAG}_ops.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -30 gpurun_out/${TAG}_prof.err; exit 1; }
cat gpurun_out/${TAG}_prof_bench.json
