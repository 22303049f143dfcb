#!/bin/bash
# kernel-only FCOS loss times, four-lane form vs CVL_DISPATCH=loss_lds1 (rocprofv3 on short bench runs)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in new lds1; do
  if [ $v = lds1 ]; then export CVL_DISPATCH=loss_lds1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/lp_$v -o p -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/lp_$v.json 2> gpurun_out/lp_$v.err || exit 1
  python3 - "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open("gpurun_out/lp_%s/p_kernel_stats.csv" % sys.argv[1])):
    if "fcos_loss" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
