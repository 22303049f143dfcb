#!/bin/bash
# kernel-only times of the small-N head weight gradient (tools/sn_probe.py) for CVL_SN_WGS values
# (measurement library): tools/sn_prof.sh wgs...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for w in "$@"; do
  CVL_SN_WGS=$w CVL_LIB=ab/libcvlite_measure.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/snp_$w -o p -- python3 tools/sn_probe.py > gpurun_out/snp_$w.txt 2>&1 || exit 1
  echo "== CVL_SN_WGS=$w"; python3 - "$w" <<'PY'
import csv, sys
for r in csv.DictReader(open("gpurun_out/snp_%s/p_kernel_stats.csv" % sys.argv[1])):
    if "sn" in r["Name"]:
        print("%-40s %6s calls  avg %.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
