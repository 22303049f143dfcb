#!/bin/bash
# kernel-only time of the small-N head weight gradient per ablation variant (tools/sn_variants.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for b in "$@"; do
  CVL_LIB=ab/libcvlite_${SNLIB:-sn}$b.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/snv_$b -o p -- python3 tools/sn_probe.py > gpurun_out/snv_$b.txt 2>&1 || exit 1
  python3 - "$b" <<'PY'
import csv, sys
for r in csv.DictReader(open("gpurun_out/snv_%s/p_kernel_stats.csv" % sys.argv[1])):
    if "conv_wgrad_sn" in r["Name"]:
        print("variant %-3s avg %.1f us" % (sys.argv[1], float(r["AverageNs"]) / 1e3))
PY
done
