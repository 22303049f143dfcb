"""Median kernel-only time of the tower weight-gradient kernel per ablation variant trace
(tools/wgx_var_prof.sh output): wgx_tower_med.py <prefix> bits..."""
import csv
import sys

for b in sys.argv[2:]:
    v = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
               for r in csv.DictReader(open("%s%s/p_kernel_trace.csv" % (sys.argv[1], b)))
               if "conv_wgrad_x_kernel<256" in r["Kernel_Name"])
    print("v%s: %d launches, median %.1f us" % (b, len(v), v[len(v) // 2]))
