"""Median kernel-only duration per (kernel, grid) from rocprofv3 kernel traces of tools/wgx_var_prof.sh:
wgx_trace_summary.py <prefix> bits..."""
import collections
import csv
import sys

pre, bits = sys.argv[1], sys.argv[2:]
res = {}
for b in bits:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open("%s%s/p_kernel_trace.csv" % (pre, b))):
        n = r["Kernel_Name"]
        if "wgrad" not in n:
            continue
        k = (n.split("(")[0].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", ""),
             int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        agg[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    res[b] = {k: sorted(v)[len(v) // 2] for k, v in agg.items() if len(v) >= 20}
keys = sorted(set().union(*[set(v) for v in res.values()]))
print("| kernel | WGs | " + " | ".join("v%s us" % b for b in bits) + " |")
print("|---|---|" + "---|" * len(bits))
for k in keys:
    print("| %s | %d | %s |" % (k[0], k[1], " | ".join("%.1f" % res[b][k] if k in res[b] else "-" for b in bits)))
