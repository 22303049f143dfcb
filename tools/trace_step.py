"""Per-dispatch timeline of the LAST profiled step of a rocprofv3 kernel trace: dispatches from the
last `lr_schedule` kernel back to the previous one (the update graph ends each step), with gaps.
usage: trace_step.py <kernel_trace.csv> [top N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "lr_schedule" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
busy = 0
gap = 0
prev_end = None
agg = []
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev_end is not None:
        gap += max(0, s - prev_end)
    prev_end = e
    busy += e - s
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    name = name[:60]
    agg.append((e - s, name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
span = int(step[-1]["End_Timestamp"]) - t0
print("dispatches %d  span %.3f ms  busy %.3f ms  gaps %.3f ms" % (len(step), span / 1e6, busy / 1e6, gap / 1e6))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if n:
    for i, (d, name, g) in enumerate(step_list := agg):
        print("%4d %8.1f us  wg %6d  %s" % (i, d / 1e3, g, name))
