"""Per-kernel time of the last profiled step of two rocprofv3 kernel traces, biggest change first.
usage: prof_diff.py <old kernel_trace.csv> <new kernel_trace.csv> [min abs change us]"""
import collections
import csv
import sys


def load(f):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "lr_schedule" in r["Kernel_Name"]]
    step = rows[idx[-2] + 1:idx[-1] + 1]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        agg[n][0] += d
        agg[n][1] += 1
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    return agg, span, len(step)


a, sa, na = load(sys.argv[1])
b, sb, nb = load(sys.argv[2])
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
print("step span %.1f -> %.1f us, dispatches %d -> %d" % (sa, sb, na, nb))
z = [0.0, 0]
for k in sorted(set(a) | set(b), key=lambda k: -(b.get(k, z)[0] - a.get(k, z)[0])):
    x, y = a.get(k, z), b.get(k, z)
    if abs(y[0] - x[0]) >= thr:
        print("%8.1f -> %8.1f  (%3d->%3d) %s" % (x[0], y[0], x[1], y[1], k[:80]))
