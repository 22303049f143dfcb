"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    n = cnt[(k, next(iter(v)))]
    print(k, "dispatches", n, "grid", next(r["Grid_Size"] for r in rows if r["Kernel_Name"][:70] == k))
    for c, x in sorted(v.items()):
        print("   %-28s %.4g" % (c, x / n))
