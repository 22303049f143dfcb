"""Per-dispatch averages of rocprofv3 --pmc counter CSVs for kernels matching a substring.
usage: pmc_summary2.py <kernel substring> <csv> [<csv> ...]"""
import csv
import sys
from collections import defaultdict

sub = sys.argv[1]
for path in sys.argv[2:]:
    by = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            by[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(path)
    for c, d in sorted(by.items()):
        print("  %-28s %16.1f  (n=%d)" % (c, sum(d.values()) / len(d), len(d)))
