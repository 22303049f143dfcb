"""Summarise a rocprofv3 --kernel-trace --stats run (kernel_stats.csv) as markdown."""
import csv
import sys


def main(path, steps, title):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("# %s\n" % title)
    print("Source: `%s` (rocprofv3 --kernel-trace --stats); %d profiled steps incl. warm-up/capture.\n" % (path, steps))
    print("Total GPU kernel time %.3f ms = %.3f ms per step.\n" % (tot / 1e6, tot / 1e6 / steps))
    print("| % | total ms | ms/step | calls | avg us | kernel |")
    print("|---|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        t = float(r["TotalDurationNs"])
        print("| %.2f | %.3f | %.3f | %s | %.1f | `%s` |" % (100 * t / tot, t / 1e6, t / 1e6 / steps, r["Calls"],
                                                         float(r["AverageNs"]) / 1e3, r["Name"][:110]))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
