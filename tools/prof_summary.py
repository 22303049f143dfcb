"""Summarise a rocprofv3 --kernel-trace --stats run as markdown.

Accepts the `*_kernel_stats.csv` of `-f csv` runs or the `*_results.db` (rocpd sqlite) of the
default output format; for a .db it also writes the equivalent kernel_stats CSV next to the
markdown so the numbers can be committed under profiles/.
usage: prof_summary.py <stats.csv|results.db> <profiled steps> <title> [csv_out]"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    out = []
    for name, calls, tot, avg, mn, mx in c.execute(
            "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
            "from kernels group by name"):
        out.append({"Name": name, "Calls": str(calls), "TotalDurationNs": str(tot), "AverageNs": str(avg),
                    "MinNs": str(mn), "MaxNs": str(mx)})
    return out


def main(path, steps, title, csv_out=None):
    rows = rows_from_db(path) if path.endswith(".db") else list(csv.DictReader(open(path)))
    if csv_out:
        with open(csv_out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
            w.writeheader()
            for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
                w.writerow({k: r.get(k, "") for k in w.fieldnames})
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
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
