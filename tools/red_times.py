"""Per-launch times of the weight-gradient kernels and split reducers in the last profiled step of
rocprofv3 kernel traces (tools/prof_quick.sh): red_times.py <tag> [tag ...]"""
import csv
import sys


def step(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "lr_schedule" in r["Kernel_Name"]]
    return rows[idx[-2] + 1:idx[-1] + 1]


for tag in sys.argv[1:]:
    st = step("gpurun_out/pq_%s/p_kernel_trace.csv" % tag)
    for key in ("reduce_batch", "wgrad_x_kernel", "wgrad_h_kernel"):
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in st if key in r["Kernel_Name"]]
        print("%s %-16s n=%2d total %7.1f us: %s" % (tag, key, len(ds), sum(ds), " ".join("%.1f" % d for d in ds)))
