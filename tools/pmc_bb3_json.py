"""Per-launch PMC of the backbone 3x3 launches from the three tools/pmc_bb3.sh passes: dispatches are
grouped by (kernel name, grid size); MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs); HBM bytes = 2 x FETCH_SIZE (gfx950 reports half of 16-B/lane streaming
reads, LDS-DMA included) + WRITE_SIZE, KB = 1024 B (MI355X_MICROARCH.md, HBM section).
usage: pmc_bb3_json.py <pass1 dir> <pass2 dir> <pass3 dir> <out.json>"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    paths = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    by = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            key = (name.split("(")[0].strip(), r["Grid_Size"])
            by[key][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return by


def mean(d):
    return sum(d.values()) / len(d) if d else None


p1, p2, p3 = (load(x) for x in sys.argv[1:4])
out = []
for key in sorted(p1):
    k, grid = key
    if "conv" not in k and "wgrad" not in k:
        continue
    c = p1[key]
    gui = mean(c.get("GRBM_GUI_ACTIVE", {}))
    mf = mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", {}))
    row = {"kernel": k, "grid": int(grid), "dispatches": len(c.get("GRBM_GUI_ACTIVE", {})),
           "mfma_busy_frac": round(mf / (1024 * gui / 8), 4) if gui and mf is not None else None,
           "grbm_gui_active": gui}
    wc = mean(c.get("SQ_WAVE_CYCLES", {}))
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            v = mean(c.get(n, {}))
            if v is not None:
                row[n.lower()[3:] + "_frac"] = round(v / wc, 4)
    f = mean(p2.get(key, {}).get("FETCH_SIZE", {}))
    w = mean(p3.get(key, {}).get("WRITE_SIZE", {}))
    if f is not None and w is not None:
        row["hbm_read_bytes"] = f * 1024 * 2
        row["hbm_write_bytes"] = w * 1024
        row["hbm_bytes"] = row["hbm_read_bytes"] + row["hbm_write_bytes"]
    out.append(row)
json.dump({"launches": out, "note": __doc__.split("usage")[0].strip()}, open(sys.argv[4], "w"), indent=1)
for r in out:
    print(r)
