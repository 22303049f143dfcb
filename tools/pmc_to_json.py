"""Reduce the two rocprofv3 --pmc passes of tools/pmc_tower.sh to the per-launch HBM traffic of the
bench's dominant kernel (MI355X_MICROARCH.md: FETCH_SIZE/WRITE_SIZE are in KB; on gfx950 FETCH_SIZE
reports half the bytes of 16-byte-per-lane streaming reads, LDS-DMA included -> x2; WRITE_SIZE is exact
for 16-byte stores).  usage: pmc_to_json.py <fetch csv> <write csv> <kernel substring> <out.json> [grid size]
(the optional grid size keeps only the dispatches of that launch shape)"""
import csv
import json
import sys


GRID = sys.argv[5] if len(sys.argv) > 5 else None


def per_launch(path, counter, sub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and sub in r["Kernel_Name"]]
    # the counter is reported per dispatch (summed over XCDs/instances by rocprofv3 per row):
    # group rows by dispatch id when several rows exist per dispatch
    by = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and sub in r["Kernel_Name"] and (GRID is None or r["Grid_Size"] == GRID):
            by.setdefault(r["Dispatch_Id"], 0.0)
            by[r["Dispatch_Id"]] += float(r["Counter_Value"])
    assert by, (path, counter, sub, len(vals))
    return sum(by.values()) / len(by), len(by)


fetch_kb, n1 = per_launch(sys.argv[1], "FETCH_SIZE", sys.argv[3])
write_kb, n2 = per_launch(sys.argv[2], "WRITE_SIZE", sys.argv[3])
out = {"kernel": sys.argv[3], "grid_size": GRID, "dispatches": [n1, n2],
       "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
       "hbm_read_bytes": fetch_kb * 1024 * 2, "hbm_write_bytes": write_kb * 1024,
       "hbm_bytes": fetch_kb * 1024 * 2 + write_kb * 1024,
       "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads incl. LDS-DMA), KB = 1024 B"}
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out))
