"""Per-launch HBM traffic of the fused update (k_update_fused / k_update_cphd) from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Guide (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE derive from the L2's
memory-side request counters; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  rocprofv3
reports both in KiB.  Writes profiles/traffic_c<config>.json, which bench.py
reports as roofline.traffic (bytes per update launch).
"""
import csv
import glob
import json
import os
import sys

cfg, out = sys.argv[1], sys.argv[2]
vals = {}
kname = None
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if ("k_update_fused" in name or "k_update_cphd" in name or "k_update_phd" in name) and row["Counter_Name"] == c:
                rows.append(float(row["Counter_Value"]))
                kname = name.split("(")[0]
    if not rows:
        sys.exit(f"no {c} samples for the update kernel under {out}")
    vals[c] = sum(rows) / len(rows)
fetch_b = 2.0 * vals["FETCH_SIZE"] * 1024.0
write_b = vals["WRITE_SIZE"] * 1024.0
res = {"config": int(cfg), "kernel": kname, "fetch_size_kib": vals["FETCH_SIZE"],
       "write_size_kib": vals["WRITE_SIZE"], "bytes_per_launch": fetch_b + write_b,
       "correction": "2 x FETCH_SIZE (gfx950 half-counting of wide reads) + WRITE_SIZE, KiB -> B",
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --steps 20"}
os.makedirs("profiles", exist_ok=True)
for path in (f"profiles/traffic_c{cfg}.json", f"{out}/traffic_c{cfg}.json"):  # out/ is merged back from the box
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
print(json.dumps(res))
