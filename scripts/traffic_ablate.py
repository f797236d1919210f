"""Per-launch HBM bytes of each update kernel for the libraries measured by
scripts/gpu_traffic_ablate.sh (FETCH_SIZE x 2 per the gfx950 calibration +
WRITE_SIZE, KiB -> B; averages over the profiled launches), and the shipped
library's L2 hit rate per kernel.

usage: python scripts/traffic_ablate.py gpurun_out/<tag> [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("k_update_cphd_a", "k_cphd_terms", "k_update_cphd_c")


def per_kernel(d, counters):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            k = next((k for k in KERNELS if k in name), None)
            if k is None or row["Counter_Name"] not in counters:
                continue
            # one row per dispatch and counter (the _sum counters are already summed)
            acc[k][(row["Counter_Name"], row.get("Dispatch_Id", row.get("Correlation_Id", "")))].append(
                float(row["Counter_Value"]))
    out = {}
    for k, m in acc.items():
        per_c = defaultdict(list)
        for (c, _), v in m.items():
            per_c[c].append(sum(v))
        out[k] = {c: sum(v) / len(v) for c, v in per_c.items()}
    return out


def main():
    root = sys.argv[1]
    res = {"source": "scripts/gpu_traffic_ablate.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, "
                     "bench.py --config 3 --steps 20 --warmup 2; bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B)",
           "libraries": {}}
    for lib in sorted(os.listdir(root)):
        if not lib.endswith(".so"):
            continue
        f = per_kernel(f"{root}/{lib}/FETCH_SIZE", {"FETCH_SIZE"})
        w = per_kernel(f"{root}/{lib}/WRITE_SIZE", {"WRITE_SIZE"})
        rows = {}
        for k in KERNELS:
            fb = 2.0 * 1024.0 * f.get(k, {}).get("FETCH_SIZE", 0.0)
            wb = 1024.0 * w.get(k, {}).get("WRITE_SIZE", 0.0)
            rows[k] = {"fetch_MB": round(fb / 1e6, 2), "write_MB": round(wb / 1e6, 2), "total_MB": round((fb + wb) / 1e6, 2)}
        res["libraries"][lib] = rows
    if os.path.isdir(f"{root}/l2"):
        l2 = per_kernel(f"{root}/l2", {"TCC_HIT_sum", "TCC_MISS_sum"})
        res["l2_shipped"] = {k: {"hit": v.get("TCC_HIT_sum"), "miss": v.get("TCC_MISS_sum"),
                                 "hit_rate": round(v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 4)}
                             for k, v in l2.items() if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v}
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
