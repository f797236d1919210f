"""Per-launch PMC figures of the update kernels of one bench configuration.

    python scripts/pmc_report.py <config> <dir>

<dir> holds rocprofv3 outputs of separate passes of `bench.py --config N`:
  FETCH_SIZE/, WRITE_SIZE/  (HBM traffic, MI355X_MICROARCH.md §HBM: gfx950
                             FETCH_SIZE counts half of wide coalesced reads, so
                             it is doubled; WRITE_SIZE as is; both KiB.
                             Calibrated on this pool with kernels of known
                             traffic, scripts/calib/calib_fetch.hip ->
                             profiles/r03_fetch_calibration.json: coalesced
                             reads of 2, 4 and 16 B per lane and the slab-
                             shaped read all give FETCH = 0.5 x bytes; 16-B
                             rows at random give 4 x the useful bytes, i.e.
                             the 128-B lines they move; WRITE = 1.0 x)
  util/                     SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES,
                            SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_ACTIVE_INST_VALU,
                            SQ_ACTIVE_INST_LDS
  stats/                    --kernel-trace --stats (average durations)
The update is the launch (PHD) or the three launches (CPHD: part A,
k_cphd_terms, part C) between predict and normalise; figures are per launch of
each kernel and summed over the update.  Utilisations, from the instruction
counts and the kernel's average duration at 2.4 GHz on 256 CUs x 4 SIMDs:
  valu_issue = SQ_INSTS_VALU * 2 cycles / (duration * 2.4e9 * 1024 SIMDs)
      (a SIMD issues one wave64 VALU instruction per 2 cycles, §CU)
  lds_issue  = SQ_INSTS_LDS / (duration * 2.4e9 * 256 CUs)
      (LDS instructions per CU-cycle; the LDS takes one per cycle)
Writes profiles/traffic_c<N>.json (bench.py's roofline.traffic) and
profiles/pmc_c<N>.json (bench.py's roofline.valu_util / lds_util).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CLK = 2.4e9
N_CU = 256
N_SIMD = 4 * N_CU
UPDATE = ("k_update_fused", "k_update_cphd", "k_update_phd", "k_cphd_terms")


def kname(full):
    return full.split("(")[0].replace("phd::", "")


def counters(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = kname(row.get("Kernel_Name", ""))
            if k.startswith(UPDATE):
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def durations(d):
    out = {}
    for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = kname(row["Name"])
            if k.startswith(UPDATE):
                out[k] = float(row["AverageNs"]) * 1e-9
    return out


def main():
    cfg, d = sys.argv[1], sys.argv[2]
    npart = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] else ""  # a per-GPU shape other than the default
    fe, wr, ut, du = counters(f"{d}/FETCH_SIZE"), counters(f"{d}/WRITE_SIZE"), counters(f"{d}/util"), durations(f"{d}/stats")
    kernels = sorted(du)
    per = {}
    for k in kernels:
        t = du[k]
        u = ut.get(k, {})
        e = {"avg_us": round(t * 1e6, 3)}
        if k in fe and k in wr:
            e["hbm_bytes"] = 2.0 * fe[k]["FETCH_SIZE"] * 1024.0 + wr[k]["WRITE_SIZE"] * 1024.0
        if u:
            e["valu_issue"] = round(u["SQ_INSTS_VALU"] * 2 / (t * CLK * N_SIMD), 4)
            e["lds_issue"] = round(u["SQ_INSTS_LDS"] / (t * CLK * N_CU), 4)
            e.update({c: u[c] for c in sorted(u)})
        per[k] = e
    tot_t = sum(du[k] for k in kernels)
    dom = max(kernels, key=lambda k: du[k])
    res = {"config": int(cfg), "kernels": per, "update_us": round(tot_t * 1e6, 3), "dominant_kernel": dom,
           "valu_util": per[dom].get("valu_issue"), "lds_util": per[dom].get("lds_issue"),
           "update_valu_util": round(sum(ut[k]["SQ_INSTS_VALU"] for k in kernels if k in ut) * 2 / (tot_t * CLK * N_SIMD), 4),
           "definitions": "valu = SQ_INSTS_VALU*2/(dur*2.4e9*1024 SIMDs); lds = SQ_INSTS_LDS/(dur*2.4e9*256 CUs)",
           "source": "rocprofv3 --pmc passes + --kernel-trace --stats of bench.py --config %s (scripts/gpu_round_pmc.sh)" % cfg}
    traffic = sum(per[k].get("hbm_bytes", 0.0) for k in kernels)
    tr = {"config": int(cfg), "kernel": "+".join(kernels), "bytes_per_launch": traffic,
          "per_kernel_bytes": {k: per[k].get("hbm_bytes") for k in kernels},
          "correction": "2 x FETCH_SIZE (gfx950 half-counting of wide reads) + WRITE_SIZE, KiB -> B",
          "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --steps 20; summed over the update's launches"}
    sfx = f"_n{npart}" if npart else ""
    if npart:
        res["particles"] = tr["particles"] = int(npart)
    os.makedirs("profiles", exist_ok=True)
    for path, obj in ((f"profiles/pmc_c{cfg}{sfx}.json", res), (f"profiles/traffic_c{cfg}{sfx}.json", tr),
                      (f"{d}/pmc_c{cfg}{sfx}.json", res), (f"{d}/traffic_c{cfg}{sfx}.json", tr)):
        with open(path, "w") as fh:
            json.dump(obj, fh, indent=1)
    print(json.dumps({k: {x: v for x, v in e.items() if not x.startswith("SQ_")} for k, e in per.items()}))
    print("update_us", res["update_us"], "traffic", traffic, "dominant", dom, res["valu_util"], res["lds_util"])


if __name__ == "__main__":
    main()
