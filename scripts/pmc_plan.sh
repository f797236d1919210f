#!/bin/bash
# PMC passes over the sharded-step plan kernel (scripts/shard_overhead.py, world 8):
# where the one-block k_shard_plan spends its cycles.
set -u
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_plan
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_IFETCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$REPO/scripts/shard_overhead.py" --config 2 --world 8 --steps 40 > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for x in csv.DictReader(open(f)):
        if "shard_plan" not in x["Kernel_Name"] and "normalize_resample" not in x["Kernel_Name"]:
            continue
        k = (x["Kernel_Name"][:24], x["Counter_Name"]); agg[k] += float(x["Counter_Value"]); cnt[(k[0], x["Dispatch_Id"])] = 1
    nd = collections.Counter(k[0] for k in cnt)
    for k, v in sorted(agg.items()):
        print(k[0], k[1], round(v / nd[k[0]], 1))
PY
