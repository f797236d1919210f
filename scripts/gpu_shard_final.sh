#!/bin/bash
# Round-6 close: the sharded step's cost on the final tree — world 1 over RCCL
# (C++ rank transport and Python ShardedFilter against the single step,
# alternating) and the emulated world-8 overhead at configs 3 and 4.
# usage: scripts/gpu_shard_final.sh <tag>
set -u
OUT=gpurun_out/${1:-shardfin}
mkdir -p $OUT
for rep in 1 2; do
  for t in single cxx torch; do
    A=""; [ $t != single ] && A="--force-sharded --transport $t"
    timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-config4-model $A > $OUT/${t}_$rep.json 2> $OUT/${t}_$rep.err || { tail -5 $OUT/${t}_$rep.err; exit 1; }
  done
  python3 - $OUT $rep <<'PY'
import json, sys
o, r = sys.argv[1], sys.argv[2]
v = {k: json.load(open(f"{o}/{k}_{r}.json")) for k in ("single", "cxx", "torch")}
print(f"rep {r}: " + "  ".join(f"{k} {d['value']:.1f} steps/s ({d['ms_per_step'] * 1e3:.1f} us)" for k, d in v.items()),
      f" overhead cxx {(v['cxx']['ms_per_step'] - v['single']['ms_per_step']) * 1e3:.1f} us,"
      f" torch {(v['torch']['ms_per_step'] - v['single']['ms_per_step']) * 1e3:.1f} us", flush=True)
PY
done
for c in 3 4; do
  timeout -k 10 300 python scripts/shard_overhead.py --config $c --world 8 --steps 200 > $OUT/w8_c$c.txt 2> $OUT/w8_c$c.err || { tail -5 $OUT/w8_c$c.err; exit 1; }
  echo "world 8 emulated, config $c:"; tail -4 $OUT/w8_c$c.txt
done
