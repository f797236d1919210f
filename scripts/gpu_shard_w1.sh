#!/bin/bash
# Round 6: the sharded step at world 1 against the single-GPU step (config 3),
# alternating: single phd_step, the C++ rank transport (GroupRank, one C call
# per step) and the Python ShardedFilter over torch.distributed (RCCL); then a
# kernel + HIP-API trace of each sharded transport.
# usage: scripts/gpu_shard_w1.sh <tag> [reps]
set -u
OUT=gpurun_out/${1:-shardw1}; REPS=${2:-2}
mkdir -p $OUT
REPO=$(pwd)
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-config4-model > $OUT/single_$rep.json 2> $OUT/single_$rep.err || { tail -5 $OUT/single_$rep.err; exit 1; }
  timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-config4-model --force-sharded --transport cxx > $OUT/cxx_$rep.json 2> $OUT/cxx_$rep.err || { tail -5 $OUT/cxx_$rep.err; exit 1; }
  timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-config4-model --force-sharded --transport torch > $OUT/torch_$rep.json 2> $OUT/torch_$rep.err || { tail -5 $OUT/torch_$rep.err; exit 1; }
  python3 - $OUT $rep <<'PY'
import json, sys
o, r = sys.argv[1], sys.argv[2]
v = {k: json.load(open(f"{o}/{k}_{r}.json")) for k in ("single", "cxx", "torch")}
print(f"rep {r}: " + "  ".join(f"{k} {d['value']:.1f} steps/s ({d['ms_per_step'] * 1e3:.1f} us)" for k, d in v.items()),
      f" overhead cxx {(v['cxx']['ms_per_step'] - v['single']['ms_per_step']) * 1e3:.1f} us,"
      f" torch {(v['torch']['ms_per_step'] - v['single']['ms_per_step']) * 1e3:.1f} us")
PY
done
for t in cxx torch; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace --stats --output-format csv -d $REPO/$OUT/trace_$t -o run -- python3 $REPO/bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-config4-model --force-sharded --transport $t > $REPO/$OUT/trace_$t.json 2> $REPO/$OUT/trace_$t.err) || { tail -5 $OUT/trace_$t.err; exit 1; }
done
echo done
# the single-GPU step's kernel trace (the gaps between its launches)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/trace_single -o run -- python3 $REPO/bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-config4-model > $REPO/$OUT/trace_single.json 2> $REPO/$OUT/trace_single.err) || { tail -5 $OUT/trace_single.err; exit 1; }
echo single traced
