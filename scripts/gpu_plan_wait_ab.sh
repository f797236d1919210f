#!/bin/bash
# The plan wait: k_wait_plan (shipped) against the cross-stream event
# (libphdslam_vevw.so, -DPHD_PLAN_WAIT_KERNEL=0), alternating by swapping the
# library file (the C++ group library binds libphdslam.so by name): the sharded
# parity tests on the shipped library, world 1 over RCCL (C++ and Python
# transports) and the emulated world-8 step at config 3, single step beside.
# usage: scripts/gpu_plan_wait_ab.sh <tag> [reps]
set -u
OUT=gpurun_out/${1:-pwab}; REPS=${2:-2}
mkdir -p $OUT
D=cuda-phdslam_amd/phdslam
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "shard or group" > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
echo "parity: $(tail -1 $OUT/parity.log)"
cp $D/libphdslam.so $D/libphdslam_wk.so
restore() { cp $D/libphdslam_wk.so $D/libphdslam.so; }
trap restore EXIT
for rep in $(seq 1 $REPS); do
  for v in wk evw; do
    if [ $v = wk ]; then cp $D/libphdslam_wk.so $D/libphdslam.so; else cp $D/libphdslam_vevw.so $D/libphdslam.so; fi
    for t in single cxx torch; do
      A=""; [ $t != single ] && A="--force-sharded --transport $t"
      timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline --no-config4-model $A > $OUT/${v}_${t}_$rep.json 2> $OUT/${v}_${t}_$rep.err || { tail -5 $OUT/${v}_${t}_$rep.err; exit 1; }
    done
    timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 200 > $OUT/${v}_w8_$rep.txt 2> $OUT/${v}_w8_$rep.err || { tail -5 $OUT/${v}_w8_$rep.err; exit 1; }
    python3 - $OUT $v $rep <<'PY'
import json, sys, ast
o, v, r = sys.argv[1:4]
d = {t: json.load(open(f"{o}/{v}_{t}_{r}.json")) for t in ("single", "cxx", "torch")}
w8 = ast.literal_eval(open(f"{o}/{v}_w8_{r}.txt").read().strip().splitlines()[-1])
us = {t: d[t]["ms_per_step"] * 1e3 for t in d}
print(f"{v} rep {r}: single {us['single']:.1f} us, cxx {us['cxx']:.1f} (+{us['cxx'] - us['single']:.1f}), "
      f"torch {us['torch']:.1f} (+{us['torch'] - us['single']:.1f}); emulated w8 {w8['sharded_step_us']:.1f} "
      f"(+{w8['sharded_minus_fused_us']:.1f})", flush=True)
PY
  done
done
