#!/bin/bash
# the sharded plan after a change: sharded / resample parity tests, the plan's
# phase stamps (vpst), the sharded-step overhead at an emulated world 8, the
# config-3 bench
# usage: scripts/gpu_plan2.sh <tag>
set -u
OUT=gpurun_out/${1:-plan2}
mkdir -p $OUT
L=$PWD/cuda-phdslam_amd/phdslam
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "shard or group or resample or normalize" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 3 4; do
  PHDSLAM_LIB=$L/libphdslam_vpst.so timeout -k 10 300 python scripts/plan_stamps.py --config $c --world 8 --plans 50 > $OUT/stamps_c$c.txt 2>&1 || { tail -20 $OUT/stamps_c$c.txt; exit 1; }
  cat $OUT/stamps_c$c.txt
done
for c in 3 4; do
  timeout -k 10 300 python scripts/shard_overhead.py --config $c --world 8 --steps 200 > $OUT/ovh_c$c.txt 2>&1 || { tail -20 $OUT/ovh_c$c.txt; exit 1; }
  echo "c$c: $(tail -1 $OUT/ovh_c$c.txt)"
done
# optional A/B against a variant library (alternating, config 3)
if [ -n "${AB:-}" ]; then
  for rep in 1 2; do
    for v in libphdslam.so $AB; do
      PHDSLAM_LIB=$L/$v timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 200 > $OUT/ab_${v}_$rep.txt 2>&1 || { tail -20 $OUT/ab_${v}_$rep.txt; exit 1; }
      echo "$v rep $rep: $(tail -1 $OUT/ab_${v}_$rep.txt)"
    done
  done
fi
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3.json'));print('c3:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'timed', d['roofline']['timed_updates'])"
