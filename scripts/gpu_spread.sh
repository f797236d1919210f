#!/bin/bash
# The spread keep / remap of k_shard_plan: the sharded parity tests, the plan's
# phase stamps before (vpst0) and after (vpst), the sharded-step overhead at an
# emulated world 8 alternating with the tail-only variant (vnospread), the
# config-3 bench.
# usage: scripts/gpu_spread.sh <tag>
set -u
OUT=gpurun_out/${1:-spread}
mkdir -p $OUT
L=$PWD/cuda-phdslam_amd/phdslam
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "shard or group" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in vpst0 vpst; do
  for c in 3 4; do
    PHDSLAM_LIB=$L/libphdslam_$v.so timeout -k 10 300 python scripts/plan_stamps.py --config $c --world 8 --plans 50 > $OUT/stamps_${v}_c$c.txt 2>&1 || { tail -20 $OUT/stamps_${v}_c$c.txt; exit 1; }
    echo "== $v"; cat $OUT/stamps_${v}_c$c.txt
  done
done
for rep in 1 2; do
  for v in libphdslam.so libphdslam_vnospread.so; do
    PHDSLAM_LIB=$L/$v timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 200 > $OUT/ovh_${v}_$rep.txt 2>&1 || { tail -20 $OUT/ovh_${v}_$rep.txt; exit 1; }
    echo "$v rep $rep: $(tail -1 $OUT/ovh_${v}_$rep.txt)"
  done
done
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3.json'));print('c3:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'timed', d['roofline']['timed_updates'])"
