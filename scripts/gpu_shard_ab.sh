#!/bin/bash
# sharded step: parity tests, then its per-step overhead (world 8, emulated transport), A (base) vs B (current)
set -u
OUT=gpurun_out/${1:-shard_ab}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sharded or global_resample or shard or resample" > $OUT/pytest_shard.log 2>&1
rc=$?; tail -2 $OUT/pytest_shard.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_base.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam.so; fi
    PHDSLAM_LIB=$LIB timeout -k 10 200 python scripts/shard_overhead.py --config 3 --world 8 --steps 100 > $OUT/ovh_${v}_$rep.txt 2>&1 || exit $?
    echo "$v rep $rep: $(tail -1 $OUT/ovh_${v}_$rep.txt)"
  done
done
