#!/bin/bash
# round 3: ablation attribution on the batched-scan merge; EAP at config-3 scale (cell-restricted kernel)
set -u
OUT=gpurun_out/${1:-r03i}
mkdir -p $OUT
for x in base 3 8 10 7 9 base; do
  if [ $x = base ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_k$x.so; fi
  PHDSLAM_LIB=$LIB timeout -k 10 120 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b_$x.json 2> $OUT/b_$x.err
  python3 -c "import json;d=json.load(open('$OUT/b_$x.json'));print('$x', d['value'], 'steps/s, update', d['roofline']['avg_kernel_ms'], 'ms')" 2>/dev/null || { echo "$x failed"; tail -2 $OUT/b_$x.err; }
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -q --timeout 500 --timeout-method thread -p no:cacheprovider -s \
  -k "expected_map" > $OUT/pytest_eap.log 2>&1
rc=$?; tail -3 $OUT/pytest_eap.log; grep -E "eap config" $OUT/pytest_eap.log; exit $rc
