#!/bin/bash
set -u
OUT=gpurun_out/${1:-r03f}
mkdir -p $OUT
timeout -k 10 300 python scripts/debug_m127.py > $OUT/debug_m127.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/debug_m127.log; [ $rc -ne 0 ] && exit $rc
PHDSLAM_WAVE_DEFAULT=1 timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 100 > $OUT/c3_wave.json 2> $OUT/c3_wave.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_wave.json'));print('config 3 wave form:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
timeout -k 10 1500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "bench_configuration or cphd_update_matches or update_matches_oracle or series_near or sharded or empty_maps or expected_map" > $OUT/pytest_new.log 2>&1
rc=$?; tail -5 $OUT/pytest_new.log; grep -E "eap config" $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 3 --mode sequence --no-cpu-baseline > $OUT/c3_seq.json 2> $OUT/c3_seq.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_seq.json'));print('config 3 sequence mode:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
