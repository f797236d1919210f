#!/bin/bash
# round 3: new parity tests (bench configuration, thread instances, CPHD edges,
# sharded CPHD, config-4 full shape) + a default bench line
set -u
OUT=gpurun_out/${1:-r03a}
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "bench_configuration or cphd_update_matches or update_matches_oracle or series_near or sharded" > $OUT/pytest_new.log 2>&1
rc=$?; tail -5 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 3 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_bench.json'));print('config 3:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms']); print(json.dumps(d.get('cpu_baseline')))"
PHDSLAM_WAVE_DEFAULT=1 timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 100 > $OUT/c3_wave_bench.json 2> $OUT/c3_wave_bench.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_wave_bench.json'));print('config 3 wave form:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
