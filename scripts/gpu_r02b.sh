#!/bin/bash
# round-2 state check: parity tests, then config-3/2 bench lines for the workgroup and wave update forms
set -u
OUT=gpurun_out/${1:-r02b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in 3 2; do
  for w in 0 1; do
    PHDSLAM_WAVE_DEFAULT=$w timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $OUT/b${c}_w$w.json 2> $OUT/b${c}_w$w.err || { tail -5 $OUT/b${c}_w$w.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b${c}_w$w.json'));print('config $c wave $w', d['value'], 'steps/s, update', d['roofline']['avg_kernel_ms'], 'ms', d['config']['update_threads'], d['config']['update_lds_bytes'], d['config']['update_resident_workgroups'])"
  done
done
exit 0
