#!/bin/bash
# round 3: fused vs three-launch CPHD update (A/B), then the new parity tests
set -u
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
for rep in 1 2; do
  for mode in 00 01 10 11; do
    f=${mode:0:1}; c=${mode:1:1}
    PHD_CPHD_FUSED=$f PHD_MERGE_CELL=$c timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3_m${mode}_$rep.json 2> $OUT/c3_m${mode}_$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$OUT/c3_m${mode}_$rep.json'));print('fused=$f cell=$c rep $rep:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
  done
done
timeout -k 10 1500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "bench_configuration or cphd_update_matches or update_matches_oracle or series_near or sharded or empty_maps" > $OUT/pytest_new.log 2>&1
rc=$?; tail -5 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 3 > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_bench.json'));print('config 3:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms']); print(json.dumps(d.get('cpu_baseline')))"
timeout -k 10 300 python bench.py --config 3 --mode sequence --no-cpu-baseline > $OUT/c3_seq.json 2> $OUT/c3_seq.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/c3_seq.json'));print('config 3 sequence mode:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
