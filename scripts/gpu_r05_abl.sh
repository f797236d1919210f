#!/bin/bash
# merge ablations at config 3 with births (timing only), the per-GPU config 4 /
# config 5 lines and the bench-configuration parity tests of the shipped build
set -u
OUT=gpurun_out/r05abl
mkdir -p $OUT
bash scripts/gpu_abn.sh r05abl 1 libphdslam.so libphdslam_k3.so libphdslam_k8.so libphdslam_k10.so libphdslam_k7.so libphdslam_k9.so libphdslam.so || exit 1
for c in "4 4096 300" "5 8192 100"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --particles $2 --steps $3 --no-cpu-baseline > $OUT/c$1_pergpu.json 2> $OUT/c$1.err || { tail -5 $OUT/c$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c$1_pergpu.json'));print('c$1 pergpu', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], d['config']['update_threads'], d['config']['update_lds_bytes'], d['config']['update_resident_workgroups'], d['config']['slow_paths'])"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bench_configuration or test_cphd_update_matches_oracle or test_update_matches_oracle" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
