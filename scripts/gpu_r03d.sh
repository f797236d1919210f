#!/bin/bash
# round 3: cell-merge emission in candidate order — M=127 debug, stamps, A/B
set -u
OUT=gpurun_out/${1:-r03d}
mkdir -p $OUT
timeout -k 10 300 python scripts/debug_m127.py > $OUT/debug_m127.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/debug_m127.log; [ $rc -ne 0 ] && exit $rc
for cell in 0 1; do
  PHD_MERGE_CELL=$cell PHDSLAM_LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_stamps.so timeout -k 10 200 python scripts/phase_stamps.py --config 3 > $OUT/stamps_cell$cell.log 2>&1 || { tail -5 $OUT/stamps_cell$cell.log; exit 1; }
  echo "== cell $cell"; grep -E "per-WG|cull|emit|screen|lfmis|bucket" $OUT/stamps_cell$cell.log
done
for rep in 1 2; do
  for cell in 0 1; do
    PHD_MERGE_CELL=$cell timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3_cell${cell}_$rep.json 2> $OUT/c3_cell${cell}_$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$OUT/c3_cell${cell}_$rep.json'));print('cell=$cell rep $rep:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
  done
done
