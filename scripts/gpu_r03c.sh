#!/bin/bash
# round 3: debug of CPHD M=127 at 1024 threads; part C phase stamps, old vs cell-ordered merge
set -u
OUT=gpurun_out/${1:-r03c}
mkdir -p $OUT
timeout -k 10 300 python scripts/debug_m127.py > $OUT/debug_m127.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/debug_m127.log; [ $rc -ne 0 ] && exit $rc
for cell in 0 1; do
  PHD_CPHD_FUSED=0 PHD_MERGE_CELL=$cell PHDSLAM_LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_stamps.so timeout -k 10 200 python scripts/phase_stamps.py --config 3 > $OUT/stamps_cell$cell.log 2>&1 || { tail -5 $OUT/stamps_cell$cell.log; exit 1; }
  echo "== cell $cell"; grep -v amdgpu.ids $OUT/stamps_cell$cell.log
done
