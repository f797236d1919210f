#!/bin/bash
set -u
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
for t in 256 1024; do
  timeout -k 10 200 python scripts/debug_m127b.py $t 2>&1 | grep -v amdgpu.ids || exit 1
  echo "-- KEEP (no context freed)"; KEEP=1 timeout -k 10 200 python scripts/debug_m127b.py $t 2>&1 | grep -v amdgpu.ids || exit 1
  echo "-- ZSYNC"; PHD_ZSYNC=1 timeout -k 10 200 python scripts/debug_m127b.py $t 2>&1 | grep -v amdgpu.ids || exit 1
done
