#!/bin/bash
# A/B (alternating) of libphdslam_base.so (previous build) against libphdslam.so at
# config 3, then the GPU parity tests on libphdslam.so.  usage: scripts/gpu_lib_ab.sh <tag> [tests-k-expr]
set -u
T=${1:-lab}; K=${2:-}
mkdir -p gpurun_out/$T
L=cuda-phdslam_amd/phdslam
for v in base new base new base new; do
  lib=$L/libphdslam.so; [ $v = base ] && lib=$L/libphdslam_base.so
  PHDSLAM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 400 --warmup 40 > gpurun_out/$T/b_$v.json 2> gpurun_out/$T/b_$v.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/$T/b_$v.json'));print('$v:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
done
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$T/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest.log; exit $rc
fi
