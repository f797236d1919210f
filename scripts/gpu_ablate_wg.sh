#!/bin/bash
# config-3 bench of the shipped library and of workgroup-update ablation builds
# (libphdslam_k<X>.so, PHD_XK): kernel time per removed phase
set -u
OUT=gpurun_out/${1:-abl}
mkdir -p $OUT
for x in base ${2:-1 2 3 4 6}; do
  if [ $x = base ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_k$x.so; fi
  PHDSLAM_LIB=$LIB timeout -k 10 120 python bench.py --config ${3:-3} --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b_$x.json 2> $OUT/b_$x.err || { tail -3 $OUT/b_$x.err; }
  python3 -c "import json;d=json.load(open('$OUT/b_$x.json'));print('$x', d['value'], 'steps/s, update', d['roofline']['avg_kernel_ms'], 'ms')" 2>/dev/null || echo "$x failed"
done
exit 0
