#!/bin/bash
# non-temporal posterior stores: traffic of the variant, then the replay A/B
# (gpu_variants.sh) and a sequence-mode pair
# usage: scripts/gpu_nt_probe.sh <tag>
set -u
T=${1:-ntp}
REPO=$(pwd)
bash scripts/gpu_traffic_ablate.sh $T/traffic libphdslam_vnt.so > gpurun_out/$T.traffic.log 2>&1 || exit 1
bash scripts/gpu_variants.sh $T 3 nt || exit 1
for rep in 1 2; do
  for v in main nt; do
    if [ $v = main ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_v$v.so; fi
    PHDSLAM_LIB=$LIB timeout -k 10 200 python3 bench.py --config 3 --mode sequence --no-cpu-baseline --no-config4-model --steps 200 --warmup 20 > gpurun_out/$T/seq_${v}_$rep.json 2> gpurun_out/$T/seq_${v}_$rep.err || exit 1
    echo "seq $v $rep $(python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["value"])' gpurun_out/$T/seq_${v}_$rep.json)"
  done
done
