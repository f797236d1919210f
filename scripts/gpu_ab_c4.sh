set -u
OUT=gpurun_out/r06nob; mkdir -p $OUT
for rep in 1 2 3; do
  for v in main nob; do
    if [ $v = main ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_vnob.so; fi
    PHDSLAM_LIB=$LIB timeout -k 10 200 python3 bench.py --config 4 --particles 4096 --no-cpu-baseline --steps 300 --warmup 20 > $OUT/c4_${v}_$rep.json 2> $OUT/c4_${v}_$rep.err || exit 1
    echo "$v rep $rep: $(python3 -c "import json; d=json.load(open('$OUT/c4_${v}_$rep.json')); print(d['value'], d['ms_per_step'])")"
  done
done
