#!/bin/bash
# bench.py default (config 3, N=1) and a 2-rank gloo rehearsal of the N>1 path on one GPU.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --cpu-budget 6 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
cat gpurun_out/bench_default.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 20 --warmup 4 --backend gloo > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || exit $?
cat gpurun_out/bench_gloo2.json
