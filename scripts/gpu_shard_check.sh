#!/bin/bash
# sharded step: parity tests (emulated + two processes), full GPU suite, overhead at world 8, gloo rehearsal
set -u
OUT=gpurun_out/${1:-shard}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "sharded" > $OUT/pytest_shard.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" $OUT/pytest_shard.log | tail -20; [ $rc -ne 0 ] && { tail -40 $OUT/pytest_shard.log; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAIL" $OUT/pytest_gpu.log | head -60; exit $rc; }
timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 100 > $OUT/overhead_c3_w8.txt 2>&1 || { tail -5 $OUT/overhead_c3_w8.txt; exit 1; }
grep -v amdgpu.ids $OUT/overhead_c3_w8.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { tail -20 $OUT/bench_gloo2.err; exit 1; }
cat $OUT/bench_gloo2.json
exit 0
