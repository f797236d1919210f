#!/bin/bash
# round-2 baseline on the GPU box: parity tests, config-3 bench line, kernel stats
set -u
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02a/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r02a/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r02a/bench_c3.json 2> gpurun_out/r02a/bench_c3.err || exit $?
cat gpurun_out/r02a/bench_c3.json
exit 0
