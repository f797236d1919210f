#!/bin/bash
# mixed-model GPU tests first (new kernels), then the whole GPU suite
set -u
mkdir -p gpurun_out/mixed
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mixed/pytest_mixed.log 2>&1
rc=$?; tail -15 gpurun_out/mixed/pytest_mixed.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mixed/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/mixed/pytest_gpu.log; exit $rc
