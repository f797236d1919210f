#!/bin/bash
# round-5: GPU suite + smoke, then the performance evidence (scripts/gpu_r05_perf.sh)
set -u
T=${1:-r05all}
bash scripts/gpu_tests.sh $T || exit $?
bash scripts/gpu_r05_perf.sh $T
