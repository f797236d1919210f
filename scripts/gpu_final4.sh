#!/bin/bash
# Round-4 end evidence on the final tree: GPU parity suite + smoke, PMC passes
# (HBM traffic, VALU / LDS issue) for configs 3 and 2, bench lines + kernel
# stats for configs 2 and 3 (profile_round.sh), and the per-GPU bench lines of
# configs 4 and 5.
# usage: scripts/gpu_final4.sh <tag>
set -u
TAG=${1:-r04end}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/gpu_tests.sh $TAG || exit $?
bash scripts/gpu_round_pmc.sh ${TAG}_pmc3 3 || exit $?
bash scripts/gpu_round_pmc.sh ${TAG}_pmc2 2 || exit $?
bash scripts/profile_round.sh $TAG || exit $?
for CFG in 4 5; do
  NP=$([ $CFG = 4 ] && echo 4096 || echo 8192)
  timeout -k 10 300 python3 bench.py --config $CFG --particles $NP --steps 60 --warmup 10 > $OUT/c${CFG}_pergpu_bench.json 2> $OUT/c${CFG}_pergpu_bench.err || { tail -5 $OUT/c${CFG}_pergpu_bench.err; exit 1; }
  head -c 400 $OUT/c${CFG}_pergpu_bench.json; echo
done
