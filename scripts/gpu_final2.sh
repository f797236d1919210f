#!/bin/bash
# Round-end evidence on the final tree: GPU parity tests + smoke, PMC passes
# (HBM traffic, VALU / LDS issue) for configs 3 and 2, then bench lines +
# kernel stats (profile_round.sh) that carry the fresh PMC numbers.
set -u
TAG=${1:-r02end}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash scripts/gpu_round_pmc.sh ${TAG}_pmc3 3 || exit $?
bash scripts/gpu_round_pmc.sh ${TAG}_pmc2 2 || exit $?
bash scripts/profile_round.sh $TAG
