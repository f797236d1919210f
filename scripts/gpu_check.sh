#!/bin/bash
# GPU-box check: parity tests, then a short bench, then a rocprofv3 kernel-trace profile.
# Each GPU step has its own time limit; a crash/timeout (rc not in {0,1}) ends the script.
set -u
REPO=$(pwd)
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
CFG=${CFG:-2}
STEPS=${STEPS:-100}
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rA > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config "$CFG" --steps "$STEPS" --warmup 10 --cpu-budget 8 > "$OUT/bench_c$CFG.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 "$OUT/bench_c$CFG.log"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c$CFG" -o run -- python3 "$REPO/bench.py" --config "$CFG" --steps "$STEPS" --warmup 10 --no-cpu-baseline > "$OUT/prof_c$CFG.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$OUT/prof_c$CFG" -name "*stats*" | head
exit $rc
