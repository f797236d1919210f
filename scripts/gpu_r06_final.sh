#!/bin/bash
# Round-6 closing evidence on the final tree: the default bench line and the
# driver's 20-step shape, kernel stats (config 3), PMC traffic / issue passes
# of every benched shape, part C stall counters, the other configs' lines
# (2, 4 and 5 per GPU, sequence mode) and config 1's CPU line.
# usage: scripts/gpu_r06_final.sh <tag> [a|b|all]   (a: config 3 lines, kernel
# stats, PMC and stall passes; b: the other configs' lines and per-GPU PMC)
set -u
T=${1:-r06fin}
STAGE=${2:-all}
OUT=gpurun_out/$T
REPO=$(pwd)
mkdir -p $OUT
b() { local name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }; echo "$name: $(python3 -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['unit'], d['roofline'] and d['roofline'].get('frac'))")"; }
if [ "$STAGE" != b ]; then
# (the PMC passes first: their report refreshes profiles/traffic_c3.json, which
# the bench lines below carry as roofline.traffic)
bash scripts/gpu_round_pmc.sh ${T}_pmc_c3 3 > $OUT/pmc_c3.txt 2>&1 || { tail -5 $OUT/pmc_c3.txt; exit 1; }
echo pmc c3 done
b bench_default
b bench_20 --steps 20 --warmup 5
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp_c3 -o run -- python3 $REPO/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-config4-model > $REPO/$OUT/rp_c3.json 2> $REPO/$OUT/rp_c3.err) || { tail -5 $OUT/rp_c3.err; exit 1; }
find $OUT/rp_c3 -name '*kernel_stats.csv' -exec cp {} $OUT/c3_kernel_stats.csv \;
bash scripts/gpu_stall.sh ${T}_stall > $OUT/stall.txt 2>&1 || { tail -5 $OUT/stall.txt; exit 1; }
echo stall done
fi
if [ "$STAGE" != a ]; then
bash scripts/gpu_pmc_pergpu.sh ${T} > $OUT/pmc_pergpu.txt 2>&1 || { tail -5 $OUT/pmc_pergpu.txt; exit 1; }
echo pmc per-GPU done
b c2 --config 2
b c4_pergpu --config 4 --particles 4096
b c5_pergpu --config 5 --particles 8192 --steps 50 --warmup 5
b c3_sequence --mode sequence --no-config4-model
b c1 --config 1
fi
echo all done
