#!/bin/bash
# round-5 closing evidence on one MI355X: GPU suite + smoke, bench lines of
# every shape (with the CPU baselines), sequence mode, sharded overhead at
# emulated world 8, kernel stats and PMC passes of the config-3 step, stamps
set -u
T=${1:-r05fin}
OUT=gpurun_out/$T
mkdir -p $OUT
bash scripts/gpu_tests.sh $T || exit $?
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'frac', d['roofline']['frac'], 'slow', d['config']['slow_paths'], 'cpu', d.get('cpu_baseline',{}).get('value'), 'c4model', (d.get('config4_model') or {}).get('filter_steps_per_s'))"
}
b c3 --steps 400 || exit 1
b c3_nobirths --births 0 --no-cpu-baseline --no-config4-model --steps 400 || exit 1
b c3_sequence --mode sequence --no-cpu-baseline --no-config4-model --steps 400 || exit 1
b c2 --config 2 --steps 400 || exit 1
b c4_pergpu --config 4 --particles 4096 --steps 300 || exit 1
b c5_pergpu --config 5 --particles 8192 --steps 100 || exit 1
b c3_sharded_w1 --force-sharded --no-cpu-baseline --steps 200 || exit 1
for c in 3 4; do
  timeout -k 10 300 python scripts/shard_overhead.py --config $c --world 8 --steps 300 > $OUT/shard_overhead_c${c}_w8.txt 2>&1 || { tail -5 $OUT/shard_overhead_c${c}_w8.txt; exit 1; }
  tail -1 $OUT/shard_overhead_c${c}_w8.txt
done
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/stamps_c3_partC.txt 2>&1 || { tail -5 $OUT/stamps_c3_partC.txt; exit 1; }
timeout -k 10 300 python scripts/phase_stamps.py --config 3 --part A > $OUT/stamps_c3_partA.txt 2>&1 || { tail -5 $OUT/stamps_c3_partA.txt; exit 1; }
bash scripts/gpu_round_pmc.sh ${T}_pmc_c3 3 || exit 1
