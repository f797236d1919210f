#!/bin/bash
# round-3 supplementary evidence on the final tree: sequence-mode and config-5
# per-GPU bench lines, part C phase stamps, the sharded-step overhead at world 8
set -u
OUT=gpurun_out/${1:-r03extra}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 3 --mode sequence --no-cpu-baseline > $OUT/c3_sequence_bench.json 2> $OUT/c3_sequence.err || exit $?
tail -c 300 $OUT/c3_sequence_bench.json; echo
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $OUT/c5_pergpu_bench.json 2> $OUT/c5_pergpu.err || exit $?
tail -c 300 $OUT/c5_pergpu_bench.json; echo
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/c3_partC_phase_stamps.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 > $OUT/shard_overhead_c3_w8.txt 2>&1 || exit $?
tail -3 $OUT/shard_overhead_c3_w8.txt
