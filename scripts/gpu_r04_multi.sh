#!/bin/bash
# round 4: RCCL at world 1 (bench.py --force-sharded, backend nccl) + its kernel
# trace, the C++ multi-GPU host at world 1 (phdslam_run --synth --gpus 1), and
# config 5's per-GPU shape in both PHD update forms (fused / split)
set -u
OUT=gpurun_out/${1:-r04multi}
mkdir -p $OUT
REPO=$(pwd)
timeout -k 10 300 python bench.py --config 3 --force-sharded --no-cpu-baseline --steps 100 --warmup 10 > $OUT/c3_rccl_w1.json 2> $OUT/c3_rccl_w1.err || { tail -20 $OUT/c3_rccl_w1.err; exit 1; }
cat $OUT/c3_rccl_w1.json | head -c 600; echo
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp_rccl -o run -- python3 $REPO/bench.py --config 3 --force-sharded --no-cpu-baseline --steps 50 --warmup 10 > $REPO/$OUT/rp_rccl.log 2>&1) || { tail -20 $OUT/rp_rccl.log; exit 1; }
find $OUT/rp_rccl -name '*kernel_stats.csv' -exec cp {} $OUT/c3_rccl_w1_kernel_stats.csv \;
head -12 $OUT/c3_rccl_w1_kernel_stats.csv | cut -c1-160
timeout -k 10 300 cuda-phdslam_amd/phdslam/phdslam_run --synth 3 --gpus 1 --replay --steps 200 > $OUT/c3_group_w1.json 2> $OUT/c3_group_w1.err || { tail -20 $OUT/c3_group_w1.err; exit 1; }
cat $OUT/c3_group_w1.json
for form in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --particles 8192 --form $form --no-cpu-baseline --steps 30 --warmup 5 > $OUT/c5_form$form.json 2> $OUT/c5_form$form.err || { tail -20 $OUT/c5_form$form.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c5_form$form.json'));c=d['config'];print('c5 form $form:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], c['update_threads'], c['update_resident_workgroups'], c['update_split'], d['roofline']['kernel'])"
done
for th in 256 512 1024; do
  timeout -k 10 300 python bench.py --config 5 --particles 8192 --form 2 --threads $th --no-cpu-baseline --steps 30 --warmup 5 > $OUT/c5_split_t$th.json 2> $OUT/c5_split_t$th.err || { tail -20 $OUT/c5_split_t$th.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c5_split_t$th.json'));c=d['config'];print('c5 split threads $th:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], c['update_resident_workgroups'])"
done
