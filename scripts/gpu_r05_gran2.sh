#!/bin/bash
set -u
bash scripts/gpu_benchab.sh r05gran2/c3 3 "--steps 300" g1280 g1280ov2 || exit 1
bash scripts/gpu_benchab.sh r05gran2/c5 1 "--config 5 --particles 8192 --steps 100" g1280 || exit 1
bash scripts/gpu_benchab.sh r05gran2/c2 2 "--config 2 --steps 400" g1280 || exit 1
for v in main g1280; do python3 -c "import json;d=json.load(open('gpurun_out/r05gran2/c5/b_${v}_1.json'));c=d['config'];print('$v c5 lds', c['update_lds_bytes'], 'resident', c['update_resident_workgroups'], 'threads', c['update_threads'])"; done
for v in main g1280; do python3 -c "import json;d=json.load(open('gpurun_out/r05gran2/c2/b_${v}_1.json'));c=d['config'];print('$v c2 lds', c['update_lds_bytes'], 'resident', c['update_resident_workgroups'], 'threads', c['update_threads'], 'split', c.get('update_split'))"; done
