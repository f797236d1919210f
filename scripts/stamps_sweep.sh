#!/bin/bash
# Phase-stamp sweep over update launch sizes (diagnostic library), configs 2 and 3.
set -u
mkdir -p gpurun_out
for cfg in 2 3; do
  for nt in 0 256 512 1024; do
    echo "=== config $cfg threads $nt" >> gpurun_out/stamps.log
    timeout -k 10 200 python scripts/phase_stamps.py --config $cfg --threads $nt >> gpurun_out/stamps.log 2>&1 || exit $?
  done
done
