#!/bin/bash
# Repeated bench A/B of an env toggle: on, off, on, off (20k steps each).
set -eo pipefail
VAR=${1:-DQZ_FUSED_FWD}
mkdir -p gpurun_out
for r in 1 2; do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 20000 --profile-iters 1 > gpurun_out/ab2_${v}_$r.json 2>> gpurun_out/ab2.err
  done
done
