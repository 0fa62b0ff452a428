#!/bin/bash
# A/B: bench with the world-1 RCCL group vs without (DQZ_BENCH_NO_GROUP=1), interleaved.
set -eo pipefail
mkdir -p gpurun_out/ab_group
for r in 1 2; do
  for G in 0 1; do
    DQZ_BENCH_NO_GROUP=$G timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 \
      > gpurun_out/ab_group/g${G}_$r.json 2> gpurun_out/ab_group/g${G}_$r.err
    python -c "import json; d=json.load(open('gpurun_out/ab_group/g${G}_$r.json')); print('nogroup=$G', $r, d['value'], d['rccl']['backend'])"
  done
done
