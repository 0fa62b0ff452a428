#!/bin/bash
# A/B of the bench's world-1 RCCL usage: in-loop stats gathers after a device
# drain (default), async gathers behind the queued graphs, no group at all.
set -eo pipefail
mkdir -p gpurun_out/ab_rccl
for r in 1 2; do
  for V in default async nogroup; do
    case $V in
      default) E="";;
      async) E="DQZ_BENCH_STATS=async";;
      nogroup) E="DQZ_BENCH_NO_GROUP=1";;
    esac
    env $E timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 \
      > gpurun_out/ab_rccl/${V}_$r.json 2> gpurun_out/ab_rccl/${V}_$r.err
    python -c "import json; d=json.loads(open('gpurun_out/ab_rccl/${V}_$r.json').read().splitlines()[-1]); print('$V', $r, d['value'], d['rccl']['backend'], d['rccl']['in_loop_gathers'])"
  done
done
