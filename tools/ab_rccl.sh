#!/bin/bash
# A/B of the bench's world-1 RCCL usage: group + dist.barrier (default),
# no group, timing barrier as an all_reduce, no timing barrier.
set -eo pipefail
mkdir -p gpurun_out/ab_rccl
for r in 1 2; do
  for V in default nogroup allreduce nobarrier; do
    case $V in
      default) E="";;
      nogroup) E="DQZ_BENCH_NO_GROUP=1";;
      allreduce) E="DQZ_BENCH_BARRIER=allreduce";;
      nobarrier) E="DQZ_BENCH_BARRIER=none";;
    esac
    env $E timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 \
      > gpurun_out/ab_rccl/${V}_$r.json 2> gpurun_out/ab_rccl/${V}_$r.err
    python -c "import json; d=json.loads(open('gpurun_out/ab_rccl/${V}_$r.json').read().splitlines()[-1]); print('$V', $r, d['value'], d['rccl']['backend'], d['rccl']['in_loop_gathers'])"
  done
done
