#!/bin/bash
# Timing-only sensitivity of the backward launch: traces and benches of the
# DQZ_EXP_SKIP variants (numerics wrong by design) against the default.
# usage: bash tools/gpu_skip.sh TAG V1 V2 ...   (variant suffixes, 0 = default)
set -eo pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = 0 ]; then T=dqn_mgsc_zoo_amd/libdqz_trace.so; else T=dqn_mgsc_zoo_amd/libdqz_trace_s$v.so; fi
  DQZ_TRACE_PREBUILT=1 DQZ_TRACE_LIB=$PWD/$T timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_$v.txt 2>&1
done
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = 0 ]; then L=dqn_mgsc_zoo_amd/libdqz.so; else L=dqn_mgsc_zoo_amd/libdqz_s$v.so; fi
    DQZ_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], {k: round(x*1e3,2) for k,x in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
  done
done
