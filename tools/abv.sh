#!/bin/bash
# Interleaved A/B of prebuilt library variants on the GPU box.
# usage: bash tools/abv.sh ROUNDS lib1.so lib2.so ...   (paths relative to the repo root)
# Each round runs the default bench config once per library (no CPU baseline).
set -eo pipefail
R=$1; shift
mkdir -p gpurun_out/abv
for r in $(seq 1 $R); do
  for L in "$@"; do
    n=$(basename $L .so)
    DQZ_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 \
      > gpurun_out/abv/${n}_$r.json 2> gpurun_out/abv/${n}_$r.err
    python -c "import json,sys; d=json.load(open('gpurun_out/abv/${n}_$r.json')); print('$n', $r, d['value'], d['handoff_status'], {k: round(v*1e3,2) for k,v in d['phase_ms'].items()})"
  done
done
