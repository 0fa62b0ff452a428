#!/bin/bash
# Interleaved A/B of prebuilt library variants on one bench workload.
# usage: DQZ_ALLOW_STALE=1 bash tools/abv_algo.sh ALGO ROUNDS lib1.so lib2.so ...
set -eo pipefail
A=$1; R=$2; shift 2
mkdir -p gpurun_out/abv
for r in $(seq 1 $R); do
  for L in "$@"; do
    n=$(basename $L .so)
    DQZ_LIB=$PWD/$L timeout -k 10 120 python bench.py --algo $A --steps 10000 --warmup 500 --cpu-seconds 0 \
      > gpurun_out/abv/${A}_${n}_$r.json 2> gpurun_out/abv/${A}_${n}_$r.err
    python -c "import json,sys; d=json.loads(open('gpurun_out/abv/${A}_${n}_$r.json').read().strip().splitlines()[-1]); print('$A', '$n', $r, d['value'])"
  done
done
