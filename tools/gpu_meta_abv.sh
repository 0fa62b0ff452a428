#!/bin/bash
# Interleaved MGSC meta-update benches (tools/meta_bench.py, M = 100, eager
# and graph-replayed, first and second order) of prebuilt library variants.
# usage: bash tools/gpu_meta_abv.sh TAG ROUNDS lib1.so lib2.so ...   (paths relative to the repo root)
set -eo pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 $R); do
  for L in "$@"; do
    n=$(basename $L .so)
    DQZ_ALLOW_STALE=1 DQZ_LIB=$PWD/$L timeout -k 10 200 python tools/meta_bench.py --steps 100 --capacity 200000 \
      > $OUT/meta_${n}_$r.json 2> $OUT/meta_${n}_$r.err
    python -c "
import json; d=json.load(open('$OUT/meta_${n}_$r.json'))
print('$n', $r, ' '.join('%s %.1f' % (k.replace('meta_M100_', ''), 1e3 * v['ms_per_step']) for k, v in d.items() if k.startswith('meta_M')))" | tee -a $OUT/meta_summary.txt
  done
done
