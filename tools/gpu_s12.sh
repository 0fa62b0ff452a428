#!/bin/bash
# Merged backward + update, timing-only decomposition: e1 (update blocks exit
# at once), e2 (no waits), base, noupd; then traces of e1 and e2.
set -eo pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/s12
mkdir -p $OUT
for r in 1 2; do
  for v in base e1 e2 noupd; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], d['handoff_status'])" | tee -a $OUT/summary.txt
  done
done
