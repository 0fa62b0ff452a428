#!/bin/bash
# Spread of the driver's 20-step bench command, and with a longer warm-up.
set -o pipefail
OUT=gpurun_out/drv
mkdir -p $OUT
for r in 1 2 3; do
  for W in 5 200; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup $W --cpu-seconds 0 > $OUT/w${W}_$r.json 2> $OUT/w${W}_$r.err || exit $?
    python -c "import json; d=json.load(open('$OUT/w${W}_$r.json')); print('warmup $W run $r', d['value'], d['ms_per_step'])" >> $OUT/drv.txt
  done
done
