#!/bin/bash
# Driver-command A/B (--steps 20 --warmup 5): one 20-step graph replay,
# eager launches, or 1 / 3 eager steps ahead of the graph replay.
# usage: bash tools/ab_lead.sh ROUNDS
set -eo pipefail
R=${1:-4}
mkdir -p gpurun_out/ablead
for r in $(seq 1 $R); do
  for V in "graph:" "eager:--graph 0" "lead1:--lead-eager 1" "lead3:--lead-eager 3"; do
    n=${V%%:*}; a=${V#*:}
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --profile-iters 10 $a \
      > gpurun_out/ablead/${n}_$r.json 2> gpurun_out/ablead/${n}_$r.err
    python -c "import json; d=json.load(open('gpurun_out/ablead/${n}_$r.json')); print('$n', $r, d['value'], d['ms_per_step'])"
  done
done
