#!/bin/bash
# SURVEY §8(d) timing protocol on the GPU box: warm-up 200, 10,000 timed
# steps, five runs; prints each run's value and the median.
# usage: bash tools/bench_median.sh [out_dir]
set -eo pipefail
OUT=${1:-gpurun_out/median}
mkdir -p $OUT
for r in 1 2 3 4 5; do
  timeout -k 10 180 python bench.py --steps 10000 --warmup 200 --cpu-seconds 0 > $OUT/run$r.json 2> $OUT/run$r.err
done
python - "$OUT" <<'PY'
import json, statistics, sys
d = sys.argv[1]
runs = [json.load(open('%s/run%d.json' % (d, r))) for r in range(1, 6)]
vals = [x['value'] for x in runs]
print(json.dumps({'metric': runs[0]['metric'], 'unit': 'steps/s', 'runs': vals,
                  'median': statistics.median(vals), 'steps': 10000, 'warmup': 200,
                  'ms_per_step_median': statistics.median(x['ms_per_step'] for x in runs)}))
PY
