#!/bin/bash
# Interleaved A/B of the default bench in this tree and in another checkout
# copied under the repo (e.g. ab_r02/ = the previous round's final commit,
# library built there).  usage: bash tools/ab_tree.sh ROUNDS OTHER_DIR
set -eo pipefail
R=$1; O=$2
mkdir -p gpurun_out/abt
for r in $(seq 1 $R); do
  timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 > gpurun_out/abt/head_$r.json 2> gpurun_out/abt/head_$r.err
  (cd $O && timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0) > gpurun_out/abt/other_$r.json 2> gpurun_out/abt/other_$r.err
  python -c "import json; a=json.loads(open('gpurun_out/abt/head_$r.json').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/abt/other_$r.json').read().strip().splitlines()[-1]); print($r, 'head', a['value'], {k: round(v*1e3,2) for k,v in a['phase_ms'].items()}); print($r, 'other', b['value'], {k: round(v*1e3,2) for k,v in b['phase_ms'].items()})"
done
