#!/bin/bash
# Interleaved default-bench A/B over several checkouts copied under the repo
# (each with its own built library).  usage: bash tools/ab_trees.sh ROUNDS DIR...
# ("." is this tree; "VAR=value@DIR" runs DIR with that environment
# variable set).  Prints value and phase times per run.
set -eo pipefail
R=$1; shift
mkdir -p gpurun_out/abt
for r in $(seq 1 $R); do
  for A in "$@"; do
    D=${A##*@}; E=""; [ "$D" != "$A" ] && E=${A%@*}
    n=$(echo $A | tr './=@' '____')
    (cd $D && env $E timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0) > gpurun_out/abt/${n}_$r.json 2> gpurun_out/abt/${n}_$r.err
    python -c "import json; a=json.loads(open('gpurun_out/abt/${n}_$r.json').read().strip().splitlines()[-1]); print($r, '$A', a['value'], {k: round(v*1e3,2) for k,v in a['phase_ms'].items()})"
  done
done
