#!/bin/bash
# Quick A/B on the GPU box (no test suite): interleaved default benches (3
# rounds, 20,000 steps, C = 200k) of libdqz_base.so against each named
# variant, then tools/meta_bench.py once per library.  Variants are prebuilt
# from the same tree (tools/build_variants.sh).
# usage: bash tools/gpu_quick_ab.sh TAG variant...
set -eo pipefail
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  for v in base "$@"; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], {k: round(x*1e3,2) for k,x in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
  done
done
for v in base "$@"; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$v.json 2> $OUT/meta_$v.err
  python -c "import json; d=json.load(open('$OUT/meta_$v.json')); print('$v', {k: round(1e3*x['ms_per_step'],1) for k,x in d.items() if k.startswith('meta')})" | tee -a $OUT/summary.txt
done
