#!/bin/bash
# Code-layout sweep: one 20,000-step default bench per prebuilt library
# (libdqz_<name>.so; e.g. DQZ_LAYOUT_PAD variants from tools/build_variants.sh),
# base first and last.  A/B arms only (DQZ_ALLOW_STALE for the variants).
# usage: bash tools/gpu_layout_sweep.sh TAG variant...
set -eo pipefail
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export DQZ_ALLOW_STALE=1
for v in base "$@" base; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_$v.json 2> $OUT/bench_$v.err
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value'])" | tee -a $OUT/summary.txt
done
