#!/bin/bash
# Merged backward + update: poll sleep 32 (base) / 8 / 127 against the update
# launch (noupd): interleaved learner benches, meta benches, a base trace.
set -eo pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/s11
mkdir -p $OUT
for r in 1 2 3; do
  for v in base s8 s127 noupd; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], d['handoff_status'], {k: round(x*1e3,2) for k,x in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
  done
done
for v in base s8 s127 noupd; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$v.json 2> $OUT/meta_$v.err
  python -c "import json; d=json.load(open('$OUT/meta_$v.json')); print('$v', {k: round(1e3*x['ms_per_step'],1) for k,x in d.items() if k.startswith('meta')})" | tee -a $OUT/summary.txt
done
DQZ_TRACE_PREBUILT=1 DQZ_TRACE_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_trace.so timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_base.txt 2>&1
