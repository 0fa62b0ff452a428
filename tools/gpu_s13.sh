#!/bin/bash
# Merged backward + update with per-block flags: the GPU suite, interleaved
# learner benches (base = poll sleep 32, s4, noupd), meta benches, traces.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/s13
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
for r in 1 2 3; do
  for v in base s4 noupd; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], d['handoff_status'])" | tee -a $OUT/summary.txt
  done
done
for v in base s4 noupd; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$v.json 2> $OUT/meta_$v.err
  python -c "import json; d=json.load(open('$OUT/meta_$v.json')); print('$v', {k: round(1e3*x['ms_per_step'],1) for k,x in d.items() if k.startswith('meta')})" | tee -a $OUT/summary.txt
done
DQZ_TRACE_PREBUILT=1 DQZ_TRACE_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_trace.so timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_base.txt 2>&1
exit 0
