#!/bin/bash
# Session: the full GPU suite, B = 1 step traces (fused forward with the fc1
# GEMV, and the two-launch forward), then meta benches base / nogemv / nofuse.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/s9
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
export DQZ_TRACE_PREBUILT=1
BATCH=1 DQZ_TRACE_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_trace.so timeout -k 10 200 python -u tools/trace_step.py > $OUT/b1_trace.txt 2>&1
BATCH=1 DQZ_TRACE_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_trace_nofuse.so timeout -k 10 200 python -u tools/trace_step.py > $OUT/b1_trace_nofuse.txt 2>&1
for r in 1 2; do
  for v in base nogemv nofuse; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_${v}_$r.json 2> $OUT/meta_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/meta_${v}_$r.json')); print('$v', $r, {k: round(1e3*x['ms_per_step'],1) for k,x in d.items() if k.startswith('meta')})" | tee -a $OUT/summary.txt
  done
done
exit 0
