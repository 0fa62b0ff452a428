#!/bin/bash
# GPU session: the full GPU suite (verbose, with the tests' printed
# measurements), then interleaved default benches (20,000 steps, 1M replay)
# of prebuilt library variants, then the driver's bench command and the
# default line at the working tree's own build.
# usage: bash tools/gpu_suite_abv.sh TAG ROUNDS lib1.so lib2.so ...   (paths relative to the repo root)
# TESTS=0 skips the GPU suite; STEPS overrides the bench length.
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
rc=0
if [ "${TESTS:-1}" != 0 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
set -e
for r in $(seq 1 $R); do
  for L in "$@"; do
    n=$(basename $L .so)
    DQZ_ALLOW_STALE=1 DQZ_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps ${STEPS:-20000} --warmup 500 --cpu-seconds 0 \
      > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err
    python -c "import json; d=json.load(open('$OUT/${n}_$r.json')); print('$n', $r, d['value'], d['handoff_status'], {k: round(v*1e3,2) for k,v in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
  done
done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err
exit $rc
