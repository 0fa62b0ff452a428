#!/bin/bash
# GPU check on the box: full GPU test suite, the driver's bench command, the default bench, a step trace.
# Test failures (pytest rc 1) do not stop the benches; any other failure (fault, abort, time limit) does.
# usage: bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
for A in per mgsc; do
  timeout -k 10 200 python bench.py --algo $A --steps 2000 --warmup 100 --cpu-seconds 0 > $OUT/bench_$A.json 2> $OUT/bench_$A.err
done
timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
exit $rc
