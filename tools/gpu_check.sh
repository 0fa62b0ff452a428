#!/bin/bash
# GPU check on the box: full GPU test suite, the driver's bench command, the default bench, a step trace.
# usage: bash tools/gpu_check.sh <tag>
set -eo pipefail
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
