#!/bin/bash
# The tail of tools/round_evidence.sh: config benches, step trace, logit add bench.
set -eo pipefail
TAG=${1:-r02}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_samplers_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/samplers.log 2>&1
timeout -k 10 300 python tools/bench_configs.py > $OUT/configs.json 2> $OUT/configs.err
timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
timeout -k 10 200 python tools/logit_add_bench.py > $OUT/logit_add.json 2>&1
