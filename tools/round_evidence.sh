#!/bin/bash
# Round evidence on the GPU box: GPU tests, the driver's bench command, the
# default bench, a kernel-trace profile, PMC passes, config benches, a step
# trace.  Each GPU step has its own time limit; a failure stops the script.
# usage: bash tools/round_evidence.sh <tag>
set -eo pipefail
TAG=${1:-r02}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
bash profiles/run_profile.sh $TAG
bash profiles/run_pmc.sh $TAG
timeout -k 10 300 python tools/bench_configs.py > $OUT/configs.json 2> $OUT/configs.err
timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
timeout -k 10 200 python tools/logit_add_bench.py > $OUT/logit_add.json 2>&1
