#!/bin/bash
# A/B on the GPU box: learner GPU tests, bench with the env toggle on/off, trace.
# usage: bash tools/ab.sh VAR  (VAR=1 vs VAR=0 benches)
set -eo pipefail
VAR=${1:-DQZ_FUSED_FWD}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_learner_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
env $VAR=1 timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/bench_on.json 2> gpurun_out/b.err
env $VAR=0 timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/bench_off.json 2>> gpurun_out/b.err
env $VAR=1 timeout -k 10 200 python -u tools/trace_step.py > gpurun_out/trace.txt 2>&1
