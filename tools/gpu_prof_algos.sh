#!/bin/bash
# Kernel-trace profiles of configs 4 (PER) and 3 (MGSC learner part) at HEAD,
# and the config-1 agent loop's line.
set -eo pipefail
bash profiles/run_profile.sh r04_per --algo per
bash profiles/run_profile.sh r04_mgsc --algo mgsc
mkdir -p gpurun_out/agent_r04
timeout -k 10 300 python bench.py --algo agent --steps 2000 --warmup 50 > gpurun_out/agent_r04/bench_agent.json 2> gpurun_out/agent_r04/bench_agent.err
