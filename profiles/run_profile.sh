#!/bin/bash
# Kernel-trace profile of the default bench config (run on the GPU box from the repo root).
# usage: bash profiles/run_profile.sh <tag> [extra bench args]
set -eo pipefail
TAG=${1:-r01}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --steps 1000 --warmup 100 --cpu-seconds 0 --profile-iters 20 "$@" \
  > "$OUT/bench.json" 2> "$OUT/bench.err"
