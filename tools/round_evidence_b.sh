#!/bin/bash
# A round's evidence on the GPU box, part B (after round_evidence_a.sh): the
# MGSC meta-update bench and its kernel trace, a kernel-trace profile of the
# default bench, the four PMC passes and a step trace of the trace build.
# usage: bash tools/round_evidence_b.sh <tag>
set -eo pipefail
TAG=${1:-r06}
ROOT=$(pwd)
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_bench.json 2> $OUT/meta_bench.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/metaprof -o run -- \
  python3 $ROOT/tools/meta_bench.py --steps 50 --graph 0 > $ROOT/$OUT/meta_prof.json 2> $ROOT/$OUT/meta_prof.err)
bash profiles/run_profile.sh ${TAG}_dqn
bash profiles/run_pmc.sh $TAG
DQZ_TRACE_PREBUILT=1 timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
