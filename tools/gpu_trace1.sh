#!/bin/bash
# Step traces of the one-sample learner (the MGSC theta' pass's shape) with
# the fused forward (libdqz_trace.so) and without (libdqz_trace_nofuse.so),
# and of the default B = 32 step.
set -eo pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/t1
mkdir -p $OUT
export DQZ_TRACE_PREBUILT=1
for v in trace trace_nofuse; do
  BATCH=1 DQZ_TRACE_LIB=$ROOT/dqn_mgsc_zoo_amd/lib$( [ $v = trace ] && echo dqz_trace || echo dqz_$v ).so timeout -k 10 200 python -u tools/trace_step.py > $OUT/b1_$v.txt 2>&1
done
timeout -k 10 200 python -u tools/trace_step.py > $OUT/b32_trace.txt 2>&1
