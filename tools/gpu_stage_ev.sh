#!/bin/bash
# Scheduling-barrier A/B (the default bench against -DDQZ_STAGE_SB=0 and
# -DDQZ_FC1_SB=0, the M = 100 meta-update), then the round-4 evidence.
set -o pipefail
OUT=gpurun_out/stage
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
bash tools/abv.sh 3 $L/libdqz.so $L/libdqz_stage0.so $L/libdqz_sb0.so > $OUT/abv.txt 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$r.json 2> $OUT/meta_$r.err || exit $?
done
bash tools/round_evidence4.sh r04
