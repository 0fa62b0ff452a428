#!/bin/bash
# Working tree against committed sources (usage: gpu_headtd.sh [out tag]):
# libdqz.so is the working tree, libdqz_oldhead.so the committed version of
# the edited files built beforehand with the working tree's build id.  GPU
# suite on the default library first, then three interleaved bench rounds,
# a step trace and the config 4 / 3 lines.  (Used for the head TD, head
# wave-partial, head DPP and fc1 dX 8-wave A/Bs of round 4.)
set -o pipefail
OUT=gpurun_out/${1:-headtd}
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 $L/libdqz.so $L/libdqz_oldhead.so > $OUT/abv.txt 2>&1
DQZ_TRACE_PREBUILT=1 timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
timeout -k 10 300 python bench.py --algo per --cpu-seconds 0 > $OUT/bench_per.json 2> $OUT/bench_per.err
timeout -k 10 300 python bench.py --algo mgsc --cpu-seconds 0 > $OUT/bench_mgsc.json 2> $OUT/bench_mgsc.err
