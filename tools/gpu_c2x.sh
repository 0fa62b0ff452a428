#!/bin/bash
# conv2 dX job count A/B: the GPU suite on the default library (16 jobs),
# the learner tests on -DDQZ_C2X_JOBS=8, an interleaved A/B of the default
# bench, and a step trace of the default build.
set -o pipefail
OUT=gpurun_out/c2x
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
DQZ_LIB=$PWD/$L/libdqz_c2x8.so timeout -k 10 300 python -u -m pytest tests/test_learner_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests_c2x8.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests_c2x8.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 $L/libdqz.so $L/libdqz_c2x8.so > $OUT/abv.txt 2>&1
DQZ_TRACE_PREBUILT=1 timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
