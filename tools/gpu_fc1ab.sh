#!/bin/bash
# fc1 split / column-vector variants: GPU suite on the default library, the
# learner tests on each variant, then an interleaved A/B of the default bench.
set -o pipefail
OUT=gpurun_out/fc1ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for V in s14 s14j2 s7j2; do
  DQZ_LIB=$PWD/dqn_mgsc_zoo_amd/libdqz_$V.so timeout -k 10 300 python -u -m pytest tests/test_learner_gpu.py tests/test_meta_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests_$V.log 2>&1
  r=$?
  echo "pytest rc=$r" >> $OUT/tests_$V.log
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then exit $r; fi
done
set -e
bash tools/abv.sh 3 dqn_mgsc_zoo_amd/libdqz.so dqn_mgsc_zoo_amd/libdqz_s14.so dqn_mgsc_zoo_amd/libdqz_s14j2.so dqn_mgsc_zoo_amd/libdqz_s7j2.so > $OUT/abv.txt 2>&1
exit $rc
