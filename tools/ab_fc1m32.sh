#!/bin/bash
# fc1 forward on 32x32x2 MFMA (-DDQZ_FC1_32=1): learner / full-size /
# actor GPU tests against that library, then an interleaved A/B.
set -o pipefail
mkdir -p gpurun_out/fc1m32
DQZ_LIB=$PWD/dqn_mgsc_zoo_amd/libdqz_fc1m32.so timeout -k 10 400 python -u -m pytest -x -q -rf \
  --timeout 120 --timeout-method thread -m gpu \
  tests/test_learner_gpu.py tests/test_fullsize_gpu.py tests/test_actor_gpu.py \
  > gpurun_out/fc1m32/tests.log 2>&1 || exit $?
bash tools/abv.sh 3 dqn_mgsc_zoo_amd/libdqz.so dqn_mgsc_zoo_amd/libdqz_fc1m32.so > gpurun_out/fc1m32/ab.txt 2>&1
