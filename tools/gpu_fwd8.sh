#!/bin/bash
# 8-job conv2 / conv3 forward for small launches: the GPU suite on the
# default library (8 jobs at Z B <= 16), the learner / actor / meta tests on
# the all-8-job build, an interleaved A/B of the default bench (4 jobs at 64
# samples) against all-8, the M = 100 meta-update and the config-1 agent
# loop against the all-4-job build, and a meta kernel trace.
set -o pipefail
OUT=gpurun_out/fwd8
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
DQZ_LIB=$PWD/$L/libdqz_fwd8all.so timeout -k 10 300 python -u -m pytest tests/test_learner_gpu.py tests/test_actor_gpu.py tests/test_meta_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests_fwd8all.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests_fwd8all.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 $L/libdqz.so $L/libdqz_fwd8all.so > $OUT/abv.txt 2>&1
for r in 1 2; do
  for V in libdqz libdqz_fwd4all; do
    DQZ_LIB=$PWD/$L/$V.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_${V}_$r.json 2> $OUT/meta_${V}_$r.err
    DQZ_LIB=$PWD/$L/$V.so timeout -k 10 300 python bench.py --algo agent --steps 1000 --warmup 50 > $OUT/agent_${V}_$r.json 2> $OUT/agent_${V}_$r.err
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
