#!/bin/bash
# MGSC meta-update iteration on the GPU box: the meta / agent / full-size /
# checkpoint GPU tests, tools/meta_bench.py, and its kernel trace.
# usage: bash tools/gpu_meta.sh <tag>
set -o pipefail
TAG=${1:-meta}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py tests/test_agents_gpu.py tests/test_fullsize_gpu.py tests/test_checkpoint_gpu.py tests/test_learner_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_bench.json 2> $OUT/meta_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
exit $rc
