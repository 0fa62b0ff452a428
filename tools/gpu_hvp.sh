#!/bin/bash
# HVP load batching: the GPU suite, the M = 100 meta-update (two runs) and a
# meta kernel trace.
set -o pipefail
OUT=gpurun_out/hvp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
for r in 1 2; do
  timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$r.json 2> $OUT/meta_$r.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
