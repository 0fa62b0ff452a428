#!/bin/bash
# HEAD check: GPU suite, smoke, default bench, M = 100 meta-update (two runs)
# and a meta kernel trace.
set -o pipefail
OUT=gpurun_out/check5
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err
for r in 1 2; do
  timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$r.json 2> $OUT/meta_$r.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
