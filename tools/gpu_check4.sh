#!/bin/bash
# Round-4 GPU check: full GPU suite, smoke, the driver's bench command, the
# default bench, config 1 (agent loop), a Z=1 forward probe under rocprof.
# Test failures (rc 1) do not stop the rest; any other failure does.
# usage: bash tools/gpu_check4.sh <tag>
set -o pipefail
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python bench.py --algo agent --steps 2000 --warmup 50 > $OUT/bench_agent.json 2> $OUT/bench_agent.err
timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_bench.json 2> $OUT/meta_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/z1 -o run -- python3 $GRAFT_REPO_ROOT/tools/z1_probe.py > $GRAFT_REPO_ROOT/$OUT/z1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/meta -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
exit $rc
