#!/bin/bash
# HEAD check on the GPU box: the full GPU suite, smoke, the driver's bench
# command and the default bench line.
# usage: bash tools/gpu_check.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err
exit $rc
