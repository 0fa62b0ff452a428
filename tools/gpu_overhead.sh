#!/bin/bash
# Fixed cost of the driver's 20-step timed region (tools/overhead_probe.py),
# then a quick GPU-suite / smoke check of HEAD.
set -o pipefail
OUT=gpurun_out/overhead
mkdir -p $OUT
timeout -k 10 300 python tools/overhead_probe.py > $OUT/probe.json 2> $OUT/probe.err || exit $?
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
exit $rc
