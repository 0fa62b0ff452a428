#!/bin/bash
# Full GPU suite at the working tree, meta bench, default + driver bench,
# then the LDS-conflict PMC passes (base, noperm, round-3 tree).
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/c3
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_bench.json 2> $OUT/meta_bench.err
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err
bash $ROOT/tools/gpu_lds.sh c3/lds noperm
exit $rc
