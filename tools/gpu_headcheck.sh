#!/bin/bash
# Short check of the library at HEAD: smoke, the driver's bench command, the
# default bench and config 4.
set -eo pipefail
OUT=gpurun_out/headcheck
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python bench.py --algo per --cpu-seconds 0 > $OUT/bench_per.json 2> $OUT/bench_per.err
tail -2 $OUT/smoke.log
