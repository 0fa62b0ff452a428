#!/bin/bash
# A round's evidence on the GPU box, part A: GPU suite, smoke, the driver's
# bench command, the default bench, configs 4 / 3 / 1 and SURVEY §8(d)'s
# median of five 10,000-step runs.  Part B (round_evidence_b.sh): the
# meta-update bench and its kernel trace, the step's kernel trace, the four
# PMC passes and a step trace.  Test failures (rc 1) do not stop the rest.
# usage: bash tools/round_evidence_a.sh <tag>
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python bench.py --algo per --cpu-seconds 0 > $OUT/bench_per.json 2> $OUT/bench_per.err
timeout -k 10 300 python bench.py --algo mgsc --cpu-seconds 0 > $OUT/bench_mgsc.json 2> $OUT/bench_mgsc.err
timeout -k 10 300 python bench.py --algo agent --steps 2000 --warmup 50 > $OUT/bench_agent.json 2> $OUT/bench_agent.err
bash tools/bench_median.sh $OUT/median > $OUT/bench_median5.json
exit $rc
