#!/bin/bash
# Round-3 evidence on the GPU box: GPU tests, the driver's bench command, the
# default bench, per / mgsc config benches, kernel-trace profiles of dqn /
# per / mgsc, PMC passes (dqn), config timings, a step trace.  Every GPU step
# has its own time limit; test failures (rc 1) do not stop the rest, any
# other failure does.
# usage: bash tools/round_evidence3.sh <tag>
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
for A in per mgsc; do
  timeout -k 10 300 python bench.py --algo $A > $OUT/bench_$A.json 2> $OUT/bench_$A.err
done
bash profiles/run_profile.sh ${TAG}_dqn
bash profiles/run_profile.sh ${TAG}_per --algo per
bash profiles/run_profile.sh ${TAG}_mgsc --algo mgsc
bash profiles/run_pmc.sh $TAG
timeout -k 10 300 python tools/bench_configs.py > $OUT/configs.json 2> $OUT/configs.err
timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
exit $rc
