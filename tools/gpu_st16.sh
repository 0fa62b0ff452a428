#!/bin/bash
# conv2 forward's y2 hand-off store width A/B: the GPU suite on the default
# library (16-byte write-through stores), the default bench against
# -DDQZ_C2F_ST16=0 (4-byte), and a step trace.
set -o pipefail
OUT=gpurun_out/st16
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 $L/libdqz.so $L/libdqz_st4.so > $OUT/abv.txt 2>&1
DQZ_TRACE_PREBUILT=1 timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
# the sampler load batching (PER tree top, learned-logit chunk sums): configs 4 and 3
timeout -k 10 300 python bench.py --algo per --cpu-seconds 0 > $OUT/bench_per.json 2> $OUT/bench_per.err
timeout -k 10 300 python bench.py --algo mgsc --cpu-seconds 0 > $OUT/bench_mgsc.json 2> $OUT/bench_mgsc.err
timeout -k 10 300 python bench.py --algo agent --steps 2000 --warmup 50 > $OUT/bench_agent.json 2> $OUT/bench_agent.err
