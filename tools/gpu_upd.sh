#!/bin/bash
# update-kernel load batching: the GPU suite, three default-bench runs, the
# M = 100 meta-update, and a kernel trace of the default bench.
set -o pipefail
OUT=gpurun_out/upd
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 dqn_mgsc_zoo_amd/libdqz.so > $OUT/abv.txt 2>&1
for r in 1 2; do
  timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_$r.json 2> $OUT/meta_$r.err
done
bash profiles/run_profile.sh upd_dqn
DQZ_TRACE_PREBUILT=1 timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_step.txt 2>&1
