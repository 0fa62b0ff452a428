#!/bin/bash
# A/B session against one prebuilt variant: the full GPU suite at the working
# tree, interleaved learner benches (3 rounds) and meta-update benches (2
# rounds) of libdqz_base.so against libdqz_<variant>.so, then a kernel trace
# of the base meta-update.
# usage: bash tools/gpu_ab2.sh TAG variant
set -o pipefail
ROOT=$(pwd)
TAG=$1; V=$2
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
export DQZ_ALLOW_STALE=1
for r in 1 2 3; do
  for v in base $V; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], d['handoff_status'])" | tee -a $OUT/summary.txt
  done
done
for r in 1 2; do
  for v in base $V; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_${v}_$r.json 2> $OUT/meta_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/meta_${v}_$r.json')); print('$v', $r, {k: round(1e3*x['ms_per_step'],1) for k,x in d.items() if k.startswith('meta')})" | tee -a $OUT/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp
DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/metaprof -o run -- python3 $ROOT/tools/meta_bench.py --steps 50 --graph 0 > $OUT/meta_prof.json 2> $OUT/meta_prof.err
exit 0
