#!/bin/bash
# Instruction-cache counters of the learner step per build (code-layout
# study): one --pmc pass of SQC_ICACHE_MISSES / SQC_ICACHE_HITS
# over a 1,000-step default bench for libdqz_base.so and each variant.
# usage: bash tools/gpu_icache.sh TAG variant...
set -eo pipefail
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export DQZ_ALLOW_STALE=1
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $OUT/pmc_$v -o run -- python3 $ROOT/bench.py --steps 1000 --warmup 100 --cpu-seconds 0 --capacity 200000 > $OUT/bench_$v.json 2> $OUT/bench_$v.err
  echo "== $v" >> $OUT/summary.txt
  python3 - $OUT/pmc_$v/run_counter_collection.csv >> $OUT/summary.txt <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
  agg[r['Kernel_Name'].split('(')[0].replace('void ', '').replace('dqz::', '')[:32]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in sorted(agg.items()):
  m, h = c.get('SQC_ICACHE_MISSES', [0]), c.get('SQC_ICACHE_HITS', [0])
  if len(m) > 50:
    print('%-32s n %5d misses %9.1f hits %10.1f' % (k, len(m), sum(m) / len(m), sum(h) / len(h)))
PY
done
cat $OUT/summary.txt
