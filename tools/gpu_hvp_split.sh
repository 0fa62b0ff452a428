#!/bin/bash
# Where the HVP launches' time goes: a kernel trace of second-order
# meta-updates for libdqz_base.so and each timing-only skip build
# (DQZ_EXP_HVP_SKIP, hvp.hpp), one rocprofv3 run each.
# usage: bash tools/gpu_hvp_split.sh TAG variant...
set -eo pipefail
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export DQZ_ALLOW_STALE=1
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 $ROOT/tools/meta_bench.py --steps 40 --graph 0 --orders 1 > $OUT/prof_$v.json 2> $OUT/prof_$v.err
  echo "== $v" >> $OUT/summary.txt
  python3 $ROOT/tools/kernel_split.py $OUT/prof_$v/run_kernel_trace.csv hvp >> $OUT/summary.txt
done
cat $OUT/summary.txt
