#!/bin/bash
# Round-5 session call: meta-update slab-dot A/B, then the backward-launch
# skip sensitivity (timing-only variants).
set -o pipefail
bash tools/gpu_meta_ab.sh metaab dqn_mgsc_zoo_amd/libdqz_metaold.so
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OUT=gpurun_out/skip
mkdir -p $OUT
for v in 0 1 6 8 15; do
  if [ "$v" = 0 ]; then T=dqn_mgsc_zoo_amd/libdqz_trace.so; else T=dqn_mgsc_zoo_amd/libdqz_trace_s$v.so; fi
  DQZ_TRACE_PREBUILT=1 DQZ_TRACE_LIB=$PWD/$T timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_$v.txt 2>&1 || exit 5
done
for v in 0 1 6 8 15; do
  if [ "$v" = 0 ]; then L=dqn_mgsc_zoo_amd/libdqz.so; else L=dqn_mgsc_zoo_amd/libdqz_s$v.so; fi
  DQZ_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit 6
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value'], {k: round(x*1e3,2) for k,x in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
done
exit $rc
