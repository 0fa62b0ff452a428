#!/bin/bash
# One A/B session on the GPU box: the full GPU suite at the working tree,
# then step traces and interleaved default benches (3 rounds, 20,000 steps,
# C = 200k) of libdqz_base.so against each named variant, PMC LDS passes of
# each, and the default / driver bench lines.  Variants are prebuilt from the
# same tree (tools/build_variants.sh); DQZ_ALLOW_STALE lets the A/B arms load.
# usage: bash tools/gpu_ab.sh TAG variant...
set -o pipefail
ROOT=$(pwd)
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver.err
timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench_default.json 2> $OUT/bench_default.err
export DQZ_ALLOW_STALE=1
for v in base "$@"; do
  if [ "$v" = base ]; then T=libdqz_trace.so; else T=libdqz_trace_$v.so; fi
  DQZ_TRACE_PREBUILT=1 DQZ_TRACE_LIB=$ROOT/dqn_mgsc_zoo_amd/$T timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_$v.txt 2>&1
done
for r in 1 2 3; do
  for v in base "$@"; do
    DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], {k: round(x*1e3,2) for k,x in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
  done
done
CTR="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/p_$v -o run -- \
    python3 $ROOT/bench.py --steps 200 --warmup 20 --graph 0 --cpu-seconds 0 --profile-iters 2 --capacity 200000 > $OUT/p_$v.json 2> $OUT/p_$v.err
done
cd $ROOT && timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_bench.json 2> $OUT/meta_bench.err
exit $rc
