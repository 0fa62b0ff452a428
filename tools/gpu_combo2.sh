#!/bin/bash
# fc1 load order / backward grid order A/B (interleaved benches + traces),
# meta tests + meta bench at HEAD, config 1 at the reference schedule, a
# kernel trace of the meta-update.  Variant runs load prebuilt libraries
# (DQZ_ALLOW_STALE=1: the arms were built together from one tree).
set -eo pipefail
OUT=gpurun_out/c2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py tests/test_fullsize_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests_meta.log 2>&1 || true
export DQZ_ALLOW_STALE=1
for v in 0 noperm fc1wf fc1last; do
  if [ "$v" = 0 ]; then T=dqn_mgsc_zoo_amd/libdqz_trace.so; else T=dqn_mgsc_zoo_amd/libdqz_trace_$v.so; fi
  DQZ_TRACE_PREBUILT=1 DQZ_TRACE_LIB=$PWD/$T timeout -k 10 200 python -u tools/trace_step.py > $OUT/trace_$v.txt 2>&1
done
for r in 1 2 3; do
  for v in base noperm fc1wf fc1last; do
    L=dqn_mgsc_zoo_amd/libdqz_$v.so
    DQZ_LIB=$PWD/$L timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 --capacity 200000 > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, d['value'], {k: round(x*1e3,2) for k,x in d['phase_ms'].items()})" | tee -a $OUT/summary.txt
  done
done
DQZ_LIB=$PWD/dqn_mgsc_zoo_amd/libdqz_base.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_bench.json 2> $OUT/meta_bench.err
DQZ_LIB=$PWD/dqn_mgsc_zoo_amd/libdqz_base.so timeout -k 10 400 python bench.py --algo agent --steps 5000 --warmup 50 > $OUT/bench_agent_refsched.json 2> $OUT/bench_agent_refsched.err
cd /tmp && export TMPDIR=/tmp
DQZ_LIB=$GRAFT_REPO_ROOT/dqn_mgsc_zoo_amd/libdqz_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/metaprof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
bash tools/gpu_lds.sh lds noperm
