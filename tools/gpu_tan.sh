#!/bin/bash
# MGSC tangent launch order A/B: meta / full-size GPU tests, then the M = 100
# meta-update against -DDQZ_TAN_FC1_FIRST=0 (three interleaved rounds) and a
# meta kernel trace.
set -o pipefail
OUT=gpurun_out/tan
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 400 python -u -m pytest tests/test_meta_gpu.py tests/test_fullsize_gpu.py tests/test_agents_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
for r in 1 2 3; do
  for V in libdqz libdqz_tan0; do
    DQZ_LIB=$PWD/$L/$V.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_${V}_$r.json 2> $OUT/meta_${V}_$r.err
    python -c "import json; d=json.load(open('$OUT/meta_${V}_$r.json')); print('$V', $r, {k[5:]: v['ms_per_step'] for k,v in d.items() if isinstance(v, dict)})" >> $OUT/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
