#!/bin/bash
# Round-4 kernel A/B: the GPU suite on the default library, an interleaved
# A/B of the default bench against -DDQZ_FC1_XCD=0 (fc1 W1 slices without the
# XCD-matched placement) and -DDQZ_C2F_JOBS=4 (conv2 forward as 4 channel-
# quarter jobs per sample), the M = 100 meta-update against
# -DDQZ_FC1_MGLOOP=0 (one block per fc1 row group), and a meta kernel trace.
set -o pipefail
OUT=gpurun_out/xcdab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 dqn_mgsc_zoo_amd/libdqz.so dqn_mgsc_zoo_amd/libdqz_noxcd.so dqn_mgsc_zoo_amd/libdqz_c2x4.so > $OUT/abv.txt 2>&1
for r in 1 2; do
  for V in libdqz libdqz_nomg; do
    DQZ_LIB=$PWD/dqn_mgsc_zoo_amd/$V.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_${V}_$r.json 2> $OUT/meta_${V}_$r.err
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
