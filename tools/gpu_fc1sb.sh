#!/bin/bash
# fc1 forward load order A/B: the GPU suite on the default library (loads
# issued before the first MFMA, two row groups per block at MG > 1), the
# default bench against -DDQZ_FC1_SB=0 (the compiler's interleaved order),
# the M = 100 meta-update against -DDQZ_FC1_SB=0 and -DDQZ_FC1_RG=1, and a
# meta kernel trace.
set -o pipefail
OUT=gpurun_out/fc1sb
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
bash tools/abv.sh 3 $L/libdqz.so $L/libdqz_sb0.so > $OUT/abv.txt 2>&1
for r in 1 2; do
  for V in libdqz libdqz_sb0 libdqz_rg1; do
    DQZ_LIB=$PWD/$L/$V.so timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_${V}_$r.json 2> $OUT/meta_${V}_$r.err
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/meta_bench.py --steps 50 --graph 0 > $GRAFT_REPO_ROOT/$OUT/meta_prof.json 2> $GRAFT_REPO_ROOT/$OUT/meta_prof.err
