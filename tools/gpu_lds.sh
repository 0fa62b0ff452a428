#!/bin/bash
# LDS bank-conflict attribution (one PMC pass per library, eager launches):
# the working tree (base), its variants, and the round-3 tree (abtrees/r03,
# its own sources, build and bench.py); then interleaved benches of base and
# noperm.  usage: bash tools/gpu_lds.sh TAG variant...
set -eo pipefail
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export DQZ_ALLOW_STALE=1
CTR="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  DQZ_LIB=$ROOT/dqn_mgsc_zoo_amd/libdqz_$v.so timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/p_$v -o run -- \
    python3 $ROOT/bench.py --steps 200 --warmup 20 --graph 0 --cpu-seconds 0 --profile-iters 2 --capacity 200000 > $OUT/p_$v.json 2> $OUT/p_$v.err
done
if [ -d $ROOT/abtrees/r03 ]; then
  cd $ROOT/abtrees/r03
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/p_r03 -o run -- \
    python3 bench.py --steps 200 --warmup 20 --graph 0 --cpu-seconds 0 --profile-iters 2 --capacity 200000 > $OUT/p_r03.json 2> $OUT/p_r03.err
fi
