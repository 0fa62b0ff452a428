#!/bin/bash
# PMC counter passes (separate runs; no tracing flags combined with --pmc).
# usage: bash profiles/run_pmc.sh <tag>
set -eo pipefail
TAG=${1:-pmc}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_F32" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 200 --warmup 20 --graph 0 --cpu-seconds 0 --profile-iters 2 \
    > "$OUT/p$i.json" 2> "$OUT/p$i.err"
done
