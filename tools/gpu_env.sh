#!/bin/bash
# HIP runtime settings A/B on the default bench (20,000 steps, interleaved):
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) and graph packet
# capture (DEBUG_CLR_GRAPH_PACKET_CAPTURE), against the runtime's defaults.
set -eo pipefail
OUT=gpurun_out/env
mkdir -p $OUT
run() {  # name, env assignments...
  local n=$1 r=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --steps 20000 --warmup 500 --cpu-seconds 0 \
    > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err
  python -c "import json; d=json.load(open('$OUT/${n}_$r.json')); print('$n', $r, d['value'], {k: round(v*1e3,2) for k,v in d['phase_ms'].items()})"
}
for r in 1 2 3; do
  run base $r DQZ_ENV_AB=base
  run devk1 $r HIP_FORCE_DEV_KERNARG=1
  run devk0 $r HIP_FORCE_DEV_KERNARG=0
  run gpc0 $r DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
done
# the driver's short command under the candidate settings
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/drv_base_$r.json 2> /dev/null
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/drv_devk1_$r.json 2> /dev/null
  python -c "import json; print('drv', $r, json.load(open('$OUT/drv_base_$r.json'))['value'], json.load(open('$OUT/drv_devk1_$r.json'))['value'])"
done
