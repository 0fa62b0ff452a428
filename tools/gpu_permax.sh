#!/bin/bash
# PER head A/B: the working tree (IS-weight batch max on DPP) against
# libdqz_oldhead.so (committed head.hpp, working tree's build id), config 4
# bench lines interleaved, after the GPU suite on the default library.
set -o pipefail
OUT=gpurun_out/permax
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
for r in 1 2 3; do
  for lib in libdqz libdqz_oldhead; do
    DQZ_LIB=$PWD/$L/$lib.so timeout -k 10 200 python bench.py --algo per --steps 20000 --warmup 500 --cpu-seconds 0 \
      > $OUT/${lib}_$r.json 2> $OUT/${lib}_$r.err
    python -c "import json; d=json.load(open('$OUT/${lib}_$r.json')); print('$lib', $r, d['value'], {k: round(v*1e3,2) for k,v in d['phase_ms'].items()})" >> $OUT/abv.txt
  done
done
cat $OUT/abv.txt
