#!/bin/bash
# fc1 copy pairing for Z = 3 (double-Q / PER): the learner / full-size GPU
# tests, then interleaved PER and DQN benches against -DDQZ_FC1_PAIR=0.
set -o pipefail
OUT=gpurun_out/pair
mkdir -p $OUT
L=dqn_mgsc_zoo_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
set -e
for r in 1 2 3; do
  for V in libdqz libdqz_pair0; do
    DQZ_LIB=$PWD/$L/$V.so timeout -k 10 200 python bench.py --algo per --steps 20000 --warmup 500 --cpu-seconds 0 > $OUT/per_${V}_$r.json 2> $OUT/per_${V}_$r.err
    python -c "import json; d=json.load(open('$OUT/per_${V}_$r.json')); print('per $V $r', d['value'], {k: round(v*1e3,2) for k,v in d['phase_ms'].items()})" >> $OUT/ab.txt
  done
done
bash tools/abv.sh 2 $L/libdqz.so $L/libdqz_pair0.so >> $OUT/ab.txt 2>&1
