#!/bin/bash
# Meta-update A/B: the meta / full-size / agent / checkpoint GPU tests on the
# default library, then tools/meta_bench.py (M = 100, both orders) on the
# default and on a variant library, interleaved.
# usage: bash tools/gpu_meta_ab.sh TAG VARIANT.so
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py tests/test_fullsize_gpu.py tests/test_agents_gpu.py tests/test_checkpoint_gpu.py -m gpu -q -rf --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
for r in 1 2; do
  timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_default_$r.json 2> $OUT/meta_default_$r.err
  DQZ_LIB=$PWD/$2 timeout -k 10 300 python tools/meta_bench.py --steps 100 > $OUT/meta_variant_$r.json 2> $OUT/meta_variant_$r.err
done
exit $rc
