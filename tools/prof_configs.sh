set -eo pipefail
ROOT=$(pwd)
mkdir -p $ROOT/gpurun_out/prof_cfg
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_cfg -o run -- python3 $ROOT/tools/bench_configs.py --steps 500 > $ROOT/gpurun_out/prof_cfg/out.json 2> $ROOT/gpurun_out/prof_cfg/err.txt
