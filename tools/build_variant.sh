#!/bin/bash
# Build a libdqz variant with extra -D flags: bash tools/build_variant.sh NAME [flags...]
# (same sources and build id as libdqz.so; only the -D flags differ)
set -e
N=$1; shift
python -c "import sys, __graft_entry__ as g; g._compile_lib('dqn_mgsc_zoo_amd/libdqz_$N.so', sys.argv[1:])" "$@"
