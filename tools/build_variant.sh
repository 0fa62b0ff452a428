#!/bin/bash
# Build a libdqz variant with extra -D flags: bash tools/build_variant.sh NAME [flags...]
set -e
N=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC "$@" -Iinclude \
  -o dqn_mgsc_zoo_amd/libdqz_$N.so dqn_mgsc_zoo_amd/csrc/learner.hip
