#!/bin/bash
# Rebuild libdqz.so and the named -D variants from the current sources (all
# carry the same build id, so the loader accepts each).  usage:
#   bash tools/build_variants.sh name1 "FLAGS1" name2 "FLAGS2" ...
# builds dqn_mgsc_zoo_amd/libdqz_<name>.so; a name starting with trace_ gets -DDQZ_TRACE too.
set -e
python -c "import __graft_entry__ as g; g.build()" | tail -1
python -c "import __graft_entry__ as g; g._compile_lib('dqn_mgsc_zoo_amd/libdqz_trace.so', ['-DDQZ_TRACE'])" &
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  ex=""; case $n in trace_*) ex="-DDQZ_TRACE";; esac
  python -c "import sys, __graft_entry__ as g; g._compile_lib('dqn_mgsc_zoo_amd/libdqz_$n.so', sys.argv[1:])" $ex $f &
done
wait
