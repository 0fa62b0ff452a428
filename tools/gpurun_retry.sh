#!/bin/bash
# Re-submit a gpurun call while it is only refused for capacity / infrastructure
# (status=transient: nothing ran, nothing charged).  usage: gpurun_retry.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  if grep -q "status=transient" $LOG; then sleep 90; continue; fi
  break
done
tail -5 $LOG
