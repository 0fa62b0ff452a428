#!/bin/bash
# Re-submit a gpurun call while it is only refused for capacity / infrastructure
# (status=transient: nothing ran, nothing charged), waiting out the back-off
# gpurun names.  usage: GPURUN=/path/to/gpurun gpurun_retry.sh LOG TIMEOUT CMD
if [ -z "$GPURUN" ]; then
  echo "gpurun_retry.sh: set GPURUN to the gpurun client's path" >&2
  exit 2
fi
LOG=$1; TO=$2; shift 2
for i in $(seq 1 40); do
  "$GPURUN" --timeout $TO -- "$@" > $LOG 2>&1
  if grep -q "status=transient" $LOG; then
    w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-60} > 60 ? ${w:-60} + 10 : 70 ))
    continue
  fi
  break
done
tail -5 $LOG
