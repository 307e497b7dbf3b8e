#!/bin/bash
# queue a gpurun call: retry only while no box/slot was available (rc 3 or a transient
# status before the command ran); any other outcome is final
log=$1; shift
for i in $(seq 1 200); do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then sleep 90; continue; fi
  echo "rc=$rc" >> "$log"; exit $rc
done
