#!/bin/bash
# Re-submit a gpurun call only while the infrastructure reports it as transient (no box / box
# not prepared: nothing ran, nothing charged).  Any real result, success or failure, ends it.
LOG=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" || [ $rc -eq 3 ]; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
