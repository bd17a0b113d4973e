#!/bin/bash
# Local-side wrapper: re-submit a gpurun call only when the pool reports an infrastructure failure before the
# command ran (status=transient / backing off / no box free: nothing ran, nothing charged).  A command that ran
# and failed is never re-submitted.   tools/gpurun_retry.sh TIMEOUT -- CMD...
T=$1; shift; [ "$1" = "--" ] && shift
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -5
  if echo "$out" | grep -q "status=transient\|backing off\|no box\|slot free"; then sleep $((30 * i)); continue; fi
  exit $rc
done
exit $rc
