#!/bin/bash
# Retry a gpurun call while the pool refuses it for infrastructure reasons only (exit 3: no box
# or slot free; or a "transient" status: box lost before the command ran).  A command that ran
# and failed is NOT retried.  usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 20); do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 120; continue; fi
  exit $rc
done
exit $rc
