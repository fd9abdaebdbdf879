#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in del keep nodestroy; do
  echo "== $m"
  timeout -k 10 120 python tools/dbg_rccl_capture.py $m > gpurun_out/rccl_dbg_$m.log 2>&1
  rc=$?; echo "rc=$rc"; grep -v "^\s*File\|Extension modules" gpurun_out/rccl_dbg_$m.log | tail -12
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
done
exit 0
