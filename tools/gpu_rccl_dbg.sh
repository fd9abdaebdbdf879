#!/bin/bash
# The RCCL-in-graph teardown modes of tools/dbg_rccl_capture.py (world 1): graph deleted before
# destroy_process_group ('del'), destroyed while the graph lives ('keep'), never destroyed
# ('nodestroy'), each with thread-local capture and 'del' / 'keep' also with global capture.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in del:thread_local keep:thread_local nodestroy:thread_local del:global keep:global; do
  m=${spec%%:*}; cm=${spec#*:}
  echo "== $m $cm"
  CAPMODE=$cm timeout -k 10 120 python tools/dbg_rccl_capture.py $m > gpurun_out/rccl_dbg_${m}_$cm.log 2>&1
  rc=$?; echo "rc=$rc"; grep -v "^\s*File\|Extension modules\|^frame #" gpurun_out/rccl_dbg_${m}_$cm.log | tail -8
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
done
exit 0
