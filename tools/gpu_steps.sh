#!/bin/bash
# Run GPU steps in order, each under its own time limit; an ordinary failure (exit 1, e.g. a
# failing test) is recorded and the next step runs, but a time-limit kill, abort or crash
# (124, 137, 134, 139, or any exit >= 128) ends the script there.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rcall=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping: $name ended with $rc"; exit $rc; fi
  [ $rc -ne 0 ] && rcall=$rc
done
exit $rcall
