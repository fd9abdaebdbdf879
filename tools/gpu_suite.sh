#!/bin/bash
# The GPU suite (optionally the files in $FIRST first, stopping there on failure), errors logged.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MDG_PARITY_LOG=gpurun_out/parity_errors.jsonl
rm -f "$MDG_PARITY_LOG"
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_first.log 2>&1; rc=$?
  echo "first rc=$rc"; grep -E "PASSED|FAILED|ERROR|Error|assert" gpurun_out/pytest_first.log | head -30
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
exit $rc
