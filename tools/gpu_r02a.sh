#!/bin/bash
# Round-2 check on one box: GPU tests (errors logged per comparison), then the bench with its
# batch sweep / f32 line.  A test FAILURE (exit 1) still runs the bench; a timeout, abort or
# crash of the test run stops the script (no further GPU work after a fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MDG_PARITY_LOG=gpurun_out/parity_errors.jsonl
rm -f "$MDG_PARITY_LOG"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -c 3000 gpurun_out/bench.log
exit $brc
