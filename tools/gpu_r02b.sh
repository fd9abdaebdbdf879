#!/bin/bash
# Training-path GPU tests (layer backward vs eager autograd, loss + grads vs the oracle) and the
# engine / rollout tests, errors logged; stops at a crash or timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MDG_PARITY_LOG=gpurun_out/parity_train.jsonl
rm -f "$MDG_PARITY_LOG"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_engine.py tests/test_gpu_geometry.py \
  -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_train.log | sed 's/.*:://' | head -60
cat "$MDG_PARITY_LOG" 2>/dev/null
exit $rc
