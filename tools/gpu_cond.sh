#!/bin/bash
# Conditioning-precompute parity first (new kernels), then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cond.py -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cond.log 2>&1; rc=$?
echo "cond rc=$rc"; grep -E "PASSED|FAILED|ERROR|Error|assert" gpurun_out/pytest_cond.log | head -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
exit $rc
