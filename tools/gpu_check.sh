#!/bin/bash
# GPU-box check: smoke -> GPU tests -> short bench.  Every GPU step has its own time limit;
# a crash / timeout (exit codes other than 0 and pytest's 1 = "tests failed") stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
