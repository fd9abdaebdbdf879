#!/bin/bash
# Same-box A/B of one build under an environment knob: AB_ENV (e.g. MDG_PACKED_PLANES=0) vs
# default, alternating.  AB_TESTS (a pytest -k filter) first runs the kernel/parity tests with
# AB_ENV set; AB_MODE adds the tools/gemm_bench.py microbench to each leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${AB_TESTS:-}" ]; then
  env $AB_ENV timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "$AB_TESTS" \
    -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 gpurun_out/pytest_ab.log
  [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for L in new old; do
    echo "== $L"
    if [ $L = old ]; then ENVSET="env $AB_ENV"; else ENVSET="env"; fi
    if [ -n "${AB_MODE:-}" ]; then
      $ENVSET timeout -k 10 100 python tools/gemm_bench.py $AB_MODE > gpurun_out/gemm_ab.log 2>&1 || exit $?
      grep -E "mdg|spa M|final M" gpurun_out/gemm_ab.log | cut -c1-90
    fi
    $ENVSET timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --sweep-batches "" --no-f32-line \
      > gpurun_out/bench_ab.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['us_per_denoise_step'], [r['avg_launch_us'] for r in [d['roofline']]+d['roofline_more']])"
  done
done
