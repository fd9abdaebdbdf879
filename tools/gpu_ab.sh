#!/bin/bash
# Same-box A/B of two builds of the library: the tree's libmdgen_hip.so vs build/ab/old.so
# (MDG_LIB_PATH), alternating: correctness of the new build's kernels first (AB_TESTS, a
# pytest -k filter), then the AB_MODE microbench (tools/gemm_bench.py) and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "$AB_TESTS" -q -x \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 gpurun_out/pytest_ab.log
  [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export MDG_LIB_PATH=$PWD/build/ab/old.so; else unset MDG_LIB_PATH; fi
    echo "== $L"
    timeout -k 10 100 python tools/gemm_bench.py ${AB_MODE:-rowln} 2>&1 | grep -E "mdg|spa M|final M" | cut -c1-90
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --sweep-batches "" --no-f32-line \
      > gpurun_out/bench_ab.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['us_per_denoise_step'], [r['avg_launch_us'] for r in [d['roofline']]+d['roofline_more']])"
  done
done
