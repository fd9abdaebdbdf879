#!/bin/bash
# Same-box A/B of one build under an environment knob: AB_ENV (e.g. MDG_PACKED_PLANES=0) vs
# default, alternating, bench only (+ the AB_MODE GEMM microbench when set).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for L in new old; do
    echo "== $L"
    if [ $L = old ]; then ENVSET="env $AB_ENV"; else ENVSET="env"; fi
    $ENVSET timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --sweep-batches "" --no-f32-line \
      > gpurun_out/bench_ab.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['us_per_denoise_step'], [r['avg_launch_us'] for r in [d['roofline']]+d['roofline_more']])"
  done
done
