#!/bin/bash
# B=8 (two lanes of 125 row tiles: just under the small-M threshold) with and without the small-M routes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for e in MDG_X=1 MDG_MLP_SPLIT=0; do
    env $e timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --sweep-batches "" --no-f32-line --batch 8 \
      > gpurun_out/bench_b8.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/bench_b8.log').read().strip().splitlines()[-1]);print('$e', d['value'], d['us_per_denoise_step'], d['kernel_plan']['mlp'][:30], d['kernel_plan']['temporal'][:20])"
  done
done
