#!/bin/bash
# Batch x lanes sweep of the headline window (bench lines only, no baselines / extra lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SWEEP=${SWEEP:-16:2 24:2 24:3 32:2 32:4 48:3}
for cfg in $SWEEP; do
  b=${cfg%%:*}; l=${cfg##*:}
  timeout -k 10 300 python -u bench.py --batch $b --lanes $l --steps 3 --warmup 1 --no-cpu-baseline --sweep-batches "" \
    --no-f32-line > gpurun_out/bench_b${b}_l$l.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_b${b}_l$l.log').read().strip().splitlines()[-1]);print('B=$b lanes=$l', d['value'], d['us_per_denoise_step'])"
done
