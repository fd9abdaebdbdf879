#!/bin/bash
# Small-M split MLP (MDG_MLP_SPLIT): GPU parity suite with it on, then B=1 / TPS lines on vs off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "${SKIP_SUITE:-}" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_split.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 gpurun_out/pytest_split.log
[ $rc -ne 0 ] && exit $rc
line() {  # $1 = env, rest = bench args
  local env=$1; shift
  env $env timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --sweep-batches "" --no-f32-line "$@" \
    > gpurun_out/bench_split.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/bench_split.log').read().strip().splitlines()[-1]);print('$env', '$*', d['value'], d['us_per_denoise_step'])"
}
for rep in 1 2; do
  for e in MDG_X=1 MDG_MLP_SPLIT_BLOCKS=160 MDG_MLP_SPLIT_BLOCKS=400; do
    line $e --batch 1 --lanes 1
    line $e --tps --frames 100 --batch 16
  done
done
