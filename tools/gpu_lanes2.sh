#!/bin/bash
# Lane / batch sweep of the bench (frames/s and us per denoise step), no CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${LANE_CFGS:-"16 2" "32 2" "32 4" "24 3" "16 4" "64 4"}; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --batch $1 --lanes $2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_lanes.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_lanes.log').read().strip().splitlines()[-1]);print('B=$1 lanes=$2', d['value'], d['us_per_denoise_step'])"
done
