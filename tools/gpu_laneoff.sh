#!/bin/bash
# Lane phase-offset A/B (MDG_LANE_OFFSET = layers of lane k-1's first step before lane k starts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lanes" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lanes.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_lanes.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for O in ${OFFSETS:-0 1 2 3}; do
  MDG_LANE_OFFSET=$O timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_off.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_off.log').read().strip().splitlines()[-1]);print('offset=$O', d['value'], d['us_per_denoise_step'])"
done
done
