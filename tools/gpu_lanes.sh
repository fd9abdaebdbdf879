#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lanes" -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lanes.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_lanes.log
[ $rc -ne 0 ] && exit $rc
for cfg in "8 1" "8 2" "16 1" "16 2" "16 4"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --batch $1 --lanes $2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_lanes.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_lanes.log').read().strip().splitlines()[-1]);print('B=$1 lanes=$2', d['value'], d['us_per_denoise_step'])"
done
