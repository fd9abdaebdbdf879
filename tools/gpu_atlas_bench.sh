#!/bin/bash
# ATLAS shape (BASELINE config 5: T=250, crop 256, B=1): HBM-traffic PMC passes of the roofline
# kernels at that shape, then the bench line with its CPU baseline (traffic read from
# profiles/traffic_r02.json, so merge the PMC result first: make_profiles.py 02 1 250 256).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${ATLAS_PMC:-1}" = 1 ]; then
  ROOF_ARGS="1 250 256" bash tools/roof_pmc.sh || exit $?
fi
timeout -k 10 400 python -u bench.py --frames 250 --crop 256 --batch 1 --lanes 1 --steps 3 --warmup 1 \
  --sweep-batches "" --no-f32-line --cpu-seconds 20 > gpurun_out/bench_atlas.log 2>&1; rc=$?
echo "atlas bench rc=$rc"; tail -1 gpurun_out/bench_atlas.log | cut -c1-400
exit $rc
