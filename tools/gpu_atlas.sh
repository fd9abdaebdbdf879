#!/bin/bash
# ATLAS long-residue path: parity tests, then a short bench at T=250 L=256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "long_residue or padded" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_atlas.log 2>&1; rc=$?
echo "atlas tests rc=$rc"; tail -12 gpurun_out/pytest_atlas.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --frames 250 --crop 256 --batch 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_atlas.log 2>&1; rc=$?
echo "atlas bench rc=$rc"; tail -2 gpurun_out/bench_atlas.log
exit $rc
