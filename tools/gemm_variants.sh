#!/bin/bash
# GEMM microbench for each tile variant (MDG_GEMM_TILE knob).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for T in ${TILES:-0 64 256}; do
  echo "== MDG_GEMM_TILE=$T" >> gpurun_out/gemm_variants.log
  MDG_GEMM_TILE=$T timeout -k 10 200 python tools/gemm_bench.py >> gpurun_out/gemm_variants.log 2>&1 || exit $?
done
