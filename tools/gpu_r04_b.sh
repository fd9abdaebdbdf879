#!/bin/bash
# Round 4 (re-entry): smoke, the GPU suite of the current tree, the training line and the
# fused attention-backward microbench, each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "smoke|240|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|600|bash tools/gpu_suite.sh" \
  "attn_bwd_bench|90|python tools/attn_bwd_bench.py > gpurun_out/attn_bwd_bench.json" \
  "train|180|python bench.py --train --batch 8 --no-cpu-baseline > gpurun_out/r04_bench_train.json"
