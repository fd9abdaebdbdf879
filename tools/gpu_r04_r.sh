#!/bin/bash
# Round 4: training-step A/B of the GEMM knobs (K-step 64 tile, 8-B epilogue) on one box, plus
# the unpack / pack tests of the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3"
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_train.py tests/test_gpu_ipa_train.py" \
  "ab_default|120|$T > gpurun_out/ab_default.json" \
  "ab_k64|120|MDG_GEMM_TILE=64 $T > gpurun_out/ab_k64.json" \
  "ab_epi8|120|MDG_WIDE_EPI=0 $T > gpurun_out/ab_epi8.json" \
  "ab_default2|120|$T > gpurun_out/ab_default2.json"
