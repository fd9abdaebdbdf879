#!/bin/bash
# Round 4: the new kernels' tests (MFMA spatial epilogue, wide-tile wgrad, segmented linears,
# local-point IPA core), then same-box A/Bs: the inference bench with MDG_SPA_MFMA=0 / 1 and the
# training line with MDG_WGRAD_WIDE=0 / 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python bench.py --steps 6 --warmup 2 --no-cpu-baseline --sweep-batches '' --no-f32-line"
bash tools/gpu_steps.sh \
  "newtests|300|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_wgrad.py tests/test_gpu_glue.py tests/test_gpu_ipa_train.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -k 'wgrad or seg or ipa or spatial or embed or final or dopri5'" \
  "ab_spa0|120|MDG_SPA_MFMA=0 $B > gpurun_out/ab_spa0.json" \
  "ab_spa1|120|MDG_SPA_MFMA=1 $B > gpurun_out/ab_spa1.json" \
  "ab_spa0b|120|MDG_SPA_MFMA=0 $B > gpurun_out/ab_spa0b.json" \
  "ab_spa1b|120|MDG_SPA_MFMA=1 $B > gpurun_out/ab_spa1b.json" \
  "ab_wg0|150|MDG_WGRAD_WIDE=0 python bench.py --train --batch 8 --no-cpu-baseline > gpurun_out/ab_wg0.json" \
  "ab_wg1|150|MDG_WGRAD_WIDE=1 python bench.py --train --batch 8 --no-cpu-baseline > gpurun_out/ab_wg1.json"
