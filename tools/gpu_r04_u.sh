#!/bin/bash
# Round 4: split-sum / unpack loops with their loads in flight; wgrad + training tests, line, trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "tests|500|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_attn_bwd.py tests/test_gpu_wgrad.py tests/test_gpu_glue.py tests/test_gpu_train.py tests/test_gpu_ipa_train.py" \
  "train|120|python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3 > gpurun_out/r04_bench_train_u.json" \
  "trainprof|200|bash tools/gpu_train_prof.sh"
