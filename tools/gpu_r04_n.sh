#!/bin/bash
# Round 4: optimizer tests, graphed-step tests, training line, training trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3"
bash tools/gpu_steps.sh \
  "optimtests|400|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_optim.py tests/test_gpu_train.py -k 'optim or fused or graphed or resume or world2'" \
  "train|120|$T > gpurun_out/r04_bench_train.json" \
  "trainprof|200|bash tools/gpu_train_prof.sh"
