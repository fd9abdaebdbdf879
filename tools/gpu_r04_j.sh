#!/bin/bash
# Round 4: K-split segmented forward for few-row linears; which PyTorch operators remain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3"
bash tools/gpu_steps.sh \
  "gluetests|300|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_glue.py tests/test_gpu_ipa_train.py tests/test_gpu_train.py -k 'seg or glue or embed or final or ipa or default_dims or gvp or small_loss'" \
  "train|120|$T > gpurun_out/r04_bench_train.json" \
  "trainprof|200|bash tools/gpu_train_prof.sh" \
  "torchops|200|python tools/torch_ops_trace.py"
