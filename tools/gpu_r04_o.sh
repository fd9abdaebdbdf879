#!/bin/bash
# Round 4: bias-slot change (attention backward + unpack tests), then the evidence traces: the
# training step (plain and with the world-1 RCCL bucket all-reduces captured), the headline bench
# line + its kernel trace, the B = 1 window trace and the dopri5 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "bwdtests|400|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_attn_bwd.py tests/test_gpu_train.py tests/test_gpu_optim.py" \
  "train|200|python bench.py --train --batch 8 > gpurun_out/r04_bench_train.json" \
  "trainprof|200|bash tools/gpu_train_prof.sh" \
  "trainprof_rccl|200|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "bench|240|python bench.py > gpurun_out/r04_bench.json" \
  "prof|200|bash tools/gpu_prof.sh" \
  "prof_b1|150|PROF_DIR=gpurun_out/prof_b1 BENCH_ARGS='--batch 1 --lanes 1' bash tools/gpu_prof.sh" \
  "dopri5|150|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r04_bench_dopri5.json"
