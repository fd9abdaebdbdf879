#!/bin/bash
# Round 4: aligned bucket slices (foreach copy) in the in-graph all-reduce; capture tests and the
# world-1 rehearsal line + trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_train.py tests/test_gpu_optim.py -k 'rccl or graphed or world2 or optim or fused or resume'" \
  "rccl_line|200|python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3 --train-rccl1 > gpurun_out/r04_bench_train_rccl1.json" \
  "plain_line|200|python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3 > gpurun_out/r04_bench_train_plain.json" \
  "trainprof_rccl|300|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh"
