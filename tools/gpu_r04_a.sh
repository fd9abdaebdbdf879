#!/bin/bash
# Round 4: the in-graph RCCL bucket all-reduce test first, then smoke, the GPU suite, the
# training line (plain and with the world-1 RCCL rehearsal) and kernel traces of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "rccl_test|300|python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_train.py -k rccl" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|600|bash tools/gpu_suite.sh" \
  "train|300|python bench.py --train --batch 8 --no-cpu-baseline > gpurun_out/r04_bench_train.json" \
  "train_rccl|300|python bench.py --train --batch 8 --no-cpu-baseline --train-rccl1 > gpurun_out/r04_bench_train_rccl1.json" \
  "trainprof_rccl|300|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "trainprof|300|bash tools/gpu_train_prof.sh"
