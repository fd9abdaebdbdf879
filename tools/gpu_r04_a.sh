#!/bin/bash
# Round 4: the new kernels' tests (fused attention backward, fused wgrad bias) and their bench,
# the in-graph RCCL bucket all-reduce test, smoke, the GPU suite, the training line (plain and
# with the world-1 RCCL rehearsal), kernel traces of both, and a torch-profiler op table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "kern_tests|300|python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_attn_bwd.py tests/test_gpu_wgrad.py tests/test_gpu_glue.py tests/test_gpu_parity.py -k \"bwd or wgrad or dopri5 or embed or final_layer\"" \
  "attn_bwd_bench|120|python tools/attn_bwd_bench.py > gpurun_out/attn_bwd_bench.json" \
  "rccl_test|300|python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_train.py -k rccl" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|600|bash tools/gpu_suite.sh" \
  "train|300|python bench.py --train --batch 8 --no-cpu-baseline > gpurun_out/r04_bench_train.json" \
  "train_rccl|300|python bench.py --train --batch 8 --no-cpu-baseline --train-rccl1 > gpurun_out/r04_bench_train_rccl1.json" \
  "trainprof_rccl|300|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "trainprof|300|bash tools/gpu_train_prof.sh" \
  "dopri5|300|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r04_bench_dopri5.json" \
  "torchprof|300|python tools/train_prof.py --train_graph 0 > gpurun_out/train_torchprof.txt"
