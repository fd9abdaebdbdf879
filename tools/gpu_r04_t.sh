#!/bin/bash
# Round 4: K-step-64 GEMM tile by default without an aux operand, DGELU pre-activation prefetch;
# kernel + training tests, the GEMM microbenchmark, the training line and trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "tests|500|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_parity.py -k 'gemm or layer_backward or default_dims or graphed or headline or forward_matches or euler_solve'" \
  "gemmbench|200|python tools/gemm_train_bench.py > gpurun_out/gemm_train_bench.log" \
  "train|120|python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3 > gpurun_out/r04_bench_train_t.json" \
  "trainprof|200|bash tools/gpu_train_prof.sh"
