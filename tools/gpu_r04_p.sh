#!/bin/bash
# Round 4: operand ring depth of the K-step-32 GEMM (MDG_B4_STAGES 2 / 3 / 4): GEMM and layer
# backward tests at each depth, then the training line at each depth.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
S="tests/test_gpu_kernels.py tests/test_gpu_train.py -k 'gemm_plain or layer_backward or default_dims'"
T="python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3"
bash tools/gpu_steps.sh \
  "ns3tests|300|MDG_B4_STAGES=3 $P $S" \
  "ns4tests|300|MDG_B4_STAGES=4 $P $S" \
  "train_ns2|120|MDG_B4_STAGES=2 $T > gpurun_out/train_ns2.json" \
  "train_ns3|120|MDG_B4_STAGES=3 $T > gpurun_out/train_ns3.json" \
  "train_ns4|120|MDG_B4_STAGES=4 $T > gpurun_out/train_ns4.json"
