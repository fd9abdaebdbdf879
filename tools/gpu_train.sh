#!/bin/bash
# Training-step throughput on one GPU (config 3 per GPU): the HIP block stack (bf16 / f32
# operands) against eager torch (fp32, bf16-mixed autocast).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u tools/train_bench.py --batch 8 --steps 5 --warmup 2 "$@" > gpurun_out/train_$tag.log 2>&1
  local rc=$?; echo "train $tag rc=$rc"; tail -1 gpurun_out/train_$tag.log
  return $rc
}
run hip_bf16 --train_backend hip --hip_dtype bf16 && \
run hip_f32 --train_backend hip --hip_dtype f32 && \
run torch_fp32 --train_backend torch && \
run torch_bf16mixed --train_backend torch --precision bf16-mixed
