#!/bin/bash
# Fused spatial kernel ring depth: parity tests at every depth, standalone timing, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for st in 2 3 4; do
  MDG_SPA_STAGES=$st timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -q -x \
    -k "spatial or golden or full_size_T1000 or padded_residues or lanes" --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_spa$st.log 2>&1 || { tail -20 gpurun_out/pytest_spa$st.log; exit 1; }
  echo "stages $st: $(tail -1 gpurun_out/pytest_spa$st.log)"
done
for rep in 1 2; do
  for st in 2 3 4; do
    MDG_SPA_STAGES=$st timeout -k 10 100 python tools/gemm_bench.py spa || exit 1
  done
done
for rep in 1 2; do
  for st in 2 3; do
    MDG_SPA_STAGES=$st timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --sweep-batches "" \
      --no-f32-line > gpurun_out/bench_spa.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/bench_spa.log').read().strip().splitlines()[-1]);print('stages $st', d['value'], d['us_per_denoise_step'])"
  done
done
