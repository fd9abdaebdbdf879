#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gate_res or lnmod" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rowln.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_rowln.log
[ $rc -ne 0 ] && exit $rc
for bm in 128 64; do
  echo "MDG_ROWLN_BM=$bm"
  MDG_ROWLN_BM=$bm timeout -k 10 120 python -u tools/gemm_bench.py rowln 2>&1 | grep -v amdgpu.ids || exit 1
  MDG_ROWLN_BM=$bm timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rowln.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/bench_rowln.log').read().strip().splitlines()[-1]);print('bench', d['value'], d['us_per_denoise_step'])"
  MDG_ROWLN_BM=$bm timeout -k 10 300 python -u bench.py --batch 8 --lanes 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rowln.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/bench_rowln.log').read().strip().splitlines()[-1]);print('bench B8 lanes1', d['value'], d['us_per_denoise_step'])"
done
