#!/bin/bash
# Same-box A/B of two builds of the library: the tree's libmdgen_hip.so vs build/ab/old.so
# (MDG_LIB_PATH), alternating, on the row-LN GEMM microbench and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export MDG_LIB_PATH=$PWD/build/ab/old.so; else unset MDG_LIB_PATH; fi
    echo "== $L"
    timeout -k 10 100 python tools/gemm_bench.py ${AB_MODE:-rowln} 2>&1 | grep mdg | cut -c1-75
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['us_per_denoise_step'])"
  done
done
