#!/bin/bash
# Timing diagnostics of the fused MLP and the temporal attention (MDG_DIAG_MLP / MDG_DIAG_ATTN in
# gemm.hip / attention.hip).  `tools/diag_mlp_attn.sh build` (CPU) links one library per variant
# under build/diag/; with no argument (GPU box) it times each variant's kernel standalone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS="mlp1 mlp2 mlp3 attn1 attn2"
if [ "${1:-}" = build ]; then
  C=mdgen_finetune_amd/csrc
  F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form"
  make -C $C -j4 >/dev/null || exit 1
  mkdir -p build/diag
  for v in $VARIANTS; do
    case $v in mlp*) src=gemm; def="-DMDG_DIAG_MLP=${v#mlp}";; attn*) src=attention; def="-DMDG_DIAG_ATTN=${v#attn}";; esac
    /opt/rocm/bin/hipcc $F $def -c $C/$src.hip -o build/diag/$src.$v.o || exit 1
    objs=""
    for o in gemm attention elementwise geometry train cond capi; do
      if [ $o = $src ]; then objs="$objs build/diag/$src.$v.o"; else objs="$objs $C/$o.o"; fi
    done
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -o build/diag/$v.so || exit 1
  done
  exit 0
fi
mkdir -p gpurun_out
for rep in 1 2; do
  unset MDG_LIB_PATH
  echo "== base"
  timeout -k 10 100 python tools/gemm_bench.py mlp 2>&1 | grep mlp | cut -c1-60 || exit 1
  timeout -k 10 100 python tools/attn_bench.py 2>&1 | grep attn || exit 1
  for v in $VARIANTS; do
    export MDG_LIB_PATH=$PWD/build/diag/$v.so
    echo "== $v"
    case $v in
      mlp*) timeout -k 10 100 python tools/gemm_bench.py mlp 2>&1 | grep mlp | cut -c1-60 || exit 1;;
      attn*) timeout -k 10 100 python tools/attn_bench.py 2>&1 | grep attn || exit 1;;
    esac
  done
done
