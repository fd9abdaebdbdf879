"""Standalone timing (GPU) of the training step's large-M GEMM shapes on mdg_gemm, with and
without their epilogue extras (the GELU pre-activation store, the DGELU read), against
torch.matmul (hipBLASLt) of the same product.  Usage: python tools/gemm_train_bench.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd import _lib  # noqa: E402

lib = _lib.load()


def tm(fn, it=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


def run(M, N, K, act=0, aux=False, out_f32=0, epi=0):
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    ax = torch.randn(M, N, device="cuda").to(torch.bfloat16) if aux else None
    d = _lib.MdgGemmDesc()
    d.dtype, d.a_mode, d.epi, d.act, d.M, d.N, d.K = 1, 0, epi, act, M, N, K
    d.A, d.lda, d.W, d.ldw, d.bias = A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr()
    d.out, d.ldo, d.out_f32 = out.data_ptr(), N, out_f32
    if ax is not None:
        d.aux, d.ldaux = ax.data_ptr(), N
    s = torch.cuda.current_stream().cuda_stream
    us = tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(d), s), "gemm"))
    ref = tm(lambda: torch.matmul(A, W.t()))
    fl = 2.0 * M * N * K
    byt = M * K * 2 + N * K * 2 + M * N * (4 if out_f32 else 2) + (M * N * 2 if aux else 0)
    print(f"M={M} N={N:5d} K={K:5d} act={act} aux={int(aux)} f32={out_f32}: mdg {us:7.1f} us "
          f"({fl / us / 1e6:6.1f} TF/s, {byt / us / 1e3:6.0f} GB/s)  torch.matmul {ref:7.1f} us "
          f"({fl / ref / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    M = 32000
    for env in (None,):
        run(M, 1536, 384)                       # plain store
        run(M, 1536, 384, act=1, aux=True)      # fc1 forward: GELU, pre-activation stored (aux)
        run(M, 1536, 384, act=3, aux=True)      # du = (dy W2) * gelu'(u): DGELU reads aux
        run(M, 384, 1536)                       # dxn3 = du W1
        run(M, 384, 1152)                       # dxn from dqkv
        run(M, 384, 384)                        # do from dy
        run(M, 384, 384, out_f32=1)
