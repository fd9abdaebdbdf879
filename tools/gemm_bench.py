"""Standalone GEMM timing on the GPU: libmdgen_hip mdg_gemm vs torch (hipBLASLt) on the
block's shapes.  Usage: python tools/gemm_bench.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd import _lib  # noqa: E402

lib = _lib.load()


def tm(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


def run(M, N, K, a_mode, epi, dt="bf16", act=0, rowln=False):
    ct = torch.bfloat16 if dt == "bf16" else torch.float32
    A = torch.randn(M, K, device="cuda").to(ct if a_mode == 0 else torch.float32)
    W = torch.randn(N, K, device="cuda").to(ct)
    bias = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=ct)
    resid = torch.zeros(M, N, device="cuda")
    mods = torch.randn(M // 4000 + 1, 9 * K, device="cuda") * 0.1
    d = _lib.MdgGemmDesc()
    d.dtype = 1 if dt == "bf16" else 0
    d.a_mode, d.epi, d.M, d.N, d.K, d.act = a_mode, epi, M, N, K, act
    d.A, d.lda, d.W, d.ldw, d.bias = A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr()
    d.mods, d.mod_stride, d.rows_per_mod, d.shift_off, d.scale_off, d.ln_eps = mods.data_ptr(), 9 * K, 4000, 0, K, 1e-6
    d.out, d.ldo, d.resid, d.ldr = out.data_ptr(), N, resid.data_ptr(), N
    if rowln:  # + LayerNorm of the updated rows into a bf16 xn (gemm_rowln_kernel)
        xn = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        d.gate, d.gate_off, d.rows_per_mod, d.mod_stride = mods.data_ptr(), 0, 4000, 9 * K
        d.xn_out, d.xn_mods, d.xn_mod_stride, d.xn_shift_off, d.xn_scale_off = (xn.data_ptr(), mods.data_ptr(),
                                                                              9 * K, 0, N)
    s = torch.cuda.current_stream().cuda_stream

    def f():
        _lib.check(lib.mdg_gemm(ctypes.byref(d), s), "gemm")

    us = tm(f)
    Ab = A.to(ct)
    ref = tm(lambda: torch.matmul(Ab, W.t()))
    fl = 2.0 * M * N * K
    print(f"M={M:6d} N={N:5d} K={K:5d} amode={a_mode} epi={epi} act={act} {dt}: mdg {us:8.1f} us ({fl/us/1e6:7.1f} TF/s)   "
          f"torch.matmul {ref:8.1f} us ({fl/ref/1e6:7.1f} TF/s)", flush=True)


def run_mlp(M, C=384, F=1536, rpm=4000):
    """mdg_mlp_fused vs mdg_gemm(fc1) + mdg_gemm(fc2) (row-LN hand-off) on one lane's shape."""
    A = (torch.randn(M, C, device="cuda") * 0.5).to(torch.bfloat16)
    W1 = (torch.randn(F, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
    W2 = (torch.randn(C, F, device="cuda") / F ** 0.5).to(torch.bfloat16)
    b1, b2 = torch.randn(F, device="cuda"), torch.randn(C, device="cuda")
    hid = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    resid, xn = torch.zeros(M, C, device="cuda"), torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    mods = torch.randn(M // rpm + 1, 9 * C, device="cuda") * 0.1
    f1, f2 = _lib.MdgGemmDesc(), _lib.MdgGemmDesc()
    f1.dtype, f1.a_mode, f1.epi, f1.act, f1.M, f1.N, f1.K = 1, 0, 0, 1, M, F, C
    f1.A, f1.lda, f1.W, f1.ldw, f1.bias, f1.out, f1.ldo = A.data_ptr(), C, W1.data_ptr(), C, b1.data_ptr(), hid.data_ptr(), F
    f2.dtype, f2.a_mode, f2.epi, f2.M, f2.N, f2.K = 1, 0, 1, M, C, F
    f2.A, f2.lda, f2.W, f2.ldw, f2.bias = hid.data_ptr(), F, W2.data_ptr(), F, b2.data_ptr()
    f2.resid, f2.ldr, f2.gate, f2.gate_off, f2.mod_stride, f2.rows_per_mod = resid.data_ptr(), C, mods.data_ptr(), 0, 9 * C, rpm
    f2.xn_out, f2.xn_mods, f2.xn_mod_stride, f2.xn_shift_off, f2.xn_scale_off, f2.ln_eps = (xn.data_ptr(), mods.data_ptr(),
                                                                                           9 * C, 0, C, 1e-6)
    s = torch.cuda.current_stream().cuda_stream
    fused = tm(lambda: _lib.check(lib.mdg_mlp_fused(ctypes.byref(f1), ctypes.byref(f2), s), "mlp"))
    t1 = tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(f1), s), "fc1"))
    t2 = tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(f2), s), "fc2"))
    fl = 4.0 * M * C * F
    print(f"mlp M={M}: mdg fused {fused:8.1f} us ({fl / fused / 1e6:7.1f} TF/s)   fc1 {t1:7.1f} + fc2 {t2:7.1f} = "
          f"{t1 + t2:7.1f} us", flush=True)


def run_rq(B=8, T=1000, L=4, H=16, D=24):
    """mdg_rowln_qkv vs mdg_gemm(out_proj row-LN) + mdg_gemm(temporal q|k|v) on one lane's shape."""
    C, M = H * D, B * T * L
    o = (torch.randn(M, C, device="cuda") * 0.5).to(torch.bfloat16)
    Wo = (torch.randn(C, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
    Wq = (torch.randn(3 * C, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
    bo, bq = torch.randn(C, device="cuda"), torch.randn(3 * C, device="cuda")
    resid, xn = torch.zeros(M, C, device="cuda"), torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    planes = torch.empty(3 * M * C, device="cuda", dtype=torch.bfloat16)
    mods = torch.randn(B, 9 * C, device="cuda") * 0.1
    rope = torch.randn(2 * (T + 1) * (D // 2), device="cuda")
    r, q = _lib.MdgGemmDesc(), _lib.MdgGemmDesc()
    r.dtype, r.a_mode, r.epi, r.M, r.N, r.K = 1, 0, 1, M, C, C
    r.A, r.lda, r.W, r.ldw, r.bias = o.data_ptr(), C, Wo.data_ptr(), C, bo.data_ptr()
    r.resid, r.ldr, r.gate, r.gate_off, r.mod_stride, r.rows_per_mod = resid.data_ptr(), C, mods.data_ptr(), 2 * C, 9 * C, T * L
    r.xn_out, r.xn_mods, r.xn_mod_stride, r.xn_shift_off, r.xn_scale_off, r.ln_eps = (xn.data_ptr(), mods.data_ptr(),
                                                                                       9 * C, 3 * C, 4 * C, 1e-6)
    q.dtype, q.a_mode, q.epi, q.M, q.N, q.K = 1, 0, 2, M, 3 * C, C
    q.A, q.lda, q.W, q.ldw, q.bias = xn.data_ptr(), C, Wq.data_ptr(), C, bq.data_ptr()
    q.qkv_layout, q.qkv_out, q.H, q.D, q.T, q.L, q.qscale = 2, planes.data_ptr(), H, D, T, L, 0.3
    q.rope, q.rope_rows = rope.data_ptr(), T + 1
    s = torch.cuda.current_stream().cuda_stream
    fused = tm(lambda: _lib.check(lib.mdg_rowln_qkv(ctypes.byref(r), ctypes.byref(q), s), "rq"))
    t1 = tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(r), s), "out_proj"))
    t2 = tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(q), s), "qkv"))
    print(f"rq M={M}: mdg fused {fused:8.1f} us   out_proj {t1:7.1f} + qkv {t2:7.1f} = {t1 + t2:7.1f} us", flush=True)


def run_spa(B=8, T=1000, L=4, H=16, D=24):
    """The fused spatial q|k|v projection + 4-residue attention (MDG_EPI_ATTN_SPATIAL) on one
    lane's shape."""
    C, M = H * D, B * T * L
    xn = (torch.randn(M, C, device="cuda") * 0.5).to(torch.bfloat16)
    W = (torch.randn(3 * C, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
    bq = torch.randn(3 * C, device="cuda")
    kvb = torch.zeros(H, 2, 32, device="cuda")
    kvb[:, :, :D] = torch.randn(H, 2, D, device="cuda")
    rope = torch.randn(2 * L * (D // 2), device="cuda")
    o = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    d = _lib.MdgGemmDesc()
    d.dtype, d.a_mode, d.epi, d.M, d.N, d.K = 1, 0, 4, M, 3 * C, C
    d.A, d.lda, d.W, d.ldw, d.bias = xn.data_ptr(), C, W.data_ptr(), C, bq.data_ptr()
    d.H, d.D, d.T, d.L, d.qscale, d.rope, d.rope_rows = H, D, T, L, D ** -0.5, rope.data_ptr(), L
    d.out, d.ldo, d.kvb = o.data_ptr(), C, kvb.data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    us = tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(d), s), "spa"))
    fl = 2.0 * M * 3 * C * C
    print(f"spa M={M}: {us:7.1f} us ({fl / us / 1e6:6.1f} TF/s)  MDG_SPA_STAGES={os.environ.get('MDG_SPA_STAGES', '2')}",
          flush=True)


def run_final(M=32000, C=384, latent=21):
    """The denoise step's FinalLayer + Euler (mdg_gemm EULER, N = 32: final_euler_kernel) vs
    the generic 64x32 GEMM (an N = 64 descriptor)."""
    xn = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    W = torch.zeros(64, C, device="cuda")
    W[:latent] = torch.randn(latent, C, device="cuda") / C ** 0.5
    W = W.to(torch.bfloat16)
    b = torch.zeros(64, device="cuda")
    xin, xo, vo = (torch.randn(M, latent, device="cuda") for _ in range(3))
    s = torch.cuda.current_stream().cuda_stream
    res = []
    for n in (32, 64):
        d = _lib.MdgGemmDesc()
        d.dtype, d.a_mode, d.epi, d.M, d.N, d.K = 1, 0, 3, M, n, C
        Wn, bn = W[:n].contiguous(), b[:n].contiguous()
        d.A, d.lda, d.W, d.ldw, d.bias = xn.data_ptr(), C, Wn.data_ptr(), C, bn.data_ptr()
        d.out, d.ldo, d.x_in, d.v_out, d.dt, d.n_valid = xo.data_ptr(), latent, xin.data_ptr(), vo.data_ptr(), 0.02, latent
        res.append(tm(lambda: _lib.check(lib.mdg_gemm(ctypes.byref(d), s), "euler")))
    mb = (M * C * 2 + 3 * M * latent * 4) / 1e6
    print(f"final M={M}: final_euler {res[0]:7.1f} us ({mb / res[0]:6.2f} TB/s)   generic {res[1]:7.1f} us", flush=True)


if __name__ == "__main__":
    import sys as _s
    if len(_s.argv) > 1 and _s.argv[1] == "spa":
        run_spa()
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "final":
        run_final()
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "rq":
        run_rq()
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "mlp":
        for M in (32000, 64000):
            run_mlp(M)
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "rowln":  # fused gated residual + LN (out_proj / fc2)
        for M in (32000, 64000):
            for K in (384, 1536):
                run(M, 384, K, 0, 1, rowln=True)
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "rowlnk":  # row-LN GEMM K sweep: epilogue vs main loop
        for K in (64, 128, 384, 768, 1536):
            run(32000, 384, K, 0, 1, rowln=True)
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "b4":  # the 128x128 streamed-A shapes (fc1, qkv)
        for M in (32000, 64000):
            run(M, 1536, 384, 0, 0, act=1)
            run(M, 1152, 384, 0, 0)
        _s.exit(0)
    if len(_s.argv) > 1 and _s.argv[1] == "ksweep":
        for K in (64, 128, 384):
            run(32000, 1536, K, 0, 0)
        run(32000, 1536, 384, 0, 0, act=1)
        _s.exit(0)
    for B in (8, 1):
        M = B * 4000
        run(M, 384, 384, 0, 1)      # out-proj gate-res
        run(M, 384, 1536, 0, 1)     # fc2 gate-res
        run(M, 1152, 384, 0, 0)     # qkv-shaped plain store
        run(M, 1536, 384, 0, 0)     # fc1-shaped plain store
        run(M, 1536, 384, 0, 0, act=1)  # fc1 with GELU
