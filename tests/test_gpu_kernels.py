"""Per-kernel numerics of libmdgen_hip.so against plain PyTorch fp32 references of the same op
(called through the C ABI: mdg_gemm / mdg_attn_temporal / mdg_attn_spatial / mdg_embed /
mdg_final_euler)."""
import ctypes
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    return _lib.load()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _tol(dt):
    return (2e-5, 2e-5) if dt == "f32" else (2e-2, 2e-2)


CT = {"f32": torch.float32, "bf16": torch.bfloat16}
ENUM = {"f32": 0, "bf16": 1}


def _desc(**kw):
    from mdgen_finetune_amd import _lib

    d = _lib.MdgGemmDesc()
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def _ln_mod(a, mods, rows_per, sh_off, sc_off, C, eps=1e-6):
    y = torch.nn.functional.layer_norm(a, (a.shape[-1],), eps=eps)
    b = torch.arange(a.shape[0], device=a.device) // rows_per
    m = mods[b]
    return y * (1 + m[:, sc_off:sc_off + C]) + m[:, sh_off:sh_off + C]


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("M,N,K,act", [(200, 384, 384, 0), (64, 1536, 384, 1), (130, 192, 1536, 2), (7, 64, 64, 0),
                                        (300, 128, 64, 0), (257, 256, 128, 1), (520, 384, 1536, 0)])
def test_gemm_plain_store(lib, dt, M, N, K, act):
    from mdgen_finetune_amd import _lib

    g = torch.Generator(device="cuda").manual_seed(M + N)
    A = torch.randn(M, K, device="cuda", generator=g).to(CT[dt])
    W = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).to(CT[dt])
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda")
    d = _desc(dtype=ENUM[dt], a_mode=0, epi=0, act=act, M=M, N=N, K=K, A=A.data_ptr(), lda=K, W=W.data_ptr(),
              ldw=K, bias=bias.data_ptr(), out=out.data_ptr(), ldo=N, out_f32=1)
    _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "mdg_gemm")
    ref = A.float() @ W.float().T + bias
    ref = {0: ref, 1: ref * 0.5 * (1 + torch.erf(ref / math.sqrt(2))), 2: torch.nn.functional.silu(ref)}[act]
    rtol, atol = _tol(dt)
    torch.testing.assert_close(out, ref, rtol=rtol, atol=atol)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_gemm_lnmod_gate_res(lib, dt):
    from mdgen_finetune_amd import _lib

    M, C, TL = 300, 384, 100
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn(M, C, device="cuda", generator=g) * 3 + 1
    W = (torch.randn(C, C, device="cuda", generator=g) / math.sqrt(C)).to(CT[dt])
    bias = torch.randn(C, device="cuda", generator=g)
    mods = torch.randn(3, 9 * C, device="cuda", generator=g) * 0.5
    resid = torch.randn(M, C, device="cuda", generator=g)
    r0 = resid.clone()
    d = _desc(dtype=ENUM[dt], a_mode=1, epi=1, M=M, N=C, K=C, A=A.data_ptr(), lda=C, W=W.data_ptr(), ldw=C,
              bias=bias.data_ptr(), mods=mods.data_ptr(), mod_stride=9 * C, rows_per_mod=TL, shift_off=3 * C,
              scale_off=4 * C, ln_eps=1e-6, resid=resid.data_ptr(), ldr=C, gate=mods.data_ptr(), gate_off=5 * C)
    _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "mdg_gemm")
    y = _ln_mod(A, mods, TL, 3 * C, 4 * C, C).to(CT[dt]).float()
    b = torch.arange(M, device="cuda") // TL
    ref = r0 + mods[b, 5 * C:6 * C] * (y @ W.float().T + bias)
    rtol, atol = _tol(dt)
    torch.testing.assert_close(resid, ref, rtol=rtol, atol=atol * 10)


@pytest.mark.parametrize("N,K,M", [(384, 384, 300), (384, 1536, 4000), (128, 256, 257), (512, 512, 130),
                                   (384, 64, 200), (256, 128, 129), (384, 192, 1000)])
def test_gemm_gate_res_fused_layernorm(lib, N, K, M):
    """bf16 full-row gated residual + next-LN epilogue (gemm_rowln_kernel): h and xn vs torch."""
    from mdgen_finetune_amd import _lib

    TL = 100
    g = torch.Generator(device="cuda").manual_seed(N + K + M)
    A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda", generator=g)
    nb = (M + TL - 1) // TL
    mods = torch.randn(nb, 9 * N, device="cuda", generator=g) * 0.5
    nmods = torch.randn(nb, 2 * N, device="cuda", generator=g) * 0.5
    resid = torch.randn(M, N, device="cuda", generator=g) * 2
    r0 = resid.clone()
    xn = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    d = _desc(dtype=1, a_mode=0, epi=1, M=M, N=N, K=K, A=A.data_ptr(), lda=K, W=W.data_ptr(), ldw=K,
              bias=bias.data_ptr(), mods=mods.data_ptr(), mod_stride=9 * N, rows_per_mod=TL, resid=resid.data_ptr(),
              ldr=N, gate=mods.data_ptr(), gate_off=8 * N, ln_eps=1e-6, xn_out=xn.data_ptr(), xn_mods=nmods.data_ptr(),
              xn_mod_stride=2 * N, xn_shift_off=0, xn_scale_off=N)
    _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "mdg_gemm")
    b = torch.arange(M, device="cuda") // TL
    href = r0 + mods[b, 8 * N:9 * N] * (A.float() @ W.float().T + bias)
    torch.testing.assert_close(resid, href, rtol=2e-3, atol=2e-3)
    xref = _ln_mod(resid, nmods, TL, 0, N, N)  # LN of the kernel's own h: isolates the epilogue LN
    torch.testing.assert_close(xn.float(), xref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,TL,with_ln", [(512, 256, True), (4000, 4000, True), (300, 150, True), (1000, 200, False),
                                         (8292, 4146, True)])
def test_mlp_fused_equals_fc1_then_fc2(lib, M, TL, with_ln):
    """mdg_mlp_fused (fc1 + GELU + fc2 + gated residual + next LN in one kernel, the hidden
    activation on chip) against the same two descriptors through mdg_gemm: h and xn
    bit-identical (same K order, same GELU, same bf16 rounding of the hidden activation), and
    against torch.  Partial last tiles (M % 128 != 0) and tiles spanning two trajectories;
    M < 8065 takes the split-hidden route, 8292 the one-pass kernel."""
    _mlp_fused_vs_unfused(lib, M, TL, with_ln)


@pytest.mark.parametrize("knob", ["MDG_MLP_WS=0", "MDG_MLP_WS=1", "MDG_MLP_WS=0 MDG_MLP_HC=256"])
def test_mlp_fused_opt_in_variants(knob):
    """The other one-pass MLP kernels (lock-step round 2, wave-specialised round 3, 256-wide hidden
    chunks; the default is round 6's wave-specialised kernel) are bit-identical to the unfused pair
    too: run in a child process (the knobs are read once per process); M = 20000 has a partial
    last tile and 100 trajectory boundaries, M = 32000 fills the chip (250 tiles)."""
    import subprocess
    import sys

    env = dict(os.environ, **dict(kv.split("=") for kv in knob.split()))
    code = ("import sys; sys.path.insert(0, '.'); from mdgen_finetune_amd import _lib; "
            "from tests.test_gpu_kernels import _mlp_fused_vs_unfused; "
            "_mlp_fused_vs_unfused(_lib.load(), 20000, 200, True); _mlp_fused_vs_unfused(_lib.load(), 8292, 4146, False); "
            "_mlp_fused_vs_unfused(_lib.load(), 32000, 4000, True); "
            "print('ok')")
    r = subprocess.run([sys.executable, "-c", code], env=env,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


@pytest.mark.parametrize("F", [6144, 7168])
def test_mlp_fused_wide_hidden(lib, F):
    """Hidden widths at the wave-specialised kernel's LDS limit (F = 6 144: H + W1 ring + b1 =
    160 KiB) and past it (7 168: the launcher takes the lock-step kernel, whose limit is 8 192):
    still bit-identical to fc1 then fc2."""
    _mlp_fused_vs_unfused(lib, 8292, 4146, True, F=F)


def test_mlp_ws2_window_equals_lockstep():
    """The round-6 wave-specialised MLP (the default) in the bench's whole inference window (B = 16,
    two concurrent lanes, hipGraph, 49 Euler steps: 2 x 250-tile launches per layer): the samples
    equal the lock-step kernel's (MDG_MLP_WS=0) bit for bit, twice over.  Its first form issued ring slot ph + 2 one phase late
    and waited on the wrong count, a race that left this window non-finite a few times in ten
    while the single-launch kernel tests passed."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sums = []
    for env in ({"MDG_MLP_WS": "0"}, {}):
        r = subprocess.run([sys.executable, "tools/window_probe.py", "2", "1", "16", "50"], env=dict(os.environ, **env),
                           cwd=root, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("lanes=")]
        assert len(lines) == 2 and all("finite=True" in ln for ln in lines), r.stdout
        sums.append([ln.split("sum=")[1] for ln in lines])
    assert sums[0][0] == sums[0][1] == sums[1][0] == sums[1][1], sums


def _mlp_fused_vs_unfused(lib, M, TL, with_ln, F=1536):
    from mdgen_finetune_amd import _lib

    C = 384
    g = torch.Generator(device="cuda").manual_seed(M + TL)
    xn = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    W1 = (torch.randn(F, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    b1 = torch.randn(F, device="cuda", generator=g) * 0.5
    W2 = (torch.randn(C, F, device="cuda", generator=g) / math.sqrt(F)).to(torch.bfloat16)
    b2 = torch.randn(C, device="cuda", generator=g)
    nb = (M + TL - 1) // TL
    mods = torch.randn(nb, 9 * C, device="cuda", generator=g) * 0.5
    nmods = torch.randn(nb, 2 * C, device="cuda", generator=g) * 0.5
    h0 = torch.randn(M, C, device="cuda", generator=g) * 2
    hid = torch.zeros(M, F, device="cuda", dtype=torch.bfloat16)
    outs = []
    for fused in (False, True):
        h = h0.clone()
        xo = torch.zeros(M, C, device="cuda", dtype=torch.bfloat16)
        f1 = _desc(dtype=1, a_mode=0, epi=0, act=1, M=M, N=F, K=C, A=xn.data_ptr(), lda=C, W=W1.data_ptr(), ldw=C,
                   bias=b1.data_ptr(), out=hid.data_ptr(), ldo=F)
        kw = dict(xn_out=xo.data_ptr(), xn_mods=nmods.data_ptr(), xn_mod_stride=2 * C, xn_shift_off=0,
                  xn_scale_off=C, ln_eps=1e-6) if with_ln else {}
        f2 = _desc(dtype=1, a_mode=0, epi=1, M=M, N=C, K=F, A=hid.data_ptr(), lda=F, W=W2.data_ptr(), ldw=F,
                   bias=b2.data_ptr(), mod_stride=9 * C, rows_per_mod=TL, resid=h.data_ptr(), ldr=C,
                   gate=mods.data_ptr(), gate_off=8 * C, **kw)
        if fused:
            _lib.check(lib.mdg_mlp_fused(ctypes.byref(f1), ctypes.byref(f2), _s()), "mdg_mlp_fused")
        else:
            _lib.check(lib.mdg_gemm(ctypes.byref(f1), _s()), "fc1")
            _lib.check(lib.mdg_gemm(ctypes.byref(f2), _s()), "fc2")
        outs.append((h, xo))
    torch.cuda.synchronize()
    (h_ref, x_ref), (h_f, x_f) = outs
    b = torch.arange(M, device="cuda") // TL
    pre = xn.float() @ W1.float().T + b1
    hidden = (pre * 0.5 * (1 + torch.erf(pre / math.sqrt(2)))).to(torch.bfloat16).float()
    href = h0 + mods[b, 8 * C:9 * C] * (hidden @ W2.float().T + b2)
    torch.testing.assert_close(h_f, href, rtol=5e-3, atol=5e-3)
    if with_ln:  # the unfused fc2 ran the same row-LN epilogue
        assert torch.equal(h_f, h_ref), (h_f - h_ref).abs().max().item()
        assert torch.equal(x_f, x_ref), (x_f.float() - x_ref.float()).abs().max().item()
    else:  # (without the LN hand-off the unfused fc2 takes the tile GEMM's gated-residual epilogue)
        torch.testing.assert_close(h_f, h_ref, rtol=1e-6, atol=1e-5)
        assert not x_f.any()


@pytest.mark.parametrize("M,TL", [(8292, 4146), (16000, 4000), (8320, 200)])
def test_rowln_mlp_equals_out_proj_then_mlp(lib, M, TL):
    """mdg_rowln_mlp (the temporal out_proj row-LN GEMM as the fused MLP's prologue, one launch:
    h and xn written and read back by the same block) against mdg_gemm(out_proj) then
    mdg_mlp_fused: h and both LayerNorm outputs bit-identical.  Partial last tile, tiles over two
    trajectories (TL = 200)."""
    from mdgen_finetune_amd import _lib

    C, F = 384, 1536
    g = torch.Generator(device="cuda").manual_seed(M + TL + 7)
    o = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    Wo = (torch.randn(C, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    bo = torch.randn(C, device="cuda", generator=g) * 0.5
    W1 = (torch.randn(F, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    b1 = torch.randn(F, device="cuda", generator=g) * 0.5
    W2 = (torch.randn(C, F, device="cuda", generator=g) / math.sqrt(F)).to(torch.bfloat16)
    b2 = torch.randn(C, device="cuda", generator=g)
    nb = (M + TL - 1) // TL
    mods = torch.randn(nb, 9 * C, device="cuda", generator=g) * 0.5
    nmods = torch.randn(nb, 2 * C, device="cuda", generator=g) * 0.5
    h0 = torch.randn(M, C, device="cuda", generator=g) * 2
    outs = []
    for fused in (False, True):
        h = h0.clone()
        xn = torch.zeros(M, C, device="cuda", dtype=torch.bfloat16)
        xo = torch.zeros(M, C, device="cuda", dtype=torch.bfloat16)
        r = _desc(dtype=1, a_mode=0, epi=1, M=M, N=C, K=C, A=o.data_ptr(), lda=C, W=Wo.data_ptr(), ldw=C,
                  bias=bo.data_ptr(), mod_stride=9 * C, rows_per_mod=TL, resid=h.data_ptr(), ldr=C,
                  gate=mods.data_ptr(), gate_off=5 * C, xn_out=xn.data_ptr(), xn_mods=mods.data_ptr(),
                  xn_mod_stride=9 * C, xn_shift_off=6 * C, xn_scale_off=7 * C, ln_eps=1e-6)
        f1 = _desc(dtype=1, a_mode=0, epi=0, act=1, M=M, N=F, K=C, A=xn.data_ptr(), lda=C, W=W1.data_ptr(), ldw=C,
                   bias=b1.data_ptr(), out=0, ldo=F)
        f2 = _desc(dtype=1, a_mode=0, epi=1, M=M, N=C, K=F, A=0, lda=F, W=W2.data_ptr(), ldw=F,
                   bias=b2.data_ptr(), mod_stride=9 * C, rows_per_mod=TL, resid=h.data_ptr(), ldr=C,
                   gate=mods.data_ptr(), gate_off=8 * C, xn_out=xo.data_ptr(), xn_mods=nmods.data_ptr(),
                   xn_mod_stride=2 * C, xn_shift_off=0, xn_scale_off=C, ln_eps=1e-6)
        if fused:
            _lib.check(lib.mdg_rowln_mlp(ctypes.byref(r), ctypes.byref(f1), ctypes.byref(f2), _s()), "mdg_rowln_mlp")
        else:
            _lib.check(lib.mdg_gemm(ctypes.byref(r), _s()), "out_proj")
            _lib.check(lib.mdg_mlp_fused(ctypes.byref(f1), ctypes.byref(f2), _s()), "mlp")
        outs.append((h, xn, xo))
    torch.cuda.synchronize()
    (h_ref, xn_ref, xo_ref), (h_f, xn_f, xo_f) = outs
    b = torch.arange(M, device="cuda") // TL
    h1 = h0 + mods[b, 5 * C:6 * C] * (o.float() @ Wo.float().T + bo)
    assert xn_ref.any() and xo_ref.any()
    assert torch.equal(xn_f, xn_ref), (xn_f.float() - xn_ref.float()).abs().max().item()
    assert torch.equal(h_f, h_ref), (h_f - h_ref).abs().max().item()
    assert torch.equal(xo_f, xo_ref), (xo_f.float() - xo_ref.float()).abs().max().item()
    pre = xn_f.float() @ W1.float().T + b1
    hidden = (pre * 0.5 * (1 + torch.erf(pre / math.sqrt(2)))).to(torch.bfloat16).float()
    torch.testing.assert_close(h_f, h1 + mods[b, 8 * C:9 * C] * (hidden @ W2.float().T + b2), rtol=5e-3, atol=5e-3)


def test_rowln_mlp_rejects_unsupported_shapes(lib):
    C, F, M = 384, 1536, 8192
    r = _desc(dtype=1, a_mode=0, epi=1, M=M, N=C, K=C, A=1, lda=C, W=1, ldw=C, resid=2, ldr=C, rows_per_mod=4096,
              xn_out=3, xn_mods=1)
    f1 = _desc(dtype=1, a_mode=0, epi=0, act=1, M=M, N=F, K=C, A=3, lda=C, W=1, ldw=C)
    f2 = _desc(dtype=1, a_mode=0, epi=1, M=M, N=C, K=F, A=1, lda=F, W=1, ldw=F, resid=2, ldr=C, rows_per_mod=4096)
    r.xn_out = 4  # xn not the MLP's input
    assert lib.mdg_rowln_mlp(ctypes.byref(r), ctypes.byref(f1), ctypes.byref(f2), _s()) == 1001
    r.xn_out = 3
    r.M = f1.M = f2.M = 4000  # < 64 row tiles: the MLP would split
    assert lib.mdg_rowln_mlp(ctypes.byref(r), ctypes.byref(f1), ctypes.byref(f2), _s()) == 1001


def test_mlp_fused_rejects_unsupported_shapes(lib):
    d1 = _desc(dtype=1, a_mode=0, epi=0, act=1, M=256, N=1536, K=256, A=1, lda=256, W=1, ldw=256)
    d2 = _desc(dtype=1, a_mode=0, epi=1, M=256, N=256, K=1536, A=1, lda=1536, W=1, ldw=1536, resid=1, ldr=256,
               rows_per_mod=256)
    assert lib.mdg_mlp_fused(ctypes.byref(d1), ctypes.byref(d2), _s()) == 1001  # MDG_E_SHAPE: C != 384
    d1.K = d2.N = 384
    d1.lda = d2.ldr = 384
    d2.rows_per_mod = 64  # tiles over > 2 trajectories
    assert lib.mdg_mlp_fused(ctypes.byref(d1), ctypes.byref(d2), _s()) == 1001


@pytest.mark.parametrize("B,T,L,rope", [(2, 37, 4, True), (8, 250, 4, True), (1, 32, 4, False), (3, 64, 5, True),
                                        (2, 37, 32, True), (3, 9, 16, True), (1, 250, 256, True), (1, 12, 48, False)])
def test_rowln_qkv_equals_out_proj_then_qkv(lib, B, T, L, rope):
    _rowln_qkv_check(lib, B, T, L, rope)


def test_rowln_qkv_frame_tiles():
    """MDG_RQ_FRAMES=1 (frame tiles, read once per process): the L % 16 == 0 cases in a child
    process, each against the two-launch path bit for bit."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r); from tests.test_gpu_kernels import _rowln_qkv_check; "
            "from mdgen_finetune_amd import _lib; lib = _lib.load(); "
            "[_rowln_qkv_check(lib, *c) for c in [(2, 37, 32, True), (3, 9, 16, True), (1, 250, 256, True), "
            "(1, 12, 48, False)]]; print('ok')") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MDG_RQ_FRAMES="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def _rowln_qkv_check(lib, B, T, L, rope):
    """mdg_rowln_qkv (spatial out_proj + gated residual + LN_t, then the temporal q|k|v into
    packed planes, LN_t(h) on chip) against the same two descriptors through mdg_gemm: h
    bit-identical (the same row-LN epilogue); q|k|v bit-identical too (the same bf16 LN rows,
    the same K order, the same epilogue arithmetic).  Partial last tiles
    (M % 128 != 0), tiles over two trajectories, with and without RoPE; xn is not written.
    With MDG_RQ_FRAMES=1 (test_rowln_qkv_frame_tiles), L % 16 == 0 takes the frame tiles (8
    frames x 16 residues; a ragged last frame group when B T % 8 != 0, groups across trajectory
    boundaries when T % 8 != 0)."""
    from mdgen_finetune_amd import _lib

    H, D = 16, 24
    C, M, TL = H * D, B * T * L, T * L
    g = torch.Generator(device="cuda").manual_seed(M + T)
    o = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    Wo = (torch.randn(C, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    bo = torch.randn(C, device="cuda", generator=g) * 0.5
    Wq = (torch.randn(3 * C, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    bq = torch.randn(3 * C, device="cuda", generator=g) * 0.5
    mods = torch.randn(B, 9 * C, device="cuda", generator=g) * 0.5
    h0 = torch.randn(M, C, device="cuda", generator=g) * 2
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2).float() / D))
    f = torch.arange(T + 1).float()[:, None] * inv
    table = torch.cat([f.cos().reshape(-1), f.sin().reshape(-1)]).cuda()
    outs = []
    for fused in (False, True):
        h = h0.clone()
        xo = torch.zeros(M, C, device="cuda", dtype=torch.bfloat16)
        planes = torch.zeros(3, B * L, H, T, D, device="cuda", dtype=torch.bfloat16)
        r = _desc(dtype=1, a_mode=0, epi=1, M=M, N=C, K=C, A=o.data_ptr(), lda=C, W=Wo.data_ptr(), ldw=C,
                  bias=bo.data_ptr(), mod_stride=9 * C, rows_per_mod=TL, resid=h.data_ptr(), ldr=C,
                  gate=mods.data_ptr(), gate_off=2 * C, xn_out=xo.data_ptr(), xn_mods=mods.data_ptr(),
                  xn_mod_stride=9 * C, xn_shift_off=3 * C, xn_scale_off=4 * C, ln_eps=1e-6)
        q = _desc(dtype=1, a_mode=0, epi=2, M=M, N=3 * C, K=C, A=xo.data_ptr(), lda=C, W=Wq.data_ptr(), ldw=C,
                  bias=bq.data_ptr(), qkv_layout=2, qkv_out=planes.data_ptr(), H=H, D=D, T=T, L=L, qscale=0.3,
                  rope=table.data_ptr() if rope else 0, rope_rows=T + 1)
        if fused:
            _lib.check(lib.mdg_rowln_qkv(ctypes.byref(r), ctypes.byref(q), _s()), "mdg_rowln_qkv")
        else:
            _lib.check(lib.mdg_gemm(ctypes.byref(r), _s()), "out_proj")
            _lib.check(lib.mdg_gemm(ctypes.byref(q), _s()), "qkv")
        outs.append((h, xo, planes))
    torch.cuda.synchronize()
    (h_ref, x_ref, p_ref), (h_f, x_f, p_f) = outs
    b = torch.arange(M, device="cuda") // TL
    href = h0 + mods[b, 2 * C:3 * C] * (o.float() @ Wo.float().T + bo)
    torch.testing.assert_close(h_f, href, rtol=5e-3, atol=5e-3)
    assert torch.equal(h_f, h_ref), (h_f - h_ref).abs().max().item()
    assert not x_f.any()  # LN_t(h) stayed on chip
    assert x_ref.any()
    # (both epilogues: + bias, x qscale, RoPE with explicit fma -> bf16)
    assert torch.equal(p_f, p_ref), ((p_f.float() - p_ref.float()).abs().max().item(), int((p_f != p_ref).sum()))


def test_rowln_qkv_rejects_unsupported_shapes(lib):
    r = _desc(dtype=1, a_mode=0, epi=1, M=256, N=384, K=384, A=1, lda=384, W=1, ldw=384, resid=1, ldr=384,
              rows_per_mod=256, xn_out=1, xn_mods=1)
    q = _desc(dtype=1, a_mode=0, epi=2, M=256, N=3 * 384, K=384, A=1, lda=384, W=1, ldw=384, qkv_layout=1,
              qkv_out=1, H=16, D=24, T=64, L=4)
    assert lib.mdg_rowln_qkv(ctypes.byref(r), ctypes.byref(q), _s()) == 1001  # padded planes
    q.qkv_layout = 2
    r.rows_per_mod = 64  # tiles over > 2 trajectories
    assert lib.mdg_rowln_qkv(ctypes.byref(r), ctypes.byref(q), _s()) == 1001
    r.rows_per_mod = 256
    q.H, q.D = 6, 64  # head_dim > 48
    assert lib.mdg_rowln_qkv(ctypes.byref(r), ctypes.byref(q), _s()) == 1001


def _rope_ref(x, pos, inv_freq):
    # x [..., D] at integer positions pos [...]
    half = x.shape[-1] // 2
    f = pos[..., None].float() * inv_freq
    c, s = torch.cat([f.cos(), f.cos()], -1), torch.cat([f.sin(), f.sin()], -1)
    rot = torch.cat([-x[..., half:], x[..., :half]], -1)
    return x * c + rot * s


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("layout", [0, 1])
def test_gemm_qkv_rope_layouts(lib, dt, layout):
    from mdgen_finetune_amd import _lib

    B, T, L, H, D = 2, 37, 4, 16, 24
    C, M = H * D, B * T * L
    g = torch.Generator(device="cuda").manual_seed(5 + layout)
    A = torch.randn(M, C, device="cuda", generator=g)
    W = (torch.randn(3 * C, C, device="cuda", generator=g) / math.sqrt(C)).to(CT[dt])
    bias = torch.randn(3 * C, device="cuda", generator=g)
    mods = torch.randn(B, 9 * C, device="cuda", generator=g) * 0.3
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2).float() / D))
    S = (L if layout == 0 else T) + 1
    f = torch.arange(S).float()[:, None] * inv
    table = torch.cat([f.cos().reshape(-1), f.sin().reshape(-1)]).cuda()
    qs = 0.2
    if layout == 0:
        out = torch.zeros(M, 3, H, D, device="cuda", dtype=CT[dt])     # unpadded spatial layout
    else:
        out = torch.zeros(3, B * L, H, T, 32, device="cuda", dtype=CT[dt])
    # the kernel contract: q/k head rows pair-interleaved (row 2i = dim i, 2i+1 = dim i + D/2)
    idx = torch.arange(D)
    within = torch.where(idx % 2 == 0, idx // 2, idx // 2 + D // 2)
    perm = (torch.arange(H)[:, None] * D + within[None]).reshape(-1).cuda()
    full = torch.cat([perm, perm + C, torch.arange(2 * C, 3 * C, device="cuda")])
    Wi, bi = W[full].contiguous(), bias[full].contiguous()
    d = _desc(dtype=ENUM[dt], a_mode=1, epi=2, M=M, N=3 * C, K=C, A=A.data_ptr(), lda=C, W=Wi.data_ptr(), ldw=C,
              bias=bi.data_ptr(), mods=mods.data_ptr(), mod_stride=9 * C, rows_per_mod=T * L, shift_off=0,
              scale_off=C, ln_eps=1e-6, qkv_layout=layout, qkv_out=out.data_ptr(), H=H, D=D, T=T, L=L, qscale=qs,
              rope=table.data_ptr(), rope_rows=S)
    _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "mdg_gemm")
    y = _ln_mod(A, mods, T * L, 0, C, C).to(CT[dt]).float()
    p = (y @ W.float().T + bias).reshape(B, T, L, 3, H, D)
    pos = (torch.arange(L) if layout == 0 else torch.arange(T)).cuda()
    posb = pos.reshape(1, 1, L, 1) if layout == 0 else pos.reshape(1, T, 1, 1)
    posb = posb.expand(B, T, L, H)
    q = _rope_ref(p[..., 0, :, :] * qs, posb, inv.cuda())
    k = _rope_ref(p[..., 1, :, :], posb, inv.cuda())
    v = p[..., 2, :, :]
    q, k = q[..., within.cuda()], k[..., within.cuda()]           # stored interleaved
    ref = torch.stack([q, k, v], 3)                               # [B,T,L,3,H,D]
    if layout == 0:
        got = out.float().reshape(B, T, L, 3, H, D)
    else:
        got = out.float().reshape(3, B, L, H, T, 32).permute(1, 4, 2, 0, 3, 5)
    rtol, atol = _tol(dt)
    torch.testing.assert_close(got[..., :D], ref, rtol=rtol, atol=atol * 5)
    assert torch.all(got[..., D:] == 0)


def _attn_ref(q, k, v, kb, vb, keyvalid, base2):
    # q [N,S,D], k/v [N,S,D], bias row kb/vb [D]; keyvalid [N,S]
    N, S, D = q.shape
    kk = torch.cat([k, kb.expand(N, 1, D)], 1)
    vv = torch.cat([v, vb.expand(N, 1, D)], 1)
    s = q @ kk.transpose(1, 2)
    if base2:
        s = s * math.log(2.0)
    valid = torch.cat([keyvalid, torch.ones(N, 1, dtype=torch.bool, device=q.device)], 1)
    s = s.masked_fill(~valid[:, None, :], float("-inf"))
    return torch.softmax(s, -1) @ vv


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("T", [1, 63, 64, 129, 600, 1000, 1024, 1300])
def test_attn_temporal(lib, dt, T):
    from mdgen_finetune_amd import _lib

    B, L, H, D = 1, 3, 4, 24
    BL = B * L
    g = torch.Generator(device="cuda").manual_seed(T)
    qkv = torch.zeros(3, BL, H, T, 32, device="cuda")
    qkv[..., :D] = torch.randn(3, BL, H, T, D, device="cuda", generator=g)
    qkv[1:, ..., D] = 1.0                       # k / v pad column D (softmax offset / row sum)
    qkv = qkv.to(CT[dt])
    mask = torch.ones(B, T, L, device="cuda")
    if T > 3:
        mask[:, T // 3: T // 2, 1] = 0          # a padded run of keys in sequence 1
        mask[:, :, 2] = 0                        # every key of sequence 2 padded: bias row only
    kvb = torch.zeros(H, 2, 32, device="cuda")
    kvb[:, :, :D] = torch.randn(H, 2, D, device="cuda", generator=g)
    kvb[:, 1, D] = 1.0
    kbias = torch.where(mask.permute(0, 2, 1).reshape(BL, T) != 0, 0.0, float("-inf")).contiguous()
    out = torch.zeros(B * T * L, H * D, device="cuda", dtype=CT[dt])
    _lib.check(lib.mdg_attn_temporal(ENUM[dt], B, T, L, H, D, qkv.data_ptr(), kbias.data_ptr(), kvb.data_ptr(),
                                     out.data_ptr(), _s()), "attn_temporal")
    qf = qkv.float()
    got = out.float().reshape(B, T, L, H, D)
    for h in range(H):
        ref = _attn_ref(qf[0, :, h, :, :D], qf[1, :, h, :, :D], qf[2, :, h, :, :D], kvb[h, 0, :D], kvb[h, 1, :D],
                        mask.permute(0, 2, 1).reshape(BL, T) != 0, base2=True)  # [BL, T, D]
        rtol, atol = _tol(dt)
        torch.testing.assert_close(got[0, :, :, h].permute(1, 0, 2), ref, rtol=rtol * 2, atol=atol * 2)


@pytest.mark.parametrize("qmul", [4.0, 40.0])
def test_attn_temporal_large_scores(lib, qmul):
    """Scores far above the bias key's: x4 (up to ~100 in log2 units: the optimistic pass,
    P up to ~2^100, stays finite) and x40 (overflows: the block reruns with the growth-tested
    offset).  Both against the fp32 softmax of the same bf16 operands."""
    from mdgen_finetune_amd import _lib

    B, L, H, D, T = 1, 2, 4, 24, 700
    BL = B * L
    g = torch.Generator(device="cuda").manual_seed(int(qmul))
    qkv = torch.zeros(3, BL, H, T, 32, device="cuda")
    qkv[..., :D] = torch.randn(3, BL, H, T, D, device="cuda", generator=g)
    qkv[0, ..., :D] *= qmul
    qkv[1:, ..., D] = 1.0
    qkv = qkv.to(torch.bfloat16)
    kvb = torch.zeros(H, 2, 32, device="cuda")
    kvb[:, :, :D] = 0.1 * torch.randn(H, 2, D, device="cuda", generator=g)
    kvb[:, 1, D] = 1.0
    kbias = torch.zeros(BL, T, device="cuda")
    out = torch.zeros(B * T * L, H * D, device="cuda", dtype=torch.bfloat16)
    _lib.check(lib.mdg_attn_temporal(1, B, T, L, H, D, qkv.data_ptr(), kbias.data_ptr(), kvb.data_ptr(),
                                     out.data_ptr(), _s()), "attn_temporal")
    qf = qkv.float()
    got = out.float().reshape(B, T, L, H, D)
    assert torch.isfinite(got).all()
    for h in range(H):
        ref = _attn_ref(qf[0, :, h, :, :D], qf[1, :, h, :, :D], qf[2, :, h, :, :D], kvb[h, 0, :D], kvb[h, 1, :D], torch.ones(BL, T, dtype=torch.bool, device="cuda"),
                        base2=True)
        rtol, atol = _tol("bf16")
        torch.testing.assert_close(got[0, :, :, h].permute(1, 0, 2), ref, rtol=rtol * 2, atol=atol * 2)


@pytest.mark.parametrize("T,D", [(1, 24), (63, 24), (1000, 24), (1300, 16), (129, 8)])
def test_attn_temporal_packed_equals_padded(lib, T, D):
    """Packed planes (row stride D, pad column synthesised while staging) give the padded
    kernel's output bit for bit; the packed q|k|v GEMM layout is the padded one minus the pads."""
    from mdgen_finetune_amd import _lib

    B, L, H = 1, 3, 4
    BL = B * L
    g = torch.Generator(device="cuda").manual_seed(T + D)
    pad = torch.zeros(3, BL, H, T, 32, device="cuda")
    pad[..., :D] = torch.randn(3, BL, H, T, D, device="cuda", generator=g)
    pad[1:, ..., D] = 1.0
    pad = pad.to(torch.bfloat16)
    packed = pad[..., :D].contiguous()
    mask = torch.ones(B, T, L, device="cuda")
    if T > 3:
        mask[:, T // 3: T // 2, 1] = 0
        mask[:, :, 2] = 0
    kvb = torch.zeros(H, 2, 32, device="cuda")
    kvb[:, :, :D] = torch.randn(H, 2, D, device="cuda", generator=g)
    kvb[:, 1, D] = 1.0
    kbias = torch.where(mask.permute(0, 2, 1).reshape(BL, T) != 0, 0.0, float("-inf")).contiguous()
    o1 = torch.zeros(B * T * L, H * D, device="cuda", dtype=torch.bfloat16)
    o2 = torch.zeros_like(o1)
    _lib.check(lib.mdg_attn_temporal(1, B, T, L, H, D, pad.data_ptr(), kbias.data_ptr(), kvb.data_ptr(),
                                     o1.data_ptr(), _s()), "attn_temporal")
    _lib.check(lib.mdg_attn_temporal_packed(1, B, T, L, H, D, packed.data_ptr(), kbias.data_ptr(), kvb.data_ptr(),
                                            o2.data_ptr(), _s()), "attn_temporal_packed")
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert lib.mdg_attn_temporal_packed(1, B, T, L, H, 20, packed.data_ptr(), kbias.data_ptr(), kvb.data_ptr(),
                                        o2.data_ptr(), _s()) == 1001  # D % 8 != 0: refused


def test_gemm_qkv_packed_layout_is_padded_minus_pads(lib):
    from mdgen_finetune_amd import _lib

    B, T, L, H, D = 2, 37, 4, 16, 24
    C, M = H * D, B * T * L
    g = torch.Generator(device="cuda").manual_seed(77)
    A = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    W = (torch.randn(3 * C, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    bias = torch.randn(3 * C, device="cuda", generator=g)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2).float() / D))
    f = torch.arange(T + 1).float()[:, None] * inv
    table = torch.cat([f.cos().reshape(-1), f.sin().reshape(-1)]).cuda()
    outs = []
    for layout, shape in ((1, (3, B * L, H, T, 32)), (2, (3, B * L, H, T, D))):
        out = torch.zeros(*shape, device="cuda", dtype=torch.bfloat16)
        d = _desc(dtype=1, a_mode=0, epi=2, M=M, N=3 * C, K=C, A=A.data_ptr(), lda=C, W=W.data_ptr(), ldw=C,
                  bias=bias.data_ptr(), qkv_layout=layout, qkv_out=out.data_ptr(), H=H, D=D, T=T, L=L, qscale=0.3,
                  rope=table.data_ptr(), rope_rows=T + 1)
        _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "mdg_gemm")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][..., :D], outs[1])


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("L,D", [(5, 24), (4, 24), (4, 16)])   # L == 4: DPP quad kernel
def test_attn_spatial(lib, dt, L, D):
    from mdgen_finetune_amd import _lib

    NF, H = 50, 16
    g = torch.Generator(device="cuda").manual_seed(1)
    qkv = torch.randn(NF * L, 3, H, D, device="cuda", generator=g).to(CT[dt])   # unpadded [token][3][H][D]
    mask = torch.ones(NF, L, device="cuda")
    mask[::3, 2] = 0
    mask[1::7, :] = 0
    kvb = torch.zeros(H, 2, 32, device="cuda")
    kvb[:, :, :D] = torch.randn(H, 2, D, device="cuda", generator=g)
    out = torch.zeros(NF * L, H * D, device="cuda", dtype=CT[dt])
    _lib.check(lib.mdg_attn_spatial(ENUM[dt], NF, L, H, D, qkv.data_ptr(), kvb.data_ptr(), mask.data_ptr(),
                                    out.data_ptr(), _s()), "attn_spatial")
    qf = qkv.float().reshape(NF, L, 3, H, D)
    got = out.float().reshape(NF, L, H, D)
    for h in range(H):
        ref = _attn_ref(qf[:, :, 0, h, :D], qf[:, :, 1, h, :D], qf[:, :, 2, h, :D], kvb[h, 0, :D], kvb[h, 1, :D],
                        mask != 0, base2=False)
        rtol, atol = _tol(dt)
        torch.testing.assert_close(got[:, :, h], ref, rtol=rtol * 2, atol=atol * 2)


def test_embed(lib):
    from mdgen_finetune_amd import _lib

    B, T, L, C, K = 2, 10, 4, 384, 21
    N = B * T * L
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(N, K, device="cuda", generator=g)
    W = torch.randn(C, K, device="cuda", generator=g)
    bias = torch.randn(C, device="cuda", generator=g)
    pos = torch.randn(L, C, device="cuda", generator=g)
    emb = torch.randn(2, C, device="cuda", generator=g)
    idx = torch.randint(0, 2, (N,), device="cuda", generator=g)
    ipa = torch.randn(B * L, C, device="cuda", generator=g)
    out = torch.empty(N, C, device="cuda")
    Wt = W.t().contiguous()
    _lib.check(lib.mdg_embed(N, T, L, C, K, x.data_ptr(), Wt.data_ptr(), bias.data_ptr(), None, pos.data_ptr(),
                             emb.data_ptr(), idx.data_ptr(), ipa.data_ptr(), out.data_ptr(), _s()), "embed")
    n = torch.arange(N, device="cuda")
    ref = x @ W.T + bias + pos[n % L] + emb[idx] + ipa[(n // (T * L)) * L + n % L]
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)



@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_final_euler_gemm(lib, dt):
    from mdgen_finetune_amd import _lib

    B, T, L, C, K = 2, 10, 4, 384, 21
    N = B * T * L
    g = torch.Generator(device="cuda").manual_seed(4)
    h = torch.randn(N, C, device="cuda", generator=g) * 2
    Wf = torch.zeros(32, C, device="cuda")
    Wf[:K] = torch.randn(K, C, device="cuda", generator=g) / 20
    bf = torch.zeros(32, device="cuda")
    bf[:K] = torch.randn(K, device="cuda", generator=g)
    mods = torch.randn(B, 2 * C, device="cuda", generator=g) * 0.3
    xin = torch.randn(N, K, device="cuda", generator=g)
    xo = torch.empty_like(xin)
    vo = torch.empty_like(xin)
    Wc = Wf.to(CT[dt]).contiguous()
    _lib.check(lib.mdg_final_euler(ENUM[dt], N, T * L, C, K, Wc.data_ptr(), bf.data_ptr(), mods.data_ptr(),
                                   h.data_ptr(), xin.data_ptr(), 0.25, xo.data_ptr(), vo.data_ptr(), _s()),
               "final_euler")
    n = torch.arange(N, device="cuda")
    b = n // (T * L)
    y = torch.nn.functional.layer_norm(h, (C,), eps=1e-6) * (1 + mods[b, C:]) + mods[b, :C]
    vref = y.to(CT[dt]).float() @ Wc.float()[:K].T + bf[:K]
    rtol, atol = _tol(dt)
    torch.testing.assert_close(vo, vref, rtol=rtol, atol=atol * 10)
    torch.testing.assert_close(xo, xin + 0.25 * vo, rtol=0, atol=1e-6)


@pytest.mark.parametrize("M,masked", [(4000, True), (132, False), (8, True)])
def test_gemm_qkv_attn_spatial_fused(lib, M, masked):
    """bf16 spatial q|k|v projection + 4-residue attention in one launch (MDG_EPI_ATTN_SPATIAL:
    gemm_qkv_attn_spatial_kernel) vs a torch fp32 reference of projection -> RoPE -> softmax
    over the bias key + unmasked residues -> P.V (latent_model.py:466-470, mha.py:255-397)."""
    from mdgen_finetune_amd import _lib

    H, D, L = 16, 24, 4
    C, NF = H * D, M // L
    g = torch.Generator(device="cuda").manual_seed(M)
    A = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    W = (torch.randn(3 * C, C, device="cuda", generator=g) / math.sqrt(C)).to(torch.bfloat16)
    bias = torch.randn(3 * C, device="cuda", generator=g) * 0.1
    inv = (1.0 / (10000 ** (torch.arange(0, D, 2).float() / D))).cuda()
    f = torch.arange(L + 1).float().cuda()[:, None] * inv
    table = torch.cat([f.cos().reshape(-1), f.sin().reshape(-1)]).contiguous()
    qs = D ** -0.5
    idx = torch.arange(D)
    within = torch.where(idx % 2 == 0, idx // 2, idx // 2 + D // 2).cuda()
    perm = (torch.arange(H, device="cuda")[:, None] * D + within[None]).reshape(-1)
    full = torch.cat([perm, perm + C, torch.arange(2 * C, 3 * C, device="cuda")])
    Wi, bi = W[full].contiguous(), bias[full].contiguous()
    kb = torch.randn(H, D, device="cuda", generator=g)
    vb = torch.randn(H, D, device="cuda", generator=g)
    kb_rot = _rope_ref(kb, torch.full((H,), L, device="cuda"), inv)   # bias_k at position S = L
    kvb = torch.zeros(H, 2, 32, device="cuda")
    kvb[:, 0, :D] = kb_rot[:, within]
    kvb[:, 1, :D] = vb
    kvb[:, 1, D] = 1.0
    mask = torch.ones(NF, L, device="cuda")
    if masked:
        mask[::3, 2] = 0
        mask[1::7, :] = 0
    out = torch.zeros(M, C, device="cuda", dtype=torch.bfloat16)
    d = _desc(dtype=1, a_mode=0, epi=_lib.MDG_EPI_ATTN_SPATIAL, M=M, N=3 * C, K=C, A=A.data_ptr(), lda=C,
              W=Wi.data_ptr(), ldw=C, bias=bi.data_ptr(), H=H, D=D, T=1, L=L, qscale=qs, rope=table.data_ptr(),
              rope_rows=L + 1, out=out.data_ptr(), ldo=C, kvb=kvb.data_ptr(), key_mask=mask.data_ptr())
    _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "mdg_gemm ATTN_SPATIAL")
    p = (A.float() @ W.float().T + bias).reshape(NF, L, 3, H, D)
    pos = torch.arange(L, device="cuda").reshape(1, L, 1).expand(NF, L, H)
    q = _rope_ref(p[:, :, 0] * qs, pos, inv)
    k = _rope_ref(p[:, :, 1], pos, inv)
    v = p[:, :, 2]
    got = out.float().reshape(NF, L, H, D)
    for h in range(H):
        ref = _attn_ref(q[:, :, h], k[:, :, h], v[:, :, h], kb_rot[h], vb[h], mask != 0, base2=False)
        torch.testing.assert_close(got[:, :, h], ref, rtol=2e-2, atol=2e-2)


def test_gemm_attn_spatial_rejects_unsupported_shapes(lib):
    from mdgen_finetune_amd import _lib

    x = torch.zeros(64, device="cuda")
    d = _desc(dtype=1, a_mode=0, epi=_lib.MDG_EPI_ATTN_SPATIAL, M=8, N=3 * 64, K=64, A=x.data_ptr(), lda=64,
              W=x.data_ptr(), ldw=64, H=4, D=16, L=4, out=x.data_ptr(), ldo=64, kvb=x.data_ptr())
    assert lib.mdg_gemm(ctypes.byref(d), _s()) == 1001  # D != 24: the two-launch path covers it


def _euler_desc(xn, W, b, xin, xo, vo, latent, dt):
    from mdgen_finetune_amd import _lib

    d = _lib.MdgGemmDesc()
    M, C = xn.shape
    d.dtype, d.a_mode, d.epi, d.M, d.N, d.K = 1, 0, 3, M, W.shape[0], C
    d.A, d.lda, d.W, d.ldw, d.bias = xn.data_ptr(), C, W.data_ptr(), C, b.data_ptr()
    d.out, d.ldo, d.x_in, d.v_out, d.dt, d.n_valid = xo.data_ptr(), latent, xin.data_ptr(), vo.data_ptr(), dt, latent
    return d


@pytest.mark.parametrize("M,C,latent", [(37, 384, 21), (1000, 384, 21), (32000, 384, 21), (4100, 384, 28),
                                        (640, 128, 32), (333, 512, 21), (96, 256, 7)])
def test_final_euler_plain_bf16(lib, M, C, latent):
    """bf16 FinalLayer + Euler on the LN'd operand (the denoise step's last launch:
    final_euler_kernel via mdg_gemm): equal bit for bit to the generic EULER GEMM (forced by
    an N = 64 descriptor: the same K order on the same MFMA), and to the fp32 product of the
    bf16 operands within accumulation-order rounding; x_out = x_in + dt * v exactly."""
    from mdgen_finetune_amd import _lib

    g = torch.Generator(device="cuda").manual_seed(M + C + latent)
    xn = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    W = torch.zeros(64, C, device="cuda")
    W[:latent] = torch.randn(latent, C, device="cuda", generator=g) / C ** 0.5
    W = W.to(torch.bfloat16)
    b = torch.zeros(64, device="cuda")
    b[:latent] = torch.randn(latent, device="cuda", generator=g)
    xin = torch.randn(M, latent, device="cuda", generator=g)
    outs = []
    for n in (32, 64):  # 32: final_euler_kernel; 64: the generic GEMM
        xo = torch.full_like(xin, float("nan"))
        vo = torch.full_like(xin, float("nan"))
        d = _euler_desc(xn, W[:n].contiguous(), b[:n].contiguous(), xin, xo, vo, latent, 0.375)
        _lib.check(lib.mdg_gemm(ctypes.byref(d), _s()), "euler gemm")
        outs.append((xo, vo))
    torch.cuda.synchronize()
    (xo, vo), (xo_g, vo_g) = outs
    assert torch.equal(vo, vo_g) and torch.equal(xo, xo_g)
    vref = xn.float() @ W.float()[:latent].T + b[:latent]
    torch.testing.assert_close(vo, vref, rtol=1e-5, atol=1e-5)
    assert torch.equal(xo, xin + 0.375 * vo)
