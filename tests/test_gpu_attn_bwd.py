"""mdg_attn_temporal_bwd (csrc/train.hip) against fp32 torch autograd of the same attention, at
the sizes config 3 trains: T = 129, 257 and 1000 frames (2, 3 and 8 chunks of 128 keys /
queries, with tails), head_dim 24 (C = 384, 16 heads), the bias_k / bias_v virtual key, RoPE
(fair-esm, bias key at position T) and key padding.  Reference op: the temporal
MultiheadAttention under loss.backward() (reference src/mdgen/model/mha.py:255-397, the
backward of 359-389; latent_model.py:482-486).

The operands are built in the kernel's own basis (q / k columns pair-interleaved per head, so
RoPE rotates neighbouring columns): q' = rope(q_lin * D^-1/2), k' = rope(k_lin), planes
[BL][H][T][32] with q' * log2(e) in the q plane and 1.0 in pad column D of the k / v planes,
lse the per-row log2-sum-exp2.  The reference differentiates
    o = softmax([q'.bk, q'.k' + kbias]) [bv; v]
with respect to q_lin, k_lin, v, bk, bv (fp64 on the device).  Bounds: f32 (scalar kernels)
||d|| / ||ref|| <= 1e-5; bf16 (MFMA kernels: P and dS rounded to bf16 as MFMA operands)
<= BF16_TOL, ~2x the worst observed (logged to MDG_PARITY_LOG).  n_pad = -1: one sequence has
every key padded (a padded residue's temporal attention: P = [1, 0, ...], exact dS = 0), which
the bf16 path gets right only through o_lo (delta = dO . (o + o_lo))."""
import json
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

BF16_TOL = 2e-2


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def _rope_tab(rows, D):
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2).float() / D))
    f = torch.einsum("i,j->ij", torch.arange(rows).float(), inv)
    return f.cos(), f.sin()


def _rope(x, cos, sin):
    """x [..., T, D] in the pair-interleaved basis; rotation of pair i at row position t."""
    a, b = x[..., 0::2], x[..., 1::2]
    out = torch.empty_like(x)
    out[..., 0::2] = a * cos - b * sin
    out[..., 1::2] = b * cos + a * sin
    return out


def _case(T, BL, H, D, n_pad_keys, seed, dev="cuda"):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)  # noqa: E731
    q_lin, k_lin, v = r(BL, H, T, D), r(BL, H, T, D), r(BL, H, T, D)
    bk_lin, bv = r(H, D), r(H, D)
    dout = r(BL, H, T, D)
    kbias = torch.zeros(BL, T, dtype=torch.float64)
    if n_pad_keys < 0:  # sequence 1 entirely padded (a padded residue): only the bias key is valid
        kbias[0, T - 3:] = -math.inf
        kbias[1, :] = -math.inf
    elif n_pad_keys:  # pad the tail frames of sequence 0 and a scattered set of sequence 1
        kbias[0, T - n_pad_keys:] = -math.inf
        if BL > 1:
            kbias[1, torch.randperm(T, generator=g)[:n_pad_keys]] = -math.inf
    return {k: v.to(dev) for k, v in dict(q_lin=q_lin, k_lin=k_lin, v=v, bk_lin=bk_lin, bv=bv, dout=dout,
                                         kbias=kbias).items()}


def _forward(c, D, T, cos, sin, qscale):
    """o (natural units) from differentiable inputs; bias key rotated at position T."""
    qn = _rope(c["q_lin"] * qscale, cos[:T], sin[:T])
    kr = _rope(c["k_lin"], cos[:T], sin[:T])
    bk = _rope(c["bk_lin"][:, None, :], cos[T:T + 1], sin[T:T + 1])[:, 0]  # [H, D]
    s = torch.einsum("shtd,shud->shtu", qn, kr) + c["kbias"][:, None, None, :]
    sb = torch.einsum("shtd,hd->sht", qn, bk)[..., None]
    p = torch.softmax(torch.cat([sb, s], -1), -1)
    o = p[..., :1] * c["bv"][None, :, None, :] + torch.einsum("shtu,shud->shtd", p[..., 1:], c["v"])
    return o, qn, kr, bk, torch.cat([sb, s], -1)


@pytest.mark.parametrize("dtype", ["bf16", "bf16-2pass", "f32"])
@pytest.mark.parametrize("T,n_pad", [(129, 0), (257, 5), (1000, 17), (300, -1), (40, 3), (513, 0)])
def test_temporal_attention_backward_multi_chunk(dtype, T, n_pad):
    """bf16: the fused single-pass kernel (generic 0: one block per (sequence, head), 256-key
    passes, 64-query chunks: T = 257 / 300 / 513 / 1000 take 2-4 passes with ragged tails);
    bf16-2pass: the two-pass MFMA kernels (generic 2); f32: the scalar kernels."""
    generic = 2 if dtype == "bf16-2pass" else 0
    _run_bwd(dtype.split("-")[0], T, n_pad, generic)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("H,D,T,n_pad", [(8, 32, 129, 5), (8, 48, 300, -1), (6, 60, 40, 3)])
def test_temporal_attention_backward_wide_heads(dtype, H, D, T, n_pad):
    """head_dim 32..63 (--embed_dim 256 --mha_heads 8 and the like; mha.py:96-102 takes any
    embed_dim // num_heads): 64-column planes (MDG_HEAD_STRIDE), generic 1 (the only value these
    heads take): bf16 on the wide MFMA kernels (round 6: each 64-column row as two 32-column
    halves, P / dS rounded to bf16 as in the head_dim-24 kernels), f32 on the scalar ones; O's
    bf16 residual from the wide forward kernel."""
    _run_bwd(dtype, T, n_pad, 1, H=H, D=D)


@pytest.mark.parametrize("H,D,T,n_pad", [(8, 32, 257, 9), (6, 60, 129, -1)])
def test_temporal_attention_backward_wide_heads_scalar_route(H, D, T, n_pad):
    """The bf16 wide heads' scalar kernels (MDG_ATTN_BWD_WIDE_MFMA=0, the round-5 route) stay
    correct: run in a child process, since the knob is read once per process."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, '.'); from tests.test_gpu_attn_bwd import _run_bwd; "
            f"_run_bwd('bf16', {T}, {n_pad}, 1, H={H}, D={D}); print('ok')")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MDG_ATTN_BWD_WIDE_MFMA="0"),
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_temporal_attention_backward_wide_heads_refuses_mfma_variants():
    """The MFMA variants' LDS images are 32 columns wide: a bf16 call with head_dim >= 32 and
    generic 0 / 2 is refused (its bias slots would not match mdg_attn_temporal_bwd_parts)."""
    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    dev = "cuda"
    B, T, L, H, D = 1, 16, 2, 8, 32
    z = lambda n, dt=torch.bfloat16: torch.zeros(n, device=dev, dtype=dt)  # noqa: E731
    rows = B * L * H * T
    for generic in (0, 2):
        rc = lib.mdg_attn_temporal_bwd(_lib.MDG_BF16, B, T, L, H, D, z(3 * rows * 64).data_ptr(),
                                       z(B * L * T, torch.float32).data_ptr(), z(H * 128, torch.float32).data_ptr(),
                                       z(rows * D).data_ptr(), None, z(rows * D).data_ptr(),
                                       z(rows, torch.float32).data_ptr(), None, T + 1,
                                       z(lib.mdg_attn_temporal_bwd_scratch(_lib.MDG_BF16, B, T, L, H, D)).data_ptr(),
                                       z(B * T * L * 3 * H * D).data_ptr(), 3 * H * D,
                                       z(H * 64 * 128, torch.float32).data_ptr(), 1.0, 1.0, generic,
                                       _lib.stream_handle())
        assert rc != 0 and b"generic" in lib.mdg_last_error_string()
    assert lib.mdg_attn_temporal_bwd_scratch(_lib.MDG_BF16, B, T, L, H, 64) == 0


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("D", [24, 48])
def test_spatial_long_route_backward_shape(dtype, D):
    """The shape the L >= 16 spatial attention hands these kernels: B*T sequences of L = 16 keys,
    one residue each (Lq = 1), padded keys."""
    _run_bwd(dtype, 16, 3, 1 if D >= 32 else 0, H=8, D=D, B=10, L=1)


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("B,T,L,H,D", [(10, 16, 1, 8, 48), (2, 5, 16, 8, 48), (10, 16, 1, 12, 32), (1, 300, 2, 8, 48),
                                       (10, 16, 1, 16, 24)])
def test_temporal_attention_forward_lse(dtype, B, T, L, H, D):
    """mdg_attn_temporal_lse (the training forward: O, its bf16 residual, the log2-sum-exp2 rows)
    against fp64 torch on the same CT operands, narrow and wide heads."""
    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    dev = "cuda"
    BL, C, DP = B * L, H * D, _lib.head_stride(D)
    ct = torch.bfloat16 if dtype == "bf16" else torch.float32
    mdt = _lib.MDG_BF16 if dtype == "bf16" else _lib.MDG_F32
    c = _case(T, BL, H, D, 3, seed=7 * T + D)
    log2e = 1.0 / math.log(2.0)
    planes = torch.zeros(3, BL, H, T, DP, device=dev, dtype=ct)
    planes[0, ..., :D] = (c["q_lin"] * D ** -0.5 * log2e).to(ct)
    planes[1, ..., :D] = c["k_lin"].to(ct)
    planes[2, ..., :D] = c["v"].to(ct)
    planes[1, ..., D] = 1.0
    planes[2, ..., D] = 1.0
    qp, kp, vp = (planes[i, ..., :D].double() for i in range(3))
    kvb = torch.zeros(H, 2, DP, device=dev)
    kvb[:, 0, :D] = c["bk_lin"].float()
    kvb[:, 1, :D] = c["bv"].float()
    kvb[:, 1, D] = 1.0  # the bias value row's pad column carries the bias key's share of the row sum
    s2 = torch.einsum("shtd,shud->shtu", qp, kp) + c["kbias"][:, None, None, :]
    sb2 = torch.einsum("shtd,hd->sht", qp, kvb[:, 0, :D].double())[..., None]
    s2 = torch.cat([sb2, s2], -1)
    lse = torch.logsumexp(s2 * math.log(2.0), -1) * log2e
    p2 = torch.exp2(s2 - lse[..., None])
    o = p2[..., :1] * kvb[None, :, 1, None, :D].double() + torch.einsum("shtu,shud->shtd", p2[..., 1:], vp)
    o_ref = o.reshape(B, L, H, T, D).permute(0, 3, 1, 2, 4).reshape(B * T * L, C)
    out = torch.full((B * T * L, C), float("nan"), device=dev, dtype=ct)
    lo = torch.full_like(out, float("nan")) if dtype == "bf16" else None
    lse_k = torch.full((BL, H, T), float("nan"), device=dev)
    _lib.check(lib.mdg_attn_temporal_lse(mdt, B, T, L, H, D, planes.data_ptr(), c["kbias"].float().contiguous().data_ptr(),
                                         kvb.data_ptr(), out.data_ptr(), _lib.ptr(lo), lse_k.data_ptr(),
                                         _lib.stream_handle()), "mdg_attn_temporal_lse")
    torch.cuda.synchronize()
    got = out.double() + (lo.double() if lo is not None else 0)
    err = float((got - o_ref).norm() / o_ref.norm())
    lerr = float((lse_k.double() - lse).abs().max())
    assert err <= (2e-3 if dtype == "bf16" else 1e-5), (err, lerr)
    assert lerr <= (2e-2 if dtype == "bf16" else 1e-4), (err, lerr)


def _run_bwd(dtype, T, n_pad, generic, H=16, D=24, B=1, L=2):
    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    dev = "cuda"
    BL, C, DP = B * L, H * D, _lib.head_stride(D)
    ct = torch.bfloat16 if dtype == "bf16" else torch.float32
    mdt = _lib.MDG_BF16 if dtype == "bf16" else _lib.MDG_F32
    qscale, log2e = D ** -0.5, 1.0 / math.log(2.0)
    c = _case(T, BL, H, D, n_pad, seed=T + n_pad)
    cos, sin = (x.double().to(dev) for x in _rope_tab(T + 1, D))
    for k in ("q_lin", "k_lin", "v", "bk_lin", "bv"):
        c[k].requires_grad_(True)
    o, qn, kr, bk, s_all = _forward(c, D, T, cos, sin, qscale)
    (o * c["dout"]).sum().backward()

    # kernel operands (rounded to CT where the kernel reads CT)
    with torch.no_grad():
        planes = torch.zeros(3, BL, H, T, DP, device=dev, dtype=ct)
        planes[0, ..., :D] = (qn * log2e).to(ct)
        planes[1, ..., :D] = kr.to(ct)
        planes[2, ..., :D] = c["v"].to(ct)
        planes[1, ..., D] = 1.0
        planes[2, ..., D] = 1.0
        qp, kp, vp = (planes[i, ..., :D].double() for i in range(3))
        # lse / o from the operands the kernel sees (log2 units)
        s2 = torch.einsum("shtd,shud->shtu", qp, kp) + c["kbias"][:, None, None, :]
        sb2 = torch.einsum("shtd,hd->sht", qp, bk.detach())[..., None]
        s2 = torch.cat([sb2, s2], -1)
        lse = torch.logsumexp(s2 * math.log(2.0), -1) * log2e
        p2 = torch.exp2(s2 - lse[..., None])
        o_k = p2[..., :1] * c["bv"].detach()[None, :, None, :] + torch.einsum("shtu,shud->shtd", p2[..., 1:], vp)

        def tok_major(x):  # [BL][H][T][D] -> [N][C], n = (b*T + t)*L + l, seq = b*L + l
            return x.reshape(B, L, H, T, D).permute(0, 3, 1, 2, 4).reshape(B * T * L, C)

        o_t = tok_major(o_k).to(ct).contiguous()
        lo_t = (tok_major(o_k) - o_t.double()).to(ct).contiguous() if dtype == "bf16" else None
        do_t = tok_major(c["dout"]).to(ct).contiguous()
        kvb = torch.zeros(H, 2, DP, device=dev)
        kvb[:, 0, :D] = bk.detach().float()
        kvb[:, 1, :D] = c["bv"].detach().float()
        kb = c["kbias"].float().contiguous()
        lse_f = lse.float().contiguous()
        rope = torch.cat([cos.float().reshape(-1), sin.float().reshape(-1)]).contiguous()
        parts = lib.mdg_attn_temporal_bwd_parts(mdt, B, T, L, generic)
        bpart = torch.full((H, parts, 2, DP), float("nan"), device=dev)  # every slot is written
        scratch = torch.empty(lib.mdg_attn_temporal_bwd_scratch(mdt, B, T, L, H, D), device=dev, dtype=torch.uint8)
        dqkv = torch.full((B * T * L, 3 * C), float("nan"), device=dev, dtype=ct)
        _lib.check(lib.mdg_attn_temporal_bwd(mdt, B, T, L, H, D, planes.data_ptr(), kb.data_ptr(), kvb.data_ptr(),
                                             o_t.data_ptr(), _lib.ptr(lo_t), do_t.data_ptr(), lse_f.data_ptr(),
                                             rope.data_ptr(), T + 1,
                                             scratch.data_ptr(), dqkv.data_ptr(), 3 * C, bpart.data_ptr(), qscale,
                                             math.log(2.0), generic, _lib.stream_handle()), "mdg_attn_temporal_bwd")
        torch.cuda.synchronize()
        got = dqkv.double()
        gb = bpart.double().sum(1)
    refs = {"dq": tok_major(c["q_lin"].grad), "dk": tok_major(c["k_lin"].grad), "dv": tok_major(c["v"].grad),
            "dbk": _rope_inv_bias(c, cos, sin, T), "dbv": c["bv"].grad}
    gots = {"dq": got[:, :C], "dk": got[:, C:2 * C], "dv": got[:, 2 * C:], "dbk": gb[:, 0, :D], "dbv": gb[:, 1, :D]}
    # f32: 1e-5 also with a fully padded sequence (its dS is exactly 0 since round 5; the rounding of
    # dpb - delta summed over its queries had left 2e-5 of the whole dbk)
    tol = BF16_TOL if dtype == "bf16" else 1e-5
    errs = {k: float((gots[k] - refs[k]).norm() / refs[k].norm()) for k in refs}
    path = os.environ.get("MDG_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": "attn_temporal_bwd", "dtype": dtype, "generic": generic, "T": T, "n_pad": n_pad,
                                "H": H, "D": D, **errs}) + "\n")
    assert torch.isfinite(got).all(), "unwritten or non-finite dq|dk|dv"
    for k, e in errs.items():
        assert e <= tol, (k, e, errs)


def _rope_inv_bias(c, cos, sin, T):
    """d loss / d (rotated bias_k) from autograd's d / d bk_lin: the kernel reports the gradient
    w.r.t. the rotated row (mdg_train_unpack_layer undoes the rotation)."""
    g = c["bk_lin"].grad  # = R^T dbk_rot  ->  dbk_rot = R g
    return _rope(g[:, None, :], cos[T:T + 1], sin[T:T + 1])[:, 0]
