"""CPU oracle: a from-scratch fp32 PyTorch-CPU restatement of MDGen's denoising hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module, and only as the checker / the timed CPU baseline — never as part
of the product path (mdgen_finetune_amd/ never imports it).

Parity status: PINNED.  Every function here is checked against golden vectors produced by
running the reference itself (oracle/gen_golden.py -> tests/golden/*.npz; tests/test_oracle.py)
to ~1e-5.  Third-party arithmetic the reference delegates (fair-esm rotary, torchdiffeq Euler)
is restated from the packages' published behaviour; their own parity is unpinned (no copy of
either package exists in the container) — see DESIGN.md §Oracle.

The one deliberate deviation from the fork, shared with the golden generator: the IPA prepend
uses mask[:, 0] (the only shape-valid reading of latent_model.py:255 for num_frames > 1;
bit-identical to the fork at T == 1).

Parameters are a dict {state-dict name -> fp32 tensor} with the reference's exact key names
(LatentMDGenModel.state_dict(), latent_model.py:44-128), so the same dict feeds the oracle,
the drop-in module and the HIP engine.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- config
@dataclass
class Cfg:
    """Model hyper-parameters (reference parsing.py:86-97 defaults)."""
    embed_dim: int = 384
    mha_heads: int = 16
    num_layers: int = 5
    ipa_heads: int = 4
    ipa_head_dim: int = 32
    ipa_qk: int = 8
    ipa_v: int = 8
    latent_dim: int = 21
    crop: int = 4
    tps: bool = False
    time_multiplier: float = 100.0

    @classmethod
    def from_flags(cls, flags, latent_dim, crop, tps):
        kv = dict(zip(flags[::2], flags[1::2]))
        c = cls(latent_dim=latent_dim, crop=crop, tps=tps)
        for k, v in kv.items():
            setattr(c, k.lstrip("-"), int(v))
        return c


def param_shapes(cfg: Cfg):
    """State-dict parameter names and shapes of LatentMDGenModel with --prepend_ipa
    --abs_pos_emb (latent_model.py:50-128; IPALayer 354-376; LatentMDGenLayer 413-454;
    MultiheadAttention mha.py:111-123; InvariantPointAttention ipa.py:66-87;
    TimestepEmbedder layers.py:21-27; FinalLayer layers.py:62-68).  Buffers excluded."""
    C, F4 = cfg.embed_dim, 4 * cfg.embed_dim
    H, c, Pq, Pv = cfg.ipa_heads, cfg.ipa_head_dim, cfg.ipa_qk, cfg.ipa_v
    out = []

    def lin(name, i, o):
        out.append((f"{name}.weight", (o, i)))
        out.append((f"{name}.bias", (o,)))

    def mha(p):
        for n in ("k_proj", "v_proj", "q_proj", "out_proj"):
            lin(f"{p}.attn.{n}", C, C)
        out.append((f"{p}.attn.bias_k", (1, 1, C)))
        out.append((f"{p}.attn.bias_v", (1, 1, C)))

    lin("latent_to_emb", cfg.latent_dim, C)
    if cfg.tps:
        lin("latent_to_emb_f", 7, C)
        lin("latent_to_emb_r", 7, C)
    lin("cond_to_emb", cfg.latent_dim, C)
    out.append(("mask_to_emb.weight", (2, C)))
    out.append(("aatype_to_emb.weight", (21, C)))
    for i in range(cfg.num_layers):
        p = f"ipa_layers.{i}"
        lin(f"{p}.adaLN_modulation.1", C, 6 * C)
        out.append((f"{p}.ipa_norm.weight", (C,)))
        out.append((f"{p}.ipa_norm.bias", (C,)))
        lin(f"{p}.ipa.linear_q", C, H * c)
        lin(f"{p}.ipa.linear_kv", C, 2 * H * c)
        lin(f"{p}.ipa.linear_q_points", C, H * Pq * 3)
        lin(f"{p}.ipa.linear_kv_points", C, H * (Pq + Pv) * 3)
        out.append((f"{p}.ipa.head_weights", (H,)))
        lin(f"{p}.ipa.linear_out", H * (c + 4 * Pv), C)
        mha(f"{p}.mha_l")
        lin(f"{p}.fc1", C, F4)
        lin(f"{p}.fc2", F4, C)
    for i in range(cfg.num_layers):
        p = f"layers.{i}"
        lin(f"{p}.adaLN_modulation.1", C, 9 * C)
        mha(f"{p}.mha_t")
        mha(f"{p}.mha_l")
        lin(f"{p}.fc1", C, F4)
        lin(f"{p}.fc2", F4, C)
    lin("emb_to_latent.linear", C, cfg.latent_dim)
    lin("emb_to_latent.adaLN_modulation.1", C, 2 * C)
    lin("t_embedder.mlp.0", 256, C)
    lin("t_embedder.mlp.2", C, C)
    return out


def seeded_params(cfg: Cfg, seed: int):
    """Parameters from the portable generator (same bits the reference model was filled with
    in oracle/gen_golden.py)."""
    from mdgen_finetune_amd.synthetic import param_value

    return {n: torch.from_numpy(param_value(seed, n, s)) for n, s in param_shapes(cfg)}


# ----------------------------------------------------------------------------- pieces
def sincos_pos_embed(dim, n):
    """get_1d_sincos_pos_embed_from_grid (latent_model.py:22-40): float64 numpy, [sin | cos]."""
    omega = np.arange(dim // 2, dtype=np.float64) / (dim / 2.0)
    omega = 1.0 / 10000 ** omega
    out = np.einsum("m,d->md", np.arange(n).astype(np.float64), omega)
    return torch.from_numpy(np.concatenate([np.sin(out), np.cos(out)], axis=1)).float()


def linear(P, name, x):
    return F.linear(x, P[f"{name}.weight"], P[f"{name}.bias"])


def ln(x, eps=1e-6, w=None, b=None):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def modulate(x, shift, scale):
    """layers.py:14-15."""
    return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1)


def gelu(x):
    """Exact-erf GELU, layers.py:78-85."""
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


def timestep_embedding(t, dim=256, max_period=10000):
    """TimestepEmbedder.timestep_embedding, layers.py:31-50: [cos | sin]."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    # (an fp64 run of the oracle — the tests' exact reference — keeps the fp32 embedding, upcast)
    return emb.double() if t.dtype == torch.float64 else emb


def t_embedder(P, t):
    """layers.py:52-55: Linear(256->C) -> SiLU -> Linear(C->C)."""
    h = linear(P, "t_embedder.mlp.0", timestep_embedding(t))
    return linear(P, "t_embedder.mlp.2", F.silu(h))


def rope_tables(d, n):
    """fair-esm RotaryEmbedding tables (restated; used at mha.py:356-357): built for n rows."""
    inv_freq = 1.0 / (10000 ** (torch.arange(0, d, 2).float() / d))
    pos = torch.arange(n).type_as(inv_freq)
    freqs = torch.einsum("i,j->ij", pos, inv_freq)
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos(), emb.sin()


def apply_rope(x, cos, sin):
    n, h = x.shape[-2], x.shape[-1] // 2
    rot = torch.cat((-x[..., h:], x[..., :h]), dim=-1)
    return x * cos[:n] + rot * sin[:n]


def mha(P, prefix, x, valid, heads):
    """MultiheadAttention.forward on the rope path (mha.py:161-407) for batch-first x [N,S,C]
    and key validity `valid` [N,S] (key_padding_mask = 1 - valid, AttentionWithRoPE
    latent_model.py:334-338).  One learned bias_k/bias_v row is appended after projection
    (mha.py:265-280), is never masked, and is RoPE-rotated at position S (the table is built
    from k's length S+1).  Scores are fp32-softmaxed (mha.py:19-23, 381)."""
    N, S, C = x.shape
    d = C // heads
    a = f"{prefix}.attn"
    q = linear(P, f"{a}.q_proj", x) * (d ** -0.5)
    k = linear(P, f"{a}.k_proj", x)
    v = linear(P, f"{a}.v_proj", x)
    k = torch.cat([k, P[f"{a}.bias_k"].reshape(1, 1, C).expand(N, 1, C)], 1)
    v = torch.cat([v, P[f"{a}.bias_v"].reshape(1, 1, C).expand(N, 1, C)], 1)
    q = q.reshape(N, S, heads, d).transpose(1, 2)          # [N,H,S,d]
    k = k.reshape(N, S + 1, heads, d).transpose(1, 2)      # [N,H,S+1,d]
    v = v.reshape(N, S + 1, heads, d).transpose(1, 2)
    cos, sin = rope_tables(d, S + 1)
    q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
    w = q @ k.transpose(-1, -2)                             # [N,H,S,S+1]
    kvalid = torch.cat([valid.bool(), torch.ones(N, 1, dtype=torch.bool)], 1)
    w = w.masked_fill(~kvalid[:, None, None, :], float("-inf"))
    w = torch.softmax(w, dim=-1, dtype=torch.float64 if w.dtype == torch.float64 else torch.float32)
    o = (w @ v).transpose(1, 2).reshape(N, S, C)
    return linear(P, f"{a}.out_proj", o)


def ipa(P, prefix, s, rots, trans, mask, cfg: Cfg):
    """InvariantPointAttention.forward with c_z = 0 (ipa.py:92-255); Rigid.apply /
    invert_apply (rigid_utils.py:1047-1073, 615-641, rot_vec_mul 64-86) in fp32."""
    B, L, _ = s.shape
    H, c, Pq, Pv = cfg.ipa_heads, cfg.ipa_head_dim, cfg.ipa_qk, cfg.ipa_v
    p = f"{prefix}.ipa"
    q = linear(P, f"{p}.linear_q", s).reshape(B, L, H, c)
    kv = linear(P, f"{p}.linear_kv", s).reshape(B, L, H, 2 * c)
    k, v = kv[..., :c], kv[..., c:]

    def points(name, n):
        raw = linear(P, f"{p}.{name}", s)                      # [B,L,3*n]
        pts = torch.stack(torch.split(raw, n, dim=-1), dim=-1)  # [B,L,n,3] (x|y|z blocks)
        r = rots[:, :, None]                                    # [B,L,1,3,3]
        x, y, z = pts.unbind(-1)
        rp = torch.stack([r[..., i, 0] * x + r[..., i, 1] * y + r[..., i, 2] * z for i in range(3)], -1)
        return rp + trans[:, :, None]

    q_pts = points("linear_q_points", H * Pq).reshape(B, L, H, Pq, 3)
    kv_pts = points("linear_kv_points", H * (Pq + Pv)).reshape(B, L, H, Pq + Pv, 3)
    k_pts, v_pts = kv_pts[..., :Pq, :], kv_pts[..., Pq:, :]

    a = torch.einsum("bihc,bjhc->bhij", q, k) * math.sqrt(1.0 / (3 * c))
    d2 = ((q_pts[:, :, None] - k_pts[:, None, :]) ** 2).sum(-1)   # [B,Li,Lj,H,Pq]
    hw = F.softplus(P[f"{p}.head_weights"]) * math.sqrt(1.0 / (3 * (Pq * 9.0 / 2)))
    pt = (d2 * hw[:, None]).sum(-1) * (-0.5)                       # [B,Li,Lj,H]
    sq = 1e5 * (mask[:, :, None] * mask[:, None, :] - 1)
    a = a + pt.permute(0, 3, 1, 2) + sq[:, None]
    a = torch.softmax(a, dim=-1)
    o = torch.einsum("bhij,bjhc->bihc", a, v).reshape(B, L, H * c)
    opt = torch.einsum("bhij,bjhpx->bihpx", a, v_pts)              # [B,L,H,Pv,3]
    opt = opt - trans[:, :, None, None]
    r = rots[:, :, None, None]
    x, y, z = opt.unbind(-1)
    opt = torch.stack([r[..., 0, i] * x + r[..., 1, i] * y + r[..., 2, i] * z for i in range(3)], -1)
    nrm = torch.sqrt((opt ** 2).sum(-1) + 1e-8).reshape(B, L, H * Pv)
    opt = opt.reshape(B, L, H * Pv, 3)
    cat = torch.cat([o, opt[..., 0], opt[..., 1], opt[..., 2], nrm], -1)
    return linear(P, f"{p}.linear_out", cat)


def ipa_layer(P, i, x, c, mask, rots, trans, cfg: Cfg):
    """IPALayer.forward (latent_model.py:378-394); adaLN 6-way chunk order (379-380)."""
    p = f"ipa_layers.{i}"
    C = cfg.embed_dim
    m = linear(P, f"{p}.adaLN_modulation.1", F.silu(c))
    sh_l, sc_l, g_l, sh_m, sc_m, g_m = m.split(C, -1)
    x = x + ipa(P, p, ln(x, 1e-5, P[f"{p}.ipa_norm.weight"], P[f"{p}.ipa_norm.bias"]),
                rots, trans, mask, cfg)
    h = modulate(ln(x), sh_l, sc_l)
    x = x + g_l.unsqueeze(1) * mha(P, f"{p}.mha_l", h, mask, cfg.mha_heads)
    h = modulate(ln(x), sh_m, sc_m)
    h = linear(P, f"{p}.fc2", gelu(linear(P, f"{p}.fc1", h)))
    return x + g_m.unsqueeze(1) * h


def latent_layer(P, i, x, c, mask, cfg: Cfg):
    """LatentMDGenLayer.forward (latent_model.py:456-493): spatial attention over L (+bias
    row), temporal attention over T (+bias row), MLP; the same no-affine LN (eps 1e-6) for
    both attentions; adaLN 9-way chunk order (459-461)."""
    p = f"layers.{i}"
    B, T, L, C = x.shape
    m = linear(P, f"{p}.adaLN_modulation.1", F.silu(c))          # c [B,1,C] -> [B,1,9C]
    sh_l, sc_l, g_l, sh_t, sc_t, g_t, sh_m, sc_m, g_m = m.split(C, -1)
    h = modulate(ln(x), sh_l, sc_l)
    h = mha(P, f"{p}.mha_l", h.reshape(B * T, L, C), mask.reshape(B * T, L), cfg.mha_heads)
    x = x + g_l.unsqueeze(1) * h.reshape(B, T, L, C)
    h = modulate(ln(x), sh_t, sc_t)
    h = mha(P, f"{p}.mha_t", h.transpose(1, 2).reshape(B * L, T, C),
            mask.transpose(1, 2).reshape(B * L, T), cfg.mha_heads)
    x = x + g_t.unsqueeze(1) * h.reshape(B, L, T, C).transpose(1, 2)
    h = modulate(ln(x), sh_m, sc_m)
    h = linear(P, f"{p}.fc2", gelu(linear(P, f"{p}.fc1", h)))
    return x + g_m.unsqueeze(1) * h


def rot_to_quat(rot):
    """rigid_utils.py:191-210 (eigenvector of the 4x4 K matrix, torch.linalg.eigh)."""
    r = [[rot[..., i, j] for j in range(3)] for i in range(3)]
    [[xx, xy, xz], [yx, yy, yz], [zx, zy, zz]] = r
    k = [[xx + yy + zz, zy - yz, xz - zx, yx - xy],
         [zy - yz, xx - yy - zz, xy + yx, xz + zx],
         [xz - zx, xy + yx, yy - xx - zz, yz + zy],
         [yx - xy, xz + zx, yz + zy, zz - xx - yy]]
    k = (1.0 / 3.0) * torch.stack([torch.stack(t, dim=-1) for t in k], dim=-2)
    _, vecs = torch.linalg.eigh(k)
    return vecs[..., -1]


def relative_tensor7(rots_a, trans_a, rots_b, trans_b):
    """a.invert().compose(b).to_tensor_7() (rigid_utils.py:1031-1045, 1075-1087, 1143-1155)."""
    ra_inv = rots_a.transpose(-1, -2)
    t_inv = -1 * torch.einsum("...ij,...j->...i", ra_inv, trans_a)
    rot = ra_inv @ rots_b
    tr = torch.einsum("...ij,...j->...i", ra_inv, trans_b) + t_inv
    return torch.cat([rot_to_quat(rot), tr], -1)


def run_ipa(P, cfg: Cfg, c, mask_b, rots, trans, end_rots, end_trans, aatype):
    """LatentMDGenModel.run_ipa (latent_model.py:179-214): sim branch (188-196) or TPS
    branch (197-211)."""
    B, L = mask_b.shape
    emb = P["aatype_to_emb.weight"][aatype]
    if not cfg.tps:
        x = torch.zeros(B, L, cfg.embed_dim) + emb
        for i in range(cfg.num_layers):
            x = ipa_layer(P, i, x, c, mask_b, rots, trans, cfg)
        return x
    x_f = linear(P, "latent_to_emb_f", relative_tensor7(rots, trans, end_rots, end_trans)) + emb
    x_r = linear(P, "latent_to_emb_r", relative_tensor7(end_rots, end_trans, rots, trans)) + emb
    for i in range(cfg.num_layers):
        x_r = ipa_layer(P, i, x_r, c, mask_b, rots, trans, cfg)
        x_f = ipa_layer(P, i, x_f, c, mask_b, end_rots, end_trans, cfg)
    return x_r + x_f


def forward(P, cfg: Cfg, x, t, mask, rots, trans, end_rots=None, end_trans=None,
            x_cond=None, x_cond_mask=None, aatype=None, capture=None):
    """LatentMDGenModel.forward (latent_model.py:216-269), sim/TPS, --prepend_ipa
    --abs_pos_emb, IPA mask = mask[:, 0]."""
    B, T, L, _ = x.shape
    if mask.dim() == 2:
        mask = mask.repeat(B, 1, 1)
    h = linear(P, "latent_to_emb", x) + sincos_pos_embed(cfg.embed_dim, cfg.crop)[None]
    if x_cond is not None:
        h = h + linear(P, "cond_to_emb", x_cond) + P["mask_to_emb.weight"][x_cond_mask]
    c = t_embedder(P, t * cfg.time_multiplier)[:, None]         # [B,1,C]
    ip = run_ipa(P, cfg, c[:, 0], mask[:, 0], rots, trans, end_rots, end_trans, aatype)
    if capture is not None:
        capture["ipa"] = ip
    h = h + ip[:, None]
    for i in range(cfg.num_layers):
        h = latent_layer(P, i, h, c, mask, cfg)
        if capture is not None:
            capture[f"layer{i}"] = h
    m = linear(P, "emb_to_latent.adaLN_modulation.1", F.silu(c))
    shift, scale = m.split(cfg.embed_dim, -1)
    return linear(P, "emb_to_latent.linear", modulate(ln(h), shift, scale))


def euler_sample(P, cfg: Cfg, zs, num_steps=50, **kw):
    """Sampler.sample_ode('euler') for the GVP/velocity transport (t0=0, t1=1,
    transport.py:407-450, 94-123) + torchdiffeq fixed-grid Euler (integrators.py:95-114):
    y_{i+1} = y_i + (t_{i+1} - t_i) * model(y_i, ones(B) * t_i).  Returns all num_steps states."""
    ts = torch.linspace(0, 1, num_steps)
    ys = [zs]
    y = zs
    for i in range(num_steps - 1):
        tt = torch.ones(zs.shape[0]) * ts[i]
        y = y + (ts[i + 1] - ts[i]) * forward(P, cfg, y, tt, **kw)
        ys.append(y)
    return torch.stack(ys)


def gvp_training_loss(P, cfg: Cfg, x1, x0, t, loss_mask, **kw):
    """Transport.training_losses, velocity + GVP path (transport.py:137-222; path.py:113-135,
    173-191): xt = sin(pi t/2) x1 + cos(pi t/2) x0, ut = pi/2 cos x1 - pi/2 sin x0,
    loss_b = sum((v - ut)^2 * m) / sum(m)  (mean_flat, transport.py:12-16)."""
    tt = t.reshape(-1, *([1] * (x1.dim() - 1)))
    xt = torch.sin(tt * np.pi / 2) * x1 + torch.cos(tt * np.pi / 2) * x0
    ut = (np.pi / 2 * torch.cos(tt * np.pi / 2)) * x1 + (-np.pi / 2 * torch.sin(tt * np.pi / 2)) * x0
    v = forward(P, cfg, xt, t, **kw)
    dims = list(range(1, x1.dim()))
    loss = ((v - ut) ** 2 * loss_mask).sum(dims) / loss_mask.sum(dims)
    return loss, v


def kwargs_from_npz(d):
    """Model kwargs from a golden fixture's in_* arrays."""
    f = lambda k: torch.from_numpy(d[f"in_{k}"])  # noqa: E731
    return dict(mask=f("mask"), rots=f("rots"), trans=f("trans"), end_rots=f("end_rots"),
                end_trans=f("end_trans"), x_cond=f("x_cond"), x_cond_mask=f("x_cond_mask"),
                aatype=f("aatype"))
