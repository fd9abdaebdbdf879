"""Parameter containers (and their eager forwards) with the reference's module names, so
``state_dict()`` keys match a reference checkpoint exactly.

Reference: src/mdgen/model/layers.py (modulate 14-15, TimestepEmbedder 17-55, FinalLayer
58-75, gelu 78-85), src/mdgen/model/mha.py (MultiheadAttention 67-159: parameter layout
only), fair-esm RotaryEmbedding (buffer ``inv_freq``), src/mdgen/model/ipa.py:34-90
(InvariantPointAttention parameters).
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.attention import SDPBackend, sdpa_kernel


class _TokenLinear(torch.autograd.Function):
    """nn.Linear over the B*T*L token rows with a tiny in or out width (latent 21 <-> C): the
    weight gradient dY^T X has K = 32 000 tokens and an output of a few tiles, which hipBLASLt
    ran as one long-K kernel (120 us each in the training step); here it is split over 16 token
    chunks (one batched GEMM + a sum of the fp32 partials)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = (g2 @ w.to(g2.dtype)).reshape(x.shape) if ctx.needs_input_grad[0] else None
        n, S = g2.shape[0], 16
        if n % S == 0 and n >= 64 * S:
            # fp32 partials (under bf16-mixed autocast g is bf16: bf16 partials would round each
            # chunk's sum before the sum over chunks)
            dw = torch.bmm(g2.float().reshape(S, n // S, -1).transpose(1, 2), x2.float().reshape(S, n // S, -1)).sum(0)
        else:
            dw = g2.t() @ x2.to(g2.dtype)
        db = g2.sum(0) if ctx.has_bias else None
        return dx, dw.to(w.dtype), db


def token_linear(lin, x):
    """lin(x), with the split-K weight gradient of _TokenLinear when autograd records a call on
    the GPU over many token rows."""
    if x.is_cuda and torch.is_grad_enabled() and x.numel() >= 4096 * x.shape[-1]:
        return _TokenLinear.apply(x, lin.weight, lin.bias)
    return lin(x)


def modulate(x, shift, scale):
    return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1)


def gelu(x):
    """Exact-erf GELU (layers.py:78-85).  On the GPU as torch's fused exact GELU (one kernel
    forward and backward instead of five and eight: the training step's eager IPA layers run it
    on 32 tokens, launch-bound); the erf argument is x * (1/sqrt 2) there, 1 ulp from x / sqrt 2."""
    if x.is_cuda:
        return F.gelu(x)
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


def timestep_freqs(dim=256, max_period=10000):
    """exp(-ln(max_period) * i / half), computed on the CPU exactly as layers.py:42-44 does."""
    half = dim // 2
    return torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)


def timestep_embedding(t, dim=256, max_period=10000, freqs=None):
    half = dim // 2
    if freqs is None:
        freqs = timestep_freqs(dim, max_period)
    freqs = freqs.to(t.device)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


class TimestepEmbedder(nn.Module):
    def __init__(self, hidden_size, frequency_embedding_size=256):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(frequency_embedding_size, hidden_size, bias=True), nn.SiLU(),
                                 nn.Linear(hidden_size, hidden_size, bias=True))
        self.frequency_embedding_size = frequency_embedding_size
        # device-resident copy (not in state_dict) so graph capture never copies host->device
        self.register_buffer("freqs", timestep_freqs(frequency_embedding_size), persistent=False)

    def forward(self, t):
        return self.mlp(timestep_embedding(t, self.frequency_embedding_size, freqs=self.freqs))


class FinalLayer(nn.Module):
    def __init__(self, hidden_size, out_channels):
        super().__init__()
        self.norm_final = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.linear = nn.Linear(hidden_size, out_channels, bias=True)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 2 * hidden_size, bias=True))

    def forward(self, x, c, mods=None):
        shift, scale = (self.adaLN_modulation(c) if mods is None else mods).chunk(2, dim=-1)
        return token_linear(self.linear, modulate(self.norm_final(x), shift, scale))


class RotaryEmbedding(nn.Module):
    """fair-esm 1.0.2 RotaryEmbedding: only the ``inv_freq`` buffer is state."""

    def __init__(self, dim):
        super().__init__()
        self.register_buffer("inv_freq", 1.0 / (10000 ** (torch.arange(0, dim, 2).float() / dim)))

    def tables(self, n, device):
        """cos, sin [n, dim/2] for positions 0..n-1 (the table is built from k's length)."""
        pos = torch.arange(n, device=self.inv_freq.device).type_as(self.inv_freq)
        freqs = torch.einsum("i,j->ij", pos, self.inv_freq)
        return freqs.cos().to(device), freqs.sin().to(device)

    def tables2(self, n, device):
        """cat([cos, cos]), cat([sin, sin]) [n, dim] (fair-esm's doubled tables), cached per
        (n, device): inv_freq is a constant buffer, and rebuilding the tables took ~8 small
        kernels per attention call in the training step's eager conditioning."""
        cache = self.__dict__.setdefault("_tab2", {})
        key = (n, str(device), self.inv_freq.data_ptr())
        t = cache.get(key)
        if t is None:
            cos, sin = self.tables(n, device)
            t = cache[key] = (torch.cat([cos, cos], -1), torch.cat([sin, sin], -1))
        return t


def apply_rope(x, cos, sin, doubled=False):
    n, h = x.shape[-2], x.shape[-1] // 2
    c = cos[:n] if doubled else torch.cat([cos[:n], cos[:n]], -1)
    s = sin[:n] if doubled else torch.cat([sin[:n], sin[:n]], -1)
    rot = torch.cat((-x[..., h:], x[..., :h]), dim=-1)
    return x * c + rot * s


class MultiheadAttention(nn.Module):
    """Parameter layout of the reference fairseq/ESM MultiheadAttention (mha.py:67-159) with
    add_bias_kv and rotary embeddings; ``forward`` is the eager rope path (mha.py:161-407)
    for batch-first input [N, S, C] and key validity [N, S]."""

    def __init__(self, embed_dim, num_heads, add_bias_kv=True, use_rotary_embeddings=True, dropout=0.0):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.scaling = self.head_dim ** -0.5
        self.dropout = dropout
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        if add_bias_kv:
            self.bias_k = nn.Parameter(torch.empty(1, 1, embed_dim))
            self.bias_v = nn.Parameter(torch.empty(1, 1, embed_dim))
        else:
            self.bias_k = self.bias_v = None
        g = 1 / math.sqrt(2)
        for lin in (self.k_proj, self.v_proj, self.q_proj):
            nn.init.xavier_uniform_(lin.weight, gain=g)
        nn.init.xavier_uniform_(self.out_proj.weight)
        nn.init.constant_(self.out_proj.bias, 0.0)
        if add_bias_kv:
            nn.init.xavier_normal_(self.bias_k)
            nn.init.xavier_normal_(self.bias_v)
        self.rot_emb = RotaryEmbedding(self.head_dim) if use_rotary_embeddings else None

    def forward(self, x, valid):
        N, S, C = x.shape
        H, d = self.num_heads, self.head_dim
        q = self.q_proj(x) * self.scaling
        k, v = self.k_proj(x), self.v_proj(x)
        kvalid = valid.bool()
        if self.bias_k is not None:
            k = torch.cat([k, self.bias_k.expand(N, 1, C)], 1)
            v = torch.cat([v, self.bias_v.expand(N, 1, C)], 1)
            kvalid = torch.cat([kvalid, torch.ones(N, 1, dtype=torch.bool, device=x.device)], 1)
        Sk = k.shape[1]
        q = q.reshape(N, S, H, d).transpose(1, 2)
        k = k.reshape(N, Sk, H, d).transpose(1, 2)
        v = v.reshape(N, Sk, H, d).transpose(1, 2)
        if self.rot_emb is not None:
            cos2, sin2 = self.rot_emb.tables2(Sk, x.device)
            q, k = apply_rope(q, cos2, sin2, doubled=True), apply_rope(k, cos2, sin2, doubled=True)
        # softmax(q k^T masked) v (mha.py:359-389) as one SDPA call, on the GPU on its math
        # backend: the default ROCm backend is wrong at some shapes (head_dim 48 over 17 keys:
        # 3e-3 rel in fp32 on random operands, 0.12 inside a training layer, against fp64 and the
        # math backend; tools/dbg/sdpa_check.py), and this eager path is the reference the HIP
        # kernels are tested against and the fallback that trains what they do not take
        bias = torch.where(kvalid[:, None, None, :], 0.0, float("-inf")).to(q.dtype)
        with sdpa_kernel(SDPBackend.MATH) if q.is_cuda else contextlib.nullcontext():
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=1.0,
                                               dropout_p=self.dropout if self.training else 0.0)
        o = o.transpose(1, 2).reshape(N, S, C)
        return self.out_proj(o)


class AttentionWithRoPE(nn.Module):
    """latent_model.py:329-338 (key_padding_mask = 1 - mask)."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.attn = MultiheadAttention(*args, **kwargs)

    def forward(self, x, mask):
        return self.attn(x, mask)


class _IpaCoreFn(torch.autograd.Function):
    """The IPA attention core (logits, softmax, value / point aggregation, inverse frame, point
    norms: ipa.py:149-250) as one HIP kernel each way (csrc/ipa_train.hip, mdg_ipa_core_fwd /
    _bwd; crops up to 32 residues on one wave per (sample, head), 33..256 on the long kernels).  flags 0: points in the global frame and hw = softplus(head_weights) * c;
    MDG_IPA_LOCAL_POINTS | MDG_IPA_RAW_HW: the raw point projections and the raw head_weights
    (the frame application and the softplus run in the kernels, ipa.py:121-140, 178-183).
    Returns the linear_out input [B, L, H*c + 4*H*Pv]."""

    @staticmethod
    def forward(ctx, q, kv, qp, kvp, mask, rots, trans, hw, wc, flags=0):
        from .. import _lib

        lib = _lib.load()
        B, L, H, c = q.shape
        Pq = (qp.shape[-1] // (3 * H)) if flags & _lib.MDG_IPA_LOCAL_POINTS else qp.shape[3]
        Pv = ((kvp.shape[-1] // (3 * H)) if flags & _lib.MDG_IPA_LOCAL_POINTS else kvp.shape[3]) - Pq
        ops = [t.detach().float().contiguous() for t in (q, kv, qp, kvp, mask, rots, trans, hw)]
        out = torch.empty(B, L, H * c + 4 * H * Pv, device=q.device)
        _lib.check(lib.mdg_ipa_core_fwd(B, L, H, c, Pq, Pv, *[t.data_ptr() for t in ops], wc, out.data_ptr(), flags,
                                        _lib.stream_handle()), "mdg_ipa_core_fwd")
        ctx.save_for_backward(*ops)
        ctx.wc, ctx.flags, ctx.P = wc, flags, (Pq, Pv)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .. import _lib

        lib = _lib.load()
        ops = ctx.saved_tensors
        q, kv, qp, kvp = ops[:4]
        B, L, H, c = q.shape
        Pq, Pv = ctx.P
        dq, dkv, dqp, dkvp = (torch.empty_like(t) for t in (q, kv, qp, kvp))
        dhw = torch.empty(B, H, device=q.device)
        _lib.check(lib.mdg_ipa_core_bwd(B, L, H, c, Pq, Pv, *[t.data_ptr() for t in ops], ctx.wc,
                                        dout.float().contiguous().data_ptr(), dq.data_ptr(), dkv.data_ptr(),
                                        dqp.data_ptr(), dkvp.data_ptr(), dhw.data_ptr(), ctx.flags,
                                        _lib.stream_handle()),
                   "mdg_ipa_core_bwd")
        return dq, dkv, dqp, dkvp, None, None, None, dhw.sum(0), None, None


class InvariantPointAttention(nn.Module):
    """Parameters of ipa.py:34-90 (c_z = 0) and the eager forward of ipa.py:92-255."""

    def __init__(self, c_s, c_z, c_hidden, no_heads, no_qk_points, no_v_points, inf=1e5, eps=1e-8, dropout=0.0):
        super().__init__()
        assert c_z == 0
        self.c_s, self.c_hidden, self.no_heads = c_s, c_hidden, no_heads
        self.no_qk_points, self.no_v_points = no_qk_points, no_v_points
        self.inf, self.eps = inf, eps
        self.hip_core = False  # set per call by LatentMDGenModel.run_ipa (HIP training path)
        hc = c_hidden * no_heads
        self.linear_q = nn.Linear(c_s, hc)
        self.linear_kv = nn.Linear(c_s, 2 * hc)
        self.linear_q_points = nn.Linear(c_s, no_heads * no_qk_points * 3)
        self.linear_kv_points = nn.Linear(c_s, no_heads * (no_qk_points + no_v_points) * 3)
        self.head_weights = nn.Parameter(torch.full((no_heads,), 0.541324854612918))
        self.linear_out = nn.Linear(no_heads * (c_hidden + no_v_points * 4), c_s)
        nn.init.zeros_(self.linear_out.weight)
        nn.init.zeros_(self.linear_out.bias)

    def forward(self, s, rots, trans, mask):
        B, L, _ = s.shape
        H, c, Pq, Pv = self.no_heads, self.c_hidden, self.no_qk_points, self.no_v_points
        hip = self.hip_core and s.is_cuda and L <= 256 and c == 32 and Pq == 8 and Pv == 8
        if hip:
            from ..train_hip import seg_linear, seg_supported

            if seg_supported(s):
                # the four projections as one library launch; the frame application of the points
                # and the head-weight softplus inside the core kernels
                from .. import _lib

                q, kv, qp, kvp = seg_linear(s, [self.linear_q, self.linear_kv, self.linear_q_points,
                                                self.linear_kv_points])
                o = _IpaCoreFn.apply(q.reshape(B, L, H, c), kv.reshape(B, L, H, 2 * c), qp, kvp, mask, rots, trans,
                                     self.head_weights, math.sqrt(1.0 / (3 * c)),
                                     _lib.MDG_IPA_LOCAL_POINTS | _lib.MDG_IPA_RAW_HW)
                return seg_linear(o, [self.linear_out])[0]
        q = self.linear_q(s).reshape(B, L, H, c)
        kv = self.linear_kv(s).reshape(B, L, H, 2 * c)
        k, v = kv[..., :c], kv[..., c:]

        # Frame applications as one broadcast product + a 3-term sum each (r x: sum_j r_ij x_j;
        # the per-component form of rigid_utils.py:64-86 costs ~17 kernels forward and ~40
        # backward per application, and the training step runs 4 per IPA layer)
        def points(raw, n):
            pts = raw.reshape(B, L, 3, n).transpose(-1, -2)  # stack(split(raw, n), -1)
            rp = (rots[:, :, None] * pts[..., None, :]).sum(-1)
            return rp + trans[:, :, None]

        q_pts = points(self.linear_q_points(s), H * Pq).reshape(B, L, H, Pq, 3)
        kv_pts = points(self.linear_kv_points(s), H * (Pq + Pv)).reshape(B, L, H, Pq + Pv, 3)
        hw = F.softplus(self.head_weights) * math.sqrt(1.0 / (3 * (Pq * 9.0 / 2)))
        if hip:
            return self.linear_out(_IpaCoreFn.apply(q, kv, q_pts, kv_pts, mask, rots, trans, hw,
                                                    math.sqrt(1.0 / (3 * c))))
        k_pts, v_pts = kv_pts[..., :Pq, :], kv_pts[..., Pq:, :]
        a = torch.einsum("bihc,bjhc->bhij", q, k) * math.sqrt(1.0 / (3 * c))
        d2 = ((q_pts[:, :, None] - k_pts[:, None, :]) ** 2).sum(-1)
        pt = (d2 * hw[:, None]).sum(-1) * (-0.5)
        sq = self.inf * (mask[:, :, None] * mask[:, None, :] - 1)
        a = torch.softmax(a + pt.permute(0, 3, 1, 2) + sq[:, None], dim=-1)
        o = torch.einsum("bhij,bjhc->bihc", a, v).reshape(B, L, H * c)
        opt = torch.einsum("bhij,bjhpx->bihpx", a, v_pts) - trans[:, :, None, None]
        opt = (rots.transpose(-1, -2)[:, :, None, None] * opt[..., None, :]).sum(-1)  # r^T x
        nrm = torch.sqrt((opt ** 2).sum(-1) + self.eps).reshape(B, L, H * Pv)
        opt = opt.reshape(B, L, H * Pv, 3)
        return self.linear_out(torch.cat([o, opt[..., 0], opt[..., 1], opt[..., 2], nrm], -1))
