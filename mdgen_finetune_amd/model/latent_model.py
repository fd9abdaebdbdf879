"""Drop-in ``LatentMDGenModel`` (reference src/mdgen/model/latent_model.py:43-326).

Same constructor ``LatentMDGenModel(args, latent_dim)``, same ``state_dict`` keys (a
reference checkpoint's ``model.*`` entries load unchanged), same
``forward(x, t, mask, start_frames=None, end_frames=None, x_cond=None, x_cond_mask=None,
aatype=None, *args, **kwargs)`` and ``forward_inference``.

Backends
  * ``"hip"`` — the MI355X path: every token-wise op of the denoiser (embedding, the
    LN/adaLN/QKV/RoPE GEMMs, spatial + temporal attention, out-proj/MLP GEMMs with fused
    gated residuals, FinalLayer + Euler) runs in libmdgen_hip.so (mdgen_finetune_amd.engine).
    Used whenever autograd is not recording (inference, sampling).  CUDA tensors only; a CPU
    tensor or a missing library raises — there is no silent fallback.
  * ``"torch"`` — eager PyTorch ops (any device).  Used for training (autograd through the
    block stack; HIP backward kernels are not built yet), and by the
    engine for the x-independent conditioning precompute (t-embedding, adaLN, IPA prepend).

Deliberate deviation shared with the oracle: the IPA prepend receives mask[:, 0]
(latent_model.py:255 passes mask.reshape(-1, L), shape-invalid for num_frames > 1;
identical at T == 1).
"""
from __future__ import annotations

import warnings

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from ..rigid_utils import Rotation, frames_to_tensors, rot_to_quat
from .layers import (AttentionWithRoPE, FinalLayer, InvariantPointAttention, TimestepEmbedder, gelu, token_linear,
                     modulate)


def get_1d_sincos_pos_embed_from_grid(embed_dim, pos):
    """latent_model.py:22-40."""
    assert embed_dim % 2 == 0
    omega = np.arange(embed_dim // 2, dtype=np.float64)
    omega /= embed_dim / 2.0
    omega = 1.0 / 10000 ** omega
    out = np.einsum("m,d->md", pos.reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


class _SmallTableEmbedding(torch.autograd.Function):
    """weight[idx] for a table of a few rows (mask_to_emb: 2 rows, indexed per token).  The
    forward is the plain gather; the backward is one [E, N] x [N, C] GEMM of the one-hot
    indices, instead of autograd's sort-based embedding_dense_backward (0.5 ms per call over
    the 32 000 tokens of a training step on MI355X)."""

    @staticmethod
    def forward(ctx, weight, idx):
        ctx.save_for_backward(idx)
        ctx.E = weight.shape[0]
        return weight[idx]

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        i2 = idx.reshape(-1)
        if ctx.E <= 4:  # masked column sums (the [E, N] x [N, C] GEMM took 0.4 ms: K = N, E rows)
            return torch.stack([(g2 * (i2 == e).to(g2.dtype)[:, None]).sum(0) for e in range(ctx.E)]), None
        onehot = F.one_hot(i2, ctx.E).to(g2.dtype)
        return onehot.t() @ g2, None


UNSUPPORTED_FLAGS = ("design", "mpnn", "dynamic_mpnn", "hyena", "interleave_ipa", "inpainting")


class IPALayer(nn.Module):
    """latent_model.py:341-394."""

    def __init__(self, embed_dim, ffn_embed_dim, mha_heads, dropout=0.0, use_rotary_embeddings=False,
                 ipa_args=None):
        super().__init__()
        self.embed_dim = embed_dim
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(embed_dim, 6 * embed_dim, bias=True))
        self.ipa_norm = nn.LayerNorm(embed_dim)
        self.ipa = InvariantPointAttention(**ipa_args)
        self.mha_l = AttentionWithRoPE(embed_dim, mha_heads, add_bias_kv=True, dropout=dropout,
                                       use_rotary_embeddings=use_rotary_embeddings)
        self.mha_layer_norm = nn.LayerNorm(embed_dim, elementwise_affine=False, eps=1e-6)
        self.fc1 = nn.Linear(embed_dim, ffn_embed_dim)
        self.fc2 = nn.Linear(ffn_embed_dim, embed_dim)
        self.final_layer_norm = nn.LayerNorm(embed_dim, elementwise_affine=False, eps=1e-6)

    hip_hl = None  # train_hip.LayerHelper while LatentMDGenModel.run_ipa runs the HIP training path

    def forward(self, x, t, mask, rots, trans, mods=None):
        m6 = self.adaLN_modulation(t) if mods is None else mods
        x = x + self.ipa(self.ipa_norm(x), rots, trans, mask)
        if self.hip_hl is not None:  # MHA + MLP sublayers on the HIP training kernels
            from ..train_hip import hip_ipa_layer_tail

            return hip_ipa_layer_tail(self.hip_hl, self, x, m6, mask)
        sh_l, sc_l, g_l, sh_m, sc_m, g_m = m6.chunk(6, dim=-1)
        x = x + g_l.unsqueeze(1) * self.mha_l(modulate(self.mha_layer_norm(x), sh_l, sc_l), mask)
        h = modulate(self.final_layer_norm(x), sh_m, sc_m)
        return x + g_m.unsqueeze(1) * self.fc2(gelu(self.fc1(h)))


class LatentMDGenLayer(nn.Module):
    """latent_model.py:397-493 (attention variant; --hyena / --interleave_ipa are out of scope)."""

    def __init__(self, embed_dim, ffn_embed_dim, mha_heads, dropout=0.0, num_frames=50,
                 use_rotary_embeddings=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(embed_dim, 9 * embed_dim, bias=True))
        self.mha_t = AttentionWithRoPE(embed_dim, mha_heads, add_bias_kv=True, dropout=dropout,
                                       use_rotary_embeddings=use_rotary_embeddings)
        self.mha_l = AttentionWithRoPE(embed_dim, mha_heads, add_bias_kv=True, dropout=dropout,
                                       use_rotary_embeddings=use_rotary_embeddings)
        self.mha_layer_norm = nn.LayerNorm(embed_dim, elementwise_affine=False, eps=1e-6)
        self.fc1 = nn.Linear(embed_dim, ffn_embed_dim)
        self.fc2 = nn.Linear(ffn_embed_dim, embed_dim)
        self.final_layer_norm = nn.LayerNorm(embed_dim, elementwise_affine=False, eps=1e-6)

    def forward(self, x, t, mask, mods=None):
        """mods: this layer's adaLN output [B, 9C] computed elsewhere (the stacked adaLN GEMM of
        the training path); None: adaLN_modulation(t) here, as the reference."""
        B, T, L, C = x.shape
        m9 = self.adaLN_modulation(t) if mods is None else mods.reshape(B, 1, 9 * C)
        (sh_l, sc_l, g_l, sh_t, sc_t, g_t, sh_m, sc_m, g_m) = m9.chunk(9, dim=-1)
        h = modulate(self.mha_layer_norm(x), sh_l, sc_l)
        h = self.mha_l(h.reshape(B * T, L, C), mask.reshape(B * T, L)).reshape(B, T, L, C)
        x = x + g_l.unsqueeze(1) * h
        h = modulate(self.mha_layer_norm(x), sh_t, sc_t)
        h = self.mha_t(h.transpose(1, 2).reshape(B * L, T, C), mask.transpose(1, 2).reshape(B * L, T))
        x = x + g_t.unsqueeze(1) * h.reshape(B, L, T, C).transpose(1, 2)
        h = modulate(self.final_layer_norm(x), sh_m, sc_m)
        return x + g_m.unsqueeze(1) * self.fc2(gelu(self.fc1(h)))


class LatentMDGenModel(nn.Module):
    def __init__(self, args, latent_dim):
        super().__init__()
        self.args = args
        for flag in UNSUPPORTED_FLAGS:
            if getattr(args, flag, False):
                raise NotImplementedError(f"--{flag} is outside this build's scope (DESIGN.md §Scope)")
        C = args.embed_dim
        self.latent_dim = latent_dim
        self.tps = bool(getattr(args, "tps_condition", False))
        self.latent_to_emb = nn.Linear(latent_dim, C)
        if self.tps:
            self.latent_to_emb_f = nn.Linear(7, C)
            self.latent_to_emb_r = nn.Linear(7, C)
        self.cond_to_emb = nn.Linear(latent_dim, C)
        self.mask_to_emb = nn.Embedding(2, C)
        ipa_args = dict(c_s=C, c_z=0, c_hidden=args.ipa_head_dim, no_heads=args.ipa_heads,
                        no_qk_points=args.ipa_qk, no_v_points=args.ipa_v, dropout=args.dropout)
        if args.prepend_ipa:
            if not getattr(args, "no_aa_emb", False):
                self.aatype_to_emb = nn.Embedding(21, C)
            self.ipa_layers = nn.ModuleList([
                IPALayer(C, 4 * C, args.mha_heads, dropout=args.dropout,
                         use_rotary_embeddings=not args.no_rope, ipa_args=ipa_args)
                for _ in range(args.num_layers)])
        self.layers = nn.ModuleList([
            LatentMDGenLayer(C, 4 * C, args.mha_heads, dropout=args.dropout, num_frames=args.num_frames,
                             use_rotary_embeddings=not args.no_rope)
            for _ in range(args.num_layers)])
        self.emb_to_latent = FinalLayer(C, latent_dim)
        self.t_embedder = TimestepEmbedder(C)
        if args.abs_pos_emb:
            self.register_buffer("pos_embed", torch.zeros(1, args.crop, C))
        if getattr(args, "abs_time_emb", False):
            self.register_buffer("time_embed", torch.zeros(1, args.num_frames, C))
        self.initialize_weights()
        self.backend = "hip"
        self.train_backend = "hip"
        self._engine = None
        # [2, B, L, 7] device tensor of relative_tensor7(start, end) / (end, start) that a
        # captured training step fills on the host before each replay (train.GraphedStep)
        self._rel7_feed = None

    # ------------------------------------------------------------------ init (latent_model.py:134-177)
    def initialize_weights(self):
        def _basic_init(m):
            if isinstance(m, nn.Linear):
                torch.nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

        self.apply(_basic_init)
        if self.args.prepend_ipa:
            for block in self.ipa_layers:
                nn.init.constant_(block.ipa.linear_out.weight, 0)
                nn.init.constant_(block.ipa.linear_out.bias, 0)
        if self.args.abs_pos_emb:
            pe = get_1d_sincos_pos_embed_from_grid(self.pos_embed.shape[-1], np.arange(self.args.crop))
            self.pos_embed.data.copy_(torch.from_numpy(pe).float().unsqueeze(0))
        if getattr(self.args, "abs_time_emb", False):
            te = get_1d_sincos_pos_embed_from_grid(self.time_embed.shape[-1], np.arange(self.args.num_frames))
            self.time_embed.data.copy_(torch.from_numpy(te).float().unsqueeze(0))
        nn.init.normal_(self.t_embedder.mlp[0].weight, std=0.02)
        nn.init.normal_(self.t_embedder.mlp[2].weight, std=0.02)
        for block in self.layers:
            nn.init.constant_(block.adaLN_modulation[-1].weight, 0)
            nn.init.constant_(block.adaLN_modulation[-1].bias, 0)
        nn.init.constant_(self.emb_to_latent.adaLN_modulation[-1].weight, 0)
        nn.init.constant_(self.emb_to_latent.adaLN_modulation[-1].bias, 0)
        nn.init.constant_(self.emb_to_latent.linear.weight, 0)
        nn.init.constant_(self.emb_to_latent.linear.bias, 0)

    @property
    def device(self):
        return next(self.parameters()).device

    # ------------------------------------------------------------------ x-independent pieces
    def embed_time(self, t):
        """c = TEmb(t * time_multiplier)  [B, C]  (latent_model.py:252).  Differentiable calls on
        the HIP training path run the MLP on the segmented library linears."""
        if self._hip_glue(t):
            from ..train_hip import seg_linear
            from .layers import timestep_embedding

            te = self.t_embedder
            e = timestep_embedding(t * self.args.time_multiplier, te.frequency_embedding_size, freqs=te.freqs)
            h = seg_linear(e, [te.mlp[0]])[0]
            return seg_linear(h, [te.mlp[2]], act="silu")[0]
        return self.t_embedder(t * self.args.time_multiplier)

    def _hip_glue(self, x):
        """The conditioning's few-row linears on mdg_seg_linear: differentiable CUDA calls with
        the HIP training backend (MDG_TRAIN_SEG=0 keeps them eager)."""
        if self.backend != "hip" or getattr(self, "train_backend", "hip") != "hip":
            return False
        from ..train_hip import seg_supported

        return seg_supported(x)

    def run_ipa(self, c, mask_b, start_frames, end_frames, aatype, ada=None, rel7=None):
        """latent_model.py:179-214 (sim / TPS branches); c [B, C], mask_b [B, L]; ada: the IPA
        layers' adaLN outputs precomputed by _stacked_adaln (None: each layer computes its own);
        rel7: TPS's two relative 7-vectors [2, B, L, 7] when the caller has them (the replicated
        conditioning's all-gathered ones)."""
        B, L = mask_b.shape
        C = self.args.embed_dim
        rots, trans = frames_to_tensors(start_frames, mask_b.device)
        use_aa = aatype is not None and hasattr(self, "aatype_to_emb")
        # differentiable calls on a ROCm device: the IPA attention core runs the HIP training
        # kernels (mdg_ipa_core_fwd / _bwd) between the autograd projections
        hip_core = (self.backend == "hip" and getattr(self, "train_backend", "hip") == "hip" and mask_b.is_cuda
                    and torch.is_grad_enabled())
        # the MHA + MLP of each IPA layer on the HIP layer Function (the block stack's kernels)
        # wherever the block stack itself takes them
        hl = self._train_helper() if hip_core and self._use_hip_layers(mask_b) else None
        for layer in self.ipa_layers:
            layer.ipa.hip_core = hip_core
            layer.hip_hl = hl
        if not self.tps:
            x = torch.zeros(B, L, C, device=mask_b.device)
            if use_aa:
                x = x + self.aatype_to_emb(aatype)
            for k, layer in enumerate(self.ipa_layers):
                x = layer(x, c, mask_b, rots, trans, mods=None if ada is None else ada[k])
            return x
        erots, etrans = frames_to_tensors(end_frames, mask_b.device)
        if rel7 is not None:
            rel_f, rel_r = rel7[0], rel7[1]
        elif self._rel7_feed is not None:  # staged by the graphed training step (host eigh outside the graph)
            rel_f, rel_r = self._rel7_feed[0], self._rel7_feed[1]
        else:
            rel_f, rel_r = relative_tensor7(rots, trans, erots, etrans), relative_tensor7(erots, etrans, rots, trans)
        x_f = self.latent_to_emb_f(rel_f)
        x_r = self.latent_to_emb_r(rel_r)
        if use_aa:
            x_f = x_f + self.aatype_to_emb(aatype)
            x_r = x_r + self.aatype_to_emb(aatype)
        for k, layer in enumerate(self.ipa_layers):
            m = None if ada is None else ada[k]
            x_r = layer(x_r, c, mask_b, rots, trans, mods=m)
            x_f = layer(x_f, c, mask_b, erots, etrans, mods=m)
        return x_r + x_f

    # ------------------------------------------------------------------ forward
    def forward(self, x, t, mask, start_frames=None, end_frames=None, x_cond=None, x_cond_mask=None,
                aatype=None, *args, **kwargs):
        if mask.dim() == 2:  # latent_model.py:233-234
            mask = mask.repeat(x.shape[0], 1, 1)
        if self._use_hip(x):
            from ..engine import get_engine

            return get_engine(self).forward(x, t, mask, start_frames, end_frames, x_cond, x_cond_mask, aatype)
        return self.forward_torch(x, t, mask, start_frames, end_frames, x_cond, x_cond_mask, aatype)

    def forward_inference(self, x, t, mask, start_frames=None, end_frames=None, x_cond=None,
                          x_cond_mask=None, aatype=None):
        return self.forward(x, t, mask, start_frames, end_frames, x_cond, x_cond_mask, aatype)

    def _needs_grad(self, x):
        """True when autograd records this call: grad mode on and x or any parameter requires
        grad — whatever the module's train/eval mode (an eval()-mode prior used for guidance
        still has to return a differentiable output)."""
        if not torch.is_grad_enabled():
            return False
        return bool(x.requires_grad) or any(p.requires_grad for p in self.parameters())

    def _use_hip(self, x):
        """The graph-captured HIP inference engine (no autograd) serves a call only when nothing
        needs a gradient; differentiable calls go through forward_torch (whose block stack runs
        the HIP autograd kernels on a ROCm device, see _hip_blocks)."""
        if self.backend == "torch":
            return False
        if self.backend != "hip":
            raise ValueError(f"unknown backend {self.backend!r}")
        return not self._needs_grad(x)

    def forward_torch(self, x, t, mask, start_frames=None, end_frames=None, x_cond=None, x_cond_mask=None,
                      aatype=None):
        """Eager PyTorch forward (latent_model.py:216-269) — the training path."""
        if mask.dim() == 2:
            mask = mask.repeat(x.shape[0], 1, 1)
        hip_layers = self._use_hip_layers(x)
        from ..train_hip import glue_supported
        # the embedding and the FinalLayer on the glue kernels (train_hip.hip_embed / hip_final)
        glue = hip_layers and glue_supported(self, x.shape[2])
        if not glue:
            h = token_linear(self.latent_to_emb, x)
            if self.args.abs_pos_emb:
                h = h + self.pos_embed
            if getattr(self.args, "abs_time_emb", False):
                h = h + self.time_embed[:, :, None]
            if x_cond is not None:
                emb = (_SmallTableEmbedding.apply(self.mask_to_emb.weight, x_cond_mask) if torch.is_grad_enabled()
                       else self.mask_to_emb(x_cond_mask))
                h = h + token_linear(self.cond_to_emb, x_cond) + emb
        ckpt = bool(getattr(self.args, "grad_checkpointing", False)) and self.training
        cg = getattr(self, "_cond_gather", None)
        if cg is not None and cg.active and self.training and torch.is_grad_enabled():
            # data-parallel training (inside the Trainer's own step only): the conditioning on
            # the ranks' global batch, local rows kept (cond_dist.CondGather: its parameters'
            # gradients come out rank-averaged)
            c, ada, ipa = self._replicated_conditioning(cg, t, mask, start_frames, end_frames, aatype)
        else:
            c = self.embed_time(t)[:, None]
            # the HIP training path: every adaLN linear of the model as one stacked GEMM
            ada = self._stacked_adaln(c[:, 0]) if hip_layers else None
            ipa = None
            if self.args.prepend_ipa:
                ipa = self.run_ipa(c[:, 0], mask[:, 0], start_frames, end_frames, aatype,
                                   ada=None if ada is None else ada[0])
        if hip_layers:
            from ..train_hip import hip_embed, hip_final, hip_layer_forward, hip_layer_forward_chain
            hl = self._train_helper()
        pre = None
        if glue:
            h = hip_embed(hl, self, x, x_cond, x_cond_mask, ipa)
        elif ipa is not None:
            h = h + ipa[:, None]
        for k, layer in enumerate(self.layers):
            if hip_layers and ckpt:  # --grad_checkpointing: the HIP Function re-runs in backward
                # (reentrant form: the first forward runs without autograd, so the Function's
                # saved activations of every layer but the one being differentiated are freed)
                h = torch.utils.checkpoint.checkpoint(hip_layer_forward, hl, layer, h, ada[1][k], mask,
                                                      use_reentrant=True)
            elif hip_layers:  # block forward + backward in libmdgen_hip.so (train_hip.py); each layer's
                # fc2 also writes the next layer's first LayerNorm (the hand-off, no separate pass)
                nxt = ada[1][k + 1] if k + 1 < len(self.layers) else None
                h, pre = hip_layer_forward_chain(hl, layer, h, ada[1][k], mask, next_mods=nxt, pre=pre)
            elif getattr(self.args, "grad_checkpointing", False) and self.training:
                h = torch.utils.checkpoint.checkpoint(layer, h, c, mask, None if ada is None else ada[1][k],
                                                      use_reentrant=False)
            else:
                h = layer(h, c, mask, mods=None if ada is None else ada[1][k])
        if glue:
            return hip_final(hl, self.emb_to_latent, h, ada[2])
        return self.emb_to_latent(h, c, mods=None if ada is None else ada[2][:, None])

    def _replicated_conditioning(self, cg, t, mask, start_frames, end_frames, aatype):
        """(c [B,1,C], (IPA mods, block mods, final mods), ipa [B,L,C]) of this rank's samples,
        computed on the all-gathered batch of every rank (cond_dist.py).  TPS: the end frames and
        the relative 7-vectors (host eigh of the local frames, or the graphed step's staged
        buffer) travel in the same gather."""
        B, L = mask.shape[0], mask.shape[2]
        C = self.args.embed_dim
        rots, trans = frames_to_tensors(start_frames, mask.device)
        if rots is None:
            rots = torch.eye(3, device=mask.device).expand(B, L, 3, 3)
            trans = torch.zeros(B, L, 3, device=mask.device)
        tps = None
        if self.tps and self.args.prepend_ipa:
            erots, etrans = frames_to_tensors(end_frames, mask.device)
            if self._rel7_feed is not None:
                rel7 = self._rel7_feed
            else:
                rel7 = torch.stack([relative_tensor7(rots, trans, erots, etrans),
                                    relative_tensor7(erots, etrans, rots, trans)])
            tps = (erots, etrans, rel7)
        gathered = cg.gather_inputs(t, mask[:, 0], rots, trans, aatype, tps=tps)
        t_g, mask_g, rots_g, trans_g, aa_g = gathered[:5]
        W = t_g.shape[0]
        c_g = self.embed_time(t_g)
        ada_g = self._stacked_adaln(c_g)
        pieces = [c_g] + list(ada_g[1]) + [ada_g[2]]
        if self.args.prepend_ipa:
            def rigid4(r, tr):
                fr = torch.zeros(W, L, 4, 4, device=mask.device)
                fr[..., :3, :3] = r
                fr[..., :3, 3] = tr
                fr[..., 3, 3] = 1.0
                return fr

            if tps is None:
                ipa_g = self.run_ipa(c_g, mask_g, rigid4(rots_g, trans_g), None, aa_g, ada=ada_g[0])
            else:
                erots_g, etrans_g, rel_g = gathered[5]
                ipa_g = self.run_ipa(c_g, mask_g, rigid4(rots_g, trans_g), rigid4(erots_g, etrans_g), aa_g,
                                     ada=ada_g[0], rel7=rel_g)
            pieces.append(ipa_g.reshape(W, L * C))
        loc = torch.split(cg.local(torch.cat(pieces, -1)), [p.shape[-1] for p in pieces], -1)
        nl = len(self.layers)
        c = loc[0][:, None]
        ada = (None, list(loc[1:1 + nl]), loc[1 + nl])
        ipa = loc[2 + nl].reshape(B, L, C) if self.args.prepend_ipa else None
        return c, ada, ipa

    def _stacked_adaln(self, c0):
        """Every adaLN linear (IPA layers 6C, blocks 9C, FinalLayer 2C: latent_model.py:341-493,
        layers.py:58-75) over SiLU(c) as ONE GEMM of the concatenated weights; returns
        ([IPA layer mods], [block mods], final mods).  The 11 separate SiLU + Linear pairs were
        ~70 forward + backward kernels of the training step on 8 rows."""
        ipa = list(self.ipa_layers) if self.args.prepend_ipa else []
        mods = [l.adaLN_modulation for l in ipa] + [l.adaLN_modulation for l in self.layers] + \
            [self.emb_to_latent.adaLN_modulation]
        lin = [m[-1] for m in mods]
        if self._hip_glue(c0) and len(lin) <= 16:  # one library launch, no concatenated weights
            from ..train_hip import seg_linear

            parts = seg_linear(c0, lin, act="silu")
        else:
            y = F.linear(F.silu(c0), torch.cat([l.weight for l in lin]), torch.cat([l.bias for l in lin]))
            parts = torch.split(y, [l.out_features for l in lin], -1)
        return list(parts[:len(ipa)]), list(parts[len(ipa):len(ipa) + len(self.layers)]), parts[-1]

    def _use_hip_layers(self, h):
        """Differentiable calls on a ROCm device run the block stack through the HIP training
        Function (train_backend 'hip', the default); dropout > 0 while training and head_dims the
        kernels do not take (>= 64, or not a multiple of 4) are not built there and take eager
        autograd, with a warning.  head_dim 32..63 runs on 64-column attention planes (ABI 23)."""
        if self.backend != "hip" or getattr(self, "train_backend", "hip") != "hip" or not h.is_cuda:
            return False
        if not torch.is_grad_enabled():
            return False
        why = None
        hd = self.args.embed_dim // self.args.mha_heads
        if hd >= 64 or hd % 4:  # the training kernels' planes: MDG_HEAD_STRIDE(D) <= 64 columns
            why = f"head_dim {hd} (the kernels take multiples of 4 below 64)"
        elif self.training and float(getattr(self.args, "dropout", 0.0) or 0.0) > 0.0:
            why = f"--dropout {self.args.dropout} (attention-probability dropout, mha.py:383)"
        if why is not None:
            if getattr(self, "_hip_refusal", None) != why:  # logged once per reason, never silent
                self._hip_refusal = why
                warnings.warn(f"LatentMDGenModel: the HIP training kernels do not take {why}; the block "
                              "stack runs eager PyTorch autograd on the device (slower, same arithmetic)",
                              RuntimeWarning, stacklevel=3)
            return False
        return True

    def _train_helper(self):
        from ..train_hip import LayerHelper

        dt = getattr(self, "hip_dtype", "bf16")
        hl = getattr(self, "_hip_train", None)
        if hl is None:
            hl = LayerHelper(self, dt)
            self._hip_train = hl
        elif hl.dtype_name != dt:
            hl.set_dtype(dt)
        return hl


def relative_tensor7(rots_a, trans_a, rots_b, trans_b):
    """a.invert().compose(b).to_tensor_7() for the TPS branch (latent_model.py:198-199), in
    the reference's exact operation order (Rigid.invert 1075-1087, Rigid.compose 1031-1045,
    rot_matmul 24-57, rot_vec_mul 64-86, to_tensor_7 1143-1155) on the HOST in fp32.

    The quaternion comes from an eigenvector (rot_to_quat, rigid_utils.py:191-210) whose sign
    flips under 1-ulp changes of the composed rotation for a sizeable fraction of residues, and
    latent_to_emb_f/_r are linear in it — so this x-independent, once-per-window precompute
    reproduces the reference's host arithmetic (CPU eigh).  The HIP engine uses this same
    function by default (engine._prepare_tps), so training and sampling condition alike; its
    device alternative (MDG_TPS_REL7=device, mdg_tps_rel7) fixes the sign to w >= 0 instead."""
    dev = rots_a.device
    ra, ta, rb, tb = (z.detach().float().cpu() for z in (rots_a, trans_a, rots_b, trans_b))
    ra_inv = ra.transpose(-1, -2)

    def rvm(r, t):
        x, y, z = torch.unbind(t, dim=-1)
        return torch.stack([r[..., i, 0] * x + r[..., i, 1] * y + r[..., i, 2] * z for i in range(3)], dim=-1)

    def rmm(a, b):
        rows = [torch.stack([a[..., i, 0] * b[..., 0, j] + a[..., i, 1] * b[..., 1, j] + a[..., i, 2] * b[..., 2, j]
                             for j in range(3)], dim=-1) for i in range(3)]
        return torch.stack(rows, dim=-2)

    t_inv = -1 * rvm(ra_inv, ta)
    rot = rmm(ra_inv, rb)
    tr = rvm(ra_inv, tb) + t_inv
    return torch.cat([rot_to_quat(rot), tr], -1).to(dev)


__all__ = ["LatentMDGenModel", "LatentMDGenLayer", "IPALayer", "Rotation", "F"]
