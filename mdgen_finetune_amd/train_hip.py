"""HIP training path: a LatentMDGenLayer's forward AND backward on libmdgen_hip.so.

The reference trains the block with eager PyTorch autograd (Transport.training_losses ->
model(xt, t, **kw) -> loss.backward(): transport.py:137-222, wrapper.py:367-403; the block
latent_model.py:456-493).  Here each block is one ``torch.autograd.Function``:

forward   ``mdg_layer_fwd_train``: LN + adaLN modulate (with row statistics) -> q|k|v GEMM +
          RoPE -> spatial / temporal attention (temporal with per-row log2-sum-exp2) -> out_proj
          GEMM with the gated residual out of place (pre-gate output kept) -> ... -> fc1 GEMM
          (pre-activation kept) -> fc2 gated residual.  Everything is saved on device for the
          backward; nothing is recomputed by torch.
backward  per sublayer, top down:
            mdg_ln_gate_bwd     LN/modulate backward of sublayer k fused with the gated-residual
                                backward of sublayer k-1 (dh, dy = dh * gate, adaLN and bias
                                gradient partials);
            mdg_gemm            input gradients dX = dY W through the HIP GEMM (W^T from the
                                forward's mdg_train_pack_layer); fc1's with the GELU-derivative
                                epilogue (MDG_ACT_DGELU);
            mdg_attn_*_bwd      flash-style attention backward (P recomputed from the saved lse),
                                RoPE / q-scale undone in the epilogue, bias_k / bias_v partials;
            mdg_wgrad           the weight and bias gradients dW = dY^T X, db = colsum(dY) from
                                the token-major operands (MFMA tiles fed by transposing LDS
                                reads, split over token chunks, fp32 partials summed in
                                chunk order: deterministic; csrc/wgrad.hip).
mdg_train_pack_layer (forward) / mdg_train_unpack_layer (backward) move the parameters into
the kernels' layouts and the gradients back (csrc/pack_train.hip), one launch each.
The adaLN modulation vectors enter as a [B, 9C] input of the Function, so the t-embedding /
adaLN linears upstream stay ordinary autograd modules (x-independent, tiny).

Parity: the f32 dtype (``model.hip_dtype = 'f32'``) runs exact-f32 MFMA / scalar kernels and
matches eager autograd to ~1e-5 relative; bf16 (the default) rounds GEMM / attention operands
to bf16 with fp32 accumulation — ``torch.set_float32_matmul_precision('medium')`` semantics, as
the reference's train.py:13 requests.  tests/test_gpu_train.py states the tolerances.
"""
from __future__ import annotations

import ctypes
import math
import os
import weakref

import torch

from . import _lib

_LN2 = math.log(2.0)
# temporal attention backward: the fused single-pass kernel (default) or the two-pass MFMA kernels
# (MDG_ATTN_BWD=2pass, for A/B measurements); see mdg_attn_temporal_bwd's `generic`
_ATTN_BWD_VARIANT = {"fused": 0, "2pass": 2}[os.environ.get("MDG_ATTN_BWD", "fused")]
_PLANE_CACHE_MAX = 64  # plane cache entries (layer x tag) before stale ones are dropped


class _PlaneLease:
    """Held by a training call's autograd context while its planes are in use."""


def pad_tokens(n):
    """Token rows of every buffer the weight-gradient kernel reads: a multiple of 32 (its
    bf16 K-step); the rows past n are zero."""
    return (n + 31) // 32 * 32


def _rows(n, cols, dtype, dev):
    """[pad_tokens(n)][cols] buffer whose pad rows are zero (kernels write rows < n)."""
    t = torch.empty(pad_tokens(n), cols, device=dev, dtype=dtype)
    if t.shape[0] > n:
        t[n:].zero_()
    return t


def _src(t):
    """Device pointer of an fp32 contiguous parameter (the pack kernel's source layout)."""
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise RuntimeError(f"HIP training layer: parameter of dtype {t.dtype} / strides {t.stride()} "
                           "(fp32 contiguous expected)")
    return t.data_ptr()


def wgrad(lib, mdg_dtype, dy, x, need_b=False):
    """(dW = dy^T x, db = colsum(dy)) in fp32 through mdg_wgrad; dy [Np][M], x [Np][K] token
    rows (pad rows zero), x None -> only db."""
    n, M = dy.shape
    K = x.shape[1] if x is not None else 8
    need_w = x is not None
    wsb = lib.mdg_wgrad_workspace_bytes(mdg_dtype, n, M, K, int(need_w), int(need_b))
    ws = torch.empty(wsb, device=dy.device, dtype=torch.uint8)
    dw = torch.empty(M, K, device=dy.device) if need_w else None
    db = torch.empty(M, device=dy.device) if need_b else None
    _lib.check(lib.mdg_wgrad(mdg_dtype, n, M, K, dy.data_ptr(), dy.stride(0), _lib.ptr(x),
                             x.stride(0) if need_w else 0, _lib.ptr(dw), K, _lib.ptr(db), ws.data_ptr(), wsb,
                             _lib.stream_handle()), "mdg_wgrad")
    return dw, db


class LayerHelper:
    """Per-model state of the HIP training path: ctypes library, RoPE tables per length, dtype."""

    def __init__(self, model, dtype="bf16"):
        self.model = model
        self.lib = _lib.load()
        a = model.args
        self.C, self.H = a.embed_dim, a.mha_heads
        self.D = self.C // self.H
        self.F = 4 * self.C
        self.rope = not a.no_rope
        self.set_dtype(dtype)
        self._tables = {}

    def __getstate__(self):
        """Picklable (the model and its IPA layers keep a reference): the ctypes library and
        the device tables are rebuilt on demand."""
        st = dict(self.__dict__)
        st["lib"], st["_tables"], st["_planes"] = None, {}, {}
        st["_kb"] = {}
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self.lib = _lib.load() if os.path.exists(_lib.LIB_PATH) else None

    def set_dtype(self, dtype):
        if dtype not in ("bf16", "f32"):
            raise ValueError(f"hip_dtype must be 'bf16' or 'f32', got {dtype!r}")
        self.dtype_name = dtype
        self.mdg_dtype = _lib.MDG_BF16 if dtype == "bf16" else _lib.MDG_F32
        self.ct = torch.bfloat16 if dtype == "bf16" else torch.float32

    def table(self, n_rows, inv_freq):
        """cos | sin [n_rows][D/2] (fair-esm: fp32 outer product on the CPU, then cos / sin)."""
        key = (n_rows, inv_freq.device)
        t = self._tables.get(key)
        if t is None:
            inv = inv_freq.detach().float().cpu()
            freqs = torch.einsum("i,j->ij", torch.arange(n_rows).type_as(inv), inv)
            t = torch.cat([freqs.cos().reshape(-1), freqs.sin().reshape(-1)]).to(inv_freq.device)
            self._tables[key] = t
        return t

    def mask_bias(self, mask, B, T, L, s, src=None):
        """(kb_t [B*L][T], kb_s [B*T][L]): the key-padding biases of the block stack's mask
        (mdg_mask_bias), computed once per mask and shared by every layer of the pass.  The
        entry holds the mask itself, so an equal (address, version, shape, strides) key is the
        same, unchanged data; inside a capture the first layer's launch is recorded and
        recomputes them on every replay, which the later layers read."""
        # (views share their base's version counter; the held reference keeps the storage, so
        # the address cannot be reused by another tensor while the entry lives)
        # (an entry made outside a stream capture is never used inside one and vice versa: a
        # captured pass must record its own launch, which every replay then repeats)
        key = (mask.data_ptr(), mask._version, tuple(mask.shape), tuple(mask.stride()), str(mask.device),
               mask.is_cuda and torch.cuda.is_current_stream_capturing())
        cache = self.__dict__.setdefault("_kb", {})
        ent = cache.get(key)
        if ent is not None:
            return ent[1], ent[2]
        dev = mask.device
        kb_t = torch.empty(B * L, T, device=dev)
        kb_s = torch.empty(B * T, L, device=dev)
        src = mask if src is None else src  # (the contiguous fp32 form of the keyed mask)
        _lib.check(self.lib.mdg_mask_bias(B, T, L, src.data_ptr(), kb_t.data_ptr(), kb_s.data_ptr(), s),
                   "mdg_mask_bias")
        if len(cache) >= 2:  # the IPA layers' and the blocks' masks
            cache.pop(next(iter(cache)))
        cache[key] = (mask, kb_t, kb_s)
        return kb_t, kb_s

    def planes(self, key, shape, device, owner):
        """(buffer, fresh): persistent padded q|k|v planes of one layer (key = (tag, layer id,
        B, T, L)); fresh = just allocated, so its pad columns still need mdg_layer_fwd_train's
        init_planes pass.  The planes are also saved activations of the call's backward, so a
        buffer is lent to one forward at a time: ``owner`` (an object the autograd context
        holds until its backward has run) marks the slot in use, and a second forward of the
        same layer and shape before that backward (TPS runs every IPA layer twice per step,
        latent_model.py:240-243) gets a slot of its own.  Only the latest shape of each layer
        is kept (a new shape drops the old slots; buffers still lent stay alive through their
        contexts)."""
        cache = self.__dict__.setdefault("_planes", {})
        tag, shape_key = key[:2] + (self.dtype_name, str(device)), key[2:]
        ent = cache.get(tag)
        if ent is None or ent[0] != shape_key:
            ent = cache[tag] = (shape_key, [])
            if len(cache) > _PLANE_CACHE_MAX:  # stale layer ids (re-allocated parameters)
                for k in [k for k, (_, slots) in cache.items() if k != tag and all(r() is None for _, r in slots)]:
                    del cache[k]
        for slot in ent[1]:
            if slot[1]() is None:
                slot[1] = weakref.ref(owner)
                return slot[0], False
        buf = torch.empty(*shape, device=device, dtype=self.ct)
        ent[1].append([buf, weakref.ref(owner)])
        return buf, True

    def dims(self, B, T, L):
        return _lib.MdgDims(B=B, T=T, L=L, C=self.C, H=self.H, D=self.D, F=self.F, latent=self.model.latent_dim,
                            num_layers=self.model.args.num_layers, dtype=self.mdg_dtype)


def _layer_params(layer):
    out = []
    for mha in (layer.mha_l.attn, layer.mha_t.attn):
        out += [mha.q_proj.weight, mha.q_proj.bias, mha.k_proj.weight, mha.k_proj.bias, mha.v_proj.weight,
                mha.v_proj.bias, mha.out_proj.weight, mha.out_proj.bias, mha.bias_k, mha.bias_v]
    out += [layer.fc1.weight, layer.fc1.bias, layer.fc2.weight, layer.fc2.bias]
    return out


def hip_layer_forward(hl, layer, h, mods, mask):
    """h [B,T,L,C] fp32, mods [B, 9C] (adaLN output), mask [B,T,L] -> layer(h) through the
    HIP training Function."""
    inv_freq = layer.mha_l.attn.rot_emb.inv_freq if hl.rope else None
    return _HipLayerFn.apply(h, mods, mask, hl, inv_freq, False, None, *_layer_params(layer))


def hip_layer_forward_chain(hl, layer, h, mods, mask, next_mods=None, pre=None):
    """hip_layer_forward with the layer-to-layer LayerNorm hand-off: the layer's fc2 also writes
    the NEXT layer's first LayerNorm + modulate (next_mods = that layer's adaLN rows [B, 9C]) and
    its row statistics, which the next call takes as ``pre`` instead of running its own pass
    (mdg_layer_saved.xn_next / xn0_given).  Returns (h_out, pre for the next layer or None)."""
    inv_freq = layer.mha_l.attn.rot_emb.inv_freq if hl.rope else None
    chain = (None if next_mods is None else next_mods.detach(), pre)
    out = _HipLayerFn.apply(h, mods, mask, hl, inv_freq, False, chain, *_layer_params(layer))
    if next_mods is None:
        return out, None
    return out[0], (out[1], out[2])


class _Mods9(torch.autograd.Function):
    """[B, 6C] adaLN rows -> [B, 9C] with three zero chunks in the temporal slots (one
    concatenation against a cached zero block forward, one concatenation of the two kept slices
    backward: autograd's cat / new_zeros pair took a fill + a copy each way and a fill, two copies
    and an add back, per IPA layer and step)."""
    _zeros = {}

    @staticmethod
    def forward(ctx, mods6, C):
        key = (mods6.shape[0], C, mods6.dtype, mods6.device)
        z = _Mods9._zeros.get(key)
        if z is None:
            z = torch.zeros(mods6.shape[0], 3 * C, dtype=mods6.dtype, device=mods6.device)
            # (a block made inside a stream capture belongs to that graph's pool: not cached; the
            # cached ones are never evicted — a captured graph may hold their address — and are a
            # few KiB per (B, C))
            if not (z.is_cuda and torch.cuda.is_current_stream_capturing()):
                _Mods9._zeros[key] = z
        ctx.C = C
        return torch.cat([mods6[:, :3 * C], z, mods6[:, 3 * C:]], -1)

    @staticmethod
    def backward(ctx, g):
        C = ctx.C
        return torch.cat([g[:, :3 * C], g[:, 6 * C:]], -1), None


def hip_ipa_layer_tail(hl, layer, x1, mods6, mask_b):
    """IPALayer (latent_model.py:341-394) after its IPA sublayer: x1 + g_l MHA_L(mod(LN x1)),
    then + g_m MLP(mod(LN .)), on the HIP training Function as a T = 1 block whose temporal
    sublayer has gate 0: adaLN rows [sh_l, sc_l, g_l, 0, 0, 0, sh_m, sc_m, g_m].  With g_t = 0
    the temporal branch adds exactly 0 forward and passes exactly 0 gradient back (dy_t = dh * 0),
    so this is the IPA layer's arithmetic; its stand-in weights (mha_l's again) would receive zero
    gradients, so the Function returns None for them (``tail``: no gradient accumulation of the
    shared parameters).  x1 [B, L, C], mods6 [B, 6C], mask_b [B, L]."""
    C = hl.C
    inv_freq = layer.mha_l.attn.rot_emb.inv_freq if hl.rope else None
    mods9 = _Mods9.apply(mods6, C)
    mha = layer.mha_l.attn
    att = [mha.q_proj.weight, mha.q_proj.bias, mha.k_proj.weight, mha.k_proj.bias, mha.v_proj.weight, mha.v_proj.bias,
           mha.out_proj.weight, mha.out_proj.bias, mha.bias_k, mha.bias_v]
    params = att + att + [layer.fc1.weight, layer.fc1.bias, layer.fc2.weight, layer.fc2.bias]
    out = _HipLayerFn.apply(x1[:, None], mods9, mask_b[:, None], hl, inv_freq, True, None, *params)
    return out[:, 0]


class _HipLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, mods, mask, hl, inv_freq, tail, chain, *params):
        """chain: None, or (next_mods [B, 9C] detached | None, pre (xn0, stats0) | None): the
        layer-to-layer LayerNorm hand-off of hip_layer_forward_chain."""
        lib = hl.lib
        B, T, L, C = h.shape
        H, D, F, ct = hl.H, hl.D, hl.F, hl.ct
        N, dev = B * T * L, h.device
        s = _lib.stream_handle()
        h = h.contiguous().float()
        mods = mods.contiguous().float()
        mask_key = mask  # the caller's tensor: the same object for every layer of a pass
        mask = mask.contiguous().float()
        # the layer's operands in the kernels' layouts (q / k rows pair-interleaved, CT casts, the
        # transposes the backward's input-gradient GEMMs read, RoPE-rotated bias key): one launch
        # (mdg_train_pack_layer; ~35 PyTorch kernels per layer before)
        ee = lambda *shape, dt=ct: torch.empty(*shape, device=dev, dtype=dt)  # noqa: E731
        P = {}
        pk = _lib.MdgTrainPack(C=C, H=H, D=D, F=F, rope=int(hl.rope), dtype=hl.mdg_dtype)
        tabs = []
        for i in range(2):
            wq, bq, wk, bk, wv, bv, wo, bo, bias_k, bias_v = [t.detach() for t in params[10 * i:10 * i + 10]]
            for name, t in (("wq", wq), ("wk", wk), ("wv", wv), ("bq", bq), ("bk", bk), ("bv", bv), ("wo", wo),
                            ("bias_k", bias_k), ("bias_v", bias_v)):
                getattr(pk, name)[i] = _src(t)
            P[f"wqkv{i}"], P[f"wqkv_t{i}"], P[f"bqkv{i}"] = ee(3 * C, C), ee(C, 3 * C), ee(3 * C, dt=torch.float32)
            P[f"wo{i}"], P[f"wo_t{i}"] = ee(C, C), ee(C, C)
            P[f"bo{i}"] = bo.float().contiguous()
            P[f"kvb{i}"] = ee(H, 2, _lib.head_stride(D), dt=torch.float32)
            S, rows = (L, L + 1) if i == 0 else (T, T + 1)
            tab = hl.table(rows, inv_freq) if hl.rope else None
            tabs.append(tab)
            pk.rope_tab[i], pk.rope_rows[i], pk.rope_pos[i] = _lib.ptr(tab), rows, S
            pk.wqkv[i], pk.wqkv_t[i], pk.bqkv[i] = P[f"wqkv{i}"].data_ptr(), P[f"wqkv_t{i}"].data_ptr(), \
                P[f"bqkv{i}"].data_ptr()
            pk.wo_p[i], pk.wo_t[i], pk.kvb[i] = P[f"wo{i}"].data_ptr(), P[f"wo_t{i}"].data_ptr(), P[f"kvb{i}"].data_ptr()
        w1, b1, w2, b2 = [t.detach() for t in params[20:24]]
        pk.w1, pk.w2 = _src(w1), _src(w2)
        P["w1"], P["w1_t"], P["w2"], P["w2_t"] = ee(F, C), ee(C, F), ee(C, F), ee(F, C)
        P["b1"], P["b2"] = b1.float().contiguous(), b2.float().contiguous()
        pk.w1_p, pk.w1_t, pk.w2_p, pk.w2_t = (P[k].data_ptr() for k in ("w1", "w1_t", "w2", "w2_t"))
        _lib.check(lib.mdg_train_pack_layer(ctypes.byref(pk), s), "mdg_train_pack_layer")
        rope_l, rope_t = tabs
        lw = _lib.MdgLayerWeights()
        for i in range(2):
            lw.wqkv[i], lw.bqkv[i] = P[f"wqkv{i}"].data_ptr(), P[f"bqkv{i}"].data_ptr()
            lw.wo[i], lw.bo[i], lw.kvb[i] = P[f"wo{i}"].data_ptr(), P[f"bo{i}"].data_ptr(), P[f"kvb{i}"].data_ptr()
        lw.w1, lw.b1, lw.w2, lw.b2 = P["w1"].data_ptr(), P["b1"].data_ptr(), P["w2"].data_ptr(), P["b2"].data_ptr()
        dims = hl.dims(B, T, L)
        long_l = L >= 16
        kb_t, kb_s = hl.mask_bias(mask_key, B, T, L, s, src=mask)
        e = lambda *shape, dt=ct: torch.empty(*shape, device=dev, dtype=dt)  # noqa: E731
        r = lambda cols: _rows(N, cols, ct, dev)  # noqa: E731  (operands of the weight gradients)
        # the padded attention planes persist per layer and shape: their pad columns (0, and 1.0 in
        # k / v column D) are written once (init_planes) instead of a memset + set_vpad pass per
        # step; the q|k|v GEMM rewrites every other column each forward
        lease = _PlaneLease()
        dp = _lib.head_stride(D)  # 32, or 64 for head_dim 32..63
        planes_t, fresh_t = hl.planes(("t", params[0].data_ptr(), B, T, L), (3, B * L, H, T, dp), dev, lease)
        planes_s, fresh_s = (hl.planes(("s", params[0].data_ptr(), B, T, L), (3, B * T, H, L, dp), dev,
                                       lease) if long_l else (e(N, 3 * C), False))
        next_mods, pre = chain if chain is not None else (None, None)
        sv = {"xn": [r(C) for _ in range(3)], "stats": [e(N, 2, dt=torch.float32) for _ in range(3)],
              "qkv_s": planes_s,
              "lse_s": e(B * T, H, L, dt=torch.float32) if long_l else None,
              "qkv_t": planes_t, "lse_t": e(B * L, H, T, dt=torch.float32),
              "o": [r(C), r(C)], "y": [e(N, C) for _ in range(3)],
              # bf16: O - bf16(O) of the attentions on the temporal kernel (the backward's delta)
              "o_lo": [e(N, C) if (ct == torch.bfloat16 and long_l) else None,
                       e(N, C) if ct == torch.bfloat16 else None],
              "h1": e(N, C, dt=torch.float32), "h2": e(N, C, dt=torch.float32), "u": e(N, F), "act": r(F)}
        if pre is not None:  # LN_s(h) from the previous layer's fc2 epilogue
            sv["xn"][0], sv["stats"][0] = pre
        nxt = None
        if next_mods is not None:
            nxt = (r(C), e(N, 2, dt=torch.float32))
            next_mods = next_mods.contiguous().float()
        cs = _lib.MdgLayerSaved()
        cs.xn0_given = int(pre is not None)
        if nxt is not None:
            cs.xn_next, cs.stats_next, cs.mods_next = nxt[0].data_ptr(), nxt[1].data_ptr(), next_mods.data_ptr()
        for i in range(3):
            cs.xn[i], cs.stats[i], cs.y[i] = sv["xn"][i].data_ptr(), sv["stats"][i].data_ptr(), sv["y"][i].data_ptr()
        cs.qkv_s, cs.lse_s = sv["qkv_s"].data_ptr(), _lib.ptr(sv["lse_s"])
        cs.qkv_t, cs.lse_t = sv["qkv_t"].data_ptr(), sv["lse_t"].data_ptr()
        cs.o[0], cs.o[1] = sv["o"][0].data_ptr(), sv["o"][1].data_ptr()
        cs.o_lo[0], cs.o_lo[1] = _lib.ptr(sv["o_lo"][0]), _lib.ptr(sv["o_lo"][1])
        cs.h1, cs.h2, cs.u, cs.act = sv["h1"].data_ptr(), sv["h2"].data_ptr(), sv["u"].data_ptr(), sv["act"].data_ptr()
        cs.init_planes = int(fresh_t or fresh_s)
        cs.skip_temporal = int(bool(tail))  # the IPA layers' tail: gate 0, h2 = h1
        h_out = torch.empty_like(h)
        _lib.check(lib.mdg_layer_fwd_train(ctypes.byref(dims), ctypes.byref(lw), _lib.ptr(rope_l), _lib.ptr(rope_t),
                                           mods.data_ptr(), mask.data_ptr(), kb_t.data_ptr(), kb_s.data_ptr(),
                                           h.data_ptr(), h_out.data_ptr(), ctypes.byref(cs), s),
                   "mdg_layer_fwd_train")
        ctx.hl, ctx.sv, ctx.P, ctx.lease = hl, sv, P, lease
        ctx.shape, ctx.tail = (B, T, L), tail
        ctx.kb = (kb_t, kb_s)
        ctx.mask = mask
        ctx.rope = (rope_l, rope_t)
        ctx.inv_freq = inv_freq
        ctx.save_for_backward(h, mods)
        if nxt is None:
            return h_out
        ctx.mark_non_differentiable(nxt[0], nxt[1])
        # the hand-off outputs' gradients stay None (materialized they were two zero fills per
        # layer and step)
        ctx.set_materialize_grads(False)
        return h_out, nxt[0], nxt[1]

    @staticmethod
    def backward(ctx, dh3, *_next_grads):  # (the hand-off outputs are non-differentiable)
        hl, sv, P = ctx.hl, ctx.sv, ctx.P
        lib = hl.lib
        h, mods = ctx.saved_tensors
        B, T, L = ctx.shape
        C, H, D, F, ct, dt = hl.C, hl.H, hl.D, hl.F, hl.ct, hl.mdg_dtype
        N, TL, dev = B * T * L, T * L, h.device
        s = _lib.stream_handle()
        rope_l, rope_t = ctx.rope
        kb_t, kb_s = ctx.kb
        if dh3 is None:  # (set_materialize_grads(False): h_out unused downstream)
            dh3 = torch.zeros(B, T, L, C, device=h.device)
        dh3 = dh3.contiguous().float().reshape(N, C)
        mods = mods.contiguous()
        nblk = lib.mdg_ln_gate_bwd_blocks(TL)
        qscale = D ** -0.5
        e = lambda *shape, dtp=ct: torch.empty(*shape, device=dev, dtype=dtp)  # noqa: E731
        r = lambda cols: _rows(N, cols, ct, dev)  # noqa: E731
        wg = lambda dy, x, need_b=False: wgrad(lib, dt, dy, x, need_b)  # noqa: E731

        def lngate(dxn, h_ln, stats, shift_off, scale_off, dh_res, dh_out, y, gate_off, dy):
            part = torch.empty(B, nblk, 4, C, device=dev)
            _lib.check(lib.mdg_ln_gate_bwd(dt, N, C, TL, _lib.ptr(dxn), _lib.ptr(h_ln), _lib.ptr(stats),
                                           mods.data_ptr(), 9 * C, shift_off, scale_off, dh_res.data_ptr(),
                                           dh_out.data_ptr(), _lib.ptr(y), gate_off, _lib.ptr(dy), part.data_ptr(), s),
                       "mdg_ln_gate_bwd")
            return part

        def dx_gemm(dy, w_t, K, Nout, act=_lib.MDG_ACT_NONE, aux=None):
            """out [N][Nout] (CT) = dy [N][K] . w_t^T with w_t = W^T [Nout][K]."""
            out = r(Nout)
            g = _lib.MdgGemmDesc()
            g.dtype, g.a_mode, g.epi, g.act = dt, _lib.MDG_A_PLAIN, _lib.MDG_EPI_STORE, act
            g.M, g.N, g.K = N, Nout, K
            g.A, g.lda, g.W, g.ldw = dy.data_ptr(), K, w_t.data_ptr(), K
            g.out, g.ldo = out.data_ptr(), Nout
            if aux is not None:
                g.aux, g.ldaux = aux.data_ptr(), Nout
            _lib.check(lib.mdg_gemm(ctypes.byref(g), s), "mdg_gemm(dX)")
            return out

        grads = {}
        # ---- MLP: h3 = h2 + g_m * (fc2(gelu(fc1(xn3))))
        dy_m = r(C)
        part_m = lngate(None, None, None, 0, 0, dh3, dh3, sv["y"][2], 8 * C, dy_m)
        grads["w2"], _ = wg(dy_m, sv["act"])
        du = dx_gemm(dy_m, P["w2_t"], C, F, _lib.MDG_ACT_DGELU, sv["u"])
        grads["w1"], grads["b1"] = wg(du, sv["xn"][2], True)
        dxn3 = dx_gemm(du, P["w1_t"], F, C)

        def attention(i, dy, o, o_lo, xn, qkv, lse):
            """out_proj + attention backward of attention i (0 spatial, 1 temporal); returns dxn."""
            grads[f"wo{i}"], _ = wg(dy, o)
            do = dx_gemm(dy, P[f"wo_t{i}"], C, C)
            dqkv = r(3 * C)
            if i == 1 or L >= 16:
                Bq, Tq, Lq = (B, T, L) if i == 1 else (B * T, L, 1)
                rope, rows = (rope_t, T + 1) if i == 1 else (rope_l, L + 1)
                kb = kb_t if i == 1 else kb_s
                # the wide heads (head_dim 32..63) take the scalar kernels (generic 1)
                variant = _ATTN_BWD_VARIANT if D < _lib.MDG_DP else 1
                parts = lib.mdg_attn_temporal_bwd_parts(dt, Bq, Tq, Lq, variant)
                bpart = torch.empty(H, parts, 2, _lib.head_stride(D), device=dev)  # every slot is written
                scratch = torch.empty(lib.mdg_attn_temporal_bwd_scratch(dt, Bq, Tq, Lq, H, D), device=dev,
                                      dtype=torch.uint8)
                _lib.check(lib.mdg_attn_temporal_bwd(dt, Bq, Tq, Lq, H, D, qkv.data_ptr(), kb.data_ptr(),
                                                     P[f"kvb{i}"].data_ptr(), o.data_ptr(), _lib.ptr(o_lo),
                                                     do.data_ptr(),
                                                     lse.data_ptr(), _lib.ptr(rope), rows, scratch.data_ptr(),
                                                     dqkv.data_ptr(), 3 * C, bpart.data_ptr(), qscale, _LN2,
                                                     variant, s),
                           "mdg_attn_temporal_bwd")
            else:
                parts = lib.mdg_attn_spatial_bwd_parts(B * T, L, H, D)
                bpart = torch.empty(H, parts, 2, _lib.head_stride(D), device=dev)
                _lib.check(lib.mdg_attn_spatial_bwd(dt, B * T, L, H, D, qkv.data_ptr(), P["kvb0"].data_ptr(),
                                                    ctx.mask.data_ptr(), do.data_ptr(), _lib.ptr(rope_l), L + 1,
                                                    dqkv.data_ptr(), bpart.data_ptr(), qscale, s),
                           "mdg_attn_spatial_bwd")
            # [H][parts][2][DP]: the unpack sums the slots (one block per head, 4 waves in order)
            grads[f"kvb{i}"] = bpart
            grads[f"wqkv{i}"], grads[f"bqkv{i}"] = wg(dqkv, xn, True)
            return dx_gemm(dqkv, P[f"wqkv_t{i}"], 3 * C, C)

        dh1 = e(N, C, dtp=torch.float32)
        dy_s = r(C)
        if ctx.tail:
            # no temporal sublayer (h2 = h1): the MLP's LN backward hands straight to the spatial
            # gated residual.  Its partials serve both the spatial and the temporal slots of the
            # unpack: d gate_l (2C), d shift_m / d scale_m (6C, 7C) and the spatial out_proj bias
            # land where they belong; the temporal slots (3C..5C, the stand-in bias) get copies,
            # and the caller drops them (zero adaLN columns, None parameter gradients)
            part_t = part_s = lngate(dxn3, sv["h1"], sv["stats"][2], 6 * C, 7 * C, dh3, dh1, sv["y"][0], 2 * C, dy_s)
        else:
            dh2 = e(N, C, dtp=torch.float32)
            dy_t = r(C)
            part_t = lngate(dxn3, sv["h2"], sv["stats"][2], 6 * C, 7 * C, dh3, dh2, sv["y"][1], 5 * C, dy_t)
            dxn2 = attention(1, dy_t, sv["o"][1], sv["o_lo"][1], sv["xn"][1], sv["qkv_t"], sv["lse_t"])
            part_s = lngate(dxn2, sv["h1"], sv["stats"][1], 3 * C, 4 * C, dh2, dh1, sv["y"][0], 2 * C, dy_s)
        dxn1 = attention(0, dy_s, sv["o"][0], sv["o_lo"][0], sv["xn"][0], sv["qkv_s"], sv["lse_s"])
        if ctx.tail:  # the unpack's temporal inputs: attention 0's again (outputs dropped)
            for k in ("wqkv", "bqkv", "kvb", "wo"):
                grads[f"{k}1"] = grads[f"{k}0"]
        dh0 = e(N, C, dtp=torch.float32)
        part_0 = lngate(dxn1, h.reshape(N, C), sv["stats"][0], 0, C, dh1, dh0, None, 0, None)

        # packed -> parameter layout, the bias-key rotation undone, adaLN / bias gradients from the
        # per-block partials: one launch (mdg_train_unpack_layer)
        f32 = lambda *shape: torch.empty(*shape, device=dev)  # noqa: E731
        up = _lib.MdgTrainUnpack(C=C, H=H, D=D, B=B, nblk=nblk, rope=int(hl.rope))
        g = {}
        for i in range(2):
            up.gwqkv[i], up.gbqkv[i] = grads[f"wqkv{i}"].data_ptr(), grads[f"bqkv{i}"].data_ptr()
            up.bpart[i], up.parts[i] = grads[f"kvb{i}"].data_ptr(), grads[f"kvb{i}"].shape[1]
            S, rows = (L, L + 1) if i == 0 else (T, T + 1)
            up.rope_tab[i], up.rope_rows[i], up.rope_pos[i] = _lib.ptr(ctx.rope[i]), rows, S
            for name, shape in (("gq", (C, C)), ("gk", (C, C)), ("gv", (C, C)), ("gbq", (C,)), ("gbk", (C,)),
                                ("gbv", (C,)), ("gbias_k", (1, 1, C)), ("gbias_v", (1, 1, C))):
                g[name, i] = f32(*shape)
                getattr(up, name)[i] = g[name, i].data_ptr()
        for k, part in enumerate((part_0, part_s, part_t, part_m)):
            up.part[k] = part.data_ptr()
        dmods, gbo0, gbo1, gb2 = f32(B, 9 * C), f32(C), f32(C), f32(C)
        up.dmods, up.gbo[0], up.gbo[1], up.gb2 = dmods.data_ptr(), gbo0.data_ptr(), gbo1.data_ptr(), gb2.data_ptr()
        _lib.check(lib.mdg_train_unpack_layer(ctypes.byref(up), s), "mdg_train_unpack_layer")
        grads["bo0"], grads["bo1"], grads["b2"] = gbo0, gbo1, gb2
        out = []
        for i in range(2):
            out += [g["gq", i], g["gbq", i], g["gk", i], g["gbk", i], g["gv", i], g["gbv", i], grads[f"wo{i}"],
                    grads[f"bo{i}"], g["gbias_k", i], g["gbias_v", i]]
        out += [grads["w1"], grads["b1"], grads["w2"], grads["b2"]]
        if ctx.tail:  # the zero-gate temporal stand-ins: exactly zero, nothing to accumulate
            out[10:20] = [None] * 10
        del ctx.sv, ctx.P, ctx.lease  # the planes go back to the layer's pool
        return (dh0.reshape(B, T, L, C), dmods, None, None, None, None, None, *out)


# ------------------------------------------------------------------------------------------
# The step's glue around the block stack on library kernels (csrc/train_glue.hip): the token
# embedding (latent_model.py:242-255, forward by mdg_embed, backward by mdg_embed_bwd) and the
# FinalLayer (layers.py:58-75, mdg_final_fwd_train / mdg_final_bwd_train), fp32 like the
# reference's parameters.  Each replaces ~20 eager kernels over the [N][C] fp32 residual.

def glue_supported(model, L):
    """The glue kernels' shapes: C = 384 (the FinalLayer kernels' row layout), L <= 8, latent 21 / 28;
    MDG_TRAIN_GLUE=0 keeps the eager embedding / FinalLayer (A/B)."""
    if os.environ.get("MDG_TRAIN_GLUE", "1") == "0":
        return False
    return model.args.embed_dim == 384 and L <= 8 and model.latent_dim in (21, 28)


class _HipEmbedFn(torch.autograd.Function):
    """h = latent_to_emb(x) + pos_embed + cond_to_emb(x_cond) + mask_to_emb[x_cond_mask]
    + ipa[b, l] (the IPA prepend broadcast over frames).  x / x_cond / the mask carry no
    gradient (the noised latents and the conditioning); ipa, both linears and the mask table do."""

    @staticmethod
    def forward(ctx, x, xc, idx, ipa, w1, b1, w2, b2, memb, pos, hl):
        lib, s = hl.lib, _lib.stream_handle()
        B, T, L, K1 = x.shape
        C, N = w1.shape[0], B * T * L
        x = x.detach().float().contiguous()
        dev = x.device
        out = torch.empty(N, C, device=dev)
        ipa_c = ipa.detach().float().contiguous() if ipa is not None else None
        pos_c = pos.detach().float().contiguous() if pos is not None else None
        w1t = w1.detach().t().contiguous()
        if xc is not None:
            xc = xc.detach().float().contiguous()
            idx = idx.to(torch.int64).contiguous()
            base = torch.empty(N, C, device=dev)
            bsum = (b1.detach() + b2.detach()).contiguous()
            _lib.check(lib.mdg_embed(N, T, L, C, xc.shape[-1], xc.data_ptr(), w2.detach().t().contiguous().data_ptr(),
                                     bsum.data_ptr(), None, _lib.ptr(pos_c), memb.detach().contiguous().data_ptr(),
                                     idx.data_ptr(), None, base.data_ptr(), s), "mdg_embed(cond)")
            _lib.check(lib.mdg_embed(N, T, L, C, K1, x.data_ptr(), w1t.data_ptr(), None, base.data_ptr(), None, None,
                                     None, _lib.ptr(ipa_c), out.data_ptr(), s), "mdg_embed(latent)")
        else:
            _lib.check(lib.mdg_embed(N, T, L, C, K1, x.data_ptr(), w1t.data_ptr(), b1.detach().contiguous().data_ptr(),
                                     None, _lib.ptr(pos_c), None, None, _lib.ptr(ipa_c), out.data_ptr(), s),
                       "mdg_embed(latent)")
        ctx.save_for_backward(x, xc, idx)
        ctx.hl, ctx.shape, ctx.E = hl, (B, T, L, C), memb.shape[0]
        ctx.has_ipa, ctx.has_cond = ipa is not None, xc is not None
        return out.view(B, T, L, C)

    @staticmethod
    def backward(ctx, dh):
        x, xc, idx = ctx.saved_tensors
        hl = ctx.hl
        lib = hl.lib
        B, T, L, C = ctx.shape
        dev = dh.device
        dh = dh.float().contiguous()
        K1 = x.shape[-1]
        K2 = xc.shape[-1] if xc is not None else 0
        E = ctx.E if ctx.has_cond else 0
        dw1 = torch.empty(C, K1, device=dev)
        db = torch.empty(C, device=dev)
        dw2 = torch.empty(C, K2, device=dev) if ctx.has_cond else None
        demb = torch.empty(E, C, device=dev) if ctx.has_cond else None
        dipa = torch.empty(B, L, C, device=dev) if ctx.has_ipa else None
        wsb = lib.mdg_embed_bwd_workspace_bytes(B, T, L, C, K1, K2, E)
        ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
        _lib.check(lib.mdg_embed_bwd(B, T, L, C, K1, x.data_ptr(), K2, _lib.ptr(xc), _lib.ptr(idx), E, dh.data_ptr(),
                                     dw1.data_ptr(), _lib.ptr(dw2), db.data_ptr(), _lib.ptr(demb), _lib.ptr(dipa),
                                     ws.data_ptr(), wsb, _lib.stream_handle()), "mdg_embed_bwd")
        return (None, None, None, dipa, dw1, db, dw2, db if ctx.has_cond else None, demb, None, None)


def hip_embed(hl, model, x, x_cond, x_cond_mask, ipa):
    """The model's token embedding + IPA prepend on the glue kernels (latent_model.py:242-255);
    x [B,T,L,lat], ipa [B,L,C] or None."""
    m = model
    pos = m.pos_embed[0] if m.args.abs_pos_emb else None
    if x_cond is not None:
        h = _HipEmbedFn.apply(x, x_cond, x_cond_mask, ipa, m.latent_to_emb.weight, m.latent_to_emb.bias,
                              m.cond_to_emb.weight, m.cond_to_emb.bias, m.mask_to_emb.weight, pos, hl)
    else:
        h = _HipEmbedFn.apply(x, None, None, ipa, m.latent_to_emb.weight, m.latent_to_emb.bias, None, None,
                              m.mask_to_emb.weight, pos, hl)
    if getattr(m.args, "abs_time_emb", False):
        h = h + m.time_embed[:, :, None]
    return h


class _HipFinalFn(torch.autograd.Function):
    """FinalLayer: LN(h) * (1 + scale) + shift -> Linear(C, latent), mods [B, 2C] = shift | scale."""

    @staticmethod
    def forward(ctx, h, mods, w, b, hl):
        lib = hl.lib
        B, T, L, C = h.shape
        N, lat = B * T * L, w.shape[0]
        h = h.detach().float().contiguous()
        mods = mods.detach().float().contiguous()
        w = w.detach().float().contiguous()
        v = torch.empty(N, lat, device=h.device)
        stats = torch.empty(N, 2, device=h.device)
        _lib.check(lib.mdg_final_fwd_train(N, T * L, C, lat, h.data_ptr(), mods.data_ptr(), w.data_ptr(),
                                           b.detach().contiguous().data_ptr(), v.data_ptr(), stats.data_ptr(),
                                           _lib.stream_handle()), "mdg_final_fwd_train")
        ctx.save_for_backward(h, stats, mods, w)
        ctx.hl = hl
        return v.view(B, T, L, lat)

    @staticmethod
    def backward(ctx, dv):
        h, stats, mods, w = ctx.saved_tensors
        lib = ctx.hl.lib
        B, T, L, C = h.shape
        N, lat = B * T * L, w.shape[0]
        dev = h.device
        dv = dv.float().contiguous()
        dh = torch.empty_like(h)
        dw = torch.empty(lat, C, device=dev)
        db = torch.empty(lat, device=dev)
        dmods = torch.empty(B, 2 * C, device=dev)
        wsb = lib.mdg_final_bwd_workspace_bytes(N, T * L, lat)
        ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
        _lib.check(lib.mdg_final_bwd_train(N, T * L, C, lat, h.data_ptr(), stats.data_ptr(), mods.data_ptr(),
                                           w.data_ptr(), dv.data_ptr(), dh.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                           dmods.data_ptr(), ws.data_ptr(), wsb, _lib.stream_handle()),
                   "mdg_final_bwd_train")
        return dh, dmods, dw, db, None


def hip_final(hl, final_layer, h, mods):
    """FinalLayer (layers.py:58-75) on the glue kernels; mods [B, 2C] (the stacked adaLN rows)."""
    return _HipFinalFn.apply(h, mods, final_layer.linear.weight, final_layer.linear.bias, hl)


# ------------------------------------------------------------------------------------------
# Few-row linears of the conditioning (t-MLP, every adaLN linear, the IPA projections and
# linear_out) on mdg_seg_linear_fwd / _bwd (csrc/linear_small.hip): nseg nn.Linear layers that
# share one input, one launch forward and two backward, no weight concatenation or output split.

_ACT = {"none": _lib.MDG_ACT_NONE, "silu": _lib.MDG_ACT_SILU}


class _SegLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act, nseg, resid, *wb):
        lib = _lib.load()
        K = x.shape[-1]
        lead = x.shape[:-1]
        x2 = x.detach().reshape(-1, K).float().contiguous()
        M = x2.shape[0]
        ws, bs = wb[:nseg], wb[nseg:]
        sl = _lib.MdgSegLinear(nseg=nseg)
        outs = []
        for i, (w, b) in enumerate(zip(ws, bs)):
            n = w.shape[0]
            y = torch.empty(M, n, device=x.device)
            sl.n[i], sl.w[i], sl.b[i], sl.y[i], sl.ldy[i] = n, _src(w.detach()), _lib.ptr(b), y.data_ptr(), n
            outs.append(y)
        if resid is not None:
            r = resid.detach().reshape(M, -1).float().contiguous()
            sl.resid[0], sl.ldr[0] = r.data_ptr(), r.shape[1]
        _lib.check(lib.mdg_seg_linear_fwd(M, K, x2.data_ptr(), K, _ACT[act], ctypes.byref(sl), _lib.stream_handle()),
                   "mdg_seg_linear_fwd")
        ctx.save_for_backward(x2, *ws)
        ctx.act, ctx.nseg, ctx.lead, ctx.has_bias = act, nseg, lead, [b is not None for b in bs]
        ctx.has_resid = resid is not None
        return tuple(y.view(*lead, y.shape[1]) for y in outs)

    @staticmethod
    def backward(ctx, *dys):
        lib = _lib.load()
        x2, *ws = ctx.saved_tensors
        M, K = x2.shape
        nseg = ctx.nseg
        sl = _lib.MdgSegLinear(nseg=nseg)
        keep, dws, dbs = [], [], []
        for i, (w, dy) in enumerate(zip(ws, dys)):
            n = w.shape[0]
            dy2 = dy.reshape(M, n).float().contiguous()
            keep.append(dy2)
            dw = torch.empty(n, K, device=x2.device) if ctx.needs_input_grad[4 + i] else None
            db = torch.empty(n, device=x2.device) if ctx.has_bias[i] and ctx.needs_input_grad[4 + nseg + i] else None
            sl.n[i], sl.w[i], sl.dy[i], sl.lddy[i] = n, w.data_ptr(), dy2.data_ptr(), n
            sl.dw[i], sl.db[i] = _lib.ptr(dw), _lib.ptr(db)
            dws.append(dw)
            dbs.append(db)
        dx = torch.empty(M, K, device=x2.device) if ctx.needs_input_grad[0] else None
        wsb = lib.mdg_seg_linear_bwd_workspace_bytes(M, K, ctypes.byref(sl)) if dx is not None else 0
        wsp = torch.empty(max(wsb, 1), device=x2.device, dtype=torch.uint8)
        _lib.check(lib.mdg_seg_linear_bwd(M, K, x2.data_ptr(), K, _ACT[ctx.act], ctypes.byref(sl), _lib.ptr(dx), K,
                                          wsp.data_ptr(), wsb, _lib.stream_handle()), "mdg_seg_linear_bwd")
        dresid = dys[0] if ctx.has_resid else None
        dxo = dx.view(*ctx.lead, K) if dx is not None else None
        return (dxo, None, None, dresid, *dws, *dbs)


def seg_linear(x, linears, act="none", resid=None):
    """[lin(act(x)) for lin in linears] (+ resid on the single output) through the segmented
    library linear; x fp32 [..., K], every lin an nn.Linear(K, n_i)."""
    if resid is not None and len(linears) != 1:
        raise ValueError("seg_linear: resid needs exactly one segment")
    ws = [l.weight for l in linears]
    bs = [l.bias for l in linears]
    return _SegLinearFn.apply(x, act, len(linears), resid, *ws, *bs)


def seg_supported(x):
    """The segmented linears serve differentiable CUDA fp32 calls with K % 4 == 0 and K <= 1024
    (MDG_TRAIN_SEG=0: eager, A/B)."""
    K = x.shape[-1]
    return (x.is_cuda and torch.is_grad_enabled() and K % 4 == 0 and K <= 1024
            and os.environ.get("MDG_TRAIN_SEG", "1") != "0")


# ------------------------------------------------------------------------------------------
# The flow-matching plan and loss (transport.py:137-222) as library launches
# (csrc/train_glue.hip, mdg_gvp_plan / mdg_gvp_loss_fwd / _bwd).

def gvp_plan(t, x0, x1, path):
    """(xt, ut) of the GVP (path 0) or Linear (1) plan; t [B], x0 / x1 [B, ...] fp32."""
    lib = _lib.load()
    x0c, x1c, tc = x0.contiguous(), x1.contiguous(), t.float().contiguous()
    xt, ut = torch.empty_like(x1c), torch.empty_like(x1c)
    B = x1c.shape[0]
    _lib.check(lib.mdg_gvp_plan(B, x1c.numel() // B, path, tc.data_ptr(), x0c.data_ptr(), x1c.data_ptr(),
                                xt.data_ptr(), ut.data_ptr(), _lib.stream_handle()), "mdg_gvp_plan")
    return xt, ut


class _GvpLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, ut, mask):
        lib = _lib.load()
        B, T, L, K = out.shape
        # the kernels read fp32: a half-precision prediction (the eager FinalLayer under bf16 /
        # fp16 autocast) is promoted here, as the reference's (out - ut) with an fp32 ut promotes
        ctx.out_dtype = out.dtype
        o, u = out.detach().float().contiguous(), ut.detach().float().contiguous()
        m = mask.detach().float().expand(B, T, L, K)
        ms = (ctypes.c_int64 * 4)(*m.stride())
        loss = torch.empty(B, device=out.device)
        den = torch.empty(B, device=out.device)
        wsb = lib.mdg_gvp_loss_workspace_bytes(B, T * L * K)
        ws = torch.empty(wsb, device=out.device, dtype=torch.uint8)
        _lib.check(lib.mdg_gvp_loss_fwd(B, T, L, K, o.data_ptr(), u.data_ptr(), m.data_ptr(), ms, loss.data_ptr(),
                                        den.data_ptr(), ws.data_ptr(), wsb, _lib.stream_handle()), "mdg_gvp_loss_fwd")
        ctx.save_for_backward(o, u, m, den)
        return loss

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        o, u, m, den = ctx.saved_tensors
        B, T, L, K = o.shape
        ms = (ctypes.c_int64 * 4)(*m.stride())
        gc = g.float().contiguous()
        dout = torch.empty_like(o)
        _lib.check(lib.mdg_gvp_loss_bwd(B, T, L, K, o.data_ptr(), u.data_ptr(), m.data_ptr(), ms, gc.data_ptr(),
                                        den.data_ptr(), dout.data_ptr(), _lib.stream_handle()), "mdg_gvp_loss_bwd")
        return dout.to(ctx.out_dtype), None, None


def gvp_loss(out, ut, mask):
    """mean_flat((out - ut) ** 2, mask) per trajectory [B] with its backward on the library."""
    return _GvpLossFn.apply(out, ut, mask)
