"""HIP execution engine for LatentMDGenModel (the MI355X hot path).

Responsibilities
  * pack the module's parameters once (re-packed when any parameter changes) into the
    operand layout of libmdgen_hip.so: fused [3C][C] QKV weights per attention, CT (bf16 or
    f32) GEMM operands, fp32 biases, RoPE tables and the RoPE-rotated bias_k / bias_v rows;
  * per (B, T, L): workspace (attention operand buffers, hidden activations), residual
    stream, and the mdg_model struct of device pointers;
  * conditioning precompute, x-independent and therefore done for ALL Euler steps of a
    window at once: t-embedding, every adaLN modulation, IPA prepend, the
    step-invariant token embedding (cond_to_emb + mask_to_emb + pos_embed + biases);
  * the Euler loop: ``sample_euler`` runs num_steps-1 ``mdg_denoise_step`` calls
    (Sampler.sample_ode('euler'), transport.py:407-450 + integrators.py:95-114), optionally
    captured with the conditioning precompute into ONE hipGraph and replayed.

The conditioning precompute runs in libmdgen_hip.so too (mdg_precompute_cond: t-embedding
MLP, one stacked adaLN GEMM, the IPA layers on S*B*L residue tokens with the TPS relative
frames computed on the device; fp32 throughout, < 1 % of a window's time), so a window's
hipGraph holds no PyTorch kernels besides input staging.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
import torch.nn.functional as F

from . import _lib
from .rigid_utils import frames_to_tensors

_DTYPES = {"bf16": (_lib.MDG_BF16, torch.bfloat16), "f32": (_lib.MDG_F32, torch.float32)}


def get_engine(model):
    dt = getattr(model, "hip_dtype", "bf16")
    eng = model._engine
    if eng is None or eng.dtype_name != dt:
        eng = HipEngine(model, dt)
        model._engine = eng
    return eng


class _ShapeState:
    pass


class HipEngine:
    def __init__(self, model, dtype="bf16"):
        if dtype not in _DTYPES:
            raise ValueError(f"hip_dtype must be one of {list(_DTYPES)}")
        self.model = model
        self.lib = _lib.load()
        self.dtype_name = dtype
        self.mdg_dtype, self.ct = _DTYPES[dtype]
        a = model.args
        self.C, self.H = a.embed_dim, a.mha_heads
        self.D = self.C // self.H
        self.F = 4 * self.C
        self.nl = a.num_layers
        self.lat = model.latent_dim
        self.rope = not a.no_rope
        self._pack_key = None
        self._packed = None
        self._states = {}
        self._graphs = {}
        self._lane_streams = []
        self._rel7 = None  # TPS relative 7-vectors staged by _prepare_tps (None: computed on the device)
        # concurrent sub-batch chains per Euler window (MDG_LANES, default 1 = one chain)
        # concurrent sub-batch chains per window; 0 = auto: 2 lanes once a window has >= 8
        # trajectories (even count) — measured best at B = 16, bit-identical to 1
        self.lanes = int(os.environ.get("MDG_LANES", "0"))
        # a single chain (no concurrent lane) may use the small-M split-K out_proj route
        self.split_alone = os.environ.get("MDG_SPLIT_ALONE", "1") != "0"
        # layers of lane k-1's first step that run before lane k starts (0 = lanes in lock-step)
        self.lane_offset = int(os.environ.get("MDG_LANE_OFFSET", "0"))

    # ------------------------------------------------------------------ packing
    def _param_key(self):
        # _weights_gen: bumped by updates that bypass autograd's version counters (the graphed
        # training step's Adam runs inside a hipGraph replay: train.GraphedStep.run)
        return (getattr(self.model, "_weights_gen", 0),) + tuple(
            (p.data_ptr(), p._version) for p in self.model.parameters())

    def _pack(self):
        key = self._param_key()
        if key == self._pack_key:
            return self._packed
        m, ct = self.model, self.ct
        dev = m.device
        if dev.type != "cuda":
            raise RuntimeError("the HIP backend needs the model on a ROCm device (model.cuda())")
        with torch.no_grad():
            P = {"layers": []}
            perm = self._pair_perm() if self.rope else None
            for layer in m.layers:
                d = {}
                for i, mha in enumerate((layer.mha_l.attn, layer.mha_t.attn)):
                    wq, wk = mha.q_proj.weight, mha.k_proj.weight
                    bq, bk = mha.q_proj.bias, mha.k_proj.bias
                    if perm is not None:  # pair-interleave q/k head rows (RoPE partner in lane^1)
                        wq, wk, bq, bk = wq[perm], wk[perm], bq[perm], bk[perm]
                    d[f"wqkv{i}"] = torch.cat([wq, wk, mha.v_proj.weight]).to(ct).contiguous()
                    d[f"bqkv{i}"] = torch.cat([bq, bk, mha.v_proj.bias]).float().contiguous()
                    d[f"wo{i}"] = mha.out_proj.weight.to(ct).contiguous()
                    d[f"bo{i}"] = mha.out_proj.bias.float().contiguous()
                    d[f"bias_k{i}"] = mha.bias_k.detach().float().reshape(-1)
                    d[f"bias_v{i}"] = mha.bias_v.detach().float().reshape(-1)
                d["w1"] = layer.fc1.weight.to(ct).contiguous()
                d["b1"] = layer.fc1.bias.float().contiguous()
                d["w2"] = layer.fc2.weight.to(ct).contiguous()
                d["b2"] = layer.fc2.bias.float().contiguous()
                P["layers"].append(d)
            P["w_l2e_t"] = m.latent_to_emb.weight.float().t().contiguous()      # [latent][C]
            P["b_l2e"] = m.latent_to_emb.bias.float().contiguous()
            P["w_c2e_t"] = m.cond_to_emb.weight.float().t().contiguous()
            P["b_base"] = (m.cond_to_emb.bias + m.latent_to_emb.bias).float().contiguous()
            lp = (self.lat + 31) // 32 * 32                                       # padded to the GEMM tile
            wf = torch.zeros(lp, self.C, device=dev)
            wf[: self.lat] = m.emb_to_latent.linear.weight.float()
            bf = torch.zeros(lp, device=dev)
            bf[: self.lat] = m.emb_to_latent.linear.bias.float()
            P["w_final"] = wf.to(ct).contiguous()
            P["b_final"] = bf
            P["inv_freq"] = m.layers[0].mha_l.attn.rot_emb.inv_freq if self.rope else None
            P["cond"] = self._pack_cond(perm)
        self._packed, self._pack_key = P, key
        self._states.clear()
        self._graphs.clear()
        return P

    def _pack_cond(self, perm):
        """fp32 operands of mdg_precompute_cond (mdg_cond_model): the t-embedder MLP, every
        adaLN Linear stacked [layers 9C | final 2C | IPA layers 6C][C], and per IPA layer the
        fused q | kv | q_points | kv_points projection (rows padded to 32), linear_out (columns
        padded to 64), the mha_l q|k|v in the pair-interleaved RoPE order, out_proj, fc1, fc2."""
        m = self.model
        f = lambda t: t.detach().float().contiguous()  # noqa: E731
        te = m.t_embedder
        cp = {"t_freqs": f(te.freqs), "t_w0": f(te.mlp[0].weight), "t_b0": f(te.mlp[0].bias),
              "t_w2": f(te.mlp[2].weight), "t_b2": f(te.mlp[2].bias)}
        ada = [l.adaLN_modulation[1] for l in m.layers] + [m.emb_to_latent.adaLN_modulation[1]]
        ipa_layers = list(m.ipa_layers) if m.args.prepend_ipa else []
        ada += [l.adaLN_modulation[1] for l in ipa_layers]
        cp["ada_w"] = f(torch.cat([a.weight for a in ada]))
        cp["ada_b"] = f(torch.cat([a.bias for a in ada]))
        cp["aa_emb"] = f(m.aatype_to_emb.weight) if hasattr(m, "aatype_to_emb") else None
        if m.tps:
            cp["l2e_f_w"], cp["l2e_f_b"] = f(m.latent_to_emb_f.weight), f(m.latent_to_emb_f.bias)
            cp["l2e_r_w"], cp["l2e_r_b"] = f(m.latent_to_emb_r.weight), f(m.latent_to_emb_r.bias)
        cp["ipa"] = []
        for layer in ipa_layers:
            ipa = layer.ipa
            w = torch.cat([ipa.linear_q.weight, ipa.linear_kv.weight, ipa.linear_q_points.weight,
                           ipa.linear_kv_points.weight])
            b = torch.cat([ipa.linear_q.bias, ipa.linear_kv.bias, ipa.linear_q_points.bias, ipa.linear_kv_points.bias])
            pp = (w.shape[0] + 31) // 32 * 32
            wp = torch.zeros(pp, self.C, device=w.device)
            wp[: w.shape[0]] = w
            bp = torch.zeros(pp, device=w.device)
            bp[: b.shape[0]] = b
            ko = ipa.linear_out.weight.shape[1]
            wo = torch.zeros(self.C, (ko + 63) // 64 * 64, device=w.device)
            wo[:, :ko] = ipa.linear_out.weight
            mha = layer.mha_l.attn
            wq, wk, bq, bk = mha.q_proj.weight, mha.k_proj.weight, mha.q_proj.bias, mha.k_proj.bias
            if perm is not None:
                wq, wk, bq, bk = wq[perm], wk[perm], bq[perm], bk[perm]
            cp["ipa"].append({
                "ln_w": f(layer.ipa_norm.weight), "ln_b": f(layer.ipa_norm.bias), "w_proj": f(wp), "b_proj": f(bp),
                "head_weights": f(ipa.head_weights), "w_out": f(wo), "b_out": f(ipa.linear_out.bias),
                "wqkv": f(torch.cat([wq, wk, mha.v_proj.weight])), "bqkv": f(torch.cat([bq, bk, mha.v_proj.bias])),
                "bias_k": f(mha.bias_k.reshape(-1)), "bias_v": f(mha.bias_v.reshape(-1)),
                "wo": f(mha.out_proj.weight), "bo": f(mha.out_proj.bias), "w1": f(layer.fc1.weight),
                "b1": f(layer.fc1.bias), "w2": f(layer.fc2.weight), "b2": f(layer.fc2.bias)})
        return cp

    def _cond_state(self, S, B, L):
        """Workspace, rope / bias-kv rows and the mdg_cond_model struct for (S, B, L)."""
        P = self._pack()
        key = ("cond", S, B, L)
        cs = self._states.get(key)
        if cs is not None:
            return cs
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"conditioning state for S={S} B={B} L={L} first requested inside a graph capture "
                               "(its tables are built on the host): create it before capturing")
        m, dev, cp = self.model, self.model.device, P["cond"]
        a = m.args
        cs = _ShapeState()
        has_ipa = bool(a.prepend_ipa)
        dims = _lib.MdgCondDims(S=S, B=B, L=L, C=self.C, H=self.H, D=self.D, num_layers=self.nl,
                                ipa_layers=len(cp["ipa"]), ipa_heads=a.ipa_heads if has_ipa else 0,
                                ipa_c=a.ipa_head_dim if has_ipa else 0, ipa_qk=a.ipa_qk if has_ipa else 0,
                                ipa_v=a.ipa_v if has_ipa else 0, tps=1 if m.tps else 0,
                                freq_dim=m.t_embedder.frequency_embedding_size)
        nbytes = self.lib.mdg_cond_workspace_bytes(ctypes.byref(dims))
        if nbytes == 0:
            _lib.check(1001, f"conditioning workspace for S={S} B={B} L={L}")
        cs.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        cs.rope_l = self._rope_table(L + 1) if self.rope else None
        cm = _lib.MdgCondModel()
        cm.dims = dims
        cm.time_multiplier = float(a.time_multiplier)
        for k in ("t_freqs", "t_w0", "t_b0", "t_w2", "t_b2", "ada_w", "ada_b", "aa_emb", "l2e_f_w", "l2e_f_b",
                  "l2e_r_w", "l2e_r_b"):
            setattr(cm, k, _lib.ptr(cp.get(k)))
        cm.rope_l = _lib.ptr(cs.rope_l)
        cs.kvb = []
        for i, d in enumerate(cp["ipa"]):
            kvb = self._kvb(d["bias_k"], d["bias_v"], L, cs.rope_l, L + 1)
            cs.kvb.append(kvb)
            lw = cm.ipa[i]
            for k in ("ln_w", "ln_b", "w_proj", "b_proj", "head_weights", "w_out", "b_out", "wqkv", "bqkv", "wo", "bo",
                      "w1", "b1", "w2", "b2"):
                setattr(lw, k, d[k].data_ptr())
            lw.kvb = kvb.data_ptr()
        cs.model_struct = cm
        cs.S, cs.B, cs.L = S, B, L
        self._states[key] = cs
        return cs

    def _pair_perm(self):
        """Row permutation of a [C] q/k projection: within each head, new row 2i = dim i and
        2i+1 = dim i + D/2 (the fair-esm rotate-half partner), see gemm.hip QKV epilogue."""
        D, half = self.D, self.D // 2
        idx = torch.arange(D)
        within = torch.where(idx % 2 == 0, idx // 2, idx // 2 + half)
        return (torch.arange(self.H)[:, None] * D + within[None]).reshape(-1).to(self.model.device)

    def _rope_table(self, n_rows):
        """cos | sin tables [n_rows][D/2] exactly as fair-esm builds them (fp32 outer product of
        positions and inv_freq, then cos/sin; computed on the CPU like the reference)."""
        inv = self._packed["inv_freq"].detach().float().cpu()
        pos = torch.arange(n_rows).type_as(inv)
        freqs = torch.einsum("i,j->ij", pos, inv)
        return torch.cat([freqs.cos().reshape(-1), freqs.sin().reshape(-1)]).to(self.model.device)

    def _kvb(self, bias_k, bias_v, S, table, n_rows):
        """[H][2][dp]: bias_k rotated at position S (the appended row's index), bias_v with 1.0
        in pad column D (the temporal kernel's softmax row sum); dp = 32 (D <= 31) or 64."""
        H, D, half = self.H, self.D, self.D // 2
        kb = bias_k.reshape(H, D)
        if table is not None:
            cos = table[: n_rows * half].reshape(n_rows, half)[S]
            sin = table[n_rows * half:].reshape(n_rows, half)[S]
            c2, s2 = torch.cat([cos, cos]), torch.cat([sin, sin])
            rot = torch.cat([-kb[:, half:], kb[:, :half]], -1)
            kb = kb * c2 + rot * s2
        if table is not None:  # same pair-interleaved order as the packed k rows
            kb = kb.reshape(-1)[self._pair_perm()].reshape(H, D)
        out = torch.zeros(H, 2, _lib.head_stride(D), device=bias_k.device, dtype=torch.float32)
        out[:, 0, :D] = kb
        out[:, 1, :D] = bias_v.reshape(H, D)
        out[:, 1, D] = 1.0
        return out.contiguous()

    def _state(self, B, T, L, lane=0):
        P = self._pack()
        key = (B, T, L, lane)
        st = self._states.get(key)
        if st is not None:
            return st
        lib, dev = self.lib, self.model.device
        st = _ShapeState()
        st.B, st.T, st.L, st.N = B, T, L, B * T * L
        st.dims = _lib.MdgDims(B=B, T=T, L=L, C=self.C, H=self.H, D=self.D, F=self.F, latent=self.lat,
                               num_layers=self.nl, dtype=self.mdg_dtype)
        nbytes = lib.mdg_workspace_bytes(ctypes.byref(st.dims))
        if nbytes == 0:
            _lib.check(1001, f"workspace for B={B} T={T} L={L}")
        st.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        _lib.check(lib.mdg_workspace_init(ctypes.byref(st.dims), st.ws.data_ptr(), _lib.stream_handle()),
                   "mdg_workspace_init")
        if os.environ.get("MDG_POISON_WS") == "1":
            # debugging: NaN bytes (0xFF) in every region the step must write before reading it,
            # applied AFTER mdg_workspace_init (which zeroes the workspace and sets the padded
            # planes' 1.0 columns): q|k|v (spatial), o, hidden, xn, key-padding biases, the split
            # partials, and the temporal planes when they are packed (no init-time pad column)
            off = _lib.workspace_offsets(st.dims)
            st.ws[off["qkv_s"]:off["qkv_t"]].fill_(0xFF)
            st.ws[off["o"]:].fill_(0xFF)
            if self.describe_plan_dims(st.dims).get("planes", "").startswith("packed"):
                st.ws[off["qkv_t"]:off["o"]].fill_(0xFF)
        st.h = torch.empty(st.N, self.C, device=dev)
        st.base = torch.empty(st.N, self.C, device=dev)
        if os.environ.get("MDG_POISON_WS") == "1":
            st.h.fill_(float("nan"))
            st.base.fill_(float("nan"))
        st.rope_l = self._rope_table(L + 1) if self.rope else None
        st.rope_t = self._rope_table(T + 1) if self.rope else None
        st.kvb = []
        mstruct = _lib.MdgModel()
        mstruct.dims = st.dims
        mstruct.w_l2e_t = P["w_l2e_t"].data_ptr()
        mstruct.w_final = P["w_final"].data_ptr()
        mstruct.b_final = P["b_final"].data_ptr()
        mstruct.rope_l = _lib.ptr(st.rope_l)
        mstruct.rope_t = _lib.ptr(st.rope_t)
        for i, d in enumerate(P["layers"]):
            kl = self._kvb(d["bias_k0"], d["bias_v0"], L, st.rope_l, L + 1)
            kt = self._kvb(d["bias_k1"], d["bias_v1"], T, st.rope_t, T + 1)
            st.kvb.append((kl, kt))
            lw = mstruct.layers[i]
            for j in range(2):
                lw.wqkv[j] = d[f"wqkv{j}"].data_ptr()
                lw.bqkv[j] = d[f"bqkv{j}"].data_ptr()
                lw.wo[j] = d[f"wo{j}"].data_ptr()
                lw.bo[j] = d[f"bo{j}"].data_ptr()
            lw.kvb[0], lw.kvb[1] = kl.data_ptr(), kt.data_ptr()
            lw.w1, lw.b1 = d["w1"].data_ptr(), d["b1"].data_ptr()
            lw.w2, lw.b2 = d["w2"].data_ptr(), d["b2"].data_ptr()
        st.model_struct = mstruct
        self._states[key] = st
        return st

    def describe_plan(self, B, T, L):
        """The kernel route mdg_denoise_step takes for (B, T, L) at this dtype (mdg_describe_plan)."""
        return self.describe_plan_dims(self._state(B, T, L).dims)

    def describe_plan_dims(self, dims):
        import json

        buf = ctypes.create_string_buffer(1024)
        _lib.check(self.lib.mdg_describe_plan(ctypes.byref(dims), buf, 1024), "mdg_describe_plan")
        return json.loads(buf.value.decode())

    # ------------------------------------------------------------------ conditioning
    def conditioning(self, t_sb, mask, rots, trans, erots, etrans, aatype, lanes=1):
        """x-independent conditioning for S time points at once (mdg_precompute_cond).
        t_sb [S, B] -> mods [S][nl][B][9C] (lanes > 1: [lanes][S][nl][B/lanes][9C]), mods_final
        [S][B][2C], ipa [S][B][L][C] (or None).  mask is the [B, T, L] token mask: its frame-0
        rows are the IPA frame mask, read in place."""
        m = self.model
        S, B = t_sb.shape
        C, L, T = self.C, mask.shape[-1], mask.shape[-2]
        cs = self._cond_state(S, B, L)
        dev = t_sb.device
        mods = (torch.empty(S, self.nl, B, 9 * C, device=dev) if lanes <= 1 else
                torch.empty(lanes, S, self.nl, B // lanes, 9 * C, device=dev))
        mods_f = torch.empty(S, B, 2 * C, device=dev)
        ipa = torch.empty(S, B, L, C, device=dev) if m.args.prepend_ipa else None
        io = _lib.MdgCondIO()
        tt = t_sb if (t_sb.dtype == torch.float32 and t_sb.is_contiguous()) else t_sb.float().contiguous()
        io.t, io.mask, io.mask_stride = tt.data_ptr(), mask.data_ptr(), T * L
        io.rots, io.trans = _lib.ptr(rots), _lib.ptr(trans)
        io.end_rots, io.end_trans = _lib.ptr(erots), _lib.ptr(etrans)
        io.rel7 = _lib.ptr(self._rel7)
        io.aatype = _lib.ptr(aatype) if hasattr(m, "aatype_to_emb") else None
        io.lanes = lanes
        io.mods, io.mods_final, io.ipa = mods.data_ptr(), mods_f.data_ptr(), _lib.ptr(ipa)
        cs.keep = (tt, mask, rots, trans, erots, etrans, aatype, self._rel7)
        _lib.check(self.lib.mdg_precompute_cond(ctypes.byref(cs.model_struct), ctypes.byref(io), cs.ws.data_ptr(),
                                                _lib.stream_handle()), "mdg_precompute_cond")
        return mods, mods_f, ipa

    def _prepare_tps(self, rots, trans, erots, etrans):
        """TPS relative 7-vectors, staged as a [2][B][L][7] tensor outside any graph.  Default:
        the reference's host arithmetic (relative_tensor7: rot_to_quat by CPU eigh, whose
        eigenvector sign is LAPACK's), the same function the training path and the eager torch
        backend use, so sampling conditions exactly as training did.  ``rel7_override`` (tests:
        the reference's own vectors) replaces it; MDG_TPS_REL7=device computes them inside
        mdg_precompute_cond instead (no host round trip; quaternion sign fixed to w >= 0, a
        documented deviation from the reference's arbitrary sign)."""
        from .model.latent_model import relative_tensor7

        self._rel7 = None
        if not self.model.tps:
            return
        ov = getattr(self, "rel7_override", None)
        if ov is not None:
            self._rel7 = torch.stack([t.to(rots.device, torch.float32) for t in ov]).contiguous()
        elif os.environ.get("MDG_TPS_REL7") != "device":
            self._rel7 = torch.stack([relative_tensor7(rots, trans, erots, etrans),
                                      relative_tensor7(erots, etrans, rots, trans)]).contiguous()

    def _base(self, st, x_cond, x_cond_mask):
        """Step-invariant embedding: cond_to_emb(x_cond) + mask_to_emb + pos_embed + both biases
        (latent_model.py:242-250 without the x-dependent latent_to_emb(x))."""
        m, P, s = self.model, self._packed, _lib.stream_handle()
        pos = m.pos_embed[0].contiguous() if m.args.abs_pos_emb else None
        if x_cond is not None:
            xc = x_cond.float().contiguous()
            idx = x_cond_mask.to(torch.int64).contiguous()
            _lib.check(self.lib.mdg_embed(st.N, st.T, st.L, self.C, self.lat, xc.data_ptr(), P["w_c2e_t"].data_ptr(),
                                          P["b_base"].data_ptr(), None, _lib.ptr(pos),
                                          m.mask_to_emb.weight.data_ptr(), idx.data_ptr(), None,
                                          st.base.data_ptr(), s), "mdg_embed(cond)")
        else:
            b = P["b_l2e"].reshape(1, 1, 1, -1)
            if pos is not None:
                b = b + pos.reshape(1, 1, st.L, -1)
            st.base.copy_(b.expand(st.B, st.T, st.L, self.C).reshape(st.N, self.C))
        if getattr(m.args, "abs_time_emb", False):
            st.base.add_(m.time_embed[0, :st.T].reshape(1, st.T, 1, self.C).expand(st.B, st.T, st.L, self.C)
                         .reshape(st.N, self.C))

    # ------------------------------------------------------------------ inputs
    def _inputs(self, x, mask, start_frames, end_frames, aatype):
        if not x.is_cuda:
            raise RuntimeError("HIP backend: inputs must be ROCm device tensors (no CPU fallback)")
        B, T, L, lat = x.shape
        if lat != self.lat:
            raise ValueError(f"latent dim {lat} != model latent {self.lat}")
        if self.model.args.abs_pos_emb and L != self.model.args.crop:
            raise ValueError(f"abs_pos_emb needs L == crop ({L} vs {self.model.args.crop})")
        mask = mask.to(x.device, torch.float32).contiguous()
        cont = lambda z: None if z is None else z.contiguous()  # noqa: E731  (the C ABI reads [B][L][...] rows)
        rots, trans = map(cont, frames_to_tensors(start_frames, x.device))
        erots, etrans = map(cont, frames_to_tensors(end_frames, x.device)) if self.model.tps else (None, None)
        if self.model.args.prepend_ipa and rots is None:
            raise ValueError("prepend_ipa needs start_frames")
        aa = None if aatype is None else aatype.to(x.device, torch.int64).contiguous()
        return B, T, L, mask, rots, trans, erots, etrans, aa

    def _step_io(self, st, x_in, x_out, v_out, ipa, mods, mods_f, dt, base=None, alone=False):
        """alone: this chain has the device to itself (no concurrent lane), so the library may
        take the small-M split-K out_proj route (mdg_step_io.chain_alone; self.split_alone
        False keeps every chain on the lane-invariant routes)."""
        io = _lib.MdgStepIO()
        io.x_in, io.x_out, io.v_out = x_in, x_out, v_out
        io.base, io.ipa = st.base.data_ptr() if base is None else base, ipa
        io.mods, io.mods_final = mods, mods_f
        io.dt = dt
        io.h = st.h.data_ptr()
        io.chain_alone = int(bool(alone) and self.split_alone)
        return io

    # ------------------------------------------------------------------ one forward
    @torch.no_grad()
    def forward(self, x, t, mask, start_frames, end_frames, x_cond, x_cond_mask, aatype):
        B, T, L, mask, rots, trans, erots, etrans, aa = self._inputs(x, mask, start_frames, end_frames, aatype)
        st = self._state(B, T, L)
        self._prepare_tps(rots, trans, erots, etrans)
        tb = t.to(x.device).float().reshape(1, B) if t.dim() else t.to(x.device).float().expand(1, B)
        mods, mods_f, ipa = self.conditioning(tb, mask, rots, trans, erots, etrans, aa)
        self._base(st, x_cond, x_cond_mask)
        xin = x.float().contiguous()
        v = torch.empty_like(xin)
        s = _lib.stream_handle()
        _lib.check(self.lib.mdg_prepare_mask(ctypes.byref(st.dims), mask.data_ptr(), st.ws.data_ptr(), s),
                   "mdg_prepare_mask")
        io = self._step_io(st, xin.data_ptr(), None, v.data_ptr(), _lib.ptr(ipa), mods.data_ptr(),
                           mods_f.data_ptr(), 0.0, alone=True)
        _lib.check(self.lib.mdg_denoise_step(ctypes.byref(st.model_struct), ctypes.byref(io), mask.data_ptr(),
                                             st.ws.data_ptr(), s), "mdg_denoise_step")
        return v

    # ------------------------------------------------------------------ Euler sampling
    @torch.no_grad()
    def sample_euler(self, zs, num_steps=50, mask=None, start_frames=None, end_frames=None, x_cond=None,
                     x_cond_mask=None, aatype=None, use_graph=True):
        """All num_steps states of the fixed-grid Euler ODE solve from t=0 to t=1
        (the tensor ``Sampler.sample_ode('euler')(zs, model)`` returns)."""
        B, T, L, mask, rots, trans, erots, etrans, aa = self._inputs(zs, mask, start_frames, end_frames, aatype)
        st = self._state(B, T, L)
        self._prepare_tps(rots, trans, erots, etrans)
        key = (B, T, L, num_steps, self._nlanes(B))
        gs = self._graphs.get(key) if use_graph else None
        if gs is None:
            gs = self._build_sampler(st, num_steps, key if use_graph else None)
        # stage inputs into the static buffers the (captured) program reads
        gs.states[0].copy_(zs)
        gs.mask.copy_(mask)
        self._copy_opt(gs, "rots", rots)
        self._copy_opt(gs, "trans", trans)
        self._copy_opt(gs, "erots", erots)
        self._copy_opt(gs, "etrans", etrans)
        self._copy_opt(gs, "aatype", aa)
        self._copy_opt(gs, "rel7", self._rel7)  # TPS relative frames staged on the host path only
        self._rel7 = gs.rel7
        gs.has_cond = x_cond is not None
        if gs.has_cond:
            self._copy_opt(gs, "x_cond", x_cond.float())
            self._copy_opt(gs, "x_cond_mask", x_cond_mask.to(torch.int64))
        if gs.graph is not None and gs.graph_has_cond == gs.has_cond:
            gs.graph.replay()
        else:
            self._run_sampler(gs, st)
            if use_graph and gs.graph is None:
                self._capture(gs, st)
        return gs.states.clone()

    # ------------------------------------------------------------------ adaptive solvers
    _VF_LANE = 64  # workspace keys of the velocity field's own states (base / mask bias hoisted)

    @torch.no_grad()
    def velocity_field(self, x_like, mask=None, start_frames=None, end_frames=None, x_cond=None, x_cond_mask=None,
                       aatype=None, use_graph=True):
        """f(t, y) -> v = model(y, ones(B)·t, **kw) for an adaptive solver (dopri5): t is a
        device scalar, y a [B,T,L,latent] device tensor.

        The Euler window's machinery, per evaluation instead of per window:
          * everything t-independent is computed ONCE here: the base embedding (cond_to_emb +
            mask_to_emb + pos_embed + biases) and the key-padding biases live in the field's own
            workspaces (keys _VF_LANE + k, never touched by the Euler sampler or forward);
          * ``f.precondition(ts)`` runs the t-dependent conditioning (t-embedding, every adaLN
            row, the IPA prepend) for ALL stage times of an adaptive step in one
            mdg_precompute_cond call (S rows of t, like the Euler window's 49), and
            ``f.stage(i, y)`` is evaluation i on those rows — the graphed dopri5 step
            (integrators.odeint_dopri5_graphed) conditions its 5 new stages at once;
          * B >= 8 runs as 2 lanes (parallel graph branches on 2 streams, the Euler window's
            lane split, bit-identical per trajectory to one chain at these shapes).
        f itself (one evaluation: precondition([t]) + stage 0) is one hipGraph replay per call,
        with no host sync inside."""
        B, T, L, mask, rots, trans, erots, etrans, aa = self._inputs(x_like, mask, start_frames, end_frames, aatype)
        self._prepare_tps(rots, trans, erots, etrans)
        dev = self.model.device
        nl = self._nlanes(B)
        st = self._state(B, T, L, lane=self._VF_LANE)
        Bl = B // nl
        lanes = [st] if nl == 1 else [self._state(Bl, T, L, lane=self._VF_LANE + 1 + k) for k in range(nl)]
        if len(self._lane_streams) < nl:
            self._lane_streams += [torch.cuda.Stream() for _ in range(nl - len(self._lane_streams))]
        vs = _ShapeState()
        vs.x = torch.empty(B, T, L, self.lat, device=dev)
        vs.v = torch.empty_like(vs.x)
        vs.t = torch.zeros(1, device=dev)
        vs.mask = mask.clone()
        for name, val in (("rots", rots), ("trans", trans), ("erots", erots), ("etrans", etrans), ("aatype", aa)):
            self._copy_opt(vs, name, val)
        self._copy_opt(vs, "rel7", self._rel7)
        vs.graph = None
        vs.ios = []
        # hoisted, t-independent: base embedding and key-padding biases, in the shape's shared
        # velocity-field workspace.  A later field of the same shape overwrites them, so the
        # workspace records its owner and ensure() re-hoists this field's before it runs again
        # (the older field used to read the newer field's conditioning).
        vs.x_cond = None if x_cond is None else x_cond.float().clone()
        vs.x_cond_mask = None if x_cond_mask is None else x_cond_mask.clone()
        vs.token = object()

        def ensure():
            if getattr(st, "vf_owner", None) is vs.token:
                return
            s = _lib.stream_handle()
            self._base(st, vs.x_cond, vs.x_cond_mask)
            for k, ls in enumerate(lanes):
                mk = vs.mask[k * Bl:(k + 1) * Bl]
                _lib.check(self.lib.mdg_prepare_mask(ctypes.byref(ls.dims), mk.data_ptr(), ls.ws.data_ptr(), s),
                           "mdg_prepare_mask")
            st.vf_owner = vs.token

        ensure()
        rows = Bl * T * L
        # conditioning states for one evaluation and for the 6 stage times of a graphed dopri5
        # step, built here: their RoPE / bias-kv tables are host work that a capture cannot record
        for S_ in (1, 6):
            self._cond_state(S_, B, L)

        def precondition(ts):
            """Conditioning rows for the stage times ts [S] (device fp32; capturable)."""
            S = ts.shape[0]
            t_sb = ts.to(torch.float32).reshape(S, 1).expand(S, B).contiguous()
            self._rel7 = vs.rel7
            vs.cond = self.conditioning(t_sb, vs.mask, vs.rots, vs.trans, getattr(vs, "erots", None),
                                        getattr(vs, "etrans", None), getattr(vs, "aatype", None), nl)

        def stage(i, y):
            """v for stage i of the last precondition() at y (capturable); returns a new tensor."""
            vs.x.copy_(y)
            mods, mods_f, ipa = vs.cond
            main = torch.cuda.current_stream()
            if nl == 1:
                io = self._step_io(st, vs.x.data_ptr(), None, vs.v.data_ptr(),
                                   None if ipa is None else ipa[i].data_ptr(), mods[i].data_ptr(),
                                   mods_f[i].data_ptr(), 0.0, alone=True)
                vs.ios.append(io)
                _lib.check(self.lib.mdg_denoise_step(ctypes.byref(st.model_struct), ctypes.byref(io),
                                                     vs.mask.data_ptr(), st.ws.data_ptr(), _lib.stream_handle()),
                           "mdg_denoise_step")
            else:
                for k, ls in enumerate(lanes):
                    strm = self._lane_streams[k]
                    strm.wait_stream(main)
                    io = self._step_io(ls, vs.x[k * Bl].data_ptr(), None, vs.v[k * Bl].data_ptr(),
                                       None if ipa is None else ipa[i, k * Bl].data_ptr(), mods[k][i].data_ptr(),
                                       mods_f[i, k * Bl].data_ptr(), 0.0, base=st.base.data_ptr() + k * rows * self.C * 4)
                    vs.ios.append(io)
                    _lib.check(self.lib.mdg_denoise_step(ctypes.byref(ls.model_struct), ctypes.byref(io),
                                                         vs.mask[k * Bl].data_ptr(), ls.ws.data_ptr(),
                                                         strm.cuda_stream), "mdg_denoise_step(lane)")
                for k in range(nl):
                    main.wait_stream(self._lane_streams[k])
            del vs.ios[:-nl]  # the launches copied their arguments; keep only the latest structs
            return vs.v.clone()

        def program():
            precondition(vs.t)
            stage(0, vs.x)

        def f(t, y):
            ensure()
            vs.x.copy_(y)
            vs.t.copy_(torch.as_tensor(t, device=dev).float().reshape(1))
            if vs.graph is not None:
                vs.graph.replay()
            else:
                program()
                if use_graph:
                    g = torch.cuda.CUDAGraph()
                    torch.cuda.synchronize()
                    with torch.cuda.graph(g):
                        program()
                    vs.graph = g
            return vs.v.clone()

        def f_capturable(t, y):
            """The same evaluation as device work only (no replay, no host read of t)."""
            vs.x.copy_(y)
            vs.t.copy_(t.to(torch.float32).reshape(1))
            program()
            return vs.v.clone()

        f_capturable.precondition = precondition
        f_capturable.stage = stage
        f_capturable.ensure = ensure  # eager: call before each replay of a graph that captured it
        f.ensure = ensure
        f.state = vs
        f.capturable = f_capturable
        f.lanes = nl
        return f

    def _copy_opt(self, gs, name, val):
        if val is None:
            if getattr(gs, name, None) is not None:
                gs.graph = None  # an input went from present to absent: the captured program read it
            setattr(gs, name, None)
            return
        buf = getattr(gs, name, None)
        if buf is None or buf.shape != val.shape or buf.dtype != val.dtype:
            buf = torch.empty_like(val)
            setattr(gs, name, buf)
            gs.graph = None  # static buffers changed: recapture
        buf.copy_(val)

    def _nlanes(self, B):
        """Concurrent sub-batch chains for a window of B trajectories (part of the graph key)."""
        want = self.lanes if self.lanes > 0 else (2 if B >= 8 else 1)
        return want if (want > 1 and B % want == 0) else 1

    def _build_sampler(self, st, num_steps, key):
        gs = _ShapeState()
        dev = self.model.device
        ts = torch.linspace(0, 1, num_steps)  # CPU fp32, as the reference's ode (integrators.py:85)
        gs.S = num_steps - 1
        gs.t_sb = ts[:-1].reshape(-1, 1).expand(gs.S, st.B).contiguous().to(dev)
        gs.dts = [float(ts[i + 1] - ts[i]) for i in range(gs.S)]
        gs.states = torch.empty(num_steps, st.B, st.T, st.L, self.lat, device=dev)
        gs.mask = torch.empty(st.B, st.T, st.L, device=dev)
        gs.graph = None
        gs.graph_has_cond = None
        if key is not None:
            self._graphs[key] = gs
        return gs

    def _run_sampler(self, gs, st):
        """The whole window: conditioning for all steps, base embedding, mask bias, S steps."""
        s = _lib.stream_handle()
        nlanes = self._nlanes(st.B)
        mods, mods_f, ipa = self.conditioning(gs.t_sb, gs.mask, gs.rots, gs.trans, getattr(gs, "erots", None),
                                              getattr(gs, "etrans", None), getattr(gs, "aatype", None), nlanes)
        gs.cond = (mods, mods_f, ipa)  # keep alive (graph-pool memory during capture)
        self._base(st, gs.x_cond if gs.has_cond else None, gs.x_cond_mask if gs.has_cond else None)
        _lib.check(self.lib.mdg_prepare_mask(ctypes.byref(st.dims), gs.mask.data_ptr(), st.ws.data_ptr(), s),
                   "mdg_prepare_mask")
        if nlanes > 1:
            self._run_lanes(gs, st, mods, mods_f, ipa, nlanes)
            return
        ios = []
        for i in range(gs.S):
            io = self._step_io(st, gs.states[i].data_ptr(), gs.states[i + 1].data_ptr(), None,
                               None if ipa is None else ipa[i].data_ptr(), mods[i].data_ptr(),
                               mods_f[i].data_ptr(), gs.dts[i], alone=True)
            ios.append(io)
            _lib.check(self.lib.mdg_denoise_step(ctypes.byref(st.model_struct), ctypes.byref(io),
                                                 gs.mask.data_ptr(), st.ws.data_ptr(), s), "mdg_denoise_step")
        gs.ios = ios

    def _run_lanes(self, gs, st, mods, mods_f, ipa, nlanes):
        """The window's S denoising steps as ``nlanes`` independent sub-batch chains, each on its
        own HIP stream (fork/join around them; inside a capture they become parallel graph
        branches).  Trajectories never interact inside a step, so the chains only share the
        read-only weights / conditioning; running them concurrently lets one chain's VALU-bound
        attention co-reside with the other's MFMA/HBM-bound GEMMs and fills each kernel's tail."""
        main = torch.cuda.current_stream()
        Bl = st.B // nlanes
        rows = Bl * st.T * st.L
        if len(self._lane_streams) < nlanes:
            self._lane_streams += [torch.cuda.Stream() for _ in range(nlanes - len(self._lane_streams))]
        lane_mods = mods  # lane-major [nlanes][S][nl][Bl][9C] straight from mdg_precompute_cond
        gs.ios = []
        # phase offset: lane k starts once lane k-1 is `lane_offset` layers into its first step,
        # so the lanes' identical kernel sequences run out of step (one lane's HBM-bound row-LN
        # GEMM beside the other's attention instead of two row-LN GEMMs splitting the CUs)
        nlay = st.dims.num_layers
        off = self.lane_offset if 0 < self.lane_offset < nlay else 0
        gs.lane_events = []
        for k in range(nlanes):
            ls = self._state(Bl, st.T, st.L, lane=1 + k)
            strm = self._lane_streams[k]
            strm.wait_stream(main)
            with torch.cuda.stream(strm):
                sk = strm.cuda_stream
                mask_k = gs.mask[k * Bl:(k + 1) * Bl]
                _lib.check(self.lib.mdg_prepare_mask(ctypes.byref(ls.dims), mask_k.data_ptr(), ls.ws.data_ptr(), sk),
                           "mdg_prepare_mask(lane)")
                if off and k > 0:
                    strm.wait_event(gs.lane_events[k - 1])
                base_k = st.base.data_ptr() + k * rows * self.C * 4
                for i in range(gs.S):
                    io = self._step_io(ls, gs.states[i, k * Bl].data_ptr(), gs.states[i + 1, k * Bl].data_ptr(), None,
                                       None if ipa is None else ipa[i, k * Bl].data_ptr(), lane_mods[k][i].data_ptr(),
                                       mods_f[i, k * Bl].data_ptr(), gs.dts[i], base=base_k)
                    gs.ios.append(io)
                    args = (ctypes.byref(ls.model_struct), ctypes.byref(io), mask_k.data_ptr(), ls.ws.data_ptr())
                    if off and i == 0 and k + 1 < nlanes:
                        _lib.check(self.lib.mdg_denoise_step_layers(*args, 0, off, sk), "mdg_denoise_step_layers")
                        ev = torch.cuda.Event()
                        ev.record(strm)
                        gs.lane_events.append(ev)
                        _lib.check(self.lib.mdg_denoise_step_layers(*args, off, nlay, sk), "mdg_denoise_step_layers")
                    else:
                        _lib.check(self.lib.mdg_denoise_step(*args, sk), "mdg_denoise_step")
        for k in range(nlanes):
            main.wait_stream(self._lane_streams[k])

    def _capture(self, gs, st):
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            self._run_sampler(gs, st)
        gs.graph = g
        gs.graph_has_cond = gs.has_cond
        g.replay()  # the capture did not execute; produce this call's result
