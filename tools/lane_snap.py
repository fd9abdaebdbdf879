"""Diagnostic: per-LAUNCH history of the lane-offset graph against the single chain.

The library's snapshot hook (capi.hip, mdg_debug_snapshots) copies a denoise step's workspace,
residual h and latents x after every launch into a device buffer, on the launch's stream, so a
captured graph replays the copies.  The chain (lanes 1, eager) is recorded once; then the 3-lane
/ offset-1 graph is captured with its own buffer and replayed REPLAYS times.  For each replay
whose result differs from the chain, the first launch (per lane) after which any region of the
lane differs from the chain's rows of the same launch is reported, with the region, the rows
and the launch before it.

usage: python tools/lane_snap.py REPLAYS [LANES OFFSET B]
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from mdgen_finetune_amd import _lib, synthetic  # noqa: E402
from mdgen_finetune_amd.engine import get_engine  # noqa: E402
from mdgen_finetune_amd.rigid_utils import Rigid, Rotation  # noqa: E402
from tests.conftest import build_model  # noqa: E402


def snap_list(lib):
    n = lib.mdg_debug_snapshot_info(-1, None, None, None, 0)
    out = []
    off, ws, lab = ctypes.c_size_t(), ctypes.c_void_p(), ctypes.create_string_buffer(64)
    for i in range(n):
        lib.mdg_debug_snapshot_info(i, ctypes.byref(off), ctypes.byref(ws), lab, 64)
        out.append((off.value, ws.value, lab.value.decode()))
    return out


def a256(x):
    return (x + 255) // 256 * 256


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    offset = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    T, L = 64, 4
    cfg = dict(flags=[], latent_dim=21, L=L, T=T, tps=False, weights_seed=3)
    m, _ = build_model(cfg, "cuda", T=T)
    m.hip_dtype = "bf16"
    eng = get_engine(m)
    lib = _lib.load()
    lib.mdg_debug_snapshots.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.mdg_debug_snapshot_info.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                            ctypes.c_size_t]
    C, H, D, LAT = eng.C, eng.H, eng.D, 21
    inp = synthetic.make_inputs(4, B, T, L, LAT)
    g = lambda k: torch.from_numpy(inp[k]).cuda()  # noqa: E731
    kw = dict(mask=g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")), x_cond=g("x_cond"),
              x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))

    cap = 12 << 30
    buf_chain = torch.empty(cap, dtype=torch.uint8, device="cuda")
    eng.lanes, eng.lane_offset = 1, 0
    lib.mdg_debug_snapshots(buf_chain.data_ptr(), cap)
    ref = eng.sample_euler(g("x"), num_steps=6, use_graph=False, **kw)
    torch.cuda.synchronize()
    chain = snap_list(lib)
    lib.mdg_debug_snapshots(None, 0)

    buf = torch.empty(cap, dtype=torch.uint8, device="cuda")
    eng.lanes, eng.lane_offset = lanes, offset
    eng._graphs.clear()
    capture = eng._capture

    def hooked(gs, st):
        lib.mdg_debug_snapshots(buf.data_ptr(), cap)
        capture(gs, st)

    eng._capture = hooked
    eng.sample_euler(g("x"), num_steps=6, use_graph=True, **kw)  # eager pass + capture + replay 0
    torch.cuda.synchronize()
    slots = snap_list(lib)
    lib.mdg_debug_snapshots(None, 0)

    def dims_of(ws):
        for st in eng._states.values():
            if hasattr(st, "ws") and st.ws.data_ptr() == ws:
                return st.dims
        raise KeyError(ws)

    chain_ws = chain[0][1]
    cd = dims_of(chain_ws)
    per_lane = {}
    for off, ws, lab in slots:
        per_lane.setdefault(ws, []).append((off, lab))
    lane_ws = sorted(per_lane, key=lambda w: [k for k, v in eng._states.items() if getattr(v, "ws", None) is not None
                                              and v.ws.data_ptr() == w][0][3])
    Bl = B // lanes
    NL = Bl * T * L

    def regions(base, d, bufr):
        """name -> tensor views of one snapshot (chain or lane), rows-first."""
        o = _lib.workspace_offsets(d)
        N = d.B * d.T * d.L
        part = o["kbias"] + a256(d.B * d.L * d.T * 4) + a256(N * 4)
        tot = part + a256(12 * N * C * 4)
        v = lambda start, n: bufr[base + start: base + start + n]  # noqa: E731
        r = {"xn": v(o["xn"], N * C * 2).view(torch.bfloat16).view(N, C),
             "o": v(o["o"], N * C * 2).view(torch.bfloat16).view(N, C),
             "qkv_t": v(o["qkv_t"], 3 * d.B * d.L * H * T * D * 2).view(torch.bfloat16).view(3, d.B * L, H, T * D),
             "mlp_part": v(part, 12 * N * C * 4).view(torch.float32).view(12, N, C),
             "qkv_s": v(o["qkv_s"], N * 3 * C * 2).view(torch.bfloat16).view(N, 3 * C)}
        hb = base + a256(tot)
        r["h"] = bufr[hb: hb + N * C * 4].view(torch.float32).view(N, C)
        xb = hb + a256(N * C * 4)
        r["x"] = bufr[xb: xb + N * LAT * 4].view(torch.float32).view(N, LAT)
        return r

    def lane_slice(name, t, k):
        if name == "qkv_t":
            return t[:, k * Bl * L:(k + 1) * Bl * L]
        if name == "mlp_part":
            return t[:, k * NL:(k + 1) * NL]
        return t[k * NL:(k + 1) * NL]

    mask_all = kw["mask"].float()

    def explain(a, o_chain, o_d, k, slot):
        """Recompute the 4-residue attention of the corrupted (frame, head pair) from the block's
        dumped q|k|v tile (bf16) and test what reproduces the lane's o instead of the chain's."""
        r0 = o_d["rows"][0]
        hp = o_d["head_pairs"][0]
        layer = ((slot % 32) - 1) // 6
        st = [v for v in eng._states.values() if getattr(v, "ws", None) is not None][0]
        kvb = st.kvb[layer][0].double().cpu()  # [H][2][dp]
        rope = st.rope_l.double().cpu()
        half = D // 2
        cos = rope[: (L + 1) * half].reshape(L + 1, half)
        sin = rope[(L + 1) * half:].reshape(L + 1, half)
        tile = a["qkv_s"][r0:r0 + 4, hp * 6 * D:(hp + 1) * 6 * D].double().cpu()  # [4][144]
        mk = mask_all[k * Bl:(k + 1) * Bl].reshape(-1)[r0:r0 + 4].double().cpu()
        o_lane = a["o"][r0:r0 + 4, hp * 2 * D:(hp + 1) * 2 * D].double().cpu()
        o_ref = o_chain[r0:r0 + 4, hp * 2 * D:(hp + 1) * 2 * D].double().cpu()

        # the same wave's rows of the block's other 64-row band (the stage is reused per band)
        rb = r0 - 64 if (r0 % 128) >= 64 else r0 + 64
        other = a["qkv_s"][rb:rb + 4, hp * 6 * D:(hp + 1) * 6 * D].double().cpu()

        def attn(qpos=None, kpos=None, valid=None, kv_head=None, qrow=None, krow=None, vrow=None, src=None):
            out = torch.zeros(4, 2 * D, dtype=torch.float64)
            valid = mk if valid is None else valid
            tq, tk, tv = (src or (tile, tile, tile))
            for hh in range(2):
                gh = hp * 2 + hh
                q = tq[:, hh * D:(hh + 1) * D].clone()
                kk = tk[:, 2 * D + hh * D:2 * D + (hh + 1) * D].clone()
                vv = tv[:, 4 * D + hh * D:4 * D + (hh + 1) * D].clone()
                if qrow is not None:
                    q = q[qrow]
                if krow is not None:
                    kk = kk[krow]
                if vrow is not None:
                    vv = vv[vrow]

                def rot(x, pos):
                    y = x.clone()
                    for j in range(4):
                        c, s_ = cos[pos[j]], sin[pos[j]]
                        x0, x1 = x[j, 0::2], x[j, 1::2]
                        y[j, 0::2] = x0 * c - x1 * s_
                        y[j, 1::2] = x1 * c + x0 * s_
                    return y

                q = rot(q, qpos or [0, 1, 2, 3])
                kk = rot(kk, kpos or [0, 1, 2, 3])
                kh = gh if kv_head is None else kv_head
                kb, bv = kvb[kh, 0, :D], kvb[kh, 1, :D]
                for jq in range(4):
                    sc = torch.cat([(q[jq] * kb).sum()[None], kk @ q[jq]])
                    ok = torch.cat([torch.ones(1, dtype=torch.float64), valid])
                    sc = torch.where(ok > 0, sc, torch.full_like(sc, -1e30))
                    pr = torch.softmax(sc, 0)
                    out[jq, hh * D:(hh + 1) * D] = pr[0] * bv + pr[1:] @ vv
            return out

        res = {"mask": mk.tolist(), "layer": layer}
        base = attn()
        res["calc_vs_chain"] = float((base - o_ref).abs().max())
        res["calc_vs_lane"] = float((base - o_lane).abs().max())
        hyp = {}
        for j in range(4):
            v = mk.clone()
            v[j] = 1 - v[j]
            hyp[f"flip_mask_{j}"] = attn(valid=v)
        hyp["qpos0"] = attn(qpos=[0, 0, 0, 0])
        hyp["kpos0"] = attn(kpos=[0, 0, 0, 0])
        hyp["qpos_rev"] = attn(qpos=[3, 2, 1, 0])
        hyp["no_rope"] = attn(qpos=[0] * 4, kpos=[0] * 4)
        for sh in (1, 2, 3):
            perm = [(j + sh) % 4 for j in range(4)]
            hyp[f"q_from_{sh}"] = attn(qrow=perm)
            hyp[f"k_from_{sh}"] = attn(krow=perm)
            hyp[f"v_from_{sh}"] = attn(vrow=perm)
        for name, srcs in (("other_band_all", (other, other, other)), ("other_band_q", (other, tile, tile)),
                           ("other_band_k", (tile, other, tile)), ("other_band_v", (tile, tile, other)),
                           ("other_band_kv", (tile, other, other)), ("other_band_qk", (other, other, tile))):
            hyp[name] = attn(src=srcs)
        for gh2 in range(H):
            if gh2 // 2 != hp:
                hyp[f"kvb_head_{gh2}"] = attn(kv_head=gh2)
        res["lane_vs"] = sorted(((float((hv - o_lane).abs().max()), name) for name, hv in hyp.items()))[:6]
        res["o_lane_minus_chain"] = (o_lane - o_ref)[:, :8].tolist()
        res["other_rows"] = rb
        return res

    n_bad = 0
    print(json.dumps({"chain_slots": len(chain), "lane_slots": {str(i): len(per_lane[w]) for i, w in enumerate(lane_ws)}}),
          flush=True)
    for r in range(reps):
        got = eng.sample_euler(g("x"), num_steps=6, use_graph=True, **kw)
        torch.cuda.synchronize()
        if torch.equal(got, ref):
            continue
        n_bad += 1
        rep = {"replay": r, "final_max_abs": float((got - ref).abs().max()), "lanes": []}
        for k, ws in enumerate(lane_ws):
            ld = dims_of(ws)
            first = None
            for i, (off, lab) in enumerate(per_lane[ws]):
                coff, _, clab = chain[i]
                a = regions(off, ld, buf)
                b = regions(coff, cd, buf_chain)
                # compare what this launch wrote: the regions the chain's same launch changed
                bp = regions(chain[i - 1][0], cd, buf_chain) if i else None
                diff = {}
                for name in a:
                    if name == "x" and lab != "final euler launch":
                        continue  # x = the step's x_out, written by the FinalLayer launch only
                    if name != "x" and (bp is None and name not in ("h", "xn") or
                                        bp is not None and torch.equal(b[name], bp[name])):
                        continue
                    x, y = a[name], lane_slice(name, b[name], k)
                    if not torch.equal(x, y):
                        bad = (x != y).reshape(x.shape[0], -1).any(1).nonzero().flatten() if name not in (
                            "qkv_t", "mlp_part") else (x != y).reshape(x.shape[0] * x.shape[1], -1).any(1).nonzero().flatten()
                        diff[name] = {"n": int(bad.numel()), "lo": int(bad[0]), "hi": int(bad[-1]),
                                      "max": float((x.float() - y.float()).abs().max())}
                        if name in ("o", "xn", "h", "qkv_s") and bad.numel() <= 16:
                            dd = (x != y)[bad]  # rows x columns that differ
                            diff[name]["rows"] = bad.tolist()
                            diff[name]["cols_per_row"] = [dd[i].nonzero().flatten().tolist()[:64]
                                                          for i in range(dd.shape[0])]
                            diff[name]["head_pairs"] = sorted({c // (2 * D if name != "qkv_s" else 6 * D)
                                                               for c in dd.nonzero()[:, 1].tolist()})
                if diff:
                    first = {"slot": i, "label": lab, "chain_label": clab,
                             "prev": per_lane[ws][i - 1][1] if i else None, "diff": diff}
                    o_d = diff.get("o")
                    if o_d is not None and "rows" in o_d and "qkv_s" in a and len(o_d["rows"]) == 4:
                        first["hypotheses"] = explain(a, lane_slice("o", b["o"], k), o_d, k, i)
                    break
            rep["lanes"].append({"lane": k, "first": first})
        print(json.dumps(rep), flush=True)
    print(json.dumps({"summary": True, "reps": reps, "n_mismatch": n_bad, "lanes": lanes, "offset": offset}),
          flush=True)


if __name__ == "__main__":
    main()
