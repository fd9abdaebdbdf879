"""Diagnostic: per-layer history of the lane-offset graph against the single chain.

Every mdg_denoise_step(_layers) call is split into single-layer calls, and after each layer the
lane's residual h and LayerNorm output xn are copied (on the lane's stream, inside the graph)
into a history buffer.  Replaying the 3-lane / offset-1 window many times, each replay whose
final states differ from the chain is reported with the first (step, layer) whose h or xn
differs, per lane, and the token rows (frames) affected.

usage: python tools/lane_hist.py REPLAYS [LANES OFFSET]
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


class HistLib:
    """ctypes library proxy: denoise-step calls run layer by layer with history copies."""

    def __init__(self, lib, eng):
        self._lib, self._eng = lib, eng
        self.hist = {}     # ws ptr -> list of (h, xn) snapshots (allocated lazily, reused by index)
        self.count = {}

    def __getattr__(self, name):
        return getattr(self._lib, name)

    def reset(self):
        self.count = {}

    def _state(self, ws):
        for st in self._eng._states.values():
            if hasattr(st, "ws") and hasattr(st, "dims") and st.ws.data_ptr() == ws:
                return st
        raise KeyError(ws)

    def regions(self, st):
        """name -> (byte offset, bytes) of the workspace regions a layer writes (bf16 packed planes)."""
        off = _lib.workspace_offsets(st.dims)
        N, C, d = st.N, self._eng.C, st.dims
        a = lambda x: (x + 255) // 256 * 256  # noqa: E731
        part = off["kbias"] + a(d.B * d.L * d.T * 4) + a(N * 4)
        return {"xn": (off["xn"], N * C * 2), "o": (off["o"], N * C * 2),
                "qkv_t": (off["qkv_t"], 3 * d.B * d.L * d.H * d.T * d.D * 2), "mlp_part": (part, 12 * N * C * 4)}

    def _snap(self, ws, stream):
        st = self._state(ws)
        i = self.count.get(ws, 0)
        self.count[ws] = i + 1
        lst = self.hist.setdefault(ws, [])
        regs = self.regions(st)
        if i == len(lst):
            lst.append({"h": torch.empty(st.N, self._eng.C, device="cuda"),
                        **{k: torch.empty(n, dtype=torch.uint8, device="cuda") for k, (o, n) in regs.items()}})
        snap = lst[i]
        with torch.cuda.stream(torch.cuda.ExternalStream(stream)):
            snap["h"].copy_(st.h)
            for k, (o, n) in regs.items():
                snap[k].copy_(st.ws[o:o + n])

    def _layers(self, m, io, mask, ws, first, last, stream):
        for k in range(first, last):
            rc = self._lib.mdg_denoise_step_layers(m, io, mask, ws, k, k + 1, stream)
            if rc:
                return rc
            self._snap(ws, stream)
        return 0

    def mdg_denoise_step(self, m, io, mask, ws, stream):
        nl = m._obj.dims.num_layers
        return self._layers(m, io, mask, ws, 0, nl, stream)

    def mdg_denoise_step_layers(self, m, io, mask, ws, first, last, stream):
        return self._layers(m, io, mask, ws, first, last, stream)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    offset = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    T, L = 64, 4
    cfg = dict(flags=[], latent_dim=21, L=L, T=T, tps=False, weights_seed=3)
    m, _ = build_model(cfg, "cuda", T=T)
    m.hip_dtype = "bf16"
    eng = get_engine(m)
    hl = HistLib(eng.lib, eng)
    eng.lib = hl
    inp = synthetic.make_inputs(4, B, T, L, 21)
    g = lambda k: torch.from_numpy(inp[k]).cuda()  # noqa: E731
    kw = dict(mask=g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")), x_cond=g("x_cond"),
              x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))
    eng.lanes, eng.lane_offset = 1, 0
    hl.reset()
    ref = eng.sample_euler(g("x"), num_steps=6, use_graph=False, **kw)
    torch.cuda.synchronize()
    chain_ws = [ws for ws in hl.hist][0]
    chain = [{k: v.clone() for k, v in snap.items()} for snap in hl.hist[chain_ws]]
    eng.lanes, eng.lane_offset = lanes, offset
    eng._graphs.clear()
    cap = eng._capture

    def capture(gs, st):  # the graph's copies write history slots 0.. (as the replays will)
        hl.reset()
        cap(gs, st)

    eng._capture = capture
    Bl = B // lanes
    nl = 5
    n_bad = 0
    for r in range(reps):
        hl.reset()
        got = eng.sample_euler(g("x"), num_steps=6, use_graph=True, **kw)
        torch.cuda.synchronize()
        if torch.equal(got, ref):
            continue
        n_bad += 1
        rep = {"replay": r, "final_max_abs": float((got - ref).abs().max()), "lanes": []}
        for ws, lst in hl.hist.items():
            if ws == chain_ws:
                continue
            st = hl._state(ws)
            k = st_lane = [key for key, v in eng._states.items() if v is st][0][3] - 1
            rows = slice(k * Bl * T * L, (k + 1) * Bl * T * L)
            first = None
            C, H, D = eng.C, eng.H, eng.D
            NL = Bl * T * L
            for i, snap in enumerate(lst[: len(chain)]):
                ref_s = chain[i]
                diff = {}
                # row regions: lane rows <-> chain rows [k NL, (k+1) NL)
                for name, width, dt in (("h", C, torch.float32), ("xn", C, torch.bfloat16), ("o", C, torch.bfloat16)):
                    a = snap[name].view(dt).view(-1, width) if name != "h" else snap[name]
                    b = (ref_s[name].view(dt).view(-1, width) if name != "h" else ref_s[name])[k * NL:(k + 1) * NL]
                    bad = (a != b).any(1).nonzero().flatten()
                    if bad.numel():
                        diff[name] = {"rows": int(bad.numel()), "lo": int(bad[0]), "hi": int(bad[-1]),
                                      "max": float((a.float() - b.float()).abs().max())}
                # planes [3][seq][H][T*D]: lane seq s <-> chain seq k*Bl*L + s
                pa = snap["qkv_t"].view(torch.bfloat16).view(3, Bl * L, H, T * D)
                pb = ref_s["qkv_t"].view(torch.bfloat16).view(3, B * L, H, T * D)[:, k * Bl * L:(k + 1) * Bl * L]
                bad = (pa != pb).any(-1).nonzero()
                if bad.numel():
                    diff["qkv_t"] = {"n": int(bad.shape[0]), "which_seq_head": bad[:6].tolist()}
                ma = snap["mlp_part"].view(torch.float32).view(12, NL, C)
                mb = ref_s["mlp_part"].view(torch.float32).view(12, B * T * L, C)[:, k * NL:(k + 1) * NL]
                bad = (ma != mb).any(-1).nonzero()
                if bad.numel():
                    diff["mlp_part"] = {"n": int(bad.shape[0]), "split_row": bad[:6].tolist()}
                if diff:
                    first = {"call": i, "step": i // nl, "layer": i % nl, "diff": diff}
                    break
            rep["lanes"].append({"lane": st_lane, "first": first})
        print(json.dumps(rep), flush=True)
    print(json.dumps({"summary": True, "reps": reps, "n_mismatch": n_bad, "lanes": lanes, "offset": offset}), flush=True)


if __name__ == "__main__":
    main()
