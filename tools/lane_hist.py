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

    def _snap(self, ws, stream):
        st = self._state(ws)
        off = _lib.workspace_offsets(st.dims)
        N, C = st.N, self._eng.C
        i = self.count.get(ws, 0)
        self.count[ws] = i + 1
        lst = self.hist.setdefault(ws, [])
        if i == len(lst):
            lst.append((torch.empty(N, C, device="cuda"), torch.empty(N * C, dtype=torch.bfloat16, device="cuda")))
        h, xn = lst[i]
        with torch.cuda.stream(torch.cuda.ExternalStream(stream)):
            h.copy_(st.h)
            xn.copy_(st.ws[off["xn"]:off["xn"] + N * C * 2].view(torch.bfloat16))

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
    B, T, L = 6, 64, 4
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
    chain = [(h.clone(), x.clone()) for h, x in hl.hist[chain_ws]]
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
            for i, (h, xn) in enumerate(lst[: len(chain)]):
                hc, xc = chain[i]
                dh = (h - hc[rows]).abs()
                dx = (xn.float().view(-1, eng.C) - xc.float().view(-1, eng.C)[rows]).abs()
                if bool((dh > 0).any()) or bool((dx > 0).any()):
                    bad_rows = ((dh > 0).any(1) | (dx > 0).any(1)).nonzero().flatten()
                    frames = sorted({int(x) // L for x in bad_rows.tolist()})
                    first = {"call": i, "step": i // nl, "layer": i % nl, "h_max": float(dh.max()),
                             "xn_max": float(dx.max()), "n_rows": int(bad_rows.numel()),
                             "frames_lo_hi": [frames[0], frames[-1]], "n_frames": len(frames),
                             "h_rows": int((dh > 0).any(1).sum()), "xn_rows": int((dx > 0).any(1).sum())}
                    break
            rep["lanes"].append({"lane": st_lane, "first": first})
        print(json.dumps(rep), flush=True)
    print(json.dumps({"summary": True, "reps": reps, "n_mismatch": n_bad, "lanes": lanes, "offset": offset}), flush=True)


if __name__ == "__main__":
    main()
