"""Diagnostic: replay the concurrent-lane Euler window many times in ONE process and report the
locus of every replay that differs from the single-chain result (step, lane, b, t, l, channel,
magnitude).  Variants are chosen by the environment (MDG_* knobs are read once per process), so
tools/gpu_lane_race.sh runs one process per variant.

usage: python tools/lane_race.py LANES OFFSET REPLAYS [B] [T] [mode]
  mode: graph (default) | eager | chain (single-chain graph replays against the eager chain)
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from mdgen_finetune_amd import synthetic  # noqa: E402
from mdgen_finetune_amd.engine import get_engine  # noqa: E402
from mdgen_finetune_amd.rigid_utils import Rigid, Rotation  # noqa: E402
from tests.conftest import build_model  # noqa: E402


def locus(got, ref, Bl):
    d = (got - ref).abs()
    bad = d > 0
    n = int(bad.sum())
    if n == 0:
        return None
    steps = bad.flatten(1).any(1).nonzero().flatten().tolist()
    s0 = steps[0]
    idx = bad[s0].nonzero()
    first = idx[0].tolist()
    lanes = sorted({int(b) // Bl for b in idx[:, 0].tolist()})
    return {"n_bad": n, "steps": steps, "first_step": s0, "lanes": lanes, "first_btlc": first,
            "max_abs": float(d.max()), "max_abs_first_step": float(d[s0].max()),
            "n_bad_first_step": int(bad[s0].sum()), "ts_first_step": sorted({int(i) for i in idx[:, 1].tolist()})[:16],
            "ls_first_step": sorted({int(i) for i in idx[:, 2].tolist()}),
            "cs_first_step": sorted({int(i) for i in idx[:, 3].tolist()})[:24]}


def order_counters():
    """The MDG_DIAG_ORDER build's launch-order counters (xn buffer, reductions done, spatial
    blocks started, blocks that started early, worst deficit), or None in other builds."""
    import ctypes

    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    if not hasattr(lib, "mdg_debug_order_counters"):
        return None
    buf = (ctypes.c_ulonglong * 320)()
    n = lib.mdg_debug_order_counters(buf, 320)
    return [{"xn": hex(buf[5 * i]), "red": buf[5 * i + 1], "spa": buf[5 * i + 2], "early": buf[5 * i + 3],
             "worst": buf[5 * i + 4]} for i in range(max(n, 0))]


def spa_diag():
    """The MDG_DIAG_SPA=9 build's log: lanes whose second evaluation of the fused spatial
    attention differed from the first (block, thread, band, column, bits 1, bits 2, row, pair)."""
    import ctypes

    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    if not hasattr(lib, "mdg_debug_spa_diag"):
        return None
    buf = (ctypes.c_uint * (4 + 32 * 128))()
    lib.mdg_debug_spa_diag(buf, 4 + 32 * 128)
    n = buf[0]
    import struct

    f = lambda u: struct.unpack("f", struct.pack("I", u))[0]  # noqa: E731
    names = ["hq", "hk", "hv", "sb", "s0", "s3", "sb_x", "s0_x", "s3_x", "pb", "p0", "inv"]
    recs = [list(buf[4 + 32 * i: 36 + 32 * i]) for i in range(min(n, 128))]
    out = []
    for r in recs:
        t1, t2 = r[8:20], r[20:32]
        out.append({"block": r[0], "tid": r[1], "band": r[2], "c": r[3], "o1": f(r[4]), "o2": f(r[5]), "m": r[6],
                    "pair": r[7], "first_diff": next((names[i] for i in range(12) if t1[i] != t2[i]), None),
                    "diffs": [names[i] for i in range(12) if t1[i] != t2[i]]})
    return {"n": n, "records": out[:48]}


def main():
    lanes, offset, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    mode = sys.argv[6] if len(sys.argv) > 6 else "graph"
    cfg = dict(flags=[], latent_dim=21, L=4, T=T, tps=False, weights_seed=3)
    m, _ = build_model(cfg, "cuda", T=T)
    m.hip_dtype = "bf16"
    eng = get_engine(m)
    inp = synthetic.make_inputs(4, B, T, 4, 21)
    g = lambda k: torch.from_numpy(inp[k]).cuda()  # noqa: E731
    kw = dict(mask=g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")), x_cond=g("x_cond"),
              x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))
    eng.lanes, eng.lane_offset = 1, 0
    ref = eng.sample_euler(g("x"), num_steps=6, use_graph=False, **kw)
    if mode != "chain":
        eng.lanes, eng.lane_offset = lanes, offset
    eng._graphs.clear()
    Bl = B // max(lanes, 1) if mode != "chain" else B
    bad = []
    for r in range(reps):
        got = eng.sample_euler(g("x"), num_steps=6, use_graph=(mode != "eager"), **kw)
        loc = locus(got, ref, Bl)
        if loc is not None:
            loc["replay"] = r
            oc = order_counters()
            if oc is not None:
                loc["order"] = oc
            bad.append(loc)
            print(json.dumps(loc), flush=True)
    env = {k: v for k, v in os.environ.items() if k.startswith("MDG_")}
    print(json.dumps({"summary": True, "lanes": lanes, "offset": offset, "B": B, "T": T, "mode": mode, "reps": reps,
                      "n_mismatch": len(bad), "env": env, "order": order_counters(), "spa_diag": spa_diag()}),
          flush=True)


if __name__ == "__main__":
    main()
