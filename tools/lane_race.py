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
            bad.append(loc)
            print(json.dumps(loc), flush=True)
    env = {k: v for k, v in os.environ.items() if k.startswith("MDG_")}
    print(json.dumps({"summary": True, "lanes": lanes, "offset": offset, "B": B, "T": T, "mode": mode, "reps": reps,
                      "n_mismatch": len(bad), "env": env}), flush=True)


if __name__ == "__main__":
    main()
