"""Finite / checksum probe of the inference window (the bench's model and inputs) for A/B of
MLP kernel variants: python tools/window_probe.py LANES GRAPH(0|1) [B] [NUM_STEPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mdgen_finetune_amd.engine import get_engine  # noqa: E402

lanes, graph = int(sys.argv[1]), bool(int(sys.argv[2]))
B = int(sys.argv[3]) if len(sys.argv) > 3 else 16
ns = int(sys.argv[4]) if len(sys.argv) > 4 else 4
T, L = 1000, 4
m = bench.make_model(T, L).to("cuda")
m.hip_dtype = "bf16"
eng = get_engine(m)
eng.lanes = lanes
zs, kw, _ = bench.inputs(B, T, L, seed=100, device="cuda")
with torch.no_grad():
    for rep in range(2):
        ys = eng.sample_euler(zs, num_steps=ns, use_graph=graph, **kw)
        torch.cuda.synchronize()
        y = ys[-1].float()
        bad = (~torch.isfinite(y)).reshape(B, -1).any(-1).nonzero().flatten().tolist()
        print(f"lanes={lanes} graph={graph} B={B} steps={ns} rep={rep}: finite={not bad} bad_traj={bad[:8]} "
              f"sum={torch.nan_to_num(y).double().sum().item():.6f}", flush=True)
