"""Launch the roofline kernels of bench.py (fused MLP, fused out_proj + q|k|v, row-LN GEMM,
temporal attention) at the bench's per-lane shape after one eager sampling window, for rocprofv3 counter passes
(tools/roof_pmc.sh).  Usage: python tools/roof_kernels.py [B T L]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

B, T, L = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (8, 1000, 4)
dev = torch.device("cuda", 0)
from mdgen_finetune_amd.engine import get_engine  # noqa: E402

m = bench.make_model(T, L).to(dev)
m.hip_dtype = "bf16"
eng = get_engine(m)
zs, kw, _ = bench.inputs(B, T, L, seed=100, device=dev)
with torch.no_grad():
    eng.sample_euler(zs, num_steps=3, use_graph=False, **kw)
    torch.cuda.synchronize()
    roofs = bench.roofline(eng, eng._state(B, T, L), "bf16", B, T, L)
torch.cuda.synchronize()
for r in roofs.values():
    print(r)
