"""Temporal / spatial attention timing at the bench shape (B=8, T=1000, L=4, H=16, D=24).
Usage: python tools/attn_bench.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd import _lib  # noqa: E402

lib = _lib.load()
it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, T, L, H, D = 8, 1000, 4, 16, 24
BL = B * L
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.zeros(3, BL, H, T, 32, device="cuda")
qkv[..., :D] = torch.randn(3, BL, H, T, D, device="cuda", generator=g) * 0.5
qkv[1:, ..., D] = 1.0
qkv = qkv.to(torch.bfloat16)
kbias = torch.zeros(BL, T, device="cuda")
kvb = torch.zeros(H, 2, 32, device="cuda")
kvb[:, :, :D] = torch.randn(H, 2, D, device="cuda", generator=g)
kvb[:, 1, D] = 1.0
out = torch.zeros(B * T * L, H * D, device="cuda", dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream


def f():
    _lib.check(lib.mdg_attn_temporal(1, B, T, L, H, D, qkv.data_ptr(), kbias.data_ptr(), kvb.data_ptr(),
                                     out.data_ptr(), s), "attn_temporal")


f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    f()
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) / it * 1e3
fl = 4.0 * BL * H * T * (T + 1) * D
print(f"attn_temporal B={B} T={T} L={L} H={H} D={D}: {us:.1f} us  {fl / us / 1e6:.1f} TFLOP/s (algorithmic, D={D})")
