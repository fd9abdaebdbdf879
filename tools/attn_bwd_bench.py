"""Time mdg_attn_temporal_bwd at the training step's shape (B=8 trajectories x L=4 residues,
T=1000 frames, 16 heads of 24): the fused single-pass kernel (generic 0) against the two-pass
MFMA kernels (generic 2), HIP events around N back-to-back calls; prints one JSON line.
The work is 4 S-sized products per pass (S, dP, dV, dK) + dQ: 2 * 5 * T * T * 32 FLOP per
(sequence, head) at the padded head dim (the kernels' MFMA work)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd import _lib  # noqa: E402


def main():
    B, L, T, H, D = int(os.environ.get("B", 8)), 4, int(os.environ.get("T", 1000)), 16, 24
    lib = _lib.load()
    dev = "cuda"
    BL, C, DP = B * L, H * D, _lib.MDG_DP
    torch.manual_seed(0)
    planes = torch.zeros(3, BL, H, T, DP, device=dev, dtype=torch.bfloat16)
    planes[..., :D] = (torch.randn(3, BL, H, T, D, device=dev) * 0.5).to(torch.bfloat16)
    planes[1:, ..., D] = 1.0
    kb = torch.zeros(BL, T, device=dev)
    kvb = torch.randn(H, 2, DP, device=dev) * 0.1
    o = torch.randn(B * T * L, C, device=dev).to(torch.bfloat16)
    do = torch.randn(B * T * L, C, device=dev).to(torch.bfloat16)
    # lse consistent with the planes (log2 units) so P is a distribution
    q, k = planes[0, ..., :D].float(), planes[1, ..., :D].float()
    lse = torch.logsumexp(torch.einsum("shtd,shud->shtu", q, k) * math.log(2.0), -1) / math.log(2.0)
    lse = lse.contiguous()
    # bias-gradient slots: the two-pass kernels need more than the fused one (one per query block and wave)
    parts = max(lib.mdg_attn_temporal_bwd_parts(_lib.MDG_BF16, B, T, L, g) for g in (0, 2))
    bpart = torch.zeros(H, parts, 2, DP, device=dev)
    scratch = torch.empty(lib.mdg_attn_temporal_bwd_scratch(_lib.MDG_BF16, B, T, L, H, D), device=dev, dtype=torch.uint8)
    dqkv = torch.empty(B * T * L, 3 * C, device=dev, dtype=torch.bfloat16)
    s = _lib.stream_handle()

    def call(generic):
        _lib.check(lib.mdg_attn_temporal_bwd(_lib.MDG_BF16, B, T, L, H, D, planes.data_ptr(), kb.data_ptr(),
                                             kvb.data_ptr(), o.data_ptr(), 0, do.data_ptr(), lse.data_ptr(), 0, T + 1,
                                             scratch.data_ptr(), dqkv.data_ptr(), 3 * C, bpart.data_ptr(),
                                             D ** -0.5, math.log(2.0), generic, s), "attn_bwd")

    out = {"shape": f"B={B} L={L} T={T} H={H} D={D}"}
    res = {}
    for name, g in (("fused", 0), ("two_pass", 2)):
        for _ in range(3):
            call(g)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            call(g)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        flops = 2 * 5 * T * T * DP * BL * H
        out[name] = {"us_per_call": round(us, 1), "tflops_padded": round(flops / us / 1e6, 1)}
        res[name] = dqkv.float().clone()
    out["max_abs_diff_fused_vs_two_pass"] = float((res["fused"] - res["two_pass"]).abs().max())
    out["ref_max"] = float(res["two_pass"].abs().max())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
