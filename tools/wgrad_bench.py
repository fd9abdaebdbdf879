"""Standalone timing (GPU) of mdg_wgrad (dW = dY^T X, db = colsum dY over the tokens) at the
training step's shapes (B=8 x T=1000 x L=4 = 32 000 tokens), checked against torch fp32 and timed
beside torch.matmul (hipBLASLt) of the same product.  Usage: python tools/wgrad_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdgen_finetune_amd import _lib  # noqa: E402
from mdgen_finetune_amd.train_hip import wgrad  # noqa: E402

lib = _lib.load()


def tm(fn, it=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


def run(N, M, K, need_b, name):
    dy = (torch.randn(N, M, device="cuda") * 0.5).to(torch.bfloat16)
    x = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    dw, db = wgrad(lib, _lib.MDG_BF16, dy, x, need_b)
    ref = dy.float().t() @ x.float()
    err = float((dw - ref).abs().max() / ref.abs().max())
    if need_b:
        err = max(err, float((db - dy.float().sum(0)).abs().max() / dy.float().sum(0).abs().max()))
    us = tm(lambda: wgrad(lib, _lib.MDG_BF16, dy, x, need_b))
    t_ref = tm(lambda: torch.matmul(dy.t(), x))
    fl = 2.0 * N * M * K
    print(f"{name:5s} N={N} M={M:5d} K={K:5d} b={int(need_b)}: mdg {us:7.1f} us ({fl / us / 1e6:6.1f} TF/s) "
          f"torch.matmul {t_ref:7.1f} us ({fl / t_ref / 1e6:6.1f} TF/s)  rel err {err:.1e}", flush=True)
    assert err < 1e-2, err


if __name__ == "__main__":
    N = 32000
    run(N, 384, 1536, False, "w2")
    run(N, 1536, 384, True, "w1")
    run(N, 1152, 384, True, "wqkv")
    run(N, 384, 384, False, "wo")
