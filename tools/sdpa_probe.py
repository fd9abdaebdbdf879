"""Which SDPA backends run (and how fast) for the training-path attention shapes on ROCm."""
import time

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

dev = "cuda"


def explicit(q, k, v, bias):
    w = q @ k.transpose(-1, -2) + bias
    w = torch.softmax(w, dim=-1, dtype=torch.float32).to(q.dtype)
    return w @ v


def bench(fn, *args, iters=10):
    for _ in range(2):
        o = fn(*args)
        o.sum().backward()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        o = fn(*args)
        o.sum().backward()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


for name, (N, H, S, d) in {"temporal": (32, 16, 1000, 24), "spatial": (8000, 16, 4, 24)}.items():
    for dt in (torch.float32, torch.bfloat16):
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(N, H, S, d, device=dev, dtype=dt, generator=g, requires_grad=True)
        k = torch.randn(N, H, S + 1, d, device=dev, dtype=dt, generator=g, requires_grad=True)
        v = torch.randn(N, H, S + 1, d, device=dev, dtype=dt, generator=g, requires_grad=True)
        bias = torch.zeros(N, 1, 1, S + 1, device=dev, dtype=dt)
        bias[::3, ..., S // 2:S] = float("-inf")
        ref = explicit(q.float(), k.float(), v.float(), bias.float())
        print(name, dt, "explicit ms", round(bench(explicit, q, k, v, bias), 3), flush=True)
        for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.MATH):
            try:
                with sdpa_kernel([be]):
                    f = lambda q, k, v, b: F.scaled_dot_product_attention(q, k, v, attn_mask=b, scale=1.0)  # noqa
                    o = f(q, k, v, bias)
                    err = (o.float() - ref).abs().max().item()
                    ms = bench(f, q, k, v, bias)
                print(name, dt, be.name, "ms", round(ms, 3), "maxerr", err, flush=True)
            except Exception as e:  # noqa: BLE001
                print(name, dt, be.name, "unavailable:", str(e).splitlines()[0][:120], flush=True)
