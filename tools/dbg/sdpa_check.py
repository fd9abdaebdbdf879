"""Debug: torch SDPA (default backend) vs the math backend with a float mask, ROCm, several head dims."""
import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

torch.manual_seed(0)
for N, H, S, Sk, d in [(10, 8, 16, 17, 48), (10, 12, 16, 17, 32), (10, 8, 16, 17, 40), (10, 8, 16, 17, 56),
                       (32, 8, 5, 6, 48), (10, 16, 16, 17, 24), (8, 8, 300, 301, 48), (10, 8, 16, 17, 64)]:
    q, k, v = (torch.randn(N, H, s, d, device="cuda") for s in (S, Sk, Sk))
    bias = torch.zeros(N, 1, 1, Sk, device="cuda")
    o0 = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=1.0)
    with sdpa_kernel(SDPBackend.MATH):
        o1 = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=1.0)
    ref = torch.softmax(q.double() @ k.double().transpose(-1, -2), -1) @ v.double()
    print(N, H, S, Sk, d, "default", float((o0.double() - ref).norm() / ref.norm()),
          "math", float((o1.double() - ref).norm() / ref.norm()), flush=True)
