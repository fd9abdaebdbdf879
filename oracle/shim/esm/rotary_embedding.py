"""Test-only restatement of fair-esm 1.0.2 `esm.rotary_embedding.RotaryEmbedding`.

Behaviour (as used at reference mha.py:13, 129-130, 356-357):
  * inv_freq[i] = 1 / 10000 ** (arange(0, dim, 2) / dim)       (buffer, fp32)
  * the cos/sin tables are built from the length of **k** (seq dim -2):
        freqs = outer(arange(S_k), inv_freq); emb = cat(freqs, freqs)
  * apply(x) = x * cos[:S_x] + rotate_half(x) * sin[:S_x],
    rotate_half(x) = cat(-x2, x1) over the two halves of the last dim.
"""
import torch


def _rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def _apply(x, cos, sin):
    n = x.shape[-2]
    return x * cos[:, :n, :] + _rotate_half(x) * sin[:, :n, :]


class RotaryEmbedding(torch.nn.Module):
    def __init__(self, dim, *_, **__):
        super().__init__()
        inv_freq = 1.0 / (10000 ** (torch.arange(0, dim, 2).float() / dim))
        self.register_buffer("inv_freq", inv_freq)

    def forward(self, q, k):
        s = k.shape[-2]
        pos = torch.arange(s, device=k.device).type_as(self.inv_freq)
        freqs = torch.einsum("i,j->ij", pos, self.inv_freq)
        emb = torch.cat((freqs, freqs), dim=-1).to(k.device)
        cos = emb.cos()[None, :, :]
        sin = emb.sin()[None, :, :]
        return _apply(q, cos, sin), _apply(k, cos, sin)
