"""The HIP IPA attention core of the training path (mdg_ipa_core_fwd / _bwd, csrc/ipa_train.hip)
against the eager autograd restatement of ipa.py:92-255 in the same module: the output and the
gradients of every IPA parameter and of the input, with padded residues masked downstream as the
model masks them (their rows are ill-conditioned in the reference itself: 1e5-offset logits)."""
import pytest
import torch

from mdgen_finetune_amd.model.layers import InvariantPointAttention

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _frames(B, L, gen):
    q = torch.randn(B, L, 4, generator=gen)
    q = q / q.norm(dim=-1, keepdim=True)
    a, b, c, d = q.unbind(-1)
    R = torch.stack([torch.stack([a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c)], -1),
                     torch.stack([2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b)], -1),
                     torch.stack([2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d], -1)], -2)
    return R, 5.0 * torch.randn(B, L, 3, generator=gen)


@pytest.mark.parametrize("seg", ["1", "0"])
@pytest.mark.parametrize("B,L,n_pad", [(8, 4, 0), (3, 6, 2), (2, 20, 3), (2, 32, 0), (2, 33, 1), (1, 100, 7),
                                       (1, 256, 51)])
def test_ipa_core_matches_eager_autograd(B, L, n_pad, seg, monkeypatch):
    """seg "1": the projections on mdg_seg_linear and the frames / softplus inside the core
    (MDG_IPA_LOCAL_POINTS | MDG_IPA_RAW_HW); "0": eager projections and global-frame points.
    L <= 32: one wave per (sample, head); L = 33 / 100 / 256 (ATLAS crop, 51 padded residues as
    in tests/test_gpu_parity.py's ATLAS case): the long kernels."""
    monkeypatch.setenv("MDG_TRAIN_SEG", seg)
    gen = torch.Generator().manual_seed(100 + L)
    C = 384
    ipa = InvariantPointAttention(C, 0, 32, 4, 8, 8)
    with torch.no_grad():
        for p in ipa.parameters():
            p.copy_(0.05 * torch.randn(p.shape, generator=gen))
    ipa = ipa.cuda()
    s0 = torch.randn(B, L, C, generator=gen).cuda()
    R, t = _frames(B, L, gen)
    R, t = R.cuda(), t.cuda()
    mask = torch.ones(B, L)
    if n_pad:
        mask[:, L - n_pad:] = 0
    mask = mask.cuda()
    G = torch.randn(B, L, C, generator=gen).cuda() * mask[..., None]
    res = []
    for hip in (False, True):
        ipa.hip_core = hip
        ipa.zero_grad(set_to_none=True)
        s = s0.clone().requires_grad_(True)
        out = ipa(s, R, t, mask)
        (out * G).sum().backward()
        res.append((out.detach() * mask[..., None], s.grad.clone(), {n: p.grad.clone() for n, p in ipa.named_parameters()}))
    (o0, ds0, g0), (o1, ds1, g1) = res

    def close(a, b, what, tol=2e-5):
        err = float((a - b).abs().max())
        assert err <= tol * max(1.0, float(b.abs().max())), (what, err, float(b.abs().max()))

    close(o1, o0, "out")
    close(ds1, ds0, "d s")
    for n in g0:
        close(g1[n], g0[n], n)
