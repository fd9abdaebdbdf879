"""The training step's glue kernels (csrc/train_glue.hip, train_hip.hip_embed / hip_final)
against eager fp32 autograd of the same ops: the token embedding + IPA prepend broadcast
(latent_model.py:242-255) and the FinalLayer (layers.py:58-75), forward values and every
gradient, at the training step's shape (C = 384, L = 4, latent 21) and the TPS latent (28),
with frame counts that leave ragged chunks.  Tolerance: fp32 reduction order only,
||d|| / ||ref|| <= 2e-6 (forward) and 1e-5 (gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


class _Hl:
    def __init__(self):
        from mdgen_finetune_amd import _lib

        self.lib = _lib.load()


@pytest.mark.parametrize("B,T,lat,cond,ipa", [(2, 70, 21, True, True), (3, 33, 28, True, True), (1, 32, 21, False, True),
                                             (2, 5, 21, True, False)])
def test_embed_forward_and_backward_match_eager(B, T, lat, cond, ipa):
    from mdgen_finetune_amd.train_hip import _HipEmbedFn

    torch.manual_seed(B * 100 + T)
    L, C, dev = 4, 384, "cuda"
    x = torch.randn(B, T, L, lat, device=dev)
    xc = torch.randn(B, T, L, lat, device=dev) if cond else None
    idx = torch.randint(0, 2, (B, T, L), device=dev) if cond else None
    p = {k: (torch.randn(*s, device=dev) * 0.3).requires_grad_(True) for k, s in
         dict(w1=(C, lat), b1=(C,), w2=(C, lat), b2=(C,), memb=(2, C), ipa=(B, L, C)).items()}
    pos = torch.randn(L, C, device=dev)
    g = torch.randn(B, T, L, C, device=dev)
    ipa_t = p["ipa"] if ipa else None
    h = _HipEmbedFn.apply(x, xc, idx, ipa_t, p["w1"], p["b1"], p["w2"] if cond else None, p["b2"] if cond else None,
                          p["memb"], pos, _Hl())
    (h * g).sum().backward()
    got = {k: v.grad.clone() for k, v in p.items() if v.grad is not None}
    for v in p.values():
        v.grad = None
    ref = x @ p["w1"].t() + p["b1"] + pos
    if cond:
        ref = ref + (xc @ p["w2"].t() + p["b2"] + p["memb"][idx])
    if ipa:
        ref = ref + p["ipa"][:, None]
    (ref * g).sum().backward()
    assert _rel(h, ref) <= 2e-6, _rel(h, ref)
    for k, v in p.items():
        if v.grad is None:
            assert k not in got or (not cond and k in ("w2", "b2")) or (not ipa and k == "ipa"), k
            continue
        assert k in got, k
        assert _rel(got[k], v.grad) <= 1e-5, (k, _rel(got[k], v.grad))


@pytest.mark.parametrize("B,T,lat", [(2, 70, 21), (3, 33, 28), (1, 1000, 21)])
def test_final_layer_forward_and_backward_match_eager(B, T, lat):
    from mdgen_finetune_amd.train_hip import _HipFinalFn

    torch.manual_seed(T + lat)
    L, C, dev = 4, 384, "cuda"
    h = (torch.randn(B, T, L, C, device=dev) * 2 + 0.5).requires_grad_(True)
    mods = (torch.randn(B, 2 * C, device=dev) * 0.2).requires_grad_(True)
    w = (torch.randn(lat, C, device=dev) * 0.05).requires_grad_(True)
    b = (torch.randn(lat, device=dev) * 0.1).requires_grad_(True)
    dv = torch.randn(B, T, L, lat, device=dev)
    v = _HipFinalFn.apply(h, mods, w, b, _Hl())
    (v * dv).sum().backward()
    got = [t.grad.clone() for t in (h, mods, w, b)]
    for t in (h, mods, w, b):
        t.grad = None
    shift, scale = mods.chunk(2, -1)
    xn = torch.nn.functional.layer_norm(h, (C,), eps=1e-6) * (1 + scale[:, None, None]) + shift[:, None, None]
    ref = xn @ w.t() + b
    (ref * dv).sum().backward()
    assert _rel(v, ref) <= 2e-6, _rel(v, ref)
    for name, a, t in zip(("h", "mods", "w", "b"), got, (h, mods, w, b)):
        assert _rel(a, t.grad) <= 1e-5, (name, _rel(a, t.grad))


@pytest.mark.parametrize("lead,K,ns,act,resid", [
    ((8,), 384, [2304] * 5 + [3456] * 5 + [768], "silu", False),  # every adaLN linear of the model
    ((8, 4), 384, [128, 256, 96, 192], "none", False),            # the IPA projections (B*L tokens)
    ((8, 4), 256, [384], "none", True),                           # linear_out + the IPA residual
    ((8,), 256, [384], "none", False),                            # t-MLP first linear
    ((37,), 100, [5, 70, 130], "silu", False),                    # ragged everything
    ((40,), 1024, [300, 17], "silu", False),                      # widest K, two token chunks
    ((5, 9), 132, [64, 64, 1], "none", False),                    # K not a multiple of 128
])
def test_seg_linear_forward_and_backward_match_fp64(lead, K, ns, act, resid):
    """mdg_seg_linear_fwd / _bwd (csrc/linear_small.hip) against float64 autograd of
    [lin(act(x)) (+ resid)]: outputs, dx, every weight and bias gradient.  fp32 FMA chains vs
    fp64: ||d|| / ||ref|| <= 2e-6."""
    from mdgen_finetune_amd.train_hip import seg_linear

    torch.manual_seed(K + len(ns))
    dev = "cuda"
    lins = [torch.nn.Linear(K, n).to(dev) for n in ns]
    for l in lins:
        torch.nn.init.normal_(l.bias, std=0.1)
    x = torch.randn(*lead, K, device=dev, requires_grad=True)
    r = torch.randn(*lead, ns[0], device=dev, requires_grad=True) if resid else None
    outs = seg_linear(x, lins, act=act, resid=r)
    gs = [torch.randn_like(o) for o in outs]
    sum((o * g).sum() for o, g in zip(outs, gs)).backward()
    got = [x.grad.clone()] + [t.grad.clone() for l in lins for t in (l.weight, l.bias)]
    if resid:
        got.append(r.grad.clone())
    xd = x.detach().double().requires_grad_(True)
    wd = [(l.weight.detach().double().requires_grad_(True), l.bias.detach().double().requires_grad_(True)) for l in lins]
    rd = r.detach().double().requires_grad_(True) if resid else None
    xa = torch.nn.functional.silu(xd) if act == "silu" else xd
    refs = [xa @ w.t() + b for w, b in wd]
    if resid:
        refs[0] = rd + refs[0]
    sum((o * g.double()).sum() for o, g in zip(refs, gs)).backward()
    for o, ref in zip(outs, refs):
        assert o.shape == ref.shape
        assert _rel(o, ref) <= 2e-6, _rel(o, ref)
    want = [xd.grad] + [t.grad for pair in wd for t in pair] + ([rd.grad] if resid else [])
    for i, (a, b) in enumerate(zip(got, want)):
        assert _rel(a, b) <= 2e-6, (i, _rel(a, b))


@pytest.mark.parametrize("path", [0, 1])
def test_gvp_plan_and_loss_match_eager(path):
    """mdg_gvp_plan / mdg_gvp_loss_fwd / _bwd (train_glue.hip) against the eager GVP / Linear plan
    and mean_flat loss of transport.py (the mask a broadcast view over frames, as prep_batch
    builds it): xt, ut to 1 ulp-level, loss and d out at ||d|| / ||ref|| <= 1e-6."""
    from mdgen_finetune_amd.train_hip import gvp_loss, gvp_plan
    from mdgen_finetune_amd.transport.transport import GVPCPlan, ICPlan, mean_flat

    torch.manual_seed(7 + path)
    B, T, L, K, dev = 3, 50, 4, 21, "cuda"
    x1 = torch.randn(B, T, L, K, device=dev)
    x0 = torch.randn_like(x1)
    t = torch.rand(B, device=dev)
    _, xt_ref, ut_ref = (GVPCPlan() if path == 0 else ICPlan()).plan(t, x0, x1)
    xt, ut = gvp_plan(t, x0, x1, path)
    assert _rel(xt, xt_ref) <= 1e-6 and _rel(ut, ut_ref) <= 1e-6, (_rel(xt, xt_ref), _rel(ut, ut_ref))
    mask = (torch.rand(B, 1, L, K, device=dev) > 0.3).float().expand(B, T, L, K)
    out = torch.randn(B, T, L, K, device=dev, requires_grad=True)
    g = torch.rand(B, device=dev)
    loss = gvp_loss(out, ut_ref, mask)
    (loss * g).sum().backward()
    d_got = out.grad.clone()
    out.grad = None
    ref = mean_flat((out - ut_ref) ** 2, mask)
    (ref * g).sum().backward()
    assert _rel(loss, ref) <= 1e-6, _rel(loss, ref)
    assert _rel(d_got, out.grad) <= 1e-6, _rel(d_got, out.grad)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gvp_loss_half_precision_prediction(dt):
    """A half-precision prediction (the eager FinalLayer under bf16 / fp16 autocast, L > 8, where
    the HIP FinalLayer is not used) is promoted to fp32 for the kernels, as the reference's
    (out - ut) with an fp32 ut promotes, and its gradient comes back in the prediction's dtype
    (the kernels read and wrote fp32 through a half-size buffer)."""
    from mdgen_finetune_amd.train_hip import gvp_loss
    from mdgen_finetune_amd.transport.transport import mean_flat

    torch.manual_seed(11)
    B, T, L, K, dev = 2, 20, 12, 21, "cuda"
    ut = torch.randn(B, T, L, K, device=dev)
    mask = (torch.rand(B, 1, L, K, device=dev) > 0.3).float().expand(B, T, L, K)
    out = torch.randn(B, T, L, K, device=dev).to(dt).requires_grad_(True)
    loss = gvp_loss(out, ut, mask)
    loss.sum().backward()
    assert loss.dtype == torch.float32 and out.grad.dtype == dt
    d_got = out.grad.float().clone()
    out.grad = None
    ref = mean_flat((out - ut) ** 2, mask)
    ref.sum().backward()
    assert _rel(loss, ref) <= 1e-6, _rel(loss, ref)
    assert _rel(d_got, out.grad.float()) <= 1e-2, _rel(d_got, out.grad.float())
