"""The graphed step's optimizer update on library kernels (csrc/optim.hip via
optim_hip.FusedClipAdam) against torch's clip_grad_norm_ + Adam / AdamW (foreach=False, the
per-tensor reference loop), three steps with fresh gradients each: parameters, exp_avg,
exp_avg_sq, step counts and the returned norm.  Tolerance: fp32 reduction order of the norm
and the update's rounding, relative 2e-6 (state) and 2e-6 of the parameter scale (parameters).
Ragged sizes (1 element, chunk boundaries 16384 +- 1), gradients at unaligned offsets (views of
one flat buffer, the scalar path) and a hipGraph capture + replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [(1,), (3, 7), (16384,), (16385,), (128, 257), (40000,)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _make(seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ps = [torch.randn(*s, generator=g).cuda().requires_grad_(True) for s in SIZES]
    return ps


def _grads(ps, step, flat=None):
    g = torch.Generator(device="cpu").manual_seed(1000 + step)
    gs = [torch.randn(p.shape, generator=g).cuda() * (0.1 + i) for i, p in enumerate(ps)]
    if flat is not None:  # views at odd offsets of one buffer (the split-mode gradient layout)
        off = 1
        for p, gg in zip(ps, gs):
            v = flat[off:off + p.numel()].view_as(p)
            v.copy_(gg)
            p.grad = v
            off += p.numel()
    else:
        for p, gg in zip(ps, gs):
            p.grad = gg.clone()


@pytest.mark.parametrize("cls,wd,max_norm", [("adam", 0.0, 1.0), ("adam", 0.0, 1e9), ("adam", 0.1, 0.5),
                                             ("adamw", 0.01, 1.0), ("adam", 0.0, 0.0)])
@pytest.mark.parametrize("unaligned", [False, True])
def test_fused_clip_adam_matches_torch(cls, wd, max_norm, unaligned):
    from mdgen_finetune_amd.optim_hip import FusedClipAdam

    C = torch.optim.AdamW if cls == "adamw" else torch.optim.Adam
    ref, got = _make(7), _make(7)
    opt_r = C(ref, lr=1e-3, weight_decay=wd, foreach=False)
    opt_g = C(got, lr=1e-3, weight_decay=wd, capturable=True, fused=True)
    fused = FusedClipAdam(opt_g, got, max_norm)
    n = sum(p.numel() for p in got)
    flat = torch.empty(n + 1, device="cuda") if unaligned else None
    for step in range(3):
        _grads(ref, step)
        _grads(got, step, flat)
        want = torch.nn.utils.clip_grad_norm_(ref, max_norm) if max_norm > 0 else None
        opt_r.step()
        norm = fused.step()
        torch.cuda.synchronize()
        if want is not None:
            assert _rel(norm, want) <= 2e-6, (step, float(norm), float(want))
        for pr, pg in zip(ref, got):
            scale = float(pr.detach().abs().max()) + 1e-3
            assert float((pr.detach() - pg.detach()).abs().max()) <= 2e-6 * scale
            sr, sg = opt_r.state[pr], opt_g.state[pg]
            assert _rel(sg["exp_avg"], sr["exp_avg"]) <= 2e-6
            assert _rel(sg["exp_avg_sq"], sr["exp_avg_sq"]) <= 2e-6
            assert float(sg["step"]) == float(sr["step"]) == step + 1


def test_fused_clip_adam_graph_replay_matches_eager():
    """Captured once, replayed twice == two eager steps, bit for bit (same kernels)."""
    from mdgen_finetune_amd.optim_hip import FusedClipAdam

    a, b = _make(3), _make(3)
    oa = torch.optim.Adam(a, lr=1e-3, capturable=True, fused=True)
    ob = torch.optim.Adam(b, lr=1e-3, capturable=True, fused=True)
    fa, fb = FusedClipAdam(oa, a, 1.0), FusedClipAdam(ob, b, 1.0)
    _grads(a, 0)
    _grads(b, 0)
    fa.step()
    fb.step()  # state exists before the capture (GraphedStep warms up the same way)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    fb.reserve()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            # temporaries freed inside the capture: their blocks go back to the graph's pool, and
            # the replay rewrites them before the optimizer runs (must not hold its table)
            junk = [torch.full((1 << 16,), 7.0, device="cuda") for _ in range(4)]
            del junk
            nb = fb.step(capturing=True)
    torch.cuda.current_stream().wait_stream(s)
    fb.finish_capture()
    for _ in range(2):
        na = fa.step()
        graph.replay()
    torch.cuda.synchronize()
    assert float(na) == float(nb)
    for pa, pb in zip(a, b):
        assert torch.equal(pa.detach(), pb.detach())
        assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])
        assert float(ob.state[pb]["step"]) == 3.0
