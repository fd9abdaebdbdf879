"""Engine behaviour around the captured sampler and the autograd boundary:
  * the per-shape hipGraph cache must not replay a program captured with an optional input
    (aatype / x_cond) that a later call omits, or captured for a different lane count;
  * a differentiable call on an eval()-mode model (guidance through a frozen prior) must
    return a tensor connected to the autograd graph, not the HIP inference engine's."""
import functools

import pytest
import torch

from tests.conftest import build_model, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def _kw(d, aatype=True):
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    f = lambda k: torch.from_numpy(d["in_" + k]).cuda()  # noqa: E731
    kw = dict(mask=f("mask"), start_frames=Rigid(Rotation(rot_mats=f("rots")), f("trans")), x_cond=f("x_cond"),
              x_cond_mask=f("x_cond_mask"))
    if aatype:
        kw["aatype"] = f("aatype")
    return kw


def test_graph_cache_alternating_optional_inputs():
    from mdgen_finetune_amd.engine import get_engine

    d, cfg = load_golden("small_sim_T8")
    m, _ = build_model(cfg, "cuda")
    m.hip_dtype = "f32"
    eng = get_engine(m)
    zs = torch.from_numpy(d["in_zs"]).cuda()
    ref_aa = eng.sample_euler(zs, num_steps=4, use_graph=False, **_kw(d, True))
    ref_no = eng.sample_euler(zs, num_steps=4, use_graph=False, **_kw(d, False))
    assert not torch.equal(ref_aa, ref_no)  # the aatype embedding matters
    for aa in (True, False, True, False):
        got = eng.sample_euler(zs, num_steps=4, use_graph=True, **_kw(d, aa))
        assert torch.equal(got, ref_aa if aa else ref_no), aa
    # changing the lane count re-keys the graph (B = 2 splits into 2 lanes of 1 when forced)
    eng.lanes = 2
    got = eng.sample_euler(zs, num_steps=4, use_graph=True, **_kw(d, True))
    eng.lanes = 0
    assert torch.equal(got, ref_aa)
    assert any(k[-1] == 2 for k in eng._graphs)


def test_eval_mode_model_is_differentiable_when_grad_enabled():
    """rtb_utils 'dps' guidance differentiates through an eval()-mode prior
    (gfn_diffusion.py:292): the output must carry grad_fn and d/dx must match eager torch."""
    d, cfg = load_golden("small_sim_T8")
    m, _ = build_model(cfg, "cuda")
    m.eval()
    m.hip_dtype = "f32"
    x = torch.from_numpy(d["in_x"]).cuda().requires_grad_(True)
    t = torch.from_numpy(d["in_t"]).cuda()
    v = m(x, t, **_kw(d))
    assert v.grad_fn is not None
    (gx,) = torch.autograd.grad(v.square().sum(), x)
    m.backend = "torch"
    x2 = x.detach().clone().requires_grad_(True)
    v2 = m(x2, t, **_kw(d))
    (gx2,) = torch.autograd.grad(v2.square().sum(), x2)
    torch.testing.assert_close(gx, gx2, rtol=1e-4, atol=1e-4)
    # and under no_grad the same call takes the HIP engine (no graph attached)
    m.backend = "hip"
    with torch.no_grad():
        v3 = m(x.detach(), t, **_kw(d))
    assert v3.grad_fn is None
    torch.testing.assert_close(v3, v.detach(), rtol=1e-4, atol=1e-4)
