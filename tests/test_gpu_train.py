"""Training on the GPU: the eager autograd step runs on the device, and after optimizer steps
the HIP inference path (which packs the weights into its own layout) follows the updated
parameters — its forward equals the eager forward of the trained module (f32 tolerance)."""
import numpy as np
import pytest
import torch

from tests.conftest import build_model, load_golden, model_args
from tests.test_train import _args, _batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def test_train_steps_then_hip_inference_tracks_weights():
    from mdgen_finetune_amd.train import Trainer

    a = _args(["--lr", "1e-3", "--embed_dim", "64", "--mha_heads", "4"])
    tr = Trainer(a, device=torch.device("cuda"))
    b = _batch(a, B=2)
    losses = [tr.step([b])[0].item() for _ in range(4)]
    assert np.isfinite(losses).all()
    w = tr.wrapper
    m = w.model.eval()
    m.hip_dtype = "f32"
    prep = w.prep_batch({k: (v.cuda() if torch.is_tensor(v) else v) for k, v in b.items()})
    x = torch.randn_like(prep["latents"])
    t = torch.full((x.shape[0],), 0.3, device="cuda")
    with torch.no_grad():
        m.backend = "hip"
        v_hip = m(x, t, **prep["model_kwargs"]).clone()
        tr.step([b])  # weights change: the engine must re-pack
        m.eval()
        v_hip2 = m(x, t, **prep["model_kwargs"])
        m.backend = "torch"
        v_ref2 = m(x, t, **prep["model_kwargs"])
    assert not torch.equal(v_hip, v_hip2)
    err = (v_hip2 - v_ref2).abs().max().item()
    assert err <= 1e-3 * max(1.0, v_ref2.abs().max().item()), err


def _loss_inputs(d, device):
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    f = lambda k: torch.from_numpy(d["in_" + k]).to(device)  # noqa: E731
    kw = dict(mask=f("mask"), start_frames=Rigid(Rotation(rot_mats=f("rots")), f("trans")), x_cond=f("x_cond"),
              x_cond_mask=f("x_cond_mask"), aatype=f("aatype"))
    return f("x"), f("x0"), f("t_loss"), f("loss_mask"), kw


def _oracle_loss_grads(d, cfg):
    """Oracle GVP loss (batch mean) and d(loss)/d(param) by autograd on the CPU restatement."""
    from oracle import mdgen_oracle as O

    _, c = model_args(cfg)
    P = O.seeded_params(c, cfg["weights_seed"])
    for v in P.values():
        v.requires_grad_(True)
    kw = O.kwargs_from_npz(d)
    f = lambda k: torch.from_numpy(d["in_" + k])  # noqa: E731
    loss, v = O.gvp_training_loss(P, c, f("x"), f("x0"), f("t_loss"), f("loss_mask"), **kw)
    loss.mean().backward()
    return loss.detach(), v.detach(), {k: p.grad for k, p in P.items()}


def _model_loss(m, d, device):
    """Transport's own GVP plan + mean_flat with the fixture's injected (t, x0)."""
    from mdgen_finetune_amd.transport import create_transport
    from mdgen_finetune_amd.transport.transport import mean_flat

    x1, x0, t, lm, kw = _loss_inputs(d, device)
    tr = create_transport(m.args, "GVP", "velocity")
    t, xt, ut = tr.path_sampler.plan(t, x0, x1)
    v = m(xt, t, **kw)
    loss = mean_flat((v - ut) ** 2, lm)
    return loss, v


def test_gvp_loss_and_grads_on_gpu_match_oracle():
    """Config 3's differentiated step on the GPU (the training forward + backward the Trainer
    runs) against tests/golden/small_loss.npz (loss, prediction: the reference's own outputs)
    and the oracle's autograd gradients for every parameter.  Tolerance: loss rel 1e-5, pred
    max|d| 2e-5, each parameter's grad ||d||/||ref|| <= 1e-4 (fp32 everywhere)."""
    d, cfg = load_golden("small_loss")
    m, _ = build_model(cfg, "cuda")
    m.train()
    loss, v = _model_loss(m, d, "cuda")
    np.testing.assert_allclose(loss.detach().cpu().numpy(), d["out_loss"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(v.detach().cpu().numpy(), d["out_pred"], rtol=0, atol=2e-5)
    loss.mean().backward()
    _, _, g_ref = _oracle_loss_grads(d, cfg)
    names = dict(m.named_parameters())
    checked = 0
    for k, gr in g_ref.items():
        if gr is None or k not in names:
            continue
        g = names[k].grad
        assert g is not None, k
        den = max(float(gr.norm()), 1e-12)
        rel = float((g.detach().cpu() - gr).norm()) / den
        assert rel <= 1e-4 or float(gr.norm()) < 1e-8, (k, rel)
        checked += 1
    assert checked > 100
