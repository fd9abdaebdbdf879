"""Training on the GPU: the eager autograd step runs on the device, and after optimizer steps
the HIP inference path (which packs the weights into its own layout) follows the updated
parameters — its forward equals the eager forward of the trained module (f32 tolerance)."""
import numpy as np
import pytest
import torch

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
