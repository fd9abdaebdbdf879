"""Property tests over random small shapes (mask / padding, B / T / L sweeps).

Each hypothesis example builds the model with seed-derived weights (synthetic.fill_module_)
and seed-derived inputs (synthetic.make_inputs), then checks two properties:

  * agreement with the pinned CPU oracle (oracle/mdgen_oracle.py) on the same weights and
    inputs.  CPU: the drop-in module's eager torch backend, max |d| <= 2e-5.  GPU (marked
    `gpu`): the HIP path, with the tolerances of tests/test_gpu_parity.py;
  * key-padding independence.  Changing x at padded residues (mask 0) leaves every unpadded
    output bit-for-bit unchanged.  Padded residues are masked as keys in both attentions and
    in the IPA prepend (latent_model.py:336, mha.py:370-376, ipa.py square_mask), and every
    other op is per token.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tests.conftest import build_model

SMALL = ["--embed_dim", "64", "--mha_heads", "4", "--ipa_heads", "2", "--ipa_head_dim", "8", "--ipa_qk", "4",
         "--ipa_v", "4", "--num_layers", "2"]


def _inputs(seed, B, T, L, n_pad, device):
    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    inp = synthetic.make_inputs(seed, B, T, L, 21, n_pad=n_pad)
    f = lambda k: torch.from_numpy(inp[k]).to(device)  # noqa: E731
    kw = dict(mask=f("mask"), start_frames=Rigid(Rotation(rot_mats=f("rots")), f("trans")), x_cond=f("x_cond"),
              x_cond_mask=f("x_cond_mask"), aatype=f("aatype"))
    return inp, f("x"), f("t"), kw


def _oracle(flags, seed, inp):
    from oracle import mdgen_oracle as O

    L = inp["x"].shape[2]
    c = O.Cfg.from_flags(flags, 21, L, False)
    P = O.seeded_params(c, seed)
    f = lambda k: torch.from_numpy(inp[k])  # noqa: E731
    with torch.no_grad():
        return O.forward(P, c, f("x"), f("t"), f("mask"), f("rots"), f("trans"), x_cond=f("x_cond"),
                         x_cond_mask=f("x_cond_mask"), aatype=f("aatype")).numpy()


def _padding_independent(m, x, t, kw, n_pad):
    """Unpadded outputs do not move when the padded residues' x changes."""
    if n_pad == 0:
        return
    x2 = x.clone()
    x2[:, :, -n_pad:] = torch.randn_like(x2[:, :, -n_pad:]) * 3.0
    with torch.no_grad():
        a = m(x, t, **kw)[:, :, :-n_pad]
        b = m(x2, t, **kw)[:, :, :-n_pad]
    assert torch.equal(a, b)


shapes = st.tuples(st.integers(1, 3), st.integers(1, 24), st.integers(2, 6), st.integers(0, 5),
                   st.integers(0, 10_000))


@settings(max_examples=10, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
@given(shapes)
def test_torch_backend_matches_oracle_and_is_padding_independent(shape):
    B, T, L, n_pad, seed = shape
    n_pad = min(n_pad, L - 1)
    cfg = dict(flags=SMALL, latent_dim=21, L=L, T=T, tps=False, weights_seed=seed)
    m, _ = build_model(cfg, "cpu", T=T)
    m.backend = "torch"
    inp, x, t, kw = _inputs(seed + 1, B, T, L, n_pad, "cpu")
    with torch.no_grad():
        v = m(x, t, **kw).numpy()
    ref = _oracle(SMALL, seed, inp)
    assert np.abs(v - ref).max() <= 2e-5
    _padding_independent(m, x, t, kw, n_pad)


@pytest.mark.gpu
@settings(max_examples=8, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow,
                                                                 HealthCheck.function_scoped_fixture])
@given(shape=st.tuples(st.integers(1, 3), st.integers(1, 80), st.sampled_from([4, 5]), st.integers(0, 2),
                       st.integers(0, 10_000)),
       dtype=st.sampled_from(["f32", "bf16"]))
def test_hip_matches_oracle_and_is_padding_independent(shape, dtype):
    """Default dims (C=384: the fused bf16 kernels at L = 4, the unfused ones at L = 5)."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    B, T, L, n_pad, seed = shape
    cfg = dict(flags=[], latent_dim=21, L=L, T=T, tps=False, weights_seed=seed)
    m, _ = build_model(cfg, "cuda", T=T)
    m.hip_dtype = dtype
    inp, x, t, kw = _inputs(seed + 1, B, T, L, n_pad, "cuda")
    with torch.no_grad():
        v = m(x, t, **kw).float().cpu().numpy()
    torch.set_num_threads(16)
    ref = _oracle([], seed, inp)
    assert np.isfinite(v).all()
    if dtype == "f32":
        assert np.abs(v - ref).max() <= 1e-3
    else:
        assert np.linalg.norm(v - ref) / np.linalg.norm(ref) <= 2.5e-2
    _padding_independent(m, x, t, kw, n_pad)
