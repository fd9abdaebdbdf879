"""head_dim >= 32 (e.g. --embed_dim 256 --mha_heads 8, or 384 / 8): the attention operands use
64-column rows (MDG_HEAD_STRIDE), the temporal attention (and the L >= 16 spatial route) runs
the generic 16x16 MFMA kernel, the spatial L = 4 path the quad kernel (D <= 32) or the generic
VALU kernel.  The reference accepts any embed_dim // num_heads (mha.py:98-102).  Forward and a
short Euler solve against the oracle, both operand types, at the tolerances of
tests/test_gpu_parity.py; and the training path's loss and gradients against the oracle's
autograd (the layer-level checks are tests/test_gpu_train.py::test_hip_layer_backward_wide_heads)."""
import pytest
import torch

from tests.conftest import build_model
from tests.test_gpu_parity import _check

pytestmark = pytest.mark.gpu


def _case(flags, T, L, B, n_pad, seed):
    from mdgen_finetune_amd import synthetic
    from oracle import mdgen_oracle as O

    c = O.Cfg.from_flags(flags, 21, L, False)
    P = O.seeded_params(c, seed)
    inp = synthetic.make_inputs(seed + 1, B, T, L, 21, n_pad=n_pad)
    f = lambda k: torch.from_numpy(inp[k])  # noqa: E731
    kw = dict(mask=f("mask"), rots=f("rots"), trans=f("trans"), x_cond=f("x_cond"), x_cond_mask=f("x_cond_mask"),
              aatype=f("aatype"))
    torch.set_num_threads(16)
    with torch.no_grad():
        v = O.forward(P, c, f("x"), f("t"), **kw)
        ys = O.euler_sample(P, c, f("x"), num_steps=4, **kw)
    cfg = dict(flags=flags, latent_dim=21, L=L, T=T, tps=False, weights_seed=seed)
    return inp, v.numpy(), ys.numpy(), cfg


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("flags,T,L,n_pad", [
    (["--embed_dim", "256", "--mha_heads", "8"], 40, 4, 0),    # D = 32: quad spatial, wide temporal
    (["--embed_dim", "384", "--mha_heads", "8"], 24, 6, 1),    # D = 48: generic spatial (L = 6), padded
    (["--embed_dim", "256", "--mha_heads", "8"], 12, 20, 3),   # D = 32, L >= 16: spatial on the MFMA kernel
])
def test_wide_head_forward_and_euler_match_oracle(flags, T, L, n_pad, dtype):
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation
    from mdgen_finetune_amd.transport import Sampler, create_transport
    import functools

    inp, ref, ys_ref, cfg = _case(flags, T, L, B=2, n_pad=n_pad, seed=41 + L)
    m, _ = build_model(cfg, "cuda", T=T)
    m.hip_dtype = dtype
    g = lambda k: torch.from_numpy(inp[k]).cuda()  # noqa: E731
    kw = dict(mask=g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")), x_cond=g("x_cond"),
              x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))
    valid = inp["mask"][0, 0] > 0
    with torch.no_grad():
        v = m(g("x"), g("t"), **kw)
        _check(v, ref, dtype, valid=valid)
        fn = Sampler(create_transport(m.args, "GVP", "velocity")).sample_ode(sampling_method="euler", num_steps=4)
        ys = fn(g("x"), functools.partial(m.forward_inference, **kw))
    _check(ys[-1], ys_ref[-1], dtype, solve=True, valid=valid)


@pytest.mark.parametrize("dtype,flags,B,T", [
    ("f32", ["--embed_dim", "256", "--mha_heads", "8"], 2, 24),   # D = 32
    ("bf16", ["--embed_dim", "256", "--mha_heads", "8"], 2, 24),
    ("f32", ["--embed_dim", "384", "--mha_heads", "8"], 1, 40),   # D = 48
    ("bf16", ["--embed_dim", "384", "--mha_heads", "8"], 1, 40),
])
def test_wide_head_training_grads_match_oracle(dtype, flags, B, T):
    """Training at head_dim 32..63 on the HIP kernels (ABI 23; the reference trains any
    embed_dim // num_heads, mha.py:96-102): the GVP loss and every parameter gradient of the whole
    model (5 layers, IPA prepend) against the oracle's CPU autograd, bounds as config 3's
    (tests/test_gpu_train.py::test_default_dims_training_grads_match_oracle); the f32 path
    against an fp64 oracle run, each gradient within max(1e-4, 2x the fp32 oracle's own error)
    (the IPA q-projection gradients are ill-conditioned here: fp32 oracle vs fp64 1.5e-3)."""
    from tests.test_gpu_train import training_grads_vs_oracle

    training_grads_vs_oracle(dtype, B, T, flags=flags, tag="wide_head_grads", ref64=True)


def test_wide_head_plan_names_the_generic_route():
    m, _ = build_model(dict(flags=["--embed_dim", "256", "--mha_heads", "8"], latent_dim=21, L=4, T=8, tps=False,
                            weights_seed=3), "cuda", T=8)
    from mdgen_finetune_amd.engine import get_engine

    plan = get_engine(m).describe_plan(1, 8, 4)
    assert "wide heads" in plan["temporal"], plan
