"""mdg_prep_latents (prep_batch on the device) against the reference's golden prep_batch
(get_offsets + LAPACK eigh quaternions, tests/golden/prep_batch.npz) and against the eager
CPU path on many random frames, including near-180-degree relative rotations."""
import numpy as np
import pytest
import torch

from tests.test_train import _args

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


@pytest.mark.parametrize("tps", [False, True])
def test_prep_batch_hip_matches_reference_golden(golden, tps):
    from mdgen_finetune_amd.wrapper import NewMDGenWrapper

    d, _ = golden("prep_batch")
    a = _args(["--tps_condition"] if tps else [])
    a.sim_condition = not tps
    w = NewMDGenWrapper(a)
    batch = {k[3:]: torch.from_numpy(d[k]).cuda() for k in d.files if k.startswith("in_")}
    p = w.prep_batch(batch)
    sfx = "_tps" if tps else ""
    np.testing.assert_allclose(p["latents"].cpu().numpy(), d["out_latents" + sfx], rtol=0, atol=5e-6)
    np.testing.assert_array_equal(p["loss_mask"].cpu().numpy(), d["out_loss_mask" + sfx])
    np.testing.assert_array_equal(p["model_kwargs"]["x_cond_mask"].cpu().numpy(), d["out_cond_mask" + sfx])
    xc = np.where(d["out_cond_mask" + sfx][..., None] == 1, d["out_latents" + sfx], 0.0)
    np.testing.assert_allclose(p["model_kwargs"]["x_cond"].cpu().numpy(), xc, rtol=0, atol=5e-6)


def test_prep_latents_random_frames_match_eager_path():
    from mdgen_finetune_amd.data import _axis_angle_to_rot
    from mdgen_finetune_amd.wrapper import NewMDGenWrapper

    rng = np.random.default_rng(3)
    B, T, L = 3, 257, 7
    v = rng.standard_normal((B, T, L, 3))
    v *= (rng.uniform(0, np.pi, (B, T, L, 1)) / np.linalg.norm(v, axis=-1, keepdims=True))
    v[:, 1::5] *= np.pi / np.linalg.norm(v[:, 1::5], axis=-1, keepdims=True) * 0.9999  # near 180 deg
    rots = torch.from_numpy(_axis_angle_to_rot(v).astype(np.float32))
    trans = torch.from_numpy((10 * rng.standard_normal((B, T, L, 3))).astype(np.float32))
    ang = rng.uniform(-np.pi, np.pi, (B, T, L, 7))
    tors = torch.from_numpy(np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32))
    batch = dict(rots=rots, trans=trans, torsions=tors, torsion_mask=torch.ones(B, L, 7), mask=torch.ones(B, L),
                 seqres=torch.zeros(B, L, dtype=torch.int64))
    for tps in (False, True):
        a = _args(["--tps_condition"] if tps else [])
        a.sim_condition = not tps
        w = NewMDGenWrapper(a)
        ref = w.prep_batch(batch)["latents"].numpy()
        got = w.prep_batch({k: x.cuda() for k, x in batch.items()})["latents"].cpu().numpy()
        err = np.abs(got - ref)
        # a real part within rounding of 0 may take either sign in both solvers
        amb = np.zeros_like(err, dtype=bool)
        for blk in range(2 if tps else 1):
            w0 = np.abs(ref[..., 7 * blk:7 * blk + 1]) < 1e-4
            amb[..., 7 * blk:7 * blk + 4] |= w0
        assert err[~amb].max() <= 2e-5, err[~amb].max()
        np.testing.assert_allclose(np.abs(got[amb]), np.abs(ref[amb]), atol=2e-4)
