"""mdg_latents_to_atom14 (HIP) against the reference's own rollout geometry
(tests/golden/geometry.npz) and the torch restatement; the GPU rollout entry end to end."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from mdgen_finetune_amd import _lib

    _lib.load()


def test_latents_to_atom14_hip_matches_reference_golden(golden):
    from mdgen_finetune_amd import geometry as G

    d, _ = golden("geometry")
    s = torch.from_numpy(d["in_samples"]).cuda()
    aa = torch.from_numpy(d["in_aatype"]).cuda()
    atom14, fr, ft = G.latents_to_atom14_hip(s, torch.from_numpy(d["in_rots0"]).cuda(),
                                             torch.from_numpy(d["in_trans0"]).cuda(), aa, want_frames=True)
    np.testing.assert_allclose(fr.cpu().numpy(), d["out_frame_rots"], atol=2e-6)
    np.testing.assert_allclose(ft.cpu().numpy(), d["out_frame_trans"], atol=2e-5)
    np.testing.assert_allclose(atom14.cpu().numpy(), d["out_atom14"], atol=5e-5)


def test_latents_to_atom14_hip_every_residue_type_and_tps_layout():
    from mdgen_finetune_amd import geometry as G

    g = torch.Generator().manual_seed(0)
    B, T, L = 2, 33, 21
    for tps in (False, True):
        s = torch.randn(B, T, L, 28 if tps else 21, generator=g)
        s[..., 4:7] *= 4
        r0 = G.atom14_to_frames(torch.randn(B, L, 14, 3, generator=g) * 3)
        aa = torch.arange(21).repeat(B, 1)  # all 20 types + X
        rots, trans, tors = G.latents_to_frames_torsions(s, r0.get_rots().get_rot_mats(), r0.get_trans(), tps=tps)
        ref = G.frames_torsions_to_atom14(rots, trans, tors, aa[:, None].expand(B, T, L))
        got = G.latents_to_atom14_hip(s.cuda(), r0.get_rots().get_rot_mats().cuda(), r0.get_trans().cuda(),
                                      aa.cuda(), tps=tps)
        np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), atol=1e-4)


def test_sim_inference_rollout_gpu(tmp_path):
    from mdgen_finetune_amd.sim_inference import main
    from tests.test_geometry import _small_ckpt

    ck = _small_ckpt(tmp_path, T=8)
    main(["--sim_ckpt", ck, "--synthetic", "AKDW", "--num_frames", "8", "--num_rollouts", "3", "--batch", "2",
          "--out_dir", str(tmp_path / "out")])
    txt = (tmp_path / "out" / "AKDW_1.pdb").read_text()
    assert txt.count("ENDMDL") == 24 and "nan" not in txt.lower()
