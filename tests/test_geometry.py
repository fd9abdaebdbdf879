"""Rollout geometry (torch restatement) and the PDB writer against the reference's own
geometry.py / utils.atom14_to_pdb outputs (tests/golden/geometry.npz, oracle/gen_golden.py)."""
import numpy as np
import torch


def _g(golden):
    d, _ = golden("geometry")
    return d


def test_latents_to_atom14_matches_reference(golden):
    from mdgen_finetune_amd import geometry as G

    d = _g(golden)
    s = torch.from_numpy(d["in_samples"])
    rots, trans, tors = G.latents_to_frames_torsions(s, torch.from_numpy(d["in_rots0"]),
                                                     torch.from_numpy(d["in_trans0"]))
    np.testing.assert_allclose(rots.numpy(), d["out_frame_rots"], atol=2e-6)
    np.testing.assert_allclose(trans.numpy(), d["out_frame_trans"], atol=2e-5)
    aa = torch.from_numpy(d["in_aatype"])
    B, T, L = s.shape[:3]
    atom14 = G.frames_torsions_to_atom14(rots, trans, tors, aa[:, None].expand(B, T, L))
    np.testing.assert_allclose(atom14.numpy(), d["out_atom14"], atol=5e-5)


def test_inverse_geometry_matches_reference(golden):
    from mdgen_finetune_amd import geometry as G

    d = _g(golden)
    last = torch.from_numpy(d["out_atom14"][:, -1])
    fr = G.atom14_to_frames(last)
    np.testing.assert_allclose(fr.get_rots().get_rot_mats().numpy(), d["out_last_rots"], atol=2e-6)
    np.testing.assert_allclose(fr.get_trans().numpy(), d["out_last_trans"], atol=1e-6)
    aa = torch.from_numpy(d["in_aatype"][0])
    a37 = G.atom14_to_atom37(last[0], aa)
    np.testing.assert_allclose(a37.numpy(), d["out_atom37"], atol=1e-6)
    tors, tmask = G.atom37_to_torsions(a37, aa)
    np.testing.assert_array_equal(tmask.numpy(), d["out_torsion_mask"])
    np.testing.assert_allclose(tors.numpy(), d["out_torsions"], atol=2e-5)


def test_pdb_text_matches_reference_byte_for_byte(golden):
    from mdgen_finetune_amd.pdb import atom14_to_pdb_string

    d = _g(golden)
    txt = atom14_to_pdb_string(d["out_atom14"][0], d["in_aatype"][0])
    assert txt == str(d["out_pdb"])


def _small_ckpt(tmp_path, T=4):
    from mdgen_finetune_amd import synthetic
    from mdgen_finetune_amd.checkpoint import save_checkpoint
    from mdgen_finetune_amd.parsing import parse_train_args
    from mdgen_finetune_amd.wrapper import NewMDGenWrapper

    a = parse_train_args(["--synthetic", "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames", str(T),
                          "--crop", "4", "--embed_dim", "64", "--mha_heads", "4", "--num_layers", "2",
                          "--ipa_heads", "2", "--ipa_head_dim", "8", "--ipa_qk", "4", "--ipa_v", "4",
                          "--sampling_method", "euler", "--model_dir", str(tmp_path)])
    w = NewMDGenWrapper(a)
    synthetic.fill_module_(w.model, 5)
    path = str(tmp_path / "sim.ckpt")
    save_checkpoint(path, w)
    return path


def test_sim_inference_rollout_cpu_writes_multimodel_pdb(tmp_path):
    from mdgen_finetune_amd.sim_inference import main

    ck = _small_ckpt(tmp_path)
    main(["--sim_ckpt", ck, "--synthetic", "AKDW", "--num_frames", "4", "--num_rollouts", "2", "--batch", "2",
          "--out_dir", str(tmp_path / "out")])
    for j in range(2):
        txt = (tmp_path / "out" / f"AKDW_{j}.pdb").read_text()
        assert txt.count("MODEL ") == 8 and txt.count("ENDMDL") == 8
        assert "nan" not in txt.lower()
