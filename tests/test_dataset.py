"""MDGenDataset (dataset.py:11-123, restated in mdgen_finetune_amd/data.py) over small atom14
``.npy`` trajectories written here from known frames and torsions: the item's frames and
torsions must be the ones the atoms were built from, the window / frame_interval / copy_frames /
ATLAS crop and pad semantics must hold, and train.py must train on it without --synthetic."""
import argparse
import os

import numpy as np
import pytest
import torch

from mdgen_finetune_amd import geometry as G
from mdgen_finetune_amd.data import RESTYPES, MDGenDataset, SyntheticMDDataset


def _write_peptide(path, seqres, F, seed):
    """An atom14 trajectory [F, L, 14, 3] (Å) built from synthetic frames + torsions."""
    L = len(seqres)
    it = SyntheticMDDataset(F, L, size=1, seed=seed)[0]
    aa = torch.tensor([RESTYPES.index(c) for c in seqres])
    tors = it["torsions"]  # (sin, cos), as the geometry and MDGenDataset take them
    atom14 = G.frames_torsions_to_atom14(it["rots"], it["trans"], tors, aa[None].expand(F, L))
    np.save(path, atom14.numpy().astype(np.float32))
    return it["rots"], it["trans"], tors


def _args(data_dir, **kw):
    a = dict(data_dir=str(data_dir), suffix="", num_frames=6, crop=4, atlas=False, frame_interval=None,
             overfit=False, overfit_peptide=None, overfit_frame=False, copy_frames=False, no_frames=False)
    a.update(kw)
    return argparse.Namespace(**a)


@pytest.fixture
def data(tmp_path):
    peps = {"AKLG": 20, "WDEY": 24, "MHRS": 18}
    truth = {}
    for i, (s, F) in enumerate(peps.items()):
        truth[s] = _write_peptide(tmp_path / f"{s}.npy", s, F, seed=50 + i)
    with open(tmp_path / "split.csv", "w") as f:
        f.write("name,seqres\n")
        for s in list(peps) + ["NOFILE"]:
            f.write(f"{s},{s if s != 'NOFILE' else 'AAAA'}\n")
    return tmp_path, truth


def test_items_recover_the_frames_and_torsions(data):
    d, truth = data
    ds = MDGenDataset(_args(d), str(d / "split.csv"), rng=np.random.default_rng(0))
    assert list(ds.df.index) == ["AKLG", "WDEY", "MHRS"]  # the row without a file is dropped
    assert len(ds) == 3
    for idx in range(3):
        it = ds[idx]
        name = it["name"]
        rots, trans, tors = truth[name]
        fs = it["frame_start"]
        assert 0 <= fs < rots.shape[0] - 6
        sl = slice(fs, fs + 6)
        assert it["rots"].shape == (6, 4, 3, 3) and it["trans"].shape == (6, 4, 3)
        np.testing.assert_allclose(it["rots"].numpy(), rots[sl].numpy(), atol=2e-5)
        np.testing.assert_allclose(it["trans"].numpy(), trans[sl].numpy(), atol=2e-4)
        m = it["torsion_mask"].bool()
        assert it["torsions"].shape == (6, 4, 7, 2) and m.shape == (4, 7)
        assert not m[0, 0] and not m[0, 1] and m[1:, :3].all()  # residue 0 has no omega / phi
        # psi and the chis place atoms (O, side chains), so they come back; omega / phi follow
        # from the frames' geometry, not from the input angles
        m[:, :2] = False
        got, want = it["torsions"][:, m], tors[sl][:, m]
        want = want / want.norm(dim=-1, keepdim=True)
        np.testing.assert_allclose(got.numpy(), want.numpy(), atol=2e-4)
        assert it["seqres"].tolist() == [RESTYPES.index(c) for c in name]
        assert it["mask"].tolist() == [1.0] * 4


def test_window_options(data):
    d, truth = data
    a = _args(d, frame_interval=2, overfit_frame=True, copy_frames=True)
    it = MDGenDataset(a, str(d / "split.csv"), rng=np.random.default_rng(1))[0]
    rots = truth["AKLG"][0]
    assert it["frame_start"] == 0
    for t in range(6):  # copy_frames: every frame is the window's first (frame 0 of the stride)
        np.testing.assert_allclose(it["rots"][t].numpy(), rots[0].numpy(), atol=2e-5)
    a = _args(d, overfit=True)
    ds = MDGenDataset(a, str(d / "split.csv"), rng=np.random.default_rng(2))
    assert {ds[i]["name"] for i in range(3)} == {"AKLG"}
    a = _args(d, overfit_peptide="WDEY")
    ds = MDGenDataset(a, str(d / "split.csv"), rng=np.random.default_rng(3))
    assert len(ds) == 1000 and ds[17]["name"] == "WDEY"
    a = _args(d, num_frames=40)
    with pytest.raises(ValueError):
        MDGenDataset(a, str(d / "split.csv"), rng=np.random.default_rng(4))[0]


def test_atlas_crop_and_pad(tmp_path):
    _write_peptide(tmp_path / "PEPTIDEA_R2.npy", "PEPTIDEA", 12, seed=9)
    _write_peptide(tmp_path / "GG_R1.npy", "GG", 12, seed=10)
    with open(tmp_path / "split.csv", "w") as f:
        f.write("name,seqres\nPEPTIDEA,PEPTIDEA\nGG,GG\n")
    rng = np.random.default_rng(5)
    a = _args(tmp_path, atlas=True, crop=4)
    # replicas are drawn from _R1.._R3: serve whichever file exists by retrying the draw
    ds = MDGenDataset(a, str(tmp_path / "split.csv"), rng=rng)
    assert len(ds.df) == 2
    seen = set()
    for _ in range(40):
        for i in range(2):
            try:
                it = ds[i]
            except FileNotFoundError:
                continue
            seen.add(it["name"])
            assert it["rots"].shape == (6, 4, 3, 3) and it["torsions"].shape == (6, 4, 7, 2)
            if it["name"] == "GG_R1":  # padded: 2 residues + 2 identity frames
                assert it["mask"].tolist() == [1, 1, 0, 0]
                assert it["seqres"].tolist()[2:] == [0, 0]
                assert torch.equal(it["rots"][:, 2:], torch.eye(3).expand(6, 2, 3, 3))
                assert float(it["trans"][:, 2:].abs().max()) == 0 and float(it["torsion_mask"][2:].abs().max()) == 0
            else:  # cropped: 4 consecutive residues of 8
                assert it["mask"].tolist() == [1, 1, 1, 1]
                seq = "".join(RESTYPES[j] for j in it["seqres"].tolist())
                assert seq in "PEPTIDEA"
    assert seen == {"PEPTIDEA_R2", "GG_R1"}


def test_trainer_trains_on_npy_dataset(data, tmp_path_factory):
    from mdgen_finetune_amd.parsing import parse_train_args
    from mdgen_finetune_amd.train import Trainer

    d, _ = data
    out = tmp_path_factory.mktemp("model")
    argv = ["--train_split", str(d / "split.csv"), "--val_split", str(d / "split.csv"), "--data_dir", str(d),
            "--sim_condition", "--prepend_ipa", "--abs_pos_emb", "--num_frames", "6", "--crop", "4",
            "--embed_dim", "32", "--mha_heads", "4", "--num_layers", "2", "--ipa_heads", "2", "--ipa_head_dim", "8",
            "--ipa_qk", "4", "--ipa_v", "4", "--batch_size", "1", "--print_freq", "1000", "--epochs", "2",
            "--num_workers", "0", "--val_batches", "2", "--model_dir", str(out)]
    a = parse_train_args(argv)
    tr = Trainer(a)
    assert isinstance(tr.dataset, MDGenDataset) and tr.val_loader is not None
    vals = []
    orig = tr.print_log
    def spy(prefix="iter"):
        m = orig(prefix)
        vals.append((prefix, m))
        return m

    tr.print_log = spy
    tr.fit()
    assert tr.global_step == 6  # 3 peptides x 2 epochs at batch 1
    val_logs = [m for p, m in vals if p == "val"]
    assert len(val_logs) == 2 and all(np.isfinite(m["val_loss"]) for m in val_logs)
    assert sorted(os.listdir(out))  # checkpoints written
