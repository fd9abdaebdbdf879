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


def _rollout_both(tmp_path, tps, n_windows=2, T=8, B=2):
    """The same multi-window rollout (sim) or batch of transition paths (tps) on the HIP path
    (f32 operands) and on the eager CPU backend, fed identical prior noise per window.

    Every window starts both sides from the SAME start batch (the CPU side's restart state,
    built on the CPU and copied to the device): a rollout is chaotic in its inputs (the
    restart re-derives frames and torsions from atoms, and the first residue's pre-omega
    torsion is degenerate; the TPS branch embeds an eigenvector quaternion whose sign flips
    with 1-ulp input changes, rigid_utils.py:191-210), so comparing two free-running rollouts
    measures that chaos, not the kernels.  The restart itself is compared separately: the
    device restart of the CPU window's atoms against the CPU restart (valid torsions only)."""
    from mdgen_finetune_amd.checkpoint import load_from_checkpoint
    from mdgen_finetune_amd.data import SyntheticMDDataset
    from mdgen_finetune_amd.sim_inference import rollout, seq_to_aatype
    from tests.test_geometry import _small_ckpt

    ck = _small_ckpt(tmp_path, T=T, tps=tps)
    lat = 28 if tps else 21
    g = torch.Generator().manual_seed(11)
    zs = [torch.randn(B, T, 4, lat, generator=g) for _ in range(n_windows)]
    w = {}
    for dev in ("cuda", "cpu"):
        w[dev] = load_from_checkpoint(ck).eval().to(dev)
        if dev == "cpu":
            w[dev].model.backend = "torch"
        else:
            w[dev].model.hip_dtype = "f32"
    outs = {"cuda": [], "cpu": [], "restart": []}
    if tps:
        import numpy as np

        from mdgen_finetune_amd.tps_inference import _synthetic_traj, collate_samples, get_sample

        arr, aat = _synthetic_traj("AKDW", 32, 4)
        rng = np.random.RandomState(0)
        batch = collate_samples([get_sample(arr, aat, [0, 3], [20, 30], num_frames=T, rng=rng) for _ in range(B)])
        for dev in ("cuda", "cpu"):
            with torch.no_grad():
                outs[dev].append(w[dev].inference({k: v.to(dev) for k, v in batch.items()}, zs0=zs[0].to(dev))[0].cpu())
        return outs
    it = SyntheticMDDataset(1, 4, size=1, seed=2)[0]
    batch = {"torsions": it["torsions"][None], "torsion_mask": it["torsion_mask"][None], "trans": it["trans"][None],
             "rots": it["rots"][None], "seqres": seq_to_aatype("AKDW")[None], "mask": torch.ones(1, 4)}
    for k in range(n_windows):
        res = {}
        for dev in ("cuda", "cpu"):
            with torch.no_grad():
                res[dev] = rollout(w[dev], {kk: v.to(dev) for kk, v in batch.items()}, T, B, zs0=zs[k].to(dev))
            outs[dev].append(res[dev][0].cpu())
        # the restart of the CPU window's last frame, on the device vs on the CPU
        from mdgen_finetune_amd import geometry as G

        last = res["cpu"][0][:, -1]
        nb = res["cpu"][1]
        fr = G.atom14_to_frames(last.cuda())
        a37 = G.atom14_to_atom37(last.cuda(), nb["seqres"].cuda())
        tors, tmask = G.atom37_to_torsions(a37, nb["seqres"].cuda())
        outs["restart"].append(((fr.get_trans().cpu() - nb["trans"][:, 0]).abs().max().item(),
                                (fr.get_rots().get_rot_mats().cpu() - nb["rots"][:, 0]).abs().max().item(),
                                ((tors.cpu() - nb["torsions"][:, 0]) * tmask.cpu()[..., None]).abs().max().item()))
        batch = {kk: v.cpu() for kk, v in nb.items()}
    return outs


def test_sim_rollout_three_windows_hip_matches_cpu_eager(tmp_path):
    """sim_inference.py:65-112 over 3 windows (window k+1 restarts from window k's last frame:
    atom14 -> frames, atom37 -> torsions).  Per window, HIP (f32) vs the eager CPU backend from
    the same start state and noise: atom14 within 2e-3 Å; the device restart of a window's last
    frame vs the CPU restart: frames within 1e-4, valid torsions within 1e-4."""
    outs = _rollout_both(tmp_path, tps=False, n_windows=3)
    for k, (a, b) in enumerate(zip(outs["cuda"], outs["cpu"])):
        err = (a - b).abs().max().item()
        assert err <= 2e-3, (k, err)
    for k, (et, er, etor) in enumerate(outs["restart"]):
        assert et <= 1e-4 and er <= 1e-4 and etor <= 1e-4, (k, et, er, etor)


def test_tps_inference_batch_hip_matches_cpu_eager(tmp_path, monkeypatch):
    """tps_inference.py:119-131: a batch of transition-path windows (frames 0 and T-1
    conditioned, latent 28) on HIP (f32) vs eager CPU with identical noise and start / end
    frames built once on the CPU.  The HIP engine takes the relative frames' quaternion sign
    from the host eigen-solve here (MDG_TPS_REL7=host), as the eager CPU path does; its default
    device frames fix the sign to w >= 0 (tests/test_gpu_cond.py)."""
    monkeypatch.setenv("MDG_TPS_REL7", "host")
    outs = _rollout_both(tmp_path, tps=True, n_windows=1)
    err = (outs["cuda"][0] - outs["cpu"][0]).abs().max().item()
    assert err <= 2e-3, err


@pytest.mark.parametrize("dtype,tol", [("f32", 1e-3), ("bf16", 5e-2)])
def test_peptides_per_window_equals_serial_gpu(tmp_path, dtype, tol):
    """sim_inference --peptides_per_window on the HIP engine: 4 tetrapeptides rolled out in one
    window (8 rows) against one window each (2 rows, the reference's serial loop): every
    peptide's atoms agree (same per-peptide noise; the kernels' plans differ with the row count,
    so equal up to their rounding), and the restart batches agree too."""
    from mdgen_finetune_amd.checkpoint import load_from_checkpoint
    from mdgen_finetune_amd.data import SyntheticMDDataset
    from mdgen_finetune_amd.sim_inference import peptide_generator, rollout_group, seq_to_aatype
    from tests.test_geometry import _small_ckpt

    ck = _small_ckpt(tmp_path, T=8)
    w = load_from_checkpoint(ck).eval().cuda()
    w.model.hip_dtype = dtype
    jobs = []
    for k, seq in enumerate(["AKDW", "GLYW", "MPEV", "AKDW"]):
        it = SyntheticMDDataset(1, 4, size=1, seed=k)[0]
        b = {"torsions": it["torsions"][None], "torsion_mask": it["torsion_mask"][None], "trans": it["trans"][None],
             "rots": it["rots"][None], "seqres": seq_to_aatype(seq)[None], "mask": torch.ones(1, 4)}
        jobs.append((f"p{k}", {key: v.cuda() for key, v in b.items()}))

    def go(K):
        out = {}
        gens = [(n, b, peptide_generator(0, i, torch.device("cuda"))) for i, (n, b) in enumerate(jobs)]
        with torch.no_grad():
            for g0 in range(0, len(gens), K):
                for name, traj, last in rollout_group(w, gens[g0:g0 + K], 8, 1, 2, 21):
                    out[name] = (traj, last)
        return out

    serial, batched = go(1), go(4)
    for name in serial:
        a, b = serial[name][0], batched[name][0]
        assert a.shape == b.shape == (2, 8, 4, 14, 3)
        assert torch.isfinite(b).all()
        assert float((a - b).abs().max()) <= tol, (name, float((a - b).abs().max()))
        for key in ("trans", "rots"):
            assert float((serial[name][1][key] - batched[name][1][key]).abs().max()) <= tol
    assert float((batched["p0"][0] - batched["p3"][0]).abs().max()) > 0.1  # same sequence, own frames / noise
