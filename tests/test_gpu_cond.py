"""GPU parity of the conditioning precompute (mdg_precompute_cond): t-embedding, every adaLN
modulation and the IPA prepend (run_ipa, latent_model.py:179-214; IPALayer 341-394;
InvariantPointAttention ipa.py:92-255), all in fp32 HIP kernels.

  * against the reference's own IPA output captured in the golden vectors (out_ipa), sim and
    TPS, small and full dims, padded residues;
  * against the eager fp32 torch modules of the same model at S > 1 time points (adaLN rows,
    FinalLayer rows, IPA) and at the ATLAS residue count (L = 256, the MFMA attention route);
  * the device TPS relative frames (mdg_tps_rel7) against the reference's 7-vectors: the
    translation exactly and the quaternion up to the eigenvector sign LAPACK leaves free.
Tolerance: max |d| <= 2e-4 * max(1, max |ref|) (fp32 arithmetic in a different order)."""
import numpy as np
import pytest
import torch

from tests.conftest import build_model, load_golden

pytestmark = pytest.mark.gpu

TOL = 2e-4


@pytest.fixture(autouse=True)
def _fp32_matmul():
    """eager references in true fp32 (the training entry sets 'medium' process-wide)"""
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    yield
    torch.set_float32_matmul_precision(old)


def _close(out, ref, tol=TOL, what=""):
    out, ref = out.detach().float().cpu(), ref.detach().float().cpu()
    err = (out - ref).abs().max().item()
    bound = tol * max(1.0, ref.abs().max().item())
    assert err <= bound, f"{what}: max|d| = {err:.3e} > {bound:.3e}"
    return err


def _frames(d, dev, key="rots", tkey="trans"):
    return torch.from_numpy(d["in_" + key]).to(dev).contiguous(), torch.from_numpy(d["in_" + tkey]).to(dev).contiguous()


@pytest.mark.parametrize("name", ["small_sim_T8", "small_sim_pad", "small_tps_T8", "full_sim_T64", "full_tps_T100"])
def test_ipa_prepend_matches_reference_golden(name):
    from mdgen_finetune_amd.engine import get_engine

    d, cfg = load_golden(name)
    m, _ = build_model(cfg, "cuda", T=d["in_x"].shape[1])
    eng = get_engine(m)
    dev = torch.device("cuda")
    rots, trans = _frames(d, dev)
    erots, etrans = _frames(d, dev, "end_rots", "end_trans")
    if m.tps:  # the reference's eigenvector signs (LAPACK) -- see the rel7 test below
        eng.rel7_override = (torch.from_numpy(d["out_rel7_f"]), torch.from_numpy(d["out_rel7_r"]))
    eng._prepare_tps(rots, trans, erots, etrans)
    mask = torch.from_numpy(d["in_mask"]).to(dev).float().contiguous()
    t = torch.from_numpy(d["in_t"]).to(dev).float().reshape(1, -1).contiguous()
    aa = torch.from_numpy(d["in_aatype"]).to(dev).long().contiguous()
    with torch.no_grad():
        mods, mods_f, ipa = eng.conditioning(t, mask, rots, trans, erots if m.tps else None,
                                             etrans if m.tps else None, aa)
    torch.cuda.synchronize()
    _close(ipa[0], torch.from_numpy(d["out_ipa"]), what=f"{name} ipa")


@pytest.mark.parametrize("L,n_pad,S", [(4, 0, 3), (6, 2, 2), (256, 51, 2)])
def test_conditioning_matches_eager_modules(L, n_pad, S):
    """S time points at once vs the eager fp32 modules evaluated per time point."""
    from mdgen_finetune_amd.engine import get_engine
    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    d, cfg = load_golden("full_sim_T1")
    cfg = dict(cfg, L=L)
    m, _ = build_model(cfg, "cuda", T=2)
    eng = get_engine(m)
    g = torch.Generator().manual_seed(7 + L)
    B = 2
    q = torch.randn(B, L, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    from mdgen_finetune_amd.rigid_utils import quat_to_rot

    rots = quat_to_rot(q).cuda().contiguous()
    trans = (5 * torch.randn(B, L, 3, generator=g)).cuda().contiguous()
    mask = torch.ones(B, 2, L)
    if n_pad:
        mask[:, :, L - n_pad:] = 0
    mask = mask.cuda().contiguous()
    aa = torch.randint(0, 20, (B, L), generator=g).cuda()
    t_sb = torch.rand(S, B, generator=g).cuda().contiguous()
    with torch.no_grad():
        mods, mods_f, ipa = eng.conditioning(t_sb, mask, rots, trans, None, None, aa)
        torch.cuda.synchronize()
        frames = Rigid(Rotation(rot_mats=rots), trans)
        for s in range(S):
            c = m.embed_time(t_sb[s])
            for i, layer in enumerate(m.layers):
                _close(mods[s, i], layer.adaLN_modulation(c), what=f"L={L} s={s} layer {i} adaLN")
            _close(mods_f[s], m.emb_to_latent.adaLN_modulation(c), what=f"L={L} s={s} final adaLN")
            ref = m.run_ipa(c, mask[:, 0], frames, None, aa)
            _close(ipa[s], ref, what=f"L={L} s={s} ipa")


@pytest.mark.parametrize("name", ["small_tps_T8", "full_tps_T100"])
def test_device_tps_rel7_matches_reference_up_to_eigen_sign(name):
    import ctypes  # noqa: F401

    from mdgen_finetune_amd import _lib

    d, _ = load_golden(name)
    dev = torch.device("cuda")
    rots, trans = _frames(d, dev)
    erots, etrans = _frames(d, dev, "end_rots", "end_trans")
    B, L = rots.shape[:2]
    out = torch.empty(2, B, L, 7, device=dev)
    lib = _lib.load()
    _lib.check(lib.mdg_tps_rel7(B, L, rots.data_ptr(), trans.data_ptr(), erots.data_ptr(), etrans.data_ptr(),
                                out.data_ptr(), _lib.stream_handle()), "mdg_tps_rel7")
    torch.cuda.synchronize()
    out = out.cpu()
    for k, key in enumerate(("out_rel7_f", "out_rel7_r")):
        ref = torch.from_numpy(d[key])
        _close(out[k, ..., 4:], ref[..., 4:], 1e-5, f"{name} {key} translation")
        sign = torch.where(ref[..., :1] < 0, -1.0, 1.0)
        _close(out[k, ..., :4], ref[..., :4] * sign, 1e-5, f"{name} {key} quaternion (w >= 0)")
        assert (out[k, ..., 0] >= 0).all()


def test_tps_window_with_device_rel7_matches_sign_fixed_oracle(monkeypatch):
    """The TPS sampler path with the device relative frames (MDG_TPS_REL7=device, no override)
    equals the same window computed with the reference's 7-vectors sign-fixed to w >= 0."""
    from mdgen_finetune_amd.engine import get_engine

    monkeypatch.setenv("MDG_TPS_REL7", "device")
    d, cfg = load_golden("small_tps_T8")
    m, _ = build_model(cfg, "cuda", T=8)
    eng = get_engine(m)
    m.hip_dtype = "f32"
    eng = get_engine(m)
    dev = torch.device("cuda")
    rots, trans = _frames(d, dev)
    erots, etrans = _frames(d, dev, "end_rots", "end_trans")
    mask = torch.from_numpy(d["in_mask"]).to(dev).float().contiguous()
    aa = torch.from_numpy(d["in_aatype"]).to(dev).long()
    t = torch.from_numpy(d["in_t"]).to(dev).float().reshape(1, -1).contiguous()

    def fixed(key):
        r = torch.from_numpy(d[key]).clone()
        r[..., :4] *= torch.where(r[..., :1] < 0, -1.0, 1.0)
        return r

    with torch.no_grad():
        eng.rel7_override = None
        eng._prepare_tps(rots, trans, erots, etrans)
        _, _, ipa_dev = eng.conditioning(t, mask, rots, trans, erots, etrans, aa)
        eng.rel7_override = (fixed("out_rel7_f"), fixed("out_rel7_r"))
        eng._prepare_tps(rots, trans, erots, etrans)
        _, _, ipa_fix = eng.conditioning(t, mask, rots, trans, erots, etrans, aa)
        eng.rel7_override = None
    torch.cuda.synchronize()
    _close(ipa_dev, ipa_fix, 1e-4, "tps ipa: device rel7 vs sign-fixed reference rel7")
    assert np.isfinite(ipa_dev.cpu().numpy()).all()


def test_tps_default_engine_conditions_like_training_path():
    """No override, default environment: the HIP engine's TPS forward stages the relative frames
    from relative_tensor7 (the host eigen-solve the training / eager path uses), so it equals the
    eager torch-backend forward of the same module (f32 tolerance) — sampling conditions exactly
    as training did (one sign convention)."""
    import os

    from mdgen_finetune_amd.rigid_utils import Rigid, Rotation

    assert os.environ.get("MDG_TPS_REL7") is None
    d, cfg = load_golden("small_tps_T8")
    m, _ = build_model(cfg, "cuda", T=8)
    m.hip_dtype = "f32"
    dev = torch.device("cuda")
    f = lambda k: torch.from_numpy(d["in_" + k]).to(dev)  # noqa: E731
    kw = dict(mask=f("mask"), start_frames=Rigid(Rotation(rot_mats=f("rots")), f("trans")),
              end_frames=Rigid(Rotation(rot_mats=f("end_rots")), f("end_trans")), x_cond=f("x_cond"),
              x_cond_mask=f("x_cond_mask"), aatype=f("aatype"))
    with torch.no_grad():
        v_hip = m(f("x"), f("t"), **kw)
        m.backend = "torch"
        v_eager = m(f("x"), f("t"), **kw)
        m.backend = "hip"
    _close(v_hip, v_eager, 1e-4, "tps forward: HIP engine (default rel7) vs eager torch backend")
