"""Generate golden vectors by running the REFERENCE model (container-only test infrastructure).

Run in the build container only (it imports /root/reference/src, which does not exist on the
GPU box).  Output: small .npz fixtures under tests/golden/ (inputs + reference outputs; the
weights are NOT stored — they are regenerated from a seed by mdgen_finetune_amd.synthetic,
which is how both the oracle restatement and the HIP path get identical weights).

What is run (reference file:line):
  * LatentMDGenModel.forward            latent_model.py:216-269 — verbatim, with ONE
    substitution: run_ipa receives mask[:, 0] instead of mask.reshape(-1, L)
    (latent_model.py:255).  The unmodified line is shape-invalid for num_frames > 1
    (SURVEY §0.3); at T == 1 the substitution is checked here to be bit-identical.
  * Sampler.sample_ode('euler', 50)      transport.py:407-450, integrators.py:95-114
  * Transport.training_losses (GVP)      transport.py:137-222 (RNG order x0 then t, :131-133)
  * MultiheadAttention (rope + bias_kv)  mha.py:161-407 (unit case)

Third-party modules the reference imports but the container lacks are replaced by the
test-only shims in oracle/shim/ (see its README; fair-esm rotary and torchdiffeq Euler are
restated there — parity to the real packages is unpinned).

Usage:  python oracle/gen_golden.py      (writes tests/golden/*.npz, ~1 min on 8 cores)
"""
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/src")
sys.path.insert(0, os.path.join(HERE, "shim"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mdgen_finetune_amd import synthetic  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")

SMALL = ["--embed_dim", "64", "--mha_heads", "4", "--ipa_heads", "2", "--ipa_head_dim", "8",
         "--ipa_qk", "4", "--ipa_v", "4", "--num_layers", "2"]


def make_args(extra):
    from mdgen.parsing import parse_train_args

    argv = sys.argv
    sys.argv = ["train", "--train_split", "x", "--val_split", "x", "--data_dir", "x"] + extra
    try:
        args = parse_train_args()
    finally:
        sys.argv = argv
    # NewMDGenWrapper backfills these (wrapper.py:178-194)
    for key in ["inpainting", "no_torsion", "hyena", "no_aa_emb", "supervise_all_torsions",
                "supervise_no_torsions", "design_key_frames", "no_design_torsion",
                "cond_interval", "mpnn", "dynamic_mpnn", "no_offsets", "no_frames"]:
        if not hasattr(args, key):
            setattr(args, key, False)
    return args


def build_model(args, latent_dim, seed):
    from mdgen.model.latent_model import LatentMDGenModel

    torch.manual_seed(0)
    model = LatentMDGenModel(args, latent_dim).eval()
    synthetic.fill_module_(model, seed)
    return model


def patch_ipa(model, capture):
    orig = model.run_ipa

    def run_ipa(t, mask2d, start_frames, end_frames, aatype, x_d=None):
        B = t.shape[0]
        mask_b = mask2d.reshape(B, -1, mask2d.shape[-1])[:, 0]
        out = orig(t, mask_b, start_frames, end_frames, aatype, x_d=x_d)
        capture["ipa"] = out.detach().clone()
        return out

    model.run_ipa = run_ipa
    return orig


def kwargs_from(inp):
    from mdgen.rigid_utils import Rigid, Rotation

    sf = Rigid(trans=torch.from_numpy(inp["trans"]), rots=Rotation(rot_mats=torch.from_numpy(inp["rots"])))
    ef = Rigid(trans=torch.from_numpy(inp["end_trans"]),
               rots=Rotation(rot_mats=torch.from_numpy(inp["end_rots"])))
    return dict(start_frames=sf, end_frames=ef, mask=torch.from_numpy(inp["mask"]),
                x_cond=torch.from_numpy(inp["x_cond"]),
                x_cond_mask=torch.from_numpy(inp["x_cond_mask"]),
                aatype=torch.from_numpy(inp["aatype"]))


def save(name, cfg, inp, out):
    os.makedirs(OUT, exist_ok=True)
    arrs = {f"in_{k}": v for k, v in inp.items()}
    arrs.update({f"out_{k}": (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in out.items()})
    arrs["config"] = np.array(json.dumps(cfg))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **arrs)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def forward_case(name, flags, latent_dim, B, T, L, seed, tps=False, n_pad=0, euler=False,
                 intermediates=False):
    args = make_args(flags + ["--num_frames", str(T), "--crop", str(L), "--prepend_ipa",
                              "--abs_pos_emb", "--sampling_method", "euler"]
                     + (["--tps_condition"] if tps else ["--sim_condition"]))
    model = build_model(args, latent_dim, seed)
    inp = synthetic.make_inputs(seed + 1, B, T, L, latent_dim, tps=tps, n_pad=n_pad)
    kw = kwargs_from(inp)
    x = torch.from_numpy(inp["x"])
    t = torch.from_numpy(inp["t"])
    cap = {}
    layer_out = []
    hooks = []
    if intermediates:
        for layer in model.layers:
            hooks.append(layer.register_forward_hook(lambda m, a, o: layer_out.append(o.detach().clone())))
    with torch.no_grad():
        if T == 1:  # the substitution is exact where the fork's own forward runs
            v_unpatched = model(x, t, **kw)
            layer_out.clear()
        orig = patch_ipa(model, cap)
        v = model(x, t, **kw)
        if T == 1:
            assert torch.equal(v, v_unpatched), "mask[:,0] substitution differs at T == 1"
            print(f"  {name}: T==1 bit-equal to the unmodified reference forward()")
    for h in hooks:
        h.remove()
    out = {"v": v, "ipa": cap["ipa"]}
    if tps:  # the relative-frame 7-vectors the TPS branch embeds (latent_model.py:198-199); their
        # quaternion half comes from an eigen-solve whose sign depends on the LAPACK build, so
        # parity on another host injects these exact values
        out["rel7_f"] = kw["start_frames"].invert().compose(kw["end_frames"]).to_tensor_7()
        out["rel7_r"] = kw["end_frames"].invert().compose(kw["start_frames"]).to_tensor_7()
    for i, o in enumerate(layer_out):
        out[f"layer{i}"] = o
    if euler:
        from mdgen.transport.transport import create_transport, Sampler
        from functools import partial

        transport = create_transport(args, args.path_type, args.prediction, None, None, None)
        sampler = Sampler(transport)
        rng = np.random.default_rng(seed + 2)
        zs = torch.from_numpy(rng.standard_normal(x.shape).astype(np.float32))
        inp["zs"] = zs.numpy()
        with torch.no_grad():
            samples = sampler.sample_ode(sampling_method="euler")(
                zs, partial(model.forward_inference, **kw))
        out["euler_step1"] = samples[1]
        out["euler_final"] = samples[-1]
        out["euler_n"] = np.array(samples.shape[0])
    cfg = dict(name=name, flags=flags, latent_dim=latent_dim, B=B, T=T, L=L, seed=seed, tps=tps,
               n_pad=n_pad, weights_seed=seed, inputs_seed=seed + 1)
    save(name, cfg, inp, out)
    model.run_ipa = orig


def loss_case(name, flags, B, T, L, seed):
    from mdgen.transport.transport import create_transport

    args = make_args(flags + ["--num_frames", str(T), "--crop", str(L), "--prepend_ipa",
                              "--abs_pos_emb", "--sim_condition"])
    model = build_model(args, 21, seed)
    inp = synthetic.make_inputs(seed + 1, B, T, L, 21)
    kw = kwargs_from(inp)
    patch_ipa(model, {})
    transport = create_transport(args, args.path_type, args.prediction, None, None, None)
    x1 = torch.from_numpy(inp["x"])
    loss_mask = torch.ones(B, T, L, 21)
    loss_mask[:, :, :, 7:] = torch.from_numpy(
        (np.random.default_rng(seed + 3).uniform(size=(B, 1, L, 14)) > 0.3).astype(np.float32))
    # the RNG draws of Transport.sample (transport.py:131-133): x0 = randn_like(x1), then t
    torch.manual_seed(1234)
    x0 = torch.randn_like(x1)
    tt = torch.rand((B,))
    torch.manual_seed(1234)
    with torch.no_grad():
        terms = transport.training_losses(model, x1, None, loss_mask, kw)
    assert torch.equal(terms["t"], tt)
    inp["x0"] = x0.numpy()
    inp["t_loss"] = tt.numpy()
    inp["loss_mask"] = loss_mask.numpy()
    cfg = dict(name=name, flags=flags, latent_dim=21, B=B, T=T, L=L, seed=seed, tps=False,
               n_pad=0, weights_seed=seed, inputs_seed=seed + 1)
    save(name, cfg, inp, {"loss": terms["loss"], "pred": terms["pred"]})


def mha_case(name, seed):
    from mdgen.model.mha import MultiheadAttention

    torch.manual_seed(0)
    C, H, S, N = 48, 2, 7, 3
    mha = MultiheadAttention(C, H, add_bias_kv=True, use_rotary_embeddings=True).eval()
    synthetic.fill_module_(mha, seed)
    rng = np.random.default_rng(seed + 1)
    x = rng.standard_normal((S, N, C)).astype(np.float32)
    kpm = np.zeros((N, S), np.float32)
    kpm[1, 5:] = 1.0   # two padded keys in sequence 1
    kpm[2, :] = 1.0    # every real key padded: only the bias_k row survives
    with torch.no_grad():
        o, _ = mha(query=torch.from_numpy(x), key=torch.from_numpy(x), value=torch.from_numpy(x),
                   key_padding_mask=torch.from_numpy(kpm))
    cfg = dict(name=name, C=C, H=H, S=S, N=N, seed=seed)
    save(name, cfg, {"x": x, "key_padding_mask": kpm}, {"o": o})


def state_dict_case(name, flags, latent_dim, tps):
    """The reference's full state_dict contract (parameter AND buffer names, shapes)."""
    args = make_args(flags + ["--num_frames", "16", "--crop", "4", "--prepend_ipa", "--abs_pos_emb"]
                     + (["--tps_condition"] if tps else ["--sim_condition"]))
    from mdgen.model.latent_model import LatentMDGenModel

    sd = LatentMDGenModel(args, latent_dim).state_dict()
    keys = np.array(list(sd.keys()))
    shapes = np.array([json.dumps(list(v.shape)) for v in sd.values()])
    save(name, dict(name=name, flags=flags, latent_dim=latent_dim, tps=tps), {}, {"keys": keys, "shapes": shapes})


def prep_batch_case(name, B, T, L, seed):
    """wrapper.py:283-365 on a synthetic trajectory batch.  The offsets come from the
    reference's own get_offsets (utils.py:7-14) on its Rigid/Rotation (rot_to_quat via eigh);
    the remaining glue (sign fix 309, masks 311-350, x_cond 362) is evaluated with the same
    tensor expressions as the reference (wrapper.py is not importable: it needs Lightning)."""
    from mdgen.rigid_utils import Rigid, Rotation
    from mdgen.utils import get_offsets
    from mdgen_finetune_amd.data import SyntheticMDDataset, collate

    ds = SyntheticMDDataset(T, L, size=B, seed=seed, n_pad=1)
    batch = collate([ds[i] for i in range(B)])
    batch["torsion_mask"][0, 0, 3] = 1.0
    inp = {k: batch[k].numpy() for k in ("torsions", "torsion_mask", "trans", "rots", "seqres", "mask")}
    rigids = Rigid(trans=batch["trans"], rots=Rotation(rot_mats=batch["rots"]))
    out = {}
    for tps in (False, True):
        offsets = get_offsets(rigids[:, 0:1], rigids)
        offsets[..., :4] *= torch.where(offsets[:, :, :, 0:1] < 0, -1, 1)
        frame_loss_mask = batch["mask"].unsqueeze(-1).expand(-1, -1, 7)
        torsion_loss_mask = batch["torsion_mask"].unsqueeze(-1).expand(-1, -1, -1, 2).reshape(B, L, 14)
        if tps:
            offsets_r = get_offsets(rigids[:, -1:], rigids)
            offsets_r[..., :4] *= torch.where(offsets_r[:, :, :, 0:1] < 0, -1, 1)
            offsets = torch.cat([offsets, offsets_r], -1)
            frame_loss_mask = torch.cat([frame_loss_mask, frame_loss_mask], -1)
        latents = torch.cat([offsets, batch["torsions"].view(B, T, L, 14)], -1)
        loss_mask = torch.cat([frame_loss_mask, torsion_loss_mask], -1).unsqueeze(1).expand(-1, T, -1, -1)
        cond_mask = torch.zeros(B, T, L, dtype=int)
        cond_mask[:, 0] = 1
        if tps:
            cond_mask[:, -1] = 1
        sfx = "_tps" if tps else ""
        out["latents" + sfx] = latents
        out["loss_mask" + sfx] = loss_mask
        out["cond_mask" + sfx] = cond_mask
    save(name, dict(name=name, B=B, T=T, L=L, seed=seed), inp, out)


def geometry_case(name, B, T, L, seed):
    """Rollout geometry through the reference's own functions: wrapper.py:480-505 (offsets ->
    frames composed on frame 0 via Rigid.from_tensor_7(normalize_quats=True), torsion
    normalisation) + geometry.frames_torsions_to_atom14, atom14_to_frames, atom14_to_atom37,
    atom37_to_torsions, and utils.atom14_to_pdb's multi-model PDB text."""
    import tempfile

    from mdgen.geometry import atom14_to_atom37, atom14_to_frames, atom37_to_torsions, frames_torsions_to_atom14
    from mdgen.rigid_utils import Rigid, Rotation
    from mdgen.utils import atom14_to_pdb
    from mdgen_finetune_amd.data import SyntheticMDDataset

    rng = np.random.default_rng(seed)
    ds = SyntheticMDDataset(1, L, size=B, seed=seed)
    rots0 = torch.stack([ds[i]["rots"][0] for i in range(B)])      # [B,L,3,3]
    trans0 = torch.stack([ds[i]["trans"][0] for i in range(B)])    # [B,L,3]
    samples = torch.from_numpy(rng.standard_normal((B, T, L, 21)).astype(np.float32))
    samples[..., 4:7] *= 3.0
    aatype = torch.from_numpy(rng.integers(0, 20, (B, L)).astype(np.int64))
    ref = Rigid(trans=trans0[:, None], rots=Rotation(rot_mats=rots0[:, None]))
    frames = ref.compose(Rigid.from_tensor_7(samples[..., :7], normalize_quats=True))
    tors = samples[..., 7:21].reshape(B, T, L, 7, 2)
    tors = tors / torch.linalg.norm(tors, dim=-1, keepdims=True)
    atom14 = frames_torsions_to_atom14(frames, tors.view(B, T, L, 7, 2), aatype[:, None].expand(B, T, L))
    last = atom14[:, -1]                                           # [B,L,14,3]
    fr = atom14_to_frames(last)
    atom37 = torch.from_numpy(np.asarray(atom14_to_atom37(last[0].numpy(), aatype[0].numpy()))).float()
    tors37, tmask = atom37_to_torsions(atom37, aatype[0])
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "x.pdb")
        atom14_to_pdb(atom14[0].numpy(), aatype[0].numpy(), path)
        pdb = open(path).read()
    inp = dict(samples=samples.numpy(), rots0=rots0.numpy(), trans0=trans0.numpy(), aatype=aatype.numpy())
    out = dict(atom14=atom14, frame_rots=frames.get_rots().get_rot_mats(), frame_trans=frames.get_trans(),
               last_rots=fr.get_rots().get_rot_mats(), last_trans=fr.get_trans(), atom37=atom37,
               torsions=tors37, torsion_mask=tmask, pdb=np.array(pdb))
    save(name, dict(name=name, B=B, T=T, L=L, seed=seed), inp, out)


def main():
    torch.set_num_threads(8)
    if sys.argv[1:] == ["geometry"]:
        geometry_case("geometry", B=2, T=5, L=6, seed=61)
        return
    if sys.argv[1:] == ["prep_batch"]:
        prep_batch_case("prep_batch", B=2, T=12, L=5, seed=51)
        return
    state_dict_case("state_dict_sim", [], 21, False)
    state_dict_case("state_dict_tps", [], 28, True)
    forward_case("small_sim_T1", SMALL, 21, B=2, T=1, L=4, seed=11, intermediates=True)
    forward_case("small_sim_T8", SMALL, 21, B=2, T=8, L=4, seed=12, intermediates=True, euler=True)
    forward_case("small_sim_pad", SMALL, 21, B=2, T=8, L=8, seed=13, n_pad=2, intermediates=True)
    forward_case("small_tps_T8", SMALL, 28, B=2, T=8, L=4, seed=14, tps=True, intermediates=True)
    forward_case("full_sim_T1", [], 21, B=2, T=1, L=4, seed=21)
    forward_case("full_sim_T64", [], 21, B=1, T=64, L=4, seed=22, euler=True)
    forward_case("full_tps_T100", [], 28, B=1, T=100, L=4, seed=23, tps=True)
    loss_case("small_loss", SMALL, B=3, T=8, L=4, seed=31)
    mha_case("mha_rope_biaskv", seed=41)
    prep_batch_case("prep_batch", B=2, T=12, L=5, seed=51)
    geometry_case("geometry", B=2, T=5, L=6, seed=61)


if __name__ == "__main__":
    main()
