"""Diagnostic: ATLAS T x 256 f32 HIP forward vs the oracle, max |d| on valid vs padded residues,
and the IPA prepend (HIP conditioning vs the oracle's IPA) likewise."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import _oracle_full
from tests.conftest import build_model
from mdgen_finetune_amd.rigid_utils import Rigid, Rotation
T = int(sys.argv[1]) if len(sys.argv) > 1 else 250
inp, ref, cfg = _oracle_full(T, seed=23, B=1, n_pad=51, L=256)
g = lambda k: torch.from_numpy(inp[k]).cuda()
valid = inp["mask"][0, 0] > 0
for mode in ("hip", "torchcond"):
    m, _ = build_model(cfg, "cuda", T=T)
    m.hip_dtype = "f32"
    if mode == "torchcond":
        from mdgen_finetune_amd import engine as E
        eng = E.get_engine(m)
        # eager-torch conditioning for comparison
        def cond(t_sb, mask, rots, trans, erots, etrans, aatype, eng=eng, m=m):
            S, B = t_sb.shape
            c = m.embed_time(t_sb.reshape(-1))
            mods = torch.stack([l.adaLN_modulation(c) for l in m.layers], 1).reshape(S, B, m.args.num_layers, -1).permute(0, 2, 1, 3).contiguous()
            mf = m.emb_to_latent.adaLN_modulation(c).reshape(S, B, -1).contiguous()
            ipa = m.run_ipa(c, mask[:, 0].repeat(S, 1), Rigid(Rotation(rot_mats=rots.repeat(S, 1, 1, 1)), trans.repeat(S, 1, 1)), None, aatype.repeat(S, 1))
            return mods, mf, ipa.reshape(S, B, mask.shape[-1], -1).contiguous()
        eng.conditioning = cond
    with torch.no_grad():
        v = m(g("x"), g("t"), g("mask"), start_frames=Rigid(Rotation(rot_mats=g("rots")), g("trans")),
              x_cond=g("x_cond"), x_cond_mask=g("x_cond_mask"), aatype=g("aatype"))
    err = np.abs(v.cpu().numpy() - ref)
    print(mode, "max all", err.max(), "valid", err[:, :, valid].max(), "padded", err[:, :, ~valid].max(),
          "rel", np.linalg.norm(v.cpu().numpy() - ref) / np.linalg.norm(ref), flush=True)
