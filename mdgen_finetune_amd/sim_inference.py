"""Forward-simulation rollouts: the drop-in for the reference's ``src/sim_inference.py``.

    python -m mdgen_finetune_amd.sim_inference --sim_ckpt forward_sim.ckpt --data_dir DIR \
        --split splits/4AA_test.csv --num_frames 1000 --num_rollouts 100 --out_dir out/

Per peptide (sim_inference.py:38-131): the first frame of its all-atom trajectory
(``{data_dir}/{name}{suffix}.npy``, atom14 in Å) gives the start frames and torsions; each
rollout window expands them over ``num_frames``, samples the window
(NewMDGenWrapper.inference: HIP Euler sampler + HIP atom14 reconstruction), and restarts the
next window from the window's last frame (atom14 -> frames, atom37 -> torsions).  All windows
are concatenated and written as one multi-model PDB.

Beyond the reference: ``--batch`` rolls out that many independent trajectories of the same
peptide at once (B rows of one window), and ``--synthetic`` starts from a synthetic frame when
no dataset is available offline.  ``--xtc`` (mdtraj) and ``--no_frames`` are not built.
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np
import torch

from . import geometry as G
from .checkpoint import load_from_checkpoint
from .pdb import atom14_to_pdb

RESTYPES = "ARNDCQEGHILKMFPSTWYV"


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--sim_ckpt", type=str, required=True)
    p.add_argument("--data_dir", type=str, default=None)
    p.add_argument("--suffix", type=str, default="")
    p.add_argument("--pdb_id", nargs="*", default=[])
    p.add_argument("--num_frames", type=int, default=1000)
    p.add_argument("--num_rollouts", type=int, default=100)
    p.add_argument("--tps", action="store_true")
    p.add_argument("--out_dir", type=str, default=".")
    p.add_argument("--split", type=str, default="splits/4AA_test.csv")
    p.add_argument("--batch", type=int, default=1, help="independent trajectories per peptide")
    p.add_argument("--synthetic", type=str, default=None, help="peptide sequence to start from a synthetic frame")
    p.add_argument("--seed", type=int, default=0)
    return p.parse_args(argv)


def seq_to_aatype(seqres):
    return torch.tensor([RESTYPES.index(c) for c in seqres], dtype=torch.int64)


def batch_from_atom14(atom14, aatype, device):
    """sim_inference.py:38-63 for the first frame: frames, torsions, masks of one peptide."""
    atom14 = atom14.to(device)
    aatype = aatype.to(device)
    fr = G.atom14_to_frames(atom14)                                     # [1,L]
    a37 = G.atom14_to_atom37(atom14, aatype[None])
    tors, tmask = G.atom37_to_torsions(a37, aatype[None])
    L = aatype.shape[0]
    return {"torsions": tors[None], "torsion_mask": tmask[0][None], "trans": fr.get_trans()[None],
            "rots": fr.get_rots().get_rot_mats()[None], "seqres": aatype[None], "mask": torch.ones(1, L, device=device)}


def rollout(model, batch, num_frames, n_traj=1, zs0=None):
    """sim_inference.py:65-93: one window from the batch's start frame; returns the window's
    atom14 [n_traj, T, L, 14, 3] and the batch restarted from each trajectory's last frame
    (``zs0``: the window's prior noise, drawn by the wrapper when None)."""
    B = batch["trans"].shape[0]
    if B != n_traj:
        batch = {k: v.expand(n_traj, *v.shape[1:]) for k, v in batch.items()}
    ex = {
        "torsions": batch["torsions"].expand(-1, num_frames, -1, -1, -1),
        "torsion_mask": batch["torsion_mask"],
        "trans": batch["trans"].expand(-1, num_frames, -1, -1),
        "rots": batch["rots"].expand(-1, num_frames, -1, -1, -1),
        "seqres": batch["seqres"],
        "mask": batch["mask"],
    }
    atom14, _ = model.inference(ex, zs0=zs0)
    last = atom14[:, -1]                                                # [n,L,14,3]
    fr = G.atom14_to_frames(last)
    a37 = G.atom14_to_atom37(last, batch["seqres"])
    tors, _ = G.atom37_to_torsions(a37, batch["seqres"])
    new = dict(batch)
    new["trans"] = fr.get_trans()[:, None]
    new["rots"] = fr.get_rots().get_rot_mats()[:, None]
    new["torsions"] = tors[:, None]
    return atom14, new


@torch.no_grad()
def run(args):
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(args.seed)
    os.makedirs(args.out_dir, exist_ok=True)
    model = load_from_checkpoint(args.sim_ckpt, map_location="cpu")
    model.args.num_frames = args.num_frames
    model = model.eval().to(device)
    if device.type != "cuda":
        model.model.backend = "torch"  # CPU run: eager denoiser (the HIP path needs a ROCm device)
    jobs = []
    if args.synthetic:
        from .data import SyntheticMDDataset

        aat = seq_to_aatype(args.synthetic)
        it = SyntheticMDDataset(1, len(args.synthetic), size=1, seed=args.seed)[0]
        start = {"torsions": it["torsions"][None], "torsion_mask": it["torsion_mask"][None],
                 "trans": it["trans"][None], "rots": it["rots"][None], "seqres": aat[None],
                 "mask": torch.ones(1, len(args.synthetic))}
        jobs.append((args.synthetic, {k: v.to(device) for k, v in start.items()}))
    else:
        import pandas as pd

        df = pd.read_csv(args.split, index_col="name")
        for name in df.index:
            if args.pdb_id and name not in args.pdb_id:
                continue
            arr = np.load(f"{args.data_dir}/{name}{args.suffix}.npy", mmap_mode="r", allow_pickle=False)
            atom14 = torch.from_numpy(np.array(arr[0:1], dtype=np.float32))
            jobs.append((name, batch_from_atom14(atom14, seq_to_aatype(df.seqres[name]), device)))
            break  # sim_inference.py:135: the reference stops after the first peptide
    timings = {}
    for name, batch in jobs:
        t0 = time.time()
        windows = []
        for _ in range(args.num_rollouts):
            atom14, batch = rollout(model, batch, args.num_frames, args.batch)
            windows.append(atom14)
        if device.type == "cuda":
            torch.cuda.synchronize()
        timings[name] = time.time() - t0
        traj = torch.cat(windows, 1)                                    # [n, rollouts*T, L, 14, 3]
        aat = batch["seqres"][0].cpu().numpy()
        for j in range(traj.shape[0]):
            sfx = "" if traj.shape[0] == 1 else f"_{j}"
            atom14_to_pdb(traj[j].cpu().numpy(), aat, os.path.join(args.out_dir, f"{name}{sfx}.pdb"))
        print(f"{name}: {args.num_rollouts} windows x {args.batch} traj x {args.num_frames} frames "
              f"in {timings[name]:.2f} s", flush=True)
    return timings


def main(argv=None):
    run(parse_args(argv))


if __name__ == "__main__":
    main()
