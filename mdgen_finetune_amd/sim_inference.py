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
peptide at once (B rows of one window); ``--all_peptides`` goes on past the first peptide of the
split (the reference stops there, sim_inference.py:135-136); ``--peptides_per_window K`` rolls
out K peptides of the same crop length in ONE window (their K*B rows side by side: the model
conditions every row on its own frames, residue types and mask, so a window of K peptides is K
windows' work in one launch sequence; tetrapeptides all have L = 4); ``--synthetic SEQ[,SEQ..]``
starts from synthetic frames when no dataset is available offline.  Every peptide draws its
windows' prior noise from its own generator (seed, position in the split), so a peptide's
trajectory does not depend on which peptides share its windows.  ``--xtc`` (mdtraj) and
``--no_frames`` are not built.
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
    p.add_argument("--all_peptides", action="store_true", help="every peptide of the split (the reference: the first)")
    p.add_argument("--peptides_per_window", type=int, default=1,
                   help="peptides of the same crop length rolled out together in one window")
    p.add_argument("--synthetic", type=str, default=None,
                   help="comma-separated peptide sequences to start from synthetic frames")
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


def peptide_generator(seed, index, device):
    """The prior-noise stream of the index-th peptide of a run."""
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) * 1000003 + int(index))
    return g


def rollout_group(model, group, num_frames, num_rollouts, n_traj, latent_dim):
    """num_rollouts windows of the peptides in ``group`` [(name, start batch, generator)], all of
    one crop length, side by side in each window (n_traj rows per peptide); returns each
    peptide's atom14 trajectory [n_traj, num_rollouts * T, L, 14, 3] and its last batch."""
    k = len(group)
    L = group[0][1]["trans"].shape[-2]
    assert all(b["trans"].shape[-2] == L for _, b, _ in group), "one window holds one crop length"
    rows = [{key: v.expand(n_traj, *v.shape[1:]) for key, v in b.items()} for _, b, _ in group]
    batch = {key: torch.cat([r[key] for r in rows]) for key in rows[0]}
    windows = []
    for _ in range(num_rollouts):
        zs0 = torch.cat([torch.randn(n_traj, num_frames, L, latent_dim, generator=g, device=g.device)
                         for _, _, g in group])
        atom14, batch = rollout(model, batch, num_frames, k * n_traj, zs0=zs0)
        windows.append(atom14)
    traj = torch.cat(windows, 1)
    out = []
    for i, (name, _, _) in enumerate(group):
        sl = slice(i * n_traj, (i + 1) * n_traj)
        out.append((name, traj[sl], {key: v[sl] for key, v in batch.items()}))
    return out


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

        for k, seq in enumerate(args.synthetic.split(",")):
            aat = seq_to_aatype(seq)
            it = SyntheticMDDataset(1, len(seq), size=1, seed=args.seed + k)[0]
            start = {"torsions": it["torsions"][None], "torsion_mask": it["torsion_mask"][None],
                     "trans": it["trans"][None], "rots": it["rots"][None], "seqres": aat[None],
                     "mask": torch.ones(1, len(seq))}
            jobs.append((seq if k == 0 or seq not in args.synthetic.split(",")[:k] else f"{seq}_{k}",
                         {key: v.to(device) for key, v in start.items()}))
    else:
        import pandas as pd

        df = pd.read_csv(args.split, index_col="name")
        for name in df.index:
            if args.pdb_id and name not in args.pdb_id:
                continue
            arr = np.load(f"{args.data_dir}/{name}{args.suffix}.npy", mmap_mode="r", allow_pickle=False)
            atom14 = torch.from_numpy(np.array(arr[0:1], dtype=np.float32))
            jobs.append((name, batch_from_atom14(atom14, seq_to_aatype(df.seqres[name]), device)))
            if not args.all_peptides:
                break  # sim_inference.py:135-136: the reference stops after the first peptide
    lat = model.latent_dim
    jobs = [(name, b, peptide_generator(args.seed, i, device)) for i, (name, b) in enumerate(jobs)]
    # windows of up to K peptides of one crop length, in split order within each length
    by_len = {}
    for job in jobs:
        by_len.setdefault(int(job[1]["trans"].shape[-2]), []).append(job)
    K = max(1, args.peptides_per_window)
    timings = {}
    for L, js in by_len.items():
        for g0 in range(0, len(js), K):
            group = js[g0:g0 + K]
            t0 = time.time()
            res = rollout_group(model, group, args.num_frames, args.num_rollouts, args.batch, lat)
            if device.type == "cuda":
                torch.cuda.synchronize()
            el = time.time() - t0
            for name, traj, last in res:
                timings[name] = el / len(group)
                aat = last["seqres"][0].cpu().numpy()
                for j in range(traj.shape[0]):
                    sfx = "" if traj.shape[0] == 1 else f"_{j}"
                    atom14_to_pdb(traj[j].cpu().numpy(), aat, os.path.join(args.out_dir, f"{name}{sfx}.pdb"))
            print(f"{','.join(n for n, _, _ in group)}: {args.num_rollouts} windows x {args.batch} traj x "
                  f"{args.num_frames} frames x {len(group)} peptides in {el:.2f} s", flush=True)
    return timings


def main(argv=None):
    run(parse_args(argv))


if __name__ == "__main__":
    main()
