"""Transition-path sampling (interpolation): the drop-in for the reference's ``src/tps_inference.py``.

    python -m mdgen_finetune_amd.tps_inference --sim_ckpt tps.ckpt --data_dir DIR \
        --split splits/4AA_test.csv --num_frames 100 --num_batches 10 --batch_size 10 \
        --start_idxs 0 5 9 --end_idxs 200 201 --out_dir out/

Per peptide (tps_inference.py:43-149): every sample is a T-frame window whose frame 0 is a
start frame and whose frame T-1 is an end frame of the peptide's all-atom trajectory
(``{data_dir}/{name}{suffix}.npy``, atom14 in Å, memory-mapped); all frames in between carry
the start frame (``get_sample``, tps_inference.py:43-79).  ``NewMDGenWrapper.inference``
(--tps_condition: frames 0 and T-1 conditioned, latent 28) samples the B = batch_size windows
of a batch at once — the HIP Euler / dopri5 sampler and the HIP atom14 reconstruction on a
ROCm device — and each window is written as a multi-model PDB plus one metadata record.

What the reference does and this build does not: it picks the start / end frames from the
two metastable states of least flux of an MSM fitted to the reference simulation
(mdgen.analysis: PyEMMA / deeptime featurisation, TICA, k-means, PCCA — tps_inference.py:81-
118), then superposes with mdtraj and writes XTC.  Those analysis libraries are not part of
the denoising path (out of scope) and not installed; the candidate frame indices
are passed instead (``--start_idxs`` / ``--end_idxs``, or ``--states_json`` with
{name: {"start_idxs": [...], "end_idxs": [...], "start_state": s, "end_state": e}}), and the
sampled window is written as PDB only.
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np
import torch

from . import geometry as G
from .checkpoint import load_from_checkpoint
from .pdb import atom14_to_pdb
from .sim_inference import RESTYPES


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--sim_ckpt", type=str, required=True)
    p.add_argument("--data_dir", type=str, default="share/4AA_data")
    p.add_argument("--suffix", type=str, default="")
    p.add_argument("--pdb_id", nargs="*", default=[])
    p.add_argument("--num_frames", type=int, default=1000)
    p.add_argument("--num_batches", type=int, default=100)
    p.add_argument("--batch_size", type=int, default=10)
    p.add_argument("--out_dir", type=str, default=".")
    p.add_argument("--split", type=str, default="splits/4AA_test.csv")
    p.add_argument("--chunk_idx", type=int, default=0)
    p.add_argument("--n_chunks", type=int, default=1)
    p.add_argument("--start_idxs", type=int, nargs="*", default=None, help="candidate start frames (state A)")
    p.add_argument("--end_idxs", type=int, nargs="*", default=None, help="candidate end frames (state B)")
    p.add_argument("--states_json", type=str, default=None, help="per-peptide start/end frame candidates")
    p.add_argument("--synthetic", type=str, default=None,
                   help="peptide sequence: sample between two frames of a synthetic trajectory (no dataset)")
    p.add_argument("--seed", type=int, default=137)
    p.add_argument("--batches_per_pass", type=int, default=1,
                   help="sample this many consecutive batches in one GPU pass (same windows, files and metadata "
                        "as one at a time; the reference's batch of 10 leaves most of an MI355X idle)")
    return p.parse_args(argv)


def _frame_features(atom14, aatype):
    """Frames + torsions of one frame [1, L, 14, 3] (tps_inference.py:50-58)."""
    fr = G.atom14_to_frames(atom14)
    a37 = G.atom14_to_atom37(atom14, aatype[None])
    tors, tmask = G.atom37_to_torsions(a37, aatype[None])
    return fr, tors, tmask


def get_sample(arr, aatype, start_idxs, end_idxs, start_state=0, end_state=1, num_frames=1000, rng=None,
               device="cpu"):
    """tps_inference.py:43-79: a window whose frame 0 is a random start-state frame and whose
    last frame is a random end-state frame; the frames in between repeat the start frame."""
    rng = rng if rng is not None else np.random
    start_idx = int(rng.choice(start_idxs, 1).item())
    end_idx = int(rng.choice(end_idxs, 1).item())
    start = torch.from_numpy(np.array(arr[start_idx:start_idx + 1], dtype=np.float32)).to(device)
    end = torch.from_numpy(np.array(arr[end_idx:end_idx + 1], dtype=np.float32)).to(device)
    aatype = aatype.to(device)
    s_fr, s_tors, s_tmask = _frame_features(start, aatype)
    e_fr, e_tors, _ = _frame_features(end, aatype)
    L = aatype.shape[0]
    tors = s_tors.expand(num_frames, -1, -1, -1).clone()
    tors[-1] = e_tors[0]
    trans = s_fr.get_trans().expand(num_frames, -1, -1).clone()
    trans[-1] = e_fr.get_trans()[0]
    rots = s_fr.get_rots().get_rot_mats().expand(num_frames, -1, -1, -1).clone()
    rots[-1] = e_fr.get_rots().get_rot_mats()[0]
    return {"torsions": tors, "torsion_mask": s_tmask[0], "trans": trans, "rots": rots, "seqres": aatype,
            "start_idx": start_idx, "end_idx": end_idx, "start_state": int(start_state), "end_state": int(end_state),
            "mask": torch.ones(L, device=device)}


def collate_samples(samples):
    out = {}
    for k in samples[0]:
        v = [s[k] for s in samples]
        out[k] = torch.stack(v) if torch.is_tensor(v[0]) else torch.tensor(v)
    return out


def sample_batches(model, name, arr, aatype, start_idxs, end_idxs, args, device, start_state=0, end_state=1,
                   zs0=None):
    """tps_inference.py:119-149 without the mdtraj superpose / XTC: per batch, B windows sampled
    together; returns the metadata records and the atom14 windows written."""
    rng = np.random.RandomState(args.seed)
    metadata, outs = [], []
    bs, k = args.batch_size, max(1, int(getattr(args, "batches_per_pass", 1) or 1))
    for i0 in range(0, args.num_batches, k):
        ids = list(range(i0, min(i0 + k, args.num_batches)))
        # the windows are drawn batch by batch in the reference's order, then stacked
        batches = [collate_samples([get_sample(arr, aatype, start_idxs, end_idxs, start_state, end_state,
                                               args.num_frames, rng, device) for _ in range(bs)]) for _ in ids]
        batch = {key: torch.cat([b[key] for b in batches]) for key in batches[0]}
        z = None if zs0 is None else torch.cat([zs0[i] for i in ids]).to(device)
        atom14s, _ = model.inference({key: v.to(device) for key, v in batch.items()}, zs0=z)
        for n, i in enumerate(ids):
            outs.append(atom14s[n * bs:(n + 1) * bs])
            for j in range(bs):
                idx, row = i * bs + j, n * bs + j
                path = os.path.join(args.out_dir, f"{name}_{idx}.pdb")
                atom14_to_pdb(atom14s[row].cpu().numpy(), batch["seqres"][0].cpu().numpy(), path)
                metadata.append({"name": name, "start_idx": int(batch["start_idx"][row]),
                                 "end_idx": int(batch["end_idx"][row]), "start_state": int(batch["start_state"][row]),
                                 "end_state": int(batch["end_state"][row]), "path": path})
    return metadata, outs


def _synthetic_traj(seq, n_frames, seed):
    """A synthetic all-atom trajectory [n_frames, L, 14, 3] of `seq` (frames + torsions of the
    synthetic dataset rebuilt to atoms), standing in for {data_dir}/{name}.npy offline."""
    from .data import SyntheticMDDataset

    it = SyntheticMDDataset(n_frames, len(seq), size=1, seed=seed)[0]
    aat = torch.tensor([RESTYPES.index(c) for c in seq], dtype=torch.int64)
    a14 = G.frames_torsions_to_atom14(it["rots"], it["trans"], it["torsions"], aat[None].expand(n_frames, -1))
    return a14.numpy().astype(np.float32), aat


@torch.no_grad()
def run(args):
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    os.makedirs(args.out_dir, exist_ok=True)
    model = load_from_checkpoint(args.sim_ckpt, map_location="cpu")
    if not model.args.tps_condition:
        raise ValueError("tps_inference needs a --tps_condition checkpoint (latent 28, frames 0 and T-1 conditioned)")
    model.args.num_frames = args.num_frames
    model = model.eval().to(device)
    if device.type != "cuda":
        model.model.backend = "torch"
    states = json.load(open(args.states_json)) if args.states_json else {}
    jobs = []
    if args.synthetic:
        arr, aat = _synthetic_traj(args.synthetic, 64, args.seed)
        jobs.append((args.synthetic, arr, aat))
    else:
        import pandas as pd

        df = pd.read_csv(args.split, index_col="name")
        names = np.array_split(np.array(df.index), args.n_chunks)[args.chunk_idx]
        for name in names:
            if args.pdb_id and name not in args.pdb_id:
                continue
            arr = np.load(f"{args.data_dir}/{name}{args.suffix}.npy", mmap_mode="r", allow_pickle=False)
            jobs.append((name, arr, torch.tensor([RESTYPES.index(c) for c in df.seqres[name]], dtype=torch.int64)))
    done = {}
    for name, arr, aat in jobs:
        st = states.get(name, {})
        s_idx = st.get("start_idxs", args.start_idxs if args.start_idxs else [0])
        e_idx = st.get("end_idxs", args.end_idxs if args.end_idxs else [len(arr) - 1])
        meta, _ = sample_batches(model, name, arr, aat, s_idx, e_idx, args, device, st.get("start_state", 0),
                                 st.get("end_state", 1))
        json.dump(meta, open(os.path.join(args.out_dir, f"{name}_metadata.json"), "w"))
        done[name] = len(meta)
        print(f"{name}: {len(meta)} transition paths of {args.num_frames} frames", flush=True)
    return done


def main(argv=None):
    run(parse_args(argv))


if __name__ == "__main__":
    main()
