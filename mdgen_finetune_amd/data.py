"""Training data in the reference's batch format (MDGenDataset.__getitem__,
src/mdgen/dataset.py:40-123): per item ``torsions`` [T,L,7,2] (sin, cos), ``torsion_mask``
[L,7], ``trans`` [T,L,3] (Å), ``rots`` [T,L,3,3], ``seqres`` [L] int64, ``mask`` [L] f32.

* ``MDGenDataset``: the reference's dataset, restated — a split CSV (``name,seqres``) of
  peptides whose atom14 trajectories are ``{data_dir}/{name}{suffix}.npy`` memmaps [F,L,14,3]
  (Å); each item is a random window of ``num_frames`` frames (every ``frame_interval``-th),
  its backbone frames (atom14_to_frames), torsions (atom14 -> atom37 -> atom37_to_torsions)
  and, for ATLAS, a random crop / identity-frame padding to ``crop`` residues.
* ``SyntheticMDDataset``: trajectories of the same shape for runs without the dataset (it
  cannot be fetched offline, README.md:26-27): per residue a backbone frame on a 3.8 Å chain
  that diffuses in orientation (random axis-angle increments) and position, and seven torsion
  angles doing a wrapped random walk.  Each item is a pure function of (seed, index), so every
  DDP rank can build its shard without communication."""
from __future__ import annotations

import os

import numpy as np
import torch

RESTYPES = "ARNDCQEGHILKMFPSTWYV"  # residue_constants.restype_order


class MDGenDataset(torch.utils.data.Dataset):
    """dataset.py:11-123.  ``rng``: the window / crop / replica draws (the reference uses numpy's
    global state; each DDP rank passes its own generator so ranks draw independent windows).

    Deviation, on purpose: the reference's ``_validate_peptides`` (dataset.py:24-38) overwrites
    the loop index with the ATLAS replica draw and so keeps random rows under ``--atlas``; here
    every row whose file exists (for ATLAS: some replica ``_R1``-``_R3``) is kept."""

    def __init__(self, args, split, repeat=1, data_dir=None, peptide=None, rng=None):
        import pandas as pd

        super().__init__()
        self.args = args
        self.repeat = repeat
        self.data_dir = data_dir if data_dir is not None else args.data_dir
        self.rng = rng if rng is not None else np.random.default_rng()
        if getattr(args, "no_frames", False):
            raise NotImplementedError("--no_frames (atom37 items) is not on the flow-matching path")
        self.df = self._validate_peptides(pd.read_csv(split, index_col="name"), peptide)

    def _path(self, name):
        return os.path.join(self.data_dir, f"{name}{self.args.suffix}.npy")

    def _validate_peptides(self, df, peptide=None):
        keep = []
        for i, name in enumerate(df.index):
            if peptide is not None and peptide != name:
                continue
            names = [f"{name}_R{r}" for r in (1, 2, 3)] if self.args.atlas else [name]
            if any(os.path.exists(self._path(n)) for n in names):
                keep.append(i)
        return df.iloc[keep]

    def __len__(self):
        if self.args.overfit_peptide:
            return 1000
        return self.repeat * len(self.df)

    def __getitem__(self, idx):
        from .geometry import atom14_to_atom37, atom14_to_frames, atom37_to_torsions

        a = self.args
        if a.overfit_peptide is None:
            idx = 0 if a.overfit else idx % len(self.df)
            name = self.df.index[idx]
            seqres = self.df.seqres[name]
        else:
            name = seqres = a.overfit_peptide
        full_name = f"{name}_R{int(self.rng.integers(1, 4))}" if a.atlas else name
        arr = np.lib.format.open_memmap(self._path(full_name), "r")
        if a.frame_interval:
            arr = arr[::a.frame_interval]
        n_start = arr.shape[0] - a.num_frames
        if n_start <= 0:  # np.random.choice(np.arange(n)) raises on an empty range
            raise ValueError(f"{full_name}: {arr.shape[0]} frames, a window needs more than {a.num_frames}")
        frame_start = 0 if a.overfit_frame else int(self.rng.integers(0, n_start))
        arr = np.array(arr[frame_start:frame_start + a.num_frames], dtype=np.float32)  # Å
        if a.copy_frames:
            arr[1:] = arr[0]
        atom14 = torch.from_numpy(arr)
        frames = atom14_to_frames(atom14)
        aa = np.array([RESTYPES.index(c) for c in seqres], dtype=np.int64)
        aatype = torch.from_numpy(aa)[None].expand(a.num_frames, -1)
        atom37 = atom14_to_atom37(atom14, aatype).float()
        torsions, torsion_mask = atom37_to_torsions(atom37, aatype)
        torsion_mask = torsion_mask[0]
        rots, trans = frames.get_rots().get_rot_mats(), frames.get_trans()
        L = rots.shape[1]
        mask = np.ones(L, dtype=np.float32)
        if a.atlas and L > a.crop:
            s = int(self.rng.integers(0, L - a.crop + 1))
            sl = slice(s, s + a.crop)
            torsions, rots, trans = torsions[:, sl], rots[:, sl], trans[:, sl]
            aa, mask, torsion_mask = aa[sl], mask[sl], torsion_mask[sl]
        elif a.atlas and L < a.crop:  # identity frames, zero torsions, aatype 0 (dataset.py:103-112)
            pad = a.crop - L
            T = a.num_frames
            rots = torch.cat([rots, torch.eye(3).expand(T, pad, 3, 3)], 1)
            trans = torch.cat([trans, torch.zeros(T, pad, 3)], 1)
            mask = np.concatenate([mask, np.zeros(pad, dtype=np.float32)])
            aa = np.concatenate([aa, np.zeros(pad, dtype=np.int64)])
            torsions = torch.cat([torsions, torch.zeros(T, pad, 7, 2)], 1)
            torsion_mask = torch.cat([torsion_mask, torch.zeros(pad, 7)])
        return {
            "name": full_name,
            "frame_start": frame_start,
            "torsions": torsions.contiguous(),
            "torsion_mask": torsion_mask.contiguous(),
            "trans": trans.contiguous(),
            "rots": rots.contiguous(),
            "seqres": torch.from_numpy(np.ascontiguousarray(aa)),
            "mask": torch.from_numpy(mask),
        }


def _axis_angle_to_rot(v: np.ndarray) -> np.ndarray:
    """Rodrigues: rotation vectors [..., 3] -> matrices [..., 3, 3]."""
    th = np.linalg.norm(v, axis=-1, keepdims=True)
    k = v / np.maximum(th, 1e-12)
    kx, ky, kz = k[..., 0], k[..., 1], k[..., 2]
    z = np.zeros_like(kx)
    K = np.stack([np.stack([z, -kz, ky], -1), np.stack([kz, z, -kx], -1), np.stack([-ky, kx, z], -1)], -2)
    th = th[..., None]
    eye = np.broadcast_to(np.eye(3), K.shape)
    return eye + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


class SyntheticMDDataset(torch.utils.data.Dataset):
    def __init__(self, num_frames: int, crop: int, size: int = 64, seed: int = 137, n_pad: int = 0):
        self.T, self.L, self.size, self.seed, self.n_pad = num_frames, crop, size, seed, n_pad

    def __len__(self):
        return self.size

    def __getitem__(self, idx):
        rng = np.random.default_rng([self.seed, idx])
        T, L = self.T, self.L
        base = rng.standard_normal((L, 3))
        rot0 = _axis_angle_to_rot(base * np.pi / np.sqrt(3))  # [L,3,3]
        dr = _axis_angle_to_rot(rng.standard_normal((T, L, 3)) * 0.05)  # per-frame increments
        rots = np.empty((T, L, 3, 3))
        r = rot0
        for t in range(T):
            r = dr[t] @ r
            rots[t] = r
        chain = np.cumsum(np.concatenate([np.zeros((1, 3)), rng.standard_normal((L - 1, 3))]), 0)
        chain *= 3.8 / np.maximum(np.linalg.norm(rng.standard_normal((1, 3)), axis=-1), 1e-6)
        trans = chain[None] + np.cumsum(rng.standard_normal((T, L, 3)) * 0.1, 0)
        ang = rng.uniform(-np.pi, np.pi, (L, 7)) + np.cumsum(rng.standard_normal((T, L, 7)) * 0.1, 0)
        torsions = np.stack([np.sin(ang), np.cos(ang)], -1)  # (sin, cos): atom37_to_torsions' order
        torsion_mask = np.zeros((L, 7), np.float32)
        torsion_mask[:, :3] = 1.0
        n_chi = rng.integers(0, 5, L)
        for l in range(L):
            torsion_mask[l, 3:3 + n_chi[l]] = 1.0
        mask = np.ones(L, np.float32)
        seqres = rng.integers(0, 20, L).astype(np.int64)
        if self.n_pad:  # dataset.py:106-118: identity frames, zero torsions, aatype 0
            p = slice(L - self.n_pad, L)
            mask[p] = 0.0
            rots[:, p] = np.eye(3)
            trans[:, p] = 0.0
            torsions[:, p] = 0.0
            torsion_mask[p] = 0.0
            seqres[p] = 0
        return {
            "name": f"synthetic_{idx}",
            "frame_start": 0,
            "torsions": torch.from_numpy(torsions.astype(np.float32)),
            "torsion_mask": torch.from_numpy(torsion_mask),
            "trans": torch.from_numpy(trans.astype(np.float32)),
            "rots": torch.from_numpy(rots.astype(np.float32)),
            "seqres": torch.from_numpy(seqres),
            "mask": torch.from_numpy(mask),
        }


def collate(items):
    """DataLoader default collate restricted to tensors (names kept as a list)."""
    out = {}
    for k in items[0]:
        vals = [it[k] for it in items]
        out[k] = torch.stack(vals) if torch.is_tensor(vals[0]) else vals
    return out
