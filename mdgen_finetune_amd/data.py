"""Training data in the reference's batch format (MDGenDataset.__getitem__,
src/mdgen/dataset.py:43-128): per item ``torsions`` [T,L,7,2] (cos, sin), ``torsion_mask``
[L,7], ``trans`` [T,L,3] (Å), ``rots`` [T,L,3,3], ``seqres`` [L] int64, ``mask`` [L] f32.

The reference reads memory-mapped all-atom trajectories from a dataset that cannot be fetched
offline (README.md:26-27), so this build trains on synthetic trajectories of the same shape:
per residue a backbone frame on a 3.8 Å chain that diffuses in orientation (random axis-angle
increments) and position, and seven torsion angles doing a wrapped random walk.  Each item is a
pure function of (seed, index), so every DDP rank can build its shard without communication."""
from __future__ import annotations

import numpy as np
import torch


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
        torsions = np.stack([np.cos(ang), np.sin(ang)], -1)
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
