"""Multi-model PDB output of a rollout (reference utils.atom14_to_pdb / prots_to_pdb,
src/mdgen/utils.py:59-103, with protein.to_pdb's ATOM/TER records, protein.py:321-440): one
``MODEL`` block per frame, atoms in the 37-atom order of each residue, absent atoms (all-zero
coordinates) skipped, chain A, residues numbered from 0."""
from __future__ import annotations

import numpy as np

from .geometry import rc


def _atom14_to_atom37_np(atom14: np.ndarray, aatype: np.ndarray) -> np.ndarray:
    t = rc()
    idx = t["restype_atom37_to_atom14"][aatype]                        # [L,37]
    out = np.take_along_axis(atom14, idx[..., None].repeat(3, -1), axis=-2)
    return out * t["restype_atom37_mask"][aatype][..., None]


def _model_lines(atom37: np.ndarray, aatype: np.ndarray):
    t = rc()
    names, res3 = [str(a) for a in t["atom_types"]], [str(r) for r in t["restype_3"]]
    mask = np.sum(np.abs(atom37), axis=-1) > 1e-7                      # utils.create_full_prot
    lines, k = [], 1
    for i in range(aatype.shape[0]):
        rn = res3[int(aatype[i])]
        for j, name in enumerate(names):
            if not mask[i, j]:
                continue
            x, y, z = atom37[i, j]
            nm = name if len(name) == 4 else f" {name}"
            lines.append(f"{'ATOM':<6}{k:>5} {nm:<4}{'':>1}{rn:>3} {'A':>1}{i:>4}{'':>1}   "
                         f"{x:>8.3f}{y:>8.3f}{z:>8.3f}{1.0:>6.2f}{0.0:>6.2f}          {name[0]:>2}{'':>2}")
            k += 1
    lines.append(f"{'TER':<6}{k:>5}      {res3[int(aatype[-1])]:>3} {'A':>1}{aatype.shape[0] - 1:>4}")
    return [ln.ljust(80) for ln in lines]  # PDB records are 80 columns


def atom14_to_pdb_string(atom14: np.ndarray, aatype: np.ndarray) -> str:
    """atom14 [T, L, 14, 3] (Å), aatype [L] -> the reference's multi-model PDB text."""
    atom14 = np.asarray(atom14, dtype=np.float64 if atom14.dtype == np.float64 else np.float32)
    aatype = np.asarray(aatype).astype(np.int64)
    out = []
    for i, pos in enumerate(atom14):
        out.append(f"MODEL      {i}\n" + "\n".join(_model_lines(_atom14_to_atom37_np(pos, aatype), aatype))
                   + "\nENDMDL\n")
    return "".join(out)


def atom14_to_pdb(atom14, aatype, path):
    with open(path, "w") as f:
        f.write(atom14_to_pdb_string(np.asarray(atom14), np.asarray(aatype)))
