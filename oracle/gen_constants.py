"""Extract the residue-geometry constant tables the rollout geometry needs (container-only).

The tables are AlphaFold/OpenFold's idealised residue geometry as the reference computes them
in src/mdgen/residue_constants.py (rigid_group_atom_positions -> default frames, atom14
literature positions, atom14<->atom37 maps, chi-angle atom indices; lines 1102-1483) and
geometry.get_chi_atom_indices (geometry.py:321-345).  They are numeric data, not code: this
script imports the reference in the build container (with the oracle shims for its missing
third-party imports) and writes them to mdgen_finetune_amd/residue_constants.npz, which the
product path loads with numpy (allow_pickle=False).  No reference source is copied.

Usage:  python oracle/gen_constants.py
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, "/root/reference/src")
sys.path.insert(0, os.path.join(HERE, "shim"))

import numpy as np  # noqa: E402


def main():
    from mdgen import residue_constants as rc
    from mdgen.geometry import get_chi_atom_indices

    restypes = list(rc.restypes) + ["X"]
    out = dict(
        restype_rigid_group_default_frame=rc.restype_rigid_group_default_frame.astype(np.float32),  # [21,8,4,4]
        restype_atom14_to_rigid_group=rc.restype_atom14_to_rigid_group.astype(np.int64),            # [21,14]
        restype_atom14_mask=rc.restype_atom14_mask.astype(np.float32),                              # [21,14]
        restype_atom14_rigid_group_positions=rc.restype_atom14_rigid_group_positions.astype(np.float32),
        restype_atom37_to_atom14=np.asarray(rc.RESTYPE_ATOM37_TO_ATOM14, np.int64),                 # [21,37]
        restype_atom14_to_atom37=np.asarray(rc.RESTYPE_ATOM14_TO_ATOM37, np.int64),                 # [21,14]
        restype_atom37_mask=np.asarray(rc.RESTYPE_ATOM37_MASK, np.float32),                         # [21,37]
        chi_angles_mask=np.asarray(list(rc.chi_angles_mask) + [[0.0] * 4], np.float32),             # [21,4]
        chi_atom_indices=np.asarray(get_chi_atom_indices(), np.int64),                              # [21,4,4]
        atom_types=np.asarray(rc.atom_types),                                                       # [37] str
        restypes=np.asarray(restypes),                                                              # [21] str
        restype_3=np.asarray([rc.restype_1to3.get(r, "UNK") for r in restypes]),                    # [21] str
    )
    path = os.path.join(REPO, "mdgen_finetune_amd", "residue_constants.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} B): " + ", ".join(f"{k}{list(v.shape)}" for k, v in out.items()))


if __name__ == "__main__":
    main()
