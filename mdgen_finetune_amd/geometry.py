"""Rollout geometry: frames + torsions -> atom14 coordinates and back (reference
src/mdgen/geometry.py), i.e. the steps on either side of the denoiser in sim_inference.py
(rollout, 59-93) and in NewMDGenWrapper.inference (wrapper.py:480-508).

Two implementations of the hot direction (latents -> atom14, once per denoised frame):
  * ``latents_to_atom14_hip`` — one HIP launch (mdg_latents_to_atom14): offsets -> frames
    composed onto frame 0, torsion normalisation, the 8 rigid-group frames per residue and
    the 14 atom positions, per token;
  * the eager torch functions below (any device), restating geometry.py:54-81, 218-317.
The inverse direction (atom14 -> frames, atom37 -> torsions) runs on the last frame of a
window only (B x L residues) and stays in torch.

Constant tables (idealised residue geometry, atom14/atom37 maps, chi atoms) are loaded from
residue_constants.npz (oracle/gen_constants.py extracted them from the reference's
residue_constants.py; numeric data only).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .rigid_utils import Rigid, Rotation, quat_to_rot

_NPZ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "residue_constants.npz")
_RC = None


def rc():
    """The constant tables as a dict of numpy arrays (loaded once, no pickle)."""
    global _RC
    if _RC is None:
        with np.load(_NPZ, allow_pickle=False) as d:
            _RC = {k: d[k] for k in d.files}
    return _RC


def _t(name, device, dtype=None):
    x = torch.from_numpy(rc()[name])
    return x.to(device=device, dtype=dtype) if dtype is not None else x.to(device)


# ------------------------------------------------------------------ rigid helpers (fp32)
def _compose(ra, ta, rb, tb):
    """(ra, ta) o (rb, tb): R = ra rb, t = ra tb + ta."""
    return ra @ rb, (ra @ tb.unsqueeze(-1)).squeeze(-1) + ta


def from_3_points(p_neg_x_axis, origin, p_xy_plane, eps=1e-8):
    """Gram-Schmidt frame (rigid_utils.py:1176-1218): columns e0, e1, e2; origin = translation."""
    e0 = origin - p_neg_x_axis
    e1 = p_xy_plane - origin
    e0 = e0 / torch.sqrt((e0 * e0).sum(-1, keepdim=True) + eps)
    e1 = e1 - e0 * (e0 * e1).sum(-1, keepdim=True)
    e1 = e1 / torch.sqrt((e1 * e1).sum(-1, keepdim=True) + eps)
    e2 = torch.cross(e0, e1, dim=-1)
    return torch.stack([e0, e1, e2], dim=-1), origin


# ------------------------------------------------------------------ forward: frames -> atoms
def torsion_angles_to_frames(rots, trans, alpha, aatype):
    """geometry.py:259-317: the 8 rigid-group frames per residue in the global frame.
    rots [*,3,3], trans [*,3], alpha [*,7,2] (sin, cos), aatype [*] -> ([*,8,3,3], [*,8,3])."""
    dev = rots.device
    d4 = _t("restype_rigid_group_default_frame", dev, torch.float32)[aatype]  # [*,8,4,4]
    dr, dt = d4[..., :3, :3], d4[..., :3, 3]
    bb = alpha.new_zeros(*alpha.shape[:-2], 1, 2)
    bb[..., 1] = 1
    a = torch.cat([bb, alpha], dim=-2)  # [*,8,2]
    ar = alpha.new_zeros(*a.shape[:-1], 3, 3)
    ar[..., 0, 0] = 1
    ar[..., 1, 1] = a[..., 1]
    ar[..., 1, 2] = -a[..., 0]
    ar[..., 2, 1] = a[..., 0]
    ar[..., 2, 2] = a[..., 1]
    fr = dr @ ar  # default_r.compose(all_rots): translation stays dt
    ft = dt
    rs, ts = [fr[..., i, :, :] for i in range(8)], [ft[..., i, :] for i in range(8)]
    for i in (5, 6, 7):  # chi2..4 chained onto chi1's frame (geometry.py:297-300)
        rs[i], ts[i] = _compose(rs[i - 1], ts[i - 1], rs[i], ts[i])
    fr, ft = torch.stack(rs, -3), torch.stack(ts, -2)
    return _compose(rots.unsqueeze(-3), trans.unsqueeze(-2), fr, ft)


def frames_torsions_to_atom14(rots, trans, torsions, aatype):
    """geometry.py:62-81 + 218-256: atom14 positions [*,14,3] (0 for absent atoms)."""
    gr, gt = torsion_angles_to_frames(rots, trans, torsions, aatype)
    dev = rots.device
    gidx = _t("restype_atom14_to_rigid_group", dev)[aatype]                      # [*,14]
    amask = _t("restype_atom14_mask", dev, torch.float32)[aatype]               # [*,14]
    lit = _t("restype_atom14_rigid_group_positions", dev, torch.float32)[aatype]  # [*,14,3]
    r = torch.gather(gr, -3, gidx[..., None, None].expand(*gidx.shape, 3, 3))
    t = torch.gather(gt, -2, gidx[..., None].expand(*gidx.shape, 3))
    pos = (r @ lit.unsqueeze(-1)).squeeze(-1) + t
    return pos * amask.unsqueeze(-1)


def latents_to_frames_torsions(samples, ref_rots, ref_trans, tps=False, renorm=True):
    """wrapper.py:480-501: offsets -> frames composed onto frame 0 (quaternions normalised),
    torsions -> unit (sin, cos) pairs.  samples [B,T,L,lat], ref [B,L] -> rots [B,T,L,3,3],
    trans [B,T,L,3], torsions [B,T,L,7,2]."""
    B, T, L, _ = samples.shape
    q = samples[..., :4]
    rr = quat_to_rot(q / torch.linalg.norm(q, dim=-1, keepdim=True))
    rots, trans = _compose(ref_rots[:, None], ref_trans[:, None], rr, samples[..., 4:7])
    tors = (samples[..., 14:28] if tps else samples[..., 7:21]).reshape(B, T, L, 7, 2)
    if renorm:
        tors = tors / torch.linalg.norm(tors, dim=-1, keepdim=True)
    return rots, trans, tors


# ------------------------------------------------------------------ inverse: atoms -> frames
def atom14_to_frames(atom14):
    """geometry.py:213-228: backbone frames from N, CA, C (with the x/z flip)."""
    N, CA, C = atom14[..., 0, :], atom14[..., 1, :], atom14[..., 2, :]
    r, t = from_3_points(C, CA, N)
    flip = torch.diag(torch.tensor([-1.0, 1.0, -1.0], device=atom14.device))
    return Rigid(Rotation(rot_mats=r @ flip), t)


def atom14_to_atom37(atom14, aatype):
    """geometry.py:9-27: gather into the 37-atom order, zero the absent atoms."""
    dev = atom14.device
    idx = _t("restype_atom37_to_atom14", dev)[aatype]                     # [*,37]
    m37 = _t("restype_atom37_mask", dev, atom14.dtype)[aatype]
    out = torch.gather(atom14, -2, idx[..., None].expand(*idx.shape, 3))
    return out * m37.unsqueeze(-1)


def atom37_to_torsions(pos, aatype, mask=None):
    """geometry.py:84-202: (sin, cos) of the 7 torsions (pre-omega, phi, psi, chi1-4) and their
    mask, residues along dim -3 of pos [*,L,37,3], aatype [*,L]."""
    dev = pos.device
    if mask is None:
        mask = _t("restype_atom37_mask", dev, pos.dtype)[aatype]
    pad = pos.new_zeros(*pos.shape[:-3], 1, 37, 3)
    prev = torch.cat([pad, pos[..., :-1, :, :]], dim=-3)
    mpad = mask.new_zeros(*mask.shape[:-2], 1, 37)
    prev_m = torch.cat([mpad, mask[..., :-1, :]], dim=-2)
    pre_omega = torch.cat([prev[..., 1:3, :], pos[..., :2, :]], dim=-2)
    phi = torch.cat([prev[..., 2:3, :], pos[..., :3, :]], dim=-2)
    psi = torch.cat([pos[..., :3, :], pos[..., 4:5, :]], dim=-2)
    pre_omega_m = prev_m[..., 1:3].prod(-1) * mask[..., :2].prod(-1)
    phi_m = prev_m[..., 2] * mask[..., :3].prod(-1)
    psi_m = mask[..., :3].prod(-1) * mask[..., 4]
    chi_idx = _t("chi_atom_indices", dev)[aatype]                         # [*,L,4,4]
    flat = chi_idx.reshape(*chi_idx.shape[:-2], 16)
    chis = torch.gather(pos, -2, flat[..., None].expand(*flat.shape, 3)).reshape(*chi_idx.shape, 3)
    chis_m = _t("chi_angles_mask", dev, pos.dtype)[aatype]
    chis_m = chis_m * torch.gather(mask, -1, flat).reshape(chi_idx.shape).prod(-1)
    atoms = torch.cat([pre_omega[..., None, :, :], phi[..., None, :, :], psi[..., None, :, :], chis], dim=-3)
    tmask = torch.cat([pre_omega_m[..., None], phi_m[..., None], psi_m[..., None], chis_m], dim=-1)
    r, t = from_3_points(atoms[..., 1, :], atoms[..., 2, :], atoms[..., 0, :], eps=1e-8)
    rel = (r.transpose(-1, -2) @ (atoms[..., 3, :] - t).unsqueeze(-1)).squeeze(-1)
    sc = torch.stack([rel[..., 2], rel[..., 1]], dim=-1)
    sc = sc / torch.sqrt((sc * sc).sum(-1, keepdim=True) + 1e-8)
    sc = sc * pos.new_tensor([1.0, 1.0, -1.0, 1.0, 1.0, 1.0, 1.0])[:, None]
    return sc, tmask


# ------------------------------------------------------------------ HIP path
_DEV_TABLES = {}


def _device_tables(device):
    key = str(device)
    if key not in _DEV_TABLES:
        _DEV_TABLES[key] = (
            _t("restype_rigid_group_default_frame", device, torch.float32).contiguous(),
            _t("restype_atom14_to_rigid_group", device, torch.int32).contiguous(),
            _t("restype_atom14_mask", device, torch.float32).contiguous(),
            _t("restype_atom14_rigid_group_positions", device, torch.float32).contiguous(),
        )
    return _DEV_TABLES[key]


def latents_to_atom14_hip(samples, ref_rots, ref_trans, aatype, tps=False, renorm=True, want_frames=False):
    """mdg_latents_to_atom14: samples [B,T,L,lat] fp32, ref frames [B,L], aatype [B,L] (or
    [B,T,L]) -> atom14 [B,T,L,14,3] (+ the composed frames' rots / trans if want_frames)."""
    from . import _lib

    lib = _lib.load()
    B, T, L, lat = samples.shape
    dev = samples.device
    s = samples.float().contiguous()
    rr = ref_rots.float().contiguous()
    rt = ref_trans.float().contiguous()
    aa = aatype.to(dev, torch.int64)
    aa = (aa[:, None].expand(B, T, L) if aa.dim() == 2 else aa).contiguous()
    dfr, gidx, amask, lit = _device_tables(dev)
    atom14 = torch.empty(B, T, L, 14, 3, device=dev)
    fr = torch.empty(B, T, L, 3, 3, device=dev) if want_frames else None
    ft = torch.empty(B, T, L, 3, device=dev) if want_frames else None
    _lib.check(lib.mdg_latents_to_atom14(B, T, L, lat, 14 if tps else 7, 1 if renorm else 0, s.data_ptr(),
                                         rr.data_ptr(), rt.data_ptr(), aa.data_ptr(), dfr.data_ptr(),
                                         gidx.data_ptr(), amask.data_ptr(), lit.data_ptr(), atom14.data_ptr(),
                                         _lib.ptr(fr), _lib.ptr(ft), _lib.stream_handle()),
               "mdg_latents_to_atom14")
    return (atom14, fr, ft) if want_frames else atom14
