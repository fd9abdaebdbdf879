"""Minimal rigid-body frames with the reference's semantics (OpenFold Rigid/Rotation,
reference src/mdgen/rigid_utils.py), enough for the drop-in call shapes:
``Rigid(rots=Rotation(rot_mats=...), trans=...)``, ``Rigid.from_tensor_7``, ``invert``,
``compose``, ``apply``, ``invert_apply``, ``to_tensor_7``, indexing, ``get_rots`` /
``get_trans`` / ``get_rot_mats``.  Rotations are forced to fp32 as in the reference
(rigid_utils.py:318-322)."""
from __future__ import annotations

import torch


def quat_to_rot(q: torch.Tensor) -> torch.Tensor:
    """Unit quaternion (w, x, y, z) -> rotation matrix (rigid_utils.py:155-189)."""
    a, b, c, d = q.unbind(-1)
    rows = [
        [a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c)],
        [2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b)],
        [2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d],
    ]
    return torch.stack([torch.stack(r, -1) for r in rows], -2)


def rot_to_quat(rot: torch.Tensor) -> torch.Tensor:
    """Rotation matrix -> quaternion via the dominant eigenvector of the 4x4 K matrix
    (rigid_utils.py:191-210).  The eigen-solve runs on the CPU so the eigenvector sign
    convention is LAPACK's — identical to the reference's CPU path."""
    r = [[rot[..., i, j] for j in range(3)] for i in range(3)]
    [[xx, xy, xz], [yx, yy, yz], [zx, zy, zz]] = r
    k = [[xx + yy + zz, zy - yz, xz - zx, yx - xy],
         [zy - yz, xx - yy - zz, xy + yx, xz + zx],
         [xz - zx, xy + yx, yy - xx - zz, yz + zy],
         [yx - xy, xz + zx, yz + zy, zz - xx - yy]]
    k = (1.0 / 3.0) * torch.stack([torch.stack(t, dim=-1) for t in k], dim=-2)
    _, vecs = torch.linalg.eigh(k.cpu())
    return vecs[..., -1].to(rot.device)


def rot_vec_mul(r: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    x, y, z = torch.unbind(t, dim=-1)
    return torch.stack([r[..., i, 0] * x + r[..., i, 1] * y + r[..., i, 2] * z for i in range(3)], -1)


class Rotation:
    def __init__(self, rot_mats=None, quats=None, normalize_quats=True):
        if (rot_mats is None) == (quats is None):
            raise ValueError("Exactly one input argument must be specified")
        if quats is not None:
            quats = quats.to(torch.float32)
            if normalize_quats:
                quats = quats / torch.linalg.norm(quats, dim=-1, keepdim=True)
        if rot_mats is not None:
            rot_mats = rot_mats.to(torch.float32)
        self._rot_mats, self._quats = rot_mats, quats

    @property
    def shape(self):
        return (self._rot_mats.shape[:-2] if self._rot_mats is not None else self._quats.shape[:-1])

    def get_rot_mats(self):
        return self._rot_mats if self._rot_mats is not None else quat_to_rot(self._quats)

    def get_quats(self):
        return self._quats if self._quats is not None else rot_to_quat(self._rot_mats)

    def __getitem__(self, idx):
        if not isinstance(idx, tuple):
            idx = (idx,)
        if self._rot_mats is not None:
            return Rotation(rot_mats=self._rot_mats[idx + (slice(None), slice(None))])
        return Rotation(quats=self._quats[idx + (slice(None),)], normalize_quats=False)

    def compose_r(self, r: "Rotation") -> "Rotation":
        a, b = self.get_rot_mats(), r.get_rot_mats()
        return Rotation(rot_mats=a @ b)

    def apply(self, pts):
        return rot_vec_mul(self.get_rot_mats(), pts)

    def invert_apply(self, pts):
        return rot_vec_mul(self.get_rot_mats().transpose(-1, -2), pts)

    def invert(self):
        return Rotation(rot_mats=self.get_rot_mats().transpose(-1, -2))

    def to(self, device):
        if self._rot_mats is not None:
            return Rotation(rot_mats=self._rot_mats.to(device))
        return Rotation(quats=self._quats.to(device), normalize_quats=False)


class Rigid:
    def __init__(self, rots: Rotation, trans: torch.Tensor):
        self._rots, self._trans = rots, trans.to(torch.float32)

    @property
    def shape(self):
        return self._trans.shape[:-1]

    def get_rots(self):
        return self._rots

    def get_trans(self):
        return self._trans

    def __getitem__(self, idx):
        if not isinstance(idx, tuple):
            idx = (idx,)
        return Rigid(self._rots[idx], self._trans[idx + (slice(None),)])

    def apply(self, pts):
        return self._rots.apply(pts) + self._trans

    def invert_apply(self, pts):
        return self._rots.invert_apply(pts - self._trans)

    def invert(self):
        rinv = self._rots.invert()
        return Rigid(rinv, -1 * rinv.apply(self._trans))

    def compose(self, r: "Rigid") -> "Rigid":
        return Rigid(self._rots.compose_r(r._rots), self._rots.apply(r._trans) + self._trans)

    def to_tensor_7(self):
        return torch.cat([self._rots.get_quats(), self._trans], -1)

    @staticmethod
    def from_tensor_7(t, normalize_quats=False):
        return Rigid(Rotation(quats=t[..., :4], normalize_quats=normalize_quats), t[..., 4:])

    def to(self, device):
        return Rigid(self._rots.to(device), self._trans.to(device))


def frames_to_tensors(frames, device=None):
    """(rot_mats [...,3,3], trans [...,3]) fp32 from a Rigid (ours or the reference's: anything
    with get_rots().get_rot_mats() and get_trans()), a [...,4,4] tensor or a [...,7] tensor."""
    if frames is None:
        return None, None
    if hasattr(frames, "get_rots"):
        rots, trans = frames.get_rots().get_rot_mats(), frames.get_trans()
    elif torch.is_tensor(frames) and frames.shape[-2:] == (4, 4):
        rots, trans = frames[..., :3, :3], frames[..., :3, 3]
    elif torch.is_tensor(frames) and frames.shape[-1] == 7:
        rots, trans = quat_to_rot(frames[..., :4].float()), frames[..., 4:]
    else:
        raise TypeError(f"unsupported frames object {type(frames)}")
    rots, trans = rots.float(), trans.float()
    if device is not None:
        rots, trans = rots.to(device), trans.to(device)
    return rots.contiguous(), trans.contiguous()
