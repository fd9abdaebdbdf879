"""Portable, seed-derived synthetic weights and inputs.

The GPU box has no checkpoint and no network, and the reference never travels there, so
every parity case and every benchmark regenerates its weights from a seed with this module.
The generator is counter-based (splitmix64 over (seed, fnv1a64(param name), index)) and
implemented in numpy uint64 arithmetic, so it yields the same bits on any host and in any
order of parameter creation; the golden fixtures under tests/golden/ were produced by the
reference model with weights from exactly this generator (oracle/gen_golden.py).

Scale rules (by state-dict name; the reference's zero-inits at latent_model.py:144-177 are
deliberately NOT kept — a zero-initialised adaLN / final layer would make every output 0):
  * 2-D ``*.weight`` (Linear):  U(-1,1) * sqrt(3 / fan_in)       (unit-variance outputs)
  * ``*.bias``:                 U(-1,1) * 0.1
  * nn.Embedding tables (``mask_to_emb``, ``aatype_to_emb``): U(-1,1) * 0.5
  * affine LayerNorm ``*norm.weight`` 1 + 0.1 U, ``*norm.bias`` 0.1 U
  * ``bias_k`` / ``bias_v``:     U(-1,1)
  * IPA ``head_weights``:        0.541324854612918 + 0.2 U   (softplus^-1(1) ± 0.2)
Buffers (``pos_embed``, ``rot_emb.inv_freq``) are never touched.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _fnv1a64(s: str) -> np.uint64:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return np.uint64(h)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, key: str, n: int) -> np.ndarray:
    """n float64 values in [-1, 1), a pure function of (seed, key, index)."""
    base = _splitmix64(np.array([seed], dtype=np.uint64))[0] ^ _fnv1a64(key)
    with np.errstate(over="ignore"):
        ctr = base + np.arange(n, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03)
    z = _splitmix64(ctr)
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return 2.0 * u - 1.0


def param_value(seed: int, name: str, shape) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    u = uniform(seed, name, n).reshape(shape)
    leaf = name.rsplit(".", 1)[-1]
    if leaf in ("bias_k", "bias_v"):
        v = u
    elif leaf == "head_weights":
        v = 0.541324854612918 + 0.2 * u
    elif leaf == "weight" and ("norm" in name.rsplit(".", 2)[-2]):
        v = 1.0 + 0.1 * u
    elif leaf == "bias" and ("norm" in name.rsplit(".", 2)[-2]):
        v = 0.1 * u
    elif leaf == "weight" and name.rsplit(".", 2)[-2] in ("mask_to_emb", "aatype_to_emb"):
        v = 0.5 * u
    elif leaf == "weight" and len(shape) == 2:
        v = u * np.sqrt(3.0 / shape[1])
    elif leaf == "bias":
        v = 0.1 * u
    else:
        v = 0.1 * u
    return v.astype(np.float32)


def fill_module_(module, seed: int) -> None:
    """Overwrite every *parameter* (not buffer) of a torch module in place."""
    import torch

    with torch.no_grad():
        for name, p in module.named_parameters():
            p.copy_(torch.from_numpy(param_value(seed, name, p.shape)))


# --------------------------------------------------------------------------- inputs
def quat_to_rotmat(q: np.ndarray) -> np.ndarray:
    """Unit quaternion (w,x,y,z) -> rotation matrix (same convention as the reference's
    rigid_utils.quat_to_rot, rigid_utils.py:155-189)."""
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    a, b, c, d = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    r = np.empty(q.shape[:-1] + (3, 3), dtype=np.float64)
    r[..., 0, 0] = a * a + b * b - c * c - d * d
    r[..., 0, 1] = 2 * (b * c - a * d)
    r[..., 0, 2] = 2 * (b * d + a * c)
    r[..., 1, 0] = 2 * (b * c + a * d)
    r[..., 1, 1] = a * a - b * b + c * c - d * d
    r[..., 1, 2] = 2 * (c * d - a * b)
    r[..., 2, 0] = 2 * (b * d - a * c)
    r[..., 2, 1] = 2 * (c * d + a * b)
    r[..., 2, 2] = a * a - b * b - c * c + d * d
    return r


def make_inputs(seed: int, B: int, T: int, L: int, latent_dim: int = 21, tps: bool = False,
                n_pad: int = 0):
    """Synthetic forward-sim (or TPS) inputs in the reference's call shape.

    Returns a dict of numpy arrays:
      x [B,T,L,latent] f32 ~ N(0,1); t [B] f32; mask [B,T,L] f32 (last n_pad residues 0);
      rots/trans (start frames) [B,L,3,3]/[B,L,3]; end_rots/end_trans (TPS);
      x_cond [B,T,L,latent] (frame 0, and frame -1 for TPS; zeros elsewhere);
      x_cond_mask [B,T,L] int64; aatype [B,L] int64 in [0,20).
    """
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, T, L, latent_dim)).astype(np.float32)
    t = rng.uniform(0.0, 1.0, size=(B,)).astype(np.float32)
    mask = np.ones((B, T, L), np.float32)
    if n_pad:
        mask[:, :, L - n_pad:] = 0.0
    q = rng.standard_normal((B, L, 4))
    rots = quat_to_rotmat(q).astype(np.float32)
    trans = (5.0 * rng.standard_normal((B, L, 3))).astype(np.float32)
    q2 = rng.standard_normal((B, L, 4))
    end_rots = quat_to_rotmat(q2).astype(np.float32)
    end_trans = (5.0 * rng.standard_normal((B, L, 3))).astype(np.float32)
    cond_mask = np.zeros((B, T, L), np.int64)
    cond_mask[:, 0] = 1
    if tps:
        cond_mask[:, -1] = 1
    lat = rng.standard_normal((B, T, L, latent_dim)).astype(np.float32)
    # torsion part as (cos, sin) pairs like prep_batch produces (wrapper.py:311-330)
    n_off = 14 if tps else 7
    ang = rng.uniform(-np.pi, np.pi, size=(B, T, L, (latent_dim - n_off) // 2))
    lat[..., n_off::2] = np.cos(ang)
    lat[..., n_off + 1::2] = np.sin(ang)
    x_cond = np.where(cond_mask[..., None].astype(bool), lat, 0.0).astype(np.float32)
    aatype = rng.integers(0, 20, size=(B, L)).astype(np.int64)
    return dict(x=x, t=t, mask=mask, rots=rots, trans=trans, end_rots=end_rots,
                end_trans=end_trans, x_cond=x_cond, x_cond_mask=cond_mask, aatype=aatype)
