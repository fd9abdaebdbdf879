"""Training / inference glue around the denoiser: the drop-in for the reference's
``NewMDGenWrapper`` (src/mdgen/wrapper.py:46-515) without PyTorch Lightning.

What it keeps from the reference, call for call:
  * ``prep_batch(batch)`` (wrapper.py:283-365): rigid offsets to frame 0 (``get_offsets``,
    utils.py:7-14) with the real-part sign fix (309), torsions appended as (cos, sin) pairs,
    loss mask ``[frame 7 | torsion 14]`` broadcast over T, the conditioning mask (frame 0 for
    --sim_condition; frames 0 and -1 for --tps_condition, which also appends the offsets to the
    last frame), ``x_cond = where(cond, latents, 0)``;
  * ``general_step(batch)`` (367-403): GVP flow-matching loss through
    ``Transport.training_losses``; returns the batch-mean loss;
  * ``inference(batch, zs0=None)`` (436-508): prior noise, ``Sampler.sample_ode`` with
    ``partial(model.forward_inference, **model_kwargs)`` (the HIP fast path on a GPU), last
    state; returns the sampled offsets/torsions and the frames composed onto frame 0;
  * optimizer (Adam / AdamW, 167-173), EMA (78-80), checkpoint hooks (120-130).

The Lightning trainer loop itself is replaced by ``mdgen_finetune_amd.train`` (DDP, one
process per GPU over RCCL).
"""
from __future__ import annotations

import time
from collections import defaultdict
from functools import partial

import torch
from torch import nn

from .ema import ExponentialMovingAverage
from .model.latent_model import LatentMDGenModel
from .rigid_utils import Rigid, Rotation
from .transport import Sampler, create_transport

# wrapper.py:40-42
DESIGN_IDX = [1, 2]
COND_IDX = [0, 3]


def get_offsets(ref_frame: Rigid, rigids: Rigid) -> torch.Tensor:
    """utils.py:7-14: ``ref.invert().compose(rigids).to_tensor_7()`` (quaternion, translation)."""
    return ref_frame.invert().compose(rigids).to_tensor_7()


def prep_latents_hip(rots, trans, torsions, tps=False, no_offsets=False, cond_first=True, cond_last=False,
                     cond_interval=0):
    """latents / x_cond / cond_mask of prep_batch in one HIP launch (mdg_prep_latents): the
    relative frames, quaternions (eigenvector of K, sign-fixed) and torsions per token."""
    from . import _lib

    lib = _lib.load()
    B, T, L = trans.shape[:3]
    lat = 28 if tps else 21
    rots = rots.float().contiguous()
    trans = trans.float().contiguous()
    tors = torsions.float().contiguous() if torsions is not None else None
    dev = trans.device
    latents = torch.empty(B, T, L, lat, device=dev)
    x_cond = torch.empty_like(latents)
    cond = torch.empty(B, T, L, dtype=torch.int64, device=dev)
    flags = ((_lib.MDG_PREP_TPS if tps else 0) | (_lib.MDG_PREP_NO_OFFSETS if no_offsets else 0)
             | (_lib.MDG_PREP_COND_FIRST if cond_first else 0) | (_lib.MDG_PREP_COND_LAST if cond_last else 0))
    _lib.check(lib.mdg_prep_latents(B, T, L, lat, flags, int(cond_interval or 0), rots.data_ptr(), trans.data_ptr(),
                                    _lib.ptr(tors), latents.data_ptr(), x_cond.data_ptr(), cond.data_ptr(),
                                    _lib.stream_handle()), "mdg_prep_latents")
    return latents, x_cond, cond


def fix_quat_sign_(offsets: torch.Tensor) -> torch.Tensor:
    """wrapper.py:309: make the quaternion's real part non-negative (in place on [..., :4])."""
    offsets[..., :4] *= torch.where(offsets[..., 0:1] < 0, -1, 1)
    return offsets


class NewMDGenWrapper(nn.Module):
    """wrapper.py:175-515 (frames + torsions variant; no design / no_frames / hyena)."""

    def __init__(self, args):
        super().__init__()
        for key in ("inpainting", "no_torsion", "hyena", "no_aa_emb", "supervise_all_torsions",
                    "supervise_no_torsions", "design_key_frames", "no_design_torsion", "cond_interval",
                    "mpnn", "dynamic_mpnn", "no_offsets", "no_frames", "design", "ema"):
            if not hasattr(args, key):  # wrapper.py:178-197
                setattr(args, key, False)
        if args.no_frames or args.design_key_frames:
            raise NotImplementedError("--no_frames / --design_key_frames are outside this build (DESIGN.md §7)")
        self.args = args
        self.latent_dim = 28 if (args.tps_condition or args.inpainting or args.dynamic_mpnn) else 21
        self.model = LatentMDGenModel(args, self.latent_dim)
        self.transport = create_transport(args, args.path_type, args.prediction, None)
        self.transport_sampler = Sampler(self.transport)
        self.ema = ExponentialMovingAverage(self.model, args.ema_decay) if args.ema else None
        self.cached_weights = None
        self._log = defaultdict(list)
        self.stage = "train"
        self.iter_step = 0
        self.last_log_time = time.time()

    @property
    def device(self):
        return next(self.model.parameters()).device

    # ------------------------------------------------------------------ logging (wrapper.py:56-62)
    def log(self, key, data):
        if isinstance(data, torch.Tensor):
            data = data.mean().item()
        if self.stage == "train" or getattr(self.args, "validate", False):
            self._log["iter_" + key].append(data)
        self._log[self.stage + "_" + key].append(data)

    # ------------------------------------------------------------------ batch preparation
    def prep_batch(self, batch):
        """wrapper.py:283-365.  On a ROCm device the offsets / quaternions / latents / x_cond
        come from one HIP launch (mdg_prep_latents) instead of the reference's per-frame CPU
        eigen-solve; CPU tensors take the eager path below."""
        a = self.args
        rigids = Rigid(Rotation(rot_mats=batch["rots"]), batch["trans"])  # B, T, L
        B, T, L = rigids.shape
        tps = bool(a.tps_condition or a.inpainting or a.dynamic_mpnn)
        frame_loss_mask = batch["mask"].unsqueeze(-1).expand(-1, -1, 7)
        torsion_loss_mask = batch["torsion_mask"].unsqueeze(-1).expand(-1, -1, -1, 2).reshape(B, L, 14)
        if tps:
            frame_loss_mask = torch.cat([frame_loss_mask, frame_loss_mask], -1)
        tors = batch["torsions"].reshape(B, T, L, 14)
        if a.no_torsion:
            tors = torch.zeros_like(tors)
        elif a.no_design_torsion:
            tors = batch["torsions"].clone()
            tors[:, :, DESIGN_IDX] = 0
            tors = tors.reshape(B, T, L, 14)
        simple_cond = not (a.inpainting or a.dynamic_mpnn or a.mpnn)
        if batch["trans"].is_cuda and simple_cond:
            latents, x_cond, cond_mask = prep_latents_hip(
                batch["rots"], batch["trans"], tors, tps=tps, no_offsets=bool(a.no_offsets),
                cond_first=bool(a.sim_condition or a.tps_condition), cond_last=bool(a.tps_condition),
                cond_interval=a.cond_interval or 0)
        else:
            offsets = rigids.to_tensor_7() if a.no_offsets else get_offsets(rigids[:, 0:1], rigids)
            fix_quat_sign_(offsets)
            if tps:
                offsets_r = fix_quat_sign_(get_offsets(rigids[:, -1:], rigids))
                offsets = torch.cat([offsets, offsets_r], -1)
            latents = torch.cat([offsets, tors.to(offsets.dtype)], -1)
            cond_mask = torch.zeros(B, T, L, dtype=torch.int64, device=offsets.device)
            if a.sim_condition:
                cond_mask[:, 0] = 1
            if a.tps_condition:
                cond_mask[:, 0] = 1
                cond_mask[:, -1] = 1
            if a.cond_interval:
                cond_mask[:, ::a.cond_interval] = 1
            if a.inpainting or a.dynamic_mpnn or a.mpnn:
                cond_mask[:, :, COND_IDX] = 1
            x_cond = torch.where(cond_mask.unsqueeze(-1).bool(), latents, 0.0)
        if a.supervise_all_torsions:
            torsion_loss_mask = torch.ones_like(torsion_loss_mask)
        elif a.supervise_no_torsions:
            torsion_loss_mask = torch.zeros_like(torsion_loss_mask)
        loss_mask = torch.cat([frame_loss_mask, torsion_loss_mask], -1).unsqueeze(1).expand(-1, T, -1, -1)
        aatype_mask = torch.ones_like(batch["seqres"])
        if a.design:
            aatype_mask[:, DESIGN_IDX] = 0
        return {
            "rigids": rigids,
            "latents": latents,
            "loss_mask": loss_mask,
            "model_kwargs": {
                "start_frames": rigids[:, 0],
                "end_frames": rigids[:, -1],
                "mask": batch["mask"].unsqueeze(1).expand(-1, T, -1),
                "aatype": torch.where(aatype_mask.bool(), batch["seqres"], 20),
                "x_cond": x_cond,
                "x_cond_mask": cond_mask,
            },
        }

    # ------------------------------------------------------------------ training step
    def general_step(self, batch, stage="train", model=None, log=True):
        """wrapper.py:367-403.  ``model`` is the module the loss differentiates through (the
        DDP wrapper of ``self.model`` in data-parallel training).  ``log=False`` (inside a graph
        capture, where .item() cannot sync) returns (batch-mean loss, per-sample losses, t)
        and leaves the logging to the caller (Trainer.log_step)."""
        self.iter_step += 1
        self.stage = stage
        start1 = time.time()
        prep = self.prep_batch(batch)
        start = time.time()
        out = self.transport.training_losses(model=model if model is not None else self.model,
                                             x1=prep["latents"], aatype1=None, mask=prep["loss_mask"],
                                             model_kwargs=prep["model_kwargs"])
        loss = out["loss"]
        if not log:
            return loss.mean(), loss, out["t"]
        self.log("model_dur", time.time() - start)
        self.log("loss", loss)
        self.log("time", out["t"])
        self.log("dur", time.time() - self.last_log_time)
        self.log("general_step_dur", time.time() - start1)
        self.last_log_time = time.time()
        return loss.mean()

    # ------------------------------------------------------------------ sampling
    def sample_prior_latent(self, B, T, L, device=None, uniform=False):
        """wrapper.py:416-434 (continuous latents)."""
        device = device or self.device
        if uniform:
            return 6 * torch.rand(B, T, L, self.latent_dim, device=device) - 3
        return torch.randn(B, T, L, self.latent_dim, device=device)

    @torch.no_grad()
    def sample_latents(self, batch, zs0=None):
        """wrapper.py:436-478: the last ODE state [B, T, L, latent] and the prepared batch."""
        prep = self.prep_batch(batch)
        B, T, L = prep["rigids"].shape
        zs = zs0 if zs0 is not None else self.sample_prior_latent(B, T, L, prep["latents"].device)
        sample_fn = self.transport_sampler.sample_ode(sampling_method=self.args.sampling_method)
        samples = sample_fn(zs, partial(self.model.forward_inference, **prep["model_kwargs"]))[-1]
        return samples, prep

    @torch.no_grad()
    def inference(self, batch, zs0=None):
        """wrapper.py:436-508: (atom14 [B,T,L,14,3], aatype [B,T,L]).  On a ROCm device the
        offsets -> frames -> 8 group frames -> 14 atoms reconstruction is one HIP launch
        (mdg_latents_to_atom14); CPU tensors take the torch restatement (geometry.py)."""
        from . import geometry as G

        samples, prep = self.sample_latents(batch, zs0)
        B, T, L, _ = samples.shape
        r0 = prep["rigids"][:, 0]
        ref_rots, ref_trans = r0.get_rots().get_rot_mats(), r0.get_trans()
        aa = batch["seqres"][:, None].expand(B, T, L)
        tps = bool(self.args.tps_condition or self.args.inpainting)
        if self.args.no_offsets:
            raise NotImplementedError("--no_offsets rollout reconstruction is outside this build")
        if samples.is_cuda:
            atom14 = G.latents_to_atom14_hip(samples, ref_rots, ref_trans, aa, tps=tps, renorm=not self.args.oracle)
        else:
            rots, trans, tors = G.latents_to_frames_torsions(samples, ref_rots, ref_trans, tps=tps,
                                                             renorm=not self.args.oracle)
            atom14 = G.frames_torsions_to_atom14(rots, trans, tors, aa)
        return atom14, aa

    # ------------------------------------------------------------------ optimizer / EMA / ckpt
    def configure_optimizers(self, params=None, capturable=False):
        """wrapper.py:167-173 (capturable: the step count on the device, for a graphed step).

        The graphed step uses the fused Adam kernel (a handful of multi-tensor launches): the
        capturable foreach form falls back to per-tensor kernels for its 0-d step / bias-correction
        arithmetic, ~600 launches per step for the model's 289 tensors (profiles/r03_train_kernels.md).
        The fused update does not bump the parameters' version counters; GraphedStep.run tells the
        inference engine's weight cache instead (model._weights_gen)."""
        cls = torch.optim.AdamW if self.args.adamW else torch.optim.Adam
        params = params if params is not None else self.model.parameters()
        kw = {"capturable": True, "fused": True} if capturable else {}
        return cls([p for p in params if p.requires_grad], lr=self.args.lr, **kw)

    def on_before_zero_grad(self):
        """wrapper.py:78-80."""
        if self.ema is not None:
            if self.ema.device != self.device:
                self.ema.to(self.device)
            self.ema.update(self.model)

    def load_ema_weights(self):
        """wrapper.py:64-71."""
        self.cached_weights = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        self.model.load_state_dict(self.ema.state_dict()["params"])

    def restore_cached_weights(self):
        """wrapper.py:73-76."""
        self.model.load_state_dict(self.cached_weights)
        self.cached_weights = None
