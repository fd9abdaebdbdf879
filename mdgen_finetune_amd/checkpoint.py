"""Checkpoints in the reference's on-disk shape (a PyTorch-Lightning ``.ckpt``): a dict with
``state_dict`` (the wrapper's parameters, every key prefixed ``model.``), ``hyper_parameters``
{``args``: the train-time Namespace} (wrapper.py:50 ``save_hyperparameters``), ``epoch``,
``global_step``, ``optimizer_states`` and — with --ema — ``ema`` = {``params``, ``decay``}
(wrapper.py:120-130).

Loading never unpickles arbitrary objects: ``torch.load(weights_only=True)`` with
``argparse.Namespace`` as the only allow-listed class.  A reference checkpoint that stores
other Python classes in its hyper-parameters is refused with the loader's message; pass the
train-time args explicitly in that case (``load_from_checkpoint(path, args=...)``)."""
from __future__ import annotations

import argparse
import os

import torch

PREFIX = "model."


def _safe_load(path, map_location="cpu"):
    with torch.serialization.safe_globals([argparse.Namespace]):
        return torch.load(path, map_location=map_location, weights_only=True)


def save_checkpoint(path, wrapper, optimizer=None, epoch=0, global_step=0, epoch_complete=True, batches_done=0,
                    grad_scaler=None):
    """Lightning layout; ``args`` is stored as a Namespace of plain values.  ``loops`` records
    where in the epoch the save happened (a mid-epoch save, e.g. at --max_steps, resumes the
    same epoch after its ``batches_done`` consumed batches, as Lightning's fit loop does)."""
    if wrapper.cached_weights is not None:  # wrapper.py:126-129
        wrapper.restore_cached_weights()
    args = argparse.Namespace(**{k: v for k, v in vars(wrapper.args).items()
                                 if isinstance(v, (int, float, str, bool, type(None)))})
    ckpt = {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": "2.1.0",
        "state_dict": {PREFIX + k: v.detach().cpu() for k, v in wrapper.model.state_dict().items()},
        "hyper_parameters": {"args": args},
        "optimizer_states": [optimizer.state_dict()] if optimizer is not None else [],
        "lr_schedulers": [],
        "loops": {"fit_loop": {"epoch_complete": bool(epoch_complete), "batches_done": int(batches_done)}},
    }
    if grad_scaler is not None:  # --precision 16-mixed: the loss-scale state (Lightning's precision-plugin entry)
        ckpt["MixedPrecision"] = grad_scaler
    if wrapper.ema is not None:
        ema = wrapper.ema.state_dict()
        ckpt["ema"] = {"params": {k: v.detach().cpu() for k, v in ema["params"].items()},
                       "decay": float(ema["decay"])}
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save(ckpt, tmp)
    os.replace(tmp, path)


def load_checkpoint(path, map_location="cpu"):
    return _safe_load(path, map_location)


def model_state_dict(ckpt):
    """The ``model.*`` entries of a checkpoint's state_dict, prefix stripped."""
    sd = ckpt["state_dict"]
    return {k[len(PREFIX):]: v for k, v in sd.items() if k.startswith(PREFIX)}


def load_from_checkpoint(path, args=None, map_location="cpu", strict=True):
    """``NewMDGenWrapper.load_from_checkpoint`` (sim_inference.py:130): rebuild the wrapper
    from the stored args (or ``args``), load the weights, and the EMA state when present."""
    from .wrapper import NewMDGenWrapper

    ckpt = _safe_load(path, map_location)
    if args is None:
        args = ckpt["hyper_parameters"]["args"]
    w = NewMDGenWrapper(args)
    w.model.load_state_dict(model_state_dict(ckpt), strict=strict)
    if w.ema is not None and "ema" in ckpt:
        w.ema.load_state_dict(ckpt["ema"])
    return w
