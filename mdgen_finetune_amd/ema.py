"""Exponential moving average of the model's state_dict (reference src/mdgen/ema.py, the
OpenFold EMA): copy <- copy - (1 - decay)·(copy - param) after every optimizer step
(wrapper.py:78-80 on_before_zero_grad); ``state_dict()`` = {"params", "decay"} as stored
under a checkpoint's "ema" key."""
from __future__ import annotations

from collections import OrderedDict

import torch


class ExponentialMovingAverage:
    def __init__(self, model: torch.nn.Module, decay: float):
        self.params = OrderedDict((k, v.detach().clone()) for k, v in model.state_dict().items())
        self.decay = decay
        self.device = next(model.parameters()).device

    def to(self, device):
        self.params = OrderedDict((k, v.to(device)) for k, v in self.params.items())
        self.device = device
        return self

    @torch.no_grad()
    def update(self, model: torch.nn.Module) -> None:
        """stored -= (stored - v) * w per floating tensor (ema.py's update), as ONE multi-tensor
        lerp pass: stored + w (v - stored) is the same update (within an ulp; the per-tensor form
        cost 3 launches per tensor, a three-pass foreach form 2.7x the bytes of this one)."""
        w = 1.0 - self.decay
        fs, fv = [], []
        for k, v in model.state_dict().items():
            stored = self.params[k]
            if torch.is_floating_point(stored):
                fs.append(stored)
                fv.append(v)
            else:
                stored.copy_(v)
        if fs:
            torch._foreach_lerp_(fs, fv, w)

    def load_state_dict(self, state_dict) -> None:
        for k, v in state_dict["params"].items():
            self.params[k] = v.clone()
        self.decay = state_dict["decay"]

    def state_dict(self):
        return OrderedDict(params=self.params, decay=self.decay)
