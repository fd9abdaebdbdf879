"""SiT flow-matching transport: the drop-in for reference src/mdgen/transport/transport.py
(create_transport 513-574, Transport.training_losses 137-222, Sampler.sample_ode 407-450)
with the GVP and Linear paths (path.py:113-135, 173-191) and velocity prediction — the
combinations the MDGen configs select.

``Sampler.sample_ode(sampling_method='euler')`` returns a function with the reference's
signature ``fn(x0, model_callable, **kw) -> Tensor[num_steps, ...]``.  When
``model_callable`` is ``partial(model.forward_inference, **model_kwargs)`` of this package's
LatentMDGenModel on the HIP backend, the whole solve is delegated to
``HipEngine.sample_euler`` (conditioning for all steps precomputed, the 49 steps captured in
one hipGraph); any other callable runs the same fixed-grid Euler loop step by step.
"""
from __future__ import annotations

import enum
import functools

import numpy as np
import torch as th


class ModelType(enum.Enum):
    NOISE = enum.auto()
    SCORE = enum.auto()
    VELOCITY = enum.auto()


class PathType(enum.Enum):
    LINEAR = enum.auto()
    GVP = enum.auto()
    VP = enum.auto()


class WeightType(enum.Enum):
    NONE = enum.auto()
    VELOCITY = enum.auto()
    LIKELIHOOD = enum.auto()


def mean_flat(x, mask):
    """transport.py:12-16."""
    dims = list(range(1, len(x.size())))
    return th.sum(x * mask, dim=dims) / th.sum(mask, dim=dims)


def _expand_t_like_x(t, x):
    return t.view(t.size(0), *([1] * (x.dim() - 1)))


class ICPlan:
    """Linear path (path.py:81-150): alpha = t, sigma = 1 - t."""

    def compute_alpha_t(self, t):
        return t, 1

    def compute_sigma_t(self, t):
        return 1 - t, -1

    def plan(self, t, x0, x1):
        te = _expand_t_like_x(t, x1)
        a, da = self.compute_alpha_t(te)
        s, ds = self.compute_sigma_t(te)
        return t, a * x1 + s * x0, da * x1 + ds * x0


class GVPCPlan(ICPlan):
    """path.py:173-191: alpha = sin(pi t/2), sigma = cos(pi t/2)."""

    def compute_alpha_t(self, t):
        return th.sin(t * np.pi / 2), np.pi / 2 * th.cos(t * np.pi / 2)

    def compute_sigma_t(self, t):
        return th.cos(t * np.pi / 2), -np.pi / 2 * th.sin(t * np.pi / 2)


class Transport:
    def __init__(self, *, args, model_type, path_type, loss_type, train_eps, sample_eps):
        if model_type != ModelType.VELOCITY or path_type == PathType.VP:
            raise NotImplementedError("only velocity prediction on the GVP / Linear paths is built "
                                      "(the configs never select score/noise/VP; DESIGN.md §Scope)")
        self.args = args
        self.model_type, self.loss_type = model_type, loss_type
        self.path_sampler = GVPCPlan() if path_type == PathType.GVP else ICPlan()
        self.train_eps, self.sample_eps = train_eps, sample_eps

    def check_interval(self, train_eps, sample_eps, *, diffusion_form="SBDM", sde=False, reverse=False,
                       eval=False, last_step_size=0.0):
        """transport.py:94-123 for velocity + GVP/Linear ODE: [0, 1]."""
        t0, t1 = 0, 1
        if sde:
            eps = train_eps if not eval else sample_eps
            t1 = 1 - eps if last_step_size == 0 else 1 - last_step_size
        if reverse:
            t0, t1 = 1 - t0, 1 - t1
        return t0, t1

    def sample(self, x1):
        """transport.py:125-135 (RNG order: x0 = randn_like(x1), then t).  The reference draws t
        on the CPU generator and copies it over; inside a graph capture (the graphed training
        step) a host-to-device copy cannot be recorded, so t is drawn on x1's device there
        (same distribution, the device generator's graph-safe stream)."""
        x0 = th.randn_like(x1)
        t0, t1 = self.check_interval(self.train_eps, self.sample_eps)
        if x1.is_cuda and th.cuda.is_current_stream_capturing():
            t = th.rand((x1.shape[0],), device=x1.device) * (t1 - t0) + t0
        else:
            t = th.rand((x1.shape[0],)) * (t1 - t0) + t0
        return t.to(x1), x0, x1

    def training_losses(self, model, x1, aatype1=None, mask=None, model_kwargs=None):
        """transport.py:137-222 (velocity branch): {'t', 'pred', 'loss'}."""
        if model_kwargs is None:
            model_kwargs = {}
        t, x0, x1 = self.sample(x1)
        if _hip_loss_ok(model, x1, mask):  # the plan and the loss as library launches (train_glue.hip)
            from ..train_hip import gvp_loss, gvp_plan

            xt, ut = gvp_plan(t, x0, x1, 0 if isinstance(self.path_sampler, GVPCPlan) else 1)
            out = model(xt, t, **model_kwargs)
            assert out.size() == xt.size()
            return {"t": t, "pred": out, "loss": gvp_loss(out, ut, mask)}
        t, xt, ut = self.path_sampler.plan(t, x0, x1)
        out = model(xt, t, **model_kwargs)
        assert out.size() == xt.size()
        return {"t": t, "pred": out, "loss": mean_flat((out - ut) ** 2, mask)}

    def get_drift(self):
        def body_fn(x, t, model, **model_kwargs):
            out = model(x, t, **model_kwargs)
            assert out.shape == x.shape, "Output shape from ODE solver must match input shape"
            return out

        return body_fn


def _hip_loss_ok(model, x1, mask):
    """The fused plan / loss serve the HIP training path: a CUDA fp32 batch under autograd, a model
    whose backend and train_backend are 'hip' (a DDP wrapper's .module counts), a [B,T,L,K]-
    broadcastable fp32 mask (MDG_TRAIN_GVP=0: eager)."""
    import os

    m = getattr(model, "module", model)
    if os.environ.get("MDG_TRAIN_GVP", "1") == "0" or not (x1.is_cuda and th.is_grad_enabled()):
        return False
    if getattr(m, "backend", None) != "hip" or getattr(m, "train_backend", None) != "hip":
        return False
    return (x1.dtype == th.float32 and x1.dim() == 4 and mask is not None and mask.dtype == th.float32
            and mask.dim() == 4)


def _hip_model_of(model, x):
    """(LatentMDGenModel, kwargs) if `model` is partial(m.forward_inference|m.forward, **kw) of
    our module on the HIP backend, else None."""
    if not isinstance(model, functools.partial) or model.args:
        return None
    fn = model.func
    owner = getattr(fn, "__self__", None)
    from ..model.latent_model import LatentMDGenModel

    if not isinstance(owner, LatentMDGenModel) or fn.__name__ not in ("forward_inference", "forward"):
        return None
    if not owner._use_hip(x):
        return None
    return owner, dict(model.keywords)


class Sampler:
    def __init__(self, transport):
        self.transport = transport
        self.drift = transport.get_drift()

    def sample_ode(self, *, sampling_method="dopri5", num_steps=50, atol=1e-6, rtol=1e-3, reverse=False):
        """transport.py:407-450 + integrators.py:74-114: 'euler' (fixed grid of num_steps points)
        or 'dopri5' (adaptive, num_steps saved points; integrators.odeint_dopri5)."""
        if sampling_method not in ("euler", "dopri5"):
            raise NotImplementedError(f"sampling_method={sampling_method!r}: the reference offers "
                                      "'dopri5' and 'euler' (parsing.py:102)")
        t0, t1 = self.transport.check_interval(self.transport.train_eps, self.transport.sample_eps,
                                               sde=False, eval=True, reverse=reverse)
        drift = self.drift
        if reverse:
            drift = lambda x, t, model, **kw: self.drift(x, th.ones_like(t) * (1 - t), model, **kw)  # noqa: E731

        if sampling_method == "dopri5":
            def _sample_dopri5(x, model, **model_kwargs):
                hip = None if (reverse or model_kwargs) else _hip_model_of(model, x)
                if hip is not None:  # each evaluation = one hipGraph replay (HipEngine.velocity_field)
                    m, kw = hip
                    from ..engine import get_engine

                    mask = kw.get("mask")
                    if mask is not None and mask.dim() == 2:
                        mask = mask.repeat(x.shape[0], 1, 1)
                    fn = get_engine(m).velocity_field(
                        x, mask=mask, start_frames=kw.get("start_frames"), end_frames=kw.get("end_frames"),
                        x_cond=kw.get("x_cond"), x_cond_mask=kw.get("x_cond_mask"), aatype=kw.get("aatype"))
                    from .integrators import odeint_dopri5_graphed

                    ts = th.linspace(t0, t1, num_steps).to(x.device)
                    # the whole adaptive step (6 evaluations + accept / reject) is one hipGraph
                    return odeint_dopri5_graphed(fn.capturable, x, ts, rtol=rtol, atol=atol, f0_func=fn,
                                                 stats=getattr(self, "dopri5_stats", None))
                else:
                    def fn(t, y):  # integrators.py:98-101
                        return drift(y, th.ones(y.size(0)).to(y.device) * t, model, **model_kwargs)
                from .integrators import odeint_dopri5

                ts = th.linspace(t0, t1, num_steps).to(x.device)
                return odeint_dopri5(fn, x, ts, rtol=rtol, atol=atol)

            return _sample_dopri5

        def _sample(x, model, **model_kwargs):
            hip = None if (reverse or model_kwargs or (t0, t1) != (0, 1)) else _hip_model_of(model, x)
            if hip is not None:
                m, kw = hip
                from ..engine import get_engine

                mask = kw.get("mask")
                if mask is not None and mask.dim() == 2:
                    mask = mask.repeat(x.shape[0], 1, 1)
                return get_engine(m).sample_euler(
                    x, num_steps=num_steps, mask=mask, start_frames=kw.get("start_frames"),
                    end_frames=kw.get("end_frames"), x_cond=kw.get("x_cond"), x_cond_mask=kw.get("x_cond_mask"),
                    aatype=kw.get("aatype"))
            ts = th.linspace(t0, t1, num_steps).to(x.device)
            ys = [x]
            y = x
            for i in range(num_steps - 1):
                tt = th.ones(x.size(0)).to(x.device) * ts[i]
                y = y + (ts[i + 1] - ts[i]) * drift(y, tt, model, **model_kwargs)
                ys.append(y)
            return th.stack(ys)

        return _sample


def create_transport(args=None, path_type="Linear", prediction="velocity", loss_weight=None, train_eps=None,
                     sample_eps=None):
    """transport.py:513-574."""
    model_type = {"noise": ModelType.NOISE, "score": ModelType.SCORE}.get(prediction, ModelType.VELOCITY)
    loss_type = {"velocity": WeightType.VELOCITY, "likelihood": WeightType.LIKELIHOOD}.get(loss_weight,
                                                                                          WeightType.NONE)
    path_type = {"Linear": PathType.LINEAR, "GVP": PathType.GVP, "VP": PathType.VP}[path_type]
    return Transport(args=args, model_type=model_type, path_type=path_type, loss_type=loss_type,
                     train_eps=0 if train_eps is None else train_eps, sample_eps=0 if sample_eps is None else sample_eps)
