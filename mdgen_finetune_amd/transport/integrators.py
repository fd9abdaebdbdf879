"""Adaptive Dormand–Prince (dopri5) ODE solver: the reference's default
``--sampling_method`` (parsing.py:102; ``ode.sample`` integrators.py:95-114 hands it to
``torchdiffeq.odeint(method='dopri5', atol=[1e-6], rtol=[1e-3])``, transport.py:407-450).

torchdiffeq 0.2.5 is not in the container, so this restates its published algorithm
(``RKAdaptiveStepsizeODESolver`` + ``Dopri5Solver``, torchdiffeq/_impl/rk_common.py and
dopri5.py) — parity against torchdiffeq itself is unpinned:

  * state dtype = y0's (fp32), time dtype = float64 (``promote_types(float64, y0.dtype)``);
  * first step from ``_select_initial_step`` (Hairer–Nørsett–Wanner II.4), order 4;
  * the 7-stage FSAL Dormand–Prince tableau, stage times t0 + alpha_i·dt except alpha = 1,
    which evaluates one ulp below t1 (``Perturb.PREV``);
  * error ratio = RMS(err / (atol + rtol·max(|y0|, |y1|))), accept iff ≤ 1;
  * step-size control: safety 0.9, ifactor 10, dfactor 0.2 (1 on accepted steps), exponent 1/5;
  * the requested output times are produced by the 4th-order dense interpolant fitted with
    the Shampine mid-point coefficients (``_interp_fit`` / ``_interp_evaluate``), so
    ``num_steps`` is the number of *saved* points, not of integration steps.

``func(t, y)`` receives t as a 0-dim tensor of y's dtype (torchdiffeq's ``_PerturbFunc``
casts it) and must return dy/dt shaped like y.  ``odeint_dopri5`` decides accept / reject on
the host after every step, as torchdiffeq does.  ``odeint_dopri5_graphed`` runs the same
arithmetic with the whole step — six stage evaluations, the error ratio, accept / reject
(``torch.where``) and the next step size — captured in ONE hipGraph, so a step is one replay
and one device→host read (the new t / dt, to decide whether the next output time is reached).
"""
from __future__ import annotations

import torch

# Dormand–Prince 5(4) tableau (torchdiffeq dopri5.py _DORMAND_PRINCE_SHAMPINE_TABLEAU)
_ALPHA = [1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0, 1.0]
_BETA = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
_C_ERROR = [
    35 / 384 - 1951 / 21600,
    0.0,
    500 / 1113 - 22642 / 50085,
    125 / 192 - 451 / 720,
    -2187 / 6784 - -12231 / 42400,
    11 / 84 - 649 / 6300,
    -1.0 / 60.0,
]
# Shampine's mid-point weights for the dense output (DPS_C_MID)
_C_MID = [
    6025192743 / 30085553152 / 2, 0.0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
    187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2,
]
ORDER = 5


def rms_norm(x):
    return x.abs().pow(2).mean().sqrt()


def _weights(vals, y):
    return torch.tensor(vals, dtype=torch.float64).to(device=y.device, dtype=y.dtype)


def _combine(y0, ks, w, dt):
    """y0 + sum_j ks[j] * (w[j] * dt): the ``k.matmul(beta * dt)`` of rk_common.py, in y's
    dtype, with the weight·dt product formed first as the matmul against (beta·dt) does."""
    wd = w * dt
    acc = None
    for j, k in enumerate(ks):
        term = k * wd[j]
        acc = term if acc is None else acc + term
    return acc if y0 is None else y0 + acc


def _select_initial_step(func, t0, y0, f0, rtol, atol):
    """rk_common.py _select_initial_step (order = ORDER - 1)."""
    scale = atol + y0.abs() * rtol
    d0 = rms_norm(y0 / scale).abs()
    d1 = rms_norm(f0 / scale).abs()
    if d0 < 1e-5 or d1 < 1e-5:
        h0 = torch.tensor(1e-6, dtype=y0.dtype, device=y0.device)
    else:
        h0 = 0.01 * d0 / d1
    h0 = h0.abs()
    y1 = y0 + h0 * f0
    f1 = func(t0 + h0, y1)
    d2 = (rms_norm((f1 - f0) / scale) / h0).abs()
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = torch.max(torch.tensor(1e-6, dtype=y0.dtype, device=y0.device), h0 * 1e-3)
    else:
        h1 = (0.01 / torch.max(d1, d2)) ** (1.0 / float(ORDER))
    h1 = h1.abs()
    return torch.min(100 * h0, h1).to(torch.float64)


def _optimal_step_size(dt, error_ratio, safety=0.9, ifactor=10.0, dfactor=0.2):
    """rk_common.py _optimal_step_size: dt·min(ifactor, max(safety/ratio^(1/5), dfactor))."""
    if error_ratio == 0:
        return dt * ifactor
    if error_ratio < 1:
        dfactor = 1.0
    er = error_ratio.to(dt.dtype)
    return dt * torch.clamp(safety / er ** (1.0 / ORDER), min=dfactor, max=ifactor)


def _interp_fit(y0, y1, y_mid, f0, f1, dt):
    """misc.py _interp_fit: coefficients [e, d, c, b, a] of the 4th-order interpolant."""
    a = 2 * dt * (f1 - f0) - 8 * (y1 + y0) + 16 * y_mid
    b = dt * (5 * f0 - 3 * f1) + 18 * y0 + 14 * y1 - 32 * y_mid
    c = dt * (f1 - 4 * f0) - 11 * y0 - 5 * y1 + 16 * y_mid
    d = dt * f0
    return [y0, d, c, b, a]


def _interp_evaluate(coeffs, t0, t1, t):
    if not bool((t0 <= t) & (t <= t1)):
        raise AssertionError(f"invalid interpolation, fails {t0} <= {t} <= {t1}")
    x = ((t - t0) / (t1 - t0)).to(coeffs[0].dtype)
    total = coeffs[0] + x * coeffs[1]
    xp = x
    for c in coeffs[2:]:
        xp = xp * x
        total = total + xp * c
    return total


class Dopri5Stats:
    """Counters of one solve: function evaluations, accepted and rejected steps."""

    def __init__(self):
        self.nfe = 0
        self.accepted = 0
        self.rejected = 0


def odeint_dopri5(func, y0, t, rtol=1e-3, atol=1e-6, max_num_steps=2 ** 31 - 1, stats=None):
    """Solution at every time of the increasing grid ``t`` (shape [len(t), *y0.shape]), as
    ``torchdiffeq.odeint(func, y0, t, method='dopri5', rtol=rtol, atol=atol)``."""
    if not torch.is_floating_point(y0):
        raise TypeError("y0 must be floating point")
    t = torch.as_tensor(t).to(device=y0.device, dtype=torch.float64)
    if t.dim() != 1 or not bool((t[1:] > t[:-1]).all()):
        raise ValueError("t must be strictly increasing")
    rtol = float(torch.as_tensor(rtol, dtype=torch.float64).reshape(-1)[0])
    atol = float(torch.as_tensor(atol, dtype=torch.float64).reshape(-1)[0])
    st = stats if stats is not None else Dopri5Stats()

    def f(tt, yy, prev=False):
        tt = tt.to(yy.dtype)
        if prev:  # Perturb.PREV: the largest representable value below t1
            tt = torch.nextafter(tt, tt - 1)
        st.nfe += 1
        return func(tt, yy)

    beta = [_weights(b, y0) for b in _BETA]
    c_err = _weights(_C_ERROR, y0)
    c_mid = _weights(_C_MID, y0)

    sol = torch.empty(len(t), *y0.shape, dtype=y0.dtype, device=y0.device)
    sol[0] = y0
    t0 = t[0]
    f0 = f(t0, y0)
    dt = _select_initial_step(f, t0, y0, f0, rtol, atol)
    y, fy, t_lo, t_hi, coeffs = y0, f0, t0, t0, [y0] * 5
    n_steps = 0
    for i in range(1, len(t)):
        nt = t[i]
        while bool(nt > t_hi):
            if n_steps >= max_num_steps:
                raise AssertionError(f"max_num_steps exceeded ({n_steps}>={max_num_steps})")
            if not bool(t_hi + dt > t_hi):
                raise AssertionError(f"underflow in dt {dt.item()}")
            t1 = t_hi + dt
            dt_y = dt.to(y.dtype)
            ks = [fy]
            for a_i, b_i in zip(_ALPHA, beta):
                yi = _combine(y, ks, b_i, dt_y)
                if a_i == 1.0:
                    ks.append(f(t1, yi, prev=True))
                else:
                    ks.append(f(t_hi + a_i * dt, yi))
            y1 = yi  # FSAL: c_sol == beta[-1] and c_sol[-1] == 0
            err = _combine(None, ks, c_err, dt_y)
            tol = atol + rtol * torch.max(y.abs(), y1.abs())
            ratio = rms_norm(err / tol)
            if bool(ratio <= 1):
                y_mid = _combine(y, ks, c_mid, dt_y)
                coeffs = _interp_fit(y, y1, y_mid, ks[0], ks[-1], dt_y)
                t_lo, t_hi = t_hi, t1
                y, fy = y1, ks[-1]
                st.accepted += 1
            else:
                st.rejected += 1
            dt = _optimal_step_size(dt, ratio)
            n_steps += 1
        sol[i] = _interp_evaluate(coeffs, t_lo, t_hi, nt)
    return sol


def odeint_dopri5_graphed(func, y0, t, rtol=1e-3, atol=1e-6, max_num_steps=2 ** 31 - 1, stats=None, f0_func=None):
    """``odeint_dopri5`` with the adaptive step on the device: ``func(t, y)`` must be
    stream-capturable (device work only, t a 0-dim tensor of y's dtype; e.g. the HIP
    velocity field's ``capturable`` program).  The initial step selection runs once, eagerly
    (``f0_func``, default func); every later step is one replay of the captured step graph and
    one host read of (t_hi, dt).  Same tableau, error norm, step-size control and dense output
    as ``odeint_dopri5``, so the accepted step sequence and the solution are the same."""
    if not torch.is_floating_point(y0):
        raise TypeError("y0 must be floating point")
    dev, dty = y0.device, y0.dtype
    t = torch.as_tensor(t).to(device=dev, dtype=torch.float64)
    if t.dim() != 1 or not bool((t[1:] > t[:-1]).all()):
        raise ValueError("t must be strictly increasing")
    rtol = float(torch.as_tensor(rtol, dtype=torch.float64).reshape(-1)[0])
    atol = float(torch.as_tensor(atol, dtype=torch.float64).reshape(-1)[0])
    st = stats if stats is not None else Dopri5Stats()
    ef = f0_func or func

    def f_eager(tt, yy):
        st.nfe += 1
        return ef(tt.to(yy.dtype), yy)

    beta = [_weights(b, y0) for b in _BETA]
    c_err = _weights(_C_ERROR, y0)
    c_mid = _weights(_C_MID, y0)
    sol = torch.empty(len(t), *y0.shape, dtype=dty, device=dev)
    sol[0] = y0
    f0 = f_eager(t[0], y0)
    # static state of the captured step
    S = {"y": y0.clone(), "fy": f0.clone(), "t_lo": t[0].clone(), "t_hi": t[0].clone(),
         "dt": _select_initial_step(f_eager, t[0], y0, f0, rtol, atol).reshape(()).clone(),
         "coeffs": [y0.clone() for _ in range(5)], "acc": torch.zeros((), dtype=torch.int64, device=dev),
         "tries": torch.zeros((), dtype=torch.int64, device=dev)}

    # a field that conditions several times at once (HipEngine.velocity_field: t-embedding, adaLN
    # rows and IPA prepend for all 5 stage times in one call) gets the step's stage times up front
    pre = getattr(func, "precondition", None)
    ensure = getattr(func, "ensure", None)  # the field's hoisted state back in place (engine)

    def step():
        y, fy, t_hi, dt = S["y"], S["fy"], S["t_hi"], S["dt"]
        t1 = t_hi + dt
        dt_y = dt.to(dty)
        ks = [fy]
        tts = []
        for a_i in _ALPHA:
            if a_i == 1.0:
                tt = t1.to(dty)
                tts.append(torch.nextafter(tt, tt - 1))
            else:
                tts.append((t_hi + a_i * dt).to(dty))
        if pre is not None:
            pre(torch.stack(tts))
        for i, b_i in enumerate(beta):
            yi = _combine(y, ks, b_i, dt_y)
            ks.append(func.stage(i, yi) if pre is not None else func(tts[i], yi))
        y1 = yi
        err = _combine(None, ks, c_err, dt_y)
        tol = atol + rtol * torch.max(y.abs(), y1.abs())
        ratio = rms_norm(err / tol)
        ok = ratio <= 1
        y_mid = _combine(y, ks, c_mid, dt_y)
        new = _interp_fit(y, y1, y_mid, ks[0], ks[-1], dt_y)
        for c, n in zip(S["coeffs"], new):
            c.copy_(torch.where(ok, n, c))
        S["t_lo"].copy_(torch.where(ok, t_hi, S["t_lo"]))
        y.copy_(torch.where(ok, y1, y))
        fy.copy_(torch.where(ok, ks[-1], fy))
        er = ratio.to(dt.dtype)  # _optimal_step_size; ratio == 0 gives min(inf, ifactor) = ifactor
        dmin = torch.where(ok, torch.ones_like(er), torch.full_like(er, 0.2))
        new_dt = dt * torch.clamp(0.9 / er ** (1.0 / ORDER), min=dmin, max=torch.full_like(er, 10.0))
        t_hi.copy_(torch.where(ok, t1, t_hi))
        dt.copy_(new_dt)
        S["acc"].add_(ok.to(torch.int64))
        S["tries"].add_(1)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=side):
            step()
    torch.cuda.current_stream().wait_stream(side)
    n_steps = 0
    th_dt = torch.stack([S["t_hi"], S["dt"]])
    for i in range(1, len(t)):
        nt = float(t[i])
        while True:
            torch.stack([S["t_hi"], S["dt"]], out=th_dt)
            t_hi_v, dt_v = th_dt.tolist()
            if not nt > t_hi_v:
                break
            if n_steps >= max_num_steps:
                raise AssertionError(f"max_num_steps exceeded ({n_steps}>={max_num_steps})")
            if not t_hi_v + dt_v > t_hi_v:
                raise AssertionError(f"underflow in dt {dt_v}")
            if ensure is not None:
                ensure()
            g.replay()
            n_steps += 1
        x = ((t[i] - S["t_lo"]) / (S["t_hi"] - S["t_lo"])).to(dty)
        c = S["coeffs"]
        total = c[0] + x * c[1]
        xp = x
        for cc in c[2:]:
            xp = xp * x
            total = total + xp * cc
        sol[i] = total
    acc, tries = int(S["acc"]), int(S["tries"])
    st.accepted += acc
    st.rejected += tries - acc
    st.nfe += 6 * tries
    return sol
