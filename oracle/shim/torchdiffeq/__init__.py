"""Test-only restatement of torchdiffeq 0.2.5 `odeint`, fixed-grid Euler only.

torchdiffeq's `_FixedGridODESolver` with `Euler._step_func` evaluates, on the given grid
(no step_size option), dy = dt * f(t0, y0) and y1 = y0 + dy, recording y at every grid
point; the solution tensor is stacked along a new leading dim.  Used by reference
integrators.py:106-113.  Adaptive methods (dopri5) are not restated here.
"""
import torch


def odeint(func, y0, t, method=None, atol=None, rtol=None, options=None):
    if method not in ("euler",):
        raise NotImplementedError(f"oracle shim supports method='euler' only, got {method!r}")
    is_tuple = isinstance(y0, tuple)
    ys = [y0]
    y = y0
    for i in range(len(t) - 1):
        t0, t1 = t[i], t[i + 1]
        dt = t1 - t0
        f = func(t0, y)
        if is_tuple:
            y = tuple(yi + dt * fi for yi, fi in zip(y, f))
        else:
            y = y + dt * f
        ys.append(y)
    if is_tuple:
        return tuple(torch.stack([yy[k] for yy in ys]) for k in range(len(y0)))
    return torch.stack(ys)
