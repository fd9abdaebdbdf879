"""dopri5 (the reference's default sampler, parsing.py:102 -> torchdiffeq.odeint, integrators.py:
95-114) restated in mdgen_finetune_amd/transport/integrators.py.  torchdiffeq is absent, so
parity with torchdiffeq itself is unpinned; these tests pin the algorithm's properties:
convergence to analytic solutions at the solver's order, the saved grid, the step-size
controller, the drop-in Sampler wiring with the model on the eager backend (the HIP side is
in tests/test_gpu_parity.py), and agreement with scipy's independent Runge-Kutta
implementations (RK45 = the same Dormand-Prince pair, DOP853 as the tight reference) on a
nonlinear system and on the model's own velocity field."""
import functools
import math

import numpy as np
import pytest
import torch

from mdgen_finetune_amd.transport import Dopri5Stats, Sampler, create_transport, odeint_dopri5
from mdgen_finetune_amd.transport import integrators as I
from tests.conftest import build_model, load_golden


def _exact(y0, t):
    # y' = -2y + sin(3t):  y = (y0 + 3/13) e^{-2t} + (2 sin 3t - 3 cos 3t) / 13
    tt = t.reshape(-1, *([1] * y0.dim()))
    return (y0 + 3 / 13) * torch.exp(-2 * tt) + (2 * torch.sin(3 * tt) - 3 * torch.cos(3 * tt)) / 13


def test_tableau_consistency():
    # row sums of beta equal alpha (stage times), c_sol == last beta row (FSAL), error weights sum to 0
    for a, b in zip(I._ALPHA, I._BETA):
        assert abs(sum(b) - a) < 1e-14
    assert abs(sum(I._BETA[-1]) - 1.0) < 1e-14
    assert abs(sum(I._C_ERROR)) < 1e-14


@pytest.mark.parametrize("rtol,err_bound", [(1e-3, 2e-3), (1e-6, 2e-6), (1e-9, 2e-9)])
def test_converges_to_analytic_solution(rtol, err_bound):
    y0 = torch.randn(4, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(0))
    t = torch.linspace(0, 1, 50, dtype=torch.float64)
    st = Dopri5Stats()
    sol = odeint_dopri5(lambda t, y: -2 * y + torch.sin(3 * t), y0, t, rtol=rtol, atol=rtol * 1e-3, stats=st)
    assert sol.shape == (50, 4, 6)
    assert torch.equal(sol[0], y0)
    err = (sol - _exact(y0, t)).abs().max().item()
    assert err < err_bound, err
    assert st.nfe == 2 + 6 * (st.accepted + st.rejected)  # f0, the initial-step probe, 6 per step


def test_fifth_order_error_decay():
    """Global error of the 5th-order solution shrinks ~ (tol)^(5/5): tighter tol, fewer errors;
    NFE grows ~ tol^(-1/5)."""
    y0 = torch.ones(3, dtype=torch.float64)
    t = torch.tensor([0.0, 2.0], dtype=torch.float64)
    nfes = []
    for rtol in (1e-4, 1e-6, 1e-8):
        st = Dopri5Stats()
        odeint_dopri5(lambda t, y: -2 * y + torch.sin(3 * t), y0, t, rtol=rtol, atol=1e-14, stats=st)
        nfes.append(st.nfe)
    r1, r2 = nfes[1] / nfes[0], nfes[2] / nfes[1]
    assert 1.6 < r1 < 4.5 and 1.6 < r2 < 4.5, nfes  # 100^(1/5) = 2.5


def test_dense_output_hits_saved_points_between_steps():
    """A linear ODE's interpolant error on 200 saved points stays within the step tolerance
    (num_steps counts saved points, the solver takes far fewer steps)."""
    y0 = torch.tensor([1.0, -0.5], dtype=torch.float64)
    t = torch.linspace(0, 1, 200, dtype=torch.float64)
    st = Dopri5Stats()
    sol = odeint_dopri5(lambda t, y: -2 * y + torch.sin(3 * t), y0, t, rtol=1e-6, atol=1e-9, stats=st)
    assert st.accepted < 40
    assert (sol - _exact(y0, t)).abs().max() < 1e-5


def test_fp32_state_and_time_dtypes():
    seen = []

    def f(t, y):
        seen.append(t.dtype)
        return -y

    sol = odeint_dopri5(f, torch.ones(5), torch.linspace(0, 1, 50))
    assert sol.dtype == torch.float32 and all(d == torch.float32 for d in seen)
    assert abs(sol[-1, 0].item() - math.exp(-1)) < 1e-3


def test_step_size_controller():
    dt = torch.tensor(0.1, dtype=torch.float64)
    assert I._optimal_step_size(dt, torch.tensor(0.0)).item() == pytest.approx(1.0)        # x ifactor
    assert I._optimal_step_size(dt, torch.tensor(1e-12)).item() == pytest.approx(1.0)      # clamp ifactor
    assert I._optimal_step_size(dt, torch.tensor(0.5)).item() == pytest.approx(0.1 * 0.9 / 0.5 ** 0.2)
    assert I._optimal_step_size(dt, torch.tensor(1e6)).item() == pytest.approx(0.02)       # clamp dfactor
    assert I._optimal_step_size(dt, torch.tensor(0.99)).item() >= 0.1 * 0.9                # accepted: no shrink below safety


def test_sampler_dopri5_with_model_matches_tight_solve():
    """Sampler.sample_ode() default (dopri5, num_steps=50) on the eager backend: the final state
    agrees with a tight-tolerance solve of the same ODE to the default rtol's accuracy."""
    d, cfg = load_golden("small_sim_T8")
    m, _ = build_model(cfg)
    m.backend = "torch"
    from tests.test_model_cpu import _kw

    kw = _kw(d)
    tr = create_transport(m.args, "GVP", "velocity")
    zs = torch.from_numpy(d["in_zs"])
    with torch.no_grad():
        ys = Sampler(tr).sample_ode()(zs, functools.partial(m.forward_inference, **kw))
        tight = Sampler(tr).sample_ode(rtol=1e-7, atol=1e-9)(zs, functools.partial(m.forward_inference, **kw))
    assert ys.shape[0] == 50
    err = (ys[-1] - tight[-1]).abs().max().item()
    scale = tight[-1].abs().max().item()
    assert err < 1e-2 * max(scale, 1.0), (err, scale)
    # and the Euler solve of the same problem is a (cruder) approximation of the same endpoint
    with torch.no_grad():
        eul = Sampler(tr).sample_ode(sampling_method="euler")(zs, functools.partial(m.forward_inference, **kw))
    assert (eul[-1] - tight[-1]).abs().max().item() < 0.2 * max(scale, 1.0)
    np.testing.assert_array_equal(ys[0].numpy(), d["in_zs"])


def test_unknown_sampler_is_refused():
    with pytest.raises(NotImplementedError):
        Sampler(create_transport(None, "GVP")).sample_ode(sampling_method="rk4")


def _vdp(t, y, mu=1.5):
    # Van der Pol, y = [..., 2]: a nonlinear, mildly stiff test problem
    x, v = y[..., 0], y[..., 1]
    return torch.stack([v, mu * (1 - x * x) * v - x], -1)


@pytest.mark.parametrize("rtol", [1e-5, 1e-8])
def test_matches_scipy_runge_kutta_on_van_der_pol(rtol):
    """An independent implementation of the same Dormand-Prince 5(4) pair (scipy RK45) and a
    higher-order one (DOP853) at tight tolerance: the restated solver lands on the same
    trajectory to its tolerance (float64, 3 initial states, 40 saved points)."""
    from scipy.integrate import solve_ivp

    y0 = torch.tensor([[2.0, 0.0], [0.5, -1.0], [-1.5, 0.7]], dtype=torch.float64)
    t = torch.linspace(0, 3, 40, dtype=torch.float64)
    ours = odeint_dopri5(_vdp, y0, t, rtol=rtol, atol=rtol * 1e-2)
    for b in range(3):
        ref = solve_ivp(lambda tt, yy: _vdp(tt, torch.from_numpy(yy)).numpy(), (0.0, 3.0), y0[b].numpy(),
                        method="DOP853", t_eval=t.numpy(), rtol=1e-12, atol=1e-14)
        rk45 = solve_ivp(lambda tt, yy: _vdp(tt, torch.from_numpy(yy)).numpy(), (0.0, 3.0), y0[b].numpy(),
                         method="RK45", t_eval=t.numpy(), rtol=rtol, atol=rtol * 1e-2)
        err_ours = np.abs(ours[:, b].numpy() - ref.y.T).max()
        err_rk45 = np.abs(rk45.y.T - ref.y.T).max()
        # same pair, same tolerance: same accuracy class as scipy's RK45 (within 10x either way)
        assert err_ours < 50 * rtol, (err_ours, rtol)
        assert err_ours < 10 * max(err_rk45, 1e-3 * rtol), (err_ours, err_rk45)


def test_model_field_matches_scipy_dop853():
    """dopri5 at the reference's tolerances (rtol 1e-3, atol 1e-6; transport.py:410-413) on the
    model's own velocity field (eager backend, float64) against scipy's DOP853 at rtol 1e-8
    (~1000 field evaluations, ~8 s)."""
    from scipy.integrate import solve_ivp

    d, cfg = load_golden("small_sim_T8")
    m, _ = build_model(cfg)
    m.backend = "torch"
    m = m.double()
    from tests.test_model_cpu import _kw

    kw = {k: (v.double() if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in _kw(d).items()}
    zs = torch.from_numpy(d["in_zs"]).double()
    shape = zs.shape
    t = torch.linspace(0, 1, 50, dtype=torch.float64)

    def field(tt, y):
        return m.forward_inference(y, torch.ones(shape[0], dtype=torch.float64) * tt, **kw)

    with torch.no_grad():
        ours = odeint_dopri5(field, zs, t, rtol=1e-3, atol=1e-6)
        assert ours.shape[0] == 50
        ref = solve_ivp(lambda tt, yy: field(torch.tensor(tt, dtype=torch.float64),
                                             torch.from_numpy(yy).reshape(shape)).reshape(-1).numpy(),
                        (0.0, 1.0), zs.reshape(-1).numpy(), method="DOP853", rtol=1e-8, atol=1e-10)
    ref_end = torch.from_numpy(ref.y[:, -1]).reshape(shape)
    scale = ref_end.abs().max().item()
    err = (ours[-1] - ref_end).abs().max().item()
    assert err < 1e-2 * max(scale, 1.0), (err, scale)
