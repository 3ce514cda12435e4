"""GPU parity: mpcqp_mpc_box_loop -- the receding-horizon loop of the
input-box MPC on a linear plant, T steps in one launch with warm-started
active sets -- against the host loop of the oracle: per step the condensed
QP (oracle/condense.py) solved by the oracle's box active set
(oracle/qp.py, KKT-checked), then x_{t+1} = A x_t + B u_0
(LinearSystem.f, session_1/LinearSystem.py:16-18, under the MPC policy of
MPCController.solve, session_4/main.py:115-116)."""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched
from oracle import condense as oc
from oracle import qp as oq

pytestmark = pytest.mark.gpu

TOL_X = 1e-9


def _fhc_plant():
    ts = 0.5                                        # FHC.py:44-48, config 2
    A = np.array([[1.0, ts], [0.0, 1.0]])
    B = np.array([[0.0], [-ts]])
    C = np.array([[1.0], [-2.0 / 3.0]])
    Q = C @ C.T + 1e-3 * np.eye(2)
    return A, B, Q, np.array([[0.1]]), Q.copy()


def _host_loop(A, B, Q, R, Qf, N, x0, lb, ub, T):
    d = oc.condense(A, B, Q, R, Qf, N)
    H, F = d["H"], d["F"]
    xs, us = [np.asarray(x0, float)], []
    for _ in range(T):
        f = F @ xs[-1]
        z = oq.box_qp(H, f, lb, ub)[0]
        assert oq.kkt_box(H, f, lb, ub, z) < 1e-9
        nu = B.shape[1]
        us.append(z[:nu])
        xs.append(A @ xs[-1] + B @ z[:nu])
    return np.array(xs), np.array(us)


def _t(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)


@pytest.mark.parametrize("N,batch", [(20, 9), (12, 4), (31, 5)])
def test_loop_matches_host_loop(dev, N, batch):
    """Config-2 plant (FHC double integrator, |u| <= 1): the device episode
    equals the oracle's host loop step for step (states and applied inputs);
    every step optimal."""
    A, B, Q, R, Qf = _fhc_plant()
    rng = np.random.default_rng(N)
    X0 = rng.uniform(-10, 10, (batch, 2))
    T = 15
    n = N
    r = batched.mpc_box_loop(_t(A, dev), _t(B, dev), _t(Q, dev), _t(R, dev), _t(Qf, dev), N,
                             _t(X0, dev), -1.0, 1.0, T, plans=True)
    torch.cuda.synchronize()
    xs, us, st = r["xs"].cpu().numpy(), r["us"].cpu().numpy(), r["status"].cpu().numpy()
    assert ((st & 0xFF) == 0).all(), np.unique(st & 0xFF)
    for i in range(batch):
        hx, hu = _host_loop(A, B, Q, R, Qf, N, X0[i], -np.ones(n), np.ones(n), T)
        assert np.abs(xs[:, i] - hx).max() < TOL_X * (1 + np.abs(hx).max()), i
        assert np.abs(us[:, i] - hu).max() < TOL_X, i


def test_loop_per_instance_plants_and_bounds(dev):
    """Per-instance plants (random stable 4x2) and per-instance bounds, nu = 2:
    the same host-loop parity; the input plans zs are the full QP solutions."""
    rng = np.random.default_rng(3)
    b, N, T = 6, 8, 10
    nx, nu = 4, 2
    As, Bs = [], []
    for _ in range(b):
        M = rng.normal(size=(nx, nx))
        As.append(0.95 * M / max(abs(np.linalg.eigvals(M))))
        Bs.append(rng.normal(size=(nx, nu)))
    As, Bs = np.array(As), np.array(Bs)
    Q, R = np.eye(nx), 0.1 * np.eye(nu)
    lb = -rng.uniform(0.2, 1.0, (b, N * nu))
    ub = rng.uniform(0.2, 1.0, (b, N * nu))
    X0 = rng.normal(size=(b, nx)) * 3
    r = batched.mpc_box_loop(_t(As, dev), _t(Bs, dev), _t(Q, dev), _t(R, dev), _t(Q, dev), N,
                             _t(X0, dev), _t(lb, dev), _t(ub, dev), T, plans=True)
    torch.cuda.synchronize()
    xs, zs, st = r["xs"].cpu().numpy(), r["zs"].cpu().numpy(), r["status"].cpu().numpy()
    assert ((st & 0xFF) == 0).all()
    for i in range(b):
        d = oc.condense(As[i], Bs[i], Q, R, Q, N)
        x = X0[i]
        for t in range(T):
            z = oq.box_qp(d["H"], d["F"] @ x, lb[i], ub[i])[0]
            assert np.abs(zs[t, i] - z).max() < 1e-9, (i, t)
            assert np.abs(xs[t, i] - x).max() < 1e-9 * (1 + np.abs(x).max())
            x = As[i] @ x + Bs[i] @ z[:nu]


def test_loop_equals_repeated_steps(dev):
    """The one-launch episode equals T separate fused MPC steps (mpcqp_mpc_box,
    cold each step) with the plant advanced in between -- the warm start
    changes the path, not the answer."""
    A, B, Q, R, Qf = _fhc_plant()
    rng = np.random.default_rng(11)
    b, N, T = 64, 20, 12
    X0 = rng.uniform(-10, 10, (b, 2))
    t = lambda a: _t(a, dev)  # noqa: E731
    r = batched.mpc_box_loop(t(A), t(B), t(Q), t(R), t(Qf), N, t(X0), -1.0, 1.0, T)
    x = t(X0)
    Ab, Bb = t(np.broadcast_to(A, (b, 2, 2))), t(np.broadcast_to(B, (b, 2, 1)))
    for k in range(T):
        z, st = batched.mpc_box(Ab, Bb, t(Q), t(R), t(Qf), N, x, -1.0, 1.0)
        assert (batched.status_code(st) == 0).all()
        assert (r["xs"][k] - x).abs().max().item() < 1e-9 * (1 + x.abs().max().item())
        assert (r["us"][k] - z[:, :1]).abs().max().item() < 1e-9
        x = x @ t(A).T + z[:, :1] @ t(B).T
    # warm starts: after the first step, the steps need far fewer sweeps +
    # iterations than the cold first step
    its = ((r["status"] >> 8) & 0xFFFF).double()
    assert its[1:].mean().item() < 0.6 * its[0].mean().item()


def test_loop_edge_cases(dev):
    """steps = 0 records x0 only; an empty box (lb > ub) reports INFEASIBLE
    for that instance at every step and leaves the others optimal; a batch
    that is not a multiple of four."""
    A, B, Q, R, Qf = _fhc_plant()
    t = lambda a: _t(a, dev)  # noqa: E731
    X0 = np.array([[1.0, 2.0], [3.0, -1.0], [0.5, 0.5]])
    r0 = batched.mpc_box_loop(t(A), t(B), t(Q), t(R), t(Qf), 10, t(X0), -1.0, 1.0, 0)
    assert torch.equal(r0["xs"][0], t(X0))
    lb = -np.ones((3, 10))
    ub = np.ones((3, 10))
    lb[1, 4] = 2.0
    r = batched.mpc_box_loop(t(A), t(B), t(Q), t(R), t(Qf), 10, t(X0), t(lb), t(ub), 4)
    code = (r["status"] & 0xFF).cpu().numpy()
    assert (code[:, 1] == 3).all() and (code[:, [0, 2]] == 0).all()
    with pytest.raises(Exception):
        batched.mpc_box_loop(t(A), t(B), t(Q), t(R), t(Qf), 40, t(X0), -1.0, 1.0, 2)  # N*nu > 32


def test_lti_loop_helper(dev):
    """closed_loop.lti_box_mpc_loop: the ControllerLog-shaped outputs of the
    same episode (success per step, input_prediction (T, b, N, nu) whose first
    input is the applied one)."""
    from model_predictive_control_amd.closed_loop import lti_box_mpc_loop

    A, B, Q, R, Qf = _fhc_plant()
    X0 = np.array([[5.0, -3.0], [-8.0, 2.0]])
    out = lti_box_mpc_loop(A, B, Q, R, Qf, 20, X0, -1.0, 1.0, 6)
    assert out["success"].all()
    assert tuple(out["input_prediction"].shape) == (6, 2, 20, 1)
    assert torch.equal(out["input_prediction"][:, :, 0], out["us"])
