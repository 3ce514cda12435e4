"""GPU parity: mpcqp_bicycle_rti (FE rollout + per-stage linearisation of the
kinematic bicycle, session_4/main.py:132-135, 250-251) against the batched
torch restatement (bicycle.fe_linearize_batched), the oracle's central finite
differences and the oracle rollout.  The ODE itself is parity unpinned
(rcracers absent): these tests pin the kernel to the restated model."""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched
from _torch_bicycle import fe_linearize_batched, fe_step_batched
from model_predictive_control_amd.parameters import VehicleParameters
from oracle import bicycle as ob

pytestmark = pytest.mark.gpu


def _case(dev, b, N, dt, seed):
    rng = np.random.default_rng(seed)
    X0 = np.stack([rng.uniform(-1, 1, b), rng.uniform(-.5, .5, b), rng.uniform(-np.pi / 4, np.pi / 4, b),
                   rng.uniform(-.3, .3, b)], -1)
    U = np.stack([rng.uniform(-1, 1, (b, N)), rng.uniform(-.38, .38, (b, N))], -1)
    return X0, U, torch.as_tensor(X0, dtype=dt, device=dev), torch.as_tensor(U, dtype=dt, device=dev)


@pytest.mark.parametrize("b,N", [(1, 1), (5, 30), (130, 7), (64, 40)])
def test_bicycle_rti_matches_torch_and_oracle(dev, b, N):
    p = VehicleParameters()
    ts = 0.08
    X0, U, X0t, Ut = _case(dev, b, N, torch.float64, 11 * b + N)
    A, B, c, X = batched.bicycle_rti(X0t, Ut, p, ts, states=True)
    # torch restatement on the same rollout
    xs = [X0t]
    for k in range(N):
        xs.append(fe_step_batched(xs[-1], Ut[:, k], p, ts))
    Xr = torch.stack(xs, 1)
    Ar, Br, cr = fe_linearize_batched(Xr[:, :N], Ut, p, ts)
    assert (X - Xr).abs().max().item() < 1e-13
    assert (A - Ar).abs().max().item() < 1e-13
    assert (B - Br).abs().max().item() < 1e-13
    assert (c - cr).abs().max().item() < 1e-13
    # oracle: independent FD Jacobians and the affine model reproduces the rollout
    An, Bn, Xn = A.cpu().numpy(), B.cpu().numpy(), X.cpu().numpy()
    for i in range(min(b, 3)):
        x = X0[i]
        for k in range(N):
            Af, Bf = ob.fe_jac_fd(x, U[i, k], ts)
            assert np.abs(An[i, k] - Af).max() < 1e-6
            assert np.abs(Bn[i, k] - Bf).max() < 1e-6
            xn = ob.fe(x, U[i, k], ts)
            assert np.abs(Xn[i, k + 1] - xn).max() < 1e-12
            x = xn
    lin = (A @ X[:, :N].unsqueeze(-1)).squeeze(-1) + (B @ Ut.unsqueeze(-1)).squeeze(-1) + c
    assert (lin - X[:, 1:]).abs().max().item() < 1e-12


def test_bicycle_rti_fp32(dev):
    p = VehicleParameters()
    X0, U, X0t, Ut = _case(dev, 257, 30, torch.float32, 3)
    A, B, c = batched.bicycle_rti(X0t, Ut, p, 0.08)
    A64, B64, c64 = batched.bicycle_rti(X0t.double(), Ut.double(), p, 0.08)
    assert (A.double() - A64).abs().max().item() < 1e-5
    assert (B.double() - B64).abs().max().item() < 1e-5
    assert (c.double() - c64).abs().max().item() < 1e-5
