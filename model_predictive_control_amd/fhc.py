"""FHC -- the call surface of session_1/FHC.py on the MI355X path.

* ``get_dynamics_continuous`` / ``get_dynamics_discrete``  (FHC.py:32-48):
  problem data, built on the host exactly as the reference does.
* ``ricatti_recursion(A, B, Q, R, P_f, N)``  (FHC.py:51-61): same signature,
  argument order (Q before R), R broadcasting (R of shape (1,)) and output
  (lists P[N+1], K[N], reversed so K[0] is the first-stage gain) -- computed
  by the batched ``mpcqp_riccati`` HIP kernel.  ``ricatti_recursion_batched``
  runs thousands of independent plants in one launch.
* ``AutoCruising``  (FHC.py:20-29): ``set_opti_gain``, ``control_law``
  (gains[0] @ x) and ``pred`` (gains[t] @ x); its closed-loop ``simulate``
  runs on the GPU (``mpcqp_rollout``) since the law is a linear feedback.
* ``compare_term_cost``  (FHC.py:117-131): returns (N list, V_N, V_inf)
  instead of plotting; V_inf from the GPU Riccati iterated to convergence.
"""
from __future__ import annotations

import numpy as np
import torch

from . import batched
from .linear_system import LinearSystem


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("model_predictive_control_amd needs a ROCm GPU (no CPU fallback)")
    return torch.device("cuda")


def get_dynamics_continuous():
    """FHC.py:32-41."""
    A = np.array([[0., 1.], [0., 0.]])
    B = np.array([[0], [-1]])
    return A, B


def get_dynamics_discrete(ts: float):
    """FHC.py:44-48 (forward Euler)."""
    A, B = get_dynamics_continuous()
    return np.eye(2) + A * ts, B * ts


def _r_matrix(R, nu):
    R = np.asarray(R, dtype=float)
    return np.broadcast_to(R, (nu, nu)).copy() if R.ndim < 2 else R


def ricatti_recursion_batched(A, B, Q, R, P_f, N: int, dtype=torch.float64):
    """Batched FHC.ricatti_recursion on device tensors: (P (b,N+1,nx,nx), K (b,N,nu,nx))."""
    dev = _device()
    B_t = torch.as_tensor(B, dtype=dtype, device=dev)
    nu = int(B_t.shape[-1])
    R_t = torch.as_tensor(R, dtype=dtype, device=dev)
    if R_t.ndim < 2:
        R_t = torch.broadcast_to(R_t, (nu, nu)).contiguous()
    return batched.riccati(torch.as_tensor(A, dtype=dtype, device=dev), B_t,
                           torch.as_tensor(Q, dtype=dtype, device=dev), R_t,
                           torch.as_tensor(P_f, dtype=dtype, device=dev), N)


def ricatti_recursion(A, B, Q, R, P_f, N: int):
    """FHC.py:51-61 -- returns (P list of N+1 (nx,nx), K list of N (nu,nx))."""
    A = np.asarray(A, dtype=float)
    B = np.asarray(B, dtype=float)
    P, K = ricatti_recursion_batched(A, B, Q, _r_matrix(R, B.shape[1]), P_f, N)
    P = P[0].cpu().numpy()
    K = K[0].cpu().numpy()
    return [P[k] for k in range(N + 1)], [K[k] for k in range(N)]


def solve_discrete_are(A, B, Q, R, tol: float = 1e-13, max_horizon: int = 1 << 14):
    """DARE solution as the limit of the GPU Riccati recursion (FHC.py:97,126
    uses scipy.linalg.solve_discrete_are for the same quantity)."""
    N = 64
    prev = None
    while N <= max_horizon:
        P, _ = ricatti_recursion(A, B, Q, R, Q, N)
        if prev is not None and np.abs(P[0] - prev).max() <= tol * max(1.0, np.abs(P[0]).max()):
            return P[0]
        prev = P[0]
        N *= 2
    # scipy.linalg.solve_discrete_are (FHC.py:97,126) raises when it fails;
    # so does this limit when the recursion has not settled by max_horizon
    raise np.linalg.LinAlgError(
        f"solve_discrete_are: Riccati recursion not converged to tol={tol:g} "
        f"within horizon {max_horizon}")


class AutoCruising(LinearSystem):
    """FHC.py:20-29."""

    def set_opti_gain(self, gains) -> None:
        self.gains = gains

    def control_law(self, x, t) -> np.ndarray:
        return self.gains[0] @ x

    def pred(self, x, t) -> np.ndarray:
        return self.gains[t] @ x

    def simulate(self, x0, control_law, steps: int) -> None:
        # The receding-horizon law gains[0] @ x is linear: run the whole
        # closed loop on device (LinearSystem.py:20-26 semantics).
        if getattr(control_law, "__func__", None) is AutoCruising.control_law and \
                getattr(control_law, "__self__", None) is self:
            x0 = np.expand_dims(np.asarray(x0, dtype=float), axis=2)[:, :, 0]
            dev = _device()
            xs = batched.rollout(torch.as_tensor(self.A, dtype=torch.float64, device=dev),
                                 torch.as_tensor(self.B, dtype=torch.float64, device=dev),
                                 torch.as_tensor(np.asarray(self.gains[0], float), device=dev),
                                 torch.as_tensor(x0.T.copy(), device=dev), max(steps, 1))
            self.x = xs.permute(2, 1, 0).cpu().numpy()
            return
        super().simulate(x0, control_law, steps)


def compare_term_cost(A, B, Q, R, P_f, x0):
    """FHC.py:117-131 without the plot: returns (N_lst, V_N, V_inf)."""
    x0 = np.asarray(x0, dtype=float)
    N_lst = list(range(1, 10))
    V_N = []
    for N in N_lst:
        P_n, _ = ricatti_recursion(A, B, Q, R, P_f, N)
        V_N.append(np.squeeze(x0.T @ P_n[0] @ x0))
    P_inf = solve_discrete_are(A, B, Q, R)
    return N_lst, np.array(V_N), np.squeeze(x0.T @ P_inf @ x0)
