"""MI355X-native batched condensed-QP MPC solver.

A drop-in for the receding-horizon inner loop of
konnpaku-youmu/Model_Predictive_Control: the reference's Python call
surfaces (session_1/FHC.py, session_1/LinearSystem.py,
session_1/session1_sol.py, session_4/main.py ``MPCController``) are kept, and
the per-step work -- condense (A, B) over the horizon into H, F, f, then solve
the box / polytope QP -- runs as hand-written gfx950 HIP kernels behind the
C ABI of include/mpcqp.h (libmpcqp.so, loaded with ctypes).

Submodules:
  batched        device API on torch tensors (condense, solve_box, solve_poly,
                 riccati, gemv, rollout)
  fhc            FHC.py surface (ricatti_recursion, AutoCruising, ...)
  linear_system  LinearSystem.py surface
  session1       session1_sol.py surface
  problems       session 2/3 problem data + ControllerLog
  parameters     VehicleParameters (session_4/parameters.py)
  bicycle        kinematic bicycle, integrators, batched FE linearisation
  mpc            MPCController (session_4/main.py) on device
  distributed    batch sharding / gather across GPUs
"""
from . import _native  # noqa: F401

__version__ = "0.1.0"


def library_path() -> str:
    return _native.LIB_PATH
