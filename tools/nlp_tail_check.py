"""Solve tests/golden/nlp_tail.npz on the device and compare each instance's
cost and solution with the fixture (the oracle's optimum).  GPU tool."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd.mpc import MPCController  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402

g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "nlp_tail.npz"))
ctl = MPCController(int(g["N"]), float(g["ts"]), VehicleParameters())
sol = ctl.solve(g["x0"])
err = np.abs(np.asarray(sol["x"]) - g["U"]).max(1)
tag = os.environ.get("TAG", "")
for i in range(len(err)):
    print(f"{tag} {i} err {err[i]:.2e} f {sol['f'][i]:.10f} fixJ {float(g['J'][i]):.10f} "
          f"kkt {float(sol['kkt'][i]):.1e} it {int(sol['iterations'][i])}")
np.save(f"gpurun_out/nlp_tail_U{tag}.npy", np.asarray(sol["x"]))
