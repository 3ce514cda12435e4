"""Vehicle data of the session-4 parking problem (session_4/parameters.py:4-54).

The reference keeps these as a flat dataclass; the solver only consumes a few
of them (the FE bicycle of bicycle.py / bicycle.hip reads ``axis_front``,
``axis_rear``, ``acceleration``, ``friction``; the QP boxes read the limits).
Here the fields are declared group by group in tables and the dataclass is
assembled from them, so the attribute names, defaults and field order stay
those of the reference while the boxes the OCP needs come out as vectors in
the solver's state order [p_x, p_y, psi, v] (main.py:58-61) and input order
[drive, steer] (main.py:68-69).
"""
from __future__ import annotations

import math
from dataclasses import field, make_dataclass

import numpy as np

# (name, default) per group, in the reference's field order
_GEOMETRY = (("length", 0.17), ("axis_front", 0.047), ("axis_rear", 0.05), ("front", 0.08),
             ("rear", 0.08), ("width", 0.08), ("height", 0.055), ("mass", 0.1735),
             ("inertia", 18.3e-5))
_INPUT_LIMITS = (("max_steer", 0.384), ("max_drive", 1.0), ("min_drive", -1.0))
_STATE_LIMITS = (("min_pos_x", -3.0), ("max_pos_x", 3.0), ("min_pos_y", -2.0), ("max_pos_y", 2.0),
                 ("min_vel", -0.5), ("max_vel", 0.5), ("max_heading", 2 * math.pi),
                 ("min_heading", -2 * math.pi))
# tyre "magic formula" factors (front/rear stiffness, shape, peak): dynamic model only
_TYRE = (("bf", 3.1355), ("cf", 2.1767), ("df", 0.4399), ("br", 2.8919), ("cr", 2.4431),
         ("dr", 0.6236))
_KINEMATIC = (("friction", 1), ("acceleration", 2))
_MOTOR = (("cm1", 0.3697), ("cm2", 0.001295), ("cr1", 0.1629), ("cr2", 0.02133))

_GROUPS = (_GEOMETRY, _INPUT_LIMITS, _STATE_LIMITS, _TYRE, _KINEMATIC, _MOTOR)


def _input_box(self) -> tuple[np.ndarray, np.ndarray]:
    """(lower, upper) of u = [drive, steer] (main.py:68-69)."""
    return (np.array([self.min_drive, -self.max_steer], float),
            np.array([self.max_drive, self.max_steer], float))


def _state_box(self) -> tuple[np.ndarray, np.ndarray]:
    """(lower, upper) of x = [p_x, p_y, psi, v] (main.py:58-61)."""
    return (np.array([self.min_pos_x, self.min_pos_y, self.min_heading, self.min_vel], float),
            np.array([self.max_pos_x, self.max_pos_y, self.max_heading, self.max_vel], float))


VehicleParameters = make_dataclass(
    "VehicleParameters",
    # every field is annotated float, as in the reference dataclass (parameters.py:4-54,
    # whose friction/acceleration defaults are written as the literals 1 and 2)
    [(name, float, field(default=value)) for group in _GROUPS for name, value in group],
    namespace={"input_box": _input_box, "state_box": _state_box,
               "__doc__": "Kinematic-bicycle parameters and bounds (session_4/parameters.py)."},
)
VehicleParameters.__module__ = __name__
