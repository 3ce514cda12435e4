"""VehicleParameters -- session_4/parameters.py:4-54 (data only)."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class VehicleParameters:
    length: float = 0.17
    axis_front: float = 0.047
    axis_rear: float = 0.05
    front: float = 0.08
    rear: float = 0.08
    width: float = 0.08
    height: float = 0.055
    mass: float = 0.1735
    inertia: float = 18.3e-5
    # input limits (parameters.py:17-19)
    max_steer: float = 0.384
    max_drive: float = 1.0
    min_drive: float = -1.
    # state limits (parameters.py:22-29)
    min_pos_x: float = -3.
    max_pos_x: float = 3.
    min_pos_y: float = -2.
    max_pos_y: float = 2.
    min_vel: float = -0.5
    max_vel: float = 0.5
    max_heading: float = 2 * np.pi
    min_heading: float = -2 * np.pi
    # Pacejka parameters (unused by the kinematic model)
    bf: float = 3.1355
    cf: float = 2.1767
    df: float = 0.4399
    br: float = 2.8919
    cr: float = 2.4431
    dr: float = 0.6236
    # kinematic approximation (parameters.py:46-48)
    friction: float = 1
    acceleration: float = 2
    # motor parameters
    cm1: float = 0.3697
    cm2: float = 0.001295
    cr1: float = 0.1629
    cr2: float = 0.02133
