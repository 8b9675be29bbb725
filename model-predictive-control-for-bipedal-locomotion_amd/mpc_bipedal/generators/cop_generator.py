"""CoP (ZMP) bounds from the footstep plan: the per-timestep boxes the Wieber QP tracks.

Behaviour of the reference ``generators/cop_generator.py:11-115`` (restated, not copied):
a walking phase machine STANDING → DOUBLE_SUPPORT ⇄ SINGLE_SUPPORT → … → STANDING sampled
every ``dt`` with a floating-point clock advanced by ``t += dt`` (the accumulation decides the
sample count, so it is kept exactly); in STANDING/DOUBLE_SUPPORT the box is the hull of the
two feet in contact, in SINGLE_SUPPORT the stance foot's box.
"""

from enum import Enum
from typing import List, Tuple

import numpy as np

from .footstep_generator import generate_footsteps


class State(Enum):
    """Walking state."""
    STANDING = 'STANDING'
    DOUBLE_SUPPORT = 'DOUBLE_SUPPORT'
    SINGLE_SUPPORT = 'SINGLE_SUPPORT'


class CoPGenerator:
    """Generates the CoP bound sequence ``z_max``/``z_min`` [n, 2] handed to the controller."""

    def __init__(self, config):
        if config.dt is None:
            raise ValueError("dt must be set in MPCConfig (it is shared with the controller)")
        self.ssp_duration = config.ssp_duration
        self.dsp_duration = config.dsp_duration
        self.standing_duration = config.standing_duration
        self.dt = config.dt
        self.distance = config.distance
        self.step_length = config.step_length
        self.foot_spread = config.foot_spread

    def _transition(self, state: State, foot: int, last: int):
        """Next (state, foot index, phase duration) when the current phase has elapsed."""
        S, D, SS = State.STANDING, State.DOUBLE_SUPPORT, State.SINGLE_SUPPORT
        if state is S:
            if foot == last:           # final standing phase: end of the walk
                return S, foot + 1, 0.0
            return D, foot, self.dsp_duration
        if state is SS:                # stance change: the swing foot lands
            return D, foot + 1, self.dsp_duration
        if state is D:
            if foot == last:
                return S, foot, self.standing_duration
            return SS, foot, self.ssp_duration
        raise ValueError(f"Invalid state: {state}")

    def generate_cop_trajectory(self, save_footsteps: bool = False,
                                output_dir: str = 'results'
                                ) -> Tuple[np.ndarray, np.ndarray, List[State]]:
        """Return (z_max [n,2], z_min [n,2], states [n]).

        ``save_footsteps`` (plotting, reference default True) is accepted for signature
        compatibility; this build does not draw.
        """
        feet = generate_footsteps(distance=self.distance, step_length=self.step_length,
                                  foot_spread=self.foot_spread)
        last = len(feet) - 1
        foot, state = 1, State.STANDING
        t, t_switch = 0., self.standing_duration
        upper, lower, states = [], [], []
        while foot <= last:
            if t > t_switch:
                state, foot, dur = self._transition(state, foot, last)
                t_switch += dur
            if foot <= last:
                if state is State.SINGLE_SUPPORT:
                    f = feet[foot]
                    upper.append([f.z_max[0], f.z_max[1]])
                    lower.append([f.z_min[0], f.z_min[1]])
                else:
                    a, b = feet[foot - 1], feet[foot]
                    upper.append([max(a.z_max[0], b.z_max[0]), max(a.z_max[1], b.z_max[1])])
                    lower.append([min(a.z_min[0], b.z_min[0]), min(a.z_min[1], b.z_min[1])])
                states.append(state)
            t += self.dt
        return np.array(upper), np.array(lower), states
