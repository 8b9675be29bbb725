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


def cop_params(config) -> List[float]:
    """The 7 producer parameters of a config, in zmpc_cop_generate's order."""
    return [float(config.distance), float(config.step_length), float(config.foot_spread),
            float(config.ssp_duration), float(config.dsp_duration),
            float(config.standing_duration), float(config.dt)]


def generate_cop_batch(params, device: int = 0):
    """Batched device CoP producer (C-ABI zmpc_cop_generate).

    params: a sequence of MPCConfig-like objects, or a [B, 7] array of (distance,
    step_length, foot_spread, ssp_duration, dsp_duration, standing_duration, dt).
    Returns device tensors (z_max [B, n_max, 2], z_min, n [B] int64, states [B, n_max] int8):
    walk b is rows [0, n_b), rows past n_b repeat its last row (the rollout's own window
    padding, so the padded batch rolls out each walk exactly); states use 0 STANDING,
    1 DOUBLE_SUPPORT, 2 SINGLE_SUPPORT, -1 padding.  Bit-exact with generate_cop_trajectory.
    """
    import ctypes
    import torch
    from .. import _native

    if not isinstance(params, (np.ndarray,)) and not hasattr(params, "shape"):
        params = [cop_params(c) for c in params]
    dev = torch.device("cuda", int(device))
    p = torch.as_tensor(np.asarray(params, dtype=np.float64), device=dev).contiguous()
    if p.dim() != 2 or p.shape[1] != 7:
        raise ValueError(f"params must be [B, 7], got {tuple(p.shape)}")
    B = int(p.shape[0])
    lib = _native.load()
    n = torch.zeros(B, dtype=torch.int64, device=dev)
    with torch.cuda.device(dev):
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        rc = lib.zmpc_cop_generate(int(device), B, p.data_ptr(), 0, None, None, None,
                                   n.data_ptr(), stream)
        _native.check(rc, "zmpc_cop_generate")
        n_cap = int(n.max().item()) if B else 0
        zmax = torch.empty((B, n_cap, 2), dtype=torch.float64, device=dev)
        zmin = torch.empty_like(zmax)
        states = torch.empty((B, n_cap), dtype=torch.int8, device=dev)
        if B and n_cap:
            rc = lib.zmpc_cop_generate(int(device), B, p.data_ptr(), n_cap, zmax.data_ptr(),
                                       zmin.data_ptr(), states.data_ptr(), None, stream)
            _native.check(rc, "zmpc_cop_generate")
    return zmax, zmin, n, states
