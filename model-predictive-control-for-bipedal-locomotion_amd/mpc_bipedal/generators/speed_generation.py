"""Reference CoM speed trajectories.

Mirrors ``SpeedTrajectoryGenerator`` of the reference
(``src/mpc_bipedal/generators/speed_generation.py:11-67``): same constructor, same
``generate_speed_and_state`` signature, modes and errors.  The "wieber" mode is a direct
caller of the hot path — the state rollout runs on the device through
``ZMPController.generate_state_trajectory_wieber``; ``generate_speed_batch`` is the batched
form (many walks per launch).
"""
from typing import List, Tuple

import numpy as np

from .cop_generator import CoPGenerator, State
from ..config import MPCConfig


class SpeedTrajectoryGenerator:
    """Generates reference CoM speed trajectories aligned with the CoP/state timeline."""

    def __init__(self, config: MPCConfig):
        from ..controllers.zmp_controller import ZMPController
        self.config = config
        self._cop_generator = CoPGenerator(config)
        self._zmp_controller = ZMPController(config)

    def generate_speed_and_state(self, save_footsteps: bool = True, output_dir: str = "results"
                                 ) -> Tuple[np.ndarray, np.ndarray, List[State]]:
        """(v_x [n], v_y [n], states [n]) — speed_generation.py:19-67.

        "classic": vx = 0.3 m/s except 0 while STANDING, vy = 0.
        "wieber": the velocity row of the Wieber state rollout from a zero initial state.
        """
        z_max, z_min, states = self._cop_generator.generate_cop_trajectory(
            save_footsteps=save_footsteps, output_dir=output_dir)
        mode = (self.config.speed_generation or "wieber").lower()
        if mode == "classic":
            v_x = [0.0 if s == State.STANDING else 0.3 for s in states]
            v_y = [0.0 for _ in states]
            return np.array(v_x), np.array(v_y), states
        if mode == "wieber":
            x_hist, y_hist = self._zmp_controller.generate_state_trajectory_wieber(
                x_init=np.zeros((3, 1)), y_init=np.zeros((3, 1)), z_max=z_max, z_min=z_min)
            return x_hist[:, 1, 0], y_hist[:, 1, 0], states
        raise ValueError(f"Unknown speed_generation mode: {self.config.speed_generation}")

    def generate_speed_batch(self, z_max, z_min, x0=None):
        """Batched "wieber" speeds: z_max/z_min [B,n,2] (or a shared [n,2]), x0 [B,2,3]
        (default zero) → (v_x [B,n], v_y [B,n]) device tensors, one rollout for all walks."""
        hist, st = self._zmp_controller.generate_state_trajectory_batch(x0, z_max, z_min)
        if self.config.strict:
            self._zmp_controller._raise_on_status(st)
        return hist[:, :, 0, 1], hist[:, :, 1, 1]
