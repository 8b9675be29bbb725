"""Unified configuration for the MPC bipedal locomotion system.

Drop-in for the reference ``MPCConfig`` (``src/mpc_bipedal/config.py:13-87``): the
same fields, the same defaults and the same ``__post_init__`` rule
(``dt = 1.5 / horizon`` when ``dt`` is None, ``config.py:84-87``).  One field is
added, ``backend``, which never changes the meaning of the existing ones: the
solver always runs on the HIP device path; ``backend`` only names the device
(``"hip"`` = the current HIP device, ``"hip:<k>"`` = device k).
"""

from dataclasses import dataclass


@dataclass
class MPCConfig:
    """Unified configuration for CoP generation and the MPC controller."""

    # --- CoP generator parameters (config.py:17-23) ---
    ssp_duration: float = 24 * 0.01
    dsp_duration: float = 1 * 0.01
    standing_duration: float = 50 * 0.01
    distance: float = 2.1
    step_length: float = 0.3
    foot_spread: float = 0.1

    # Time step shared by the CoP generator and the controller (config.py:25-27).
    dt: float = None

    # --- MPC parameters (config.py:29-39) ---
    horizon: int = 150
    Q: float = 1.0
    R: float = 1e-6
    S: float = 1.0
    h: float = 0.75
    g: float = 9.81
    m: float = 40.0
    F_ext: float = 400.0
    strict: bool = True
    add_force: bool = True

    # --- method selection and Herdt parameters (config.py:41-82) ---
    method: str = "wieber"
    alpha: float = 1e-6
    beta: float = 1.0
    gamma: float = 1.0
    vx_ref: float = 0.0
    vy_ref: float = 0.0
    foot_length: float = 0.11
    foot_width: float = 0.05
    v_max_x: float = 0.9
    v_max_y: float = 0.5
    speed_generation: str = "classic"
    left_foot_polytope: tuple = (
        (-0.1, -0.3), (-0.1, -0.4), (0.0, -0.4), (0.0, -0.2), (0.1, -0.17), (0.2, -0.13),
        (0.3, -0.1), (0.7, -0.05), (0.8, -0.05), (0.8, -0.3), (0.4, -0.35),
    )
    right_foot_polytope: tuple = (
        (-0.1, 0.3), (-0.1, 0.4), (0.0, 0.4), (0.0, 0.2), (0.1, 0.17), (0.2, 0.13),
        (0.3, 0.1), (0.7, 0.05), (0.8, 0.05), (0.8, 0.3), (0.4, 0.35),
    )

    # --- addition: which HIP device the solver uses (never a CPU path) ---
    backend: str = "hip"

    def __post_init__(self):
        """Calculate dt from horizon if not explicitly provided (config.py:84-87)."""
        if self.dt is None:
            self.dt = 1.5 / self.horizon
