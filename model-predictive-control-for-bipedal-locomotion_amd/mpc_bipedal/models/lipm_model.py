"""Linear inverted pendulum model (LIPM) with jerk input, and its prediction matrices.

The reference documents ``models/lipm_model.py`` (README.md:119-121, ARCHITECTURE.md:15-19)
but ships it only as stale bytecode (``__pycache__/model.cpython-312.pyc``: class
``LIPMModel`` with ``step``, ``get_zmp``, ``get_state_dimension``); the live code
inlines the same matrices in ``ZMPController.__init__`` (``zmp_controller.py:18-20``)
and rebuilds ``Px``/``Pu`` on every call (``zmp_controller.py:162-171``).

This module is the host-side model definition.  The device plan
(``csrc/plan.hip``) builds the same quantities on the GPU from the scalar
constants returned by :func:`plan_constants`, which are evaluated here with the
exact Python expressions the reference uses so that ``Px``/``Pu`` agree bit for bit.
"""

from dataclasses import dataclass

import numpy as np


def plan_constants(dt: float, h: float, g: float) -> dict:
    """Scalar constants of ``zmp_controller.py:18-20,166-171`` as the reference evaluates them.

    ``T ** 3`` in Python is ``pow`` (not ``T*T*T``); computing these on the host and passing
    them to the device keeps the device-built ``Px``/``Pu`` bit-identical to the reference.
    """
    T = float(dt)
    return dict(
        T=T,
        T2_2=(T ** 2) / 2,            # A[0,2], B[1], Px[:,2] factor
        T3_6=(T ** 3) / 6,            # B[0], Pu factor
        hg=h / g,                     # Px[:,2] offset, -C[2]
        Thg=T * h / g,                # Pu offset
    )


def lipm_matrices(dt: float, h: float, g: float):
    """``A`` (3,3), ``B`` (3,1), ``C`` (3,) exactly as ``zmp_controller.py:18-20``."""
    T = dt
    A = np.array([[1., T, T ** 2 / 2.], [0., 1., T], [0., 0., 1.]])
    B = np.array([T ** 3 / 6., T ** 2 / 2., T]).reshape((3, 1))
    C = np.array([1., 0., -h / g])
    return A, B, C


def toeplitz_column(N: int, dt: float, h: float, g: float) -> np.ndarray:
    """First column ``p`` of the lower-triangular Toeplitz ``Pu``: ``Pu[i,j] = p[i-j]``.

    ``p(d) = T³/6·(1+3d+3d²) − T·h/g`` (``zmp_controller.py:171``), same operation order.
    """
    c = plan_constants(dt, h, g)
    d = np.arange(N, dtype=np.int64)
    return c["T3_6"] * (1 + 3 * d + 3 * d ** 2).astype(np.float64) - c["Thg"]


def prediction_matrices(N: int, dt: float, h: float, g: float):
    """``Px`` (N,3) and ``Pu`` (N,N) as ``zmp_controller.py:162-171`` builds them."""
    c = plan_constants(dt, h, g)
    i = np.arange(N, dtype=np.int64)
    Px = np.empty((N, 3))
    Px[:, 0] = 1
    Px[:, 1] = c["T"] * (i + 1).astype(np.float64)
    Px[:, 2] = c["T2_2"] * ((i + 1) ** 2).astype(np.float64) - c["hg"]
    p = toeplitz_column(N, dt, h, g)
    D = i[:, None] - i[None, :]
    Pu = np.where(D >= 0, p[np.clip(D, 0, None)], 0.0)
    return Px, Pu


@dataclass
class ModelConfig:
    """Model parameters (legacy ``ModelConfig`` of the reference's root ``config.py``)."""
    dt: float = 0.01
    h: float = 0.75
    g: float = 9.81


class LIPMModel:
    """Discrete LIPM with jerk input: ``x⁺ = A x + B u``, ``zmp = C x``.

    Mirrors the legacy reference class (``__pycache__/model.cpython-312.pyc``):
    ``LIPMModel(config)`` stores ``g``, ``h``, ``dt`` and builds ``A``, ``B``, ``C``.
    """

    def __init__(self, config):
        self.g = config.g
        self.h = config.h
        self.dt = config.dt
        self.A, self.B, self.C = lipm_matrices(self.dt, self.h, self.g)

    def step(self, x: np.ndarray, u: float) -> np.ndarray:
        return self.A @ x + self.B * u

    def get_zmp(self, x: np.ndarray) -> float:
        return self.C @ x

    def get_state_dimension(self) -> int:
        return self.A.shape[0]

    def prediction_matrices(self, N: int):
        return prediction_matrices(N, self.dt, self.h, self.g)
