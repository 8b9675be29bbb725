"""MPC bipedal locomotion — MI355X-native batched Wieber ZMP-MPC solver.

Mirrors the reference package layout (``src/mpc_bipedal``): ``config.MPCConfig``,
``controllers.ZMPController``, ``generators`` (CoP / footstep input producer) and the
``models.lipm_model`` the reference documents.  The QP solves run in HIP kernels for gfx950
(``../csrc``) behind the C-ABI ``include/zmpc.h``.
"""

__version__ = "0.1.0"
