"""Diagnostic: the device Herdt solver on the default walk of tests/golden/herdt_default.npz
(reference-driven rollout, exact QPs) and on its saved single steps; prints the errors."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd"))
import torch  # noqa: E402
from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.controllers import ZMPController  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "herdt_default.npz"))
cfg = MPCConfig(method="herdt", add_force=True)
c = ZMPController(cfg)
t = time.time()
com, y_hist, foot = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                              v_ref=d["v_ref"], state_ref=d["states"])
print(f"rollout {time.time() - t:.2f}s")
e_com = np.abs(com - d["com"]).max()
rm = float(np.sqrt(np.mean((com - d["com"]) ** 2)))
print(f"com max err {e_com:.3e} rmse {rm:.3e}; foot max err {np.abs(foot - d['foot_hist']).max():.3e}; "
      f"y max err {np.abs(y_hist[:, :, 0] - d['y_hist']).max():.3e}")
bad = np.nonzero(np.abs(com - d["com"]).max(axis=1) > 1e-9)[0]
print("first diverging rows", bad[:10])
A, B = c.A, c.B
for k in range(int(d["n_steps_saved"])):
    g = lambda key: d[f"step{k}_{key}"]
    N, m = int(g("N")), int(g("m"))
    side = "left" if int(g("side")) == 0 else "right"
    from mpc_bipedal.controllers.herdt import STANDING  # noqa: F401
    xn, yn, fx, fy = c.predict_herdt_joint(g("x"), g("y"), g("v"), g("fx"), g("fy"), int(g("cur")),
                                           g("win"), N, (1, 1), None, None, side, k)
    sol = g("sol")
    xr = A @ g("x").reshape(3, 1) + B * sol[0]
    yr = A @ g("y").reshape(3, 1) + B * sol[N + m]
    ef = (abs(fx - sol[N]) if fx is not None else 0.0, abs(fy - sol[2 * N + m]) if fy is not None else 0.0)
    print(f"step {k}: m={m} dx {np.abs(xn - xr).max():.2e} dy {np.abs(yn - yr).max():.2e} "
          f"dfoot {ef[0]:.2e} {ef[1]:.2e} (none: {fx is None})")
