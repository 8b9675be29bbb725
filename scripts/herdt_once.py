"""One batched Herdt rollout (config 6 inputs) after a warm-up, for rocprofv3 counter passes:
python scripts/herdt_once.py [B] [out.npy]  (out.npy: the history, for bitwise A/B of builds)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd"))
import torch  # noqa: E402
from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.controllers import herdt as H  # noqa: E402
from mpc_bipedal.generators import SpeedTrajectoryGenerator  # noqa: E402
from mpc_bipedal.solver import Plan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
cfg = MPCConfig(method="herdt", add_force=True)
vx, vy, states = SpeedTrajectoryGenerator(cfg).generate_speed_and_state(save_footsteps=False)
st = H.encode_states(states)
n, N = len(st), cfg.horizon
pad = H.pad_states(st, N)
nb = np.array([t[0] for t in H.find_nb_steps(pad)][:n], np.int32)
prm = H.make_params(cfg, H.max_footsteps(pad[None], N, n))
dev = torch.device("cuda", 0)
plan = Plan(0, N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, False)
rng = np.random.default_rng(1)
x0 = torch.zeros((B, 2, 3), dtype=torch.float64, device=dev)
kick = torch.as_tensor(cfg.dt * rng.uniform(0, 800, B) / cfg.m, device=dev)
v = torch.as_tensor(np.stack([vx, vy], 1), device=dev)
s_t = torch.as_tensor(st, device=dev)
nb_t = torch.as_tensor(nb, device=dev)
for _ in range(2):
    hist, foot, status = plan.herdt_rollout(prm, v, s_t, nb_t, x0, kick=kick, kick_step=n // 2)
torch.cuda.synchronize()
print("status max", int(status.abs().max()), plan.counters())
if len(sys.argv) > 2:
    np.save(sys.argv[2], torch.cat([hist.reshape(B, -1), foot.reshape(B, -1)], 1).cpu().numpy())
