"""Zero Moment Point (ZMP) controller using Model Predictive Control — HIP device path.

Drop-in for the reference ``ZMPController`` (``src/mpc_bipedal/controllers/zmp_controller.py``):
same constructor, same attributes (``config``, ``A``, ``B``, ``C``, ``external_force``), same
method names, argument meanings, shapes, return values and errors for the Wieber path.  Every
QP solve runs in hand-written HIP kernels (``csrc/``) reached through the C-ABI of
``include/zmpc.h``; NumPy inputs are staged to the device and results copied back, which is
the only host work.  There is no CPU solver behind this class.

The Herdt joint footstep QP (``method="herdt"``, :203-531) runs on the device as well
(``csrc/herdt.hip``); its host bookkeeping is in ``controllers/herdt.py``.

Additions (not in the reference): ``generate_com_trajectory_batch`` /
``generate_state_trajectory_batch`` / ``generate_com_trajectory_herdt_batch`` for many walks or
disturbance scenarios at once, taking and returning torch device tensors.
"""

import warnings
from typing import Optional, Tuple

import numpy as np
import torch

from ..config import MPCConfig
from ..models.lipm_model import lipm_matrices
from ..solver import get_plan
from . import herdt

_FAILED = "QP solver did not find a solution (infeasible or other)."
_ST_MAXITER = 1  # include/zmpc.h ZMPC_ST_MAXITER
_ST_INFEASIBLE = 8  # include/zmpc.h ZMPC_ST_INFEASIBLE


class ZMPController:
    """ZMP Controller using Model Predictive Control for bipedal locomotion."""

    def __init__(self, config: MPCConfig):
        # zmp_controller.py:15-21
        self.config = config
        self.A, self.B, self.C = lipm_matrices(config.dt, config.h, config.g)
        self.external_force = True

    # ------------------------------------------------------------------ plans / helpers
    def _plan(self, horizon: Optional[int] = None):
        cfg = self.config
        if horizon is not None and int(horizon) != int(cfg.horizon):
            # predict_wieber_axis takes nb_steps explicitly (zmp_controller.py:149)
            from dataclasses import replace
            cfg = replace(cfg, horizon=int(horizon), dt=cfg.dt)
        return get_plan(cfg)

    def _raise_on_status(self, status):
        if int(status.max().item() if status.numel() else 0) != 0:
            raise RuntimeError(_FAILED)

    def _herdt_status(self, status):
        """Herdt drop-ins: the reference never raises on a failed joint QP — it prints a message,
        substitutes zero jerk and the air foot's centre and continues (zmp_controller.py:796-802).
        The kernel applies that same fallback to a solve whose swing polytope is infeasible
        (ZMPC_ST_INFEASIBLE, the analogue of OSQP returning no solution); a solve that reached the
        active-set pass cap (ZMPC_ST_MAXITER) keeps its last iterate, as OSQP returns its iterate
        at its own iteration limit.  Both warn; any other flag (non-finite state, footstep
        factorisation, more footsteps than the kernel was built for) raises RuntimeError."""
        st = status.cpu().numpy() if isinstance(status, torch.Tensor) else np.asarray(status)
        soft = _ST_MAXITER | _ST_INFEASIBLE
        if st.size and np.any(st & ~soft):
            raise RuntimeError(_FAILED)
        if st.size and np.any(st & soft):
            msg = (f"Joint QP solver failed in {int(np.count_nonzero(st & soft))} walk(s) "
                   f"(pass cap, last iterate kept: {int(np.count_nonzero(st & _ST_MAXITER))}; "
                   f"infeasible swing polytope, zero jerk and the air foot's centre used: "
                   f"{int(np.count_nonzero(st & _ST_INFEASIBLE))})")
            print(msg)
            warnings.warn(msg, RuntimeWarning, stacklevel=3)

    def _kick(self) -> float:
        # zmp_controller.py:106: dt * F_ext / m, subtracted from the y velocity
        return self.config.dt * self.config.F_ext / self.config.m

    # ------------------------------------------------------------------ reference API
    def generate_com_trajectory(self, x_init: np.ndarray, y_init: np.ndarray,
                                z_max: np.ndarray = None, z_min: np.ndarray = None,
                                v_ref: np.ndarray = None, state_ref: np.ndarray = None,
                                ) -> Tuple[np.ndarray, np.ndarray]:
        """Route on ``config.method`` (zmp_controller.py:23-57)."""
        method = self.config.method.lower()
        if method == "wieber":
            if z_max is None or z_min is None:
                raise ValueError("z_max and z_min are required for wieber method")
            return self.generate_com_trajectory_wieber(x_init, y_init, z_max, z_min)
        elif method == "herdt":
            if v_ref is None or state_ref is None:
                raise ValueError("v_ref and state_ref are required for herdt method")
            return self.generate_com_trajectory_herdt(x_init, y_init, v_ref, state_ref)
        else:
            raise ValueError(f"Unknown method: {method}. Must be 'wieber' or 'herdt'")

    def generate_com_trajectory_wieber(self, x_init: np.ndarray, y_init: np.ndarray,
                                       z_max: np.ndarray, z_min: np.ndarray
                                       ) -> Tuple[np.ndarray, np.ndarray]:
        """COM trajectory (n,2) and y state history (n,3,1) (zmp_controller.py:59-108)."""
        z_max = np.asarray(z_max, dtype=np.float64)
        z_min = np.asarray(z_min, dtype=np.float64)
        n_steps = len(z_min)
        force_time = n_steps // 2
        print(f"Time of the external force: {(force_time*self.config.dt):.2f}s")
        hist = self._rollout_host(x_init, y_init, z_max, z_min,
                                  self._kick() if self.config.add_force else None, force_time)
        com = hist[:, :, 0].copy()
        y_hist = hist[:, 1, :].reshape(n_steps, 3, 1).copy()
        return com, y_hist

    def generate_state_trajectory_wieber(self, x_init: np.ndarray, y_init: np.ndarray,
                                         z_max: np.ndarray, z_min: np.ndarray
                                         ) -> Tuple[np.ndarray, np.ndarray]:
        """Full x and y state histories (n,3,1) each, no force (zmp_controller.py:110-147)."""
        z_max = np.asarray(z_max, dtype=np.float64)
        z_min = np.asarray(z_min, dtype=np.float64)
        n_steps = len(z_min)
        hist = self._rollout_host(x_init, y_init, z_max, z_min, None, -1)
        return (hist[:, 0, :].reshape(n_steps, 3, 1).copy(),
                hist[:, 1, :].reshape(n_steps, 3, 1).copy())

    def predict_wieber_axis(self, x_init: np.ndarray, nb_steps: int, z_max: np.ndarray,
                            z_min: np.ndarray) -> np.ndarray:
        """One-axis next state (3,1) after the first optimal jerk (zmp_controller.py:149-201)."""
        plan = self._plan(nb_steps)
        x = np.asarray(x_init, dtype=np.float64).reshape(1, 3)
        zx = np.asarray(z_max, dtype=np.float64).reshape(1, -1)
        zn = np.asarray(z_min, dtype=np.float64).reshape(1, -1)
        if zx.shape[1] != nb_steps or zn.shape[1] != nb_steps:
            raise ValueError(f"z_max/z_min must hold nb_steps={nb_steps} rows")
        out, st = plan.step(x, zx, zn)
        if plan.strict:
            self._raise_on_status(st)
        return out.cpu().numpy().reshape(3, 1)

    # ------------------------------------------------------------------ Herdt
    def find_nb_steps(self, state_ref) -> list:
        """(steps to the next footstep change, steps of the current footstep phase) per index
        (zmp_controller.py:203-433)."""
        return herdt.find_nb_steps(state_ref)

    def _polytope_halfspace(self, vertices):
        """Convex polygon → (A, b) with A d <= b (zmp_controller.py:828-865)."""
        return herdt.polytope_halfspace(vertices)

    def generate_com_trajectory_herdt(self, x_init: np.ndarray, y_init: np.ndarray,
                                      v_ref: np.ndarray, state_ref: np.ndarray):
        """COM trajectory (n,2), y state history (n,3,1) and foot positions (n,2) of the Herdt
        joint footstep QP (zmp_controller.py:435-531), every QP on the device."""
        v_ref = np.asarray(v_ref, dtype=np.float64)
        n = len(v_ref)
        x0 = np.stack([np.asarray(x_init, np.float64).reshape(3),
                       np.asarray(y_init, np.float64).reshape(3)])[None]
        kick = np.array([self._kick()]) if self.config.add_force else None
        hist, foot, _ = self._herdt_rollout(x0, v_ref, herdt.encode_states(state_ref), kick,
                                            n // 2)
        hist, foot = hist[0].cpu().numpy(), foot[0].cpu().numpy()
        for i in np.nonzero(np.any(foot[1:] != foot[:-1], axis=1))[0]:
            # zmp_controller.py:510 (the footstep adopted when a single support ends)
            print(f"Je change : de ({foot[i, 0], foot[i, 1]}) à ({foot[i + 1, 0], foot[i + 1, 1]})")
        com = hist[:, :, 0].copy()
        return com, hist[:, 1, :].reshape(n, 3, 1).copy(), foot

    def predict_herdt_joint(self, x_init, y_init, v_ref, x_fc, y_fc, current_state, state_ref,
                            nb_steps, nb_steps_to_next_state, x_airc, y_airc, foot_side, idx):
        """One joint x/y step (zmp_controller.py:533-826): (next x state (3,1), next y state
        (3,1), first planned x footstep or None, first planned y footstep or None).  A solve whose
        swing polytope is infeasible takes the reference's fallback (:796-802): zero jerk (the
        kernel) and the air foot's centre x_airc / y_airc as the first footstep (here; the C-ABI
        step knows only the current foot); one at the pass cap keeps its last iterate."""
        plan = self._plan(nb_steps)
        v = np.asarray(v_ref, np.float64).reshape(1, nb_steps, 2)
        win = herdt.encode_states(state_ref).reshape(1, nb_steps)
        cur = herdt.encode_states([current_state])
        pad = herdt.pad_states(np.concatenate([cur, win[0]]), 0)[None]
        prm = herdt.make_params(self.config, herdt.max_footsteps(pad, nb_steps, 2))
        x = np.stack([np.asarray(x_init, np.float64).reshape(3),
                      np.asarray(y_init, np.float64).reshape(3)])[None]
        foot = np.array([[float(np.asarray(x_fc).reshape(-1)[0]),
                          float(np.asarray(y_fc).reshape(-1)[0])]])
        side = np.array([0 if foot_side == "left" else 1], np.int8)
        xn, step, st = plan.herdt_step(prm, x, v, win, cur, foot, side)
        self._herdt_status(st)
        failed = int(st[0]) & _ST_INFEASIBLE
        xn, step = xn[0].cpu().numpy(), step[0].cpu().numpy()
        fx = None if np.isnan(step[0]) else float(step[0])
        fy = None if np.isnan(step[1]) else float(step[1])
        if failed and fx is not None and x_airc is not None and y_airc is not None:
            fx = float(np.asarray(x_airc).reshape(-1)[0])
            fy = float(np.asarray(y_airc).reshape(-1)[0])
        return xn[0].reshape(3, 1), xn[1].reshape(3, 1), fx, fy

    def generate_com_trajectory_herdt_batch(self, x_init, v_ref, state_ref, F_ext=None,
                                            return_status: bool = False):
        """Many Herdt walks at once (addition): x_init [B,2,3] or None; v_ref [B,n,2] or a
        shared [n,2]; state_ref [B,n] or a shared [n] (State enums or int8 codes); F_ext [B]
        or None.  Returns (com [B,n,2], hist [B,n,2,3], foot [B,n,2]) on the device; with
        return_status=True also the per-walk status [B] (ZMPC_ST_* flags) instead of raising
        or warning on a failed walk."""
        v = torch.as_tensor(v_ref, dtype=torch.float64)
        n = int(v.shape[-2])
        st = herdt.encode_states(state_ref) if not isinstance(state_ref, torch.Tensor) \
            else state_ref.cpu().numpy().astype(np.int8)
        if x_init is not None:
            B = int(np.shape(x_init)[0])
        elif v.dim() == 3:
            B = int(v.shape[0])
        elif st.ndim == 2:
            B = int(st.shape[0])
        else:
            B = 1 if F_ext is None else int(np.size(F_ext))
        x0 = np.zeros((B, 2, 3)) if x_init is None else x_init
        kick = None
        if F_ext is not None:
            kick = self.config.dt * np.asarray(F_ext, np.float64).reshape(B) / self.config.m
        hist, foot, status = self._herdt_rollout(x0, v_ref, st, kick, n // 2,
                                                 check=not return_status)
        if return_status:
            return hist[..., 0], hist, foot, status
        return hist[..., 0], hist, foot

    def _herdt_rollout(self, x0, v_ref, st, kick, kick_step, check=True):
        plan = self._plan()
        N = plan.N
        st2 = np.atleast_2d(st)
        pad = np.concatenate([st2, np.repeat(st2[:, -1:], N, axis=1)], axis=1)
        n = st2.shape[1]
        prm = herdt.make_params(self.config, herdt.max_footsteps(pad, N, n))
        nb = np.array([[t[0] for t in herdt.find_nb_steps(p)][:n] for p in pad], np.int32)
        if st.ndim == 1:
            nb = nb[0]
        hist, foot, status = plan.herdt_rollout(prm, v_ref, st, nb, x0, kick=kick,
                                                kick_step=kick_step)
        if check:
            self._herdt_status(status)
        return hist, foot, status

    # ------------------------------------------------------------------ batched additions
    def generate_state_trajectory_batch(self, x_init, z_max, z_min, F_ext=None,
                                        force_step: Optional[int] = None, walk_lengths=None):
        """Many walks at once; every input may be NumPy or a torch tensor.

        x_init : [B,2,3] initial (x-axis, y-axis) states, or None for zeros
        z_max, z_min : [B,n,2] per-walk CoP bounds, or [n,2] one CoP for every walk
        F_ext : None (no disturbance) or [B] forces in N; the y velocity at history index
                force_step+1 drops by dt·F_ext/m (default force_step = n//2, as
                zmp_controller.py:90,105-106)
        walk_lengths : [B] sample counts of ragged walks padded to n with their last row
                (CoPGenerator.generate_cop_batch); the force then hits step n_b//2 of each
                walk and hist[b, :n_b] is walk b's history
        Returns (hist [B,n,2,3], status [B]) on the plan's device.
        """
        plan = self._plan()
        dev = torch.device("cuda", plan.device)
        zmax_t = torch.as_tensor(z_max, dtype=torch.float64, device=dev)
        n = int(zmax_t.shape[-2])
        if x_init is None:
            B = 1 if zmax_t.dim() == 2 else int(zmax_t.shape[0])
            x0 = torch.zeros((B, 2, 3), dtype=torch.float64, device=dev)
        else:
            x0 = torch.as_tensor(x_init, dtype=torch.float64, device=dev)
            B = int(x0.shape[0])
        kick = None
        if F_ext is not None:
            F = torch.as_tensor(F_ext, dtype=torch.float64, device=dev).reshape(B)
            kick = self.config.dt * F / self.config.m
        if walk_lengths is not None:
            step = torch.as_tensor(walk_lengths, dtype=torch.int64, device=dev).reshape(B) // 2
        else:
            step = (n // 2) if force_step is None else int(force_step)
        hist, st = plan.rollout(zmax_t, z_min, x0, kick=kick, kick_step=step)
        if plan.strict:
            self._raise_on_status(st)
        return hist, st

    def generate_com_trajectory_batch(self, x_init, z_max, z_min, F_ext=None,
                                      force_step: Optional[int] = None, walk_lengths=None):
        """Batched generate_com_trajectory_wieber: (com [B,n,2], hist [B,n,2,3]) on device."""
        hist, _ = self.generate_state_trajectory_batch(x_init, z_max, z_min, F_ext, force_step,
                                                       walk_lengths)
        return hist[..., 0], hist

    def zmp(self, hist):
        """ZMP estimate C·state (run_mpc.py:294) for a [..., 3] state tensor or array."""
        C = self.C
        if isinstance(hist, torch.Tensor):
            return hist @ torch.as_tensor(C, dtype=hist.dtype, device=hist.device)
        return np.asarray(hist) @ C

    # ------------------------------------------------------------------ internals
    def _rollout_host(self, x_init, y_init, z_max, z_min, kick, kick_step) -> np.ndarray:
        if z_max.ndim != 2 or z_max.shape[1] != 2 or z_min.shape != z_max.shape:
            raise ValueError("z_max and z_min must both be [n_steps, 2]")
        plan = self._plan()
        x0 = np.stack([np.asarray(x_init, dtype=np.float64).reshape(3),
                       np.asarray(y_init, dtype=np.float64).reshape(3)])[None]
        kick_arr = None if kick is None else np.array([kick], dtype=np.float64)
        hist, st = plan.rollout(z_max[None], z_min[None], x0, kick=kick_arr, kick_step=kick_step)
        if plan.strict:
            self._raise_on_status(st)
        return hist[0].cpu().numpy()
