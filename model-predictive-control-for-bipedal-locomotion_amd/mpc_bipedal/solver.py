"""Device-side solver objects on top of the C-ABI (``include/zmpc.h``).

``Plan`` owns one ``zmpc_plan`` (batch-invariant matrices on one HIP device).  Its methods
take torch tensors that live on that device (PyTorch-ROCm is used for device buffers and
streams only) and launch the HIP kernels on torch's current stream.
"""

import ctypes
import os
import weakref
from collections import OrderedDict

import numpy as np
import torch

from . import _native
from .models.lipm_model import plan_constants

# get_plan's cache: least recently used plans beyond ZMPC_PLAN_CACHE (default 8) are dropped
# (a plan holds N² matrices and the FFT tables; a caller sweeping horizons, as
# run_compare_runtime.py:139 does, would otherwise keep one per N)
_PLAN_CACHE = OrderedDict()
PLAN_CACHE_MAX = max(1, int(os.environ.get("ZMPC_PLAN_CACHE", "8")))


def _device_index(backend: str) -> int:
    if not torch.cuda.is_available():
        raise RuntimeError("the ZMP-MPC solver needs a HIP device (torch.cuda.is_available() is "
                           "False); there is no CPU fallback")
    if backend in ("hip", "cuda", None):
        return torch.cuda.current_device()
    for prefix in ("hip:", "cuda:"):
        if backend.startswith(prefix):
            return int(backend[len(prefix):])
    raise ValueError(f"unknown backend {backend!r} (expected 'hip' or 'hip:<index>')")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Plan:
    """Batch-invariant solver plan for one (N, dt, h, g, Q, R, strict) on one device."""

    def __init__(self, device: int, N: int, dt: float, h: float, g: float, Q: float, R: float,
                 strict: bool):
        lib = _native.load()
        self.device = int(device)
        self.N = int(N)
        self.dt, self.h, self.g, self.Q, self.R = float(dt), float(h), float(g), float(Q), float(R)
        self.strict = bool(strict)
        c = plan_constants(self.dt, self.h, self.g)
        self.consts = c
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = lib.zmpc_plan_create(self.device, self.N, c["T"], c["T2_2"], c["T3_6"], c["hg"],
                                      c["Thg"], self.Q, self.R, int(self.strict),
                                      ctypes.c_void_p(stream), ctypes.byref(handle))
        _native.check(rc, "zmpc_plan_create")
        self._h = handle
        self._finalizer = weakref.finalize(self, lib.zmpc_plan_destroy, handle)

    @property
    def handle(self):
        return self._live()

    def _live(self):
        if self._h is None:
            raise RuntimeError("plan was destroyed")
        return self._h

    def destroy(self):
        """Free the device plan now (zmpc_plan_destroy) instead of at garbage collection; the
        object is unusable afterwards.  Idempotent."""
        if self._h is not None:
            self._finalizer()
            self._h = None

    def export(self, what: int) -> np.ndarray:
        n = {0: self.N, 1: 3 * self.N, 2: self.N ** 2, 3: self.N, 4: 3, 5: self.N ** 2,
             6: self.N ** 2, 7: self.N ** 2}[what]
        buf = np.empty(n, dtype=np.float64)
        rc = _native.load().zmpc_plan_export(
            self._live(), what, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n)
        _native.check(rc, "zmpc_plan_export")
        if what in (1,):
            return buf.reshape(self.N, 3)
        if what in (2, 5, 6, 7):
            return buf.reshape(self.N, self.N)
        return buf

    def counters(self, reset: bool = False) -> dict:
        """Active-set solver work counters (zmpc_plan_counters, include/zmpc.h), summed over this
        plan's launches since creation or the last reset; synchronises the device.  Strict
        solver: wave_passes .. launches; Herdt solver: the herdt_* keys."""
        buf = (ctypes.c_uint64 * _native.NCOUNTERS)()
        rc = _native.load().zmpc_plan_counters(self._live(), buf, _native.NCOUNTERS, int(reset))
        _native.check(rc, "zmpc_plan_counters")
        return {"wave_passes": int(buf[0]), "instance_passes": int(buf[1]),
                "working_set_slots": int(buf[2]), "launches": int(buf[3]),
                "herdt_wave_passes": int(buf[4]), "herdt_instance_passes": int(buf[5]),
                "herdt_footsteps": int(buf[6]), "herdt_footsteps_sq": int(buf[7]),
                "max_passes_per_solve": int(buf[8]), "herdt_max_passes_per_solve": int(buf[9])}

    def set_option(self, option, value: int) -> "Plan":
        """zmpc_plan_set_option: choose between forms that compute the same solution (cross-checks
        and A/B timing).  option: a name of _native.OPTIONS ("correlation", "long_walk",
        "rollout_kernel", "kick_order", "strict_solver", "strict_bounds") or its ZMPC_OPT_* number."""
        opt = _native.OPTIONS[option] if isinstance(option, str) else int(option)
        rc = _native.load().zmpc_plan_set_option(self._live(), opt, int(value))
        _native.check(rc, "zmpc_plan_set_option")
        return self

    def get_option(self, option) -> int:
        opt = _native.OPTIONS[option] if isinstance(option, str) else int(option)
        v = ctypes.c_int64()
        rc = _native.load().zmpc_plan_get_option(self._live(), opt, ctypes.byref(v))
        _native.check(rc, "zmpc_plan_get_option")
        return int(v.value)

    def timings(self) -> dict:
        """Plan-build stage durations in ms (zmpc_plan_timings; HIP events on the creation
        stream): name → ms, names as _native.PLAN_STAGE_NAMES."""
        buf = (ctypes.c_float * _native.PLAN_STAGES)()
        rc = _native.load().zmpc_plan_timings(self._live(), buf, _native.PLAN_STAGES)
        _native.check(rc, "zmpc_plan_timings")
        return {name: float(buf[i]) for i, name in enumerate(_native.PLAN_STAGE_NAMES)}

    # -- launches --------------------------------------------------------------------------
    def _dev(self):
        return torch.device("cuda", self.device)

    def _as_dev(self, a, shape=None):
        t = torch.as_tensor(a, dtype=torch.float64, device=self._dev())
        t = t.contiguous()
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    def step(self, x, zmax_win, zmin_win, status=None):
        """Batched predict_wieber_axis: x [B,3], windows [B,N] → x_next [B,3] (device)."""
        x = self._as_dev(x)
        B = x.shape[0]
        zmax_win = self._as_dev(zmax_win, (B, self.N))
        zmin_win = self._as_dev(zmin_win, (B, self.N))
        x = x.reshape(B, 3)
        out = torch.empty((B, 3), dtype=torch.float64, device=self._dev())
        st = status if status is not None else torch.empty(B, dtype=torch.int32,
                                                           device=self._dev())
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = _native.load().zmpc_step(self._live(), B, _ptr(x), _ptr(zmax_win), _ptr(zmin_win),
                                          _ptr(out), _ptr(st), ctypes.c_void_p(stream))
        _native.check(rc, "zmpc_step")
        return out, st

    def rollout_launcher(self, zmax, zmin, x0, kick=None, kick_step=-1, hist=None, status=None):
        """Validate once and return a zero-argument callable that re-issues the same rollout
        launch on the current stream (one ctypes call, no tensor checks): for timing loops
        and graph capture.  The tensors must stay alive while the launcher is used."""
        hist, status, (name, args, keep) = self._rollout_args(zmax, zmin, x0, kick, kick_step,
                                                              hist, status)
        fn = getattr(_native.load(), name)
        dev = self.device

        def launch():
            stream = torch.cuda.current_stream(dev).cuda_stream
            rc = fn(*args, ctypes.c_void_p(stream))
            if rc != 0:
                _native.check(rc, name)
        launch.hist, launch.status, launch.inputs = hist, status, keep
        return launch

    def rollout(self, zmax, zmin, x0, kick=None, kick_step=-1, hist=None, status=None):
        """Batched Wieber rollout → hist [B,n,2,3] (device), status [B] (see _rollout_args)."""
        hist, status, (name, args, _) = self._rollout_args(zmax, zmin, x0, kick, kick_step, hist,
                                                           status)
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = getattr(_native.load(), name)(*args, ctypes.c_void_p(stream))
        _native.check(rc, name)
        return hist, status

    def _rollout_args(self, zmax, zmin, x0, kick, kick_step, hist, status):
        """Batched Wieber rollout → hist [B,n,2,3] (device), status [B].

        zmax/zmin: [B,n,2] per-walk CoP bounds, or [n,2] one CoP shared by every walk;
        x0: [B,2,3]; kick: [B] velocity impulse subtracted from y at step kick_step — an int,
        or a [B] array of per-walk steps (ragged walks: zmpc_rollout_kicks).
        """
        zmax = self._as_dev(zmax)
        x0 = self._as_dev(x0)
        if x0.dim() != 3 or x0.shape[1:] != (2, 3):
            raise ValueError(f"x0 must be [B, 2, 3], got {tuple(x0.shape)}")
        B = int(x0.shape[0])
        if zmax.dim() == 2 and zmax.shape[1] == 2:
            n = int(zmax.shape[0])
            zmin = self._as_dev(zmin, (n, 2))
            bstride = 0
        elif zmax.dim() == 3 and zmax.shape[2] == 2 and zmax.shape[0] == B:
            n = int(zmax.shape[1])
            zmin = self._as_dev(zmin, (B, n, 2))
            bstride = 2 * n
        else:
            raise ValueError(f"z_max must be [B, n, 2] or [n, 2], got {tuple(zmax.shape)}")
        kick_t = None if kick is None else self._as_dev(kick, (B,))
        if hist is None:
            hist = torch.empty((B, n, 2, 3), dtype=torch.float64, device=self._dev())
        elif tuple(hist.shape) != (B, n, 2, 3) or hist.dtype != torch.float64 or \
                hist.device != self._dev() or not hist.is_contiguous():
            raise ValueError("hist must be a contiguous float64 [B, n, 2, 3] tensor on the "
                             "plan's device")
        if status is None:
            status = torch.empty(B, dtype=torch.int32, device=self._dev())
        if isinstance(kick_step, (int, np.integer)):
            args = (self._live(), B, n, _ptr(zmax), _ptr(zmin), bstride, _ptr(x0), _ptr(kick_t),
                    int(kick_step), _ptr(hist), _ptr(status))
            return hist, status, ("zmpc_rollout", args, (zmax, zmin, x0, kick_t))
        ks = torch.as_tensor(kick_step, dtype=torch.int64, device=self._dev()).contiguous()
        if tuple(ks.shape) != (B,):
            raise ValueError(f"per-walk kick_step must be [B], got {tuple(ks.shape)}")
        args = (self._live(), B, n, _ptr(zmax), _ptr(zmin), bstride, _ptr(x0), _ptr(kick_t),
                _ptr(ks), _ptr(hist), _ptr(status))
        return hist, status, ("zmpc_rollout_kicks", args, (zmax, zmin, x0, kick_t, ks))


    # -- Herdt joint footstep QP (zmpc_herdt_rollout / zmpc_herdt_step) --------------------
    def herdt_rollout(self, params, v_ref, states, nb_next, x0, kick=None, kick_step=-1):
        """Batched generate_com_trajectory_herdt → (hist [B,n,2,3], foot [B,n,2], status [B]).

        v_ref [B,n,2] or a shared [n,2]; states [B,n] or [n] int8 codes; nb_next [B,n] or [n]
        int32 (find_nb_steps of the padded states, first element); x0 [B,2,3]; kick [B] or
        None: y-velocity impulse at kick_step.  params: controllers.herdt.HerdtParams.
        """
        x0 = self._as_dev(x0)
        if x0.dim() != 3 or x0.shape[1:] != (2, 3):
            raise ValueError(f"x0 must be [B, 2, 3], got {tuple(x0.shape)}")
        B = int(x0.shape[0])
        v = self._as_dev(v_ref)
        if v.dim() not in (2, 3) or v.shape[-1] != 2:
            raise ValueError(f"v_ref must be [B, n, 2] or [n, 2], got {tuple(v.shape)}")
        n = int(v.shape[-2])
        if v.dim() == 2:
            vs = 0
        elif v.shape[0] == B:
            vs = 2 * n
        else:
            raise ValueError(f"v_ref must be [B, n, 2] or [n, 2], got {tuple(v.shape)}")
        dev = self._dev()
        st = torch.as_tensor(np.asarray(states, dtype=np.int8) if not isinstance(
            states, torch.Tensor) else states, dtype=torch.int8, device=dev).contiguous()
        nb = torch.as_tensor(np.asarray(nb_next, dtype=np.int32) if not isinstance(
            nb_next, torch.Tensor) else nb_next, dtype=torch.int32, device=dev).contiguous()
        # per-walk [B, n] or shared [n]: a 2-D array must carry one row per walk (the kernel
        # reads row b of walk b)
        for name, t in (("states", st), ("nb_next", nb)):
            if t.dim() not in (1, 2) or t.shape[-1] != n or (t.dim() == 2 and t.shape[0] != B):
                raise ValueError(f"{name} must be [B, n] = [{B}, {n}] or [n], got "
                                 f"{tuple(t.shape)}")
        ss = 0 if st.dim() == 1 else n
        ns = 0 if nb.dim() == 1 else n
        kick_t = None if kick is None else self._as_dev(kick, (B,))
        hist = torch.empty((B, n, 2, 3), dtype=torch.float64, device=dev)
        foot = torch.empty((B, n, 2), dtype=torch.float64, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = _native.load().zmpc_herdt_rollout(
                self._live(), ctypes.byref(params), B, n, _ptr(v), vs, _ptr(st), ss, _ptr(nb), ns,
                _ptr(x0), _ptr(kick_t), int(kick_step), _ptr(hist), _ptr(foot), _ptr(status),
                ctypes.c_void_p(stream))
        _native.check(rc, "zmpc_herdt_rollout")
        return hist, foot, status

    def herdt_step(self, params, x, v_win, s_win, current, foot, side):
        """Batched predict_herdt_joint: x [B,2,3], v_win [B,N,2], s_win [B,N] int8,
        current [B] int8, foot [B,2], side [B] int8 (0 left) → (x_next [B,2,3],
        first footstep [B,2] (NaN: none), status [B])."""
        x = self._as_dev(x)
        B = int(x.shape[0])
        dev = self._dev()
        v = self._as_dev(v_win, (B, self.N, 2))
        f = self._as_dev(foot, (B, 2))
        i8 = lambda a, shape: torch.as_tensor(np.asarray(a, dtype=np.int8).reshape(shape),
                                              device=dev).contiguous()
        sw, cu, sd = i8(s_win, (B, self.N)), i8(current, (B,)), i8(side, (B,))
        xn = torch.empty((B, 2, 3), dtype=torch.float64, device=dev)
        step = torch.empty((B, 2), dtype=torch.float64, device=dev)
        status = torch.empty(B, dtype=torch.int32, device=dev)
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = _native.load().zmpc_herdt_step(
                self._live(), ctypes.byref(params), B, _ptr(x), _ptr(v), _ptr(sw), _ptr(cu), _ptr(f),
                _ptr(sd), _ptr(xn), _ptr(step), _ptr(status), ctypes.c_void_p(stream))
        _native.check(rc, "zmpc_herdt_step")
        return xn, step, status


def get_plan(config, device=None) -> Plan:
    """Cached plan for an MPCConfig (keyed on every field the hot path reads)."""
    dev = _device_index(getattr(config, "backend", "hip")) if device is None else int(device)
    key = (dev, int(config.horizon), float(config.dt), float(config.h), float(config.g),
           float(config.Q), float(config.R), bool(config.strict))
    p = _PLAN_CACHE.get(key)
    if p is not None and p._h is not None:
        _PLAN_CACHE.move_to_end(key)
        return p
    p = Plan(dev, key[1], key[2], key[3], key[4], key[5], key[6], key[7])
    _PLAN_CACHE[key] = p
    while len(_PLAN_CACHE) > PLAN_CACHE_MAX:
        # drop the cache's reference only: a caller still holding the plan keeps it alive,
        # the device memory is freed when the last reference goes (weakref finalizer)
        _PLAN_CACHE.popitem(last=False)
    return p


def clear_plan_cache(destroy: bool = False):
    """Empty get_plan's cache; with destroy=True also free every cached plan now (callers must
    not use those plans afterwards)."""
    plans = list(_PLAN_CACHE.values())
    _PLAN_CACHE.clear()
    if destroy:
        for p in plans:
            p.destroy()
