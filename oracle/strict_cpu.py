"""ctypes binding of ``oracle/strict_lq_cpu.c`` — TEST INFRASTRUCTURE ONLY.

The strict (ZMP box-constrained) rollout of zmp_controller.py:173-195 in the device kernel's
LQ / primal-dual active-set form, in C on the host's cores (OpenMP over (walk, axis)
instances).  Two uses, both outside the product: the checker of the kernel's algorithm
(tests/test_oracle.py pins it to the reference-driven strict fixtures and to the exact
box-QP oracle), and bench.py's optimized multi-core strict CPU baseline.  Built by
``make -C oracle`` (``__graft_entry__.build()``) into ``oracle/_build/``.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libstrict_cpu.so")
_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        f = lib.zmpc_cpu_strict_rollout
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int] + [ctypes.c_double] * 6 + \
            [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
             ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def rollout_strict(zmax, zmin, x0, N, dt, h, g, Q, R, kick=None, kick_step=-1, threads=0):
    """zmax/zmin [B,n,2] (or one shared [n,2]), x0 [B,2,3], kick [B] → (hist [B,n,2,3],
    status [B] int32, passes [B] uint64).  The LIPM constants are evaluated as the reference
    evaluates them (zmp_controller.py:18-20)."""
    zmax = np.ascontiguousarray(zmax, np.float64)
    zmin = np.ascontiguousarray(zmin, np.float64)
    x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 2, 3)
    B = x0.shape[0]
    if zmax.ndim == 2:
        n, bstride = zmax.shape[0], 0
    else:
        n, bstride = zmax.shape[1], 2 * zmax.shape[1]
    T = float(dt)
    kk = None if kick is None else np.ascontiguousarray(kick, np.float64).reshape(B)
    hist = np.empty((B, n, 2, 3))
    status = np.zeros(B, np.int32)
    passes = np.zeros(B, np.uint64)
    rc = load().zmpc_cpu_strict_rollout(B, n, int(N), T, (T ** 2) / 2, (T ** 3) / 6, h / g,
                                        float(Q), float(R), _p(zmax), _p(zmin), bstride, _p(x0),
                                        _p(kk), int(kick_step), _p(hist), _p(status),
                                        _p(passes), int(threads))
    if rc != 0:
        raise RuntimeError(f"zmpc_cpu_strict_rollout failed ({rc})")
    return hist, status, passes
