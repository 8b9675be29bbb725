"""Host side of the Herdt joint footstep QP (zmp_controller.py:203-531, :828-865).

Everything here is bookkeeping around the device solver (``csrc/herdt.hip`` through
``zmpc_herdt_rollout`` / ``zmpc_herdt_step``): the footstep-phase counters of
``find_nb_steps``, the swing polytopes in half-space form, the support-state encoding and the
per-batch footstep bound that sizes the kernel.  No QP is solved on the host.
"""
import ctypes
from typing import List, Sequence, Tuple

import numpy as np

from .. import _native
from ..generators.cop_generator import State

# int8 codes of cop_generator.State on the device (include/zmpc.h)
STANDING, DOUBLE_SUPPORT, SINGLE_SUPPORT = 0, 1, 2
_CODE = {State.STANDING: STANDING, State.DOUBLE_SUPPORT: DOUBLE_SUPPORT,
         State.SINGLE_SUPPORT: SINGLE_SUPPORT}


def encode_states(states) -> np.ndarray:
    """State enums (or their names, or the int8 codes) → int8 codes."""
    out = []
    for s in np.asarray(states, dtype=object).ravel():
        if isinstance(s, State):
            out.append(_CODE[s])
        elif isinstance(s, str):
            out.append(_CODE[State(s)])
        else:
            out.append(int(s))
    return np.asarray(out, dtype=np.int8).reshape(np.shape(states))


def find_nb_steps(states) -> List[Tuple[int, int]]:
    """``find_nb_steps`` (zmp_controller.py:203-433): for each index, (timesteps to the next
    footstep change, timesteps of the current footstep phase), vectorised over the sequence."""
    s = encode_states(states).astype(np.int64)
    n = len(s)
    idx = np.arange(n)
    big = n

    def next_index(mask):
        # first j > i with mask[j] (n if none)
        pos = np.where(mask, idx, big)
        nxt = np.minimum.accumulate(pos[::-1])[::-1]
        return np.append(nxt[1:], big)

    def prev_index(mask):
        # last j < i with mask[j] (-1 if none)
        pos = np.where(mask, idx, -1)
        prv = np.maximum.accumulate(pos)
        return np.insert(prv[:-1], 0, -1)

    ds = s == DOUBLE_SUPPORT
    nds = next_index(ds)
    nss = next_index(s == SINGLE_SUPPORT)
    rem = n - idx
    # steps to the next change
    after_ds_ss = np.where(nds < n, np.append(nss, big)[np.minimum(nds, n)], big)
    nb_stand = np.where(nds >= n, rem, np.where(after_ds_ss >= n, rem, after_ds_ss - idx - 1))
    nb_walk = np.where(nds < n, nds - idx, rem)
    nb = np.where(s == STANDING, nb_stand, nb_walk)
    # first index of the DS run containing each DS sample
    run_start = np.where(ds & ~np.insert(ds[:-1], 0, False), idx, -1)
    run_start = np.maximum.accumulate(run_start)
    pds = prev_index(ds)
    tot_ds = nds - run_start
    tot_ss = np.where(pds >= 0, nds - run_start[np.maximum(pds, 0)], rem)
    tot = np.where(s == DOUBLE_SUPPORT, tot_ds, np.where(s == SINGLE_SUPPORT, tot_ss, 0))
    tot0 = nb[0] if s[0] == STANDING else tot[0]
    stand_tot = np.where(pds >= 0, nb[np.maximum(pds, 0)], tot0)
    tot = np.where(s == STANDING, stand_tot, tot)
    if n:
        tot[0] = tot0
    return [(int(a), int(b)) for a, b in zip(nb, tot)]


def polytope_halfspace(vertices) -> Tuple[np.ndarray, np.ndarray]:
    """``_polytope_halfspace`` (zmp_controller.py:828-865): A d <= b of the convex hull of
    the polygon (outward normals), with the reference's checks and errors."""
    from scipy.spatial import ConvexHull
    verts = np.asarray(vertices, dtype=float)
    if verts.ndim != 2 or verts.shape[1] != 2 or len(verts) < 3:
        raise ValueError("Polytope must be array-like of shape (k, 2), k>=3")
    eq = ConvexHull(verts).equations
    vals = (eq[:, :2] @ verts.T).T + eq[:, 2].reshape(1, -1)
    if np.max(vals) > 1e-10:
        raise ValueError(f"Polytope half-space conversion failed: max violation = {np.max(vals)}")
    return eq[:, :2], -eq[:, 2]


def max_footsteps(padded_states: np.ndarray, horizon: int, n_steps: int) -> int:
    """Most footsteps inside one horizon window of a rollout: at step i the window is
    samples i+1..i+N of the padded sequence and the current state is sample i, so the
    footsteps are the phase breaks (a state change other than DOUBLE→SINGLE support,
    zmp_controller.py:561-573) among transitions i..i+N−1.  padded_states [B, n+N] int8."""
    s = np.asarray(padded_states, dtype=np.int64)
    a, b = s[:, :-1], s[:, 1:]
    brk = ((a != b) & ~((a == DOUBLE_SUPPORT) & (b == SINGLE_SUPPORT))).astype(np.int64)
    cs = np.concatenate([np.zeros((len(s), 1), np.int64), np.cumsum(brk, axis=1)], axis=1)
    i = np.arange(max(n_steps - 1, 1))
    win = cs[:, i + horizon] - cs[:, i]
    return int(win.max()) if win.size else 0


class HerdtParams(ctypes.Structure):
    """zmpc_herdt_params (include/zmpc.h)."""
    _fields_ = [("alpha", ctypes.c_double), ("beta", ctypes.c_double),
                ("gamma", ctypes.c_double), ("foot_length", ctypes.c_double),
                ("foot_width", ctypes.c_double), ("foot_spread", ctypes.c_double),
                ("nfacets", ctypes.c_int32 * 2),
                ("facets", ((ctypes.c_double * 3) * _native.HERDT_MAX_FACETS) * 2),
                ("max_footsteps", ctypes.c_int32), ("max_passes", ctypes.c_int32)]


def make_params(config, max_steps: int) -> HerdtParams:
    p = HerdtParams()
    p.alpha, p.beta, p.gamma = float(config.alpha), float(config.beta), float(config.gamma)
    p.foot_length, p.foot_width = float(config.foot_length), float(config.foot_width)
    p.foot_spread = float(config.foot_spread)
    for side, verts in enumerate((config.left_foot_polytope, config.right_foot_polytope)):
        A, b = polytope_halfspace(np.array(verts))
        if len(b) > _native.HERDT_MAX_FACETS:
            raise ValueError(f"swing polytope has {len(b)} facets "
                             f"(at most {_native.HERDT_MAX_FACETS})")
        p.nfacets[side] = len(b)
        for f in range(len(b)):
            p.facets[side][f][0] = float(A[f, 0])
            p.facets[side][f][1] = float(A[f, 1])
            p.facets[side][f][2] = float(b[f])
    if max_steps > 8:
        raise ValueError(f"{max_steps} footsteps inside one horizon window (at most 8 are "
                         "supported by the device solver)")
    p.max_footsteps = int(max_steps)
    return p


def pad_states(states: Sequence, horizon: int) -> np.ndarray:
    """Pad with `horizon` copies of the last state (zmp_controller.py:466-469)."""
    s = encode_states(states)
    return np.concatenate([s, np.repeat(s[-1:], horizon)])
