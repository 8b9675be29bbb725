"""CPU ORACLE of the Herdt joint footstep QP — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker.  The product path (mpc_bipedal) never imports it.

Restates, in NumPy, the Herdt path of the reference controller
(src/mpc_bipedal/controllers/zmp_controller.py, reference @ 2025-12-26):
  find_nb_steps                   :203-433   footstep-phase counters
  generate_com_trajectory_herdt   :435-531   rollout driver (foot bookkeeping, force kick)
  predict_herdt_joint             :533-826   the joint x/y QP with footstep variables
  _polytope_halfspace             :828-865   footstep polytope → A d <= b
The reference solves the QP with cvxpy → OSQP (polish=False).  Neither cvxpy (pinned only as
cvxpy>=1.2.0, requirements.txt:2) nor OSQP (no pin) is installed here, and there is no
network: parity with OSQP is UNPINNED.  This oracle returns the exact, KKT-certified optimum of
the same QP (Goldfarb–Idnani dual active set); OSQP's answer differs from it by up to its
tolerances.  The QP data themselves are pinned to the reference: tests/golden/
make_herdt_golden.py runs the reference's own predict_herdt_joint / generate_com_trajectory_herdt
with a recording stand-in for cvxpy that captures the problem at the reference's call site
(zmp_controller.py:785-787) and answers solve() with qp_solve below.
"""
import numpy as np

from .zmp_oracle import lipm, prediction_matrices

STANDING, DOUBLE_SUPPORT, SINGLE_SUPPORT = 0, 1, 2  # cop_generator.State order


# ----------------------------------------------------------------------------- exact QP

def qp_solve(Q, p, G=None, h=None, maxit=10000, tol=1e-12):
    """Exact solve of min ½xᵀQx + pᵀx s.t. G x <= h (Q symmetric positive definite) by the
    Goldfarb–Idnani dual active-set method (Math. Programming 27, 1983): start at the
    unconstrained minimum, add the most violated constraint, take the dual step (dropping
    active constraints whose multiplier would turn negative) until every constraint holds.
    Returns (x, lam) with lam >= 0 the multipliers of all rows of G.
    """
    Q = np.asarray(Q, np.float64)
    p = np.asarray(p, np.float64).ravel()
    n = len(p)
    L = np.linalg.cholesky(Q)

    def qinv(v):
        return np.linalg.solve(L.T, np.linalg.solve(L, v))

    x = -qinv(p)
    if G is None or len(G) == 0:
        return x, np.zeros(0)
    G = np.asarray(G, np.float64)
    h = np.asarray(h, np.float64).ravel()
    m = len(h)
    act = []          # active constraint indices
    u = np.zeros(0)   # their multipliers
    scale = np.maximum(1.0, np.abs(h)) * np.maximum(1.0, np.linalg.norm(G, axis=1))
    for _ in range(maxit):
        viol = (G @ x - h) / scale
        viol[act] = -np.inf
        j = int(np.argmax(viol))
        if viol[j] <= tol:
            break
        uplus = np.append(u, 0.0)
        while True:
            nj = G[j]
            # the step directions in the Q metric: r = S⁻¹NᵀQ⁻¹nj, S = NᵀQ⁻¹N by a Cholesky of S
            # while it is well conditioned, else (consecutive ZMP rows nearly parallel) from a
            # Householder QR of L⁻¹N, which stays accurate where S loses its digits
            b = np.linalg.solve(L, nj)
            if act:
                Bm = np.linalg.solve(L, G[act].T)     # L⁻¹N, n × q
                c = Bm.T @ b
                Ls = None
                try:
                    Ls = np.linalg.cholesky(Bm.T @ Bm)
                    dg = np.diag(Ls)
                    if dg.min() < 1e-6 * dg.max():
                        Ls = None
                except np.linalg.LinAlgError:
                    Ls = None
                if Ls is not None:
                    r = np.linalg.solve(Ls.T, np.linalg.solve(Ls, c))
                    zb = b - Bm @ r
                else:
                    U, Rf = np.linalg.qr(Bm)
                    cu = U.T @ b
                    r = np.linalg.solve(Rf, cu)        # N⁺-coefficients of nj
                    zb = b - U @ cu
            else:
                r = np.zeros(0)
                zb = b
            if np.linalg.norm(zb) <= 1e-13 * np.linalg.norm(b):
                zb = np.zeros_like(zb)                # nj depends on the active normals
            z = np.linalg.solve(L.T, zb)
            # dual step length (drop a constraint whose multiplier hits zero first)
            t1, k_drop = np.inf, -1
            for i in range(len(act)):
                if r[i] > 0:
                    ti = uplus[i] / r[i]
                    if ti < t1:
                        t1, k_drop = ti, i
            zn = z @ nj
            s = nj @ x - h[j]
            t2 = np.inf if abs(zn) <= 1e-300 else s / zn
            if not np.isfinite(t1) and not np.isfinite(t2):
                raise RuntimeError("QP infeasible")
            if not np.isfinite(t2):           # dual step only
                uplus[:-1] -= t1 * r
                uplus[-1] += t1
                del act[k_drop]
                uplus = np.delete(uplus, k_drop)
                continue
            t = min(t1, t2)
            x = x - t * z
            uplus[:-1] -= t * r
            uplus[-1] += t
            if t2 <= t1:                          # constraint j becomes active
                act.append(j)
                u = uplus
                break
            del act[k_drop]                       # partial step: drop and retry j
            uplus = np.delete(uplus, k_drop)
    lam = np.zeros(m)
    lam[act] = u
    return x, lam


def qp_kkt(Q, p, G, h, x, lam):
    """KKT residuals of (x, lam) for min ½xᵀQx + pᵀx s.t. G x <= h."""
    out = {"stationarity": float(np.abs(Q @ x + p + (G.T @ lam if len(lam) else 0)).max())}
    if len(lam):
        s = G @ x - h
        out["primal"] = float(max(0.0, s.max()))
        out["dual"] = float(max(0.0, -lam.min()))
        out["complementarity"] = float(np.abs(lam * s).max())
    return out


# ----------------------------------------------------------------------------- problem

def find_nb_steps(states):
    """find_nb_steps (zmp_controller.py:203-433) as an O(n) scan: result[i] =
    (steps to the next footstep change, total steps of the current footstep phase)."""
    s = np.asarray(states)
    n = len(s)
    nxt_ds = np.full(n + 1, n, np.int64)   # first DS index > i
    nxt_ss = np.full(n + 1, n, np.int64)   # first SS index > i
    for i in range(n - 1, -1, -1):
        nxt_ds[i] = i + 1 if i + 1 < n and s[i + 1] == DOUBLE_SUPPORT else nxt_ds[i + 1]
        nxt_ss[i] = i + 1 if i + 1 < n and s[i + 1] == SINGLE_SUPPORT else nxt_ss[i + 1]
    nb = np.zeros(n, np.int64)
    for i in range(n):
        rem = n - i
        if s[i] == STANDING:
            ids = nxt_ds[i]
            if ids >= n:
                nb[i] = rem
            else:
                iss = nxt_ss[ids]
                nb[i] = rem if iss >= n else iss - i - 1
        else:  # DS or SS: steps to the next DS
            j = nxt_ds[i]
            nb[i] = j - i if j < n else rem
    # start index of the DS run ending at or before j
    ds_start = np.zeros(n, np.int64)
    prev_ds = np.full(n, -1, np.int64)     # last DS index < i
    last = -1
    for i in range(n):
        prev_ds[i] = last
        if s[i] == DOUBLE_SUPPORT:
            ds_start[i] = ds_start[i - 1] if i > 0 and s[i - 1] == DOUBLE_SUPPORT else i
            last = i

    def total(i):
        rem = n - i
        if s[i] == DOUBLE_SUPPORT:
            return nxt_ds[i] - ds_start[i]
        if s[i] == SINGLE_SUPPORT:
            pd = prev_ds[i]
            return nxt_ds[i] - ds_start[pd] if pd >= 0 else rem
        return None

    tot = np.zeros(n, np.int64)
    t0 = total(0)
    tot[0] = nb[0] if s[0] == STANDING else t0
    for i in range(1, n):
        if s[i] == STANDING:
            pd = prev_ds[i]
            tot[i] = nb[pd] if pd >= 0 else tot[0]
        else:
            tot[i] = total(i)
    return [(int(a), int(b)) for a, b in zip(nb, tot)]


def support_segments(current, window):
    """Support-phase lengths l (zmp_controller.py:561-573): l[0] rows (counting one extra, as
    the reference does) for the current foot, then one entry per future footstep."""
    s = current
    lst = []
    c = 1
    for st in window:
        if st == s:
            c += 1
        elif s == DOUBLE_SUPPORT and st == SINGLE_SUPPORT:
            c += 1
        else:
            lst.append(c)
            c = 1
        s = st
    lst.append(c)
    return lst


def velocity_matrices(N, dt):
    """Pvs (N,3), Pvu (N,N) of zmp_controller.py:553-559 (velocity at steps 1..N)."""
    T = dt
    Pvs = np.zeros((N, 3))
    Pvs[:, 1] = 1.0
    Pvs[:, 2] = np.arange(1, N + 1) * T
    d = np.subtract.outer(np.arange(N), np.arange(N)).astype(np.float64)
    Pvu = np.where(d >= 0, (T ** 2) / 2.0 * (2 * d + 1), 0.0)
    return Pvs, Pvu


def polytope_halfspace(vertices):
    """A d <= b of the convex hull of the polygon's vertices (zmp_controller.py:828-865):
    outward normals, via scipy's ConvexHull as the reference."""
    from scipy.spatial import ConvexHull
    verts = np.asarray(vertices, np.float64)
    eq = ConvexHull(verts).equations
    return eq[:, :2], -eq[:, 2]


def herdt_qp(cfg, x_init, y_init, v_ref, x_fc, y_fc, current, window, foot_side):
    """The joint QP of predict_herdt_joint (zmp_controller.py:533-787) as (Q, p, G, h, N, m):
    variables u = [J_x (N), f_x (m), J_y (N), f_y (m)], objective ½uᵀQu + pᵀu, G u <= h."""
    N = len(window)
    T, h_, g_ = cfg.dt, cfg.h, cfg.g
    Px, Pu = prediction_matrices(N, T, h_, g_)
    Pvs, Pvu = velocity_matrices(N, T)
    lst = support_segments(current, window)
    m = len(lst) - 1
    U = np.zeros((N, m))
    Uc = np.zeros((N, 1))
    Uc[: lst[0], 0] = 1
    nc = lst[0]
    for i, nf in enumerate(lst[1:]):
        U[nc: nc + nf, i] = 1
        nc += nf
    al, be, ga = cfg.alpha, cfg.beta, cfg.gamma
    Qxx = al * np.eye(N) + be * (Pvu.T @ Pvu) + ga * (Pu.T @ Pu)
    Qxf = -ga * (Pu.T @ U)
    Qa = np.block([[Qxx, Qxf], [Qxf.T, ga * (U.T @ U)]])
    Qa = 0.5 * (Qa + Qa.T)
    n1 = N + m
    Q = np.zeros((2 * n1, 2 * n1))
    Q[:n1, :n1] = Qa
    Q[n1:, n1:] = Qa
    ps = []
    for st, vr, fc in ((x_init, v_ref[:, 0:1], x_fc), (y_init, v_ref[:, 1:2], y_fc)):
        st = np.asarray(st, np.float64).reshape(3, 1)
        ev = Pvs @ st - vr
        ez = Px @ st - Uc * float(fc)
        ps.append(np.vstack([be * (Pvu.T @ ev) + ga * (Pu.T @ ez), -ga * (U.T @ ez)]).ravel())
    p = np.concatenate(ps)
    rows, rhs = [], []
    window = np.asarray(window)
    standing = np.where(window == STANDING)[0]
    keep = np.ones(N, bool)
    keep[standing] = False
    for ax, (st, fc, bnd) in enumerate(((x_init, x_fc, cfg.foot_length),
                                        (y_init, y_fc, cfg.foot_width))):
        st = np.asarray(st, np.float64).reshape(3, 1)
        zn = (Px @ st).ravel()
        fcv = (Uc * float(fc)).ravel()
        b = 0.5 * bnd
        off = ax * n1
        for k in np.where(keep)[0]:
            r = np.zeros(2 * n1)
            r[off: off + N] = Pu[k]
            r[off + N: off + n1] = -U[k]
            rows.append(r)
            rhs.append(b - zn[k] + fcv[k])
        for k in np.where(keep)[0]:
            r = np.zeros(2 * n1)
            r[off: off + N] = -Pu[k]
            r[off + N: off + n1] = U[k]
            rows.append(r)
            rhs.append(b + zn[k] - fcv[k])
    if (current == STANDING or keep.sum() == 0) and len(standing) > 0:
        fs = cfg.foot_spread
        yl, yr = (float(y_fc), float(y_fc) - 2 * fs) if foot_side == "left" else \
            (float(y_fc) + 2 * fs, float(y_fc))
        lims = ((float(x_fc) - 0.5 * cfg.foot_length, float(x_fc) + 0.5 * cfg.foot_length),
                (min(yl, yr) - 0.5 * cfg.foot_width, max(yl, yr) + 0.5 * cfg.foot_width))
        for ax, st in enumerate((x_init, y_init)):
            st = np.asarray(st, np.float64).reshape(3, 1)
            zn = (Px @ st).ravel()
            lo, hi = lims[ax]
            off = ax * n1
            for k in standing:
                r = np.zeros(2 * n1)
                r[off: off + N] = Pu[k]
                rows.append(r)
                rhs.append(hi - zn[k])
            for k in standing:
                r = np.zeros(2 * n1)
                r[off: off + N] = -Pu[k]
                rows.append(r)
                rhs.append(-lo + zn[k])
    if m > 0:
        verts = cfg.left_foot_polytope if foot_side == "left" else cfg.right_foot_polytope
        Ap, bp = polytope_halfspace(verts)
        for a, b in zip(Ap, bp):
            r = np.zeros(2 * n1)
            r[N] = a[0]
            r[n1 + N] = a[1]
            rows.append(r)
            rhs.append(b + a[0] * float(x_fc) + a[1] * float(y_fc))
    G = np.array(rows) if rows else np.zeros((0, 2 * n1))
    return Q, p, G, np.array(rhs), N, m


def herdt_solve(Q, p, G, h, N, m):
    """Exact solution of herdt_qp's problem.  A footstep variable whose support segment lies
    past the horizon (the reference's U column is empty: U[N:N+1]) does not enter the
    objective: it is fixed to the previous footstep, the first one to the point of the
    polytope nearest the current foot (OSQP's choice there is whatever its iterate was —
    unpinned)."""
    n1 = N + m
    colsum = np.abs(Q[N:n1, N:n1]).sum(axis=1) if m else np.zeros(0)
    empty = [i for i in range(m) if colsum[i] == 0.0]
    if not empty:
        return qp_solve(Q, p, G, h)
    keep = np.ones(2 * n1, bool)
    fixed = np.zeros(2 * n1)
    for i in empty:
        keep[N + i] = keep[n1 + N + i] = False
    if 0 in empty:
        # nearest polytope point to the current foot: rows of G on (f_x0, f_y0) only
        poly = np.where((np.abs(G[:, N]) + np.abs(G[:, n1 + N]) > 0)
                        & (np.abs(np.delete(G, [N, n1 + N], axis=1)).sum(axis=1) == 0))[0]
        A2 = G[poly][:, [N, n1 + N]]
        d2, _ = qp_solve(np.eye(2), np.zeros(2), A2, h[poly])
        fixed[N], fixed[n1 + N] = d2
    for i in empty:
        if i > 0:
            fixed[N + i] = fixed[N + i - 1]
            fixed[n1 + N + i] = fixed[n1 + N + i - 1]
    # reduced problem
    Qr = Q[np.ix_(keep, keep)]
    pr = p[keep] + Q[np.ix_(keep, ~keep)] @ fixed[~keep]
    Gr = G[:, keep]
    hr = h - G[:, ~keep] @ fixed[~keep]
    live = np.abs(Gr).sum(axis=1) > 0
    xr, lr = qp_solve(Qr, pr, Gr[live], hr[live])
    x = fixed.copy()
    x[keep] = xr
    lam = np.zeros(len(h))
    lam[live] = lr
    return x, lam


def herdt_step(cfg, x_init, y_init, v_ref, x_fc, y_fc, current, window, foot_side):
    """predict_herdt_joint (zmp_controller.py:533-826) with the exact QP: returns
    (x_next (3,), y_next (3,), first_x_footstep or None, first_y_footstep or None)."""
    Q, p, G, h, N, m = herdt_qp(cfg, x_init, y_init, v_ref, x_fc, y_fc, current, window,
                                foot_side)
    u, _ = herdt_solve(Q, p, G, h, N, m)
    A, B, _ = lipm(cfg.dt, cfg.h, cfg.g)
    n1 = N + m
    xs = A @ np.asarray(x_init, np.float64).reshape(3) + B[:, 0] * u[0]
    ys = A @ np.asarray(y_init, np.float64).reshape(3) + B[:, 0] * u[n1]
    fx = u[N] if m > 0 else None
    fy = u[n1 + N] if m > 0 else None
    return xs, ys, fx, fy


def herdt_rollout(cfg, x_init, y_init, v_ref, states):
    """generate_com_trajectory_herdt (zmp_controller.py:435-531) with the exact QP.
    Returns (com [n,2], y_hist [n,3], foot_hist [n,2], x_hist [n,3])."""
    v_ref = np.asarray(v_ref, np.float64)
    states = np.asarray(states)
    n = len(v_ref)
    N = cfg.horizon
    force_time = n // 2
    x_fc, y_fc = 0.0, float(cfg.foot_spread)
    foot_side = "left"
    x_air, y_air = x_fc, y_fc
    fxh, fyh = [x_fc], [y_fc]
    cur = states[0]
    vpad = np.vstack([v_ref, np.repeat(v_ref[-1:], N, axis=0)])
    spad = np.concatenate([states, np.repeat(states[-1:], N)])
    nb = find_nb_steps(spad)
    xh = [np.asarray(x_init, np.float64).reshape(3)]
    yh = [np.asarray(y_init, np.float64).reshape(3)]
    for i in range(n - 1):
        xn, yn, fx, fy = herdt_step(cfg, xh[-1], yh[-1], vpad[i + 1: i + 1 + N], fxh[-1],
                                    fyh[-1], cur, spad[i + 1: i + 1 + N], foot_side)
        xh.append(xn)
        yh.append(yn)
        if fx is not None:
            x_air += (1 / nb[i][0]) * (fx - x_air)
        if fy is not None:
            y_air += (1 / nb[i][0]) * (fy - y_air)
        if spad[i + 1] != cur and cur == SINGLE_SUPPORT:
            foot_side = "left" if foot_side == "right" else "right"
            if fx is not None and fy is not None:
                fxh.append(float(fx))
                fyh.append(float(fy))
            else:
                fxh.append(x_air)
                fyh.append(y_air)
            x_air, y_air = fxh[-1], fyh[-1]
        else:
            fxh.append(fxh[-1])
            fyh.append(fyh[-1])
        if cfg.add_force and i == force_time:
            yh[-1] = yh[-1] - np.array([0.0, cfg.dt * cfg.F_ext / cfg.m, 0.0])
        if spad[i + 1] != cur:
            cur = spad[i + 1]
    xh, yh = np.array(xh), np.array(yh)
    com = np.stack([xh[:, 0], yh[:, 0]], 1)
    return com, yh, np.stack([fxh, fyh], 1), xh
