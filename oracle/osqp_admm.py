"""ORACLE (test infrastructure only) — restatement of the OSQP solver the reference calls.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

The reference builds one ``osqp.OSQP()`` per solver and drives it through its update API
(src/osqp_solver.py:38-40 setup with the CSC templates and ``verbose=False`` only;
:137-143 ``update(Px)``, ``update(Ax)``, ``update(q, l, u)``, ``solve()`` per QP).  OSQP is a
third-party dependency that is neither vendored nor pinned; this file restates
the published algorithm of the OSQP C library with its default settings:

  rho 0.1, sigma 1e-6, alpha 1.6, scaling 10 (Ruiz), eps_abs = eps_rel = 1e-3,
  eps_prim_inf = eps_dual_inf = 1e-4, max_iter 4000, check_termination 25, warm start on,
  polishing off, scaled_termination off, adaptive rho with tolerance 5, and (OSQP 1.x)
  check_dualgap on;

and the library's constants RHO_MIN 1e-6, RHO_MAX 1e6, RHO_EQ_OVER_RHO_INEQ 1e3, RHO_TOL 1e-4,
MIN_SCALING 1e-4, MAX_SCALING 1e4, OSQP_INFTY 1e30, OSQP_DIVISION_TOL 1e-30.

What is restated, routine by routine (names are OSQP's):
  * ``scale_data`` / ``unscale_data``: Ruiz equilibration of the KKT matrix [P A'; A 0], 10
    passes, each followed by the cost normalisation c; ``update_P`` / ``update_A`` unscale the
    stored data, write the new values and re-run the whole scaling on it — with the linear cost
    that is stored *at that moment*, i.e. the previous QP's q (the reference updates q last).
  * ``osqp_solve``: warm start from the stored (scaled) iterates x, z, y — they are not
    re-scaled when the scaling changes; per iteration ``update_xz_tilde`` (the quasi-definite KKT
    [P + sigma I, A'; A, -diag(1/rho)] solved exactly here; OSQP factors it with QDLDL, so the
    two agree to rounding), ``update_x``, ``update_z`` (projection on [l, u]), ``update_y``;
    every 25th iteration ``update_info`` + ``check_termination`` on the unscaled residuals,
    including the primal / dual infeasibility certificates; every ``adaptive_rho_interval``-th
    iteration ``adapt_rho`` from the scaled residuals.
    OSQP 1.x also requires the duality gap x'Px + q'x + SC(y) (SC the support function of
    [l, u]) below eps_abs + eps_rel max(|x'Px|, |q'x|, |SC(y)|) (``check_dualgap``).
  * ``store_solution``: x = D x, y = E y / c.

Two settings are not fixed by the reference's files: the OSQP version (0.6 has no duality-gap
test) and the adaptive-rho interval, which OSQP's timed builds (the PyPI wheels) set during the
first ``solve`` from the measured setup time (``adaptive_rho_fraction`` 0.4, rounded to a
multiple of 25; if the first solve ends earlier it stays 0 = never adapt).  Both are pinned by
the reference's own output: ``oracle/studies/osqp_trace.py`` re-runs the notebook's closed loop
(notebooks/pin_mpc_indy7.ipynb cell 2, the 500 goal distances it prints) through this class, and
with the gap test on and no rho adaptation the first 20 printed distances are reproduced to
6e-10 (the exact KKT solve: 1.1e-6; without the gap test: 6.7e-6; adaptive interval 25: 1.1e-5),
the first three to 1e-14.  These are the defaults below.
"""
from __future__ import annotations

import numpy as np
from scipy.sparse import bmat, csc_matrix, diags, identity
from scipy.sparse.linalg import splu

RHO_MIN, RHO_MAX, RHO_EQ_OVER_RHO_INEQ, RHO_TOL = 1e-6, 1e6, 1e3, 1e-4
MIN_SCALING, MAX_SCALING = 1e-4, 1e4
OSQP_INFTY, OSQP_DIVISION_TOL = 1e30, 1e-30

DEFAULTS = dict(rho=0.1, sigma=1e-6, alpha=1.6, scaling=10, eps_abs=1e-3, eps_rel=1e-3,
                eps_prim_inf=1e-4, eps_dual_inf=1e-4, max_iter=4000, check_termination=25,
                warm_start=True, adaptive_rho=True, adaptive_rho_interval=0,
                adaptive_rho_tolerance=5.0, infeasibility_checks=True, check_dualgap=True)


def _limit(v):
    v = np.where(v < MIN_SCALING, 1.0, v)
    return np.where(v > MAX_SCALING, MAX_SCALING, v)


class _Csc:
    """A CSC matrix whose structure stays fixed (explicit zeros included, as OSQP keeps them):
    the reference writes its value arrays by position (src/osqp_solver.py:140-141)."""

    def __init__(self, M):
        M = csc_matrix(M, copy=True)
        M.sort_indices()
        self.shape = M.shape
        self.indptr, self.indices = M.indptr.copy(), M.indices.copy()
        self.row = self.indices
        self.col = np.repeat(np.arange(M.shape[1]), np.diff(self.indptr))
        self.data = M.data.astype(float).copy()

    def mat(self):
        return csc_matrix((self.data, self.indices, self.indptr), shape=self.shape)

    def cols(self):
        out = np.zeros(self.shape[1])
        np.maximum.at(out, self.col, np.abs(self.data))
        return out

    def rows(self):
        out = np.zeros(self.shape[0])
        np.maximum.at(out, self.row, np.abs(self.data))
        return out

    def cols_sym_triu(self):
        """inf-norm of every column of the symmetric matrix whose upper triangle this stores."""
        a = np.abs(self.data)
        out = np.zeros(self.shape[1])
        np.maximum.at(out, self.col, a)
        np.maximum.at(out, self.row, a)
        return out


def _sym(P):
    """full symmetric matrix from the stored upper triangle."""
    M = P.mat()
    return (M + M.T - diags(M.diagonal())).tocsc()


class OSQP:
    """One OSQP workspace (osqp.OSQP) as the reference uses it."""

    def setup(self, P, q, A, l, u, **settings):
        self.s = dict(DEFAULTS)
        self.s.update(settings)
        self.n, self.m = P.shape[0], A.shape[0]
        # the workspace's own copies (OSQP copies the data at setup)
        self.P = _Csc(P)
        self.A = _Csc(A)
        self.q = np.array(q, float)
        self.l = np.clip(np.array(l, float), -OSQP_INFTY, OSQP_INFTY)
        self.u = np.clip(np.array(u, float), -OSQP_INFTY, OSQP_INFTY)
        self.D = np.ones(self.n)
        self.E = np.ones(self.m)
        self.c = 1.0
        self.Dinv, self.Einv, self.cinv = np.ones(self.n), np.ones(self.m), 1.0
        if self.s["scaling"]:
            self._scale_data()
        self.rho = self.s["rho"]
        self._set_rho_vec()
        self.x = np.zeros(self.n)
        self.z = np.zeros(self.m)
        self.y = np.zeros(self.m)
        self._lu = None
        self.info = {}
        self.history = []  # per solve: (iters, rho at exit, rho updates, checks, rho estimates, status)

    # ---- scaling (OSQP scaling.c) ----
    def _scale_data(self):
        n, m = self.n, self.m
        D, E, c = np.ones(n), np.ones(m), 1.0
        P, A, q = self.P, self.A, self.q
        for _ in range(self.s["scaling"]):
            Dt = np.maximum(P.cols_sym_triu(), A.cols())
            Et = A.rows()
            Dt = 1.0 / np.sqrt(_limit(Dt))
            Et = 1.0 / np.sqrt(_limit(Et))
            P.data = P.data * Dt[P.row] * Dt[P.col]
            A.data = A.data * Et[A.row] * Dt[A.col]
            q = Dt * q
            D = D * Dt
            E = E * Et
            ct = float(np.mean(P.cols_sym_triu()))
            nq = float(_limit(np.array([np.abs(q).max(initial=0.0)]))[0])
            ct = max(ct, nq)
            ct = float(_limit(np.array([ct]))[0])
            ct = 1.0 / ct
            P.data = P.data * ct
            q = q * ct
            c = c * ct
        self.q = q
        self.D, self.E, self.c = D, E, c
        self.Dinv, self.Einv, self.cinv = 1.0 / D, 1.0 / E, 1.0 / c
        self.l = E * self.l
        self.u = E * self.u

    def _unscale_data(self):
        P, A = self.P, self.A
        P.data = P.data * self.cinv * self.Dinv[P.row] * self.Dinv[P.col]
        self.q = self.Dinv * (self.q * self.cinv)
        A.data = A.data * self.Einv[A.row] * self.Dinv[A.col]
        self.l = self.Einv * self.l
        self.u = self.Einv * self.u

    # ---- rho (OSQP auxil.c set_rho_vec / osqp_update_rho) ----
    def _set_rho_vec(self):
        self.rho = min(max(self.rho, RHO_MIN), RHO_MAX)
        loose = (self.l < -OSQP_INFTY * MIN_SCALING) & (self.u > OSQP_INFTY * MIN_SCALING)
        eq = np.abs(self.u - self.l) < RHO_TOL
        self.rho_vec = np.where(loose, RHO_MIN, np.where(eq, RHO_EQ_OVER_RHO_INEQ * self.rho, self.rho))
        self.rho_inv = 1.0 / self.rho_vec
        self._lu = None

    def _factor(self):
        A = self.A.mat()
        K = bmat([[_sym(self.P) + self.s["sigma"] * identity(self.n), A.T],
                  [A, diags(-self.rho_inv)]], format="csc")
        self._lu = splu(K)

    # ---- updates (osqp_update_P / _A / _lin_cost / _bounds) ----
    def update(self, q=None, l=None, u=None, Px=None, Ax=None):
        if Px is not None:
            self._new_matrix("P", Px)
        if Ax is not None:
            self._new_matrix("A", Ax)
        if q is not None:
            self.q = self.c * (self.D * np.asarray(q, float))
        if l is not None or u is not None:
            ln = self.Einv * self.l if l is None else np.clip(np.asarray(l, float), -OSQP_INFTY, OSQP_INFTY)
            un = self.Einv * self.u if u is None else np.clip(np.asarray(u, float), -OSQP_INFTY, OSQP_INFTY)
            self.l = self.E * ln
            self.u = self.E * un
            self._set_rho_vec()  # osqp_update_bounds re-derives the constraint types

    def _new_matrix(self, which, vals):
        if self.s["scaling"]:
            self._unscale_data()
        M = getattr(self, which)
        assert len(vals) == len(M.data)
        M.data = np.asarray(vals, float).copy()
        if self.s["scaling"]:
            self._scale_data()
        self._lu = None

    # ---- residuals (OSQP auxil.c) ----
    def _info(self, x, z, y):
        A, Ps = self.A.mat(), _sym(self.P)
        Ax, Px, Aty = A @ x, Ps @ x, A.T @ y
        rp = Ax - z
        rd = self.q + Px + Aty
        # duality gap (OSQP 1.0 compute_duality_gap): x'Px + q'x + SC(y), unscaled by 1/c
        xPx = float(x @ Px) * self.cinv
        qx = float(self.q @ x) * self.cinv
        sc = float(self.u @ np.maximum(y, 0.0) + self.l @ np.minimum(y, 0.0)) * self.cinv
        return dict(Ax=Ax, Px=Px, Aty=Aty, rp=rp, rd=rd, gap=xPx + qx + sc, gap_terms=(xPx, qx, sc),
                    pri_res=float(np.abs(self.Einv * rp).max(initial=0.0)),
                    dua_res=float(self.cinv * np.abs(self.Dinv * rd).max(initial=0.0)))

    def _pri_tol(self, f, z, eps_abs, eps_rel):
        return eps_abs + eps_rel * max(np.abs(self.Einv * z).max(initial=0.0), np.abs(self.Einv * f["Ax"]).max(initial=0.0))

    def _dua_tol(self, f, eps_abs, eps_rel):
        r = max(np.abs(self.Dinv * self.q).max(initial=0.0), np.abs(self.Dinv * f["Aty"]).max(initial=0.0),
                np.abs(self.Dinv * f["Px"]).max(initial=0.0))
        return eps_abs + eps_rel * self.cinv * r

    def _primal_infeasible(self, dy, eps):
        dy = dy.copy()
        upinf = self.u > OSQP_INFTY * MIN_SCALING
        loinf = self.l < -OSQP_INFTY * MIN_SCALING
        dy[upinf & loinf] = 0.0
        dy[upinf & ~loinf] = np.minimum(dy[upinf & ~loinf], 0.0)
        dy[~upinf & loinf] = np.maximum(dy[~upinf & loinf], 0.0)
        nrm = np.abs(self.E * dy).max(initial=0.0)
        if nrm > OSQP_DIVISION_TOL:
            lhs = float(np.sum(self.u * np.maximum(dy, 0) + self.l * np.minimum(dy, 0)))
            if lhs < eps * nrm:
                return bool(np.abs(self.Dinv * (self.A.mat().T @ dy)).max() < eps * nrm)
        return False

    def _dual_infeasible(self, dx, eps):
        nrm = np.abs(self.D * dx).max(initial=0.0)
        cs = self.c
        if nrm > OSQP_DIVISION_TOL and float(self.q @ dx) < cs * eps * nrm:
            if np.abs(self.Dinv * (_sym(self.P) @ dx)).max() < cs * eps * nrm:
                Adx = self.Einv * (self.A.mat() @ dx)
                bad = ((self.u < OSQP_INFTY * MIN_SCALING) & (Adx > eps * nrm)) | \
                      ((self.l > -OSQP_INFTY * MIN_SCALING) & (Adx < -eps * nrm))
                return not bad.any()
        return False

    def _check(self, f, z, dx, dy, approximate=False):
        s = self.s
        ea, er, epi, edi = s["eps_abs"], s["eps_rel"], s["eps_prim_inf"], s["eps_dual_inf"]
        if f["pri_res"] > OSQP_INFTY or f["dua_res"] > OSQP_INFTY:
            return "non_convex"
        if approximate:
            ea, er, epi, edi = 10 * ea, 10 * er, 10 * epi, 10 * edi
        prim_ok = dual_ok = prim_inf = dual_inf = False
        self.checks.append((f["pri_res"], self._pri_tol(f, z, ea, er), f["dua_res"], self._dua_tol(f, ea, er)))
        if self.m == 0:
            prim_ok = True
        elif f["pri_res"] < self._pri_tol(f, z, ea, er):
            prim_ok = True
        elif s["infeasibility_checks"]:
            prim_inf = self._primal_infeasible(dy, epi)
        if f["dua_res"] < self._dua_tol(f, ea, er):
            dual_ok = True
        elif s["infeasibility_checks"]:
            dual_inf = self._dual_infeasible(dx, edi)
        if s["check_dualgap"] and prim_ok and dual_ok:
            gtol = ea + er * max(abs(t) for t in f["gap_terms"])
            self.checks[-1] = self.checks[-1] + (abs(f["gap"]), gtol)
            dual_ok = abs(f["gap"]) < gtol
        if prim_ok and dual_ok:
            return "solved_inaccurate" if approximate else "solved"
        if prim_inf:
            return "primal_infeasible"
        if dual_inf:
            return "dual_infeasible"
        return None

    def _rho_estimate(self, f):
        pri = np.abs(f["rp"]).max(initial=0.0)
        dua = np.abs(f["rd"]).max(initial=0.0)
        pn = max(np.abs(self.z).max(initial=0.0), np.abs(f["Ax"]).max(initial=0.0))
        pri = pri / (pn + OSQP_DIVISION_TOL)
        dn = max(np.abs(self.q).max(initial=0.0), np.abs(f["Aty"]).max(initial=0.0), np.abs(f["Px"]).max(initial=0.0))
        dua = dua / (dn + OSQP_DIVISION_TOL)
        r = self.rho * np.sqrt(pri / (dua + OSQP_DIVISION_TOL))
        return min(max(r, RHO_MIN), RHO_MAX)

    # ---- osqp_solve ----
    def solve(self):
        s = self.s
        if not s["warm_start"]:
            self.x[:], self.z[:], self.y[:] = 0.0, 0.0, 0.0
        if self._lu is None:
            self._factor()
        n, alpha, sigma = self.n, s["alpha"], s["sigma"]
        x, z, y = self.x, self.z, self.y
        status, f, it, can_check, rho_updates = None, None, 0, False, 0
        dx = np.zeros(n)
        dy = np.zeros(self.m)
        self.checks = []
        self.rho_estimates = []
        for it in range(1, s["max_iter"] + 1):
            xp, zp = x, z
            rhs = np.concatenate([sigma * xp - self.q, zp - self.rho_inv * y])
            sol = self._lu.solve(rhs)
            xt = sol[:n]
            zt = rhs[n:] + self.rho_inv * sol[n:]
            x = alpha * xt + (1.0 - alpha) * xp
            dx = x - xp
            zr = alpha * zt + (1.0 - alpha) * zp
            z = np.minimum(np.maximum(zr + self.rho_inv * y, self.l), self.u)
            dy = self.rho_vec * (zr - z)
            y = y + dy
            can_check = bool(s["check_termination"]) and it % s["check_termination"] == 0
            if can_check:
                f = self._info(x, z, y)
                self.z = z
                status = self._check(f, z, dx, dy)
                if status:
                    break
            if s["adaptive_rho"] and s["adaptive_rho_interval"] and it % s["adaptive_rho_interval"] == 0:
                if not can_check:
                    f = self._info(x, z, y)
                self.z = z
                rn = self._rho_estimate(f)
                self.rho_estimates.append((it, rn / self.rho))
                if rn > self.rho * s["adaptive_rho_tolerance"] or rn < self.rho / s["adaptive_rho_tolerance"]:
                    self.rho = rn
                    self._set_rho_vec()
                    self._factor()
                    rho_updates += 1
        if not can_check:
            f = self._info(x, z, y)
            status = self._check(f, z, dx, dy)
            it = it  # OSQP records iter - 1 here; the iterate count is what matters below
        if status is None:
            status = self._check(f, z, dx, dy, approximate=True) or "max_iter_reached"
        self.x, self.z, self.y = x, z, y
        self.info = dict(iter=it, status=status, pri_res=f["pri_res"], dua_res=f["dua_res"],
                         rho=self.rho, rho_updates=rho_updates)
        self.history.append((it, self.rho, rho_updates, list(self.checks), list(self.rho_estimates), status))
        if status in ("primal_infeasible", "dual_infeasible", "non_convex"):
            self.x[:], self.z[:], self.y[:] = 0.0, 0.0, 0.0
            return np.full(n, np.nan), np.full(self.m, np.nan)
        return self.D * x, self.cinv * (self.E * y)
