"""ORACLE (test infrastructure only) — restatement of the reference's SQP-MPC hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

Restates, function by function:
  * ``OSQPSolver``          reference src/osqp_solver.py:6-155
        - ``initialize_P``    :48-52   CSC upper-triangular template, nnz = 27N + 6(N-1)
        - ``initialize_A``    :54-68   block-bidiagonal CSC template, nnz = 360(N-1) + 144
        - ``compute_dynamics_jacobians`` :70-81
        - ``update_constraint_matrix``   :83-101  (Adata value order, l)
        - ``update_cost_matrix``         :103-135 (Pdata value order, g)
        - ``setup_and_solve_qp``         :137-143
        - ``eepos`` / ``d_eepos``        :146-155
  * ``SQP_OSQP``            reference src/osqp_sqp.py:4-96 (eepos_cost :13-30, integrator_err
                            :32-47, linesearch :49-74, sqp :76-93)

The QP solve: the reference calls OSQP (third-party, un-vendored, unpinned; default
eps_abs = eps_rel = 1e-3).  The QP is equality-constrained (l == u, src/osqp_solver.py:142)
and strictly convex on null(A), so it has one solution, which OSQP approximates.  The oracle
returns that solution EXACTLY: a sparse LU (scipy ``splu``) of the full KKT system
[[P, A^T], [A, 0]] [x; y] = [-g; l].  This is the "tight-tolerance oracle" SURVEY.md §7/§8c
prescribes.  ``solve_qp_admm`` restates OSQP's ADMM iteration (rho, sigma, alpha, equality
rows at 1e3*rho) for the ADMM-mode tests.

Pure-Python loops over knots mirror the reference's structure; sizes are small.
"""
from __future__ import annotations

import numpy as np
from scipy.sparse import bmat, csc_matrix, triu, diags
from scipy.sparse.linalg import splu

from . import rbd


class QPResult:
    def __init__(self, x, y=None, iters=0):
        self.x = x
        self.y = y
        self.info = type("info", (), {"iter": iters, "status": "solved"})()


class OSQPSolverRef:
    """Restates OSQPSolver (src/osqp_solver.py:6-155); QP solved exactly."""

    def __init__(self, dt=0.01, N=32, dQ_cost=0.01, R_cost=1e-5, QN_cost=100, regularize=True, eps=1,
                 qp="exact", P=None, box_mask=7, box_tol=1e-8, box_max_iters=30, fext6=None, fext_frame="local",
                 osqp_settings=None, osqp_box=0):
        self.P_ = P or rbd.params()
        # external wrench on joint 6 in every dynamics evaluation (batch_sqp's
        # set_external_wrench_batch; frame "world": converted per configuration, rbd.fext_list)
        self.fext6 = None if fext6 is None else np.asarray(fext6, float)
        self.fext_frame = fext_frame
        self.N, self.dt = N, dt
        self.nq = self.nv = rbd.NJ
        self.nx = self.nq + self.nv
        self.nu = rbd.NJ
        self.nxu = self.nx + self.nu
        self.traj_len = (self.nx + self.nu) * self.N - self.nu
        self.dQ_cost, self.R_cost, self.QN_cost = dQ_cost, R_cost, QN_cost
        self.regularize, self.eps = regularize, eps
        self.A = self.initialize_A()
        self.l = np.zeros(self.N * self.nx)
        self.P = self.initialize_P()
        self.g = np.zeros(self.traj_len)
        self.Pdata = np.zeros(self.P.nnz)
        self.Adata = np.zeros(self.A.nnz)
        self.qp = qp
        # config 4 box mode (oracle/box_ipm.py)
        self.box_mask, self.box_tol, self.box_max_iters = box_mask, box_tol, box_max_iters
        self.last_ipm = None
        nq = self.nq
        self.A_k = np.vstack([-1.0 * np.eye(self.nx),
                              np.vstack([np.hstack([np.eye(nq), self.dt * np.eye(nq)]), np.ones((nq, 2 * nq))])])
        self.B_k = np.zeros((self.nx, self.nq))
        self.cx_k = np.zeros(self.nx)
        if qp == "osqp":
            # src/osqp_solver.py:38-40: one OSQP workspace, set up on the templates.  osqp_box
            # (config 4 in ADMM mode, no reference counterpart): box rows l_b <= x_b <= u_b appended
            # to A for the bounded entries of box_ipm.box_bounds(mask = osqp_box), values 1
            from .osqp_admm import OSQP
            self.osqp = OSQP()
            A, l, u = self.A, self.l, self.l
            self.osqp_box = osqp_box
            if osqp_box:
                from scipy.sparse import vstack, identity
                from . import box_ipm
                lo, hi, bm = box_ipm.box_bounds(self.P_, N, osqp_box)
                self._bidx = np.flatnonzero(bm)
                self._blo, self._bhi = lo[bm], hi[bm]
                # where A's values and the box rows' land in the stacked matrix's CSC value order
                At = A.copy()
                At.data = np.arange(1, At.nnz + 1, dtype=float)
                Ib = identity(self.traj_len, format="csc")[self._bidx]
                Ib.data = -np.arange(1, Ib.nnz + 1, dtype=float)
                code = vstack([At, Ib], format="csc")
                code.sort_indices()
                self._pos_a = np.flatnonzero(code.data > 0)[np.argsort(code.data[code.data > 0])]
                self._pos_b = np.flatnonzero(code.data < 0)
                self._nnz_full = code.nnz
                A = vstack([A, identity(self.traj_len, format="csc")[self._bidx]], format="csc")
                l = np.concatenate([self.l, self._blo])
                u = np.concatenate([self.l, self._bhi])
            self.osqp.setup(P=self.P, q=self.g, A=A, l=l, u=u, **(osqp_settings or {}))

    # src/osqp_solver.py:48-52
    def initialize_P(self):
        block = np.eye(self.nxu)
        block[: self.nq, : self.nq] = np.ones((self.nq, self.nq))
        bd = np.kron(np.eye(self.N), block)[: -self.nu, : -self.nu]
        return csc_matrix(triu(bd), shape=(self.traj_len, self.traj_len))

    # src/osqp_solver.py:54-68
    def initialize_A(self):
        nx, nu, N = self.nx, self.nu, self.N
        blocks = [[np.ones((nx, nx))] + [None] * (2 * N)]
        for i in range(N - 1):
            row = [None] * (2 * i)
            row += [np.ones((nx, nx)), 2 * np.ones((nx, nu)), -1 * np.ones((nx, nx))]
            row += [None] * (2 * N + 1 - len(row))
            blocks.append(row)
        return bmat(blocks, format="csc")

    # src/osqp_solver.py:70-81
    def compute_dynamics_jacobians(self, q, v, u):
        d_dq, d_dv, d_du, a = rbd.aba_derivatives(q, v, u, self.P_, self.fext6, self.fext_frame)
        nx, nq = self.nx, self.nq
        self.A_k[nx + nq:, :nq] = d_dq * self.dt
        self.A_k[nx + nq:, nq:2 * nq] = d_dv * self.dt + np.eye(self.nv)
        self.B_k[nq:, :] = d_du * self.dt
        qnext = rbd.integrate(q, v * self.dt)
        vnext = v + a * self.dt
        xnext = np.hstack([qnext, vnext])
        xcur = np.hstack([q, v])
        self.cx_k = xnext - self.A_k[nx:] @ xcur - self.B_k @ u

    # src/osqp_solver.py:83-101
    def update_constraint_matrix(self, xu, xs):
        nx, nq, nu = self.nx, self.nq, self.nu
        self.l[:nx] = -1 * xs
        Aind = 0
        s = nx + nu
        for k in range(self.N - 1):
            qcur = xu[k * s: k * s + nq]
            vcur = xu[k * s + nq: k * s + nx]
            ucur = xu[k * s + nx: (k + 1) * s]
            self.compute_dynamics_jacobians(qcur, vcur, ucur)
            self.Adata[Aind: Aind + nx * nx * 2] = self.A_k.T.reshape(-1)
            Aind += nx * nx * 2
            self.Adata[Aind: Aind + nx * nu] = self.B_k.T.reshape(-1)
            Aind += nx * nu
            self.l[(k + 1) * nx: (k + 2) * nx] = -1.0 * self.cx_k
        self.Adata[Aind:] = -1.0 * np.eye(nx).reshape(-1)

    # src/osqp_solver.py:103-135
    def update_cost_matrix(self, XU, eepos_g):
        nx, nq, nu, N = self.nx, self.nq, self.nu, self.N
        Pind = 0
        for k in range(N):
            if k < N - 1:
                XU_k = XU[k * (nx + nu): (k + 1) * (nx + nu)]
            else:
                XU_k = XU[k * (nx + nu): (k + 1) * (nx + nu) - nu]
            eepos, deepos = self.d_eepos(XU_k[:nq])
            eepos_err = np.array(eepos.T) - eepos_g[k * 3: (k + 1) * 3]
            nrm = abs(np.linalg.norm(eepos_err))
            dQm = self.dQ_cost if not self.regularize else self.dQ_cost * (1 / (nrm + self.eps))
            Rm = self.R_cost if not self.regularize else self.R_cost * (1 / (nrm + self.eps))
            Qm = self.QN_cost if k == N - 1 else 1
            joint_err = eepos_err @ deepos
            g0 = k * (nx + nu)
            self.g[g0: g0 + nx] = np.concatenate([Qm * joint_err, dQm * XU_k[nq:nx]])
            ph = np.outer(joint_err, joint_err)
            pos = Qm * ph[np.tril_indices_from(ph)]
            self.Pdata[Pind: Pind + len(pos)] = pos
            Pind += len(pos)
            self.Pdata[Pind: Pind + self.nv] = dQm
            Pind += self.nv
            if k < N - 1:
                self.Pdata[Pind: Pind + nu] = Rm
                Pind += nu
                self.g[g0 + nx: g0 + nx + nu] = Rm * XU_k[nx: nx + nu]

    def matrices(self):
        """Current (P upper CSC, A CSC) with the value arrays written in."""
        P = self.P.copy()
        P.data = self.Pdata.copy()
        A = self.A.copy()
        A.data = self.Adata.copy()
        return P, A

    def solve_qp_exact(self):
        P, A = self.matrices()
        Pf = P + P.T - diags(P.diagonal())
        n, m = self.traj_len, self.N * self.nx
        K = bmat([[Pf, A.T], [A, None]], format="csc")
        rhs = np.concatenate([-self.g, self.l])
        z = splu(K).solve(rhs)
        return QPResult(z[:n], z[n:])

    def solve_qp_admm(self, rho=0.1, sigma=1e-6, alpha=1.6, iters=4000, eps_abs=1e-9, eps_rel=1e-9,
                      x0=None, y0=None):
        """OSQP's ADMM iteration (unscaled; l == u rows use rho_eq = 1e3 rho)."""
        P, A = self.matrices()
        Pf = (P + P.T - diags(P.diagonal())).tocsc()
        n, m = self.traj_len, self.N * self.nx
        rho_v = np.full(m, 1e3 * rho)  # every row is an equality row
        K = bmat([[Pf + sigma * diags(np.ones(n)), A.T], [A, diags(-1.0 / rho_v)]], format="csc")
        lu = splu(K)
        x = np.zeros(n) if x0 is None else x0.copy()
        y = np.zeros(m) if y0 is None else y0.copy()
        z = A @ x
        it = 0
        for it in range(1, iters + 1):
            rhs = np.concatenate([sigma * x - self.g, z - y / rho_v])
            sol = lu.solve(rhs)
            xt, nu_ = sol[:n], sol[n:]
            zt = z + (nu_ - y) / rho_v
            x = alpha * xt + (1 - alpha) * x
            zr = alpha * zt + (1 - alpha) * z
            znew = np.clip(zr + y / rho_v, self.l, self.l)
            y = y + rho_v * (zr - znew)
            z = znew
            rp = np.abs(A @ x - z).max()
            rd = np.abs(Pf @ x + self.g + A.T @ y).max()
            if rp < eps_abs + eps_rel * max(np.abs(A @ x).max(), np.abs(z).max()) and \
               rd < eps_abs + eps_rel * max(np.abs(Pf @ x).max(), np.abs(A.T @ y).max(), np.abs(self.g).max()):
                break
        return QPResult(x, y, it)

    # src/osqp_solver.py:137-143
    def setup_and_solve_qp(self, xu, xs, eepos_g):
        self.update_constraint_matrix(xu, xs)
        self.update_cost_matrix(xu, eepos_g)
        if self.qp == "osqp":
            # src/osqp_solver.py:140-143
            self.osqp.update(Px=self.Pdata)
            if self.osqp_box:
                ax = np.empty(self._nnz_full)
                ax[self._pos_a] = self.Adata
                ax[self._pos_b] = 1.0
                self.osqp.update(Ax=ax)
                self.osqp.update(q=self.g, l=np.concatenate([self.l, self._blo]), u=np.concatenate([self.l, self._bhi]))
            else:
                self.osqp.update(Ax=self.Adata)
                self.osqp.update(q=self.g, l=self.l, u=self.l)
            x, y = self.osqp.solve()
            return QPResult(x, y, self.osqp.info["iter"])
        if self.qp == "admm":
            return self.solve_qp_admm()
        if self.qp == "box":
            return self.solve_qp_box()
        return self.solve_qp_exact()

    def solve_qp_box(self):
        """Config 4: box rows on q, v, u (oracle/box_ipm.py), from the equality-only optimum."""
        from . import box_ipm
        x_eq = self.solve_qp_exact().x
        P, A = self.matrices()
        Pf = (P + P.T - diags(P.diagonal())).tocsc()
        lo, hi, bm = box_ipm.box_bounds(self.P_, self.N, self.box_mask)
        r = box_ipm.ipm_box(Pf, self.g, A, self.l, x_eq, lo, hi, bm, tol=self.box_tol, max_iters=self.box_max_iters)
        self.last_ipm = r
        return QPResult(r.x, None, r.iters)

    # src/osqp_solver.py:146-155
    def eepos(self, q):
        return rbd.eepos(q, self.P_)

    def d_eepos(self, q):
        return rbd.d_eepos(q, self.P_)


class SQPRef:
    """Restates SQP_OSQP (src/osqp_sqp.py:4-96)."""

    ALPHAS = np.array([1.0, 0.5, 0.25, 0.125, 0.0625, 0.03125, 0.015625, 0.0078125])

    def __init__(self, solver: OSQPSolverRef, stats=None):
        self.solver = solver
        self.stats = stats or {
            "qp_iters": {"values": [], "unit": "", "multiplier": 1},
            "linesearch_alphas": {"values": [], "unit": "", "multiplier": 1},
            "sqp_stepsizes": {"values": [], "unit": "", "multiplier": 1},
        }

    # src/osqp_sqp.py:13-30
    def eepos_cost(self, eepos_goals, XU):
        s = self.solver
        qcost = vcost = ucost = 0
        for k in range(s.N):
            if k < s.N - 1:
                XU_k = XU[k * (s.nx + s.nu): (k + 1) * (s.nx + s.nu)]
                Qm = 1
            else:
                XU_k = XU[k * (s.nx + s.nu): (k + 1) * (s.nx + s.nu) - s.nu]
                Qm = s.QN_cost
            e = s.eepos(XU_k[: s.nq]) - eepos_goals[k * 3: (k + 1) * 3]
            qcost += Qm * np.dot(e, e)
            vk = XU_k[s.nq: s.nx]
            vcost += s.dQ_cost * np.dot(vk, vk)
            if k < s.N - 1:
                uk = XU_k[s.nx: s.nx + s.nu]
                ucost += s.R_cost * np.dot(uk, uk)
        return qcost, vcost, ucost

    # src/osqp_sqp.py:32-47
    def integrator_err(self, XU):
        s = self.solver
        err = 0
        st = s.nx + s.nu
        for k in range(s.N - 1):
            q = XU[k * st: k * st + s.nq]
            v = XU[k * st + s.nq: k * st + s.nx]
            u = XU[k * st + s.nx: (k + 1) * st]
            a = rbd.aba(q, v, u, s.P_, rbd.fext_list(q, s.fext6, s.fext_frame, s.P_))
            qn = rbd.integrate(q, v * s.dt)
            vn = v + a * s.dt
            err += np.linalg.norm(qn - XU[(k + 1) * st: (k + 1) * st + s.nq]) + \
                np.linalg.norm(vn - XU[(k + 1) * st + s.nq: (k + 1) * st + s.nx])
        return err

    def merit_terms(self, XU, XU_ref, goals):
        q, v, u = self.eepos_cost(goals, XU)
        cv = self.integrator_err(XU) + np.linalg.norm(XU[: self.solver.nx] - XU_ref[: self.solver.nx])
        return q + v + u + 10.0 * cv

    # src/osqp_sqp.py:49-74
    def linesearch(self, XU, XU_fullstep, eepos_goals, record=None):
        basemerit = self.merit_terms(XU, XU, eepos_goals)
        diff = XU_fullstep - XU
        merits = []
        alpha_ok = 0.0
        for alpha in self.ALPHAS:
            XU_new = XU + alpha * diff
            m = self.merit_terms(XU_new, XU, eepos_goals)
            merits.append(m)
            if m <= basemerit:
                alpha_ok = alpha
                break
        if record is not None:
            record.append(dict(base=basemerit, merits=merits))
        self.stats["linesearch_alphas"]["values"].append(alpha_ok)
        return alpha_ok

    # src/osqp_sqp.py:76-93
    def sqp(self, xcur, eepos_goals, XU, record=None):
        qp = 0
        for qp in range(2):
            sol = self.solver.setup_and_solve_qp(XU, xcur, eepos_goals)
            if record is not None:
                record.append(dict(sol=sol.x.copy()))
            alpha = self.linesearch(XU, sol.x, eepos_goals, record)
            if alpha == 0.0:
                continue
            step = alpha * (sol.x - XU)
            XU = XU + step
            stepsize = np.linalg.norm(step)
            self.stats["sqp_stepsizes"]["values"].append(stepsize)
            if stepsize < 1e-3:
                break
        self.stats["qp_iters"]["values"].append(qp + 1)
        return XU

    def get_stats(self):
        return self.stats


def synthetic_batch(B, N, seed, P=None):
    """Bench/test inputs: q ~ U(+-lim/2), v ~ U(-.5,.5), goal = FK(q_goal)
    tiled N times, XU = 0 with XU[:12] = xcur (src/gato_mpc_batch.py:97-99)."""
    P = P or rbd.params()
    rng = np.random.default_rng(seed)
    lo, hi = 0.5 * P.q_lower, 0.5 * P.q_upper
    q0 = rng.uniform(lo, hi, size=(B, 6))
    v0 = rng.uniform(-0.5, 0.5, size=(B, 6))
    qg = rng.uniform(lo, hi, size=(B, 6))
    xcur = np.hstack([q0, v0])
    goals = np.stack([np.tile(rbd.eepos(qg[b], P), N) for b in range(B)])
    T = 18 * N - 6
    XU = np.zeros((B, T))
    XU[:, :12] = xcur
    return xcur, goals, XU
