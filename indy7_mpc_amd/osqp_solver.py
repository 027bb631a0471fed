"""Drop-in for reference ``OSQPSolver`` (src/osqp_solver.py:6-155).

Same constructor, attributes and methods.  The numbers come from the GPU:
  * ``setup_and_solve_qp`` linearises on the device (k_linearize) and, by default
    (``qp_mode="admm"``), runs OSQP's own algorithm on it (k_admm_scale, k_admm_factor,
    k_admm_iter; i7m_admm.h) from a warm-started per-problem OSQP state, as the reference's
    ``self.osqp`` object does (:38-40, 140-143): the trajectories are the reference's own
    (oracle/osqp_admm.py pins them against the notebook's printed closed loop).
    ``qp_mode="direct"`` instead solves each QP EXACTLY with the block-tridiagonal Riccati kernel
    (k_riccati): the optimum OSQP (eps 1e-3) only approximates, so its trajectories differ from
    the reference's by OSQP's own tolerance — median 5e-5, over 1e-4 on ~30 % of config-3
    problems, up to ~0.2 (tests/test_admm_oracle.py pins that distribution).
  * ``Pdata/Adata/l/g`` (the CSC value arrays the reference fills, :95-135) are assembled on
    the host from the device linearisation, in the reference's exact value order.  The solve
    itself does not need them, so after ``setup_and_solve_qp`` they are filled lazily: the call
    records its linearisation point and the first read of any of the four arrays assembles them
    (one device linearisation of that point, bit-identical to the solve's), as the reference
    leaves them filled as a side effect of :137-143.  ``update_constraint_matrix`` /
    ``update_cost_matrix`` fill them at once, like the reference's.
  * ``eepos`` / ``d_eepos`` are device FK / Jacobian queries.
Extra (not in the reference): ``max_batch`` / ``device_id`` kwargs size the device buffers
for the batched entry point ``SQP_OSQP.sqp_batch``.
"""
from __future__ import annotations

import numpy as np
from scipy.sparse import bmat, csc_matrix, triu

from . import _lib


# i7m_get_admm_status values -> OSQP's (status, status_val)
ADMM_STATUS = {1: ("solved", 1), 2: ("solved inaccurate", 2), 0: ("maximum iterations reached", -2)}


class QPSolution:
    """What ``osqp.OSQP().solve()`` returns: ``.x`` (the only field the reference reads,
    src/osqp_solver.py:143, src/osqp_sqp.py:80), ``.y`` and ``.info.status`` / ``.info.iter``.
    ADMM mode: OSQP's status string ("solved"; "solved inaccurate" or "maximum iterations
    reached" when the termination test never passed within max_iter), its iteration count and the
    unscaled dual y = E y_s / c.  Direct mode: the exact KKT solve ("solved", 0 iterations, y None)."""

    def __init__(self, x, status="solved", iters=0, y=None):
        self.x = x
        self.y = y
        val = {s: v for s, v in ADMM_STATUS.values()}[status]
        self.info = type("info", (), {"status": status, "iter": iters, "status_val": val})()

    @classmethod
    def from_admm(cls, x, code, iters, y):
        """From i7m_get_admm_status's code; -1 (no QP ran) is an error, not "solved"."""
        code = int(code)
        if code not in ADMM_STATUS:
            raise RuntimeError(f"no OSQP result for this QP (status code {code})")
        return cls(x, status=ADMM_STATUS[code][0], iters=int(iters), y=y)


class OSQPSolver:
    def __init__(self, model, dt=0.01, N=32, dQ_cost=0.01, R_cost=1e-5, QN_cost=100, regularize=True, eps=1,
                 max_batch=1, device_id=0, box_constraints=False, box_mask=_lib.BOX_Q | _lib.BOX_V | _lib.BOX_U,
                 box_max_iters=30, box_tol=1e-8, qp_mode=None, admm=None):
        """Reference signature (src/osqp_solver.py:7) plus: max_batch / device_id (device
        buffers); the config-4 extension ``box_constraints``: box rows on
        q, v, u from the model's URDF limits, solved by the interior-point mode (I7M_QP_BOX);
        ``qp_mode``: "admm" (the default: OSQP's iteration with its carried state, i.e. the
        reference's numbers; ``admm`` overrides OSQP settings, keys of _lib.ADMM_DEFAULTS) or
        "direct" (the exact KKT solve, the optimum OSQP approximates).  With box_constraints the
        QP is the interior-point mode's (qp_mode must then be left unset or "direct")."""
        if qp_mode is None:
            qp_mode = "direct" if box_constraints else "admm"
        if qp_mode not in ("direct", "admm"):
            raise ValueError("qp_mode must be 'direct' or 'admm'")
        if qp_mode == "admm" and box_constraints:
            raise ValueError("box_constraints use the interior-point mode; qp_mode='admm' is the reference's equality QP")
        self.model = model
        self.data = model.createData()
        self.N = N
        self.dt = dt
        self.nq = model.nq
        self.nv = model.nv
        self.nx = self.nq + self.nv
        self.nu = len(model.joints) - 1
        self.nxu = self.nx + self.nu
        self.traj_len = (self.nx + self.nu) * self.N - self.nu
        self.dQ_cost = dQ_cost
        self.R_cost = R_cost
        self.QN_cost = QN_cost
        self.regularize = regularize
        self.eps = eps
        self.A = self.initialize_A()
        self.P = self.initialize_P()
        self._l = np.zeros(self.N * self.nx)
        self._g = np.zeros(self.traj_len)
        self._Pdata = np.zeros(self.P.nnz)
        self._Adata = np.zeros(self.A.nnz)
        self._pending_A = self._pending_P = None  # linearisation point of the last setup_and_solve_qp
        self.A_k = np.vstack([-1.0 * np.eye(self.nx),
                              np.vstack([np.hstack([np.eye(self.nq), self.dt * np.eye(self.nq)]),
                                         np.ones((self.nq, 2 * self.nq))])])
        self.B_k = np.zeros((self.nx, self.nq))
        self.cx_k = np.zeros(self.nx)
        mode = _lib.QP_ADMM if qp_mode == "admm" else (_lib.QP_BOX if box_constraints else _lib.QP_DIRECT)
        # the QP-mode keyword arguments every handle of this solver is created with
        self.box = dict(qp_mode=mode, box_mask=box_mask, box_max_iters=box_max_iters, box_tol=box_tol, admm=admm)
        self.handle = _lib.Handle(model, N=N, dt=dt, dQ_cost=dQ_cost, R_cost=R_cost, QN_cost=QN_cost,
                                  regularize=regularize, eps=eps, max_batch=max_batch, device_id=device_id, **self.box)

    # ---- sparsity templates (src/osqp_solver.py:48-68) -----------------------------------
    def initialize_P(self):
        block = np.eye(self.nxu)
        block[: self.nq, : self.nq] = np.ones((self.nq, self.nq))
        bd = np.kron(np.eye(self.N), block)[: -self.nu, : -self.nu]
        return csc_matrix(triu(bd), shape=(self.traj_len, self.traj_len))

    def initialize_A(self):
        nx, nu, N = self.nx, self.nu, self.N
        blocks = [[np.ones((nx, nx))] + [None] * (2 * N)]
        for i in range(N - 1):
            row = [None] * (2 * i) + [np.ones((nx, nx)), 2 * np.ones((nx, nu)), -1 * np.ones((nx, nx))]
            row += [None] * (2 * N + 1 - len(row))
            blocks.append(row)
        return bmat(blocks, format="csc")

    # ---- linearisation (src/osqp_solver.py:70-135), values from the device --------------
    def compute_dynamics_jacobians(self, q, v, u):
        dq, dv, Minv, a = self.handle.aba_derivatives(q, v, u)
        nx, nq = self.nx, self.nq
        self.A_k[nx + nq:, :nq] = dq[0] * self.dt
        self.A_k[nx + nq:, nq:2 * nq] = dv[0] * self.dt + np.eye(self.nv)
        self.B_k[nq:, :] = Minv[0] * self.dt
        xnext = np.hstack([q + v * self.dt, v + a[0] * self.dt])
        self.cx_k = xnext - self.A_k[nx:] @ np.hstack([q, v]) - self.B_k @ u

    def _linearisation(self, xu, eepos_g):
        lin, cost = self.handle.linearize(xu, eepos_g)
        return lin[0], cost[0]

    def update_constraint_matrix(self, xu, xs, _lin=None):
        lin = self._linearisation(xu, np.zeros(3 * self.N))[0] if _lin is None else _lin
        self._pending_A = None
        self._Adata[:], self._l[:] = assemble_A(lin, np.asarray(xu, float), np.asarray(xs, float), self.dt, self.N)

    def update_cost_matrix(self, XU, eepos_g, _cost=None):
        cost = self._linearisation(XU, eepos_g)[1] if _cost is None else _cost
        self._pending_P = None
        self._Pdata[:], self._g[:] = assemble_P(cost, np.asarray(XU, float), self.N)

    def setup_and_solve_qp(self, xu, xs, eepos_g):
        """reference :137-143 — linearise at xu, solve the QP; returns an object with ``.x``.
        Pdata / Adata / l / g describe this QP afterwards (assembled on first read)."""
        xu, xs, eepos_g = (np.array(a, dtype=float) for a in (xu, xs, eepos_g))
        x = self.handle.qp(xu, xs, eepos_g)[0]
        if self.box["qp_mode"] == _lib.QP_ADMM:
            its, _, solved = self.handle.admm_stats(1, with_status=True)
            y = self.handle.admm_dual(1)[0]
            sol = QPSolution.from_admm(x, solved[0, 0], its[0, 0], y)
        else:
            sol = QPSolution(x)
        self._pending_A = (xu, xs)
        self._pending_P = (xu, eepos_g)
        return sol

    def _flush(self):
        """Assemble the arrays of the last setup_and_solve_qp that have not been read yet."""
        pa, pp = self._pending_A, self._pending_P
        if pa is None and pp is None:
            return
        xu = (pa or pp)[0]
        goals = pp[1] if pp is not None else np.zeros(3 * self.N)
        lin, cost = self._linearisation(xu, goals)
        if pa is not None:
            self.update_constraint_matrix(xu, pa[1], _lin=lin)
        if pp is not None:
            self.update_cost_matrix(xu, goals, _cost=cost)

    @property
    def Pdata(self):
        self._flush()
        return self._Pdata

    @Pdata.setter
    def Pdata(self, value):
        self._flush()
        self._Pdata = np.asarray(value, dtype=float)

    @property
    def Adata(self):
        self._flush()
        return self._Adata

    @Adata.setter
    def Adata(self, value):
        self._flush()
        self._Adata = np.asarray(value, dtype=float)

    @property
    def l(self):  # noqa: E743 - the reference's attribute name
        self._flush()
        return self._l

    @l.setter
    def l(self, value):
        self._flush()
        self._l = np.asarray(value, dtype=float)

    @property
    def g(self):
        self._flush()
        return self._g

    @g.setter
    def g(self, value):
        self._flush()
        self._g = np.asarray(value, dtype=float)

    def assemble(self, xu, xs, eepos_g):
        """Fill Pdata/Adata/l/g exactly as the reference's update_* methods do."""
        lin, cost = self._linearisation(xu, eepos_g)
        self.update_constraint_matrix(xu, xs, _lin=lin)
        self.update_cost_matrix(xu, eepos_g, _cost=cost)

    # ---- end effector (src/osqp_solver.py:146-155) -------------------------------------
    def eepos(self, q):
        return self.handle.eepos(q)[0]

    def d_eepos(self, q):
        p, J = self.handle.eepos(q, jacobian=True)
        return p[0], J[0]


def assemble_A(lin, xu, xs, dt, N):
    """CSC values of A and l in the order of src/osqp_solver.py:83-101, from the device
    linearisation lin (N-1, 114) = Aq | Av | Bu | a per knot."""
    nx = 12
    Adata = np.empty(360 * (N - 1) + 144)
    l = np.empty(N * nx)
    l[:nx] = -xs
    Ak = np.zeros((24, 12))
    Ak[:12] = -np.eye(12)
    Ak[12:18, :6] = np.eye(6)
    Ak[12:18, 6:] = dt * np.eye(6)
    Bk = np.zeros((12, 6))
    ind = 0
    for k in range(N - 1):
        Aq = lin[k, 0:36].reshape(6, 6)
        Av = lin[k, 36:72].reshape(6, 6)
        Bu = lin[k, 72:108].reshape(6, 6)
        a = lin[k, 108:114]
        Ak[18:, :6] = Aq
        Ak[18:, 6:] = Av
        Bk[6:] = Bu
        Adata[ind:ind + 288] = Ak.T.reshape(-1)
        ind += 288
        Adata[ind:ind + 72] = Bk.T.reshape(-1)
        ind += 72
        x = xu[18 * k:18 * k + 12]
        u = xu[18 * k + 12:18 * k + 18]
        xnext = np.hstack([x[:6] + x[6:] * dt, x[6:] + a * dt])
        c = xnext - Ak[12:] @ x - Bk @ u
        l[(k + 1) * nx:(k + 2) * nx] = -c
    Adata[ind:] = -np.eye(nx).reshape(-1)
    return Adata, l


def assemble_P(cost, xu, N):
    """CSC values of P (upper) and g in the order of src/osqp_solver.py:103-135, from the device
    cost linearisation cost (N, 10) = j(6) | Qm | dQm | Rm | |e|."""
    Pdata = np.empty(27 * N + 6 * (N - 1))
    g = np.empty(18 * N - 6)
    tri = np.tril_indices(6)
    ind = 0
    for k in range(N):
        j = cost[k, :6]
        Qm, dQm, Rm = cost[k, 6], cost[k, 7], cost[k, 8]
        g0 = 18 * k
        g[g0:g0 + 6] = Qm * j
        g[g0 + 6:g0 + 12] = dQm * xu[g0 + 6:g0 + 12]
        ph = np.outer(j, j)
        Pdata[ind:ind + 21] = Qm * ph[tri]
        ind += 21
        Pdata[ind:ind + 6] = dQm
        ind += 6
        if k < N - 1:
            Pdata[ind:ind + 6] = Rm
            ind += 6
            g[g0 + 12:g0 + 18] = Rm * xu[g0 + 12:g0 + 18]
    return Pdata, g
