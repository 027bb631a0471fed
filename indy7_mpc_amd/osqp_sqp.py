"""Drop-in for reference ``SQP_OSQP`` (src/osqp_sqp.py:4-96).

``sqp`` runs the whole <=2-iteration SQP (linearise -> exact QP -> parallel backtracking line
search -> step) on the GPU in one library call and fills the same stats keys.
``sqp_batch`` is the batched entry point the reference lacks on this path: B independent
problems laid out as (B, traj_len) like src/gato_mpc_batch.py:41,97-99.
"""
from __future__ import annotations

import numpy as np

from . import _lib


class SQP_OSQP:
    def __init__(self, solver, stats=None):
        self.solver = solver
        self.stats = stats or {
            "qp_iters": {"values": [], "unit": "", "multiplier": 1},
            "linesearch_alphas": {"values": [], "unit": "", "multiplier": 1},
            "sqp_stepsizes": {"values": [], "unit": "", "multiplier": 1},
        }
        self._batch_handle = None

    # ---- merit pieces (src/osqp_sqp.py:13-47) --------------------------------------------
    def eepos_cost(self, eepos_goals, XU):
        m = self.solver.handle.merit(XU, XU, eepos_goals)[0]
        return m[0], m[1], m[2]

    def integrator_err(self, XU):
        m = self.solver.handle.merit(XU, XU, np.zeros(3 * self.solver.N))[0]
        return m[3]

    def linesearch(self, XU, XU_fullstep, eepos_goals):
        """src/osqp_sqp.py:49-74 (all alphas evaluated on the device, first accepted wins)."""
        alpha = float(self.solver.handle.linesearch(XU, XU_fullstep, eepos_goals)[0])
        self.stats["linesearch_alphas"]["values"].append(alpha)
        return alpha

    # ---- SQP (src/osqp_sqp.py:76-93) ----------------------------------------------------
    def _record(self, st):
        for s in np.atleast_1d(st):
            self.stats["linesearch_alphas"]["values"].extend(float(a) for a in s["alphas"][: s["n_alphas"]])
            self.stats["sqp_stepsizes"]["values"].extend(float(a) for a in s["stepsizes"][: s["n_steps"]])
            self.stats["qp_iters"]["values"].append(int(s["qp_iters"]))

    def sqp(self, xcur, eepos_goals, XU):
        out, st = self.solver.handle.solve(xcur, eepos_goals, XU)
        self._record(st)
        return out[0]

    def _handle_for(self, B):
        h = self.solver.handle
        if B <= h.max_batch:
            return h
        if self._batch_handle is None or self._batch_handle.max_batch < B:
            s = self.solver
            self._batch_handle = _lib.Handle(s.model, N=s.N, dt=s.dt, dQ_cost=s.dQ_cost, R_cost=s.R_cost,
                                             QN_cost=s.QN_cost, regularize=s.regularize, eps=s.eps, max_batch=B,
                                             device_id=h.cfg.device_id, **s.box)
        return self._batch_handle

    def sqp_batch(self, xcur_batch, eepos_goals_batch, XU_batch):
        """Batched ``sqp``: xcur (B,12), goals (B,3N) or (B,6N), XU (B,traj_len) -> (B,traj_len)."""
        XU_batch = np.asarray(XU_batch, dtype=float)
        h = self._handle_for(XU_batch.shape[0])
        out, st = h.solve(xcur_batch, eepos_goals_batch, XU_batch)
        self._record(st)
        return out

    def get_stats(self):
        return self.stats
