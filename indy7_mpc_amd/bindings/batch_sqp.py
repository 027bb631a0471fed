"""Drop-in for the ``bindings.batch_sqp`` module the reference's GATO controllers import
(gato_controller.py:53-68,95,106,129,132-138; src/gato_mpc_batch.py:12-29,43).

The reference binding is an external CUDA module (absent).  This one keeps its
Python surface — ``SQPSolverfloat_{1..256}`` with ``solve``, ``reset``, ``resetRho``,
``resetLambda``, ``set_external_wrench_batch`` and ``sim_forward`` — and solves the OSQP
formulation of src/osqp_solver.py (fp64) on the GPU, each QP by default (``qp_mode="admm"``)
with OSQP's own iteration from a per-problem warm-started state, as the reference's OSQP path
does (``resetRho`` / ``resetLambda`` reset OSQP's rho / duals, gato_controller.py:132-138), or
with ``qp_mode="direct"`` exactly (the optimum OSQP approximates to eps 1e-3).  N is taken
from the XU width (traj_len = 18N - 6); goals use the GATO layout (B, 6N), first 3 of every 6 used.

External wrench convention (``set_external_wrench_batch``): by default each row is what the
reference's callers put there — a WORLD-frame force [f; n] (gato_controller.py:77-81,120-129 and
src/gato_mpc_batch_sample.py:37-40 draw f and zero n), which the reference's own host code turns
into joint 6's local frame at the current configuration with ``data.oMi[6].actInv``
(src/gato_mpc_batch_sample.py:151-161,270-279).  Here every dynamics evaluation does that
conversion at its own configuration (the linearisation differentiates it too), and
``sim_forward`` converts once at the start state, like the reference's host rk4 plant.
``frame="local"`` keeps a constant wrench in joint 6's frame instead (pinocchio's f_ext as is).
"""
from __future__ import annotations

import time

import numpy as np

from .. import _lib
from ..model import default_model

_SIZES = (1, 2, 4, 8, 16, 32, 64, 128, 256)


class _SQPSolverBatch:
    batch_size = 1

    def __init__(self, model=None, device_id=0, wrench_frame="world", qp_mode="admm"):
        if wrench_frame not in ("world", "local"):
            raise ValueError("wrench_frame must be 'world' or 'local'")
        if qp_mode not in ("direct", "admm"):
            raise ValueError("qp_mode must be 'direct' or 'admm'")
        self.qp_mode = _lib.QP_ADMM if qp_mode == "admm" else _lib.QP_DIRECT
        self.model = model or default_model()
        self.device_id = device_id
        self.wrench_frame = wrench_frame
        self._h = None
        self._key = None
        self._fext = np.zeros((self.batch_size, 6))
        self._sim = _lib.Handle(self.model, N=2, max_batch=max(self.batch_size, 1), device_id=device_id)

    def _handle(self, N, dt):
        if self._key != (N, dt):
            self._h = _lib.Handle(self.model, N=N, dt=dt, max_batch=self.batch_size, device_id=self.device_id,
                                  qp_mode=self.qp_mode)
            self._key = (N, dt)
            if np.any(self._fext):
                self._h.set_external_wrench(self._fext, self.wrench_frame)
        return self._h

    def solve(self, XU_batch, dt, xcur_batch, eepos_goals_batch):
        XU = np.asarray(XU_batch, dtype=float).reshape(self.batch_size, -1)
        T = XU.shape[1]
        if (T + 6) % 18:
            raise ValueError(f"XU width {T} is not 18N-6")
        N = (T + 6) // 18
        h = self._handle(N, float(dt))
        t0 = time.perf_counter()
        out, st = h.solve(np.asarray(xcur_batch, float).reshape(self.batch_size, 12),
                          np.asarray(eepos_goals_batch, float).reshape(self.batch_size, -1), XU)
        t1 = time.perf_counter()
        iters = int(st["qp_iters"].max()) if len(st) else 0
        ls = []
        for it in range(iters):
            ls.append({"step_size": np.array([s["alphas"][it] if it < s["n_alphas"] else 0.0 for s in st])})
        if self.qp_mode == _lib.QP_ADMM:  # inner iterations per SQP iteration: OSQP's
            adm = h.admm_stats(self.batch_size)[0]
            inner = [{"pcg_iterations": np.maximum(adm[:, it], 0)} for it in range(iters)]
        else:
            inner = [{"pcg_iterations": 0} for _ in range(iters)]  # exact KKT solve, no PCG
        return {
            "xu_trajectory": out,
            "solve_time_us": (t1 - t0) * 1e6,
            "sqp_iterations": st["qp_iters"].copy(),
            "pcg_stats": inner,
            "line_search_stats": ls,
        }

    def reset(self):
        """Solver state reset (i7m_reset): ADMM mode starts every problem's OSQP state afresh;
        the exact solve keeps no warm start, so its results are unchanged; the wrench hypotheses
        are kept."""
        for h in (self._h, self._sim):
            if h is not None:
                h.reset()

    def resetRho(self):
        """Penalty reset: ADMM mode puts OSQP's rho back to its setting (the iterates stay);
        the exact solve has no penalty, so there it is i7m_reset."""
        if self.qp_mode == _lib.QP_ADMM and self._h is not None:
            self._h.admm_reset(what=_lib.ADMM_RESET_RHO)
        else:
            self.reset()

    def resetLambda(self):
        """Dual reset: ADMM mode zeroes OSQP's y; the exact solve keeps no duals, so there it is
        i7m_reset."""
        if self.qp_mode == _lib.QP_ADMM and self._h is not None:
            self._h.admm_reset(what=_lib.ADMM_RESET_DUAL)
        else:
            self.reset()

    def set_external_wrench_batch(self, f_ext_batch):
        f = np.asarray(f_ext_batch, dtype=float).reshape(self.batch_size, 6)
        self._fext = f.copy()
        if self._h is not None:
            self._h.set_external_wrench(self._fext, self.wrench_frame)

    def sim_forward(self, x, u, dt):
        """One rk4 step of x (12,) under u (6,) for every wrench hypothesis -> (B, 12)
        (gato_controller.py:109-118 compares these with the measured state)."""
        x = np.asarray(x, float).reshape(12)
        u = np.asarray(u, float).reshape(6)
        B = self.batch_size
        qo, vo = self._sim.rk4(np.tile(x[:6], (B, 1)), np.tile(x[6:], (B, 1)), np.tile(u, (B, 1)), float(dt),
                               fext=self._fext, frame=self.wrench_frame)
        return np.hstack([qo, vo])


def world_to_local_wrench(model, q, f_world):
    """World-frame wrench [f; n] at the joint-6 origin's world placement -> local frame
    (pinocchio ``oMi[6].actInv(Force)``, src/gato_mpc_batch_sample.py:151-161)."""
    from ..utils import query_handle

    q = np.asarray(q, float).reshape(6)
    p, _ = query_handle(model).eepos(q, jacobian=True)
    R = _rotation_joint6(model, q)
    f = np.asarray(f_world, float).reshape(6)
    fl = R.T @ f[:3]
    nl = R.T @ (f[3:] - np.cross(p[0], f[:3]))
    return np.concatenate([fl, nl])


def _rotation_joint6(model, q):
    R = np.eye(3)
    for i in range(6):
        c, s = np.cos(q[i]), np.sin(q[i])
        Rz = np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
        R = R @ np.asarray(model.params["placement_R"][i]) @ Rz
    return R


for _n in _SIZES:
    globals()[f"SQPSolverfloat_{_n}"] = type(f"SQPSolverfloat_{_n}", (_SQPSolverBatch,), {"batch_size": _n})

__all__ = [f"SQPSolverfloat_{n}" for n in _SIZES] + ["world_to_local_wrench"]
