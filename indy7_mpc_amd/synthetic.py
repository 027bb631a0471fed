"""Synthetic MPC problems for the bench.

q_start, q_goal ~ U(+-1/2 URDF limit) (description/indy7.urdf:203-238), v_start ~ U(-0.5, 0.5),
goal = FK(q_goal) tiled N times (src/osqp_mpc.py:23), XU = 0 with XU[:12] = x_start
(src/gato_mpc_batch.py:97-99).  Goals are computed by the device FK (i7m_eepos), so this
module needs the GPU library like everything else in the package.
"""
from __future__ import annotations

import numpy as np


def draw_states(model, B: int, seed: int):
    rng = np.random.default_rng(seed)
    lo, hi = 0.5 * model.lowerPositionLimit, 0.5 * model.upperPositionLimit
    q0 = rng.uniform(lo, hi, size=(B, 6))
    v0 = rng.uniform(-0.5, 0.5, size=(B, 6))
    qg = rng.uniform(lo, hi, size=(B, 6))
    return np.hstack([q0, v0]), qg


def make_batch(handle, model, B: int, N: int, seed: int):
    """(xcur (B,12), goals (B,3N), XU (B,18N-6)) — same draws as oracle.synthetic_batch."""
    xcur, qg = draw_states(model, B, seed)
    p = handle.eepos(qg)
    goals = np.tile(p, (1, N))
    XU = np.zeros((B, 18 * N - 6))
    XU[:, :12] = xcur
    return xcur, goals, XU
