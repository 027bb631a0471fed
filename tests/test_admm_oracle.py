"""ADMM mode (OSQP's algorithm, the reference's QP solver: src/osqp_solver.py:38-40, 137-143).

oracle/osqp_admm.py restates OSQP (scaling, warm start, termination with the duality-gap test)
and is pinned by the reference's own output: the closed loop the notebook prints
(notebooks/pin_mpc_indy7.ipynb cell 2, tests/golden/notebook_kats.json "mpc_trace").  The C++
port (oracle/cpp/i7m_cpu.cpp ``admm``) runs the same algorithm in the block form the GPU's
the device kernels use, and is checked against the numpy restatement here.
"""
import json
import os

import numpy as np
import pytest

from oracle import cpu, rbd
from oracle.mpc_ref import run_mpc_ref
from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch

GOLD = os.path.join(os.path.dirname(__file__), "golden", "notebook_kats.json")


@pytest.fixture(scope="module")
def trace():
    return json.load(open(GOLD))["mpc_trace"]


def test_osqp_restatement_reproduces_notebook_closed_loop(trace):
    """The first 12 printed goal distances to 1e-9 (the exact KKT solve: 1.1e-6), the first
    three to 1e-13: the reference's OSQP iterates, not just its limit."""
    ends = [rbd.eepos(np.array(q)) for q in trace["endpoint_q"]]
    s = OSQPSolverRef(N=32, qp="osqp")
    _, d = run_mpc_ref(SQPRef(s), np.array(trace["xstart"]), ends, num_steps=12)
    err = np.abs(np.array(d) - np.array(trace["goal_distances"][:12]))
    assert err[:3].max() < 1e-13, err
    assert err.max() < 1e-9, err
    assert all(st == "solved" for st in [s.osqp.info["status"]])
    assert {h[0] for h in s.osqp.history} <= {25, 50, 75}


def _port_closed_loop(xstart, ends, steps, N=32):
    """MPC_OSQP.run_mpc (src/osqp_mpc.py:14-72, as oracle/mpc_ref.py) with every SQP solve by the
    C++ port's ADMM mode and the OSQP state carried from call to call."""
    nq, nx, nu = 6, 12, 6
    st = cpu.AdmmState(1, N)
    xcur = np.asarray(xstart, float)
    ei = 0
    goal = np.tile(ends[ei], N)
    XU = np.zeros(N * 18 - 6)

    def sqp(x, g, xu):
        out, *_ = cpu.solve_admm(x[None], g[None], xu[None], N, st)
        return out[0]

    XU = sqp(xcur, goal, XU)
    dists = []
    for i in range(steps):
        d = np.linalg.norm(rbd.eepos(xcur[:nq]) - goal[:3])
        if d < 1e-1:
            ei = (ei + 1) % len(ends)
            goal = np.tile(ends[ei], N)
        dists.append(d)
        xu_new = sqp(xcur, goal, XU)
        u = XU[nx:nx + nu]
        qn, vn = rbd.rk4(xcur[:nq], xcur[nq:nx], u, 0.01)
        xcur = np.concatenate([qn, vn])
        XU[:-(nx + nu)] = xu_new[nx + nu:]
        XU[:nx] = xcur
        XU[-nx:] = np.hstack([np.ones(nq), np.zeros(nq)])
    return np.array(dists)


def test_port_admm_closed_loop_matches_notebook(trace):
    ends = [rbd.eepos(np.array(q)) for q in trace["endpoint_q"]]
    d = _port_closed_loop(np.array(trace["xstart"]), ends, 16)
    err = np.abs(d - np.array(trace["goal_distances"][:16]))
    assert err[:3].max() < 1e-13, err
    assert err.max() < 1e-9, err


@pytest.mark.parametrize("N,seed", [(16, 41), (32, 43)])
def test_port_admm_matches_numpy_osqp(N, seed):
    """Block Cholesky of the reduced system (port, GPU) vs OSQP's quasi-definite KKT (numpy,
    sparse LU): same OSQP iteration counts and line-search steps, XU to 1e-8."""
    B = 6
    xcur, goals, XU = synthetic_batch(B, N, seed)
    st = cpu.AdmmState(B, N)
    out, qp, al, _, it = cpu.solve_admm(xcur, goals, XU, N, st)
    # a second call from the carried state (the reference's warm start across solves)
    out2, qp2, al2, _, it2 = cpu.solve_admm(xcur, goals, out, N, st)
    for b in range(B):
        s = OSQPSolverRef(N=N, qp="osqp")
        sq = SQPRef(s)
        x = sq.sqp(xcur[b], goals[b], XU[b].copy())
        its = [h[0] for h in s.osqp.history]
        assert its == list(it[b, :qp[b]]), (b, its, it[b])
        np.testing.assert_array_equal(sq.stats["linesearch_alphas"]["values"], al[b, :qp[b]])
        assert np.linalg.norm(x - out[b]) <= 1e-8 * np.linalg.norm(x)
        x2 = sq.sqp(xcur[b], goals[b], x.copy())
        its2 = [h[0] for h in s.osqp.history][len(its):]
        assert its2 == list(it2[b, :qp2[b]])
        assert np.linalg.norm(x2 - out2[b]) <= 1e-8 * np.linalg.norm(x2)
        assert s.osqp.info["status"] == "solved"


def test_admm_tight_tolerance_reaches_the_exact_qp():
    """With a tight tolerance OSQP's iterate is the QP's minimiser: the ADMM-mode SQP takes the
    exact-KKT SQP's (direct mode) steps and ends within 1e-7 of it."""
    N, B = 16, 4
    xcur, goals, XU = synthetic_batch(B, N, 42)
    ref, qp_r, al_r, _ = cpu.solve(xcur, goals, XU, N)
    st = cpu.AdmmState(B, N)
    out, qp, al, _, it = cpu.solve_admm(xcur, goals, XU, N, st,
                                        admm=cpu.admm_cfg(eps_abs=1e-12, eps_rel=1e-12, max_iter=20000))
    np.testing.assert_array_equal(al, al_r)
    rel = np.linalg.norm(out - ref, axis=1) / np.linalg.norm(ref, axis=1)
    assert rel.max() < 1e-7, rel
