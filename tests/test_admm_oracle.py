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
    # (the block LDL' solve of round 5 reads 1.1e-13 at step 3, the block Cholesky's C form 7e-15:
    # rounding of the x-update, which the closed loop doubles every ~1.5 steps; over 16 steps the
    # LDL' form with the row-sum u-part reads 1.2e-9, the C form 0.9e-9 — the exact KKT solve is
    # 1.1e-6 off there)
    assert err[:3].max() < 3e-13, err
    assert err.max() < 5e-9, err


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


@pytest.mark.parametrize("N,seed", [(16, 44), (32, 45)])
def test_port_admm_adaptive_rho_matches_numpy_osqp(N, seed):
    """OSQP's adaptive rho (the reference's OSQP default adapts; its interval is timing-based,
    oracle/osqp_admm.py) at a fixed interval of 25 and a tolerance tight enough that rho moves:
    the port (block form, re-factoring in place) takes the numpy restatement's OSQP iteration
    counts, line-search steps and final rho, XU to 1e-8.  rho starts at 0.005 (a setting's
    choice), so that the estimate leaves the tolerance band of 5 and rho moves."""
    B = 4
    xcur, goals, XU = synthetic_batch(B, N, seed)
    kw = dict(rho=0.005, adaptive_rho_interval=25)
    st = cpu.AdmmState(B, N, rho=0.005)
    out, qp, al, _, it = cpu.solve_admm(xcur, goals, XU, N, st, admm=cpu.admm_cfg(**kw))
    moved = 0
    for b in range(B):
        s = OSQPSolverRef(N=N, qp="osqp", osqp_settings=dict(kw))
        sq = SQPRef(s)
        x = sq.sqp(xcur[b], goals[b], XU[b].copy())
        its = [h[0] for h in s.osqp.history]
        assert its == list(it[b, :qp[b]]), (b, its, it[b])
        np.testing.assert_array_equal(sq.stats["linesearch_alphas"]["values"], al[b, :qp[b]])
        assert np.linalg.norm(x - out[b]) <= 1e-8 * np.linalg.norm(x)
        assert abs(s.osqp.rho - st.rho[b]) <= 1e-8 * s.osqp.rho, (s.osqp.rho, st.rho[b])
        moved += s.osqp.rho != 0.005
    assert moved > 0, "rho never adapted: the test would not exercise the re-factorisation"


def test_direct_mode_vs_osqp_distribution_is_pinned():
    """The exact KKT solve (qp_mode "direct", the optimum) against OSQP's own iterate (qp_mode
    "admm", the reference's numbers, eps 1e-3) on config-3 draws (seed 45, 1024 problems, cold
    OSQP state): same line-search steps on every problem, but XU differs by OSQP's tolerance —
    measured median 5.8e-5, p90 2.0e-4, max 1.0e-3, 31 % of problems above north_star's 1e-4.
    Pinned here so the gap between the two modes cannot drift unseen (VERDICT r4 "What's weak" 1);
    the device's direct mode equals the port's direct mode to 1e-12 (tests/test_gpu_solver.py),
    so these are also the device's numbers, and bench.py reports them as `exact_mode.parity_vs_port_admm`."""
    B, N = 1024, 32
    xcur, goals, XU = synthetic_batch(B, N, 45)
    d, qp_d, al_d, _ = cpu.solve(xcur, goals, XU, N, nthreads=8)
    a, qp_a, al_a, _, _ = cpu.solve_admm(xcur, goals, XU, N, cpu.AdmmState(B, N), nthreads=8)
    rel = np.linalg.norm(d - a, axis=1) / np.linalg.norm(a, axis=1)
    same = np.all(np.where(np.isnan(al_d) & np.isnan(al_a), True, al_d == al_a), axis=1)
    assert same.all() and (qp_d == qp_a).all()
    assert 3e-5 < np.median(rel) < 1.2e-4, np.median(rel)
    assert 0.2 < (rel > 1e-4).mean() < 0.45, (rel > 1e-4).mean()
    assert rel.max() < 1e-2, rel.max()


def _world_forces(B, seed):
    """World-frame wrench hypotheses as gato_controller.py:77-81,120-129 draws them: forces only
    (torque part zero), row 0 zero."""
    f = np.random.default_rng(seed).normal(0, 30, (B, 6))
    f[:, 3:] = 0.0
    f[0] = 0.0
    return f


def test_port_world_wrench_direct_matches_numpy_oracle():
    """The port's world-frame wrench (cfg fext_frame "world": F0 -= f_w in the linearisation with
    the +S_r.(S_j x* f_w) term a world-fixed force adds to d tau / dq, actInv per configuration in
    the merit) against the numpy oracle, whose derivatives are complex-step through rbd.fext_list:
    alpha sequences identical, XU 1e-8 (exact QP both sides)."""
    N, B = 16, 4
    xcur, goals, XU = synthetic_batch(B, N, 13)
    f = _world_forces(B, 1)
    f[3, 3:] = [0.5, -0.5, 1.0]
    out, qp, al, _ = cpu.solve(xcur, goals, XU, N, fext=f, fext_frame="world")
    loc, *_ = cpu.solve(xcur, goals, XU, N, fext=f, fext_frame="local")
    for b in range(B):
        sq = SQPRef(OSQPSolverRef(N=N, fext6=f[b], fext_frame="world"))
        x = sq.sqp(xcur[b], goals[b], XU[b].copy())
        np.testing.assert_array_equal(sq.stats["linesearch_alphas"]["values"], al[b, :qp[b]])
        assert np.linalg.norm(x - out[b]) <= 1e-8 * np.linalg.norm(x), b
        if b:
            assert not np.allclose(out[b], loc[b])  # the frames are different models


def test_port_admm_world_wrench_matches_numpy_osqp():
    """batch_sqp's default (ADMM mode, world-frame wrench, gato_controller.py:90,95,129-138) on the
    port against the numpy OSQP restatement with the same wrench: two consecutive solves with
    resetLambda (OSQP's y = 0) between them; OSQP iterations and alphas identical, XU 1e-8."""
    N, B = 16, 4
    xcur, goals, XU = synthetic_batch(B, N, 17)
    f = _world_forces(B, 3)
    st = cpu.AdmmState(B, N)
    out, qp, al, _, it = cpu.solve_admm(xcur, goals, XU, N, st, fext=f, fext_frame="world")
    st.y[:] = 0.0  # resetLambda
    out2, qp2, al2, _, it2 = cpu.solve_admm(xcur, goals, out, N, st, fext=f, fext_frame="world")
    for b in range(B):
        s = OSQPSolverRef(N=N, qp="osqp", fext6=f[b], fext_frame="world")
        sq = SQPRef(s)
        x = sq.sqp(xcur[b], goals[b], XU[b].copy())
        its = [h[0] for h in s.osqp.history]
        assert its == list(it[b, :qp[b]]), (b, its, it[b])
        np.testing.assert_array_equal(sq.stats["linesearch_alphas"]["values"], al[b, :qp[b]])
        assert np.linalg.norm(x - out[b]) <= 1e-8 * np.linalg.norm(x), b
        s.osqp.y[:] = 0.0
        n0 = len(sq.stats["linesearch_alphas"]["values"])
        x2 = sq.sqp(xcur[b], goals[b], x.copy())
        assert [h[0] for h in s.osqp.history][len(its):] == list(it2[b, :qp2[b]]), b
        np.testing.assert_array_equal(sq.stats["linesearch_alphas"]["values"][n0:], al2[b, :qp2[b]])
        assert np.linalg.norm(x2 - out2[b]) <= 1e-8 * np.linalg.norm(x2), b


STATUS_CODE = {"solved": 1, "solved_inaccurate": 2, "max_iter_reached": 0}


@pytest.mark.parametrize("max_iter,eps", [(10, 1e-3), (20, 1e-3), (50, 1e-8)])
def test_port_admm_status_after_max_iter_matches_numpy_osqp(max_iter, eps):
    """OSQP's status when max_iter stops the iteration: the test once more at the final
    iterate unless the last iteration ran it, then the approximate test (eps x 10, "solved
    inaccurate").  max_iter 10 / 20: the closing exact test runs (no multiple of 25); 50 (eps
    1e-8): only the approximate one.  Port status per QP (i7m_get_admm_status's codes) = the numpy
    restatement's, OSQP iterations and alphas identical."""
    N, B = 16, 8
    xcur, goals, XU = synthetic_batch(B, N, 41)
    st = cpu.AdmmState(B, N)
    cfg = dict(max_iter=max_iter, eps_abs=eps, eps_rel=eps)
    out, qp, al, _, it = cpu.solve_admm(xcur, goals, XU, N, st, admm=cpu.admm_cfg(**cfg))
    seen = set()
    for b in range(B):
        s = OSQPSolverRef(N=N, qp="osqp", osqp_settings=cfg)
        sq = SQPRef(s)
        x = sq.sqp(xcur[b], goals[b], XU[b].copy())
        assert [h[0] for h in s.osqp.history] == list(it[b, :qp[b]]), b
        codes = [STATUS_CODE[h[5]] for h in s.osqp.history]
        assert codes == list(st.status[b, :qp[b]]), (b, codes, st.status[b])
        assert (st.status[b, qp[b]:] == -1).all()
        np.testing.assert_array_equal(sq.stats["linesearch_alphas"]["values"], al[b, :qp[b]])
        assert np.linalg.norm(x - out[b]) <= 1e-8 * np.linalg.norm(x), b
        seen.update(codes)
    # the cases each setting is for: no test can pass / inaccurate after the closing tests /
    # inaccurate after the approximate test alone
    assert {10: {0}, 20: {0, 2}, 50: {1, 2}}[max_iter] <= seen, seen
