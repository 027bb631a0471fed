"""ADMM mode on the GPU (I7M_QP_ADMM, k_admm_scale / k_admm_factor / k_admm_iter): OSQP's algorithm — the reference's QP solver,
src/osqp_solver.py:38-40, 137-143 — with its warm-started per-problem state, through the C-ABI.

Checked against the C++ port's ADMM mode (oracle/cpp/i7m_cpu.cpp, the same block form; itself
checked against the numpy OSQP restatement in tests/test_admm_oracle.py) and against the
reference's own output (the notebook's printed closed loop).

Tolerances (fp64):
  OSQP iteration counts per QP, line-search steps   : identical
  XU after a solve, carried state (x, z, y, q, rho) : 1e-8 relative (a termination test every 25
      iterations; between them rounding of the two builds' sums stays ~1e-12)
  closed loop vs the notebook's printed distances   : 1e-12 over the first 3 steps, 2e-9 over 8,
      5e-8 over 16 (the loop amplifies a 1e-12 difference ~2x per step; the exact KKT solve is
      already 1.1e-6 off at step 16)
"""
import json
import os

import numpy as np
import pytest

from oracle import cpu
from oracle.osqp_ref import synthetic_batch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "notebook_kats.json")


@pytest.fixture(scope="module")
def lib():
    from indy7_mpc_amd import _lib
    _lib.load()
    if _lib.device_count() < 1:
        pytest.fail("no GPU visible but the gpu tests were requested")
    return _lib


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-300)


@pytest.mark.parametrize("N,B,seed", [(16, 8, 41), (32, 64, 43), (16, 512, 41)])
def test_admm_solves_match_port(lib, model, N, B, seed):
    """Two consecutive solves (the second warm-started from the first's OSQP state) on the GPU and
    on the port: same OSQP iterations and steps, same XU and state.  (16, 512, 41) holds problems
    whose first line search finds no step (alpha = 0): src/osqp_sqp.py:81-82 re-solves the same QP,
    which OSQP's warm start makes a different iterate — the GPU re-solves too (k_linesearch mode 2)."""
    xcur, goals, XU = synthetic_batch(B, N, seed)
    h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
    st = cpu.AdmmState(B, N)
    xin = XU
    for call in range(2):
        out, s = h.solve(xcur, goals, xin)
        it, rho = h.admm_stats(B)
        ref, qp, al, _, it_r = cpu.solve_admm(xcur, goals, xin, N, st)
        np.testing.assert_array_equal(s["qp_iters"], qp)
        if (N, B, seed) == (16, 512, 41) and call == 0:
            assert (al[:, 0] == 0.0).sum() >= 5  # the case this parameter set is for
        for b in range(B):
            n = qp[b]
            np.testing.assert_array_equal(it[b, :n], it_r[b, :n], err_msg=f"call {call} problem {b}")
            np.testing.assert_array_equal(s["alphas"][b, :s["n_alphas"][b]], al[b, :n])
        assert _rel(out, ref).max() < 1e-8, _rel(out, ref).max()
        x, z, y, q, r = h.admm_state(B)
        np.testing.assert_allclose(r, st.rho, rtol=0, atol=0)
        for a, b_ in ((x, st.x), (z, st.z), (y, st.y), (q, st.q)):
            assert _rel(a, b_).max() < 1e-8
        xin = out


def test_admm_reset_is_a_fresh_solver(lib, model):
    N, B = 16, 4
    xcur, goals, XU = synthetic_batch(B, N, 44)
    h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
    first, _ = h.solve(xcur, goals, XU)
    second, _ = h.solve(xcur, goals, first)
    h.reset()
    again, _ = h.solve(xcur, goals, XU)
    np.testing.assert_array_equal(again, first)
    # the warm start matters: the second call from the carried state is not a cold solve
    h2 = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
    cold, _ = h2.solve(xcur, goals, first)
    assert not np.array_equal(cold, second)
    # resetRho / resetLambda touch only their part of the state
    h.admm_reset(what=lib.ADMM_RESET_DUAL)
    x, z, y, q, rho = h.admm_state(B)
    assert not y.any() and x.any() and q.any()
    h.admm_reset(what=lib.ADMM_RESET_RHO)
    assert (h.admm_state(B)[4] == 0.1).all()


def test_admm_closed_loop_reproduces_notebook(lib, model):
    """MPC_OSQP.run_mpc on the device (i7m_mpc_run) in ADMM mode from the notebook's start: the
    printed goal distances of the reference's OSQP run (pin_mpc_indy7.ipynb cell 2)."""
    tr = json.load(open(GOLD))["mpc_trace"]
    h = lib.Handle(model, N=32, max_batch=1, qp_mode=lib.QP_ADMM)
    ends = h.eepos(np.array(tr["endpoint_q"]))
    d, *_ = h.mpc_run(np.array([tr["xstart"]]), ends, 16)
    err = np.abs(d[:, 0] - np.array(tr["goal_distances"][:16]))
    assert err[:3].max() < 1e-12, err
    assert err[:8].max() < 2e-9, err
    assert err.max() < 5e-8, err


def test_admm_drop_in_surfaces(lib, model):
    """OSQPSolver(qp_mode="admm").setup_and_solve_qp returns OSQP's iterate and iteration count;
    batch_sqp's ADMM mode reports OSQP iterations as its inner-solver stats."""
    from indy7_mpc_amd.bindings import batch_sqp
    from indy7_mpc_amd.osqp_solver import OSQPSolver
    N = 16
    xcur, goals, XU = synthetic_batch(1, N, 45)
    s = OSQPSolver(model, N=N, qp_mode="admm")
    sol = s.setup_and_solve_qp(XU[0], xcur[0], goals[0])
    st = cpu.AdmmState(1, N)
    ref, qp, *_ , it_r = cpu.solve_admm(xcur, goals, XU, N, st, max_iters=1)
    assert sol.info.iter == it_r[0, 0] and sol.info.iter % 25 == 0
    b = batch_sqp.SQPSolverfloat_4(model, qp_mode="admm")
    xc4, g4, XU4 = synthetic_batch(4, N, 46)
    g6 = np.zeros((4, 6 * N))
    g6.reshape(4, N, 6)[:, :, :3] = g4.reshape(4, N, 3)
    r = b.solve(XU4, 0.01, xc4, g6)
    assert all((p["pcg_iterations"] % 25 == 0).all() and (p["pcg_iterations"] >= 0).all() for p in r["pcg_stats"])
    b.resetLambda()
    b.resetRho()
    b.reset()


def test_admm_chunked_host_to_host_equals_one_piece(lib, model):
    """i7m_solve's chunked host-to-host pipeline (h2h_chunks = 3) hands each chunk its own rows of
    the OSQP state: two consecutive solves equal a one-piece handle's bit for bit, state included."""
    N, B = 16, 600
    xcur, goals, XU = synthetic_batch(B, N, 47)
    h1 = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, h2h_chunks=1)
    h3 = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, h2h_chunks=3)
    a1, _ = h1.solve(xcur, goals, XU)
    a3, _ = h3.solve(xcur, goals, XU)
    np.testing.assert_array_equal(a1, a3)
    b1, _ = h1.solve(xcur, goals, a1)
    b3, _ = h3.solve(xcur, goals, a3)
    np.testing.assert_array_equal(b1, b3)
    for u, v in zip(h1.admm_state(B), h3.admm_state(B)):
        np.testing.assert_array_equal(u, v)
    np.testing.assert_array_equal(h1.admm_stats(B)[0], h3.admm_stats(B)[0])
