"""ADMM mode on the GPU (I7M_QP_ADMM, k_admm_scale / k_admm_factor / k_admm_iter): OSQP's algorithm — the reference's QP solver,
src/osqp_solver.py:38-40, 137-143 — with its warm-started per-problem state, through the C-ABI.

Checked against the C++ port's ADMM mode (oracle/cpp/i7m_cpu.cpp, the same block form; itself
checked against the numpy OSQP restatement in tests/test_admm_oracle.py) and against the
reference's own output (the notebook's printed closed loop).

Tolerances (fp64):
  OSQP iteration counts per QP, line-search steps   : identical
  XU after a solve, carried state (x, z, y, q, rho) : 5e-8 relative.  The x-update's rounding is
      ~1e-12 per solve, but the SQP step of a few problems amplifies it: problem 48 of seed 43
      moves by 1.2e-8 between two port builds whose x-updates differ only in summation order (the
      block Cholesky's C form of round 4 and the LDL' form of round 5), and the device reads
      1.9e-8 there; every discrete outcome (OSQP and SQP iterations, alpha) is identical
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


@pytest.mark.parametrize("N,B,seed", [(16, 8, 41), (32, 64, 43), (16, 512, 41), (64, 24, 48), (5, 16, 49), (32, 13, 50),
                                       (2, 6, 51)])
def test_admm_solves_match_port(lib, model, N, B, seed):
    """Two consecutive solves (the second warm-started from the first's OSQP state) on the GPU and
    on the port: same OSQP iterations and steps, same XU and state.  (16, 512, 41) holds problems
    whose first line search finds no step (alpha = 0): src/osqp_sqp.py:81-82 re-solves the same QP,
    which OSQP's warm start makes a different iterate — the GPU re-solves too (k_linesearch mode 2).
    N = 64 runs the scaling kernel's wide variant; N = 5 a short horizon, N = 2 the shortest (every
    sweep step a segment end); B = 13 and 6 leave rows of k_admm_iter's last wave (four problems per
    wave) empty."""
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
        assert _rel(out, ref).max() < 5e-8, _rel(out, ref).max()
        x, z, y, q, r = h.admm_state(B)
        np.testing.assert_allclose(r, st.rho, rtol=0, atol=0)
        for a, b_ in ((x, st.x), (z, st.z), (y, st.y), (q, st.q)):
            assert _rel(a, b_).max() < 5e-8
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


def test_admm_adaptive_rho_matches_port(lib, model):
    """OSQP's adaptive rho (admm_adaptive_rho_interval > 0: k_admm_iter's in-place re-factorisation)
    against the port (itself pinned to the numpy OSQP restatement with the same settings,
    tests/test_admm_oracle.py): OSQP iteration counts identical, the rho after every solve to 1e-6
    (OSQP's estimate is the square root of a ratio of residual maxima, measured <= 3.2e-8), XU to 5e-8; rho starts at 0.005 so that it actually moves."""
    N, B = 32, 48
    kw = dict(rho=0.005, adaptive_rho_interval=25)
    xcur, goals, XU = synthetic_batch(B, N, 50)
    h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, admm=kw)
    st = cpu.AdmmState(B, N, rho=0.005)
    xin = XU
    for call in range(2):
        out, s = h.solve(xcur, goals, xin)
        it, rho = h.admm_stats(B)
        ref, qp, al, _, it_r = cpu.solve_admm(xcur, goals, xin, N, st, admm=cpu.admm_cfg(**kw))
        np.testing.assert_array_equal(s["qp_iters"], qp)
        for b in range(B):
            np.testing.assert_array_equal(it[b, :qp[b]], it_r[b, :qp[b]], err_msg=f"call {call} problem {b}")
            np.testing.assert_array_equal(s["alphas"][b, :s["n_alphas"][b]], al[b, :qp[b]])
        np.testing.assert_allclose(rho, st.rho, rtol=1e-6)
        assert (rho != 0.005).sum() >= B // 2, rho  # the re-factorisation ran on most problems
        assert _rel(out, ref).max() < 5e-8, _rel(out, ref).max()
        xin = out


def test_admm_full_size_every_problem_matches_port(lib, model):
    """Config 3 at full size in ADMM mode (B = 4096, N = 32, seed 45, cold OSQP state): every
    problem's SQP iterations, OSQP iterations per QP and line-search steps equal the port's, XU to
    1e-7 (measured max 1.4e-8, median 3.9e-10: the M of a second SQP iteration has cond ~4e7, so
    the linearisations' 1e-16 differences reach x at ~1e-9) — the same comparison the bench's headline `parity_vs_port` makes, as a test."""
    B, N = 4096, 32
    xcur, goals, XU = synthetic_batch(B, N, 45)
    h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
    out, s = h.solve(xcur, goals, XU)
    it, _ = h.admm_stats(B)
    ref, qp, al, _, it_r = cpu.solve_admm(xcur, goals, XU, N, cpu.AdmmState(B, N), nthreads=16)
    np.testing.assert_array_equal(s["qp_iters"], qp)
    used = np.arange(8)[None, :] < qp[:, None]
    np.testing.assert_array_equal(np.where(used, it, -1), np.where(used, it_r, -1))
    ga = s["alphas"][:, :al.shape[1]]
    used_a = np.arange(ga.shape[1])[None, :] < s["n_alphas"][:, None]
    assert np.array_equal(used_a, ~np.isnan(al)) and np.array_equal(ga[used_a], al[used_a])
    rel = _rel(out, ref)
    assert rel.max() < 1e-7 and np.median(rel) < 5e-9, (rel.max(), np.median(rel))


def test_admm_staggered_device_ranges_equal_one_range(lib, model, monkeypatch):
    """i7m_solve_device in ADMM mode at B >= 3072 runs the batch as two ranges on streams of their
    own, the second started behind the first's first scaling + factor (I7M_ADMM_STAGGER 1, the
    default): two consecutive solves equal a one-range handle's (I7M_ADMM_STAGGER 0) bit for bit,
    the OSQP state, iteration records, statuses and duals included."""
    import torch
    B, N = 4096, 32
    xcur, goals, XU = synthetic_batch(B, N, 45)
    dev = torch.device("cuda", 0)
    res = []
    for mode in ("0", "1"):
        monkeypatch.setenv("I7M_ADMM_STAGGER", mode)
        h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
        t_xu, t_xs, t_g = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (XU, xcur, goals))
        outs = []
        for call in range(2):
            t_out = torch.empty_like(t_xu)
            torch.cuda.synchronize()
            h.solve_device(B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr())
            h.synchronize()
            outs.append(t_out.cpu().numpy())
            t_xu = t_out
        res.append((outs, h.admm_stats(B, with_status=True), h.admm_state(B), h.admm_dual(B)))
        h.close()
    (o0, st0, x0, s0), (o1, st1, x1, s1) = res
    for a, b in zip(o0, o1):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(st0 + x0, st1 + x1):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(s0, s1)
    assert (st1[0][:, 0] >= 25).all()  # every problem ran its first QP


def test_admm_staggered_closed_loop_equals_one_range(lib, model, monkeypatch):
    """i7m_mpc_run in ADMM mode at B >= 3072 runs each half of the instances through every MPC
    step on its own stream (the second half behind the first's first scaling + factor): the
    distances, q histories, final states and trajectories equal a one-range run's bit for bit
    (NaN where an instance stopped, in the same places)."""
    tr = json.load(open(GOLD))["mpc_trace"]
    B, N = 4096, 32
    xcur, _, _ = synthetic_batch(B, N, 45)
    res = []
    for mode in ("0", "1"):
        monkeypatch.setenv("I7M_ADMM_STAGGER", mode)
        h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
        ends = h.eepos(np.array(tr["endpoint_q"]))
        res.append(h.mpc_run(xcur, ends, 3))
        h.close()
    for a, b in zip(*res):
        np.testing.assert_array_equal(a, b)
    assert np.isfinite(res[1][0][0]).all()


def test_admm_staggered_host_to_host_equals_one_piece(lib, model, monkeypatch):
    """i7m_solve in ADMM mode at B >= 3072 runs two chunks (copy-in, solve, copy-out each), the
    second chunk's solve behind the first's first scaling + factor: two consecutive solves equal a
    one-piece handle's (h2h_chunks = 1, no stagger) bit for bit, state and OSQP records included."""
    B, N = 3072, 32
    xcur, goals, XU = synthetic_batch(B, N, 46)
    monkeypatch.setenv("I7M_ADMM_STAGGER", "0")
    h1 = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, h2h_chunks=1)
    monkeypatch.setenv("I7M_ADMM_STAGGER", "1")
    h2 = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM)
    a1, s1 = h1.solve(xcur, goals, XU)
    a2, s2 = h2.solve(xcur, goals, XU)
    np.testing.assert_array_equal(a1, a2)
    b1, _ = h1.solve(xcur, goals, a1)
    b2, _ = h2.solve(xcur, goals, a2)
    np.testing.assert_array_equal(b1, b2)
    for u, v in zip(h1.admm_state(B), h2.admm_state(B)):
        np.testing.assert_array_equal(u, v)
    for u, v in zip(h1.admm_stats(B, with_status=True), h2.admm_stats(B, with_status=True)):
        np.testing.assert_array_equal(u, v)
    h1.close()
    h2.close()


def test_admm_status_and_dual(lib, model):
    """OSQP's result fields through QPSolution: status "solved" with the default settings and
    "maximum iterations reached" when max_iter stops OSQP before its termination test passes; y
    is the unscaled dual (OSQP's result.y), so P x + q + A'y is OSQP's dual residual, within its
    tolerance eps_abs + eps_rel * scale, and A x = l within the primal tolerance."""
    from indy7_mpc_amd.osqp_solver import OSQPSolver
    N = 16
    xcur, goals, XU = synthetic_batch(1, N, 51)
    s = OSQPSolver(model, N=N)  # qp_mode "admm" is the default
    sol = s.setup_and_solve_qp(XU[0], xcur[0], goals[0])
    assert sol.info.status == "solved" and sol.info.iter % 25 == 0
    P = s.P.copy()
    P.data[:] = s.Pdata
    Pf = P + P.T - np.diag(P.diagonal())
    A = s.A.copy()
    A.data[:] = s.Adata
    x, y = sol.x, sol.y
    dres = Pf @ x + s.g + A.T @ y
    scale = max(np.abs(Pf @ x).max(), np.abs(s.g).max(), np.abs(A.T @ y).max())
    assert np.abs(dres).max() <= 1e-3 + 1e-3 * scale, (np.abs(dres).max(), scale)
    pres = A @ x - s.l
    assert np.abs(pres).max() <= 1e-3 + 1e-3 * max(np.abs(A @ x).max(), np.abs(s.l).max())
    s2 = OSQPSolver(model, N=N, admm={"max_iter": 10})
    sol2 = s2.setup_and_solve_qp(XU[0], xcur[0], goals[0])
    assert sol2.info.status == "maximum iterations reached" and sol2.info.iter == 10


def test_admm_iteration_record_is_reset_every_solve(lib, model):
    """i7m_get_admm_stats after a solve reports -1 for the SQP iterations that solve did not run,
    even where an earlier solve ran them.  The step tolerance is chosen from the port's
    first-iteration step lengths of two consecutive solves (1 % away from every one of them), so
    that some problems run two QPs in solve 1 and stop after one in solve 2."""
    N, B = 16, 16
    xcur, goals, XU = synthetic_batch(B, N, 52)
    st = cpu.AdmmState(B, N)
    o1, _, _, s1c, _ = cpu.solve_admm(xcur, goals, XU, N, st)
    _, _, _, s2c, _ = cpu.solve_admm(xcur, goals, o1, N, st)
    a, b_ = s1c[:, 0], s2c[:, 0]
    allst = np.concatenate([a, b_])
    cands = [t for t in np.unique(np.round(allst, 1)) + 0.5
             if ((a > t) & (b_ < t)).any() and np.min(np.abs(allst - t) / allst) > 0.01]
    assert cands, (a, b_)
    h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, step_tol=float(cands[len(cands) // 2]))
    out, r1 = h.solve(xcur, goals, XU)
    it1 = h.admm_stats(B)[0]
    out, r2 = h.solve(xcur, goals, out)
    it2, _, st2 = h.admm_stats(B, with_status=True)
    stale = (r1["qp_iters"] == 2) & (r2["qp_iters"] == 1)
    assert stale.any(), (r1["qp_iters"], r2["qp_iters"])
    assert (it1[stale, 1] > 0).all()
    for b in range(B):
        n = r2["qp_iters"][b]
        assert (it2[b, :n] > 0).all() and (it2[b, n:] == -1).all(), (b, n, it2[b])
        assert (st2[b, :n] >= 0).all() and (st2[b, n:] == -1).all(), (b, n, st2[b])


def test_admm_state_over_2gib_is_refused(lib, model):
    """k_admm_iter addresses the handle's ADMM state with 32-bit offsets: i7m_create refuses a
    max_batch x N whose state would pass 2 GiB (before allocating anything), with a message."""
    with pytest.raises(Exception, match="2 GiB"):
        lib.Handle(model, N=64, max_batch=200000, qp_mode=lib.QP_ADMM)



@pytest.mark.parametrize("max_iter,eps", [(20, 1e-3), (50, 1e-8)])
def test_admm_status_after_max_iter_matches_port(lib, model, max_iter, eps):
    """OSQP's closing tests after max_iter (oracle/osqp_admm.py OSQP.solve :344-349):
    k_admm_iter runs the termination test at the final iterate unless the last iteration ran it, then
    the approximate test (eps x 10) -> status 2 "solved inaccurate".  (20, 1e-3): 20 is no multiple
    of check_termination 25, so both closing tests run — statuses 0, 1 and 2 all occur; (50, 1e-8):
    only the approximate one.  Status, OSQP iterations, alphas = the port's (itself = the numpy
    restatement's, tests/test_admm_oracle.py::test_port_admm_status_after_max_iter_matches_numpy_osqp);
    QPSolution maps the codes to OSQP's strings."""
    from indy7_mpc_amd.osqp_solver import QPSolution
    N, B = 16, 64
    cfg = dict(max_iter=max_iter, eps_abs=eps, eps_rel=eps)
    xcur, goals, XU = synthetic_batch(B, N, 41)
    h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, admm=cfg)
    out, s = h.solve(xcur, goals, XU)
    it, _, stat = h.admm_stats(B, with_status=True)
    st = cpu.AdmmState(B, N)
    ref, qp, al, _, it_r = cpu.solve_admm(xcur, goals, XU, N, st, admm=cpu.admm_cfg(**cfg))
    np.testing.assert_array_equal(s["qp_iters"], qp)
    ran = np.arange(8)[None, :] < qp[:, None]
    np.testing.assert_array_equal(np.where(ran, it, -1), np.where(ran, it_r, -1))
    np.testing.assert_array_equal(np.where(ran, stat, -9), np.where(ran, st.status, -9))
    assert (stat[~ran] == -1).all()
    seen = set(stat[ran].tolist())
    assert ({0, 1, 2} if max_iter == 20 else {1, 2}) <= seen, seen
    assert _rel(out, ref).max() < 5e-8
    assert [QPSolution.from_admm(None, c, 1, None).info.status for c in (1, 2, 0)] == \
        ["solved", "solved inaccurate", "maximum iterations reached"]
    assert [QPSolution.from_admm(None, c, 1, None).info.status_val for c in (1, 2, 0)] == [1, 2, -2]
    with pytest.raises(RuntimeError, match="no OSQP result"):
        QPSolution.from_admm(None, -1, 0, None)


KERNELS = (("res", {"I7M_ADMM_RES": "1", "I7M_ADMM_ITER2": "-1"}),
           ("iter2", {"I7M_ADMM_RES": "0", "I7M_ADMM_ITER2": "1"}),
           ("iter4", {"I7M_ADMM_RES": "0", "I7M_ADMM_ITER2": "0"}))


@pytest.mark.parametrize("B,N,admm", [(13, 32, None), (600, 32, None), (1, 32, None), (13, 16, None),
                                      (13, 32, {"max_iter": 20})])
def test_admm_iteration_kernels_bit_identical(lib, model, monkeypatch, B, N, admm):
    """The three OSQP iteration kernels run the same arithmetic per problem: k_admm_iter_res (one
    problem per workgroup, LDS-resident: launches of <= 256 problems at N <= 32), k_admm_iter2 (two
    per wave: <= 512) and k_admm_iter (four), each forced (I7M_ADMM_RES, I7M_ADMM_ITER2): two
    consecutive solves are equal bit for bit, carried state, OSQP records and statuses included
    (B = 13: empty rows in the streaming kernels' last wave; max_iter 20: the closing tests)."""
    xcur, goals, XU = synthetic_batch(B, N, 54)
    res = []
    for _, env in KERNELS:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        kw = {"admm": admm} if admm else {}
        h = lib.Handle(model, N=N, max_batch=B, qp_mode=lib.QP_ADMM, **kw)
        o1, _ = h.solve(xcur, goals, XU)
        o2, _ = h.solve(xcur, goals, o1)
        res.append((o1, o2) + h.admm_state(B) + h.admm_stats(B, with_status=True))
        h.close()
    for other in res[1:]:
        for a, b in zip(res[0], other):
            np.testing.assert_array_equal(a, b)
