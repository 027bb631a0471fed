"""CPU: pin the oracle against the reference's own known-answer data, and check its internal
consistency.  (The reference has no tests; its notebooks' printed outputs are the only KATs,
SURVEY.md §4.)"""
import json
import os

import numpy as np
import pytest

from oracle import rbd
from oracle.mpc_ref import run_mpc_ref
from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def kats():
    with open(os.path.join(GOLD, "notebook_kats.json")) as f:
        return json.load(f)


def test_fk_matches_notebook_kats(kats):
    assert len(kats["fk"]) == 16
    for k in kats["fk"]:
        p = rbd.eepos(np.array(k["q"]))
        exp = np.array(k["eepos"])
        # printed with `digits` significant/decimal digits -> half-ulp of the print
        tol = 0.5 * 10.0 ** (-k["digits"]) * max(1.0, np.abs(exp).max()) + 1e-12
        assert np.abs(p - exp).max() <= tol, (k, p)


def test_first_goal_distance_exact(kats):
    tr = kats["mpc_trace"]
    p0 = rbd.eepos(np.ones(6))
    g = rbd.eepos(np.array(tr["endpoint_q"][0]))
    assert abs(np.linalg.norm(p0 - g) - tr["goal_distances"][0]) < 1e-15


def test_closed_loop_trace_matches_notebook(kats):
    """Oracle (exact QP) vs the reference's OSQP (eps 1e-3) closed loop: the first steps agree
    to ~1e-6; the residual is OSQP's approximation, growing slowly along the trajectory."""
    tr = kats["mpc_trace"]
    ends = [rbd.eepos(np.array(q)) for q in tr["endpoint_q"]]
    _, d = run_mpc_ref(SQPRef(OSQPSolverRef(N=32)), np.array(tr["xstart"]), ends, num_steps=8)
    ref = np.array(tr["goal_distances"][:8])
    err = np.abs(np.array(d) - ref)
    assert err[0] < 1e-15
    assert err.max() < 2e-6, err


def test_dynamics_self_consistency():
    rng = np.random.default_rng(5)
    for _ in range(5):
        q, v, t = rng.uniform(-3, 3, 6), rng.uniform(-2, 2, 6), rng.uniform(-50, 50, 6)
        a = rbd.aba(q, v, t)
        np.testing.assert_allclose(rbd.rnea(q, v, a), t, atol=1e-9)  # RNEA(ABA) = id
        M = rbd.crba(q)
        np.testing.assert_allclose(M, M.T, atol=1e-14)
        assert np.linalg.eigvalsh(M).min() > 0
        b = rbd.rnea(q, v, np.zeros(6))
        np.testing.assert_allclose(np.linalg.solve(M, t - b), a, rtol=1e-9, atol=1e-9)
        dq, dv, Mi, _ = rbd.aba_derivatives(q, v, t)
        np.testing.assert_allclose(Mi @ M, np.eye(6), atol=1e-9)
        h = 1e-6
        fdq = np.array([(rbd.aba(q + h * e, v, t) - rbd.aba(q - h * e, v, t)) / (2 * h) for e in np.eye(6)]).T
        fdv = np.array([(rbd.aba(q, v + h * e, t) - rbd.aba(q, v - h * e, t)) / (2 * h) for e in np.eye(6)]).T
        assert np.abs(fdq - dq).max() <= 1e-5 * max(1, np.abs(dq).max())  # central FD, h=1e-6
        assert np.abs(fdv - dv).max() <= 1e-5 * max(1, np.abs(dv).max())
        p, J = rbd.d_eepos(q)
        fdj = np.array([(rbd.eepos(q + h * e) - rbd.eepos(q - h * e)) / (2 * h) for e in np.eye(6)]).T
        np.testing.assert_allclose(J, fdj, atol=1e-8)


def test_fext_consistency():
    """ABA with a local joint-6 wrench: RNEA(q, v, a, fext) == tau."""
    rng = np.random.default_rng(9)
    q, v, t = rng.uniform(-3, 3, 6), rng.uniform(-2, 2, 6), rng.uniform(-50, 50, 6)
    f = [np.zeros(6)] * 5 + [rng.normal(0, 20, 6)]
    a = rbd.aba(q, v, t, fext=f)
    np.testing.assert_allclose(rbd.rnea(q, v, a, fext=f), t, atol=1e-9)


def test_world_wrench_oracle():
    """World-frame joint-6 wrench (gato_controller.py:77-81 draws them; the reference converts
    with oMi[6].actInv, src/gato_mpc_batch_sample.py:151-161):
      * the conversion is pinocchio's actInv: the converted local force, moved back to the
        world origin by oMi[6], is the world force again;
      * the complex-step derivatives of the world-wrench dynamics match central differences of
        ABA with the wrench re-converted at every perturbed q;
      * rk4 with a world wrench converts once at the start q (the host plant, :270-279)."""
    rng = np.random.default_rng(11)
    q, v, t = rng.uniform(-2, 2, 6), rng.uniform(-1, 1, 6), rng.uniform(-30, 30, 6)
    fw = np.concatenate([rng.normal(0, 30, 3), rng.normal(0, 3, 3)])
    R, p = rbd.fk(q)[-1]
    fl = rbd.wrench_world_to_local(q, fw)
    f_back = R @ fl[:3]
    np.testing.assert_allclose(f_back, fw[:3], atol=1e-12)
    np.testing.assert_allclose(R @ fl[3:] + np.cross(p, f_back), fw[3:], atol=1e-12)
    dq, dv, Mi, a = rbd.aba_derivatives(q, v, t, fext6=fw, frame="world")
    np.testing.assert_allclose(a, rbd.aba(q, v, t, fext=rbd.fext_list(q, fw, "world")), rtol=1e-12)
    h = 1e-6

    def aw(qq, vv):
        return rbd.aba(qq, vv, t, fext=rbd.fext_list(qq, fw, "world"))

    fdq = np.array([(aw(q + h * e, v) - aw(q - h * e, v)) / (2 * h) for e in np.eye(6)]).T
    fdv = np.array([(aw(q, v + h * e) - aw(q, v - h * e)) / (2 * h) for e in np.eye(6)]).T
    assert np.abs(fdq - dq).max() <= 1e-5 * max(1, np.abs(dq).max())
    assert np.abs(fdv - dv).max() <= 1e-5 * max(1, np.abs(dv).max())
    # a local-frame wrench of the same value at q gives the same a but different d/dq
    dql, _, _, al = rbd.aba_derivatives(q, v, t, fext6=fl, frame="local")
    np.testing.assert_allclose(al, a, rtol=1e-10)
    assert np.abs(dql - dq).max() > 1e-3 * np.abs(dq).max()
    qw, vw = rbd.rk4(q, v, t, 0.01, fext6_world=fw)
    ql, vl = rbd.rk4(q, v, t, 0.01, fext=[np.zeros(6)] * 5 + [fl])
    np.testing.assert_array_equal(qw, ql)
    np.testing.assert_array_equal(vw, vl)


@pytest.mark.parametrize("N", [16, 32, 64])
def test_csc_templates(N):
    s = OSQPSolverRef(N=N)
    assert s.P.nnz == 27 * N + 6 * (N - 1)
    assert s.A.nnz == 360 * (N - 1) + 144
    assert s.A.shape == (12 * N, 18 * N - 6)
    assert s.P.has_sorted_indices and s.A.has_sorted_indices


def test_exact_kkt_and_admm():
    N = 16
    xcur, goals, XU = synthetic_batch(1, N, seed=3)
    s = OSQPSolverRef(N=N)
    sol = s.setup_and_solve_qp(XU[0], xcur[0], goals[0])
    P, A = s.matrices()
    Pf = (P + P.T).toarray() - np.diag(P.diagonal())
    r_p = A @ sol.x - s.l
    r_d = Pf @ sol.x + s.g + A.T @ sol.y
    assert np.abs(r_p).max() < 1e-10 * max(1, np.abs(s.l).max())
    assert np.abs(r_d).max() < 1e-8 * max(1, np.abs(s.g).max())
    ad = s.solve_qp_admm(iters=3000, eps_abs=1e-10, eps_rel=1e-10)
    assert np.linalg.norm(ad.x - sol.x) / np.linalg.norm(sol.x) < 1e-6


def test_fixtures_reproduce():
    """Re-derive a slice of each committed fixture with the oracle (guards the fixtures)."""
    for N in (16, 32):
        f = np.load(os.path.join(GOLD, f"sqp_N{N}.npz"))
        s = OSQPSolverRef(N=N)
        x = s.setup_and_solve_qp(f["XU_lin"][0], f["xcur"][0], f["goals"][0]).x
        np.testing.assert_allclose(s.Pdata, f["Pdata"][0], rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(s.Adata, f["Adata"][0], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(s.l, f["l"][0], rtol=1e-11, atol=1e-12)
        np.testing.assert_allclose(x, f["qp_sol"][0], rtol=1e-9, atol=1e-10)
    f = np.load(os.path.join(GOLD, "sqp_N16.npz"))
    out = SQPRef(OSQPSolverRef(N=16)).sqp(f["xcur"][0], f["goals"][0], f["XU"][0].copy())
    np.testing.assert_allclose(out, f["sqp_out"][0], rtol=1e-9, atol=1e-10)
    d = np.load(os.path.join(GOLD, "dynamics.npz"))
    for i in range(0, 48, 12):
        dq, dv, Mi, a = rbd.aba_derivatives(d["q"][i], d["v"][i], d["tau"][i])
        np.testing.assert_allclose(dq, d["dq"][i], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(a, d["a"][i], rtol=1e-12, atol=1e-12)


def test_linesearch_first_accept_semantics():
    """alpha is the FIRST accepted candidate in 1, 1/2, ..., 1/128 (src/osqp_sqp.py:58-72)."""
    N = 16
    xcur, goals, XU = synthetic_batch(1, N, seed=4)
    s = OSQPSolverRef(N=N)
    sq = SQPRef(s)
    sol = s.setup_and_solve_qp(XU[0], xcur[0], goals[0]).x
    rec = []
    alpha = sq.linesearch(XU[0], sol, goals[0], rec)
    merits, base = rec[0]["merits"], rec[0]["base"]
    if alpha > 0:
        idx = list(SQPRef.ALPHAS).index(alpha)
        assert merits[idx] <= base and all(m > base for m in merits[:idx])
    else:
        assert len(merits) == 8 and all(m > base for m in merits)


@pytest.mark.parametrize("N", [16, 32, 64])
def test_cpp_port_matches_numpy_oracle(N):
    """oracle/cpp (the bench's CPU baseline + flop counter) == the numpy restatement."""
    from oracle import cpu

    f = np.load(os.path.join(GOLD, f"sqp_N{N}.npz"))
    out, qp, al, st = cpu.solve(f["xcur"], f["goals"], f["XU"], N, nthreads=2)
    for b in range(out.shape[0]):
        assert np.linalg.norm(out[b] - f["sqp_out"][b]) <= 1e-9 * np.linalg.norm(f["sqp_out"][b])
        assert qp[b] == f["qp_iters"][b]
        np.testing.assert_array_equal(al[b][~np.isnan(al[b])], f["alphas"][b][~np.isnan(f["alphas"][b])])
    fl = cpu.count_flops(f["xcur"][0], f["goals"][0], f["XU"][0], N)
    assert fl["linearize"] > 0 and fl["qp"] > 0 and fl["iters"] == f["qp_iters"][0]
