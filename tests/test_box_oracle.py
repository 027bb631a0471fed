"""Config 4: the box-constrained QP mode's oracle (oracle/box_ipm.py).

The reference has no box rows, so this mode is pinned by its KKT certificate rather than by
reference outputs ("parity unpinned" against the reference): stationarity with
least-squares equality multipliers, complementarity, primal feasibility, bound satisfaction
and dual signs, each to a stated tolerance.
"""
import numpy as np
import pytest
from scipy.sparse import diags

from oracle import box_ipm, rbd
from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch


def _qp(s, xu, xc, g):
    s.setup_and_solve_qp(xu, xc, g)
    P, A = s.matrices()
    return (P + P.T - diags(P.diagonal())).tocsc(), A


def test_box_bounds_layout():
    P = rbd.params()
    lo, hi, bm = box_ipm.box_bounds(P, 3)
    assert lo.shape == (48,) and not bm[:12].any() and bm[12:].all()
    np.testing.assert_array_equal(hi[12:18], P.effort_limit)
    np.testing.assert_array_equal(lo[18:24], P.q_lower)
    np.testing.assert_array_equal(hi[24:30], P.v_limit)
    _, _, bq = box_ipm.box_bounds(P, 3, box_ipm.MASK_U)
    assert bq.sum() == 12 and bq[12:18].all() and bq[30:36].all()


def test_box_ipm_kkt_certificate():
    N = 16
    xcur, goals, XU = synthetic_batch(3, N, 46)
    s = OSQPSolverRef(N=N, qp="box")
    lo, hi, bm = box_ipm.box_bounds(s.P_, N)
    n_active = 0
    for b in range(3):
        r = s.setup_and_solve_qp(XU[b], xcur[b], goals[b])
        ipm = s.last_ipm
        assert ipm.converged and ipm.iters <= 30
        Pf, A = _qp(s, XU[b], xcur[b], goals[b])
        c = box_ipm.kkt_certificate(Pf, s.g, A, s.l, r.x, ipm.zl, ipm.zu, lo, hi, bm)
        assert c["stationarity"] <= 1e-7 * c["scale"], c
        assert c["complementarity"] <= 1e-5, c
        assert c["primal_eq"] <= 1e-9 * max(1.0, np.abs(r.x).max()), c
        assert c["bound_violation"] == 0.0 and c["dual_sign"] == 0.0, c
        n_active += int(((r.x - lo)[bm] < 1e-4).sum() + ((hi - r.x)[bm] < 1e-4).sum())
    assert n_active > 0  # the fixture really exercises the box rows


def test_box_without_rows_is_the_exact_qp():
    N = 16
    xcur, goals, XU = synthetic_batch(1, N, 46)
    ex = OSQPSolverRef(N=N).setup_and_solve_qp(XU[0], xcur[0], goals[0]).x
    bx = OSQPSolverRef(N=N, qp="box", box_mask=0).setup_and_solve_qp(XU[0], xcur[0], goals[0]).x
    np.testing.assert_array_equal(ex, bx)


def test_box_sqp_keeps_the_box():
    N = 16
    xcur, goals, XU = synthetic_batch(2, N, 46)
    s = OSQPSolverRef(N=N, qp="box")
    lo, hi, bm = box_ipm.box_bounds(s.P_, N)
    sq = SQPRef(s)
    for b in range(2):
        out = sq.sqp(xcur[b], goals[b], XU[b].copy())
        assert (out[bm] >= lo[bm]).all() and (out[bm] <= hi[bm]).all()


def test_mu_aff_expansion_matches_direct_product_sum():
    """The predictor's mu_aff is formed from four sums of one pass (bilinear in the two step
    lengths; i7m_box.h ipm_pred_body does the same).  Pinned here against the direct product sum
    sum((s_l + ap dx)(z_l + ad dz_l) + (s_u - ap dx)(z_u + ad dz_u)) / 2nb, which the oracle keeps
    for exactly this check: the two agree to rounding of mu, every iteration."""
    for N in (16, 32):
        xcur, goals, XU = synthetic_batch(3, N, 46)
        s = OSQPSolverRef(N=N, qp="box")
        n = 0
        for b in range(3):
            s.setup_and_solve_qp(XU[b], xcur[b], goals[b])
            for mua, direct, mu in s.last_ipm.mua:
                assert abs(mua - direct) <= 1e-10 * mu, (N, b, mua, direct, mu)
                assert direct >= -1e-10 * mu
                n += 1
        assert n > 10


@pytest.mark.parametrize("N", [16, 32])
def test_cpp_port_box_mode_matches_numpy_oracle(N):
    """oracle/cpp's config-4 mode (the CPU baseline and the bench-scale parity reference of the
    box QP) against the numpy oracle: every SQP iteration's interior-point iteration count and
    convergence, the alpha sequence, and XU to 1e-5 relative (the GPU box test's tolerance; the
    two Newton solves differ by Riccati vs sparse LU rounding, amplified by Sigma ~ z/s)."""
    from oracle import cpu

    B = 4
    xcur, goals, XU = synthetic_batch(B, N, 46)
    out, qp, al, _, it, conv, mu = cpu.solve_box(xcur, goals, XU, N, nthreads=2)
    s = OSQPSolverRef(N=N, qp="box")
    for b in range(B):
        its = []
        orig = s.setup_and_solve_qp

        def rec(*a):
            r = orig(*a)
            its.append((s.last_ipm.iters, s.last_ipm.converged))
            return r

        s.setup_and_solve_qp = rec
        sq = SQPRef(s)
        ref = sq.sqp(xcur[b], goals[b], XU[b].copy())
        s.setup_and_solve_qp = orig
        assert qp[b] == len(its)
        assert list(it[b][: qp[b]]) == [i for i, _ in its], (b, it[b], its)
        assert conv[b] == its[-1][1]
        np.testing.assert_array_equal(al[b][: qp[b]], sq.stats["linesearch_alphas"]["values"])
        assert np.abs(out[b] - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    fl = cpu.count_flops(xcur[0], goals[0], XU[0], N, box=cpu.box_cfg())
    assert fl["ipm"] > fl["linearize"] and fl["ipm_iters"] == it[0][: qp[0]].sum()
