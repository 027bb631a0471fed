"""The Riccati recursion on an ill-conditioned H: k_riccati_mfma's QP
solution and its cost-to-go V~_0 (i7m_qp_value) against the sparse-LU KKT of the same QP.

The fp64 MFMA recursion is accurate only because it stays on ONE matrix: the 16x16 products take
V~'s accumulators as their A operand, i.e. use V~' throughout, and V~ = Qxx + K~'G~ is symmetric
only to the accuracy of K~ = -H^-1 G~.  H = Bu' V_vv Bu + R with R = 1e-5 w (src/osqp_solver.py:
103-135) is ill-conditioned; reading V~_vv un-transposed for H (one 6x6 block) gave 1e-4 errors at
N = 64.  This test makes H worse still (R_cost 1e-8, QN_cost 1e4, besides the
reference's 1e-5 / 100) and pins, at N = 32 and N = 64 (the largest horizon the library takes):

  QP minimiser vs sparse-LU KKT                 : 1e-8 relative (SURVEY.md 8d's per-QP gate)
  V~_0's 12x12 block vs d y_0 / d xs            : 1e-8 relative (y_0: the KKT multipliers of the
      x_0 rows l[:12] = -xs, src/osqp_solver.py:85; dJ*/dxs = y_0, so d2J*/dxs2 = dy_0/dxs, a
      12-column solve with the same LU; checked against finite differences in the oracle tests)
  V~_0's linear column vs y_0 - Vxx xs          : 1e-8 relative
  asymmetry of the 12x12 block, relative          : <= 1e-10 (V~ is symmetric in exact arithmetic;
      the recursion keeps it to ~1e-13 on these problems, measured; the constant V~[12][12] is not
      formed, I7M_RIC_44X)

A build that forms H from V~_vv instead of V~_vv' (-DI7M_RIC_VV_PLAIN=1) fails the first two
gates (profiles/r04_vv_plain_variant.log).
"""
import numpy as np
import pytest
from scipy.sparse import bmat, diags
from scipy.sparse.linalg import splu

from oracle.osqp_ref import OSQPSolverRef, synthetic_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from indy7_mpc_amd import _lib
    _lib.load()
    if _lib.device_count() < 1:
        pytest.fail("no GPU visible but the gpu tests were requested")
    return _lib


def kkt_reference(s, xu, xs, goals):
    """Exact minimiser, y_0 and Vxx = d y_0 / d xs of the QP the oracle builds at xu."""
    s.setup_and_solve_qp(xu, xs, goals)
    P, A = s.matrices()
    Pf = (P + P.T - diags(P.diagonal())).tocsc()
    K = bmat([[Pf, A.T], [A, None]], format="csc")
    n = Pf.shape[0]
    lu = splu(K)
    z = lu.solve(np.concatenate([-s.g, s.l]))
    rhs = np.zeros((K.shape[0], 12))
    rhs[n:n + 12, :] = -np.eye(12)
    Vxx = lu.solve(rhs)[n:n + 12, :]
    return z[:n], z[n:n + 12], Vxx


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("N", [32, 64])
@pytest.mark.parametrize("R_cost,QN_cost", [(1e-5, 100.0), (1e-8, 1e4)])
def test_riccati_ill_conditioned_matches_kkt(lib, model, N, R_cost, QN_cost):
    B = 4
    xcur, goals, XU = synthetic_batch(B, N, seed=61)
    # a second linearisation point away from the trivial start: a quarter step to the minimiser
    s = OSQPSolverRef(N=N, R_cost=R_cost, QN_cost=QN_cost)
    XU[2:] += 0.25 * (np.stack([s.setup_and_solve_qp(XU[b], xcur[b], goals[b]).x for b in range(2, B)]) - XU[2:])
    h = lib.Handle(model, N=N, max_batch=B, R_cost=R_cost, QN_cost=QN_cost)
    sol = h.qp(XU, xcur, goals)
    V0 = h.qp_value(XU, xcur, goals)
    for b in range(B):
        x, y0, Vxx = kkt_reference(s, XU[b], xcur[b], goals[b])
        assert _rel(sol[b], x) <= 1e-8, (b, _rel(sol[b], x))
        V = V0[b]
        assert _rel(V[:12, :12], Vxx) <= 1e-8, (b, _rel(V[:12, :12], Vxx))
        assert _rel(V[:12, 12], y0 - Vxx @ xcur[b]) <= 1e-8, (b, _rel(V[:12, 12], y0 - Vxx @ xcur[b]))
        asym = np.abs(V[:12, :12] - V[:12, :12].T).max() / np.abs(V[:12, :12]).max()
        assert asym <= 1e-10, (b, asym)
