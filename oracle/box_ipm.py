"""ORACLE (test infrastructure only) — box-constrained QP mode.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

The reference QP (src/osqp_solver.py:137-143) has equality rows only (l == u).  Config 4
adds box rows on every decision variable after the fixed initial state:

    q_lower <= q_k <= q_upper, |v_k| <= v_limit, |u_k| <= effort_limit
    (description/indy7.urdf:203-238 <limit lower upper velocity effort>)

The reference has no semantics for these rows (SURVEY.md §8f-3 "define and test it via KKT
certificate"), so the mode is defined here as: the exact optimum of the box-constrained QP,
to a tolerance, computed by a primal-dual interior-point method (Mehrotra predictor-corrector)
whose Newton systems keep the dynamics rows exact.  This file is the restatement the GPU
path (k_ipm_* + k_riccati_mfma<BOX>) follows step by step:

  init      x = clip(x_eq, lo + theta (hi - lo), hi - theta (hi - lo)) on bounded variables,
            x_eq = the equality-only QP solution; z_l = z0 / s_l, z_u = z0 / s_u (a centred
            start: every complementarity product equals z0, so mu_0 = z0).  theta = 0.2 and
            z0 = 0.1 take 6.9 iterations per config-4 QP against 12.2 for theta = 0.01, z = 1
            (oracle/studies/ipm_iters.py).
  iterate   Sigma = z_l / s_l + z_u / s_u        (s_l = x - lo, s_u = hi - x)
            each Newton step is the equality-constrained QP
                min 1/2 y'(P + Sigma) y + l'y   s.t.  A y = b
            whose minimiser is y = x + dx, with
                l = g - z_l + z_u + r_l / s_l - r_u / s_u - Sigma x
            (r_l = s_l z_l - tau_l, r_u = s_u z_u - tau_u; predictor tau = 0 -> l = g - Sigma x).
            The equality multipliers never appear: dx does not depend on them.
  step      one common step alpha = min(1, eta * max feasible) for primal and dual, so the
            primal (A x - b) and dual residuals both shrink by exactly (1 - alpha).
  stop      mu < tol and prod(1 - alpha) < tol (both residuals are below tol times their
            initial values), or max_iters.

The KKT certificate (``kkt_certificate``) is independent of the iteration: it recovers the
equality multipliers by least squares and reports stationarity, complementarity, primal
feasibility and bound violation.  ADMM was measured first and rejected for this QP: with
R = 1e-5 on u the problem is very flat, and OSQP-style ADMM needed 40-2000+ iterations per
QP to reach 1e-3 residuals.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
from scipy.sparse import bmat, diags, csc_matrix
from scipy.sparse.linalg import splu, lsqr

MASK_Q, MASK_V, MASK_U = 1, 2, 4


def box_bounds(P, N: int, mask: int = MASK_Q | MASK_V | MASK_U):
    """(lo, hi, bm) over the trajectory vector [q v u]_0 ... [q v]_{N-1}; bm marks bounded
    entries.  The initial state (fixed by the equality rows) is never bounded."""
    T = 18 * N - 6
    lo = np.concatenate([np.concatenate([P.q_lower, -P.v_limit, -P.effort_limit])] * N)[:T]
    hi = np.concatenate([np.concatenate([P.q_upper, P.v_limit, P.effort_limit])] * N)[:T]
    cls = np.concatenate([np.repeat([MASK_Q, MASK_V, MASK_U], 6)] * N)[:T]
    bm = (cls & mask) != 0
    bm[:12] = False
    lo = np.where(bm, lo, -np.inf)
    hi = np.where(bm, hi, np.inf)
    return lo, hi, bm


@dataclass
class IPMResult:
    x: np.ndarray
    zl: np.ndarray
    zu: np.ndarray
    iters: int
    converged: bool
    mu: list = field(default_factory=list)
    alpha: list = field(default_factory=list)
    mua: list = field(default_factory=list)  # per iteration: (expanded mu_aff, direct product sum, mu)


def _ratio(v, dv, bm):
    """max t in (0, 1] with v + t dv >= 0 on bm (v > 0)."""
    neg = bm & (dv < 0)
    if not neg.any():
        return 1.0
    return float(min(1.0, np.min(-v[neg] / dv[neg])))


def ipm_box(Pf, g, A, b, x_eq, lo, hi, bm, tol=1e-8, max_iters=30, theta=0.2, eta=0.99, z0=0.1) -> IPMResult:
    """Mehrotra predictor-corrector on the box-constrained QP (module docstring)."""
    n = len(g)
    nb = int(bm.sum())
    x = x_eq.copy()
    if nb == 0:
        return IPMResult(x, np.zeros(n), np.zeros(n), 0, True)
    w = np.where(bm, hi - lo, 0.0)
    x[bm] = np.clip(x_eq[bm], (lo + theta * w)[bm], (hi - theta * w)[bm])
    # (every term divides by the slacks through their reciprocals, formed once per pass — as the
    # GPU's i7m_box.h and the C++ port do)
    zl = np.where(bm, z0 * (1.0 / np.where(bm, x - lo, 1.0)), 0.0)
    zu = np.where(bm, z0 * (1.0 / np.where(bm, hi - x, 1.0)), 0.0)
    K0 = bmat([[Pf, A.T], [A, None]], format="csc")
    res = IPMResult(x, zl, zu, 0, False)
    rfrac = 1.0
    it = 0
    for it in range(max_iters):
        sl = np.where(bm, x - lo, 1.0)
        su = np.where(bm, hi - x, 1.0)
        mu = float((sl[bm] @ zl[bm] + su[bm] @ zu[bm]) / (2 * nb))
        res.mu.append(mu)
        if mu < tol and rfrac < tol:
            res.converged = True
            break
        isl, isu = 1.0 / sl, 1.0 / su
        sig = np.where(bm, zl * isl + zu * isu, 0.0)
        K = (K0 + bmat([[diags(sig), None], [None, csc_matrix((A.shape[0], A.shape[0]))]])).tocsc()
        lu = splu(K)

        def newton(ell):
            return lu.solve(np.concatenate([-ell, b]))[:n] - x

        # predictor (tau = 0)
        dxa = newton(g - sig * x)
        dzla = np.where(bm, -zl - zl * dxa * isl, 0.0)
        dzua = np.where(bm, -zu + zu * dxa * isu, 0.0)
        ap = min(_ratio(sl, dxa, bm), _ratio(su, -dxa, bm))
        ad = min(_ratio(zl, dzla, bm), _ratio(zu, dzua, bm))
        # the complementarity after the affine step is bilinear in (ap, ad): four sums
        # (i7m_box.h ipm_pred_body forms it the same way, in the pass that finds ap, ad)
        s00 = float(np.sum((sl * zl + su * zu)[bm]))
        s01 = float(np.sum((sl * dzla + su * dzua)[bm]))
        s10 = float(np.sum((dxa * zl - dxa * zu)[bm]))
        s11 = float(np.sum((dxa * dzla - dxa * dzua)[bm]))
        mua = ((s00 + ad * s01) + ap * (s10 + ad * s11)) / (2 * nb)
        # the direct product sum, independent of the expansion (tests/test_box_oracle.py pins the
        # two together); near convergence s00 ~ 2 nb mu cancels against the other terms, so the
        # expanded form is clamped at 0 (a negative sigma mu would push away from the centre)
        mua_direct = float(np.sum(((sl + ap * dxa) * (zl + ad * dzla) + (su - ap * dxa) * (zu + ad * dzua))[bm])) / (2 * nb)
        res.mua.append((mua, mua_direct, mu))
        mua = max(mua, 0.0)
        smu = (mua / mu) ** 3 * mu
        # corrector
        rl = np.where(bm, sl * zl + dxa * dzla - smu, 0.0)
        ru = np.where(bm, su * zu - dxa * dzua - smu, 0.0)
        ell = g - zl + zu + np.where(bm, rl * isl - ru * isu, 0.0) - sig * x
        dx = newton(ell)
        dzl = np.where(bm, (-rl - zl * dx) * isl, 0.0)
        dzu = np.where(bm, (-ru + zu * dx) * isu, 0.0)
        a = min(_ratio(sl, dx, bm), _ratio(su, -dx, bm), _ratio(zl, dzl, bm), _ratio(zu, dzu, bm))
        a = min(1.0, eta * a)
        res.alpha.append(a)
        x = x + a * dx
        zl = zl + a * dzl
        zu = zu + a * dzu
        rfrac *= 1.0 - a
    else:
        it = max_iters
    res.x, res.zl, res.zu, res.iters = x, zl, zu, it
    return res


def kkt_certificate(Pf, g, A, b, x, zl, zu, lo, hi, bm) -> dict:
    """Optimality residuals of x for the box QP; equality multipliers by least squares."""
    r0 = Pf @ x + g - zl + zu
    lam = lsqr(A.T, -r0, atol=1e-15, btol=1e-15, iter_lim=20000)[0]
    stat = r0 + A.T @ lam
    sl = np.where(bm, x - lo, 0.0)
    su = np.where(bm, hi - x, 0.0)
    return {
        "stationarity": float(np.abs(stat).max()),
        "complementarity": float(max(np.abs(sl * zl).max(), np.abs(su * zu).max())),
        "primal_eq": float(np.abs(A @ x - b).max()),
        "bound_violation": float(max(0.0, (lo - x)[bm].max(initial=0.0), (x - hi)[bm].max(initial=0.0))),
        "dual_sign": float(max(0.0, -zl.min(), -zu.min())),
        "scale": float(max(1.0, np.abs(g).max(), np.abs(Pf @ x).max())),
    }
