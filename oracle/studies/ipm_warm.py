"""STUDY (test infrastructure, not shipped): warm-starting the second SQP iteration's box QP
(config 4, oracle/box_ipm.py) from the first QP's solution.

Each config-4 solve hands the interior point two QPs: the linearisation at XU, then at
XU + alpha (sol_1 - XU).  The second QP's optimum is close to the first's, so its interior point
could start there instead of at the centred cold start (x = clip(x_eq) with a 20 % margin,
z = 0.1 / s).  This script captures the (QP1 solution, QP2) pairs of the SQP oracle on config-4
draws and re-solves QP2 from several warm starts, reporting iterations and the KKT certificate.

Warm start "x1, mu_t, theta_w": x = x1 (QP1's box solution) clipped into the box with margin
theta_w of the width; z_l = max(z1_l, mu_t / s_l), z_u likewise (QP1's duals, pushed so every
complementarity product is >= mu_t); or z centred at mu_t ("centred").  Both stopping rules are
reported: the shipping one (mu < tol and prod(1 - alpha) < tol: the equality residual shrank by
tol from the start) and an absolute one on the measured residual.

    python -m oracle.studies.ipm_warm [--problems 12] [--N 64]
"""
from __future__ import annotations

import argparse

import numpy as np
from scipy.sparse import bmat, diags, csc_matrix
from scipy.sparse.linalg import splu

from oracle import box_ipm
from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch


def ipm_from(Pf, g, A, b, x, zl, zu, lo, hi, bm, tol=1e-8, max_iters=40, eta=0.99, rule="rfrac", res0=None):
    """box_ipm.ipm_box's iteration from a given interior (x, zl, zu).  rule "rfrac": the shipping
    stop (mu < tol and prod(1 - alpha) < tol); "abs": mu < tol and |A x - b|_inf <= tol (1 + |b|_inf)."""
    n = len(g)
    nb = int(bm.sum())
    K0 = bmat([[Pf, A.T], [A, None]], format="csc")
    rfrac = 1.0
    it = 0
    conv = False
    scale_b = 1.0 + np.abs(b).max()
    for it in range(max_iters):
        sl = np.where(bm, x - lo, 1.0)
        su = np.where(bm, hi - x, 1.0)
        mu = float((sl[bm] @ zl[bm] + su[bm] @ zu[bm]) / (2 * nb))
        if rule == "rfrac":
            ok = rfrac < tol
        else:
            ok = np.abs(A @ x - b).max() <= tol * scale_b
        if mu < tol and ok:
            conv = True
            break
        sig = np.where(bm, zl / sl + zu / su, 0.0)
        K = (K0 + bmat([[diags(sig), None], [None, csc_matrix((A.shape[0], A.shape[0]))]])).tocsc()
        lu = splu(K)

        def newton(ell):
            return lu.solve(np.concatenate([-ell, b]))[:n] - x

        dxa = newton(g - sig * x)
        dzla = np.where(bm, -zl - zl * dxa / sl, 0.0)
        dzua = np.where(bm, -zu + zu * dxa / su, 0.0)
        ap = min(box_ipm._ratio(sl, dxa, bm), box_ipm._ratio(su, -dxa, bm))
        ad = min(box_ipm._ratio(zl, dzla, bm), box_ipm._ratio(zu, dzua, bm))
        mua = max(0.0, float(((sl + ap * dxa)[bm] @ (zl + ad * dzla)[bm] + (su - ap * dxa)[bm] @ (zu + ad * dzua)[bm]) / (2 * nb)))
        smu = (mua / mu) ** 3 * mu
        rl = np.where(bm, sl * zl + dxa * dzla - smu, 0.0)
        ru = np.where(bm, su * zu - dxa * dzua - smu, 0.0)
        ell = g - zl + zu + np.where(bm, rl / sl - ru / su, 0.0) - sig * x
        dx = newton(ell)
        dzl = np.where(bm, (-rl - zl * dx) / sl, 0.0)
        dzu = np.where(bm, (-ru + zu * dx) / su, 0.0)
        a = min(box_ipm._ratio(sl, dx, bm), box_ipm._ratio(su, -dx, bm), box_ipm._ratio(zl, dzl, bm),
                box_ipm._ratio(zu, dzu, bm))
        a = min(1.0, eta * a)
        x = x + a * dx
        zl = zl + a * dzl
        zu = zu + a * dzu
        rfrac *= 1.0 - a
    else:
        it = max_iters
    return x, zl, zu, it, conv


def cold(x_eq, lo, hi, bm, theta=0.2, z0=0.1):
    w = np.where(bm, hi - lo, 0.0)
    x = x_eq.copy()
    x[bm] = np.clip(x_eq[bm], (lo + theta * w)[bm], (hi - theta * w)[bm])
    zl = np.where(bm, z0 / np.where(bm, x - lo, 1.0), 0.0)
    zu = np.where(bm, z0 / np.where(bm, hi - x, 1.0), 0.0)
    return x, zl, zu


def warm(x1, zl1, zu1, lo, hi, bm, mu_t, theta_w, centred):
    w = np.where(bm, hi - lo, 0.0)
    x = x1.copy()
    x[bm] = np.clip(x1[bm], (lo + theta_w * w)[bm], (hi - theta_w * w)[bm])
    sl = np.where(bm, x - lo, 1.0)
    su = np.where(bm, hi - x, 1.0)
    if centred:
        zl = np.where(bm, mu_t / sl, 0.0)
        zu = np.where(bm, mu_t / su, 0.0)
    else:
        zl = np.where(bm, np.maximum(zl1, mu_t / sl), 0.0)
        zu = np.where(bm, np.maximum(zu1, mu_t / su), 0.0)
    return x, zl, zu


def capture(nprob: int, N: int, seed: int):
    """Per solve of the SQP oracle on config-4 draws: the box QPs in order, each with its
    solution (x, z_l, z_u)."""
    xcur, goals, XU = synthetic_batch(nprob, N, seed)
    s = OSQPSolverRef(N=N, qp="box")
    solves = []
    orig = box_ipm.ipm_box

    def grab(Pf, g, A, b, x_eq, lo, hi, bm, **kw):
        r = orig(Pf, g, A, b, x_eq, lo, hi, bm, **kw)
        solves[-1].append(((Pf, g.copy(), A, b.copy(), x_eq.copy(), lo, hi, bm), r))
        return r

    box_ipm.ipm_box = grab
    try:
        sq = SQPRef(s)
        for i in range(nprob):
            solves.append([])
            sq.sqp(xcur[i], goals[i], XU[i].copy())
    finally:
        box_ipm.ipm_box = orig
    return solves


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=12)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--seed", type=int, default=46)
    a = ap.parse_args()
    solves = capture(a.problems, a.N, a.seed)
    pairs = [(s[0][1], s[1][0]) for s in solves if len(s) >= 2]
    print(f"{len(pairs)} (QP1 solution, QP2) pairs, N = {a.N}")
    variants = [("cold (shipping)", None)]
    for centred in (False, True):
        for mu_t in (1e-2, 1e-3, 1e-4):
            for theta_w in (1e-3, 1e-2, 0.05):
                variants.append((f"warm {'centred' if centred else 'z1 pushed'} mu_t {mu_t:.0e} theta_w {theta_w:g}",
                                 (mu_t, theta_w, centred)))
    for rule in ("rfrac", "abs"):
        for name, v in variants:
            its, worst, comp = [], 0.0, 0.0
            for r1, (Pf, g, A, b, x_eq, lo, hi, bm) in pairs:
                x0 = cold(x_eq, lo, hi, bm) if v is None else warm(r1.x, r1.zl, r1.zu, lo, hi, bm, *v)
                x, zl, zu, it, conv = ipm_from(Pf, g, A, b, *x0, lo, hi, bm, rule=rule)
                its.append(it if conv else 99)
                c = box_ipm.kkt_certificate(Pf, g, A, b, x, zl, zu, lo, hi, bm)
                worst = max(worst, c["stationarity"] / c["scale"])
                comp = max(comp, c["complementarity"])
            its = np.array(its)
            print(f"[{rule:5s}] {name:46s} QP2 iters mean {its.mean():5.2f} max {its.max():3d}  "
                  f"stat/scale {worst:.1e}  compl {comp:.1e}", flush=True)
    q1 = np.array([s[0][1].iters for s in solves])
    print(f"QP1 (cold) iters mean {q1.mean():.2f}")


if __name__ == "__main__":
    main()
