"""STUDY (test infrastructure, not shipped): interior-point iteration counts of the config-4 box
QP (oracle/box_ipm.py) under variants of its starting point and step rule.

k_ipm_fused is bound by the bytes each Newton step streams, so its time per QP
is proportional to the iteration count.  This script captures the QPs the SQP oracle hands the
box solver on config-4 draws (N = 64, seed 48 like bench.py's config 4) and re-solves each one
with every variant, reporting iterations and the KKT certificate of the result.

    python -m oracle.studies.ipm_iters [--problems 16] [--N 64]
"""
from __future__ import annotations

import argparse

import numpy as np
from scipy.sparse import bmat, diags, csc_matrix
from scipy.sparse.linalg import splu

from oracle import box_ipm
from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch


def ipm_variant(Pf, g, A, b, x_eq, lo, hi, bm, tol=1e-8, max_iters=30, theta=0.01, eta=0.99,
                zinit="one", eta_rule="const", second_order=True, sigma_pow=3.0):
    """box_ipm.ipm_box with knobs: zinit 'one' (z = 1) or 'mu' (z = mu0 / s, centred start);
    eta_rule 'const' or 'adapt' (eta = max(eta, 1 - mu))."""
    n = len(g)
    nb = int(bm.sum())
    x = x_eq.copy()
    w = np.where(bm, hi - lo, 0.0)
    x[bm] = np.clip(x_eq[bm], (lo + theta * w)[bm], (hi - theta * w)[bm])
    sl = np.where(bm, x - lo, 1.0)
    su = np.where(bm, hi - x, 1.0)
    if zinit == "one":
        zl = np.where(bm, 1.0, 0.0)
        zu = np.where(bm, 1.0, 0.0)
    else:
        m0 = float(zinit)
        zl = np.where(bm, m0 / sl, 0.0)
        zu = np.where(bm, m0 / su, 0.0)
    K0 = bmat([[Pf, A.T], [A, None]], format="csc")
    rfrac = 1.0
    it = 0
    conv = False
    for it in range(max_iters):
        sl = np.where(bm, x - lo, 1.0)
        su = np.where(bm, hi - x, 1.0)
        mu = float((sl[bm] @ zl[bm] + su[bm] @ zu[bm]) / (2 * nb))
        if mu < tol and rfrac < tol:
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
        mua = float(((sl + ap * dxa)[bm] @ (zl + ad * dzla)[bm] + (su - ap * dxa)[bm] @ (zu + ad * dzua)[bm]) / (2 * nb))
        smu = (mua / mu) ** sigma_pow * mu
        so = 1.0 if second_order else 0.0
        rl = np.where(bm, sl * zl + so * dxa * dzla - smu, 0.0)
        ru = np.where(bm, su * zu - so * dxa * dzua - smu, 0.0)
        ell = g - zl + zu + np.where(bm, rl / sl - ru / su, 0.0) - sig * x
        dx = newton(ell)
        dzl = np.where(bm, (-rl - zl * dx) / sl, 0.0)
        dzu = np.where(bm, (-ru + zu * dx) / su, 0.0)
        a = min(box_ipm._ratio(sl, dx, bm), box_ipm._ratio(su, -dx, bm), box_ipm._ratio(zl, dzl, bm),
                box_ipm._ratio(zu, dzu, bm))
        e = eta if eta_rule == "const" else max(eta, 1.0 - mu)
        a = min(1.0, e * a)
        x = x + a * dx
        zl = zl + a * dzl
        zu = zu + a * dzu
        rfrac *= 1.0 - a
    else:
        it = max_iters
    return x, zl, zu, it, conv


def capture(nprob: int, N: int, seed: int = 48):
    """The box QPs of the SQP oracle's solves (both SQP iterations) on config-4 draws."""
    xcur, goals, XU = synthetic_batch(nprob, N, seed)
    s = OSQPSolverRef(N=N, qp="box")
    qps = []
    orig = box_ipm.ipm_box

    def grab(Pf, g, A, b, x_eq, lo, hi, bm, **kw):
        qps.append((Pf, g.copy(), A, b.copy(), x_eq.copy(), lo, hi, bm))
        return orig(Pf, g, A, b, x_eq, lo, hi, bm, **kw)

    box_ipm.ipm_box = grab
    try:
        sq = SQPRef(s)
        for i in range(nprob):
            sq.sqp(xcur[i], goals[i], XU[i].copy())
    finally:
        box_ipm.ipm_box = orig
    return qps


VARIANTS = {
    "baseline (theta .01, z = 1, eta .99)": {},
    "eta .995": {"eta": 0.995},
    "eta adaptive max(.99, 1 - mu)": {"eta_rule": "adapt"},
    "theta .05": {"theta": 0.05},
    "theta .1": {"theta": 0.1},
    "z = 1 / s": {"zinit": "1.0"},
    "z = 10 / s": {"zinit": "10.0"},
    "z = 0.1 / s": {"zinit": "0.1"},
    "theta .1, z = 0.1 / s": {"theta": 0.1, "zinit": "0.1"},
    "theta .2, z = 0.1 / s": {"theta": 0.2, "zinit": "0.1"},
    "theta .2, z = 1 / s": {"theta": 0.2, "zinit": "1.0"},
    "theta .3": {"theta": 0.3},
    "theta .2": {"theta": 0.2},
    "theta .1, z = 0.01 / s": {"theta": 0.1, "zinit": "0.01"},
    "theta .2, z = 0.01 / s": {"theta": 0.2, "zinit": "0.01"},
    "theta .2, z = 0.1 / s, eta adapt": {"theta": 0.2, "zinit": "0.1", "eta_rule": "adapt"},
    "n centred, no second-order term": {"theta": 0.2, "zinit": "0.1", "second_order": False},
    "n centred, no second-order term, sigma^2": {"theta": 0.2, "zinit": "0.1", "second_order": False, "sigma_pow": 2.0},
    "n centred, no second-order term, sigma^1": {"theta": 0.2, "zinit": "0.1", "second_order": False, "sigma_pow": 1.0},
    "g theta .15, z = 0.1 / s": {"theta": 0.15, "zinit": "0.1"},
    "g theta .25, z = 0.1 / s": {"theta": 0.25, "zinit": "0.1"},
    "g theta .3, z = 0.1 / s": {"theta": 0.3, "zinit": "0.1"},
    "g theta .5, z = 0.1 / s": {"theta": 0.5, "zinit": "0.1"},
    "g theta .2, z = 0.03 / s": {"theta": 0.2, "zinit": "0.03"},
    "g theta .2, z = 0.3 / s": {"theta": 0.2, "zinit": "0.3"},
    "g theta .3, z = 0.3 / s": {"theta": 0.3, "zinit": "0.3"},
    "g theta .3, z = 0.03 / s": {"theta": 0.3, "zinit": "0.03"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=12)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--seed", type=int, default=48)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    qps = capture(a.problems, a.N, a.seed)
    print(f"{len(qps)} QPs (N = {a.N})")
    sel = a.only.split("|") if a.only else None
    for name, kw in VARIANTS.items():
        if sel and not any(t in name for t in sel):
            continue
        its, worst = [], 0.0
        for (Pf, g, A, b, x_eq, lo, hi, bm) in qps:
            x, zl, zu, it, conv = ipm_variant(Pf, g, A, b, x_eq, lo, hi, bm, **kw)
            its.append(it if conv else 99)
            c = box_ipm.kkt_certificate(Pf, g, A, b, x, zl, zu, lo, hi, bm)
            worst = max(worst, c["stationarity"] / c["scale"])
        its = np.array(its)
        print(f"{name:40s} iters mean {its.mean():5.2f}  max {its.max():3d}  worst stat/scale {worst:.1e}")


if __name__ == "__main__":
    main()
