"""Probe behind DESIGN.md §4.4 (not a test; run by hand): iterations OSQP-style ADMM needs on
the config-4 box QP versus the interior point, on oracle QPs (test infrastructure only).

    python tests/probes/box_admm_vs_ipm.py admm N RHO [scalar|class]
    python tests/probes/box_admm_vs_ipm.py ipm N
"""
import sys


def admm_main():
    import numpy as np, time
    from scipy.sparse import bmat, diags, csc_matrix, identity
    from scipy.sparse.linalg import splu
    sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))))
    from oracle import osqp_ref, rbd
    P_ = rbd.params()
    N = int(sys.argv[2]); rho = float(sys.argv[3]); mode = sys.argv[4] if len(sys.argv) > 4 else "scalar"
    B = 8
    xcur, goals, XU = osqp_ref.synthetic_batch(B, N, 46)
    s = osqp_ref.OSQPSolverRef(N=N)
    T = s.traj_len
    blk = np.concatenate([P_.q_upper, P_.v_limit, P_.effort_limit])
    hi = np.concatenate([blk] * N)[:T]; lo = np.concatenate([np.concatenate([P_.q_lower, -P_.v_limit, -P_.effort_limit])] * N)[:T]
    sigma, alpha = 1e-6, 1.6
    def admm(Pf, g, A, l, rhov, x0, iters=20000, eps=1e-3, every=5):
        n = len(g); m = A.shape[0]
        K = bmat([[Pf + diags(sigma + rhov), A.T], [A, None]], format="csc")
        lu = splu(K)
        x = x0.copy(); z = np.clip(x, lo, hi); y = np.zeros(n)
        for it in range(1, iters + 1):
            rhs = np.concatenate([sigma * x - g + rhov * z - y, l])
            xt = lu.solve(rhs)[:n]
            xr = alpha * xt + (1 - alpha) * z
            x = alpha * xt + (1 - alpha) * x
            zn = np.clip(xr + y / rhov, lo, hi)
            y = y + rhov * (xr - zn)
            dz = zn - z; z = zn
            if it % every == 0:
                rp = np.abs(x - z).max(); rd = np.abs(rhov * dz).max()
                ep = eps + eps * max(np.abs(x).max(), np.abs(z).max())
                ed = eps + eps * np.abs(y).max()
                if rp < ep and rd < ed: return x, z, y, it
        return x, z, y, iters
    its = []
    for b in range(B):
        Xb = XU[b].copy()
        sol_eq = s.setup_and_solve_qp(Xb, xcur[b], goals[b]).x
        Pm, A = s.matrices(); Pf = (Pm + Pm.T - diags(Pm.diagonal())).tocsc()
        if mode == "scalar": rhov = np.full(T, rho)
        else:  # per-class: scale by the cost diagonal magnitude
            d = np.abs(Pf.diagonal()); rhov = rho * np.maximum(d, 1e-3)
        x, z, y, it = admm(Pf, s.g, A, s.l, rhov, sol_eq)
        xx, zz, yy, it2 = admm(Pf, s.g, A, s.l, rhov, sol_eq, eps=1e-9)
        print(b, "iters(1e-3)", it, "iters(1e-9)", it2, "dist %.3g" % (np.abs(x - xx).max()), "viol %.3g" % np.abs(zz - xx).max(), "active", int((np.abs(yy) > 1e-9).sum()))
        its.append(it)
    print("mean", np.mean(its))


def ipm_main():
    import numpy as np
    from scipy.sparse import bmat, diags
    from scipy.sparse.linalg import splu
    sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))))
    from oracle import osqp_ref, rbd
    P_ = rbd.params()
    N = int(sys.argv[2]); B = 8
    xcur, goals, XU = osqp_ref.synthetic_batch(B, N, 46)
    s = osqp_ref.OSQPSolverRef(N=N)
    T = s.traj_len
    hi = np.concatenate([np.concatenate([P_.q_upper, P_.v_limit, P_.effort_limit])] * N)[:T]
    lo = np.concatenate([np.concatenate([P_.q_lower, -P_.v_limit, -P_.effort_limit])] * N)[:T]
    bm = np.ones(T, bool); bm[:12] = False  # knot-0 state fixed by the equality
    def ipm(Pf, g, A, b, x0, tol=1e-8, maxit=60):
        n = len(g); m = A.shape[0]
        x = np.clip(x0, lo + 1e-2 * (hi - lo), hi - 1e-2 * (hi - lo)); x[~bm] = x0[~bm]
        sl = np.where(bm, x - lo, 1.0); su = np.where(bm, hi - x, 1.0)
        zl = np.where(bm, 1.0, 0.0); zu = np.where(bm, 1.0, 0.0); lam = np.zeros(m)
        nb = bm.sum()
        for it in range(maxit):
            rd = Pf @ x + g + A.T @ lam - zl + zu
            rp = A @ x - b
            mu = (sl[bm] @ zl[bm] + su[bm] @ zu[bm]) / (2 * nb)
            if np.abs(rd).max() < tol * (1 + np.abs(g).max()) and np.abs(rp).max() < tol * (1 + np.abs(b).max()) and mu < tol:
                return x, it
            Sig = np.where(bm, zl / sl + zu / su, 0.0)
            lu = splu(bmat([[Pf + diags(Sig), A.T], [A, None]], format="csc"))
            def solve(rl, ru):  # complementarity residuals rl = sl*zl - target, ru likewise
                # dz_l = -(rl + zl*dx)/sl ; dz_u = -(ru - zu*dx)/su
                rhs1 = -rd - np.where(bm, rl / sl, 0) + np.where(bm, ru / su, 0)
                sol = lu.solve(np.concatenate([rhs1, -rp]))
                dx, dl = sol[:n], sol[n:]
                dzl = np.where(bm, -(rl + zl * dx) / sl, 0); dzu = np.where(bm, -(ru - zu * dx) / su, 0)
                return dx, dl, dzl, dzu
            def step(v, dv):
                neg = (dv < 0) & bm
                return min(1.0, (-v[neg] / dv[neg]).min()) if neg.any() else 1.0
            dx, dl, dzl, dzu = solve(sl * zl, su * zu)
            ap = min(step(sl, dx), step(su, -dx)); ad = min(step(zl, dzl), step(zu, dzu))
            mua = ((sl + ap * dx)[bm] @ (zl + ad * dzl)[bm] + (su - ap * dx)[bm] @ (zu + ad * dzu)[bm]) / (2 * nb)
            sgm = (mua / mu) ** 3
            dx, dl, dzl, dzu = solve(sl * zl + dx * dzl - sgm * mu, su * zu - dx * dzu - sgm * mu)
            ap = 0.99 * min(step(sl, dx), step(su, -dx)); ad = 0.99 * min(step(zl, dzl), step(zu, dzu))
            x = x + ap * dx; sl = np.where(bm, x - lo, 1.0); su = np.where(bm, hi - x, 1.0)
            lam = lam + ad * dl; zl = zl + ad * dzl; zu = zu + ad * dzu
        return x, maxit
    for b in range(B):
        sol_eq = s.setup_and_solve_qp(XU[b].copy(), xcur[b], goals[b]).x
        Pm, A = s.matrices(); Pf = (Pm + Pm.T - diags(Pm.diagonal())).tocsc()
        x, it = ipm(Pf, s.g, A, s.l, sol_eq)
        print(b, "iters", it, "obj", 0.5 * x @ (Pf @ x) + s.g @ x, "eq", np.abs(A @ x - s.l).max(), "box", max((x - hi)[bm].max(), (lo - x)[bm].max()))


if __name__ == "__main__":
    admm_main() if sys.argv[1] == "admm" else ipm_main()
