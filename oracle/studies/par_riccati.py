"""Design study (test infrastructure, not product code): a parallel-in-time Riccati for the
SQP subproblem QP (the equality-constrained QP the reference hands OSQP, src/osqp_solver.py:
137-143), checked against the exact KKT solution of oracle/osqp_ref.py.

* the sequential Riccati recursion (what k_riccati_mfma runs);
* the associative element scan of Sarkka & Garcia-Fernandez (elements (A, b, C, eta, J), a
  Hillis-Steele suffix scan in log2 N combine rounds);
* the chunked variant: W chunks, (1) each chunk's element total, (2) a suffix over the totals
  as value functions, (3) the Riccati recursion inside each chunk from its successor's value.

DESIGN.md §7 ("Next", item 5) uses its results: all variants solve the QP to ~1e-12, but a
combine inverts a 12x12 matrix, so the chunked depth is barely below the sequential one.

    python oracle/studies/par_riccati.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.osqp_ref import OSQPSolverRef, synthetic_batch  # noqa: E402

N = 32
xcur, goals, XU = synthetic_batch(2, N, seed=7)
XU = XU + np.random.default_rng(1).normal(0, 0.2, XU.shape)
s = OSQPSolverRef(N=N)
b = 0
s.update_constraint_matrix(XU[b], xcur[b]); s.update_cost_matrix(XU[b], goals[b])
P, A = s.matrices()
Pf = (P + P.T).toarray() - np.diag(P.diagonal())
Ad = A.toarray(); g = s.g.copy(); l = s.l.copy()
ref = s.solve_qp_exact().x
nx, nu = 12, 6
T = 18 * N - 6
def xi(k): return slice(18 * k, 18 * k + 12)
def ui(k): return slice(18 * k + 12, 18 * k + 18)
# per stage data
Qs = [Pf[xi(k), xi(k)] for k in range(N)]
qs = [g[xi(k)] for k in range(N)]
Rs = [Pf[ui(k), ui(k)] for k in range(N - 1)]
rs = [g[ui(k)] for k in range(N - 1)]
As, Bs, cs = [], [], []
for k in range(N - 1):
    rows = slice(12 * (k + 1), 12 * (k + 2))
    Ak = Ad[rows, xi(k)]; Bk = Ad[rows, ui(k)]; nxt = Ad[rows, xi(k + 1)]
    assert np.allclose(nxt, -np.eye(12))
    As.append(Ak); Bs.append(Bk); cs.append(-l[rows])   # A x + B u - x' = -c  -> x' = A x + B u + c
xs0 = -l[:12]
# sequential Riccati check
Pn, pn = Qs[-1].copy(), qs[-1].copy()
Ks, ks = [None] * (N - 1), [None] * (N - 1)
for k in range(N - 2, -1, -1):
    A_, B_, c_ = As[k], Bs[k], cs[k]
    H = Rs[k] + B_.T @ Pn @ B_
    G = B_.T @ Pn @ A_
    h = rs[k] + B_.T @ (Pn @ c_ + pn)
    K = -np.linalg.solve(H, G); kf = -np.linalg.solve(H, h)
    Ks[k], ks[k] = K, kf
    pn = qs[k] + A_.T @ (Pn @ c_ + pn) + G.T @ kf
    Pn = Qs[k] + A_.T @ Pn @ A_ + G.T @ K
x = xs0.copy(); z = np.zeros(T); z[xi(0)] = x
for k in range(N - 1):
    u = Ks[k] @ x + ks[k]; z[ui(k)] = u
    x = As[k] @ x + Bs[k] @ u + cs[k]; z[xi(k + 1)] = x
print("sequential riccati vs KKT rel", np.linalg.norm(z - ref) / np.linalg.norm(ref))

# parallel elements (Sarkka & Garcia-Fernandez): V(x,y) = 1/2 x'Jx - eta'x + max_l l'(y - A x - b) - 1/2 l'C l
I = np.eye(12)
def elem(k):
    if k == N - 1:
        return (np.zeros((12, 12)), np.zeros(12), np.zeros((12, 12)), -qs[k], Qs[k])
    Ri = np.linalg.inv(Rs[k])
    C = Bs[k] @ Ri @ Bs[k].T
    bb = cs[k] - Bs[k] @ Ri @ rs[k]
    return (As[k], bb, C, -qs[k], Qs[k])
def comb(ei, ej):
    Ai, bi, Ci, ei_, Ji = ei
    Aj, bj, Cj, ej_, Jj = ej
    M = np.linalg.inv(I + Ci @ Jj)
    Aij = Aj @ M @ Ai
    bij = Aj @ M @ (bi + Ci @ ej_) + bj
    Cij = Aj @ M @ Ci @ Aj.T + Cj
    Mt = M.T  # (I + J C)^-1
    eij = Ai.T @ Mt @ (ej_ - Jj @ bi) + ei_
    Jij = Ai.T @ Mt @ Jj @ Ai + Ji
    return (Aij, bij, Cij, eij, Jij)
E = [elem(k) for k in range(N)]
# suffix scan (Hillis-Steele, backward): S_k = E_k (x) E_{k+1} (x) ... (x) E_{N-1}
S = list(E)
d = 1
while d < N:
    S = [comb(S[k], S[k + d]) if k + d < N else S[k] for k in range(N)]
    d *= 2
# value functions P_k = J, p_k = -eta
maxerr = 0
Pn2 = [None] * N; pn2 = [None] * N
for k in range(N):
    Pn2[k] = S[k][4]; pn2[k] = -S[k][3]
# compare with sequential value functions by recomputing
Pn, pn = Qs[-1].copy(), qs[-1].copy()
errs = []
for k in range(N - 2, -1, -1):
    A_, B_, c_ = As[k], Bs[k], cs[k]
    H = Rs[k] + B_.T @ Pn @ B_; G = B_.T @ Pn @ A_; h = rs[k] + B_.T @ (Pn @ c_ + pn)
    K = -np.linalg.solve(H, G); kf = -np.linalg.solve(H, h)
    pn = qs[k] + A_.T @ (Pn @ c_ + pn) + G.T @ kf
    Pn = Qs[k] + A_.T @ Pn @ A_ + G.T @ K
    errs.append((np.abs(Pn2[k] - Pn).max() / np.abs(Pn).max(), np.abs(pn2[k] - pn).max() / max(1e-300, np.abs(pn).max())))
print("value fn rel err max (P, p):", max(e[0] for e in errs), max(e[1] for e in errs))
# controls from P_{k+1}, p_{k+1}, then rollout
x = xs0.copy(); z2 = np.zeros(T); z2[xi(0)] = x
for k in range(N - 1):
    Pk1, pk1 = Pn2[k + 1], pn2[k + 1]
    H = Rs[k] + Bs[k].T @ Pk1 @ Bs[k]
    u = -np.linalg.solve(H, Bs[k].T @ Pk1 @ (As[k] @ x + cs[k]) + Bs[k].T @ pk1 + rs[k])
    z2[ui(k)] = u
    x = As[k] @ x + Bs[k] @ u + cs[k]; z2[xi(k + 1)] = x
print("parallel-scan solution vs KKT rel", np.linalg.norm(z2 - ref) / np.linalg.norm(ref))
conds = [np.linalg.cond(I + E[k][2] @ E[k+1][4]) for k in range(N-1)]
print("cond(I + C J) elementary max", max(conds))

# ---- chunked: W chunks of L elements; phase 1 chunk totals, phase 2 suffix over totals, phase 3 Riccati fix-up
def vf_comb(e, P, p):
    """element (x) value function (P, p): the Riccati step in information form."""
    Ai, bi, Ci, ei_, Ji = e
    M = np.linalg.inv(I + P @ Ci)          # (I + J_j C_i)^-1 with J_j = P
    eta = Ai.T @ M @ (-p - P @ bi) + ei_   # eta_j = -p
    J = Ai.T @ M @ P @ Ai + Ji
    return J, -eta
for W in (2, 4, 8):
    L = -(-N // W)
    chunks = [(w * L, min(N, (w + 1) * L)) for w in range(W)]
    tot = []
    for (a, bnd) in chunks:
        acc = E[bnd - 1]
        for k in range(bnd - 2, a - 1, -1):
            acc = comb(E[k], acc)
        tot.append(acc)
    # phase 2: suffix value functions at chunk starts
    Vstart = [None] * W
    P_, p_ = tot[-1][4], -tot[-1][3]          # last chunk total is a value function (contains the terminal)
    Vstart[W - 1] = (P_, p_)
    for w in range(W - 2, -1, -1):
        P_, p_ = vf_comb(tot[w], P_, p_)
        Vstart[w] = (P_, p_)
    # phase 3: within each chunk, value functions from the next chunk's start value
    Vk = [None] * N
    for w, (a, bnd) in enumerate(chunks):
        P_, p_ = (Qs[-1], qs[-1]) if w == W - 1 else Vstart[w + 1]
        if w == W - 1:
            Vk[N - 1] = (P_, p_)
            rng_ = range(bnd - 2, a - 1, -1)
        else:
            rng_ = range(bnd - 1, a - 1, -1)
        for k in rng_:
            P_, p_ = vf_comb(E[k], P_, p_)
            Vk[k] = (P_, p_)
    x = xs0.copy(); z3 = np.zeros(T); z3[xi(0)] = x
    for k in range(N - 1):
        Pk1, pk1 = Vk[k + 1]
        H = Rs[k] + Bs[k].T @ Pk1 @ Bs[k]
        u = -np.linalg.solve(H, Bs[k].T @ Pk1 @ (As[k] @ x + cs[k]) + Bs[k].T @ pk1 + rs[k])
        z3[ui(k)] = u
        x = As[k] @ x + Bs[k] @ u + cs[k]; z3[xi(k + 1)] = x
    print(f"chunked W={W}: vs KKT rel", np.linalg.norm(z3 - ref) / np.linalg.norm(ref))
