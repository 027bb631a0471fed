"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference for the notebook outputs):
    python tests/golden/make_golden.py

Outputs (data only — inputs and expected outputs):
  notebook_kats.json  numbers PRINTED in the reference notebooks (the reference's only
                      known-answer data):
                        * FK of joint-6 origin: notebooks/pin_mpc_indy7.ipynb cell 1,
                          gato_mpc_indy7.ipynb cell 1, gato_mpc_indy7_sample.ipynb cell 1
                        * the closed-loop OSQP-MPC goal-distance trace (500 values),
                          notebooks/pin_mpc_indy7.ipynb cell 2
  dynamics.npz        oracle ABA / complex-step ABA derivatives / Minv at random states
  sqp_N{16,32,64}.npz oracle CSC values (Pdata, Adata, l, g), exact QP solution and the
                      full SQP result + stats on synthetic problems (SURVEY.md §8d draws)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import rbd  # noqa: E402
from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch  # noqa: E402

REF = "/root/reference"


def _outputs(nb, cell):
    out = []
    for o in nb["cells"][cell].get("outputs", []):
        out.append("".join(o.get("text", [])) or "".join(o.get("data", {}).get("text/plain", [])))
    return "\n".join(out)


def _matrix(txt):
    rows = []
    for line in txt.replace("[", " ").replace("]", " ").splitlines():
        vals = line.split()
        try:
            nums = [float(v) for v in vals]
        except ValueError:
            continue
        if len(nums) == 3:
            rows.append(nums)
    return rows


def notebook_kats():
    nbdir = os.path.join(REF, "notebooks")
    pin = json.load(open(os.path.join(nbdir, "pin_mpc_indy7.ipynb")))
    gato = json.load(open(os.path.join(nbdir, "gato_mpc_indy7.ipynb")))
    samp = json.load(open(os.path.join(nbdir, "gato_mpc_indy7_sample.ipynb")))
    kats = []
    ones = np.ones(6)
    # pin_mpc_indy7.ipynb cell 1: endpoints printed with 8 decimals
    qs = [0.3 * ones, 0.9 * ones, np.array([-3.0, 1.0, 1.0, 1.0, 0.0, 0.0])]
    for q, p in zip(qs, _matrix(_outputs(pin, 1))[:3]):
        kats.append({"q": q.tolist(), "eepos": p, "digits": 8, "source": "notebooks/pin_mpc_indy7.ipynb cell 1"})
    # gato_mpc_indy7.ipynb cell 1: 6 endpoints, 9 significant digits
    qs = [0 * ones, np.array([-3.0, 1.0, 1.0, 1.0, 0.0, 0.0]), 0.8 * ones, 0 * ones, -1.6 * ones, 0 * ones]
    for q, p in zip(qs, _matrix(_outputs(gato, 1))[:6]):
        kats.append({"q": q.tolist(), "eepos": p, "digits": 9, "source": "notebooks/gato_mpc_indy7.ipynb cell 1"})
    # gato_mpc_indy7_sample.ipynb cell 1
    qs = [1.6 * ones, 0.5 * ones, 0.2 * ones, -0.5 * ones, -0.9 * ones, 0.5 * ones, np.array([0.5, 1.5, 2.0, 0, 0, 0])]
    rows = _matrix(_outputs(samp, 2))  # endpoints defined in cell 1, printed by cell 2
    for q, p in zip(qs, rows[:7]):
        kats.append({"q": q.tolist(), "eepos": p, "digits": 8, "source": "notebooks/gato_mpc_indy7_sample.ipynb cells 1-2"})
    txt = _outputs(pin, 2)
    trace = [float(l) for l in txt.splitlines() if l.strip() and l.strip()[0].isdigit()]
    return {
        "fk": kats,
        "mpc_trace": {
            "source": "notebooks/pin_mpc_indy7.ipynb cell 2 (MPC_OSQP.run_mpc, N=32, OSQP eps 1e-3)",
            "xstart": [1.0] * 12,
            "endpoint_q": [[0.3] * 6, [0.9] * 6, [-3.0, 1.0, 1.0, 1.0, 0.0, 0.0]],
            "goal_distances": trace,
        },
    }


def dynamics(n=48, seed=11):
    rng = np.random.default_rng(seed)
    q = rng.uniform(-3, 3, (n, 6))
    v = rng.uniform(-2, 2, (n, 6))
    tau = rng.uniform(-60, 60, (n, 6))
    out = {k: [] for k in ("a", "dq", "dv", "Minv", "M", "eepos", "J")}
    for i in range(n):
        dq, dv, Mi, a = rbd.aba_derivatives(q[i], v[i], tau[i])
        p, J = rbd.d_eepos(q[i])
        out["a"].append(a)
        out["dq"].append(dq)
        out["dv"].append(dv)
        out["Minv"].append(Mi)
        out["M"].append(rbd.crba(q[i]))
        out["eepos"].append(p)
        out["J"].append(J)
    return dict(q=q, v=v, tau=tau, **{k: np.array(v_) for k, v_ in out.items()})


def sqp_fixture(N, B, seed, n_csc=2):
    xcur, goals, XU = synthetic_batch(B, N, seed)
    res = dict(xcur=xcur, goals=goals, XU=XU)
    # linearisation point for the CSC/QP fixture: a perturbed trajectory
    XUl = XU + np.random.default_rng(seed + 1).normal(0, 0.3, XU.shape)
    XUl[:, :12] = xcur
    res["XU_lin"] = XUl
    P, A, l, g, sol = [], [], [], [], []
    for b in range(B):
        s = OSQPSolverRef(N=N)
        x = s.setup_and_solve_qp(XUl[b], xcur[b], goals[b]).x
        sol.append(x)
        if b < n_csc:
            P.append(s.Pdata.copy())
            A.append(s.Adata.copy())
            l.append(s.l.copy())
            g.append(s.g.copy())
    res.update(Pdata=np.array(P), Adata=np.array(A), l=np.array(l), g=np.array(g), qp_sol=np.array(sol))
    outs, qp_iters, alphas, steps = [], [], [], []
    for b in range(B):
        sq = SQPRef(OSQPSolverRef(N=N))
        outs.append(sq.sqp(xcur[b], goals[b], XU[b].copy()))
        st = sq.get_stats()
        qp_iters.append(st["qp_iters"]["values"][0])
        a = st["linesearch_alphas"]["values"]
        alphas.append(list(a) + [np.nan] * (8 - len(a)))
        s_ = st["sqp_stepsizes"]["values"]
        steps.append(list(s_) + [np.nan] * (8 - len(s_)))
    res.update(sqp_out=np.array(outs), qp_iters=np.array(qp_iters), alphas=np.array(alphas), stepsizes=np.array(steps))
    return res


def main():
    if os.path.isdir(REF):
        with open(os.path.join(HERE, "notebook_kats.json"), "w") as f:
            json.dump(notebook_kats(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "dynamics.npz"), **dynamics())
    for N, B in ((16, 8), (32, 6), (64, 3)):
        np.savez_compressed(os.path.join(HERE, f"sqp_N{N}.npz"), **sqp_fixture(N, B, seed=100 + N))
        print("N", N, "done", flush=True)


if __name__ == "__main__":
    main()
