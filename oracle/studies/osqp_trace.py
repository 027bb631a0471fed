"""STUDY (test infrastructure, not shipped): which QP solver reproduces the reference's printed
closed loop (notebooks/pin_mpc_indy7.ipynb cell 2, 500 goal distances, OSQP eps 1e-3)?

    python -m oracle.studies.osqp_trace [--steps 20] [--intervals exact,0,25,0g,25g]

For every variant the numpy oracle runs MPC_OSQP.run_mpc (oracle/mpc_ref.py) from the notebook's
start with the QP solved either exactly (``exact``) or by the OSQP 0.6 restatement
(oracle/osqp_admm.py) with the given adaptive-rho interval (suffix g: with OSQP 1.x's
duality-gap test), and prints the largest deviation from
the printed trace over the first 8, 20, ... steps.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np

from oracle import rbd
from oracle.mpc_ref import run_mpc_ref
from oracle.osqp_ref import OSQPSolverRef, SQPRef

GOLD = os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "notebook_kats.json")


def run(variant, steps):
    tr = json.load(open(GOLD))["mpc_trace"]
    ends = [rbd.eepos(np.array(q)) for q in tr["endpoint_q"]]
    if variant == "exact":
        s = OSQPSolverRef(N=32)
    else:
        gap = variant.endswith("g")
        s = OSQPSolverRef(N=32, qp="osqp", osqp_settings=dict(adaptive_rho_interval=int(variant.rstrip("g")), check_dualgap=gap))
    sqp = SQPRef(s)
    _, d = run_mpc_ref(sqp, np.array(tr["xstart"]), ends, num_steps=steps)
    ref = np.array(tr["goal_distances"][:len(d)])
    hist = getattr(getattr(s, "osqp", None), "history", [])
    return np.abs(np.array(d) - ref), hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--intervals", default="exact,0,25,0g,25g")
    a = ap.parse_args()
    for v in a.intervals.split(","):
        t0 = time.time()
        err, hist = run(v, a.steps)
        marks = [k for k in (8, 20, 50, 100, 200, 500) if k <= len(err)]
        s = "  ".join(f"<= {k}: {err[:k].max():.1e}" for k in marks)
        its = [h[0] for h in hist]
        extra = f"  ADMM iters/QP median {np.median(its):.0f} max {max(its)}, rho updates {sum(h[2] for h in hist)}" if its else ""
        print(f"{v:>6s}: max |d - d_notebook| {s}{extra}  ({time.time() - t0:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
