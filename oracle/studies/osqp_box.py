"""STUDY (test infrastructure, not shipped): config 4 (box rows on q, v, u) through OSQP itself.

SURVEY.md §8d names config 4 "ADMM mode".  This runs config-4 QPs through the OSQP restatement
(oracle/osqp_admm.py — the reference's solver, pinned by the notebook's closed loop) with the box
rows appended to A (l_b <= x_b <= u_b on every bounded entry, oracle/box_ipm.box_bounds), and
compares with the interior point of the box mode (oracle/box_ipm.py, I7M_QP_BOX):

    python -m oracle.studies.osqp_box [--B 8] [--N 32] [--seed 46]

Per problem (first SQP iteration's QP): OSQP's status, iterations and distance from the interior
point's optimum with the settings that reproduce the reference (defaults, rho fixed), then with
adaptive rho every 25 iterations.
"""
from __future__ import annotations

import argparse

import numpy as np

from oracle.osqp_ref import OSQPSolverRef, synthetic_batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--seed", type=int, default=46)
    a = ap.parse_args()
    xcur, goals, XU = synthetic_batch(a.B, a.N, a.seed)
    rows = []
    for b in range(a.B):
        ipm = OSQPSolverRef(N=a.N, qp="box").setup_and_solve_qp(XU[b], xcur[b], goals[b]).x
        s = OSQPSolverRef(N=a.N, qp="osqp", osqp_box=7)
        s.setup_and_solve_qp(XU[b], xcur[b], goals[b])
        st0, it0 = s.osqp.info["status"], s.osqp.info["iter"]
        x0 = s.osqp.D * s.osqp.x
        rel0 = float(np.linalg.norm(x0 - ipm) / np.linalg.norm(ipm))
        s = OSQPSolverRef(N=a.N, qp="osqp", osqp_box=7, osqp_settings=dict(adaptive_rho_interval=25))
        x = s.setup_and_solve_qp(XU[b], xcur[b], goals[b]).x
        rel = float(np.linalg.norm(x - ipm) / np.linalg.norm(ipm))
        rows.append((st0, it0, rel0, s.osqp.info["status"], s.osqp.info["iter"], rel))
        print(f"problem {b}: defaults -> {st0} at {it0} iterations, |x - x_ipm| / |x_ipm| = {rel0:.1e}; adaptive rho "
              f"(every 25) -> {s.osqp.info['status']} at {s.osqp.info['iter']}, {rel:.1e}", flush=True)
    print(f"defaults: {sum(r[0] == 'solved' for r in rows)} of {a.B} solved, iterations median "
          f"{np.median([r[1] for r in rows]):.0f}, distance from the interior point median "
          f"{np.median([r[2] for r in rows]):.1e}; adaptive rho: {sum(r[3] == 'solved' for r in rows)} solved, "
          f"iterations median {np.median([r[4] for r in rows]):.0f}, distance median {np.median([r[5] for r in rows]):.1e}")


if __name__ == "__main__":
    main()
