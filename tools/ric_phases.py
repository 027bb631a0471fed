"""Per-stage phase timing of the Riccati backward sweep at B = 1 (diagnostic build
I7M_ABLATE=19: s_memtime stamps of problem 0, results invalid): operand staging + first
MFMAs, the G~ MFMAs, the Gauss-Jordan elimination, the V~ update.  python tools/ric_phases.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ["I7M_ABLATE"] = "19"
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    model = default_model()
    N = 32
    h = _lib.Handle(model, N=N, max_batch=1)
    xcur, goals, XU = make_batch(h, model, 1, N, seed=44)
    rows = []
    for _ in range(20):
        sol = h.qp(XU, xcur, goals)
        rows.append(sol[0, : 8 * (N - 1)].reshape(N - 1, 8))
    t = np.median(np.stack(rows), axis=0)  # (stage, phase) cycles
    names = ["stash LDS + operands + MFMA chains", "W0 MFMA chain", "wait for the stage's stash loads", "G~ issue",
             "H, G~ -> LDS -> columns", "six pivots", "K~ -> LDS", "V~ update"]
    per = t.mean(axis=0)
    for n, v in zip(names, per):
        print(f"{n:32s} {v:8.0f} cycles/stage")
    print(f"{'total':32s} {per.sum():8.0f} cycles/stage over {N - 1} stages")


if __name__ == "__main__":
    main()
