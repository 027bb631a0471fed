"""How close the device's ADMM mode is to the C++ port's (oracle/cpp) on one batch, to the bit:
share of problems whose solution / carried state are bitwise identical, max relative difference,
OSQP iteration agreement; exact mode beside it (diagnostic: A/B of FMA contraction builds).

    [I7M_LIB=...] python tools/port_diff.py [B] [N] [seed]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 61
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from oracle import cpu
    from oracle.osqp_ref import synthetic_batch
    xc, g, xu = synthetic_batch(B, N, seed)
    res = {"lib": os.path.basename(_lib.LIB_PATH), "B": B, "N": N}
    for mode in ("admm", "exact"):
        h = _lib.Handle(default_model(), N=N, max_batch=B, qp_mode=_lib.QP_ADMM if mode == "admm" else _lib.QP_DIRECT)
        out = h.solve(xc, g, xu)[0]
        if mode == "admm":
            st = [s.copy() for s in h.admm_state(B)[:3]]
            it = np.array(h.admm_stats(B)[0])
            stp = cpu.AdmmState(B, N)
            ref, _, _, _, rit = cpu.solve_admm(xc, g, xu, N, stp, nthreads=16)
            rst = [stp.x, stp.z, stp.y]
            res["admm_state_bitwise_share"] = [float(np.all(a == b_, axis=1).mean()) for a, b_ in zip(st, rst)]
            res["admm_state_max_abs"] = [float(np.abs(a - b_).max()) for a, b_ in zip(st, rst)]
            res["osqp_iters_agree"] = float(np.all(np.where(rit >= 0, it == rit, True), axis=1).mean())
        else:
            ref = cpu.solve(xc, g, xu, N, nthreads=16)[0]
        h.close()
        rel = np.abs(out - ref).max(axis=1) / np.maximum(np.abs(ref).max(axis=1), 1e-300)
        res[mode] = {"bitwise_share": float(np.all(out == ref, axis=1).mean()), "rel_max": float(rel.max()),
                     "rel_median": float(np.median(rel))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
