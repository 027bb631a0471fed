"""Bitwise comparison of two library builds on the same inputs (tools/ only).

    I7M_LIB=<a.so> python tools/lib_diff.py dump A.npz    (one process per build)
    python tools/lib_diff.py cmp A.npz B.npz

dump: one config-3 solve (B = 4096, N = 32, bench.py's draws), one config-4 solve (B = 256,
N = 64, box rows) and the notebook's 500-step closed loop (B = 1, N = 32).
cmp: per output, how many problems differ at all, the largest relative difference, and for the
closed loop the first step at which the goal distances differ.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path):
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from oracle.osqp_ref import synthetic_batch  # goals by the CPU FK: identical inputs for both builds
    m = default_model()
    out = {}
    xc, g, xu = synthetic_batch(4096, 32, 45)
    h = _lib.Handle(m, N=32, max_batch=4096)
    out["c3"] = h.solve(xc, g, xu)[0]
    h.close()
    xc, g, xu = synthetic_batch(256, 64, 48)
    h = _lib.Handle(m, N=64, max_batch=256, qp_mode=_lib.QP_BOX)
    out["c4"] = h.solve(xc, g, xu)[0]
    h.close()
    tr = json.load(open(os.path.join(ROOT, "tests", "golden", "notebook_kats.json")))["mpc_trace"]
    h = _lib.Handle(m, N=32, max_batch=1)
    ends = h.eepos(np.array(tr["endpoint_q"]))
    out["mpc"] = h.mpc_run(np.array([tr["xstart"]]), ends, 500)[0][:, 0]
    h.close()
    # ADMM mode (the drop-in default): config 3 twice (cold, then warm from the carried state), the
    # carried state after it, N = 64 and an odd batch (empty rows of the 3- and 4-problem waves)
    for key, (B, N, seed) in {"a3": (4096, 32, 45), "a64": (24, 64, 48), "a13": (13, 32, 50)}.items():
        xc, g, xu = synthetic_batch(B, N, seed)
        h = _lib.Handle(m, N=N, max_batch=B, qp_mode=_lib.QP_ADMM)
        o1 = h.solve(xc, g, xu)[0]
        o2 = h.solve(xc, g, o1)[0]
        out[key] = np.concatenate([o1, o2], axis=1)
        out[key + "_state"] = np.concatenate(h.admm_state(B)[:4], axis=1)
        out[key + "_iters"] = h.admm_stats(B)[0]
        h.close()
    h = _lib.Handle(m, N=32, max_batch=1, qp_mode=_lib.QP_ADMM)
    out["mpca"] = h.mpc_run(np.array([tr["xstart"]]), ends, 40)[0][:, 0]
    h.close()
    out["ver"] = np.array(_lib.version())
    np.savez(path, **out)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    print("A:", str(A["ver"]), "\nB:", str(B["ver"]))
    for k in ("c3", "c4", "a3", "a3_state", "a3_iters", "a64", "a64_state", "a13", "a13_state"):
        if k not in A or k not in B:
            continue
        x, y = A[k].astype(float), B[k].astype(float)
        diff = (x != y).any(axis=1)
        rel = np.linalg.norm(x - y, axis=1) / np.maximum(np.linalg.norm(x, axis=1), 1e-300)
        print(f"{k}: {int(diff.sum())} of {len(x)} problems differ; max rel {rel.max():.2e}")
    for k in ("mpc", "mpca"):
        if k not in A or k not in B:
            continue
        x, y = A[k], B[k]
        nz = np.nonzero((x != y) & ~(np.isnan(x) & np.isnan(y)))[0]
        print(f"{k}: first differing step {nz[0] if len(nz) else None}; max |diff| {np.nanmax(np.abs(x - y)):.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
