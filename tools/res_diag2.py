"""k_admm_iter_res against the streaming kernels (I7M_ADMM_ITER2 1 / 0) after 1-3 OSQP iterations
(no termination test): which entries of the carried x, z, y differ (stage, row) (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(env, B, N, seed, iters):
    os.environ.update(env)
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from oracle.osqp_ref import synthetic_batch
    xc, g, xu = synthetic_batch(B, N, seed)
    h = _lib.Handle(default_model(), N=N, max_batch=B, qp_mode=_lib.QP_ADMM, max_sqp_iters=1,
                    admm={"max_iter": iters, "check_termination": 0})
    h.solve(xc, g, xu)
    st = [s.copy() for s in h.admm_state(B)[:3]]
    h.close()
    return st


if __name__ == "__main__":
    B, N, seed = 1, 32, 51
    for iters in (1, 2, 3):
        r = {k: run(e, B, N, seed, iters) for k, e in
             (("res", {"I7M_ADMM_RES": "1", "I7M_ADMM_ITER2": "-1"}), ("it2", {"I7M_ADMM_RES": "0", "I7M_ADMM_ITER2": "1"}),
              ("it4", {"I7M_ADMM_RES": "0", "I7M_ADMM_ITER2": "0"}))}
        for a, b in (("res", "it2"),):
            for name, x, y in zip("xzy", r[a], r[b]):
                d = np.nonzero(x[0] != y[0])[0]
                per = 18 if name == "x" else 12
                locs = [(int(i) // per, int(i) % per, float(x[0, i]).hex(), float(y[0, i]).hex()) for i in d[:6]]
                print(f"iters={iters} {a} vs {b} {name}: {len(d)} differ; {locs}", flush=True)
