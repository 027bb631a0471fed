"""A/B of the ADMM mode's launch shape (I7M_ADMM_CHUNK, read at handle creation): cold OSQP
state every step, B problems at horizon N, ADMM kernels' time per launch and solves/s, one JSON line
per setting.

    python tools/admm_ab.py [--B 4096] [--N 32] [--chunks 0,2048,1024] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--chunks", default="0,2048,1024")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--scaling", type=int, default=None, help="OSQP's Ruiz passes (default: the reference's 10)")
    ap.add_argument("--admm", default=None, help='further OSQP settings as JSON, e.g. \'{"max_iter": 50, "check_termination": 0}\'')
    a = ap.parse_args()
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    model = default_model()
    dev = torch.device("cuda", 0)
    for rep in range(2):
        for c in [int(x) for x in a.chunks.split(",")]:
            os.environ["I7M_ADMM_CHUNK"] = str(c)
            st = {} if a.scaling is None else {"scaling": a.scaling}
            st.update(json.loads(a.admm) if a.admm else {})
            kw = {"admm": st} if st else {}
            h = _lib.Handle(model, N=a.N, max_batch=a.B, qp_mode=_lib.QP_ADMM, **kw)
            xcur, goals, XU = make_batch(h, model, a.B, a.N, seed=45)
            t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
            t_out = torch.empty_like(t_xu)
            h.solve_device(a.B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr())
            h.synchronize()
            h.reset_kernel_times()
            h.set_timing(True)
            el = []
            for _ in range(a.steps):
                h.admm_reset()
                t0 = time.perf_counter()
                h.solve_device(a.B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr())
                h.synchronize()
                el.append(time.perf_counter() - t0)
            kt = h.kernel_times()
            it = h.admm_stats(a.B)[0]
            h.close()
            used = it[it >= 0]
            print(json.dumps({"rep": rep, "chunk": c, "B": a.B, "N": a.N, "solves_per_s": a.B / float(np.mean(el)),
                              "ms_per_step": 1e3 * float(np.mean(el)), "osqp_iters_mean": float(used.mean()),
                              "kernels": {k: {"avg_us": round(1e3 * ms / max(n, 1), 1), "launches": n}
                                          for k, (ms, n) in kt.items()}}), flush=True)


if __name__ == "__main__":
    main()
