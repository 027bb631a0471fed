"""A/B of the host-to-host solve (i7m_solve: numpy in, numpy out) split into chunks
(i7m_config.h2h_chunks; I7M_H2H_PIPE=0 for the alternating two-stream layout instead of the pipeline) at config 3 (B = 4096, N = 32): median of 20 timed calls after 3
warm-up calls per chunk count (BASELINE.md §4's procedure), each output checked bit for bit
against the one-piece solve.  Prints one JSON line per setting.

    python tools/h2h_ab.py [--batch 4096] [--N 32] [--chunks 1,2,3,4,8] [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--chunks", default="1,2,3,4,8")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pinned", action="store_true", help="inputs and outputs in pinned host memory (torch pin_memory)")
    ap.add_argument("--mode", default="direct", choices=["direct", "admm"],
                    help="QP mode; admm: every call from a cold OSQP state (admm_reset outside the timing)")
    a = ap.parse_args()
    import numpy as np

    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    model = default_model()
    ref = None
    for nch in [int(c) for c in a.chunks.split(",")]:
        h = _lib.Handle(model, N=a.N, max_batch=a.batch, h2h_chunks=nch,
                        qp_mode=_lib.QP_ADMM if a.mode == "admm" else _lib.QP_DIRECT)
        xcur, goals, XU = make_batch(h, model, a.batch, a.N, 45)
        out = st = None
        if a.pinned:
            import torch

            def pin(x):
                t = torch.empty(x.shape, dtype=torch.float64, pin_memory=True)
                t.numpy()[...] = x
                return t

            keep = [pin(x) for x in (xcur, goals, XU, np.zeros_like(XU))]
            st_t = torch.empty(a.batch * _lib.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
            keep.append(st_t)
            xcur, goals, XU, out = (t.numpy() for t in keep[:4])
            st = st_t.numpy().view(_lib.STATS_DTYPE)
        ts = []
        for i in range(a.reps + 3):
            if a.mode == "admm":
                h.admm_reset()
            t0 = time.perf_counter()
            out, st = h.solve(xcur, goals, XU, out=out, stats=st)
            if i >= 3:
                ts.append(time.perf_counter() - t0)
        if ref is None:
            ref = (out.copy(), st.copy())
        same = bool(np.array_equal(out, ref[0]) and np.array_equal(st, ref[1]))
        med = statistics.median(ts)
        print(json.dumps({"mode": a.mode, "h2h_chunks": nch, "pipe": os.environ.get("I7M_H2H_PIPE", "2"), "taper": os.environ.get("I7M_H2H_TAPER", "1"), "pinned": a.pinned, "batch": a.batch, "N": a.N, "median_ms": 1e3 * med,
                          "host_to_host_solves_per_s": a.batch / med, "min_ms": 1e3 * min(ts),
                          "bit_identical_to_first": same}), flush=True)
        h.close()


if __name__ == "__main__":
    main()
