"""A/B: config 3 in ADMM mode (or --mode box / direct) as one batch on one stream against K sub-batches on K streams, the
k-th sub-batch started `--offset-us` × k later (a device sleep on its stream), so that one
sub-batch's latency-bound phases (the factor, the OSQP tail after the first termination check)
overlap another's stream-bound ones.  Cold OSQP state every step; one JSON line per setting.

    python tools/admm_streams_ab.py [--B 4096] [--N 32] [--ks 1,2,4] [--offsets 0,1000,2000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--ks", default="1,2,4")
    ap.add_argument("--offsets", default="0,1000,2000")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--mode", default="admm", choices=["admm", "box", "direct"])
    a = ap.parse_args()
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    model = default_model()
    dev = torch.device("cuda", 0)
    # device clock for torch.cuda._sleep: cycles per microsecond, measured
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    torch.cuda._sleep(10_000_000)
    s1.record()
    torch.cuda.synchronize()
    cyc_per_us = 10_000_000 / (1e3 * s0.elapsed_time(s1))
    for rep in range(2):
        for K in [int(x) for x in a.ks.split(",")]:
            for off in [float(x) for x in a.offsets.split(",")] if K > 1 else [0.0]:
                b = a.B // K
                hs, ss, bufs = [], [], []
                for i in range(K):
                    qm = {"admm": _lib.QP_ADMM, "box": _lib.QP_BOX, "direct": _lib.QP_DIRECT}[a.mode]
                    h = _lib.Handle(model, N=a.N, max_batch=b, qp_mode=qm)
                    s = torch.cuda.Stream(dev)
                    h.set_stream(s.cuda_stream)
                    xcur, goals, XU = make_batch(h, model, a.B, a.N, seed=45)
                    sl = slice(i * b, (i + 1) * b)
                    t = [torch.from_numpy(np.ascontiguousarray(x[sl])).to(dev) for x in (XU, xcur, goals)]
                    t.append(torch.empty_like(t[0]))
                    hs.append(h)
                    ss.append(s)
                    bufs.append(t)

                def run():
                    for h in hs:
                        if a.mode == "admm":
                            h.admm_reset()
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ends = []
                    for i, (h, s, t) in enumerate(zip(hs, ss, bufs)):
                        s.wait_event(e0)
                        with torch.cuda.stream(s):
                            if i and off > 0:
                                torch.cuda._sleep(int(i * off * cyc_per_us))
                            h.solve_device(b, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), 3, t[3].data_ptr())
                            ev = torch.cuda.Event()
                            ev.record(s)
                            ends.append(ev)
                    for ev in ends:
                        torch.cuda.current_stream().wait_event(ev)
                    e1.record()
                    torch.cuda.synchronize()
                    return e0.elapsed_time(e1)

                run()  # warm-up
                ms = [run() for _ in range(a.steps)]
                its = np.concatenate([h.admm_stats(b)[0] for h in hs]) if a.mode == "admm" else np.zeros(1)
                for h in hs:
                    h.close()
                used = its[its >= 0]
                print(json.dumps({"mode": a.mode, "rep": rep, "K": K, "offset_us": off, "B": a.B, "N": a.N,
                                  "ms_per_batch": float(np.mean(ms)), "solves_per_s": a.B / (1e-3 * float(np.mean(ms))),
                                  "osqp_iters_mean": float(used.mean())}), flush=True)


if __name__ == "__main__":
    main()
