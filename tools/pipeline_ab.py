"""A/B of the launch pipelines (include/indy7_mpc.h I7M_PIPE_*): split (3 kernels per SQP
iteration), fused (k_sqp_fused, one launch per solve) and fused_iter (one launch per SQP
iteration), device-resident, over batch sizes.  Per mode and B: throughput over back-to-back
solves (no syncs between), p50 host-to-host latency of one solve, per-kernel launch durations.
Every mode's output is compared with the split one (bit-identical expected).

    python tools/pipeline_ab.py [--N 32] [--batches 1,64,256,1024,4096] [--steps 50]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(B, N, pipe, steps):
    import numpy as np
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    model = default_model()
    h = _lib.Handle(model, N=N, max_batch=B, pipeline=pipe)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    h.set_stream(s.cuda_stream)
    xcur, goals, XU = make_batch(h, model, B, N, seed=45)
    t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
    t_out = torch.empty_like(t_xu)

    def step():
        h.solve_device(B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), None)

    for _ in range(5):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    thr = B * steps / (time.perf_counter() - t0)
    lat = []
    for _ in range(min(steps, 30)):
        a = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        lat.append(1e3 * (time.perf_counter() - a))
    h.reset_kernel_times()
    h.set_timing(True)
    for _ in range(10):
        step()
    torch.cuda.synchronize(dev)
    h.set_timing(False)
    kt = h.kernel_times()
    out = t_out.cpu().numpy()
    h.close()
    return out, {"solves_per_s": thr, "ms_per_step": 1e3 * B / thr, "p50_h2h_ms": statistics.median(lat),
                 "kernels_us": {k: round(1e3 * ms / max(c, 1), 2) for k, (ms, c) in kt.items()},
                 "launches_per_step": {k: c / 10 for k, (ms, c) in kt.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--batches", default="1,64,256,1024,4096")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--modes", default="split,fused,fused_iter")
    a = ap.parse_args()
    import numpy as np
    from indy7_mpc_amd import _lib

    codes = {"split": _lib.PIPE_SPLIT, "fused": _lib.PIPE_FUSED, "fused_iter": _lib.PIPE_FUSED_ITER}
    res = []
    for B in [int(x) for x in a.batches.split(",")]:
        ref = None
        for mode in a.modes.split(","):
            out, r = run(B, a.N, codes[mode], a.steps)
            if ref is None:
                ref = out
            r.update(B=B, N=a.N, mode=mode, equal_to_first=bool(np.array_equal(out, ref)))
            print(json.dumps(r), flush=True)
            res.append(r)
    return res


if __name__ == "__main__":
    main()
