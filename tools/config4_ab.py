"""Config 4 (B = 4096, N = 64, box rows) on one GPU: solves/s, IPM iterations and per-kernel
times of the library in I7M_LIB (k_ipm_fused; the split-launch and factorisation-reuse forms
measured in round 2 were removed in round 3).
    python tools/config4_ab.py [--steps 3] [--B 4096] [--N 64]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, B, N, steps):
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    model = default_model()
    dev = torch.device("cuda", 0)
    h = _lib.Handle(model, N=N, max_batch=B, device_id=0, qp_mode=_lib.QP_BOX)
    stream = torch.cuda.Stream(dev)
    h.set_stream(stream.cuda_stream)
    xcur, goals, XU = make_batch(h, model, B, N, seed=42 + 4)
    t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
    t_out = torch.empty_like(t_xu)

    def step():
        h.solve_device(B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), None)

    step()
    torch.cuda.synchronize(dev)
    h.reset_kernel_times()
    h.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    h.set_timing(False)
    kt = h.kernel_times()
    it, conv, _ = h.box_stats(B)
    out = t_out.cpu().numpy()
    h.close()
    return out, {"mode": mode, "solves_per_s": B * steps / el, "ms_per_step": 1e3 * el / steps,
                 "ipm_iters_mean": float(it.mean()), "ipm_iters_max": int(it.max()),
                 "ipm_iters_hist": np.bincount(it).tolist(), "converged": float(conv.mean()),
                 "kernels": {k: {"avg_us": 1e3 * ms / max(c, 1), "launches": c} for k, (ms, c) in kt.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--modes", default="fused")
    a = ap.parse_args()
    res, outs = {}, {}
    modes = a.modes.split(",")
    for mode in modes:
        outs[mode], res[mode] = run(mode, a.B, a.N, a.steps)
        res[mode].pop("ipm_iters_hist")
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
