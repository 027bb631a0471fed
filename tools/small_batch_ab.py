"""Small-batch latency A/B (config 2 shape): per-step time and per-kernel launch durations of
the solve at B in {1, 64, 256} for the default kernels and the variants selected by environment
knobs read at handle creation (I7M_RICCATI=valu, I7M_GRAPH=1).
python tools/small_batch_ab.py"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(B, N, env, steps=100, **handle_kw):
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        model = default_model()
        h = _lib.Handle(model, N=N, max_batch=B, **handle_kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    h.set_stream(s.cuda_stream)
    xcur, goals, XU = make_batch(h, model, B, N, seed=44)
    t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
    t_out = torch.empty_like(t_xu)

    def step():
        h.solve_device(B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), None)

    for _ in range(10):
        step()
    torch.cuda.synchronize(dev)
    lat = []
    for _ in range(steps):
        a = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        lat.append(1e3 * (time.perf_counter() - a))
    h.reset_kernel_times()
    h.set_timing(True)
    for _ in range(20):
        step()
    torch.cuda.synchronize(dev)
    h.set_timing(False)
    kt = h.kernel_times()
    h.close()
    return {"B": B, "env": env, "p50_ms": statistics.median(lat),
            "kernels_us": {k: round(1e3 * ms / max(c, 1), 2) for k, (ms, c) in kt.items()}}


def main():
    out = []
    for B in (1, 64, 256):
        for env in ({}, {"I7M_RICCATI": "valu"}, {"I7M_GRAPH": "1"}):
            r = run(B, 32, env)
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
