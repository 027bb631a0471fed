"""A/B of hipGraph replay (I7M_GRAPH) on device-resident solves: B=4096 throughput without
per-launch events, and B=1 / B=64 p50 latency.  Run twice with I7M_GRAPH=0 / 1."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch
    dev = torch.device("cuda", 0)
    model = default_model()
    B, N = 4096, 32
    h = _lib.Handle(model, N=N, max_batch=B)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    h.set_stream(s.cuda_stream)
    xc, g, XU = make_batch(h, model, B, N, seed=45)
    t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xc, g))
    out = torch.empty_like(t_xu)
    res = {}
    for b in (4096, 64, 1):
        for _ in range(5):
            h.solve_device(b, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, out.data_ptr(), None)
        torch.cuda.synchronize(dev)
        reps = 20 if b == 4096 else 200
        if b == 4096:
            t0 = time.perf_counter()
            for _ in range(reps):
                h.solve_device(b, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, out.data_ptr(), None)
            torch.cuda.synchronize(dev)
            res["solves_per_s_4096"] = b * reps / (time.perf_counter() - t0)
        else:
            lat = []
            for _ in range(reps):
                a = time.perf_counter()
                h.solve_device(b, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, out.data_ptr(), None)
                torch.cuda.synchronize(dev)
                lat.append((time.perf_counter() - a) * 1e3)
            res[f"p50_ms_B{b}"] = statistics.median(lat)
    print(os.environ.get("I7M_GRAPH", "0"), res)


if __name__ == "__main__":
    main()
