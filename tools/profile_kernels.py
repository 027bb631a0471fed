"""Run only the bench workload's device solves (no CPU leg, no latency loop) so rocprofv3
kernel-trace / PMC summaries contain exactly the timed kernels.

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- python tools/profile_kernels.py
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o fetch -- python tools/profile_kernels.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--box", action="store_true", help="config 4: box rows (I7M_QP_BOX), seed 46")
    ap.add_argument("--admm", action="store_true", help="config 3 in ADMM mode (I7M_QP_ADMM), cold OSQP state per solve")
    ap.add_argument("--pipeline", default="split", choices=["split", "fused", "fused_iter"])
    a = ap.parse_args()
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    dev = torch.device("cuda", 0)
    model = default_model()
    pipe = {"split": _lib.PIPE_SPLIT, "fused": _lib.PIPE_FUSED, "fused_iter": _lib.PIPE_FUSED_ITER}[a.pipeline]
    mode = {"qp_mode": _lib.QP_BOX} if a.box else ({"qp_mode": _lib.QP_ADMM} if a.admm else {})
    h = _lib.Handle(model, N=a.N, max_batch=a.batch, pipeline=pipe, **mode)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    h.set_stream(s.cuda_stream)
    xcur, goals, XU = make_batch(h, model, a.batch, a.N, seed=46 if a.box else 45)
    t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
    t_out = torch.empty_like(t_xu)
    for _ in range(a.warmup + a.steps):
        if a.admm:
            h.admm_reset()
        h.solve_device(a.batch, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), None)
    torch.cuda.synchronize(dev)
    print("profiled", a.warmup + a.steps, "solves of B", a.batch, "N", a.N)


if __name__ == "__main__":
    main()
