"""A/B of the batched closed loop (i7m_mpc_run) in one process per setting: B instances, N = 32,
`--steps` MPC steps, wall clock of the whole run as the bench's `closed_loop` line, `--reps` runs.

    I7M_ADMM_STAGGER=0 python tools/mpc_loop_ab.py [--mode admm|direct] [--B 4096] [--steps 10]
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", default="admm", choices=["admm", "direct"])
    ap.add_argument("--torch-stream", action="store_true", help="run on a torch stream (i7m_set_stream), as bench.py")
    a = ap.parse_args()
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import draw_states

    model = default_model()
    qm = _lib.QP_ADMM if a.mode == "admm" else _lib.QP_DIRECT
    h = _lib.Handle(model, N=a.N, max_batch=a.B, qp_mode=qm)
    if a.torch_stream:
        import torch
        stream = torch.cuda.Stream(torch.device("cuda", 0))
        h.set_stream(stream.cuda_stream)
    xs, qg = draw_states(model, a.B, seed=42 + 3)
    ends = np.vstack([h.eepos(qg[:1]), h.eepos(qg[1:2])])
    h.mpc_run(xs, ends, 2)
    for rep in range(a.reps):
        if qm == _lib.QP_ADMM:
            h.admm_reset()
        t0 = time.perf_counter()
        d, q, _, _ = h.mpc_run(xs, ends, a.steps)
        el = time.perf_counter() - t0
        print(json.dumps({"mode": a.mode, "rep": rep, "stagger": os.environ.get("I7M_ADMM_STAGGER", "default"), "torch_stream": a.torch_stream,
                          "instance_steps_per_s": a.B * a.steps / el, "ms_per_mpc_step": 1e3 * el / a.steps,
                          "alive_at_end": int(np.isfinite(d[-1]).sum())}), flush=True)
    h.close()


if __name__ == "__main__":
    main()
