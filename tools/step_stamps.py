"""Where one sweep step of k_admm_iter spends its cycles (diagnostic library, I7M_ABLATE
100000 + 100 IT + S: s_memtime stamps at nine points of step S of OSQP iteration IT in
workgroup 0, written to the timeline buffer's record area 5).  Segments, in shader cycles:
wait (the slot's DMA), dma (issuing step S + 2's), lds (the step's vector and first coefficient
reads issued), pre (right-hand side, J' u), lmul (Linv r), ltmul (Linv' y), st (stores), jmul
(the coupling J h / the block's rows).  The stamps fence the schedule and drain LDS reads: read
the shares, not the total.

    I7M_LIB=indy7_mpc_amd/lib/libindy7mpc_diag.so python tools/step_stamps.py [--B 1] [--it 3]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SEG = ["wait", "dma", "lds", "pre", "lmul", "ltmul", "st", "jmul"]
# k_admm_iter_res (launches of <= 256 problems): no ring, so no wait or DMA segment; its fifth and
# sixth segments are the stores then J h (forward) or J xt then the rows' update and stores (backward)
SEG_RES = ["lds", "pre", "lmul", "ltmul", "st|jmul", "jmul|upd+st"]
# k_admm_factor (--factor: stage S of workgroup 0): the stage's operands and J staged, S formed,
# the Cholesky, L written back, the inverse and the record stored, C_k
SEG_FAC = ["wait+J", "S", "chol", "Lwrite", "inv+store", "Ck"]
# k_admm_scale (--scale: Ruiz pass S of workgroup 0): the stage owners' v-row maxima, the column
# norms, the row norms, D / E / q updated, the cost normalisation
SEG_SCL = ["reg", "cols", "rows", "update", "cost"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--it", type=int, default=3)
    ap.add_argument("--steps", default="1,2,5,10,20,30,31,33,34,35,40,50,60,63")
    ap.add_argument("--factor", action="store_true", help="stamp the factor's stage S instead of a sweep step")
    ap.add_argument("--scale", action="store_true", help="stamp the scaling's Ruiz pass S instead of a sweep step")
    a = ap.parse_args()
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    lib = _lib.load()
    if not hasattr(lib, "i7m_diag_timeline"):
        raise SystemExit("needs the diagnostic library (I7M_LIB=.../libindy7mpc_diag.so)")
    lib.i7m_diag_timeline.argtypes = [C.c_void_p]
    model = default_model()
    dev = torch.device("cuda", 0)
    cap = 6 << 16
    buf = torch.zeros(8 + 4 * cap, dtype=torch.int64, device=dev)
    buf[1] = cap
    base = 8 + 4 * (5 << 16)
    rows = []
    for S in [int(x) for x in a.steps.split(",")]:
        os.environ["I7M_ABLATE"] = str(300000 + S if a.scale else (200000 + S if a.factor else 100000 + 100 * a.it + S))
        h = _lib.Handle(model, N=a.N, max_batch=a.B, max_sqp_iters=1, qp_mode=_lib.QP_ADMM)
        os.environ.pop("I7M_ABLATE")
        xcur, goals, XU = make_batch(h, model, a.B, a.N, seed=44)
        t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
        t_out = torch.empty_like(t_xu)
        for rep in range(3):
            buf[base:base + 16] = 0
            if lib.i7m_diag_timeline(C.c_void_p(buf.data_ptr())) != 0:
                raise SystemExit("i7m_diag_timeline failed")
            h.admm_reset(a.B)
            h.solve_device(a.B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), None)
            torch.cuda.synchronize(dev)
            lib.i7m_diag_timeline(C.c_void_p(0))
        t = buf[base:base + 11].cpu().tolist()
        h.close()
        res, fac, scl = t[10] == 1, t[10] == 2, t[10] == 3
        ns = 5 if scl else (6 if (res or fac) else 8)
        d = [t[i + 1] - t[i] if t[i + 1] and t[i] else None for i in range(ns)]
        kind = "fwd" if S < a.N - 1 else ("fwd_last" if S == a.N - 1 else ("turn" if S == a.N else "bwd"))
        if fac or scl:
            kind = "factor stage" if fac else "Ruiz pass"
        r = {"B": a.B, "it": a.it, "step": S, "kind": kind, "tag": t[9],
             "kernel": "scale" if scl else ("factor" if fac else ("res" if res else "streaming")),
             "cycles": dict(zip(SEG_SCL if scl else (SEG_FAC if fac else (SEG_RES if res else SEG)), d)),
             "total": (t[ns] - t[0]) if t[ns] and t[0] else None}
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
