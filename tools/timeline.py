"""Per-wave timeline of one solve (diagnostic library, i7m_timeline.h): how each launch's waves
spread over the SIMDs and how long each SIMD sat idle inside the launch (load imbalance, tails).

    I7M_LIB=indy7_mpc_amd/lib/libindy7mpc_diag.so python tools/timeline.py [--B 4096] [--N 32] [--box]

Per launch (kernel, in stream order): span (first wave start to last wave end), waves, SIMDs
used, max waves resident per SIMD, wave duration p10 / p50 / p90 / max, `busy` = summed per-SIMD
busy time (union of its waves' intervals) / (SIMDs x span), and `tail` = span minus the time at
which 90 % of the SIMDs had finished their last wave.  Times in microseconds (100 MHz clock).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KNAMES = {1: "k_linearize", 2: "k_riccati", 3: "k_linesearch", 4: "k_ipm_fused"}


def analyse(rec):
    t0, t1, hw, kw = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64), rec[:, 2], rec[:, 3]
    kid = (kw & 0xFF).astype(int)
    # SIMD identity: XCC (hi word) + HW_ID bits 4..15 (simd, pipe, cu, sh, se); wave slot bits 0..3 dropped
    simd = ((hw >> 32) << 16) | (hw & 0xFFF0)
    order = np.argsort(t0, kind="stable")
    # launches: consecutive runs of one kernel id in start order (a stream runs them in turn)
    launches, cur = [], [order[0]]
    for i in order[1:]:
        if kid[i] != kid[cur[-1]]:
            launches.append(cur)
            cur = []
        cur.append(i)
    launches.append(cur)
    out = []
    for L in launches:
        L = np.asarray(L)
        s0, s1 = t0[L].min(), t1[L].max()
        span = (s1 - s0) / 100.0
        dur = (t1[L] - t0[L]) / 100.0
        busy, last_end, maxres = 0.0, [], 0
        for sid in np.unique(simd[L]):
            M = L[simd[L] == sid]
            iv = sorted(zip(t0[M], t1[M]))
            # union of intervals and the largest number resident at once
            u, ce, cs = 0, None, None
            ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv], key=lambda e: (e[0], e[1]))
            r = 0
            for _, d in ev:
                r += d
                maxres = max(maxres, r)
            for a, b in iv:
                if ce is None or a > ce:
                    if ce is not None:
                        u += ce - cs
                    cs, ce = a, b
                else:
                    ce = max(ce, b)
            u += ce - cs
            busy += u / 100.0
            last_end.append((max(b for _, b in iv) - s0) / 100.0)
        ns = len(last_end)
        out.append({
            "kernel": KNAMES.get(int(kid[L[0]]), str(kid[L[0]])), "span_us": round(span, 2), "waves": int(len(L)),
            "simds": ns, "max_resident": maxres,
            "wave_us": [round(float(np.percentile(dur, p)), 2) for p in (10, 50, 90)] + [round(float(dur.max()), 2)],
            "busy": round(busy / (ns * span), 3),
            "tail_us": round(span - float(np.percentile(last_end, 90)), 2),
            "simd_last_end_us_p10_p50": [round(float(np.percentile(last_end, p)), 2) for p in (10, 50)],
        })
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--box", action="store_true")
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    import torch
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.synthetic import make_batch

    lib = _lib.load()
    if not hasattr(lib, "i7m_diag_timeline"):
        raise SystemExit("load the diagnostic library (I7M_LIB=.../libindy7mpc_diag.so)")
    lib.i7m_diag_timeline.argtypes = [C.c_void_p]
    model = default_model()
    kw = {"qp_mode": _lib.QP_BOX} if a.box else {}
    # one SQP iteration: the record buffer holds one launch per kernel (i7m_timeline.h)
    h = _lib.Handle(model, N=a.N, max_batch=a.B, max_sqp_iters=1, **kw)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    h.set_stream(s.cuda_stream)
    xcur, goals, XU = make_batch(h, model, a.B, a.N, seed=46 if a.box else 45)
    t_xu, t_xs, t_g = (torch.from_numpy(x).to(dev) for x in (XU, xcur, goals))
    t_out = torch.empty_like(t_xu)

    def step():
        h.solve_device(a.B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), None)

    for _ in range(3):
        step()
    cap = 5 << 16
    buf = torch.zeros(8 + 4 * cap, dtype=torch.int64, device=dev)
    buf[1] = cap
    torch.cuda.synchronize(dev)
    if lib.i7m_diag_timeline(C.c_void_p(buf.data_ptr())) != 0:
        raise SystemExit("i7m_diag_timeline failed")
    step()
    torch.cuda.synchronize(dev)
    lib.i7m_diag_timeline(C.c_void_p(0))
    rec = buf[8:].view(-1, 4).cpu().numpy().astype(np.uint64)
    rec = rec[rec[:, 1] != 0]
    n = len(rec)
    if a.dump:
        np.save(a.dump, rec)
    res = analyse(rec)
    print(json.dumps({"B": a.B, "N": a.N, "box": a.box, "records": n, "launches": res}))
    for r in res:
        print(json.dumps(r), file=sys.stderr)


if __name__ == "__main__":
    main()
