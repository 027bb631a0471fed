"""Multi-rank check of the sharded path on ONE GPU (tests/test_gpu_multiproc.py runs it as a
fresh child process): W ranks are spawned (torch.multiprocessing, gloo process group as in
bench.py), each creates its own library handle on device 0 and solves its contiguous shard
(sharding.shard_range) of one batch, `--calls` times in a row (each call fed the previous one's
output, as an MPC loop does); this process (which has not touched the GPU before the ranks
finish) then solves the whole batch the same way in one handle and checks that the concatenation
of the ranks' outputs equals it bit for bit, call by call.

--qp-mode admm (the drop-in default, as OSQPSolver / batch_sqp / ShardedSQP): every problem's
OSQP state (x, z, y, the previous q, rho) lives in its rank's handle and is carried from call to
call; the check then also covers the OSQP iteration records and statuses of every call and the
carried state after the last one, rank rows against the single handle's rows.  A handle's ADMM
state is limited to 2 GiB (16 670 problems at N = 32), so the single-handle side of a larger
batch runs as the fewest contiguous pieces that fit (config 5: two 16384-problem handles), each
itself a different split of the batch than the ranks'.

With --port every problem is also solved by the C++ CPU port (oracle/cpp/i7m_cpu.cpp, test
infrastructure; its ADMM mode carries its own state over the same calls, fed the GPU's outputs):
alpha sequences, SQP iterations (and, in ADMM mode, OSQP iterations and statuses) identical, XU
within 1e-9 (direct) / 5e-8 (ADMM, tests/test_gpu_admm.py's tolerance) relative.  Prints one JSON
line; exit status 0 iff everything holds.

    python tools/shard_ranks.py [--world 2] [--batch 96] [--N 32] [--seed 45] [--qp-mode admm]
                                [--calls 2] [--port]

Config 5: --world 8 --batch 32768 --N 32 --seed 47 --port.
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _mode(lib, name):
    return lib.QP_ADMM if name == "admm" else lib.QP_DIRECT


def _solve_calls(h, xcur, goals, XU, calls, admm):
    """`calls` consecutive solves on one handle: per call (out, stats[, OSQP iterations, statuses]);
    ADMM mode also the carried state after the last call."""
    recs, xin = [], XU
    for _ in range(calls):
        out, st = h.solve(xcur, goals, xin)
        rec = {"out": out, "qp_iters": st["qp_iters"], "alphas": st["alphas"], "n_alphas": st["n_alphas"]}
        if admm:
            its, _, stat = h.admm_stats(len(out), with_status=True)
            rec.update(osqp_iters=its, status=stat)
        recs.append(rec)
        xin = out
    state = h.admm_state(len(XU)) if admm else None
    return recs, state


def _rank(r, world, port, B, N, seed, qp_mode, calls, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world))
    import numpy as np
    import torch.distributed as dist

    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from indy7_mpc_amd.sharding import shard_range
    from oracle.osqp_ref import synthetic_batch

    dist.init_process_group("gloo", rank=r, world_size=world)
    xcur, goals, XU = synthetic_batch(B, N, seed=seed)
    lo, hi = shard_range(B, r, world)
    admm = qp_mode == "admm"
    h = _lib.Handle(default_model(), N=N, max_batch=max(hi - lo, 1), device_id=0, qp_mode=_mode(_lib, qp_mode))
    dist.barrier()
    recs, state = _solve_calls(h, xcur[lo:hi], goals[lo:hi], XU[lo:hi], calls, admm)
    arrs = {f"{k}_{c}": v for c, rec in enumerate(recs) for k, v in rec.items()}
    if admm:
        arrs.update({f"state_{i}": a for i, a in enumerate(state)})
    np.savez(os.path.join(out_dir, f"rank{r}.npz"), lo=lo, hi=hi, **arrs)
    h.close()
    dist.barrier()
    dist.destroy_process_group()


def _single(lib, model, xcur, goals, XU, N, qp_mode, calls):
    """The whole batch on one handle (ADMM mode: the fewest contiguous pieces whose state fits a
    handle's 2 GiB), call by call; returns (records, state, piece ranges)."""
    import numpy as np

    B = len(XU)
    admm = qp_mode == "admm"
    pieces = 1
    while True:
        from indy7_mpc_amd.sharding import shard_ranges

        rngs = shard_ranges(B, pieces)
        try:
            h = lib.Handle(model, N=N, max_batch=max(hi - lo for lo, hi in rngs), device_id=0,
                           qp_mode=_mode(lib, qp_mode))
            break
        except lib.I7MError as e:
            if "2 GiB" not in str(e):
                raise
            pieces *= 2
    parts = []
    for lo, hi in rngs:
        h.reset()
        parts.append(_solve_calls(h, xcur[lo:hi], goals[lo:hi], XU[lo:hi], calls, admm))
    h.close()
    recs = [{k: np.concatenate([p[0][c][k] for p in parts]) for k in parts[0][0][c]} for c in range(calls)]
    state = tuple(np.concatenate([p[1][i] for p in parts]) for i in range(5)) if admm else None
    return recs, state, rngs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--batch", type=int, default=96)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--seed", type=int, default=45)
    ap.add_argument("--qp-mode", choices=("admm", "direct"), default="admm")
    ap.add_argument("--calls", type=int, default=None, help="consecutive solves (default: 2 in ADMM mode, 1 direct)")
    ap.add_argument("--port", action="store_true", help="also compare every problem with the C++ CPU port")
    a = ap.parse_args()
    calls = a.calls or (2 if a.qp_mode == "admm" else 1)
    admm = a.qp_mode == "admm"
    import numpy as np
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_rank, args=(a.world, port, a.batch, a.N, a.seed, a.qp_mode, calls, td), nprocs=a.world, join=True)
        parts = [dict(np.load(os.path.join(td, f"rank{r}.npz"))) for r in range(a.world)]
    t_ranks = time.perf_counter() - t0
    keys = ["out", "qp_iters", "alphas", "n_alphas"] + (["osqp_iters", "status"] if admm else [])
    got = [{k: np.concatenate([p[f"{k}_{c}"] for p in parts]) for k in keys} for c in range(calls)]
    ranges = [(int(p["lo"]), int(p["hi"])) for p in parts]
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from oracle.osqp_ref import synthetic_batch

    xcur, goals, XU = synthetic_batch(a.batch, a.N, seed=a.seed)
    ref, ref_state, pieces = _single(_lib, default_model(), xcur, goals, XU, a.N, a.qp_mode, calls)
    ok = all(np.array_equal(g[k], r[k]) for g, r in zip(got, ref) for k in keys)
    res = {"world": a.world, "batch": a.batch, "N": a.N, "seed": a.seed, "qp_mode": a.qp_mode, "calls": calls,
           "ranges": ranges, "single_handle_pieces": [list(p) for p in pieces], "equal": ok,
           "max_abs_diff": float(max(np.abs(g["out"] - r["out"]).max() for g, r in zip(got, ref))),
           "ranks_wall_s": t_ranks}
    if admm:
        st_eq = all(np.array_equal(np.concatenate([p[f"state_{i}"] for p in parts]), ref_state[i]) for i in range(5))
        res["state_equal"] = st_eq
        res["osqp_iters_per_qp_mean"] = float(got[0]["osqp_iters"][got[0]["osqp_iters"] > 0].mean())
        ok = ok and st_eq
    if a.port:
        from oracle import cpu

        nt = min(16, os.cpu_count() or 1)
        st = cpu.AdmmState(a.batch, a.N) if admm else None
        xin, agg = XU, {"alpha_sequence_agreement": 1.0, "qp_iters_agreement": 1.0, "xu_rel_err_max": 0.0}
        if admm:
            agg.update(osqp_iters_agreement=1.0, status_agreement=1.0)
        for c in range(calls):
            g = got[c]
            if admm:
                pref, pqp, pal, _, pit = cpu.solve_admm(xcur, goals, xin, a.N, st, nthreads=nt)
            else:
                pref, pqp, pal, _ = cpu.solve(xcur, goals, xin, a.N, nthreads=nt)
            used_g = np.arange(pal.shape[1])[None, :] < g["n_alphas"][:, None]
            same_alpha = np.all(used_g == ~np.isnan(pal), axis=1) & np.all(
                np.where(used_g, g["alphas"][:, :pal.shape[1]] == pal, True), axis=1)
            rel = np.linalg.norm(g["out"] - pref, axis=1) / np.maximum(np.linalg.norm(pref, axis=1), 1e-300)
            agg["alpha_sequence_agreement"] = min(agg["alpha_sequence_agreement"], float(same_alpha.mean()))
            agg["qp_iters_agreement"] = min(agg["qp_iters_agreement"], float((g["qp_iters"] == pqp).mean()))
            agg["xu_rel_err_max"] = max(agg["xu_rel_err_max"], float(rel.max()))
            if admm:
                ran = np.arange(8)[None, :] < pqp[:, None]
                agg["osqp_iters_agreement"] = min(agg["osqp_iters_agreement"], float(
                    np.all(np.where(ran, g["osqp_iters"] == pit, True), axis=1).mean()))
                agg["status_agreement"] = min(agg["status_agreement"], float(
                    np.all(np.where(ran, g["status"] == st.status, True), axis=1).mean()))
            xin = g["out"]
        res["port"] = agg
        tol = 5e-8 if admm else 1e-9
        ok = ok and agg["alpha_sequence_agreement"] == 1.0 and agg["qp_iters_agreement"] == 1.0 and \
            agg["xu_rel_err_max"] <= tol and (not admm or (agg["osqp_iters_agreement"] == 1.0 and
                                                          agg["status_agreement"] == 1.0))
    print(json.dumps(res))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
