"""Multi-rank check of the sharded path on ONE GPU (tests/test_gpu_multiproc.py runs it as a
fresh child process): W ranks are spawned (torch.multiprocessing, gloo process group as in
bench.py), each creates its own library handle on device 0 and solves its contiguous shard
(sharding.shard_range) of one batch; this process (which has not touched the GPU before the
ranks finish) then solves the whole batch in one handle and checks that the concatenation of the
ranks' outputs equals it bit for bit.  With --port it also solves the whole batch with the C++
CPU port (oracle/cpp/i7m_cpu.cpp, test infrastructure) and reports the alpha-sequence agreement,
the SQP iteration agreement and the largest per-problem XU relative error.  Prints one JSON
line; exit status 0 iff the sharded and single-handle solves are equal (and, with --port, the
port agrees: alphas and iterations identical, XU <= 1e-9 relative).

    python tools/shard_ranks.py [--world 2] [--batch 96] [--N 32] [--seed 45] [--port]

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


def _rank(r, world, port, B, N, seed, out_dir):
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
    h = _lib.Handle(default_model(), N=N, max_batch=max(hi - lo, 1), device_id=0)
    dist.barrier()
    out, st = h.solve(xcur[lo:hi], goals[lo:hi], XU[lo:hi])
    np.savez(os.path.join(out_dir, f"rank{r}.npz"), out=out, qp_iters=st["qp_iters"], alphas=st["alphas"],
             n_alphas=st["n_alphas"], lo=lo, hi=hi)
    h.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--batch", type=int, default=96)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--seed", type=int, default=45)
    ap.add_argument("--port", action="store_true", help="also compare every problem with the C++ CPU port")
    a = ap.parse_args()
    import numpy as np
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_rank, args=(a.world, port, a.batch, a.N, a.seed, td), nprocs=a.world, join=True)
        parts = [np.load(os.path.join(td, f"rank{r}.npz")) for r in range(a.world)]
        out = np.concatenate([p["out"] for p in parts])
        qp = np.concatenate([p["qp_iters"] for p in parts])
        al = np.concatenate([p["alphas"] for p in parts])
        na = np.concatenate([p["n_alphas"] for p in parts])
        ranges = [(int(p["lo"]), int(p["hi"])) for p in parts]
    t_ranks = time.perf_counter() - t0
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.model import default_model
    from oracle.osqp_ref import synthetic_batch

    xcur, goals, XU = synthetic_batch(a.batch, a.N, seed=a.seed)
    h = _lib.Handle(default_model(), N=a.N, max_batch=a.batch, device_id=0)
    ref, st = h.solve(xcur, goals, XU)
    h.close()
    ok = bool(np.array_equal(out, ref) and np.array_equal(qp, st["qp_iters"]) and np.array_equal(al, st["alphas"]))
    res = {"world": a.world, "batch": a.batch, "N": a.N, "seed": a.seed, "ranges": ranges, "equal": ok,
           "max_abs_diff": float(np.abs(out - ref).max()) if out.shape == ref.shape else None,
           "ranks_wall_s": t_ranks}
    if a.port:
        from oracle import cpu

        pref, pqp, pal, _ = cpu.solve(xcur, goals, XU, a.N, nthreads=min(16, os.cpu_count() or 1))
        used_g = np.arange(pal.shape[1])[None, :] < na[:, None]
        same_alpha = np.all(used_g == ~np.isnan(pal), axis=1) & np.all(
            np.where(used_g, al[:, :pal.shape[1]] == pal, True), axis=1)
        rel = np.linalg.norm(out - pref, axis=1) / np.maximum(np.linalg.norm(pref, axis=1), 1e-300)
        res["port"] = {"alpha_sequence_agreement": float(same_alpha.mean()),
                       "qp_iters_agreement": float((qp == pqp).mean()), "xu_rel_err_max": float(rel.max())}
        ok = ok and bool(same_alpha.all() and (qp == pqp).all() and rel.max() <= 1e-9)
    print(json.dumps(res))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
