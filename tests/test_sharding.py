"""CPU, world_size 2 (gloo): the multi-GPU path shards the batch into contiguous ranges with
no data-path collective; per-rank results concatenated == the single-process result.  The
per-rank compute here is the oracle (no GPU in this container); the GPU version of the same
check is tests/test_gpu_solver.py::test_sharded_solver_matches_single."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _rank_main(rank, world, port, N, B, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from indy7_mpc_amd.sharding import shard_range
    from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch

    xcur, goals, XU = synthetic_batch(B, N, seed=77)
    lo, hi = shard_range(B, rank, world)
    outs = np.stack([SQPRef(OSQPSolverRef(N=N)).sqp(xcur[b], goals[b], XU[b].copy()) for b in range(lo, hi)])
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), outs)
    # the bench's timing reduction: max over ranks
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert t.item() == world
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_process(tmp_path):
    N, B, world = 16, 5, 2
    port = 29500 + os.getpid() % 1000
    mp.spawn(_rank_main, args=(world, port, N, B, str(tmp_path)), nprocs=world, join=True)
    from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch

    xcur, goals, XU = synthetic_batch(B, N, seed=77)
    single = np.stack([SQPRef(OSQPSolverRef(N=N)).sqp(xcur[b], goals[b], XU[b].copy()) for b in range(B)])
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    np.testing.assert_array_equal(got, single)


def _bench_rank_main(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    rows = bench.gather_rank_rows(dist, rank % 1, 0.1 * (rank + 1), 1000.0 * (rank + 1))
    if rank == 0:
        with open(os.path.join(out_dir, "per_rank.json"), "w") as f:
            json.dump(bench.per_rank_summary(rows, 4096, 20), f)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_per_rank_keys_two_ranks(tmp_path):
    """bench.py's multi-rank line carries per-rank elapsed (min / median / max) and per-rank
    solve and host-to-host rates: the gather and the summary under gloo,
    world size 2, as the ranks of `bench.py --gpus 2` run them."""
    import json

    world = 2
    port = 29500 + (os.getpid() + 7) % 1000
    mp.spawn(_bench_rank_main, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    d = json.load(open(tmp_path / "per_rank.json"))
    assert d["elapsed_s"] == {"min": 0.1, "median": pytest.approx(0.15), "max": 0.2}
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    assert d["ranks"][1]["host_to_host_solves_per_s"] == 2000.0
    assert d["ranks"][0]["solves_per_s"] == pytest.approx(4096 * 20 / 0.1)
    assert set(d["ranks"][0]) == {"rank", "device", "elapsed_s", "solves_per_s", "host_to_host_solves_per_s"}
