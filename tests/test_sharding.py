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
