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


def _admm_line_rank_main(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import json
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    B, N, steps = 4096, 32, 20
    own = 0.2 + 0.01 * rank  # this rank's barrier-to-barrier time of pass 1
    t = torch.tensor([own], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.Leg.timed's reduction
    rows = bench.gather_rank_rows(dist, rank, own, 3.0e5)
    # what pass 2 of the ADMM leg records: two staggered ranges x two SQP iterations per step
    it = np.full((B, 8), -1, dtype=np.int32)
    it[:, 0] = 25
    it[: B // 2, 1] = 50
    kt = {"k_admm_iter": (steps * 4 * 3.0, steps * 4), "k_admm_prep": (steps * 4 * 1.0, steps * 4),
          "k_linearize": (steps * 4 * 0.05, steps * 4)}
    roof = bench.admm_roofline(kt, steps, it, B, N, float(t.item()) / steps)
    line = bench.headline_line(value=B * world * steps / float(t.item()), elapsed=float(t.item()), steps=steps,
                               warmup=3, world=world, B=B, N=N, seed=47, devs=[r[0] for r in rows],
                               step_ms=[10.0] * steps, ktimes=kt, roofline=roof,
                               osqp_iters=bench.osqp_iter_summary(it), qp_iters_mean=1.5, el_ev=0.21,
                               rank_rows=rows)
    if rank == 0:
        with open(os.path.join(out_dir, "line.json"), "w") as f:
            json.dump(line, f)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_admm_leg_line_keys_two_ranks(tmp_path):
    """bench.py's multi-rank line in the drop-in default mode (ADMM, config 5): world size 2 under
    gloo as `bench.py --gpus 2` runs its ranks — value from the max over ranks, qp_mode "admm" and
    the cold-state definition in config, k_admm_iter's roofline with its factor stream and the
    staggered launch's traffic key, per_rank rows."""
    import json

    world = 2
    port = 29500 + (os.getpid() + 13) % 1000
    mp.spawn(_admm_line_rank_main, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    d = json.load(open(tmp_path / "line.json"))
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["unit"] == "solves/s" and d["dtype"] == "f64"
    assert d["value"] == pytest.approx(4096 * 2 * 20 / 0.21)
    assert d["config"]["qp_mode"] == "admm" and d["config"]["workload"].startswith("config5: B=8192")
    assert "cold" in d["config"]["osqp_state"] and d["config"]["global_batch"] == 8192
    r = d["roofline"]
    assert r["kernel"] == "k_admm_iter" and r["traffic_key"] == "k_admm_iter:B2048:N32:stagger"
    assert r["launches_per_step"] == 4 and r["problems_per_launch"] == pytest.approx((4096 + 2048) / 4)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0)
    assert r["factor_stream"]["osqp_iters_per_launch"] == pytest.approx((4096 * 25 + 2048 * 50) / 4)
    assert d["osqp_iters_per_qp"]["max"] == 50
    assert [x["rank"] for x in d["per_rank"]["ranks"]] == [0, 1]
    assert d["per_rank"]["elapsed_s"]["max"] == pytest.approx(0.21)
