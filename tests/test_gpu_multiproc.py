"""GPU: the multi-rank sharded path for real — several processes, each with its own library
handle on the one GPU, solving contiguous shards (sharding.shard_range, as bench.py's ranks do);
their concatenated outputs must equal the single-process solve bit for bit.

The ranks are spawned by a fresh child process (tools/shard_ranks.py) that has not touched the
GPU, so no GPU-initialised process forks ranks.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,batch,mode", [(2, 96, "admm"), (3, 50, "admm"), (2, 96, "direct")])
def test_ranks_on_shards_equal_single_process(world, batch, mode):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shard_ranks.py"), "--world", str(world),
                        "--batch", str(batch), "--qp-mode", mode], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["equal"] and len(res["ranges"]) == world and res["qp_mode"] == mode
    assert res["ranges"][0][0] == 0 and res["ranges"][-1][1] == batch
    if mode == "admm":
        assert res["calls"] == 2 and res["state_equal"]


@pytest.mark.timeout(540)
@pytest.mark.parametrize("mode", ["admm", "direct"])
def test_config5_eight_shards_equal_single_handle_and_port(mode):
    """SURVEY.md §8d config 5 (B = 32768, N = 32, seed 47) as 8 ranks x 4096 — bench.py's
    `--gpus 8` sharding — here all on the one GPU, in the drop-in default (ADMM: OSQP's iteration,
    each problem's OSQP state carried in its rank's handle over two consecutive calls) and in the
    exact mode.  The concatenated shards equal the single-handle solve bit for bit (ADMM: call by
    call, OSQP iteration records, statuses and the carried state included; the single-handle side
    is two 16384-problem handles, the most a handle's 2 GiB of ADMM state holds at N = 32), and all
    32768 problems match the C++ CPU port: alpha sequences, SQP iterations (ADMM: OSQP iterations
    and statuses) identical, XU <= 1e-9 (direct) / 5e-8 (ADMM) relative (SURVEY.md 8d's gate is 1e-4)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shard_ranks.py"), "--world", "8",
                        "--batch", "32768", "--N", "32", "--seed", "47", "--qp-mode", mode, "--port"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["equal"] and len(res["ranges"]) == 8
    assert all(hi - lo == 4096 for lo, hi in res["ranges"])
    assert res["port"]["alpha_sequence_agreement"] == 1.0 and res["port"]["qp_iters_agreement"] == 1.0
    if mode == "admm":
        assert res["calls"] == 2 and res["state_equal"] and len(res["single_handle_pieces"]) == 2
        assert res["port"]["osqp_iters_agreement"] == 1.0 and res["port"]["status_agreement"] == 1.0
        assert res["port"]["xu_rel_err_max"] <= 5e-8
    else:
        assert res["port"]["xu_rel_err_max"] <= 1e-9
