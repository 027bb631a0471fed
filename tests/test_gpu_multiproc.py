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


@pytest.mark.parametrize("world,batch", [(2, 96), (3, 50)])
def test_ranks_on_shards_equal_single_process(world, batch):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shard_ranks.py"), "--world", str(world),
                        "--batch", str(batch)], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["equal"] and len(res["ranges"]) == world
    assert res["ranges"][0][0] == 0 and res["ranges"][-1][1] == batch


@pytest.mark.timeout(540)
def test_config5_eight_shards_equal_single_handle_and_port():
    """SURVEY.md §8d config 5 (B = 32768, N = 32, seed 47) as 8 ranks x 4096 — bench.py's
    `--gpus 8` sharding — here all on the one GPU: the concatenated shards equal one B = 32768
    handle's solve bit for bit, and all 32768 problems match the C++ CPU port (alpha sequences and
    SQP iteration counts identical, XU <= 1e-9 relative; SURVEY.md 8d's gate is 1e-4)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shard_ranks.py"), "--world", "8",
                        "--batch", "32768", "--N", "32", "--seed", "47", "--port"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["equal"] and len(res["ranges"]) == 8
    assert all(hi - lo == 4096 for lo, hi in res["ranges"])
    assert res["port"]["alpha_sequence_agreement"] == 1.0 and res["port"]["qp_iters_agreement"] == 1.0
    assert res["port"]["xu_rel_err_max"] <= 1e-9
