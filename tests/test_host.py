"""CPU: host-side logic of the package (no GPU compute): URDF parsing, packed model layout,
CSC value assembly in the reference's order, sharding arithmetic, stats bookkeeping."""
import os

import numpy as np
import pytest

from indy7_mpc_amd.model import RobotModel, default_model, parse_urdf
from indy7_mpc_amd.osqp_solver import assemble_A, assemble_P
from indy7_mpc_amd.sharding import shard_range, shard_ranges
from oracle import rbd
from oracle.osqp_ref import OSQPSolverRef, synthetic_batch

URDF = "/root/reference/description/indy7.urdf"


def test_model_surface(model):
    assert model.nq == model.nv == 6
    assert len(model.joints) - 1 == 6  # nu as src/osqp_solver.py:20 computes it
    np.testing.assert_array_equal(model.gravity.linear, [0, 0, -9.81])
    assert model.packed().shape == (159,)
    d = model.createData()
    assert len(d.oMi) == model.njoints


@pytest.mark.skipif(not os.path.exists(URDF), reason="reference URDF only in the build container")
def test_urdf_parse_matches_committed_params():
    p = parse_urdf(URDF)
    assert np.array_equal(RobotModel(p).packed(), default_model().packed())


def test_model_rejects_non_z_axis(tmp_path):
    urdf = tmp_path / "bad.urdf"
    urdf.write_text("""<robot name="r"><link name="a"/><link name="b"/>
      <joint name="j" type="revolute"><parent link="a"/><child link="b"/><axis xyz="1 0 0"/>
      <limit lower="-1" upper="1" effort="1" velocity="1"/></joint></robot>""")
    with pytest.raises(ValueError):
        parse_urdf(str(urdf))


def _device_format_lin(xu, N):
    """The device linearisation layout (Aq | Av | Bu | a per knot) built with the oracle."""
    lin = np.zeros((N - 1, 114))
    dt = 0.01
    for k in range(N - 1):
        q, v, u = xu[18 * k:18 * k + 6], xu[18 * k + 6:18 * k + 12], xu[18 * k + 12:18 * k + 18]
        dq, dv, Mi, a = rbd.aba_derivatives(q, v, u)
        lin[k, :36] = (dt * dq).reshape(-1)
        lin[k, 36:72] = (np.eye(6) + dt * dv).reshape(-1)
        lin[k, 72:108] = (dt * Mi).reshape(-1)
        lin[k, 108:] = a
    return lin


def _device_format_cost(xu, goals, N, dQ=0.01, R=1e-5, QN=100.0, eps=1.0):
    cost = np.zeros((N, 10))
    for k in range(N):
        p, J = rbd.d_eepos(xu[18 * k:18 * k + 6])
        e = p - goals[3 * k:3 * k + 3]
        w = 1.0 / (np.linalg.norm(e) + eps)
        cost[k, :6] = e @ J
        cost[k, 6] = QN if k == N - 1 else 1.0
        cost[k, 7] = dQ * w
        cost[k, 8] = R * w
        cost[k, 9] = np.linalg.norm(e)
    return cost


def test_csc_assembly_matches_reference_order():
    N = 16
    xcur, goals, XU = synthetic_batch(1, N, seed=21)
    xu = XU[0] + np.random.default_rng(0).normal(0, 0.2, XU.shape[1])
    s = OSQPSolverRef(N=N)
    s.update_constraint_matrix(xu, xcur[0])
    s.update_cost_matrix(xu, goals[0])
    Adata, l = assemble_A(_device_format_lin(xu, N), xu, xcur[0], 0.01, N)
    Pdata, g = assemble_P(_device_format_cost(xu, goals[0], N), xu, N)
    np.testing.assert_allclose(Adata, s.Adata, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(l, s.l, rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(Pdata, s.Pdata, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(g, s.g, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("B,world", [(0, 1), (1, 1), (7, 2), (32768, 8), (5, 8), (4097, 3)])
def test_shard_ranges_partition(B, world):
    rs = shard_ranges(B, world)
    assert rs[0][0] == 0 and rs[-1][1] == B
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c
    sizes = [b - a for a, b in rs]
    assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(B, world, world)


def test_stats_recording_layout():
    """SQP_OSQP._record turns device stats rows into the reference's stats lists."""
    from indy7_mpc_amd import _lib
    from indy7_mpc_amd.osqp_sqp import SQP_OSQP

    st = np.zeros(2, dtype=_lib.STATS_DTYPE)
    st[0]["qp_iters"], st[0]["n_alphas"], st[0]["n_steps"] = 2, 2, 2
    st[0]["alphas"][:2] = [0.125, 0.015625]
    st[0]["stepsizes"][:2] = [27.1, 2.8]
    st[1]["qp_iters"], st[1]["n_alphas"], st[1]["n_steps"] = 1, 1, 1
    st[1]["alphas"][0] = 1.0
    st[1]["stepsizes"][0] = 1e-4

    class _S:
        pass

    sq = SQP_OSQP(_S())
    sq._record(st)
    s = sq.get_stats()
    assert s["qp_iters"]["values"] == [2, 1]
    assert s["linesearch_alphas"]["values"] == [0.125, 0.015625, 1.0]
    assert s["sqp_stepsizes"]["values"] == [27.1, 2.8, 1e-4]
    assert set(s) == {"qp_iters", "linesearch_alphas", "sqp_stepsizes"}


def test_bench_refuses_more_ranks_than_devices():
    """bench.py --gpus N without a launcher starts N ranks itself only when N devices are
    visible (or --share-devices asks for a rehearsal); here there is no GPU, so it refuses with
    exit status 2 before starting anything (no silently shared devices)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--share-devices" in r.stderr
