"""GPU edge cases beyond the bench shapes: ragged horizons (N not a power of two, which takes
k_linesearch's LDS-reduction path and short Riccati sweeps; N = 2 is the minimum), the other
cost options of OSQPSolver (regularize=False, another dt / costs), batch sizes 0 and 1, and
problems that differ wildly within one batch.  Each against the CPU oracle through the C-ABI.

Tolerances as in test_gpu_parity.py: QP 1e-8 relative vs the exact KKT solve; full SQP 1e-6
relative per problem with the alpha sequence and qp_iters identical.
"""
import numpy as np
import pytest

from oracle.osqp_ref import OSQPSolverRef, SQPRef, synthetic_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from indy7_mpc_amd import _lib
    _lib.load()
    if _lib.device_count() < 1:
        pytest.fail("no GPU visible but the gpu tests were requested")
    return _lib


def _check_sqp(out, st, xcur, goals, XU, **kw):
    for b in range(out.shape[0]):
        sq = SQPRef(OSQPSolverRef(**kw))
        ref = sq.sqp(xcur[b], goals[b], XU[b].copy())
        s = sq.get_stats()
        assert st["qp_iters"][b] == s["qp_iters"]["values"][0], b
        na = st["n_alphas"][b]
        np.testing.assert_array_equal(st["alphas"][b][:na], s["linesearch_alphas"]["values"])
        rel = np.linalg.norm(out[b] - ref) / np.linalg.norm(ref)
        assert rel < 1e-6, (b, rel)


@pytest.mark.parametrize("N", [2, 5, 20, 48])
def test_ragged_horizon_qp_and_sqp(lib, model, N):
    B = 3
    xcur, goals, XU = synthetic_batch(B, N, seed=100 + N)
    h = lib.Handle(model, N=N, max_batch=B)
    XUp = XU + np.random.default_rng(N).normal(0, 0.2, XU.shape)
    sol = h.qp(XUp, xcur, goals)
    for b in range(B):
        ref = OSQPSolverRef(N=N).setup_and_solve_qp(XUp[b], xcur[b], goals[b]).x
        assert np.linalg.norm(sol[b] - ref) / np.linalg.norm(ref) < 1e-8
        np.testing.assert_array_equal(sol[b][:12], xcur[b])
    out, st = h.solve(xcur, goals, XU)
    _check_sqp(out, st, xcur, goals, XU, N=N)


def test_cost_options(lib, model):
    N, B = 16, 3
    kw = dict(N=N, dt=0.02, dQ_cost=0.05, R_cost=1e-4, QN_cost=50.0, regularize=False)
    xcur, goals, XU = synthetic_batch(B, N, seed=5)
    h = lib.Handle(model, max_batch=B, **kw)
    out, st = h.solve(xcur, goals, XU)
    _check_sqp(out, st, xcur, goals, XU, **kw)


def test_batch_of_one_and_empty(lib, model):
    N = 32
    xcur, goals, XU = synthetic_batch(2, N, seed=9)
    h = lib.Handle(model, N=N, max_batch=2)
    out, st = h.solve(xcur[:1], goals[:1], XU[:1])
    _check_sqp(out, st, xcur[:1], goals[:1], XU[:1], N=N)
    e_out, e_st = h.solve(xcur[:0], goals[:0], XU[:0])
    assert e_out.shape == (0, XU.shape[1]) and e_st.shape == (0,)


def test_mixed_batch_extremes(lib, model):
    """A batch mixing a start at rest on its goal, a start at the joint limits with large
    velocities, and ordinary draws: each problem still equals its own oracle solve."""
    from oracle import rbd

    N, B = 32, 5
    xcur, goals, XU = synthetic_batch(B, N, seed=21)
    lim = rbd.params().q_upper
    # problem 0: at rest exactly on its goal
    g0 = rbd.eepos(xcur[0][:6])
    goals[0] = np.tile(g0, N)
    xcur[0][6:] = 0.0
    # problem 1: near the position limits, fast
    xcur[1][:6] = 0.95 * lim
    xcur[1][6:] = np.array([2.0, -2.0, 1.5, -1.5, 3.0, -3.0])
    for b in range(2):
        XU[b] = 0.0
        XU[b][:12] = xcur[b]
    h = lib.Handle(model, N=N, max_batch=B)
    out, st = h.solve(xcur, goals, XU)
    assert np.isfinite(out).all()
    _check_sqp(out, st, xcur, goals, XU, N=N)


@pytest.mark.parametrize("graph", ["0", "1"])
def test_device_solve_out_of_place(lib, model, graph, monkeypatch):
    """i7m_solve_device with xu_out != xu_in: the input is only read, every output row is
    written (including a row whose line search fails: problem 5 has NaN goals, so it must come
    back unchanged and leave its neighbours alone), and the result equals the in-place
    host-path solve; a second call on the same buffers gives the same answer (no state leaks
    through the in-kernel initialisation of the active flags and stats).  graph = "1": the
    solve captured once into a hipGraph and replayed (I7M_GRAPH=1), against direct launches."""
    import torch

    N, B = 32, 37
    xcur, goals, XU = synthetic_batch(B, N, seed=77)
    goals[5] = np.nan  # a poisoned problem: every merit is NaN, so no alpha is accepted
    monkeypatch.setenv("I7M_GRAPH", "0")
    h0 = lib.Handle(model, N=N, max_batch=B)
    ref, st_ref = h0.solve(xcur, goals, XU)
    h0.close()
    monkeypatch.setenv("I7M_GRAPH", graph)
    h = lib.Handle(model, N=N, max_batch=B)
    np.testing.assert_array_equal(ref[5], XU[5])  # returned unchanged (src/osqp_sqp.py:81-82)
    assert st_ref["alphas"][5][0] == 0.0
    others = np.arange(B) != 5
    assert np.isfinite(ref[others]).all()
    dev = torch.device("cuda", 0)
    t_xu, t_xs, t_g = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (XU, xcur, goals))
    t_out = torch.full_like(t_xu, float("nan"))
    t_st = torch.zeros(B * lib.STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    # torch filled the buffers on its current stream: order the solve after it;
    # the default stream is the null stream (0), which the handle's own blocking stream follows
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(3):
        h.solve_device(B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), t_st.data_ptr())
        torch.cuda.synchronize(dev)
        np.testing.assert_array_equal(t_out.cpu().numpy(), ref)
        np.testing.assert_array_equal(t_xu.cpu().numpy(), XU)
        st = np.frombuffer(t_st.cpu().numpy().tobytes(), dtype=lib.STATS_DTYPE)
        np.testing.assert_array_equal(st["qp_iters"], st_ref["qp_iters"])
        np.testing.assert_array_equal(st["alphas"], st_ref["alphas"])


@pytest.mark.parametrize("N", [32, 20, 64])
def test_linesearch_one_and_four_waves_agree(lib, model, N, monkeypatch):
    """k_linesearch with one wave per problem (the B > 256 path) and with four (the small-batch
    path: all candidates of a round spread over four waves) computes the same merits and the
    same first-accept alpha, so whole solves are bit-identical; N = 20 takes the non-power-of-2
    reduction, N = 64 one candidate per wave."""
    B = 9
    xcur, goals, XU = synthetic_batch(B, N, seed=300 + N)
    outs = []
    for nw in ("1", "4"):
        monkeypatch.setenv("I7M_LS_WAVES", nw)
        h = lib.Handle(model, N=N, max_batch=B)
        outs.append(h.solve(xcur, goals, XU))
        h.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1]["alphas"], outs[1][1]["alphas"])
    _check_sqp(outs[1][0], outs[1][1], xcur, goals, XU, N=N)


def test_release_library_refuses_ablation_knob(lib, model, monkeypatch):
    """I7M_ABLATE selects invalid-result timing kernels that exist only in the -DI7M_DIAG build:
    the shipping library refuses to create a handle while it is set (no silent wrong answers)."""
    assert "release" in lib.version()
    monkeypatch.setenv("I7M_ABLATE", "4")
    with pytest.raises(lib.I7MError, match="I7M_ABLATE"):
        lib.Handle(model, N=16)
    monkeypatch.delenv("I7M_ABLATE")
    lib.Handle(model, N=16).close()


def test_reset_and_wrench_clear_with_captured_graphs(lib, model, monkeypatch):
    """i7m_reset keeps results (the exact solve has no warm start) and the wrench; clearing the
    wrench afterwards must not replay a graph captured with the wrench kernels (I7M_GRAPH=1)."""
    monkeypatch.setenv("I7M_GRAPH", "1")
    N, B = 16, 5
    xcur, goals, XU = synthetic_batch(B, N, seed=23)
    f = np.random.default_rng(6).normal(0, 30, (B, 6))
    plain, _ = lib.Handle(model, N=N, max_batch=B).solve(xcur, goals, XU)
    h = lib.Handle(model, N=N, max_batch=B)
    h.set_external_wrench(f, "world")
    w1, _ = h.solve(xcur, goals, XU)
    h.reset()
    w2, _ = h.solve(xcur, goals, XU)
    np.testing.assert_array_equal(w1, w2)
    assert not np.array_equal(w1, plain)
    h.set_external_wrench(None)
    np.testing.assert_array_equal(h.solve(xcur, goals, XU)[0], plain)


def test_zero_step_accepts_alpha_one(lib, model):
    """A QP minimiser equal to XU (sol == XU): the reference's merit_new == basemerit exactly, so
    alpha = 1 is accepted (src/osqp_sqp.py:58-72).  The line-search hook (base evaluated by the
    candidate function) must agree."""
    N, B = 16, 3
    xcur, goals, XU = synthetic_batch(B, N, seed=19)
    XU = XU + np.random.default_rng(3).normal(0, 0.2, XU.shape)
    h = lib.Handle(model, N=N, max_batch=B)
    al = h.linesearch(XU, XU, goals)
    np.testing.assert_array_equal(al, np.ones(B))


@pytest.mark.parametrize("N,B", [(32, 5), (32, 300), (20, 7), (64, 3), (2, 4)])
def test_fused_pipelines_equal_split(lib, model, N, B):
    """k_sqp_fused (one launch per solve, and one per SQP iteration) runs the same bodies as the
    three-kernel path, so its solves are bit-identical to it; B <= 256 takes the 4-wave
    workgroups, B = 300 the 1-wave ones; a few problems also against the oracle."""
    xcur, goals, XU = synthetic_batch(B, N, seed=400 + N + B)
    outs = {}
    for pipe in (lib.PIPE_SPLIT, lib.PIPE_FUSED, lib.PIPE_FUSED_ITER):
        h = lib.Handle(model, N=N, max_batch=B, pipeline=pipe)
        outs[pipe] = h.solve(xcur, goals, XU)
        h.close()
    for pipe in (lib.PIPE_FUSED, lib.PIPE_FUSED_ITER):
        np.testing.assert_array_equal(outs[pipe][0], outs[lib.PIPE_SPLIT][0])
        for key in ("qp_iters", "n_alphas", "alphas", "n_steps", "stepsizes"):
            np.testing.assert_array_equal(outs[pipe][1][key], outs[lib.PIPE_SPLIT][1][key])
    idx = [0, B - 1]
    _check_sqp(outs[lib.PIPE_FUSED][0][idx], outs[lib.PIPE_FUSED][1][idx], xcur[idx], goals[idx], XU[idx], N=N)


@pytest.mark.parametrize("N,B", [(32, 5), (32, 300), (20, 7), (2, 4), (32, 2050)])
def test_riccati_broadcast_variants_bit_identical(lib, model, N, B, monkeypatch):
    """k_riccati_mfma's cross-lane broadcasts (riccati_mfma_body BC: v_readlane, or DPP
    row_newbcast with H's columns duplicated in a second 16-lane row for the pivots) move the
    same values: whole solves are bit-identical for every variant (I7M_RIC_BC=0..3), and with the
    progress-priority bit (6, 7: s_setprio per stage changes only the issue order); B = 2050
    also runs the automatic choice (DPP pivots and rollout at every size, priority from 768
    problems)."""
    xcur, goals, XU = synthetic_batch(B, N, seed=600 + N + B)
    outs = {}
    for bc in ("0", "1", "2", "3", "6", "7", "auto"):
        if bc == "auto":
            monkeypatch.delenv("I7M_RIC_BC", raising=False)
        else:
            monkeypatch.setenv("I7M_RIC_BC", bc)
        h = lib.Handle(model, N=N, max_batch=B)
        outs[bc] = h.solve(xcur, goals, XU)
        h.close()
    for bc in ("1", "2", "3", "6", "7", "auto"):
        np.testing.assert_array_equal(outs[bc][0], outs["0"][0])
        for key in ("qp_iters", "n_alphas", "alphas", "n_steps", "stepsizes"):
            np.testing.assert_array_equal(outs[bc][1][key], outs["0"][1][key])
    idx = [0, B - 1]
    _check_sqp(outs["3"][0][idx], outs["3"][1][idx], xcur[idx], goals[idx], XU[idx], N=N)


@pytest.mark.parametrize("N,B", [(32, 5), (2, 4), (20, 7), (64, 3), (32, 2050)])
def test_riccati_two_wave_body_bit_identical(lib, model, N, B, monkeypatch):
    """k_riccati_mfma_w2 (two waves per problem: W0 / G~ / elimination on wave 0, W1 / H / Qxx on
    wave 1, V~ formed by both from the same operands) gives bit-identical solves to the one-wave
    kernel, with either pivot broadcast (B = 2050 takes the DPP pivots)."""
    xcur, goals, XU = synthetic_batch(B, N, seed=700 + N + B)
    outs = {}
    for w2 in ("0", "1"):
        monkeypatch.setenv("I7M_RIC_W2", w2)
        h = lib.Handle(model, N=N, max_batch=B)
        outs[w2] = h.solve(xcur, goals, XU)
        h.close()
    np.testing.assert_array_equal(outs["1"][0], outs["0"][0])
    for key in ("qp_iters", "n_alphas", "alphas", "n_steps", "stepsizes"):
        np.testing.assert_array_equal(outs["1"][1][key], outs["0"][1][key])
    idx = [0, B - 1]
    _check_sqp(outs["1"][0][idx], outs["1"][1][idx], xcur[idx], goals[idx], XU[idx], N=N)


@pytest.mark.parametrize("frame", ["local", "world"])
def test_fused_pipeline_with_wrench(lib, model, frame):
    N, B = 16, 6
    xcur, goals, XU = synthetic_batch(B, N, seed=41)
    f = np.random.default_rng(4).normal(0, 20, (B, 6))
    outs = []
    for pipe in (lib.PIPE_SPLIT, lib.PIPE_FUSED):
        h = lib.Handle(model, N=N, max_batch=B, pipeline=pipe)
        h.set_external_wrench(f, frame)
        outs.append(h.solve(xcur, goals, XU))
        h.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1]["alphas"], outs[1][1]["alphas"])


def test_fused_device_solve_out_of_place(lib, model):
    """The fused path on device buffers: input only read, every output row written (a poisoned
    problem comes back unchanged), repeated calls give the same answer."""
    import torch

    N, B = 32, 37
    xcur, goals, XU = synthetic_batch(B, N, seed=77)
    goals[5] = np.nan
    ref, st_ref = lib.Handle(model, N=N, max_batch=B, pipeline=lib.PIPE_SPLIT).solve(xcur, goals, XU)
    h = lib.Handle(model, N=N, max_batch=B, pipeline=lib.PIPE_FUSED)
    dev = torch.device("cuda", 0)
    t_xu, t_xs, t_g = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (XU, xcur, goals))
    t_out = torch.full_like(t_xu, float("nan"))
    t_st = torch.zeros(B * lib.STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(2):
        h.solve_device(B, t_xu.data_ptr(), t_xs.data_ptr(), t_g.data_ptr(), 3, t_out.data_ptr(), t_st.data_ptr())
        torch.cuda.synchronize(dev)
        np.testing.assert_array_equal(t_out.cpu().numpy(), ref)
        np.testing.assert_array_equal(t_xu.cpu().numpy(), XU)
        st = np.frombuffer(t_st.cpu().numpy().tobytes(), dtype=lib.STATS_DTYPE)
        np.testing.assert_array_equal(st["alphas"], st_ref["alphas"])


@pytest.mark.parametrize("layout", ["pipeline", "taper", "two_solve_streams", "alternating", "copy_out_thread"])
@pytest.mark.parametrize("chunks", [2, 3, 7])
def test_chunked_host_to_host_solve_bit_identical(lib, model, monkeypatch, chunks, layout):
    """i7m_solve split into chunks (h2h_chunks, copies overlapping solves) gives the one-piece
    solve's XU and stats bit for bit, also for chunks that do not divide B: the default pipeline
    (copy-in / solve / copy-out streams), its tapered chunk sizes (I7M_H2H_TAPER), the solves on
    two alternating streams (I7M_H2H_PIPE=2), the copies out from a second host thread
    (I7M_H2H_PIPE=3, tapered) and the alternating two-stream layout (I7M_H2H_PIPE=0)."""
    from oracle.osqp_ref import synthetic_batch

    monkeypatch.setenv("I7M_H2H_PIPE", {"alternating": "0", "two_solve_streams": "2", "copy_out_thread": "3"}.get(layout, "1"))
    monkeypatch.setenv("I7M_H2H_TAPER", "1" if layout in ("taper", "copy_out_thread") else "0")
    B, N = 300, 32
    xcur, goals, XU = synthetic_batch(B, N, seed=71)
    h1 = lib.Handle(model, N=N, max_batch=B, h2h_chunks=1)
    hc = lib.Handle(model, N=N, max_batch=B, h2h_chunks=chunks)
    o1, s1 = h1.solve(xcur, goals, XU)
    oc, sc = hc.solve(xcur, goals, XU)
    np.testing.assert_array_equal(oc, o1)
    assert np.array_equal(sc, s1)
    # a smaller batch than the handle's, and B < chunks
    o1, s1 = h1.solve(xcur[:5], goals[:5], XU[:5])
    oc, sc = hc.solve(xcur[:5], goals[:5], XU[:5])
    np.testing.assert_array_equal(oc, o1)
    assert np.array_equal(sc, s1)


@pytest.mark.parametrize("mode", ["box", "fused"])
@pytest.mark.parametrize("chunks", [2, 3])
def test_chunked_host_to_host_box_and_fused_bit_identical(lib, model, chunks, mode):
    """Chunked i7m_solve (default pipeline, tapered) in the two modes whose per-chunk buffers differ
    from the split QP: config 4's box mode (the chunk's interior-point buffers through
    bufs_at, and its box stats) and the fused pipeline (launch_fused with the chunk's offsets), each
    against the same mode's one-piece call, bit for bit."""
    from oracle.osqp_ref import synthetic_batch

    B, N = 200, 16
    xcur, goals, XU = synthetic_batch(B, N, seed=73)
    kw = {"qp_mode": lib.QP_BOX} if mode == "box" else {"pipeline": lib.PIPE_FUSED}
    h1 = lib.Handle(model, N=N, max_batch=B, h2h_chunks=1, **kw)
    hc = lib.Handle(model, N=N, max_batch=B, h2h_chunks=chunks, **kw)
    o1, s1 = h1.solve(xcur, goals, XU)
    oc, sc = hc.solve(xcur, goals, XU)
    np.testing.assert_array_equal(oc, o1)
    assert np.array_equal(sc, s1)
    if mode == "box":
        for a, b in zip(h1.box_stats(B), hc.box_stats(B)):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("tail", ["1", "2", "3"])
def test_split_line_search_bit_identical(lib, model, monkeypatch, tail):
    """I7M_LS_TAIL=r: the line search as two launches — r rounds of one wave per problem, then
    two waves per problem for the problems that have not accepted a candidate (base merit handed
    over) — gives the one-launch search's alphas, stats and XU bit for bit (B = 800 > 768, so the
    one-wave kernel is the reference; both wrench frames)."""
    B, N = 800, 32
    xcur, goals, XU = synthetic_batch(B, N, seed=90 + int(tail))
    fx = np.random.default_rng(3).normal(0.0, 20.0, (B, 6))
    outs = {}
    for t in ("0", tail):
        monkeypatch.setenv("I7M_LS_TAIL", t)
        h = lib.Handle(model, N=N, max_batch=B)
        outs[t] = [h.solve(xcur, goals, XU)]
        h.set_external_wrench(fx, frame="world")
        outs[t].append(h.solve(xcur, goals, XU))
        h.close()
    for (o0, s0), (o1, s1) in zip(outs["0"], outs[tail]):
        np.testing.assert_array_equal(o1, o0)
        assert np.array_equal(s1, s0)
    # the split really happened: some problem needed more than the first launch's candidates
    st = outs["0"][0][1]
    used = np.arange(st["alphas"].shape[1])[None, :] < st["n_alphas"][:, None]
    assert (used & (st["alphas"] < 0.5 ** (2 * int(tail) - 1))).any()
