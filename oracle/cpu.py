"""ORACLE (test/bench infrastructure only) — ctypes wrapper of oracle/build/libi7m_cpu.so,
the C++ CPU restatement (oracle/cpp/i7m_cpu.cpp).  Used by tests/ (cross-check) and by
bench.py's cpu_baseline leg and flop count.  Never imported by indy7_mpc_amd."""
import ctypes as C
import os

import numpy as np

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libi7m_cpu.so")
# -march=native build for the host it is built on (bench.py builds it on the GPU box)
LIB_NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libi7m_cpu_native.so")
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int)
_lib = None


def load(path=None):
    """dlopen the port (once; `path` selects a build, default the portable one)."""
    global _lib
    if _lib is None:
        path = path or LIB
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle/cpp`")
        _lib = C.CDLL(path)
        _lib.i7m_cpu_solve.argtypes = [_DP, C.c_int, _DP, C.c_int, _DP, _DP, _DP, C.c_int, _DP, _DP, _IP, _DP, _DP,
                                       C.c_int]
        _lib.i7m_cpu_count_flops.argtypes = [_DP, C.c_int, _DP, _DP, _DP, _DP, C.c_int, _DP]
        _lib.i7m_cpu_solve_box.argtypes = [_DP, C.c_int, _DP, _DP, C.c_int, _DP, _DP, _DP, C.c_int, _DP, _DP, _IP,
                                           _DP, _DP, _IP, _IP, _DP, C.c_int]
        _lib.i7m_cpu_count_flops_box.argtypes = [_DP, C.c_int, _DP, _DP, _DP, _DP, _DP, C.c_int, _DP]
        _lib.i7m_cpu_solve_admm.argtypes = [_DP, C.c_int, _DP, _DP, C.c_int, _DP, _DP, _DP, C.c_int, _DP, _DP, _IP,
                                            _DP, _DP, _DP, _DP, _DP, _DP, _DP, _IP, _IP, C.c_int]
    return _lib


def _p(a):
    return a.ctypes.data_as(_DP)


def _cfg(dt=0.01, dQ=0.01, R=1e-5, QN=100.0, eps=1.0, mu=10.0, step_tol=1e-3, regularize=True, max_iters=2,
         fext_frame="local"):
    """fext_frame: "local" = the wrench is constant in joint 6's frame (pinocchio f_ext); "world" =
    a world-frame spatial force about the world origin, converted per configuration by
    oMi[6].actInv like the GPU's I7M_WRENCH_WORLD (batch_sqp's default)."""
    if fext_frame not in ("local", "world"):
        raise ValueError("fext_frame must be 'local' or 'world'")
    return np.array([dt, dQ, R, QN, eps, mu, step_tol, float(regularize), float(max_iters),
                     float(fext_frame == "world")])


def model_packed():
    import json
    from . import rbd
    with open(rbd.PARAMS_PATH) as f:
        p = json.load(f)
    out = []
    for j in range(6):
        out += list(np.asarray(p["placement_R"][j], float).reshape(9))
    for j in range(6):
        out += list(p["placement_t"][j])
    out += list(p["mass"])
    for j in range(6):
        out += list(p["com"][j])
    for j in range(6):
        I = np.asarray(p["inertia_com"][j], float)
        out += [I[0, 0], I[0, 1], I[0, 2], I[1, 1], I[1, 2], I[2, 2]]
    out += list(p.get("gravity", [0, 0, -9.81]))
    out += list(p["q_lower"]) + list(p["q_upper"]) + list(p["v_limit"]) + list(p["effort_limit"])
    return np.asarray(out, dtype=np.float64)


def box_cfg(mask=7, max_iters=30, tol=1e-8, theta=0.2, eta=0.99, z0=0.1):
    """Config 4's interior-point settings (oracle/box_ipm.py::ipm_box defaults, i7m_box.h BoxParams)."""
    return np.array([mask, max_iters, tol, theta, eta, z0], dtype=np.float64)


def solve_box(xcur, goals, XU, N, nthreads=1, fext=None, box=None, **cfg):
    """Config 4 (box rows on q, v, u): (XU out, qp_iters, alphas, steps, ipm_iters (B, 8) per SQP
    iteration, last QP's converged flag, last QP's mu)."""
    lib = load()
    XU = np.ascontiguousarray(XU, float)
    B = XU.shape[0]
    xcur = np.ascontiguousarray(xcur, float)
    goals = np.ascontiguousarray(goals, float)
    stride = goals.shape[1] // N
    out = np.empty_like(XU)
    qp = np.zeros(B, dtype=np.int32)
    al = np.full((B, 8), np.nan)
    st = np.full((B, 8), np.nan)
    it = np.full((B, 8), -1, dtype=np.int32)
    conv = np.zeros(B, dtype=np.int32)
    mu = np.zeros(B)
    f = np.ascontiguousarray(fext, float) if fext is not None else None
    m = model_packed()
    c = _cfg(**cfg)
    bc = box_cfg() if box is None else np.asarray(box, float)
    rc = lib.i7m_cpu_solve_box(_p(m), N, _p(c), _p(bc), B, _p(XU), _p(xcur), _p(goals), stride,
                               _p(f) if f is not None else None, _p(out), qp.ctypes.data_as(_IP), _p(al), _p(st),
                               it.ctypes.data_as(_IP), conv.ctypes.data_as(_IP), _p(mu), int(nthreads))
    if rc != 0:
        raise RuntimeError("i7m_cpu_solve_box failed")
    return out, qp, al, st, it, conv, mu


def admm_cfg(rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, max_iter=4000, check_termination=25,
             scaling=10, check_dualgap=True, adaptive_rho_interval=0, adaptive_rho_tolerance=5.0):
    """ADMM mode settings: OSQP's defaults as oracle/osqp_admm.py pins them (gap test on, no rho
    adaptation)."""
    return np.array([rho, sigma, alpha, eps_abs, eps_rel, max_iter, check_termination, scaling, float(check_dualgap),
                     adaptive_rho_interval, adaptive_rho_tolerance], dtype=np.float64)


class AdmmState:
    """Per-problem OSQP solver state (scaled x, z, y, the previous QP's q, rho), carried from
    call to call as the reference's OSQP object carries it."""

    def __init__(self, B, N, rho=0.1):
        T, m = 18 * N - 6, 12 * N
        self.x = np.zeros((B, T))
        self.z = np.zeros((B, m))
        self.y = np.zeros((B, m))
        self.q = np.zeros((B, T))
        self.rho = np.full(B, float(rho))
        # OSQP's status of every SQP iteration's QP in the last solve_admm (B, 8): 1 solved,
        # 2 solved inaccurate, 0 max_iter reached, -1 no QP (i7m_get_admm_status's codes)
        self.status = np.full((B, 8), -1, dtype=np.int32)


def solve_admm(xcur, goals, XU, N, state, nthreads=1, fext=None, admm=None, **cfg):
    """ADMM mode: (XU out, qp_iters, alphas, steps, OSQP iterations (B, 8) per SQP iteration);
    `state` (AdmmState) is updated in place.  fext (B, 6) with cfg fext_frame "local" (default) or
    "world" (batch_sqp's default, gato_controller.py's hypotheses)."""
    lib = load()
    XU = np.ascontiguousarray(XU, float)
    B = XU.shape[0]
    xcur = np.ascontiguousarray(xcur, float)
    goals = np.ascontiguousarray(goals, float)
    stride = goals.shape[1] // N
    out = np.empty_like(XU)
    qp = np.zeros(B, dtype=np.int32)
    al = np.full((B, 8), np.nan)
    st = np.full((B, 8), np.nan)
    it = np.full((B, 8), -1, dtype=np.int32)
    f = np.ascontiguousarray(fext, float) if fext is not None else None
    m = model_packed()
    c = _cfg(**cfg)
    ac = admm_cfg() if admm is None else np.asarray(admm, float)
    for a in (state.x, state.z, state.y, state.q, state.rho):
        assert a.flags.c_contiguous and a.dtype == np.float64 and a.shape[0] == B
    state.status[:] = -1
    rc = lib.i7m_cpu_solve_admm(_p(m), N, _p(c), _p(ac), B, _p(XU), _p(xcur), _p(goals), stride,
                                _p(f) if f is not None else None, _p(out), qp.ctypes.data_as(_IP), _p(al), _p(st),
                                _p(state.x), _p(state.z), _p(state.y), _p(state.q), _p(state.rho),
                                it.ctypes.data_as(_IP), state.status.ctypes.data_as(_IP), int(nthreads))
    if rc != 0:
        raise RuntimeError("i7m_cpu_solve_admm failed")
    return out, qp, al, st, it


def solve(xcur, goals, XU, N, nthreads=1, fext=None, **cfg):
    lib = load()
    XU = np.ascontiguousarray(XU, float)
    B = XU.shape[0]
    xcur = np.ascontiguousarray(xcur, float)
    goals = np.ascontiguousarray(goals, float)
    stride = goals.shape[1] // N
    out = np.empty_like(XU)
    qp = np.zeros(B, dtype=np.int32)
    al = np.full((B, 8), np.nan)
    st = np.full((B, 8), np.nan)
    f = np.ascontiguousarray(fext, float) if fext is not None else None
    m = model_packed()
    c = _cfg(**cfg)
    rc = lib.i7m_cpu_solve(_p(m), N, _p(c), B, _p(XU), _p(xcur), _p(goals), stride, _p(f) if f is not None else None,
                           _p(out), qp.ctypes.data_as(_IP), _p(al), _p(st), int(nthreads))
    if rc != 0:
        raise RuntimeError("i7m_cpu_solve failed")
    return out, qp, al, st


def count_flops(xcur, goals, XU, N, box=None, **cfg):
    """Instrumented flops of one SQP solve: dict by stage (box: config 4's settings, box_cfg(),
    adds the interior point's flops — inside "qp" — and its iterations)."""
    lib = load()
    out = np.zeros(8)
    m = model_packed()
    c = _cfg(**cfg)
    g = np.ascontiguousarray(goals, float)
    bc = None if box is None else np.asarray(box, float)
    lib.i7m_cpu_count_flops_box(_p(m), N, _p(c), _p(bc) if bc is not None else None,
                                _p(np.ascontiguousarray(XU, float)), _p(np.ascontiguousarray(xcur, float)),
                                _p(g), g.shape[0] // N, _p(out))
    d = {"linearize": out[0], "qp": out[1], "linesearch": out[2], "step": out[3], "iters": out[4],
         "merit_evals": out[5], "total": out[:4].sum()}
    if bc is not None:
        d.update(ipm=out[6], ipm_iters=out[7])
    return d
