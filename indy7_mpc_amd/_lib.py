"""ctypes binding of libindy7mpc.so (the C-ABI in include/indy7_mpc.h).

The library is built in-tree by ``__graft_entry__.build()`` into ``indy7_mpc_amd/lib/``.
There is no CPU fallback: if the library or a gfx950 device is missing every entry point
raises :class:`I7MError`.

One HIP runtime per process: torch-ROCm bundles its own ``libamdhip64.so`` (SONAME
``libamdhip64.so.7``, the same SONAME as /opt/rocm's).  If torch is importable we import it
*before* dlopen-ing our library so the dynamic loader binds our NEEDED entry to the runtime
torch already mapped, instead of mapping a second HIP runtime into the process.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("I7M_LIB", os.path.join(LIB_DIR, "libindy7mpc.so"))  # I7M_LIB: A/B builds

ABI_VERSION = 6  # I7M_ABI_VERSION of include/indy7_mpc.h this binding's SIGNATURES follow
NJ, NX, NU = 6, 12, 6
MAX_SQP = 8
MAX_N = 64
LIN_STRIDE, COST_STRIDE = 114, 10

(I7M_K_LIN, I7M_K_RICCATI, I7M_K_LINESEARCH, I7M_K_RICCATI_BOX, I7M_K_IPM, I7M_K_IPM_FUSED, I7M_K_SQP_FUSED,
 I7M_K_LINESEARCH_TAIL, I7M_K_ADMM, I7M_K_ADMM_PREP) = range(10)
I7M_K_COUNT = 10
KERNEL_NAMES = ("k_linearize", "k_riccati", "k_linesearch", "k_riccati_box", "k_ipm", "k_ipm_fused", "k_sqp_fused",
                "k_linesearch_tail", "k_admm_iter", "k_admm_prep")


class I7MError(RuntimeError):
    pass


class i7m_model(C.Structure):
    _fields_ = [
        ("placement_R", (C.c_double * 9) * 6),
        ("placement_t", (C.c_double * 3) * 6),
        ("mass", C.c_double * 6),
        ("com", (C.c_double * 3) * 6),
        ("inertia", (C.c_double * 6) * 6),
        ("gravity", C.c_double * 3),
        ("q_lower", C.c_double * 6),
        ("q_upper", C.c_double * 6),
        ("v_limit", C.c_double * 6),
        ("effort_limit", C.c_double * 6),
    ]


class i7m_config(C.Structure):
    _fields_ = [
        ("N", C.c_int32),
        ("regularize", C.c_int32),
        ("dt", C.c_double),
        ("dQ_cost", C.c_double),
        ("R_cost", C.c_double),
        ("QN_cost", C.c_double),
        ("eps", C.c_double),
        ("mu", C.c_double),
        ("step_tol", C.c_double),
        ("max_sqp_iters", C.c_int32),
        ("max_batch", C.c_int32),
        ("device_id", C.c_int32),
        ("qp_mode", C.c_int32),
        ("model", i7m_model),
        ("box_mask", C.c_int32),
        ("box_max_iters", C.c_int32),
        ("box_tol", C.c_double),
        ("pipeline", C.c_int32),
        ("h2h_chunks", C.c_int32),
        ("admm_rho", C.c_double),
        ("admm_sigma", C.c_double),
        ("admm_alpha", C.c_double),
        ("admm_eps_abs", C.c_double),
        ("admm_eps_rel", C.c_double),
        ("admm_max_iter", C.c_int32),
        ("admm_check_termination", C.c_int32),
        ("admm_scaling", C.c_int32),
        ("admm_check_dualgap", C.c_int32),
        ("admm_adaptive_rho_interval", C.c_int32),
        ("precision", C.c_int32),
        ("admm_adaptive_rho_tolerance", C.c_double),
    ]


QP_DIRECT, QP_BOX, QP_ADMM = 0, 1, 2
PREC_F64, PREC_F32 = 0, 1  # i7m_config.precision (only PREC_F64 is built)
ADMM_RESET_RHO, ADMM_RESET_DUAL, ADMM_RESET_PRIMAL, ADMM_RESET_ALL = 1, 2, 4, 7
# OSQP's settings as i7m_config_default sets them (oracle/osqp_admm.py DEFAULTS)
ADMM_DEFAULTS = dict(rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, max_iter=4000, check_termination=25,
                     scaling=10, check_dualgap=True, adaptive_rho_interval=0, adaptive_rho_tolerance=5.0)
PIPE_AUTO, PIPE_SPLIT, PIPE_FUSED, PIPE_FUSED_ITER = 0, 1, 2, 3
WRENCH_LOCAL, WRENCH_WORLD = 0, 1
_FRAMES = {"local": WRENCH_LOCAL, "world": WRENCH_WORLD, WRENCH_LOCAL: WRENCH_LOCAL, WRENCH_WORLD: WRENCH_WORLD}
BOX_Q, BOX_V, BOX_U = 1, 2, 4


class i7m_problem_stats(C.Structure):
    _fields_ = [
        ("qp_iters", C.c_int32),
        ("n_alphas", C.c_int32),
        ("n_steps", C.c_int32),
        ("pad", C.c_int32),
        ("alphas", C.c_double * MAX_SQP),
        ("stepsizes", C.c_double * MAX_SQP),
    ]


STATS_DTYPE = np.dtype(
    [("qp_iters", "<i4"), ("n_alphas", "<i4"), ("n_steps", "<i4"), ("pad", "<i4"),
     ("alphas", "<f8", (MAX_SQP,)), ("stepsizes", "<f8", (MAX_SQP,))]
)
assert STATS_DTYPE.itemsize == C.sizeof(i7m_problem_stats)

_DP = C.POINTER(C.c_double)
_H = C.c_void_p

# (name, restype, argtypes) — every symbol declared in include/indy7_mpc.h
SIGNATURES = [
    ("i7m_last_error", C.c_char_p, []),
    ("i7m_version", C.c_char_p, []),
    ("i7m_abi_version", C.c_int, []),
    ("i7m_config_default", C.c_int, [C.POINTER(i7m_config)]),
    ("i7m_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("i7m_create", C.c_int, [C.POINTER(i7m_config), C.POINTER(_H)]),
    ("i7m_destroy", None, [_H]),
    ("i7m_set_stream", C.c_int, [_H, C.c_void_p]),
    ("i7m_synchronize", C.c_int, [_H]),
    ("i7m_set_external_wrench", C.c_int, [_H, C.c_int32, _DP, C.c_int32]),
    ("i7m_solve", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, C.c_int32, _DP, C.c_void_p]),
    ("i7m_solve_device", C.c_int, [_H, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p,
                                   C.c_void_p]),
    ("i7m_qp", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, C.c_int32, _DP]),
    ("i7m_qp_value", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, C.c_int32, _DP]),
    ("i7m_get_box_stats", C.c_int, [_H, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), _DP]),
    ("i7m_admm_reset", C.c_int, [_H, C.c_int32, C.c_int32]),
    ("i7m_get_admm_stats", C.c_int, [_H, C.c_int32, C.POINTER(C.c_int32), _DP]),
    ("i7m_get_admm_state", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, _DP, _DP]),
    ("i7m_get_admm_status", C.c_int, [_H, C.c_int32, C.POINTER(C.c_int32)]),
    ("i7m_get_admm_dual", C.c_int, [_H, C.c_int32, _DP]),
    ("i7m_linearize", C.c_int, [_H, C.c_int32, _DP, _DP, C.c_int32, _DP, _DP]),
    ("i7m_merit", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, C.c_int32, _DP]),
    ("i7m_linesearch", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, C.c_int32, _DP]),
    ("i7m_eepos", C.c_int, [_H, C.c_int32, _DP, _DP, _DP]),
    ("i7m_aba", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, _DP, C.c_int32, _DP]),
    ("i7m_aba_derivatives", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, _DP, _DP, _DP, _DP]),
    ("i7m_rk4", C.c_int, [_H, C.c_int32, _DP, _DP, _DP, C.c_double, _DP, C.c_int32, _DP, _DP]),
    ("i7m_mpc_run", C.c_int, [_H, C.c_int32, _DP, _DP, C.c_int32, C.c_int32, _DP, _DP, _DP, _DP]),
    ("i7m_set_timing", C.c_int, [_H, C.c_int]),
    ("i7m_get_kernel_times", C.c_int, [_H, _DP, C.POINTER(C.c_int32), C.c_int32]),
    ("i7m_reset_kernel_times", C.c_int, [_H]),
    ("i7m_reset", C.c_int, [_H]),
]

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """dlopen libindy7mpc.so (once).  Raises I7MError if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise I7MError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:  # share torch's HIP runtime if torch is present (see module docstring)
            import torch  # noqa: F401
        except Exception:
            pass
        lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.i7m_abi_version() != ABI_VERSION:
            raise I7MError(f"{path} has C-ABI revision {lib.i7m_abi_version()}, this binding expects {ABI_VERSION}")
        _lib = lib
        return lib


def _check(rc: int):
    if rc != 0:
        msg = _lib.i7m_last_error().decode(errors="replace")
        raise I7MError(f"libindy7mpc error {rc}: {msg}")


def version() -> str:
    """i7m_version(): build kind and the sha256 prefix of the sources it was compiled from
    (__graft_entry__.src_hash)."""
    return load().i7m_version().decode()


def device_count() -> int:
    lib = load()
    n = C.c_int(0)
    rc = lib.i7m_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def _f64(a, shape=None) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_DP)


class Handle:
    """One device handle (= one OSQPSolver-like solver state on one GPU)."""

    def __init__(self, model, N=32, dt=0.01, dQ_cost=0.01, R_cost=1e-5, QN_cost=100.0, regularize=True, eps=1.0,
                 max_batch=1, device_id=0, mu=10.0, step_tol=1e-3, max_sqp_iters=2, qp_mode=QP_DIRECT,
                 box_mask=BOX_Q | BOX_V | BOX_U, box_max_iters=30, box_tol=1e-8, pipeline=PIPE_AUTO, h2h_chunks=0,
                 admm=None):
        """admm: OSQP settings for qp_mode=QP_ADMM (keys of ADMM_DEFAULTS; missing keys keep the
        defaults)."""
        lib = load()
        cfg = i7m_config()
        _check(lib.i7m_config_default(C.byref(cfg)))
        cfg.N, cfg.dt, cfg.dQ_cost, cfg.R_cost, cfg.QN_cost = int(N), float(dt), float(dQ_cost), float(R_cost), float(QN_cost)
        cfg.regularize, cfg.eps, cfg.mu, cfg.step_tol = int(bool(regularize)), float(eps), float(mu), float(step_tol)
        cfg.max_sqp_iters, cfg.max_batch, cfg.device_id = int(max_sqp_iters), int(max_batch), int(device_id)
        cfg.qp_mode, cfg.box_mask, cfg.box_max_iters, cfg.box_tol = int(qp_mode), int(box_mask), int(box_max_iters), float(box_tol)
        cfg.pipeline = int(pipeline)
        cfg.h2h_chunks = int(h2h_chunks)
        if admm:
            unknown = set(admm) - set(ADMM_DEFAULTS)
            if unknown:
                raise ValueError(f"unknown ADMM settings {sorted(unknown)}")
            for k, v in admm.items():
                f = "admm_" + k
                setattr(cfg, f, type(getattr(cfg, f))(v) if not isinstance(v, bool) else int(v))
        packed = np.ascontiguousarray(model.packed(), dtype=np.float64)
        assert packed.nbytes == C.sizeof(i7m_model), (packed.nbytes, C.sizeof(i7m_model))
        C.memmove(C.byref(cfg.model), packed.ctypes.data, packed.nbytes)
        h = _H()
        _check(lib.i7m_create(C.byref(cfg), C.byref(h)))
        self._lib, self._h, self.cfg = lib, h, cfg
        self.N, self.T, self.max_batch = int(N), 18 * int(N) - 6, int(max_batch)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.i7m_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- batched entry points (numpy in / numpy out) -------------------------------------
    def _batch(self, xu, goals, xcur=None):
        xu = _f64(xu)
        if xu.ndim == 1:
            xu = xu[None]
        B = xu.shape[0]
        if xu.shape[1] != self.T:
            raise ValueError(f"XU must have {self.T} columns, got {xu.shape[1]}")
        goals = _f64(goals)
        if goals.ndim == 1:
            goals = goals[None]
        if goals.shape[0] != B:
            raise ValueError("goals batch mismatch")
        stride = goals.shape[1] // self.N
        if stride not in (3, 6) or goals.shape[1] != stride * self.N:
            raise ValueError(f"goals must have 3N or 6N columns (N={self.N}), got {goals.shape[1]}")
        out = [xu, goals, B, stride]
        if xcur is not None:
            xc = _f64(xcur)
            if xc.ndim == 1:
                xc = xc[None]
            if xc.shape != (B, NX):
                raise ValueError(f"xcur must be ({B}, 12)")
            out.append(xc)
        return out

    def solve(self, xcur, goals, xu, out=None, stats=None):
        """out / stats: optional preallocated (B, T) float64 / (B,) STATS_DTYPE arrays (e.g. views
        of pinned host memory, which the chunked host-to-host path can copy asynchronously)."""
        xu, goals, B, stride, xc = self._batch(xu, goals, xcur)
        if out is None:
            out = np.empty_like(xu)
        elif out.shape != xu.shape or out.dtype != np.float64 or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous float64 array shaped like XU")
        st = np.zeros(B, dtype=STATS_DTYPE) if stats is None else stats
        if st.shape != (B,) or st.dtype != STATS_DTYPE:
            raise ValueError("stats must be a (B,) STATS_DTYPE array")
        _check(self._lib.i7m_solve(self._h, B, _ptr(xu), _ptr(xc), _ptr(goals), stride, _ptr(out),
                                   st.ctypes.data_as(C.c_void_p)))
        return out, st

    def solve_device(self, B, d_xu_in, d_xcur, d_goals, goal_stride, d_xu_out, d_stats=None):
        """Device pointers (ints, e.g. torch ``data_ptr()``); async on the handle's stream."""
        _check(self._lib.i7m_solve_device(self._h, int(B), C.c_void_p(d_xu_in), C.c_void_p(d_xcur),
                                          C.c_void_p(d_goals), int(goal_stride), C.c_void_p(d_xu_out),
                                          C.c_void_p(d_stats) if d_stats else None))

    def qp(self, xu, xcur, goals):
        xu, goals, B, stride, xc = self._batch(xu, goals, xcur)
        sol = np.empty_like(xu)
        _check(self._lib.i7m_qp(self._h, B, _ptr(xu), _ptr(xc), _ptr(goals), stride, _ptr(sol)))
        return sol

    def qp_value(self, xu, xcur, goals):
        """The QP's cost-to-go at the first knot, V~_0 (B, 13, 13) (i7m_qp_value): [[Vxx, vx], [vx', c]]
        in the homogeneous coordinates [x_0; 1], as the Riccati recursion ends with it."""
        xu, goals, B, stride, xc = self._batch(xu, goals, xcur)
        V = np.empty((B, 13, 13))
        _check(self._lib.i7m_qp_value(self._h, B, _ptr(xu), _ptr(xc), _ptr(goals), stride, _ptr(V)))
        return V

    def box_stats(self, B):
        """Interior-point record of the last QP (box mode): (iters, converged, mu), each (B,)."""
        it = np.zeros(B, dtype=np.int32)
        cv = np.zeros(B, dtype=np.int32)
        mu = np.zeros(B)
        ip = C.POINTER(C.c_int32)
        _check(self._lib.i7m_get_box_stats(self._h, int(B), it.ctypes.data_as(ip), cv.ctypes.data_as(ip), _ptr(mu)))
        return it, cv.astype(bool), mu

    def admm_reset(self, B=None, what=ADMM_RESET_ALL):
        """I7M_QP_ADMM: start the OSQP state of problems [0, B) afresh (what: ADMM_RESET_* bits;
        RHO = batch_sqp resetRho, DUAL = resetLambda, ALL = a new OSQP object)."""
        _check(self._lib.i7m_admm_reset(self._h, int(self.max_batch if B is None else B), int(what)))

    def admm_stats(self, B, with_status=False):
        """I7M_QP_ADMM: (OSQP iterations per SQP iteration of the last solve (B, 8), -1 = none;
        rho (B,)); with_status also OSQP's status per SQP iteration (B, 8): 1 solved, 2 solved inaccurate, 0 maximum
        iterations reached, -1 no QP."""
        it = np.zeros((B, MAX_SQP), dtype=np.int32)
        rho = np.zeros(B)
        _check(self._lib.i7m_get_admm_stats(self._h, int(B), it.ctypes.data_as(C.POINTER(C.c_int32)), _ptr(rho)))
        if not with_status:
            return it, rho
        stat = np.zeros((B, MAX_SQP), dtype=np.int32)
        _check(self._lib.i7m_get_admm_status(self._h, int(B), stat.ctypes.data_as(C.POINTER(C.c_int32))))
        return it, rho, stat

    def admm_dual(self, B):
        """I7M_QP_ADMM: each problem's last QP's dual y, unscaled as OSQP returns it (B, 12N)."""
        y = np.empty((B, 12 * self.N))
        _check(self._lib.i7m_get_admm_dual(self._h, int(B), _ptr(y)))
        return y

    def admm_state(self, B):
        """I7M_QP_ADMM: the carried OSQP state (scaled x (B, T), z, y (B, 12N), previous q (B, T),
        rho (B,))."""
        m = 12 * self.N
        x, q = np.empty((B, self.T)), np.empty((B, self.T))
        z, y = np.empty((B, m)), np.empty((B, m))
        rho = np.empty(B)
        _check(self._lib.i7m_get_admm_state(self._h, int(B), _ptr(x), _ptr(z), _ptr(y), _ptr(q), _ptr(rho)))
        return x, z, y, q, rho

    def linearize(self, xu, goals):
        xu, goals, B, stride = self._batch(xu, goals)
        lin = np.empty((B, self.N - 1, LIN_STRIDE))
        cost = np.empty((B, self.N, COST_STRIDE))
        _check(self._lib.i7m_linearize(self._h, B, _ptr(xu), _ptr(goals), stride, _ptr(lin), _ptr(cost)))
        return lin, cost

    def merit(self, xu, xu_ref, goals):
        xu, goals, B, stride = self._batch(xu, goals)
        xr = _f64(xu_ref).reshape(B, self.T)
        out = np.empty((B, 5))
        _check(self._lib.i7m_merit(self._h, B, _ptr(xu), _ptr(xr), _ptr(goals), stride, _ptr(out)))
        return out

    def linesearch(self, xu, xu_full, goals):
        xu, goals, B, stride = self._batch(xu, goals)
        xf = _f64(xu_full).reshape(B, self.T)
        out = np.empty(B)
        _check(self._lib.i7m_linesearch(self._h, B, _ptr(xu), _ptr(xf), _ptr(goals), stride, _ptr(out)))
        return out

    # ---- query hooks ---------------------------------------------------------------------
    def eepos(self, q, jacobian=False):
        q = _f64(q).reshape(-1, NJ)
        n = q.shape[0]
        p = np.empty((n, 3))
        J = np.empty((n, 3, NJ)) if jacobian else None
        _check(self._lib.i7m_eepos(self._h, n, _ptr(q), _ptr(p), _ptr(J) if J is not None else None))
        return (p, J) if jacobian else p

    def aba(self, q, v, tau, fext=None, frame="local"):
        """fext (n, 6) joint-6 wrench, in joint 6's frame ("local") or the world frame ("world",
        converted at q by oMi[6].actInv)."""
        q, v, tau = (_f64(x).reshape(-1, NJ) for x in (q, v, tau))
        n = q.shape[0]
        a = np.empty((n, NJ))
        f = _f64(fext).reshape(n, 6) if fext is not None else None
        _check(self._lib.i7m_aba(self._h, n, _ptr(q), _ptr(v), _ptr(tau), _ptr(f) if f is not None else None,
                                 _FRAMES[frame], _ptr(a)))
        return a

    def aba_derivatives(self, q, v, tau):
        q, v, tau = (_f64(x).reshape(-1, NJ) for x in (q, v, tau))
        n = q.shape[0]
        dq, dv, Mi = (np.empty((n, NJ, NJ)) for _ in range(3))
        a = np.empty((n, NJ))
        _check(self._lib.i7m_aba_derivatives(self._h, n, _ptr(q), _ptr(v), _ptr(tau), _ptr(dq), _ptr(dv), _ptr(Mi),
                                             _ptr(a)))
        return dq, dv, Mi, a

    def rk4(self, q, v, u, dt, fext=None, frame="local"):
        """utils.rk4 per row; a "world" wrench is converted once at the start q (the reference's
        host plant, src/gato_mpc_batch_sample.py:270-279)."""
        q, v, u = (_f64(x).reshape(-1, NJ) for x in (q, v, u))
        n = q.shape[0]
        qo, vo = np.empty((n, NJ)), np.empty((n, NJ))
        f = _f64(fext).reshape(n, 6) if fext is not None else None
        _check(self._lib.i7m_rk4(self._h, n, _ptr(q), _ptr(v), _ptr(u), float(dt), _ptr(f) if f is not None else None,
                                 _FRAMES[frame], _ptr(qo), _ptr(vo)))
        return qo, vo

    def mpc_run(self, xstart, endpoints, num_steps):
        """Closed-loop MPC of B instances on the device (i7m_mpc_run): returns (dists
        (num_steps, B), q (num_steps, B, 6), xcur (B, 12), XU (B, T))."""
        xs = _f64(xstart).reshape(-1, NX)
        ep = _f64(endpoints).reshape(-1, 3)
        B = xs.shape[0]
        d = np.empty((num_steps, B))
        q = np.empty((num_steps, B, NJ))
        xc = np.empty((B, NX))
        xu = np.empty((B, self.T))
        _check(self._lib.i7m_mpc_run(self._h, B, _ptr(xs), _ptr(ep), ep.shape[0], int(num_steps), _ptr(d), _ptr(q),
                                     _ptr(xc), _ptr(xu)))
        return d, q, xc, xu

    # ---- timing --------------------------------------------------------------------------
    def set_stream(self, stream_ptr: int):
        _check(self._lib.i7m_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None))

    def set_external_wrench(self, fext, frame="local"):
        """(B, 6) joint-6 wrench per problem ([f; n]; frame "local" = joint 6's frame, "world" =
        world frame about the origin, converted per configuration), or None to clear."""
        if fext is None:
            _check(self._lib.i7m_set_external_wrench(self._h, 0, None, 0))
            return
        f = _f64(fext).reshape(-1, 6)
        _check(self._lib.i7m_set_external_wrench(self._h, f.shape[0], _ptr(f), _FRAMES[frame]))

    def synchronize(self):
        _check(self._lib.i7m_synchronize(self._h))

    def set_timing(self, on: bool):
        _check(self._lib.i7m_set_timing(self._h, int(bool(on))))

    def kernel_times(self):
        ms = (C.c_double * I7M_K_COUNT)()
        cnt = (C.c_int32 * I7M_K_COUNT)()
        _check(self._lib.i7m_get_kernel_times(self._h, ms, cnt, I7M_K_COUNT))
        return {KERNEL_NAMES[i]: (ms[i], cnt[i]) for i in range(I7M_K_COUNT) if cnt[i] > 0}

    def reset_kernel_times(self):
        _check(self._lib.i7m_reset_kernel_times(self._h))

    def reset(self):
        """i7m_reset: back to the post-create solver state (ADMM mode: every problem's OSQP state
        afresh; drops captured graphs and timing sums; the external wrench is kept)."""
        _check(self._lib.i7m_reset(self._h))
