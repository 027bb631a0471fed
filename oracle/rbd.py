"""ORACLE (test infrastructure only) — rigid-body dynamics restated in numpy.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
The product path (indy7_mpc_amd) never does.

What it restates: the pinocchio calls the reference's hot path makes (pinocchio is an
un-vendored third-party dependency, version unpinned):
  * ``pin.forwardKinematics`` + ``data.oMi[6].translation``   (src/osqp_solver.py:146-148)
  * ``pin.computeJointJacobians`` + ``getJointJacobian(6, LOCAL_WORLD_ALIGNED)[:3]``
                                                                (src/osqp_solver.py:150-155)
  * ``pin.aba``                                                 (src/osqp_sqp.py:40, src/utils.py:4-11)
  * ``pin.computeABADerivatives`` -> (da/dq, da/dv, Minv), ``data.ddq``
                                                                (src/osqp_solver.py:71,76)
  * ``pin.integrate`` on revolute joints = q + v                (src/osqp_solver.py:77)
Algorithms (published, Featherstone / Carpentier-Mansard conventions as pinocchio uses):
local-frame RNEA, articulated-body ABA, RNEA-column CRBA; derivatives by complex-step
differentiation of RNEA (exact to rounding, independent of the GPU's dual-number scheme):
da/dq = -Minv dRNEA/dq |_(q,v,a),  da/dv = -Minv dRNEA/dv,  da/dtau = Minv.
Spatial vectors are [linear; angular] (pinocchio ordering). Every function accepts
complex dtypes so complex-step works through it.

Model constants come from indy7_mpc_amd/params/indy7.json (numbers generated from the
reference URDF, description/indy7.urdf:49-245) — read as data, not imported.
"""
from __future__ import annotations

import json
import os

import numpy as np

PARAMS_PATH = os.path.join(os.path.dirname(__file__), "..", "indy7_mpc_amd", "params", "indy7.json")
NJ = 6
H_CS = 1e-30  # complex-step size


class Params:
    def __init__(self, path: str = PARAMS_PATH):
        with open(path) as f:
            p = json.load(f)
        self.Rp = [np.array(r, dtype=float) for r in p["placement_R"]]
        self.tp = [np.array(t, dtype=float) for t in p["placement_t"]]
        self.mass = np.array(p["mass"], dtype=float)
        self.com = [np.array(c, dtype=float) for c in p["com"]]
        self.Ic = [np.array(i, dtype=float) for i in p["inertia_com"]]
        self.gravity = np.array(p.get("gravity", [0, 0, -9.81]), dtype=float)
        self.q_lower = np.array(p["q_lower"])
        self.q_upper = np.array(p["q_upper"])
        self.v_limit = np.array(p["v_limit"])
        self.effort_limit = np.array(p["effort_limit"])


_P = None


def params() -> Params:
    global _P
    if _P is None:
        _P = Params()
    return _P


def _rz(q):
    c, s = np.cos(q), np.sin(q)
    z = 0.0 * q
    o = z + 1.0
    return np.array([[c, -s, z], [s, c, z], [z, z, o]])


def joint_transforms(q, P: Params = None):
    """liMi for each joint: (R_i, t_i) with x_parent = R_i x_i + t_i."""
    P = P or params()
    return [(P.Rp[i] @ _rz(q[i]), P.tp[i]) for i in range(NJ)]


def fk(q, P: Params = None):
    """World placements oMi[1..6] (pinocchio forwardKinematics)."""
    P = P or params()
    R = np.eye(3, dtype=np.result_type(q, float))
    p = np.zeros(3, dtype=R.dtype)
    out = []
    for Ri, ti in joint_transforms(q, P):
        p = p + R @ ti
        R = R @ Ri
        out.append((R, p))
    return out


def eepos(q, P: Params = None):
    """data.oMi[6].translation  (src/osqp_solver.py:146-148)."""
    return fk(q, P)[-1][1]


def d_eepos(q, P: Params = None):
    """(eepos, J[:3]) with J the LOCAL_WORLD_ALIGNED joint-6 Jacobian (src/osqp_solver.py:150-155)."""
    oM = fk(q, P)
    pe = oM[-1][1]
    J = np.zeros((3, NJ), dtype=pe.dtype)
    for j, (R, p) in enumerate(oM):
        J[:, j] = np.cross(R[:, 2], pe - p)
    return pe, J


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]])


def _inertia_mul(P: Params, i, v, w):
    """Spatial inertia (local, about the joint origin) times motion (v, w)."""
    m, c, Ic = P.mass[i], P.com[i], P.Ic[i]
    lin = m * (v - _cross(c, w))
    ang = Ic @ w + _cross(c, lin)
    return lin, ang


def _rnea_impl(q, v, a, P: Params, grav, fext):
    dt = np.result_type(q, v, a, float)
    X = joint_transforms(q, P)
    vl = np.zeros(3, dtype=dt)
    vw = np.zeros(3, dtype=dt)
    al = np.array(-P.gravity if grav else np.zeros(3), dtype=dt)
    aw = np.zeros(3, dtype=dt)
    ez = np.array([0.0, 0.0, 1.0])
    F = []
    for i in range(NJ):
        R, t = X[i]
        vl, vw = R.T @ (vl - _cross(t, vw)), R.T @ vw
        al, aw = R.T @ (al - _cross(t, aw)), R.T @ aw
        vw = vw + ez * v[i]
        # a_i += S qdd + v_i x (S qd)
        al = al + _cross(vl, ez * v[i])
        aw = aw + ez * a[i] + _cross(vw, ez * v[i])
        hl, hn = _inertia_mul(P, i, vl, vw)
        il, iN = _inertia_mul(P, i, al, aw)
        # f = I a + v x* (I v)
        fl = il + _cross(vw, hl)
        fn = iN + _cross(vw, hn) + _cross(vl, hl)
        if fext is not None:
            fl = fl - fext[i][:3]
            fn = fn - fext[i][3:]
        F.append([fl, fn])
    tau = np.zeros(NJ, dtype=dt)
    for i in range(NJ - 1, -1, -1):
        fl, fn = F[i]
        tau[i] = fn[2]
        if i > 0:
            R, t = X[i]
            pf = R @ fl
            pn = R @ fn + _cross(t, pf)
            F[i - 1][0] = F[i - 1][0] + pf
            F[i - 1][1] = F[i - 1][1] + pn
    return tau


def rnea(q, v, a, P: Params = None, gravity=True, fext=None):
    """Inverse dynamics tau = M a + C v + g (local-frame RNEA, pinocchio conventions).

    ``fext``: optional list of 6 local spatial forces [f; n] applied to each body
    (pinocchio's f_ext argument; used only by the rk4 plant, src/utils.py:3-18)."""
    return _rnea_impl(q, v, a, P or params(), gravity, fext)


def crba(q, P: Params = None):
    """Joint-space inertia M(q), column j = RNEA(q, 0, e_j) without gravity."""
    P = P or params()
    dt = np.result_type(q, float)
    M = np.zeros((NJ, NJ), dtype=dt)
    z = np.zeros(NJ)
    for j in range(NJ):
        e = np.zeros(NJ)
        e[j] = 1.0
        M[:, j] = _rnea_impl(q, z, e, P, False, None)
    return M


def aba(q, v, tau, P: Params = None, fext=None):
    """Articulated-body algorithm (pinocchio pin.aba), local frames, 3 passes."""
    P = P or params()
    dt = np.result_type(q, v, tau, float)
    X = joint_transforms(q, P)

    def Xinv_mat(R, t):  # 6x6 motion transform parent -> child
        tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
        M6 = np.zeros((6, 6), dtype=dt)
        M6[:3, :3] = R.T
        M6[:3, 3:] = -R.T @ tx
        M6[3:, 3:] = R.T
        return M6

    def skew(w):
        return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]], dtype=dt)

    def inertia6(i):
        m, c, Ic = P.mass[i], P.com[i], P.Ic[i]
        cx = skew(c)
        I6 = np.zeros((6, 6), dtype=float)
        I6[:3, :3] = m * np.eye(3)
        I6[:3, 3:] = -m * cx
        I6[3:, :3] = m * cx
        I6[3:, 3:] = Ic - m * cx @ cx
        return I6

    def mcross(m):  # motion cross matrix
        v_, w_ = m[:3], m[3:]
        C = np.zeros((6, 6), dtype=dt)
        C[:3, :3] = skew(w_)
        C[:3, 3:] = skew(v_)
        C[3:, 3:] = skew(w_)
        return C

    S = np.array([0, 0, 0, 0, 0, 1.0])
    Xi = [Xinv_mat(R, t) for R, t in X]
    V = [None] * NJ
    c = [None] * NJ
    IA = [None] * NJ
    pA = [None] * NJ
    vp = np.zeros(6, dtype=dt)
    for i in range(NJ):
        V[i] = Xi[i] @ vp + S * v[i]
        c[i] = mcross(V[i]) @ (S * v[i])
        IA[i] = inertia6(i).astype(dt)
        pA[i] = -mcross(V[i]).T @ (IA[i] @ V[i])  # v x* I v
        if fext is not None:
            pA[i] = pA[i] - np.asarray(fext[i], dtype=dt)
        vp = V[i]
    U = [None] * NJ
    D = [None] * NJ
    u = [None] * NJ
    for i in range(NJ - 1, -1, -1):
        U[i] = IA[i] @ S
        D[i] = S @ U[i]
        u[i] = tau[i] - S @ pA[i]
        if i > 0:
            Ia = IA[i] - np.outer(U[i], U[i]) / D[i]
            pa = pA[i] + Ia @ c[i] + U[i] * u[i] / D[i]
            IA[i - 1] = IA[i - 1] + Xi[i].T @ Ia @ Xi[i]
            pA[i - 1] = pA[i - 1] + Xi[i].T @ pa
    qdd = np.zeros(NJ, dtype=dt)
    ap = np.array(list(-P.gravity) + [0, 0, 0], dtype=dt)
    for i in range(NJ):
        a_ = Xi[i] @ ap + c[i]
        qdd[i] = (u[i] - U[i] @ a_) / D[i]
        ap = a_ + S * qdd[i]
    return qdd


def wrench_world_to_local(q, fw, P: Params = None):
    """World-frame spatial force [f; n] (about the world origin) -> joint 6's local frame:
    data.oMi[6].actInv(pin.Force(f, n)) at configuration q (src/gato_mpc_batch_sample.py:151-161),
    f_l = R' f, n_l = R' (n - p x f).  Complex-step safe."""
    R, p = fk(q, P)[-1]
    fw = np.asarray(fw)
    f, n = fw[:3], fw[3:]
    return np.concatenate([R.T @ f, R.T @ (n - _cross(p, f))])


def fext_list(q, fext6=None, frame="local", P: Params = None):
    """pinocchio's f_ext vector (6 local spatial forces) for a wrench on joint 6 given in
    `frame` ("local": as it is; "world": converted at q), or None."""
    if fext6 is None:
        return None
    f = wrench_world_to_local(q, fext6, P) if frame == "world" else np.asarray(fext6)
    return [np.zeros(6)] * (NJ - 1) + [f]


def aba_derivatives(q, v, tau, P: Params = None, fext6=None, frame="local"):
    """pin.computeABADerivatives -> (da/dq, da/dv, da/dtau=Minv) and ddq.

    Complex-step on RNEA at (q, v, a=ddq): exact to rounding.  With a joint-6 wrench fext6
    (frame "local" or "world", see fext_list) the derivatives include it; a world-frame wrench's
    conversion to the local frame depends on q and is differentiated through."""
    P = P or params()
    M = crba(q, P)
    Minv = np.linalg.inv(M)
    Minv = 0.5 * (Minv + Minv.T)
    a = aba(q, v, tau, P, fext_list(q, fext6, frame, P))
    dtq = np.zeros((NJ, NJ))
    dtv = np.zeros((NJ, NJ))
    fv = fext_list(q, fext6, frame, P)
    for j in range(NJ):
        e = np.zeros(NJ, dtype=complex)
        e[j] = 1j * H_CS
        fq = fext_list(q + e, fext6, frame, P)
        dtq[:, j] = np.imag(_rnea_impl(q + e, v.astype(complex), a.astype(complex), P, True, fq)) / H_CS
        dtv[:, j] = np.imag(_rnea_impl(q.astype(complex), v + e, a.astype(complex), P, True, fv)) / H_CS
    return -Minv @ dtq, -Minv @ dtv, Minv, a


def integrate(q, dq):
    """pin.integrate on revolute joints (src/osqp_solver.py:77)."""
    return q + dq


def rk4(q, v, u, dt, fext=None, P: Params = None, fext6_world=None):
    """Plant integrator restating src/utils.py:3-18 (4 x pin.aba with optional f_ext).
    fext6_world: a world-frame joint-6 wrench, converted ONCE at the start q and held over the
    four stages, as the reference's host plant does (src/gato_mpc_batch_sample.py:270-279)."""
    if fext6_world is not None:
        fext = fext_list(q, fext6_world, "world", P)
    k1q = v
    k1v = aba(q, v, u, P, fext)
    q2 = integrate(q, k1q * dt / 2)
    k2q = v + k1v * dt / 2
    k2v = aba(q2, k2q, u, P, fext)
    q3 = integrate(q, k2q * dt / 2)
    k3q = v + k2v * dt / 2
    k3v = aba(q3, k3q, u, P, fext)
    q4 = integrate(q, k3q * dt)
    k4q = v + k3v * dt
    k4v = aba(q4, k4q, u, P, fext)
    v_next = v + (dt / 6) * (k1v + 2 * k2v + 2 * k3v + k4v)
    avg_v = (k1q + 2 * k2q + 2 * k3q + k4q) / 6
    q_next = integrate(q, avg_v * dt)
    return q_next, v_next
