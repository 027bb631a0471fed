"""ORACLE (test infrastructure only) — restatement of MPC_OSQP.run_mpc (reference
src/osqp_mpc.py:14-72): goal switching (:31-43), sqp warm-start (:46), rk4 plant step with
the PREVIOUS trajectory's first control (:48-61, quirk kept), shift (:64-65) and the
first/last state pins (:68-70).  rk4 without f_ext, as the notebook run used
(notebooks/pin_mpc_indy7.ipynb cell 2; src/utils.py:3-18 later gained an f_ext arg)."""
import numpy as np

from . import rbd


def run_mpc_ref(sqp, xstart, endpoints, num_steps=500, on_step=None):
    s = sqp.solver
    nq, nv, nx, nu = s.nq, s.nv, s.nx, s.nu
    xcur = np.asarray(xstart, dtype=float)
    ei = 0
    goal = np.tile(endpoints[ei], s.N)
    XU = np.zeros(s.N * (nx + nu) - nu)
    XU = sqp.sqp(xcur, goal, XU)
    dists, xpath = [], []
    for i in range(num_steps):
        d = np.linalg.norm(s.eepos(xcur[:nq]) - goal[:3])
        if d < 1e-1:
            ei = (ei + 1) % len(endpoints)
            goal = np.tile(endpoints[ei], s.N)
        dists.append(d)
        if on_step:
            on_step(i, d)
        if d > 1.1:
            break
        xu_new = sqp.sqp(xcur, goal, XU)
        sim_time, sim_steps = 0.01, 0
        while sim_time > 0:
            ts = min(sim_time, s.dt)
            u = XU[sim_steps * (nx + nu) + nx:(sim_steps + 1) * (nx + nu)]
            qn, vn = rbd.rk4(xcur[:nq], xcur[nq:nx], u, ts)
            xcur = np.concatenate([qn, vn])
            if ts > 0.5 * s.dt:
                sim_steps += 1
            sim_time -= ts
            xpath.append(xcur[:nq].copy())
        if sim_steps > 0:
            XU[:-(sim_steps) * (nx + nu) or len(XU)] = xu_new[sim_steps * (nx + nu):]
        XU[:nx] = xcur
        XU[-nx:] = np.hstack([np.ones(nq), np.zeros(nv)])
    return xpath, dists
