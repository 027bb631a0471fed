"""Drop-in for reference ``MPC_OSQP`` (src/osqp_mpc.py:5-72): the closed-loop driver.

Each MPC step is one GPU SQP solve (SQP_OSQP.sqp) plus the GPU rk4 plant step.  The
reference's quirks are kept on purpose: the plant is driven with the PREVIOUS trajectory's
first control (``XU``, not ``xu_new``, :56), the warm start is shifted by the number of full
dt steps simulated (:64-65), and the first/last states are pinned to xcur and
[1,...,1, 0,...,0] (:68-70).  The reference's rk4 call passes no f_ext (:56); the external
force is zero here as in the notebook run (notebooks/pin_mpc_indy7.ipynb cell 2).
"""
from __future__ import annotations

import numpy as np

from .utils import rk4


class MPC_OSQP:
    def __init__(self, model, sqp_optimizer, solver):
        self.model = model
        self.model.gravity.linear = np.array([0, 0, -9.81])  # reference :8-9
        self.sqp_optimizer = sqp_optimizer
        self.solver = solver
        self.xpath = []
        self.goal_distances = []

    def run_mpc(self, xstart, endpoints, num_steps=500, verbose=True):
        nq, nv, nx, nu = self.solver.nq, self.solver.nv, self.solver.nx, self.solver.nu
        xcur = np.asarray(xstart, dtype=float)
        endpoint_ind = 0
        endpoint = endpoints[endpoint_ind]
        eepos_goal = np.tile(endpoint, self.solver.N).T
        XU = np.zeros(self.solver.N * (nx + nu) - nu)
        XU = self.sqp_optimizer.sqp(xcur, eepos_goal, XU)
        for i in range(num_steps):
            cur_eepos = self.solver.eepos(xcur[:nq])
            goaldist = np.linalg.norm(cur_eepos - eepos_goal[:3])
            if goaldist < 1e-1:
                if verbose:
                    print("switching goals")
                endpoint_ind = (endpoint_ind + 1) % len(endpoints)
                endpoint = endpoints[endpoint_ind]
                eepos_goal = np.tile(endpoint, self.solver.N).T
            if verbose:
                print(goaldist)
            self.goal_distances.append(goaldist)
            if goaldist > 1.1:
                if verbose:
                    print("breaking on big goal dist")
                break
            xu_new = self.sqp_optimizer.sqp(xcur, eepos_goal, XU)
            trajopt_time = 0.01
            sim_time = trajopt_time
            sim_steps = 0
            while sim_time > 0:
                timestep = min(sim_time, self.solver.dt)
                control = XU[sim_steps * (nx + nu) + nx:(sim_steps + 1) * (nx + nu)]
                qn, vn = rk4(self.model, self.solver.data, xcur[:nq], xcur[nq:nx], control, timestep)
                xcur = np.concatenate([qn, vn])
                if timestep > 0.5 * self.solver.dt:
                    sim_steps += 1
                sim_time -= timestep
                self.xpath.append(xcur[:nq])
            if sim_steps > 0:
                XU[:-(sim_steps) * (nx + nu) or len(XU)] = xu_new[(sim_steps) * (nx + nu):]
            XU[:nx] = xcur.reshape(-1)
            XU[-nx:] = np.hstack([np.ones(nq), np.zeros(nv)])
        return self.xpath

    def run_mpc_batch(self, xstart_batch, endpoints, num_steps=500):
        """``run_mpc`` for B independent instances at once, every step on the GPU (i7m_mpc_run:
        goal switching, the batched SQP, the rk4 plant and the warm-start shift and pins of
        :14-72 per instance; the batch axis of src/gato_mpc_batch.py:76-217).  Returns
        (q_path (num_steps, B, 6), goal_distances (num_steps, B)); an instance that stops (goal
        distance > 1.1) has NaN from the step after its last distance on."""
        xs = np.asarray(xstart_batch, dtype=float).reshape(-1, self.solver.nx)
        h = self.sqp_optimizer._handle_for(xs.shape[0])
        d, q, xc, xu = h.mpc_run(xs, np.asarray(endpoints, dtype=float).reshape(-1, 3), num_steps)
        self.batch_xcur, self.batch_XU = xc, xu
        return q, d

