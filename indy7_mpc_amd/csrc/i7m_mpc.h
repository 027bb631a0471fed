// i7m_mpc.h — the closed-loop MPC driver of the reference (MPC_OSQP.run_mpc, src/osqp_mpc.py:
// 14-72) for B independent instances on the device: per MPC step a goal kernel, the batched SQP
// solve (i7m_api.hip run_sqp) and an advance kernel, the instance state (xcur, XU, goal, goal
// index, alive flag) resident in HBM for the whole run.
#pragma once

#include "i7m_kernels.h"

namespace i7m {

// src/osqp_mpc.py:31-43, thread per instance: the goal distance of the current state (FK of the
// joint-6 origin), the cyclic goal switch below 0.1 (the goal rows re-tiled), the recorded
// distance (w.r.t. the goal before the switch, as the reference appends it), and the break
// above 1.1 (the instance stops; its later distances are NaN).
__global__ void __launch_bounds__(256) k_mpc_goal(const DevModel* __restrict__ Mg, int B, int N,
                                                  const double* __restrict__ xs, double* __restrict__ goals,
                                                  const double* __restrict__ endpoints, int n_endpoints,
                                                  int* __restrict__ goal_idx, int* __restrict__ alive,
                                                  double* __restrict__ dist_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (!alive[b]) {
    dist_out[b] = __builtin_nan("");
    return;
  }
  double c[6], s[6], p[3];
  sincos6(xs + 12L * b, c, s);
  fk_pos(*Mg, c, s, p);
  double* g = goals + (long)b * 3 * N;
  const double e0 = p[0] - g[0], e1 = p[1] - g[1], e2 = p[2] - g[2];
  const double d = sqrt(e0 * e0 + e1 * e1 + e2 * e2);
  if (d < 1e-1) {
    const int ei = (goal_idx[b] + 1) % n_endpoints;
    goal_idx[b] = ei;
    const double* ep = endpoints + 3 * ei;
    for (int k = 0; k < N; ++k) {
      g[3 * k] = ep[0];
      g[3 * k + 1] = ep[1];
      g[3 * k + 2] = ep[2];
    }
  }
  dist_out[b] = d;
  if (d > 1.1) alive[b] = 0;
}

// src/osqp_mpc.py:48-70, one wave per instance: the plant (lane 0) integrates the reference's
// hard-coded 0.01 s of trajectory-optimisation time in rk4 steps of min(remaining, dt), each with
// the control of knot sim_steps of the PREVIOUS trajectory XU (the reference's quirk, :56),
// counting the steps longer than dt / 2 (:51-61; for dt = 0.01 one step, sim_steps = 1); then
// XU[:-18 s] = xu_new[18 s:] for s = sim_steps > 0 (the warm-start shift, :64-65; XU's last 18 s
// entries keep their old values) and the pins XU[:12] = xcur, XU[-12:] = [1]*6 + [0]*6 (:68-70).
// q_out: each instance's q after the plant step (NaN for a stopped instance).
__global__ void __launch_bounds__(64) k_mpc_advance(const DevModel* __restrict__ Mg, int B, int N, double dt,
                                                    double* __restrict__ xs, double* __restrict__ XU,
                                                    const double* __restrict__ xu_new, const int* __restrict__ alive,
                                                    double* __restrict__ q_out) {
  const int b = blockIdx.x;
  if (b >= B) return;
  const int l = threadIdx.x;
  if (!alive[b]) {
    if (l < 6) q_out[6L * b + l] = __builtin_nan("");
    return;
  }
  const int T = 18 * N - 6;
  __shared__ double xn[12];
  __shared__ int steps;
  double* X = XU + (long)b * T;
  const double* Xn = xu_new + (long)b * T;
  double* x = xs + 12L * b;
  if (l == 0) {
    double q[6], v[6], qo[6], vo[6];
    for (int r = 0; r < 6; ++r) {
      q[r] = x[r];
      v[r] = x[6 + r];
    }
    double sim_time = 0.01;
    int sim_steps = 0;
    while (sim_time > 0.0) {
      const double ts = fmin(sim_time, dt);
      const int kk = sim_steps < N - 1 ? sim_steps : N - 2;  // (the reference would index past XU)
      rk4_step(*Mg, q, v, X + 18 * kk + 12, ts, nullptr, false, qo, vo);
      for (int r = 0; r < 6; ++r) {
        q[r] = qo[r];
        v[r] = vo[r];
      }
      if (ts > 0.5 * dt) ++sim_steps;
      sim_time -= ts;
    }
    for (int r = 0; r < 6; ++r) {
      xn[r] = q[r];
      xn[6 + r] = v[r];
    }
    steps = sim_steps;
  }
  __syncthreads();  // the controls X[...] are read before the shift overwrites them
  const int sh = 18 * steps;
  if (sh > 0)
    for (int e = l; e < T - sh; e += 64) X[e] = Xn[e + sh];
  __syncthreads();
  if (l < 12) {
    x[l] = xn[l];
    X[l] = xn[l];
    X[T - 12 + l] = l < 6 ? 1.0 : 0.0;
  }
  if (l < 6) q_out[6L * b + l] = xn[l];
}

}  // namespace i7m
