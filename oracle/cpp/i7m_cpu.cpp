// ORACLE (test/bench infrastructure only) — C++ CPU restatement of the reference hot path.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the
// product (indy7_mpc_amd) never does.  Two uses:
//   * bench.py's CPU baseline ("port"): the same SQP as src/osqp_sqp.py:76-93 with the QP of
//     src/osqp_solver.py:137-143 solved exactly, timed on the host cores (OpenMP over problems);
//   * the instrumented flop count of that algorithm (template on an op-counting scalar) that
//     bench.py's FP64 roofline uses (SURVEY.md §8d asks for an instrumented count).
// Follows, function by function:
//   rnea / crba / forward_dynamics   pin.aba / computeABADerivatives (src/osqp_solver.py:71-77,
//                                    src/osqp_sqp.py:40) — local-frame RNEA, forward-mode dual
//                                    tangents for the derivatives (da/dx = -Minv dRNEA/dx)
//   fk_jac                           eepos / d_eepos (src/osqp_solver.py:146-155)
//   linearize                        update_constraint_matrix / update_cost_matrix (:83-135)
//   riccati                          the equality-constrained QP (:137-143), exact
//   merit / linesearch               eepos_cost, integrator_err, linesearch (src/osqp_sqp.py:13-74)
//   sqp                              src/osqp_sqp.py:76-93
//   ipm (box_mask != 0)              config 4's box rows (no reference
//                                    counterpart): oracle/box_ipm.py::ipm_box, Newton steps by
//                                    riccati with the (Sigma, h) shifts, as i7m_box.h on the GPU
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <vector>

namespace {

// ---------------------------------------------------------------- op-counting scalar
struct CountD {
  double v;
  static thread_local uint64_t flops;
  CountD() : v(0) {}
  CountD(double x) : v(x) {}
};
thread_local uint64_t CountD::flops = 0;
inline CountD operator+(CountD a, CountD b) { ++CountD::flops; return CountD(a.v + b.v); }
inline CountD operator-(CountD a, CountD b) { ++CountD::flops; return CountD(a.v - b.v); }
inline CountD operator*(CountD a, CountD b) { ++CountD::flops; return CountD(a.v * b.v); }
inline CountD operator/(CountD a, CountD b) { ++CountD::flops; return CountD(a.v / b.v); }
inline CountD operator-(CountD a) { return CountD(-a.v); }
inline CountD& operator+=(CountD& a, CountD b) { a = a + b; return a; }
inline CountD& operator-=(CountD& a, CountD b) { a = a - b; return a; }
inline bool operator<(CountD a, CountD b) { return a.v < b.v; }
inline bool operator<=(CountD a, CountD b) { return a.v <= b.v; }
inline CountD sqrt(CountD a) { ++CountD::flops; return CountD(std::sqrt(a.v)); }
inline CountD fabs(CountD a) { return CountD(std::fabs(a.v)); }
inline void sincos2(CountD q, CountD* s, CountD* c) { CountD::flops += 2; *s = std::sin(q.v); *c = std::cos(q.v); }
inline void sincos2(double q, double* s, double* c) { *s = std::sin(q); *c = std::cos(q); }
inline double val(double x) { return x; }
inline double val(CountD x) { return x.v; }
using std::sqrt;
using std::fabs;

template <class R>
struct Dual {
  R v, d;
  Dual() : v(0), d(0) {}
  Dual(R a) : v(a), d(0) {}
  Dual(R a, R b) : v(a), d(b) {}
};
template <class R> inline Dual<R> operator+(Dual<R> a, Dual<R> b) { return {a.v + b.v, a.d + b.d}; }
template <class R> inline Dual<R> operator-(Dual<R> a, Dual<R> b) { return {a.v - b.v, a.d - b.d}; }
template <class R> inline Dual<R> operator*(Dual<R> a, Dual<R> b) { return {a.v * b.v, a.v * b.d + a.d * b.v}; }
template <class R> inline Dual<R> operator*(R a, Dual<R> b) { return {a * b.v, a * b.d}; }

struct Model {
  double Rp[6][9], tp[6][3], m[6], h[6][3], Io[6][6], g[3];
  double qlo[6], qhi[6], vlim[6], ulim[6];  // description/indy7.urdf:203-238 <limit>
};

Model make_model(const double* p) {
  // packed layout == i7m_model (include/indy7_mpc.h)
  Model M;
  const double* R = p;
  const double* t = p + 54;
  const double* mass = p + 72;
  const double* com = p + 78;
  const double* I = p + 96;
  const double* g = p + 132;
  for (int i = 0; i < 6; ++i) {
    for (int k = 0; k < 9; ++k) M.Rp[i][k] = R[9 * i + k];
    for (int k = 0; k < 3; ++k) M.tp[i][k] = t[3 * i + k];
    M.m[i] = mass[i];
    const double* c = com + 3 * i;
    for (int k = 0; k < 3; ++k) M.h[i][k] = mass[i] * c[k];
    const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    const double* Ic = I + 6 * i;
    M.Io[i][0] = Ic[0] + mass[i] * (cc - c[0] * c[0]);
    M.Io[i][1] = Ic[1] - mass[i] * c[0] * c[1];
    M.Io[i][2] = Ic[2] - mass[i] * c[0] * c[2];
    M.Io[i][3] = Ic[3] + mass[i] * (cc - c[1] * c[1]);
    M.Io[i][4] = Ic[4] - mass[i] * c[1] * c[2];
    M.Io[i][5] = Ic[5] + mass[i] * (cc - c[2] * c[2]);
  }
  for (int k = 0; k < 3; ++k) M.g[k] = g[k];
  for (int k = 0; k < 6; ++k) {
    M.qlo[k] = p[135 + k];
    M.qhi[k] = p[141 + k];
    M.vlim[k] = p[147 + k];
    M.ulim[k] = p[153 + k];
  }
  return M;
}

// Local-frame RNEA on scalar type T (R or Dual<R>) with base scalar R for constants.
template <class R, class T>
void rnea(const Model& M, const T* c, const T* s, const T* qd, const T* qdd, bool grav, const double* f6, T* tau) {
  auto K = [](double x) -> T { return T(R(x)); };
  T vl[3] = {K(0), K(0), K(0)}, vw[3] = {K(0), K(0), K(0)};
  T al[3] = {K(grav ? -M.g[0] : 0), K(grav ? -M.g[1] : 0), K(grav ? -M.g[2] : 0)}, aw[3] = {K(0), K(0), K(0)};
  T f[6][6];
  for (int i = 0; i < 6; ++i) {
    const double* Rp = M.Rp[i];
    const double* t = M.tp[i];
    auto to_child = [&](T* l, T* w) {
      T x0 = l[0] - (K(t[1]) * w[2] - K(t[2]) * w[1]);
      T x1 = l[1] - (K(t[2]) * w[0] - K(t[0]) * w[2]);
      T x2 = l[2] - (K(t[0]) * w[1] - K(t[1]) * w[0]);
      T y0 = K(Rp[0]) * x0 + K(Rp[3]) * x1 + K(Rp[6]) * x2;
      T y1 = K(Rp[1]) * x0 + K(Rp[4]) * x1 + K(Rp[7]) * x2;
      T y2 = K(Rp[2]) * x0 + K(Rp[5]) * x1 + K(Rp[8]) * x2;
      T z0 = K(Rp[0]) * w[0] + K(Rp[3]) * w[1] + K(Rp[6]) * w[2];
      T z1 = K(Rp[1]) * w[0] + K(Rp[4]) * w[1] + K(Rp[7]) * w[2];
      T z2 = K(Rp[2]) * w[0] + K(Rp[5]) * w[1] + K(Rp[8]) * w[2];
      l[0] = c[i] * y0 + s[i] * y1; l[1] = c[i] * y1 - s[i] * y0; l[2] = y2;
      w[0] = c[i] * z0 + s[i] * z1; w[1] = c[i] * z1 - s[i] * z0; w[2] = z2;
    };
    to_child(vl, vw);
    to_child(al, aw);
    vw[2] = vw[2] + qd[i];
    al[0] = al[0] + vl[1] * qd[i];
    al[1] = al[1] - vl[0] * qd[i];
    aw[0] = aw[0] + vw[1] * qd[i];
    aw[1] = aw[1] - vw[0] * qd[i];
    aw[2] = aw[2] + qdd[i];
    auto imul = [&](const T* l, const T* w, T* fl, T* fn) {
      const double m = M.m[i];
      const double* h = M.h[i];
      const double* I = M.Io[i];
      fl[0] = K(m) * l[0] - (K(h[1]) * w[2] - K(h[2]) * w[1]);
      fl[1] = K(m) * l[1] - (K(h[2]) * w[0] - K(h[0]) * w[2]);
      fl[2] = K(m) * l[2] - (K(h[0]) * w[1] - K(h[1]) * w[0]);
      fn[0] = K(I[0]) * w[0] + K(I[1]) * w[1] + K(I[2]) * w[2] + (K(h[1]) * l[2] - K(h[2]) * l[1]);
      fn[1] = K(I[1]) * w[0] + K(I[3]) * w[1] + K(I[4]) * w[2] + (K(h[2]) * l[0] - K(h[0]) * l[2]);
      fn[2] = K(I[2]) * w[0] + K(I[4]) * w[1] + K(I[5]) * w[2] + (K(h[0]) * l[1] - K(h[1]) * l[0]);
    };
    T hl[3], hn[3], il[3], in[3];
    imul(vl, vw, hl, hn);
    imul(al, aw, il, in);
    f[i][0] = il[0] + (vw[1] * hl[2] - vw[2] * hl[1]);
    f[i][1] = il[1] + (vw[2] * hl[0] - vw[0] * hl[2]);
    f[i][2] = il[2] + (vw[0] * hl[1] - vw[1] * hl[0]);
    f[i][3] = in[0] + (vw[1] * hn[2] - vw[2] * hn[1]) + (vl[1] * hl[2] - vl[2] * hl[1]);
    f[i][4] = in[1] + (vw[2] * hn[0] - vw[0] * hn[2]) + (vl[2] * hl[0] - vl[0] * hl[2]);
    f[i][5] = in[2] + (vw[0] * hn[1] - vw[1] * hn[0]) + (vl[0] * hl[1] - vl[1] * hl[0]);
  }
  if (f6)
    for (int k = 0; k < 6; ++k) f[5][k] = f[5][k] - K(f6[k]);
  for (int i = 5; i >= 0; --i) {
    tau[i] = f[i][5];
    if (i == 0) break;
    const double* Rp = M.Rp[i];
    const double* t = M.tp[i];
    T x0 = c[i] * f[i][0] - s[i] * f[i][1], x1 = s[i] * f[i][0] + c[i] * f[i][1], x2 = f[i][2];
    T F0 = K(Rp[0]) * x0 + K(Rp[1]) * x1 + K(Rp[2]) * x2;
    T F1 = K(Rp[3]) * x0 + K(Rp[4]) * x1 + K(Rp[5]) * x2;
    T F2 = K(Rp[6]) * x0 + K(Rp[7]) * x1 + K(Rp[8]) * x2;
    x0 = c[i] * f[i][3] - s[i] * f[i][4]; x1 = s[i] * f[i][3] + c[i] * f[i][4]; x2 = f[i][5];
    T N0 = K(Rp[0]) * x0 + K(Rp[1]) * x1 + K(Rp[2]) * x2;
    T N1 = K(Rp[3]) * x0 + K(Rp[4]) * x1 + K(Rp[5]) * x2;
    T N2 = K(Rp[6]) * x0 + K(Rp[7]) * x1 + K(Rp[8]) * x2;
    f[i - 1][0] = f[i - 1][0] + F0;
    f[i - 1][1] = f[i - 1][1] + F1;
    f[i - 1][2] = f[i - 1][2] + F2;
    f[i - 1][3] = f[i - 1][3] + N0 + (K(t[1]) * F2 - K(t[2]) * F1);
    f[i - 1][4] = f[i - 1][4] + N1 + (K(t[2]) * F0 - K(t[0]) * F2);
    f[i - 1][5] = f[i - 1][5] + N2 + (K(t[0]) * F1 - K(t[1]) * F0);
  }
}

template <class R>
void chol6(R A[6][6]) {
  for (int j = 0; j < 6; ++j) {
    R d = A[j][j];
    for (int k = 0; k < j; ++k) d = d - A[j][k] * A[j][k];
    d = sqrt(d);
    A[j][j] = d;
    for (int i = j + 1; i < 6; ++i) {
      R v = A[i][j];
      for (int k = 0; k < j; ++k) v = v - A[i][k] * A[j][k];
      A[i][j] = v / d;
    }
  }
}
template <class R>
void chol6_solve(const R L[6][6], R* b) {
  for (int i = 0; i < 6; ++i) {
    R v = b[i];
    for (int k = 0; k < i; ++k) v = v - L[i][k] * b[k];
    b[i] = v / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    R v = b[i];
    for (int k = i + 1; k < 6; ++k) v = v - L[k][i] * b[k];
    b[i] = v / L[i][i];
  }
}

// Composite-rigid-body M(q) (same recursion as the GPU's crba), then a = M^-1 (tau - b).
template <class R>
void crba(const Model& Md, const R* c, const R* s, R Mq[6][6]) {
  R cm[6], ch[6][3], cI[6][6];
  for (int i = 0; i < 6; ++i) {
    cm[i] = R(Md.m[i]);
    for (int k = 0; k < 3; ++k) ch[i][k] = R(Md.h[i][k]);
    for (int k = 0; k < 6; ++k) cI[i][k] = R(Md.Io[i][k]);
  }
  for (int i = 5; i >= 0; --i) {
    R fl[3] = {R(0) - ch[i][1], ch[i][0], R(0)};
    R fn[3] = {cI[i][2], cI[i][4], cI[i][5]};
    Mq[i][i] = fn[2];
    for (int j = i; j >= 1; --j) {
      const double* Rp = Md.Rp[j];
      const double* t = Md.tp[j];
      R x0 = c[j] * fl[0] - s[j] * fl[1], x1 = s[j] * fl[0] + c[j] * fl[1], x2 = fl[2];
      R F0 = R(Rp[0]) * x0 + R(Rp[1]) * x1 + R(Rp[2]) * x2;
      R F1 = R(Rp[3]) * x0 + R(Rp[4]) * x1 + R(Rp[5]) * x2;
      R F2 = R(Rp[6]) * x0 + R(Rp[7]) * x1 + R(Rp[8]) * x2;
      x0 = c[j] * fn[0] - s[j] * fn[1]; x1 = s[j] * fn[0] + c[j] * fn[1]; x2 = fn[2];
      R N0 = R(Rp[0]) * x0 + R(Rp[1]) * x1 + R(Rp[2]) * x2;
      R N1 = R(Rp[3]) * x0 + R(Rp[4]) * x1 + R(Rp[5]) * x2;
      R N2 = R(Rp[6]) * x0 + R(Rp[7]) * x1 + R(Rp[8]) * x2;
      fn[0] = N0 + (R(t[1]) * F2 - R(t[2]) * F1);
      fn[1] = N1 + (R(t[2]) * F0 - R(t[0]) * F2);
      fn[2] = N2 + (R(t[0]) * F1 - R(t[1]) * F0);
      fl[0] = F0; fl[1] = F1; fl[2] = F2;
      Mq[i][j - 1] = fn[2];
      Mq[j - 1][i] = fn[2];
    }
    if (i > 0) {
      const double* Rp = Md.Rp[i];
      const double* t = Md.tp[i];
      const R m = cm[i];
      R hz[3] = {c[i] * ch[i][0] - s[i] * ch[i][1], s[i] * ch[i][0] + c[i] * ch[i][1], ch[i][2]};
      R hr[3];
      for (int r = 0; r < 3; ++r) hr[r] = R(Rp[3 * r]) * hz[0] + R(Rp[3 * r + 1]) * hz[1] + R(Rp[3 * r + 2]) * hz[2];
      const R* I = cI[i];
      const R cc = c[i] * c[i], ss = s[i] * s[i], cs = c[i] * s[i];
      R A[3][3];
      A[0][0] = cc * I[0] - R(2.0) * cs * I[1] + ss * I[3];
      A[1][1] = ss * I[0] + R(2.0) * cs * I[1] + cc * I[3];
      A[0][1] = cs * (I[0] - I[3]) + (cc - ss) * I[1];
      A[0][2] = c[i] * I[2] - s[i] * I[4];
      A[1][2] = s[i] * I[2] + c[i] * I[4];
      A[2][2] = I[5];
      A[1][0] = A[0][1]; A[2][0] = A[0][2]; A[2][1] = A[1][2];
      R RA[3][3], Bm[3][3];
      for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) RA[r][q] = R(Rp[3 * r]) * A[0][q] + R(Rp[3 * r + 1]) * A[1][q] + R(Rp[3 * r + 2]) * A[2][q];
      for (int r = 0; r < 3; ++r)
        for (int q = r; q < 3; ++q) Bm[r][q] = RA[r][0] * R(Rp[3 * q]) + RA[r][1] * R(Rp[3 * q + 1]) + RA[r][2] * R(Rp[3 * q + 2]);
      const R ht = hr[0] * R(t[0]) + hr[1] * R(t[1]) + hr[2] * R(t[2]);
      const R tt = R(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
      const R dg = R(2.0) * ht + m * tt;
      const int iu[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
      for (int k = 0; k < 6; ++k) {
        const int r = iu[k][0], q = iu[k][1];
        R v = Bm[r][q] - (R(t[r]) * hr[q] + hr[r] * R(t[q])) - m * R(t[r]) * R(t[q]);
        if (r == q) v = v + dg;
        cI[i - 1][k] = cI[i - 1][k] + v;
      }
      for (int k = 0; k < 3; ++k) ch[i - 1][k] = ch[i - 1][k] + hr[k] + m * R(t[k]);
      cm[i - 1] = cm[i - 1] + m;
    }
  }
}

template <class R>
void forward_dynamics(const Model& Md, const R* c, const R* s, const R* v, const R* tau, const double* f6, R L[6][6],
                      R* a) {
  R z[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
  crba(Md, c, s, L);
  chol6(L);
  R b[6];
  rnea<R, R>(Md, c, s, v, z, true, f6, b);
  for (int i = 0; i < 6; ++i) a[i] = tau[i] - b[i];
  chol6_solve(L, a);
}

// World-frame wrench [f; n] about the world origin -> joint 6's local frame at (c, s) = cos / sin(q):
// data.oMi[6].actInv (src/gato_mpc_batch_sample.py:151-161): f_l = R' f, n_l = R' (n - p x f)
template <class R>
void wrench_world_to_local(const Model& Md, const R* c, const R* s, const double* fw, double* fl) {
  double Rw[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, p[3] = {0, 0, 0};
  for (int i = 0; i < 6; ++i) {
    const double* Rp = Md.Rp[i];
    const double* t = Md.tp[i];
    const double ci = val(c[i]), si = val(s[i]);
    double np_[3], RR[3][3];
    for (int r = 0; r < 3; ++r) np_[r] = p[r] + Rw[r][0] * t[0] + Rw[r][1] * t[1] + Rw[r][2] * t[2];
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q) RR[r][q] = Rw[r][0] * Rp[q] + Rw[r][1] * Rp[3 + q] + Rw[r][2] * Rp[6 + q];
    for (int r = 0; r < 3; ++r) {
      Rw[r][0] = RR[r][0] * ci + RR[r][1] * si;
      Rw[r][1] = RR[r][1] * ci - RR[r][0] * si;
      Rw[r][2] = RR[r][2];
      p[r] = np_[r];
    }
  }
  const double m0 = fw[3] - (p[1] * fw[2] - p[2] * fw[1]);
  const double m1 = fw[4] - (p[2] * fw[0] - p[0] * fw[2]);
  const double m2 = fw[5] - (p[0] * fw[1] - p[1] * fw[0]);
  for (int q = 0; q < 3; ++q) {
    fl[q] = Rw[0][q] * fw[0] + Rw[1][q] * fw[1] + Rw[2][q] * fw[2];
    fl[3 + q] = Rw[0][q] * m0 + Rw[1][q] * m1 + Rw[2][q] * m2;
  }
}

template <class R>
void fk_jac(const Model& Md, const R* c, const R* s, R* p, R J[3][6]) {
  R Rw[3][3] = {{R(1), R(0), R(0)}, {R(0), R(1), R(0)}, {R(0), R(0), R(1)}};
  R pos[3] = {R(0), R(0), R(0)}, zs[6][3], ps[6][3];
  for (int i = 0; i < 6; ++i) {
    const double* Rp = Md.Rp[i];
    const double* t = Md.tp[i];
    R np_[3], RR[3][3];
    for (int r = 0; r < 3; ++r) np_[r] = pos[r] + Rw[r][0] * R(t[0]) + Rw[r][1] * R(t[1]) + Rw[r][2] * R(t[2]);
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q) RR[r][q] = Rw[r][0] * R(Rp[q]) + Rw[r][1] * R(Rp[3 + q]) + Rw[r][2] * R(Rp[6 + q]);
    for (int r = 0; r < 3; ++r) {
      Rw[r][0] = RR[r][0] * c[i] + RR[r][1] * s[i];
      Rw[r][1] = RR[r][1] * c[i] - RR[r][0] * s[i];
      Rw[r][2] = RR[r][2];
      zs[i][r] = RR[r][2];
      ps[i][r] = np_[r];
      pos[r] = np_[r];
    }
  }
  for (int r = 0; r < 3; ++r) p[r] = pos[r];
  if (J)
    for (int j = 0; j < 6; ++j) {
      R d0 = pos[0] - ps[j][0], d1 = pos[1] - ps[j][1], d2 = pos[2] - ps[j][2];
      J[0][j] = zs[j][1] * d2 - zs[j][2] * d1;
      J[1][j] = zs[j][2] * d0 - zs[j][0] * d2;
      J[2][j] = zs[j][0] * d1 - zs[j][1] * d0;
    }
}

struct Params {
  int N, regularize, max_iters, goal_stride;
  // external wrench frame: 0 = constant in joint 6's frame (pinocchio f_ext), 1 = a WORLD-frame
  // spatial force about the world origin, as batch_sqp's callers give it (gato_controller.py:
  // 77-81,120-129), converted per configuration by oMi[6].actInv (src/gato_mpc_batch_sample.py:
  // 151-161) — the GPU's I7M_WRENCH_WORLD (i7m_dynamics.h wrench_world_to_local)
  int fext_world;
  double dt, dQ, R, QN, eps, mu, step_tol;
  // config 4 box rows (oracle/box_ipm.py; 0 = the reference's equality-only QP)
  int box_mask, box_max_iters;
  double box_tol, box_theta, box_eta, box_z0;
};

// ADMM mode settings (OSQP's defaults; oracle/osqp_admm.py DEFAULTS)
struct AdmmParams {
  double rho0 = 0.1, sigma = 1e-6, alpha = 1.6, eps_abs = 1e-3, eps_rel = 1e-3, adapt_tol = 5.0;
  int max_iter = 4000, check = 25, scaling = 10, gap = 1, adapt_interval = 0;
};

template <class R>
struct Solver {
  const Model& Md;
  Params P;
  int T;
  std::vector<R> lin, cost, K, sol;  // lin (N-1)*114, cost N*10, K (N-1)*84
  // box mode: the interior point's iterate, bound duals, Newton shifts and predictor step
  std::vector<R> bx, bzl, bzu, bsig, bh, bdxa;
  int ipm_iters = 0, ipm_conv = 0;
  double ipm_mu = 0.0;
  Solver(const Model& m, const Params& p) : Md(m), P(p), T(18 * p.N - 6) {
    lin.resize((P.N - 1) * 114);
    cost.resize(P.N * 10);
    K.resize((P.N - 1) * 84);
    sol.resize(T);
    if (P.box_mask) {
      bx.resize(T); bzl.resize(T); bzu.resize(T); bsig.resize(T); bh.resize(T); bdxa.resize(T);
    }
  }

  // Analytic world-frame O(n^2) derivatives (the algorithm of the GPU's k_linearize,
  // indy7_mpc_amd/csrc/i7m_linearize.h), executed once per knot.
  static void mcross(const R* a, const R* b, R* o) {
    o[0] = a[4] * b[2] - a[5] * b[1] + a[1] * b[5] - a[2] * b[4];
    o[1] = a[5] * b[0] - a[3] * b[2] + a[2] * b[3] - a[0] * b[5];
    o[2] = a[3] * b[1] - a[4] * b[0] + a[0] * b[4] - a[1] * b[3];
    o[3] = a[4] * b[5] - a[5] * b[4];
    o[4] = a[5] * b[3] - a[3] * b[5];
    o[5] = a[3] * b[4] - a[4] * b[3];
  }
  static void fcross(const R* m, const R* f, R* o) {
    o[0] = m[4] * f[2] - m[5] * f[1];
    o[1] = m[5] * f[0] - m[3] * f[2];
    o[2] = m[3] * f[1] - m[4] * f[0];
    o[3] = m[4] * f[5] - m[5] * f[4] + m[1] * f[2] - m[2] * f[1];
    o[4] = m[5] * f[3] - m[3] * f[5] + m[2] * f[0] - m[0] * f[2];
    o[5] = m[3] * f[4] - m[4] * f[3] + m[0] * f[1] - m[1] * f[0];
  }
  static R dot6(const R* a, const R* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5]; }
  static void imul(R m, const R* h, const R* I, const R* x, R* o) {
    o[0] = m * x[0] - (h[1] * x[5] - h[2] * x[4]);
    o[1] = m * x[1] - (h[2] * x[3] - h[0] * x[5]);
    o[2] = m * x[2] - (h[0] * x[4] - h[1] * x[3]);
    o[3] = I[0] * x[3] + I[1] * x[4] + I[2] * x[5] + (h[1] * x[2] - h[2] * x[1]);
    o[4] = I[1] * x[3] + I[3] * x[4] + I[4] * x[5] + (h[2] * x[0] - h[0] * x[2]);
    o[5] = I[2] * x[3] + I[4] * x[4] + I[5] * x[5] + (h[0] * x[1] - h[1] * x[0]);
  }
  static void imul0(const R* h, const R* I, const R* x, R* o) {  // rate form: zero mass
    o[0] = R(0) - (h[1] * x[5] - h[2] * x[4]);
    o[1] = R(0) - (h[2] * x[3] - h[0] * x[5]);
    o[2] = R(0) - (h[0] * x[4] - h[1] * x[3]);
    o[3] = I[0] * x[3] + I[1] * x[4] + I[2] * x[5] + (h[1] * x[2] - h[2] * x[1]);
    o[4] = I[1] * x[3] + I[3] * x[4] + I[4] * x[5] + (h[2] * x[0] - h[0] * x[2]);
    o[5] = I[2] * x[3] + I[4] * x[4] + I[5] * x[5] + (h[0] * x[1] - h[1] * x[0]);
  }

  void linearize(const R* X, const double* goal, const double* f6) {
    const R dt = R(P.dt);
    static const int iu[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
    for (int k = 0; k < P.N - 1; ++k) {
      const R* x = X + 18 * k;
      const R* v = x + 6;
      R c[6], s[6];
      for (int i = 0; i < 6; ++i) sincos2(x[i], &s[i], &c[i]);
      R Rw[6][9], pw[6][3], S[6][6], V[6][6], A0[6][6];
      {
        R Rc[9] = {R(1), R(0), R(0), R(0), R(1), R(0), R(0), R(0), R(1)}, pc[3] = {R(0), R(0), R(0)};
        R Vc[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
        R Ac[6] = {R(-Md.g[0]), R(-Md.g[1]), R(-Md.g[2]), R(0), R(0), R(0)};
        for (int i = 0; i < 6; ++i) {
          const double* Rp = Md.Rp[i];
          const double* t = Md.tp[i];
          R np_[3], RR[9];
          for (int r = 0; r < 3; ++r) np_[r] = pc[r] + Rc[3 * r] * R(t[0]) + Rc[3 * r + 1] * R(t[1]) + Rc[3 * r + 2] * R(t[2]);
          for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) RR[3 * r + q] = Rc[3 * r] * R(Rp[q]) + Rc[3 * r + 1] * R(Rp[3 + q]) + Rc[3 * r + 2] * R(Rp[6 + q]);
          for (int r = 0; r < 3; ++r) {
            Rc[3 * r] = RR[3 * r] * c[i] + RR[3 * r + 1] * s[i];
            Rc[3 * r + 1] = RR[3 * r + 1] * c[i] - RR[3 * r] * s[i];
            Rc[3 * r + 2] = RR[3 * r + 2];
            pc[r] = np_[r];
          }
          R* Si = S[i];
          Si[3] = Rc[2]; Si[4] = Rc[5]; Si[5] = Rc[8];
          Si[0] = pc[1] * Si[5] - pc[2] * Si[4];
          Si[1] = pc[2] * Si[3] - pc[0] * Si[5];
          Si[2] = pc[0] * Si[4] - pc[1] * Si[3];
          for (int r = 0; r < 6; ++r) Vc[r] = Vc[r] + Si[r] * v[i];
          R VS[6];
          mcross(Vc, Si, VS);
          for (int r = 0; r < 6; ++r) Ac[r] = Ac[r] + VS[r] * v[i];
          for (int r = 0; r < 9; ++r) Rw[i][r] = Rc[r];
          for (int r = 0; r < 3; ++r) pw[i][r] = pc[r];
          for (int r = 0; r < 6; ++r) { V[i][r] = Vc[r]; A0[i][r] = Ac[r]; }
        }
      }
      // per link: world inertia, rate, momentum, bias force
      R m_[6], h[6][3], Ib[6][6], hd[6][3], Ibd[6][6], hV[6][6], F0[6][6];
      for (int i = 0; i < 6; ++i) {
        const R m = R(Md.m[i]);
        const double* hl = Md.h[i];
        const double* Io = Md.Io[i];
        const R* Rj = Rw[i];
        const R* t = pw[i];
        R Iof[9] = {R(Io[0]), R(Io[1]), R(Io[2]), R(Io[1]), R(Io[3]), R(Io[4]), R(Io[2]), R(Io[4]), R(Io[5])};
        R RI[9], hr[3];
        for (int r = 0; r < 3; ++r)
          for (int q = 0; q < 3; ++q) RI[3 * r + q] = Rj[3 * r] * Iof[q] + Rj[3 * r + 1] * Iof[3 + q] + Rj[3 * r + 2] * Iof[6 + q];
        for (int r = 0; r < 3; ++r) hr[r] = Rj[3 * r] * R(hl[0]) + Rj[3 * r + 1] * R(hl[1]) + Rj[3 * r + 2] * R(hl[2]);
        const R ht = hr[0] * t[0] + hr[1] * t[1] + hr[2] * t[2];
        const R tt = t[0] * t[0] + t[1] * t[1] + t[2] * t[2];
        const R dg = R(2.0) * ht + m * tt;
        for (int e = 0; e < 6; ++e) {
          const int r = iu[e][0], q = iu[e][1];
          R val = RI[3 * r] * Rj[3 * q] + RI[3 * r + 1] * Rj[3 * q + 1] + RI[3 * r + 2] * Rj[3 * q + 2];
          val = val - ((t[r] * hr[q] + hr[r] * t[q]) + m * t[r] * t[q]);
          if (r == q) val = val + dg;
          Ib[i][e] = val;
        }
        for (int r = 0; r < 3; ++r) h[i][r] = hr[r] + m * t[r];
        m_[i] = m;
        imul(m, h[i], Ib[i], V[i], hV[i]);
        R IA[6], VxH[6];
        imul(m, h[i], Ib[i], A0[i], IA);
        fcross(V[i], hV[i], VxH);
        for (int r = 0; r < 6; ++r) F0[i][r] = IA[r] + VxH[r];
        if (f6 && i == 5 && P.fext_world) {
          // a world-frame wrench acts on link 6 as it is (GPU: i7m_linearize.h, FW)
          for (int r = 0; r < 6; ++r) F0[i][r] = F0[i][r] - R(f6[r]);
        } else if (f6 && i == 5) {
          R fw[3], nw[3];
          for (int r = 0; r < 3; ++r) {
            fw[r] = Rj[3 * r] * R(f6[0]) + Rj[3 * r + 1] * R(f6[1]) + Rj[3 * r + 2] * R(f6[2]);
            nw[r] = Rj[3 * r] * R(f6[3]) + Rj[3 * r + 1] * R(f6[4]) + Rj[3 * r + 2] * R(f6[5]);
          }
          for (int r = 0; r < 3; ++r) F0[i][r] = F0[i][r] - fw[r];
          F0[i][3] = F0[i][3] - (nw[0] + (t[1] * fw[2] - t[2] * fw[1]));
          F0[i][4] = F0[i][4] - (nw[1] + (t[2] * fw[0] - t[0] * fw[2]));
          F0[i][5] = F0[i][5] - (nw[2] + (t[0] * fw[1] - t[1] * fw[0]));
        }
        const R* vl = V[i];
        const R* w = V[i] + 3;
        hd[i][0] = m * vl[0] + (w[1] * h[i][2] - w[2] * h[i][1]);
        hd[i][1] = m * vl[1] + (w[2] * h[i][0] - w[0] * h[i][2]);
        hd[i][2] = m * vl[2] + (w[0] * h[i][1] - w[1] * h[i][0]);
        R Ibf[9] = {Ib[i][0], Ib[i][1], Ib[i][2], Ib[i][1], Ib[i][3], Ib[i][4], Ib[i][2], Ib[i][4], Ib[i][5]};
        R WI[9];
        for (int q = 0; q < 3; ++q) {
          WI[q] = w[1] * Ibf[6 + q] - w[2] * Ibf[3 + q];
          WI[3 + q] = w[2] * Ibf[q] - w[0] * Ibf[6 + q];
          WI[6 + q] = w[0] * Ibf[3 + q] - w[1] * Ibf[q];
        }
        const R vh = vl[0] * h[i][0] + vl[1] * h[i][1] + vl[2] * h[i][2];
        for (int e = 0; e < 6; ++e) {
          const int r = iu[e][0], q = iu[e][1];
          R val = WI[3 * r + q] + WI[3 * q + r] - (h[i][r] * vl[q] + vl[r] * h[i][q]);
          if (r == q) val = val + R(2.0) * vh;
          Ibd[i][e] = val;
        }
      }
      // subtree sums (suffix), a_j, e_j, tau0, M
      R cm[6], ch[6][3], cI[6][6], chd[6][3], cId[6][6], HC[6][6], Fc[6][6];
      for (int j = 5; j >= 0; --j) {
        cm[j] = m_[j];
        for (int r = 0; r < 3; ++r) { ch[j][r] = h[j][r]; chd[j][r] = hd[j][r]; }
        for (int r = 0; r < 6; ++r) { cI[j][r] = Ib[j][r]; cId[j][r] = Ibd[j][r]; HC[j][r] = hV[j][r]; Fc[j][r] = F0[j][r]; }
        if (j < 5) {
          cm[j] = cm[j] + cm[j + 1];
          for (int r = 0; r < 3; ++r) { ch[j][r] = ch[j][r] + ch[j + 1][r]; chd[j][r] = chd[j][r] + chd[j + 1][r]; }
          for (int r = 0; r < 6; ++r) {
            cI[j][r] = cI[j][r] + cI[j + 1][r]; cId[j][r] = cId[j][r] + cId[j + 1][r];
            HC[j][r] = HC[j][r] + HC[j + 1][r]; Fc[j][r] = Fc[j][r] + Fc[j + 1][r];
          }
        }
      }
      R aj[6][6], ej[6][6], tau0[6], Lm[6][6];
      for (int j = 0; j < 6; ++j) {
        tau0[j] = dot6(S[j], Fc[j]);
        imul(cm[j], ch[j], cI[j], S[j], aj[j]);
        R bj[6], cj[6];
        imul0(chd[j], cId[j], S[j], bj);
        fcross(S[j], HC[j], cj);
        for (int r = 0; r < 6; ++r) ej[j][r] = bj[r] - cj[r];
      }
      for (int j = 0; j < 6; ++j)
        for (int kk = 0; kk <= j; ++kk) Lm[j][kk] = Lm[kk][j] = dot6(aj[j], S[kk]);
      chol6(Lm);
      R acc[6];
      for (int r = 0; r < 6; ++r) acc[r] = x[12 + r] - tau0[r];
      chol6_solve(Lm, acc);
      // accelerations, full subtree forces
      R dA[6][6], gI[6][6];
      for (int j = 0; j < 6; ++j) {
        for (int r = 0; r < 6; ++r) dA[j][r] = (j ? dA[j - 1][r] : R(0)) + S[j][r] * acc[j];
        imul(m_[j], h[j], Ib[j], dA[j], gI[j]);
      }
      for (int j = 4; j >= 0; --j)
        for (int r = 0; r < 6; ++r) gI[j][r] = gI[j][r] + gI[j + 1][r];
      R W[6][6], Z[6][6], y[6][6], z[6][6];
      for (int j = 0; j < 6; ++j) {
        R Aj[6], t1[6], t2[6], a1[6], a2[6], a3[6], a4[6], b2[6];
        for (int r = 0; r < 6; ++r) { Aj[r] = A0[j][r] + dA[j][r]; Fc[j][r] = Fc[j][r] + gI[j][r]; }
        mcross(S[j], V[j], W[j]);
        mcross(S[j], Aj, t1);
        mcross(W[j], V[j], t2);
        for (int r = 0; r < 6; ++r) Z[j][r] = t1[r] - t2[r];
        fcross(S[j], Fc[j], a1);
        imul(cm[j], ch[j], cI[j], Z[j], a2);
        imul0(chd[j], cId[j], W[j], a3);
        fcross(W[j], HC[j], a4);
        for (int r = 0; r < 6; ++r) y[j][r] = a1[r] - a2[r] - a3[r] - a4[r];
        R b1[6], b3[6];
        imul0(chd[j], cId[j], S[j], b1);
        imul(cm[j], ch[j], cI[j], W[j], b2);
        fcross(S[j], HC[j], b3);
        for (int r = 0; r < 6; ++r) z[j][r] = b1[r] - R(2.0) * b2[r] + b3[r];
      }
      R* o = &lin[114 * k];
      for (int j = 0; j < 6; ++j) {
        R dq[6], dv[6], em[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
        for (int r = 0; r < 6; ++r) {
          if (r >= j) {
            dq[r] = R(0) - (dot6(aj[r], Z[j]) + dot6(ej[r], W[j]));
            dv[r] = dot6(ej[r], S[j]) - R(2.0) * dot6(aj[r], W[j]);
          } else {
            dq[r] = dot6(S[r], y[j]);
            dv[r] = dot6(S[r], z[j]);
          }
        }
        if (f6 && P.fext_world) {
          // the formulas above differentiate forces that turn with the bodies; a world-frame
          // wrench does not, so d tau_r / d q_j gains +S_r . (S_j x* f_w) (i7m_linearize.h)
          R fw6[6], tS[6];
          for (int r = 0; r < 6; ++r) fw6[r] = R(f6[r]);
          fcross(S[j], fw6, tS);
          for (int r = 0; r < 6; ++r) dq[r] = dq[r] + dot6(S[r], tS);
        }
        chol6_solve(Lm, dq);
        chol6_solve(Lm, dv);
        em[j] = R(1);
        chol6_solve(Lm, em);
        for (int r = 0; r < 6; ++r) {
          o[6 * r + j] = R(0) - dt * dq[r];
          o[36 + 6 * r + j] = (r == j ? R(1) : R(0)) - dt * dv[r];
          if (r <= j) o[72 + 6 * r + j] = o[72 + 6 * j + r] = dt * em[r];
        }
      }
      for (int i = 0; i < 6; ++i) o[108 + i] = acc[i];
    }
    for (int k = 0; k < P.N; ++k) {
      const R* q = X + 18 * k;
      R c[6], s[6], p[3], J[3][6];
      for (int i = 0; i < 6; ++i) sincos2(q[i], &s[i], &c[i]);
      fk_jac(Md, c, s, p, J);
      const double* g = goal + (size_t)k * P.goal_stride;
      R e0 = p[0] - R(g[0]), e1 = p[1] - R(g[1]), e2 = p[2] - R(g[2]);
      R nrm = sqrt(e0 * e0 + e1 * e1 + e2 * e2);
      R w = P.regularize ? R(1) / (fabs(nrm) + R(P.eps)) : R(1);
      R* o = &cost[10 * k];
      for (int j = 0; j < 6; ++j) o[j] = e0 * J[0][j] + e1 * J[1][j] + e2 * J[2][j];
      o[6] = R(k == P.N - 1 ? P.QN : 1.0);
      o[7] = R(P.dQ) * w;
      o[8] = R(P.R) * w;
      o[9] = nrm;
    }
  }

  // sg / hs (box mode): the interior point's Newton step solves the same QP with Hessian
  // P + diag(sg) and linear term g + hs (oracle/box_ipm.py, i7m_box.h); null = the plain QP.
  void riccati(const R* X, const R* xs, const R* sg = nullptr, const R* hs = nullptr) {
    const int N = P.N;
    const R dt = R(P.dt);
    R V[12][12], v[12];
    const R* cw = &cost[10 * (N - 1)];
    for (int r = 0; r < 12; ++r)
      for (int c = 0; c < 12; ++c) V[r][c] = (r < 6 && c < 6) ? cw[6] * (cw[r] * cw[c]) : (r == c ? cw[7] : R(0));
    for (int r = 0; r < 12; ++r) v[r] = r < 6 ? cw[6] * cw[r] : cw[7] * X[18 * (N - 1) + r];
    if (sg)
      for (int r = 0; r < 12; ++r) {
        V[r][r] = V[r][r] + sg[18 * (N - 1) + r];
        v[r] = v[r] + hs[18 * (N - 1) + r];
      }
    for (int k = N - 2; k >= 0; --k) {
      const R* L = &lin[114 * k];
      const R* w = &cost[10 * k];
      const R* x = X + 18 * k;
      const R *Aq = L, *Av = L + 36, *Bu = L + 72, *a = L + 108;
      R cv[6];
      for (int i = 0; i < 6; ++i) {
        R acc = R(0);
        for (int j = 0; j < 6; ++j) acc = acc + Aq[6 * i + j] * x[j] + Av[6 * i + j] * x[6 + j] + Bu[6 * i + j] * x[12 + j];
        cv[i] = (x[6 + i] + a[i] * dt) - acc;
      }
      R VA[12][12], Tm[6][6], s_[12];
      for (int r = 0; r < 12; ++r) {
        for (int c = 0; c < 6; ++c) {
          R a1 = V[r][c], a2 = dt * V[r][c];
          for (int m = 0; m < 6; ++m) {
            a1 = a1 + V[r][6 + m] * Aq[6 * m + c];
            a2 = a2 + V[r][6 + m] * Av[6 * m + c];
          }
          VA[r][c] = a1;
          VA[r][6 + c] = a2;
        }
        R acc = v[r];
        for (int m = 0; m < 6; ++m) acc = acc + V[r][6 + m] * cv[m];
        s_[r] = acc;
      }
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) {
          R acc = R(0);
          for (int m = 0; m < 6; ++m) acc = acc + V[6 + r][6 + m] * Bu[6 * m + c];
          Tm[r][c] = acc;
        }
      R AtVA[12][12], G[6][12], H[6][6], h[6], vA[12];
      for (int r = 0; r < 12; ++r)
        for (int c = r; c < 12; ++c) {
          R acc = r < 6 ? VA[r][c] : dt * VA[r - 6][c];
          for (int m = 0; m < 6; ++m) acc = acc + (r < 6 ? Aq[6 * m + r] : Av[6 * m + r - 6]) * VA[6 + m][c];
          AtVA[r][c] = AtVA[c][r] = acc;
        }
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 12; ++c) {
          R acc = R(0);
          for (int m = 0; m < 6; ++m) acc = acc + Bu[6 * m + r] * VA[6 + m][c];
          G[r][c] = acc;
        }
      const R* sgk = sg ? sg + 18 * k : nullptr;
      const R* hsk = sg ? hs + 18 * k : nullptr;
      for (int r = 0; r < 6; ++r)
        for (int c = r; c < 6; ++c) {
          R acc = r == c ? (sgk ? w[8] + sgk[12 + r] : w[8]) : R(0);
          for (int m = 0; m < 6; ++m) acc = acc + Bu[6 * m + r] * Tm[m][c];
          H[r][c] = H[c][r] = acc;
        }
      for (int r = 0; r < 6; ++r) {
        R acc = sgk ? w[8] * x[12 + r] + hsk[12 + r] : w[8] * x[12 + r];
        for (int m = 0; m < 6; ++m) acc = acc + Bu[6 * m + r] * s_[6 + m];
        h[r] = acc;
      }
      for (int r = 0; r < 12; ++r) {
        R acc = r < 6 ? w[6] * w[r] + s_[r] : w[7] * x[6 + r - 6] + dt * s_[r - 6];
        if (sgk) acc = acc + hsk[r];
        for (int m = 0; m < 6; ++m) acc = acc + (r < 6 ? Aq[6 * m + r] : Av[6 * m + r - 6]) * s_[6 + m];
        vA[r] = acc;
      }
      chol6(H);
      R* Kk = &K[84 * k];
      for (int c = 0; c < 13; ++c) {
        R rhs[6];
        for (int i = 0; i < 6; ++i) rhs[i] = c < 12 ? G[i][c] : h[i];
        chol6_solve(H, rhs);
        for (int i = 0; i < 6; ++i) Kk[c < 12 ? 12 * i + c : 72 + i] = R(0) - rhs[i];
      }
      for (int i = 0; i < 6; ++i) Kk[78 + i] = cv[i];
      for (int r = 0; r < 12; ++r)
        for (int c = r; c < 12; ++c) {
          R acc = AtVA[r][c];
          if (r < 6 && c < 6) acc = acc + w[6] * (w[r] * w[c]);
          else if (r == c) acc = acc + w[7];
          if (sgk && r == c) acc = acc + sgk[r];
          for (int m = 0; m < 6; ++m) acc = acc + G[m][r] * Kk[12 * m + c];
          V[r][c] = V[c][r] = acc;
        }
      for (int r = 0; r < 12; ++r) {
        R acc = vA[r];
        for (int m = 0; m < 6; ++m) acc = acc + G[m][r] * Kk[72 + m];
        v[r] = acc;
      }
    }
    R xk[12];
    for (int i = 0; i < 12; ++i) sol[i] = xk[i] = xs[i];
    for (int k = 0; k < N - 1; ++k) {
      const R* Kk = &K[84 * k];
      const R* L = &lin[114 * k];
      R u[6];
      for (int i = 0; i < 6; ++i) {
        R acc = Kk[72 + i];
        for (int j = 0; j < 12; ++j) acc = acc + Kk[12 * i + j] * xk[j];
        u[i] = acc;
        sol[18 * k + 12 + i] = acc;
      }
      R xn[12];
      for (int i = 0; i < 6; ++i) {
        xn[i] = xk[i] + dt * xk[6 + i];
        R acc = Kk[78 + i];
        for (int j = 0; j < 6; ++j) acc = acc + L[6 * i + j] * xk[j] + L[36 + 6 * i + j] * xk[6 + j] + L[72 + 6 * i + j] * u[j];
        xn[6 + i] = acc;
      }
      for (int i = 0; i < 12; ++i) sol[18 * (k + 1) + i] = xk[i] = xn[i];
    }
  }

  // ---- config 4: the box-constrained QP by Mehrotra predictor-corrector (oracle/box_ipm.py
  // ::ipm_box, step for step as i7m_box.h's ipm_init/pred/corr bodies), every Newton step the
  // Riccati solve above with the (Sigma, h) shifts; equality rows exact.  sol holds x_eq on
  // entry and the box-QP minimiser on exit.
  bool box_of(int e, double& lo, double& hi) const {
    const int k = e / 18, j = e - 18 * k;
    if (k == 0 && j < 12) return false;  // the fixed initial state
    if (j < 6) {
      if (!(P.box_mask & 1)) return false;
      lo = Md.qlo[j]; hi = Md.qhi[j];
    } else if (j < 12) {
      if (!(P.box_mask & 2)) return false;
      hi = Md.vlim[j - 6]; lo = -hi;
    } else {
      if (!(P.box_mask & 4)) return false;
      hi = Md.ulim[j - 12]; lo = -hi;
    }
    return true;
  }
  static R ratio_min(R t, R v, R dv) {
    if (!(dv < R(0))) return t;
    const R q = -v / dv;
    return q < t ? q : t;
  }

  void ipm(const R* X, const R* xs) {
    const double theta = P.box_theta, z0 = P.box_z0;
    // init (ipm_init_body): x = clip(x_eq) into the interior, centred duals z = z0 / s
    R acc = R(0);
    int nb = 0;
    for (int e = 0; e < T; ++e) {
      double lo, hi;
      R xv = sol[e], a = R(0), c = R(0), s = R(0);
      if (box_of(e, lo, hi)) {
        const double w = hi - lo;
        const double l1 = lo + theta * w, h1 = hi - theta * w;
        if (xv < R(l1)) xv = R(l1);
        if (R(h1) < xv) xv = R(h1);
        const R sl = xv - R(lo), su = R(hi) - xv, isl = R(1) / sl, isu = R(1) / su;
        a = R(z0) * isl;
        c = R(z0) * isu;
        acc = acc + (sl * a + su * c);
        s = a * isl + c * isu;
        ++nb;
      }
      bx[e] = xv; bzl[e] = a; bzu[e] = c; bsig[e] = s;
      bh[e] = -(s * xv);
    }
    R mu = nb ? acc / R(2.0 * nb) : R(0);
    double rfrac = 1.0;
    int it = 0;
    bool conv = nb == 0;
    while (!conv && it < P.box_max_iters) {
      // predictor Newton step (tau = 0): y = argmin with l = g - Sigma x
      riccati(X, xs, bsig.data(), bh.data());
      R ap = R(1), ad = R(1), s00 = R(0), s01 = R(0), s10 = R(0), s11 = R(0);
      for (int e = 0; e < T; ++e) {
        const R d = sol[e] - bx[e];
        bdxa[e] = d;
        double lo, hi;
        if (box_of(e, lo, hi)) {
          const R xx = bx[e], sl = xx - R(lo), su = R(hi) - xx, a = bzl[e], c = bzu[e];
          const R isl = R(1) / sl, isu = R(1) / su;
          const R dzl = (-a) - a * d * isl, dzu = (-c) + c * d * isu;
          ap = ratio_min(ratio_min(ap, sl, d), su, -d);
          ad = ratio_min(ratio_min(ad, a, dzl), c, dzu);
          s00 = s00 + (sl * a + su * c);
          s01 = s01 + (sl * dzl + su * dzu);
          s10 = s10 + (d * a - d * c);
          s11 = s11 + (d * dzl - d * dzu);
        }
      }
      // mu after the affine step, bilinear in (ap, ad); clamped at 0 (cancellation near the end)
      R mua = ((s00 + ad * s01) + ap * (s10 + ad * s11)) / R(2.0 * nb);
      if (mua < R(0)) mua = R(0);
      const R r = mua / mu;
      const R smu = r * r * r * mu;
      // the corrector's linear-term shift
      for (int e = 0; e < T; ++e) {
        double lo, hi;
        R hv = R(0);
        if (box_of(e, lo, hi)) {
          const R d = bdxa[e], xx = bx[e], sl = xx - R(lo), su = R(hi) - xx, a = bzl[e], c = bzu[e];
          const R isl = R(1) / sl, isu = R(1) / su;
          const R dzl = (-a) - a * d * isl, dzu = (-c) + c * d * isu;
          const R rl = sl * a + d * dzl - smu, ru = su * c - d * dzu - smu;
          const R s = a * isl + c * isu;
          hv = (-a) + c + (rl * isl - ru * isu) - s * xx;
        }
        bh[e] = hv;
      }
      // corrector Newton step
      riccati(X, xs, bsig.data(), bh.data());
      R t = R(1);
      for (int e = 0; e < T; ++e) {
        double lo, hi;
        if (!box_of(e, lo, hi)) continue;
        const R d = sol[e] - bx[e], da = bdxa[e];
        const R xx = bx[e], sl = xx - R(lo), su = R(hi) - xx, a = bzl[e], c = bzu[e];
        const R isl = R(1) / sl, isu = R(1) / su;
        const R dzla = (-a) - a * da * isl, dzua = (-c) + c * da * isu;
        const R rl = sl * a + da * dzla - smu, ru = su * c - da * dzua - smu;
        const R dzl = ((-rl) - a * d) * isl, dzu = ((-ru) + c * d) * isu;
        t = ratio_min(ratio_min(t, sl, d), su, -d);
        t = ratio_min(ratio_min(t, a, dzl), c, dzu);
      }
      const R al = (R(P.box_eta) * t < R(1)) ? R(P.box_eta) * t : R(1);
      R acc2 = R(0);
      for (int e = 0; e < T; ++e) {
        const R d = sol[e] - bx[e], xx = bx[e];
        double lo, hi;
        if (box_of(e, lo, hi)) {
          const R da = bdxa[e], sl = xx - R(lo), su = R(hi) - xx, a = bzl[e], c = bzu[e];
          const R isl = R(1) / sl, isu = R(1) / su;
          const R dzla = (-a) - a * da * isl, dzua = (-c) + c * da * isu;
          const R rl = sl * a + da * dzla - smu, ru = su * c - da * dzua - smu;
          const R dzl = ((-rl) - a * d) * isl, dzu = ((-ru) + c * d) * isu;
          const R xn = xx + al * d, an = a + al * dzl, cn = c + al * dzu;
          bx[e] = xn; bzl[e] = an; bzu[e] = cn;
          const R sln = xn - R(lo), sun = R(hi) - xn;
          acc2 = acc2 + (sln * an + sun * cn);
          const R s = an * (R(1) / sln) + cn * (R(1) / sun);
          bsig[e] = s;
          bh[e] = -(s * xn);
        } else {
          bx[e] = xx + al * d;
          bsig[e] = R(0);
          bh[e] = R(0);
        }
      }
      mu = acc2 / R(2.0 * nb);
      rfrac *= 1.0 - val(al);
      ++it;
      conv = val(mu) < P.box_tol && rfrac < P.box_tol;
    }
    for (int e = 0; e < T; ++e) sol[e] = bx[e];
    ipm_iters = it;
    ipm_conv = conv ? 1 : 0;
    ipm_mu = val(mu);
  }

  // merit of Xn (initial-state term relative to X0)
  R merit(const R* Xn, const R* X0, const double* goal, const double* f6) {
    R qc = R(0), vc = R(0), uc = R(0), cv = R(0);
    const R dt = R(P.dt);
    for (int k = 0; k < P.N; ++k) {
      const R* x = Xn + 18 * k;
      R c[6], s[6], p[3];
      for (int i = 0; i < 6; ++i) sincos2(x[i], &s[i], &c[i]);
      fk_jac(Md, c, s, p, (R(*)[6]) nullptr);
      const double* g = goal + (size_t)k * P.goal_stride;
      R e0 = p[0] - R(g[0]), e1 = p[1] - R(g[1]), e2 = p[2] - R(g[2]);
      qc = qc + R(k == P.N - 1 ? P.QN : 1.0) * (e0 * e0 + e1 * e1 + e2 * e2);
      R vv = R(0);
      for (int i = 0; i < 6; ++i) vv = vv + x[6 + i] * x[6 + i];
      vc = vc + R(P.dQ) * vv;
      if (k < P.N - 1) {
        R uu = R(0);
        for (int i = 0; i < 6; ++i) uu = uu + x[12 + i] * x[12 + i];
        uc = uc + R(P.R) * uu;
        R L[6][6], a[6];
        double fl[6];
        const double* fk = f6;
        if (f6 && P.fext_world) {
          wrench_world_to_local(Md, c, s, f6, fl);
          fk = fl;
        }
        forward_dynamics(Md, c, s, x + 6, x + 12, fk, L, a);
        const R* xn = Xn + 18 * (k + 1);
        R eq = R(0), ev = R(0);
        for (int i = 0; i < 6; ++i) {
          R dq = (x[i] + x[6 + i] * dt) - xn[i];
          R dv = (x[6 + i] + a[i] * dt) - xn[6 + i];
          eq = eq + dq * dq;
          ev = ev + dv * dv;
        }
        cv = cv + (sqrt(eq) + sqrt(ev));
      }
    }
    R d0 = R(0);
    for (int i = 0; i < 12; ++i) d0 = d0 + (Xn[i] - X0[i]) * (Xn[i] - X0[i]);
    cv = cv + sqrt(d0);
    return qc + vc + uc + R(P.mu) * cv;
  }

  // ---- ADMM mode: OSQP's algorithm (oracle/osqp_admm.py, which reproduces the reference's
  // printed closed loop) in the block form the GPU's k_admm runs (indy7_mpc_amd/csrc/i7m_admm.h):
  // Ruiz scaling in place on the per-stage blocks, the x-update by a block Cholesky of the
  // reduced matrix M = P + sigma I + A' diag(rho) A (block tridiagonal: 18 x 18 diagonal blocks,
  // 12 x 18 couplings), kept as explicit inverses Linv_k of the diagonal factors and the coupling
  // blocks C_k, so that every solve is mat-vecs.  A's rows are the reference's (src/osqp_solver.py:
  // 54-68, 83-101): block 0 = -x_0, block k+1 = J_k z_k - x_{k+1} with J_k = [[I, dt I, 0],
  // [Aq, Av, Bu]]; l = u = [-xs; -(0, cv_k)].  The iterates live in the caller's state (scaled,
  // as OSQP keeps them between solves: the reference's solver object, src/osqp_solver.py:38-40).
  struct AdmmState {
    double *x, *z, *y, *qold, *rho;  // T, m, m, T, 1 (scaled x, z, y; the previous QP's q; rho)
  };
  AdmmParams A_;
  int admm_it = 0, admm_solved = 0;
  // per-stage scaled data (in place, as OSQP's scale_data multiplies its stored matrices)
  std::vector<double> aPq, aPd, aJ, aI, aqs, als, aD, aE;
  double rho_cur = 0.1;  // the rho the current factor was built with
  double ac = 1.0;

  static double limit_sc(double v) { return v < 1e-4 ? 1.0 : (v > 1e4 ? 1e4 : v); }

  void admm_alloc() {
    const int N = P.N, m = 12 * N;
    aPq.assign(36 * N, 0.0); aPd.assign(T, 0.0); aJ.assign(216 * (N - 1), 0.0); aI.assign(m, 0.0);
    aqs.assign(T, 0.0); als.assign(m, 0.0); aD.assign(T, 1.0); aE.assign(m, 1.0);
    aLinv.assign(324 * N, 0.0);
  }

  // unscaled data of the QP at X (after linearize): P blocks, J_k, the -I entries, l; then the
  // Ruiz passes with the previous QP's q (OSQP re-scales inside update(Ax), before update(q)).
  void admm_setup(const R* X, const R* xs, const double* qold) {
    const int N = P.N, m = 12 * N;
    for (int k = 0; k < N; ++k) {
      const R* w = &cost[10 * k];
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) aPq[36 * k + 6 * i + j] = val(w[6] * (w[i] * w[j]));
      for (int i = 0; i < 6; ++i) aPd[18 * k + i] = 0.0;  // the q diagonal lives in aPq
      for (int i = 6; i < 12; ++i) aPd[18 * k + i] = val(w[7]);
      if (k < N - 1)
        for (int i = 12; i < 18; ++i) aPd[18 * k + i] = val(w[8]);
    }
    for (int k = 0; k + 1 < N; ++k) {
      const R* L = &lin[114 * k];
      double* G = &aJ[216 * k];
      for (int i = 0; i < 12; ++i)
        for (int j = 0; j < 18; ++j) {
          double v;
          if (i < 6) v = (j == i) ? 1.0 : (j == 6 + i ? P.dt : 0.0);
          else if (j < 6) v = val(L[6 * (i - 6) + j]);
          else if (j < 12) v = val(L[36 + 6 * (i - 6) + j - 6]);
          else v = val(L[72 + 6 * (i - 6) + j - 12]);
          G[18 * i + j] = v;
        }
      // l of block k+1: -(x_next - J_k z_k) with the q rows' offset exactly 0
      const R* x = X + 18 * k;
      for (int i = 0; i < 6; ++i) {
        R acc = R(0);
        for (int j = 0; j < 6; ++j) acc = acc + L[6 * i + j] * x[j] + L[36 + 6 * i + j] * x[6 + j] + L[72 + 6 * i + j] * x[12 + j];
        const R cv = (x[6 + i] + L[108 + i] * R(P.dt)) - acc;
        als[12 * (k + 1) + i] = 0.0;
        als[12 * (k + 1) + 6 + i] = -val(cv);
      }
    }
    for (int i = 0; i < 12; ++i) als[i] = -val(xs[i]);
    for (int r = 0; r < m; ++r) aI[r] = -1.0;
    for (int e = 0; e < T; ++e) { aqs[e] = qold[e]; aD[e] = 1.0; }
    for (int r = 0; r < m; ++r) aE[r] = 1.0;
    ac = 1.0;
    std::vector<double> Dt(T), Et(m);
    for (int pass = 0; pass < A_.scaling; ++pass) {
      // column inf-norms of [P; A] and row inf-norms of A (OSQP compute_inf_norm_cols_KKT)
      for (int e = 0; e < T; ++e) Dt[e] = 0.0;
      for (int r = 0; r < m; ++r) Et[r] = 0.0;
      admm_colP(Dt.data());
      for (int r = 0; r < m; ++r) {
        const int col = 18 * (r / 12) + r % 12;
        const double a = std::fabs(aI[r]);
        Dt[col] = std::max(Dt[col], a);
        Et[r] = std::max(Et[r], a);
      }
      for (int k = 0; k + 1 < N; ++k)
        for (int i = 0; i < 12; ++i)
          for (int j = 0; j < 18; ++j) {
            const double a = std::fabs(aJ[216 * k + 18 * i + j]);
            Dt[18 * k + j] = std::max(Dt[18 * k + j], a);
            Et[12 * (k + 1) + i] = std::max(Et[12 * (k + 1) + i], a);
          }
      for (int e = 0; e < T; ++e) Dt[e] = 1.0 / std::sqrt(limit_sc(Dt[e]));
      for (int r = 0; r < m; ++r) Et[r] = 1.0 / std::sqrt(limit_sc(Et[r]));
      // P <- D P D, A <- E A D, q <- D q (row factor first, as mat_premult_diag then postmult)
      for (int k = 0; k < N; ++k) {
        for (int i = 0; i < 6; ++i)
          for (int j = i; j < 6; ++j) {
            const double v = aPq[36 * k + 6 * i + j] * Dt[18 * k + i] * Dt[18 * k + j];
            aPq[36 * k + 6 * i + j] = aPq[36 * k + 6 * j + i] = v;
          }
        const int hi = k < N - 1 ? 18 : 12;
        for (int i = 6; i < hi; ++i) aPd[18 * k + i] = aPd[18 * k + i] * Dt[18 * k + i] * Dt[18 * k + i];
      }
      for (int r = 0; r < m; ++r) aI[r] = aI[r] * Et[r] * Dt[18 * (r / 12) + r % 12];
      for (int k = 0; k + 1 < N; ++k)
        for (int i = 0; i < 12; ++i)
          for (int j = 0; j < 18; ++j) aJ[216 * k + 18 * i + j] = aJ[216 * k + 18 * i + j] * Et[12 * (k + 1) + i] * Dt[18 * k + j];
      for (int e = 0; e < T; ++e) { aqs[e] = Dt[e] * aqs[e]; aD[e] = aD[e] * Dt[e]; }
      for (int r = 0; r < m; ++r) aE[r] = aE[r] * Et[r];
      // cost normalisation
      for (int e = 0; e < T; ++e) Dt[e] = 0.0;
      admm_colP(Dt.data());
      double mean = 0.0;
      for (int e = 0; e < T; ++e) mean += Dt[e];
      mean /= T;
      double qn = 0.0;
      for (int e = 0; e < T; ++e) qn = std::max(qn, std::fabs(aqs[e]));
      qn = limit_sc(qn);
      double ct = 1.0 / limit_sc(std::max(mean, qn));
      for (int k = 0; k < N; ++k) {
        for (int i = 0; i < 36; ++i) aPq[36 * k + i] *= ct;
        const int hi = k < N - 1 ? 18 : 12;
        for (int i = 6; i < hi; ++i) aPd[18 * k + i] *= ct;
      }
      for (int e = 0; e < T; ++e) aqs[e] *= ct;
      ac *= ct;
    }
    for (int r = 0; r < m; ++r) als[r] = aE[r] * als[r];
  }
  // max(|P_s| column) into out (symmetric P: the q block's full columns, the v / u diagonals)
  void admm_colP(double* out) const {
    for (int k = 0; k < P.N; ++k) {
      for (int j = 0; j < 6; ++j) {
        double mx = out[18 * k + j];
        for (int i = 0; i < 6; ++i) mx = std::max(mx, std::fabs(aPq[36 * k + 6 * i + j]));
        out[18 * k + j] = mx;
      }
      const int hi = k < P.N - 1 ? 18 : 12;
      for (int i = 6; i < hi; ++i) out[18 * k + i] = std::max(out[18 * k + i], std::fabs(aPd[18 * k + i]));
    }
  }
  // the new QP's linear cost, scaled (update(q)): q = c D g, g of src/osqp_solver.py:125-134
  void admm_q(const R* X) {
    for (int k = 0; k < P.N; ++k) {
      const R* w = &cost[10 * k];
      for (int i = 0; i < 6; ++i) aqs[18 * k + i] = val(w[6] * w[i]);
      for (int i = 6; i < 12; ++i) aqs[18 * k + i] = val(w[7] * X[18 * k + i]);
      if (k < P.N - 1)
        for (int i = 12; i < 18; ++i) aqs[18 * k + i] = val(w[8] * X[18 * k + i]);
    }
  }

  // The x-update's matrix M = P_s + sigma I + A_s' rho A_s (every row an equality row here:
  // rho_vec = 1e3 rho, OSQP's RHO_EQ_OVER_RHO_INEQ) is block tridiagonal: an 18 x 18 block per knot
  // (x_k, u_k) and the coupling M_{k+1,k} = re diag(I_{k+1}) J_k (x_{k+1} <- z_k).  Its block
  // Cholesky keeps the inverted diagonal factors Linv_k (S_k = L_k L_k', S_k = M_kk - C_{k-1}
  // C_{k-1}', C_k = M_{k+1,k} Linv_k'); the solve never needs C, only Linv and J (the device's
  // stage record: Linv_k packed, J_k compact), as the block LDL' with S_k^-1 = Linv_k' Linv_k:
  //   forward   g_k = rhs_k - [re I_k (J_{k-1} h_{k-1}); 0],  h_k = Linv_k' (Linv_k g_k)
  //   backward  xt_k = h_k - Linv_k' (Linv_k (J_k' (re I_{k+1} xt_{k+1}[:12])))
  // every product an fma chain over its 18 (or 12) terms in ascending order, as the device's
  // sweeps (indy7_mpc_amd/csrc/i7m_admm.h, k_admm_iter).  (An explicit S_k^-1 instead of the
  // triangular pair reads the same bytes but lost 5 orders of accuracy on the ill-conditioned M of
  // a second SQP iteration, cond ~4e7: forward error 1e-5 vs 3e-10)
  std::vector<double> aLinv;  // (N, 18, 18) Linv_k, zeros above the diagonal and in the last knot's padding
  // block Cholesky of M = P_s + sigma I + A_s' rho A_s; every row is an equality row here
  // (rho_vec = 1e3 rho, OSQP's RHO_EQ_OVER_RHO_INEQ)
  void admm_factor(double rho) {
    const int N = P.N;
    const double re = 1e3 * rho;
    rho_cur = rho;
    double Cp[12][18];
    for (int k = 0; k < N; ++k) {
      const int nk = k < N - 1 ? 18 : 12;
      double S[18][18];
      for (int a = 0; a < 18; ++a)
        for (int b = 0; b < 18; ++b) S[a][b] = 0.0;
      for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) S[a][b] = aPq[36 * k + 6 * a + b];
      for (int a = 6; a < nk; ++a) S[a][a] = aPd[18 * k + a];
      for (int a = 0; a < nk; ++a) S[a][a] += A_.sigma;
      for (int a = 0; a < 12; ++a) S[a][a] += re * (aI[12 * k + a] * aI[12 * k + a]);
      if (k < N - 1) {
        const double* G = &aJ[216 * k];
        for (int a = 0; a < 18; ++a)
          for (int b = 0; b < 18; ++b) {
            double acc = 0.0;
            for (int i = 0; i < 12; ++i) acc += G[18 * i + a] * G[18 * i + b];
            S[a][b] += re * acc;
          }
      }
      if (k > 0)
        for (int a = 0; a < 12; ++a)
          for (int b = 0; b < 12; ++b) {
            double acc = 0.0;
            for (int j = 0; j < 18; ++j) acc += Cp[a][j] * Cp[b][j];
            S[a][b] -= acc;
          }
      // right-looking Cholesky (the GPU's lane-parallel order); the pivots' reciprocals kept for
      // the inverse (the device's: a product by 1 / L_ii, not a quotient)
      double idv[18];
      for (int p = 0; p < nk; ++p) {
        const double d = std::sqrt(S[p][p]);
        S[p][p] = d;
        const double id = 1.0 / d;
        idv[p] = id;
        for (int i = p + 1; i < nk; ++i) S[i][p] = S[i][p] * id;
        for (int i = p + 1; i < nk; ++i)
          for (int j = p + 1; j <= i; ++j) S[i][j] = S[i][j] - S[i][p] * S[j][p];
      }
      double* Li = &aLinv[324 * k];
      for (int i = 0; i < 324; ++i) Li[i] = 0.0;
      for (int j = 0; j < nk; ++j) {
        Li[18 * j + j] = idv[j];
        for (int i = j + 1; i < nk; ++i) {
          double acc = 0.0;
          for (int l = j; l < i; ++l) acc += S[i][l] * Li[18 * l + j];
          Li[18 * i + j] = -acc * idv[i];
        }
      }
      if (k < N - 1) {
        // C_k = M_{x_{k+1}, z_k} Linv_k', M_{x_{k+1}, z_k} = re diag(aI_{k+1}) G_k
        const double* G = &aJ[216 * k];
        for (int a = 0; a < 12; ++a)
          for (int j = 0; j < 18; ++j) {
            double acc = 0.0;
            for (int l = 0; l <= j; ++l) acc += G[18 * a + l] * Li[18 * j + l];
            Cp[a][j] = re * aI[12 * (k + 1) + a] * acc;
          }
      }
    }
  }
  // compact J_k entry (i, j) (the dense 12 x 18 block; the device reads it from its record)
  double Jkc(int k, int i, int j) const { return aJ[216 * k + 18 * i + j]; }
  // The device's dot products (indy7_mpc_amd/csrc/i7m_admm.h a4_dot16 / a4_dot6, here adm_dot16 / adm_dot6): 16 terms as four
  // interleaved fma chains (l mod 4) combined (a0 + a1) + (a2 + a3); 6 terms as two (r even, odd)
  static double adm_dot16(const double* cf, const double* v) {
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int l = 0; l < 16; ++l) a[l % 4] = std::fma(cf[l], v[l], a[l % 4]);
    return (a[0] + a[1]) + (a[2] + a[3]);
  }
  static double adm_dot6(const double* cf, const double* v) {
    double a0 = 0.0, a1 = 0.0;
    for (int r = 0; r < 6; r += 2) {
      a0 = std::fma(cf[r], v[r], a0);
      a1 = std::fma(cf[r + 1], v[r + 1], a1);
    }
    return a0 + a1;
  }
  // sum_{c < 16} cf[c] v[c] as the device's a4_rowsum: t[c] = fma(cf[c], v[c], cf[c-1] v[c-1]),
  // then t[c] += t[c - d] for d = 2, 4, 8 (a pairwise tree), the result t[15]
  static double adm_rowsum(const double* cf, const double* v) {
    double p[16], t[16];
    for (int c = 0; c < 16; ++c) p[c] = cf[c] * v[c];
    for (int c = 1; c < 16; ++c) t[c] = std::fma(cf[c], v[c], p[c - 1]);
    t[0] = p[0];
    for (int d = 2; d < 16; d *= 2)
      for (int c = 15; c >= d; --c) t[c] = t[c] + t[c - d];
    return t[15];
  }
  // Linv_k (lower) and Linv_k' (upper) times an 18-vector, in the device's order (rows / columns
  // 0..15 by adm_dot16, rows 16, 17 by adm_rowsum, then the u-part's terms; the zeros above the
  // diagonal add nothing)
  void lmul(int k, const double* v, double* o) const {
    const double* Li = &aLinv[324 * k];
    for (int c = 0; c < 16; ++c) o[c] = adm_dot16(Li + 18 * c, v);
    o[16] = std::fma(Li[18 * 16 + 16], v[16], adm_rowsum(Li + 18 * 16, v));
    o[17] = std::fma(Li[18 * 17 + 17], v[17], std::fma(Li[18 * 17 + 16], v[16], adm_rowsum(Li + 18 * 17, v)));
  }
  void ltmul(int k, const double* v, double* o) const {
    const double* Li = &aLinv[324 * k];
    for (int c = 0; c < 16; ++c) {
      double col[16];
      for (int l = 0; l < 16; ++l) col[l] = Li[18 * l + c];
      o[c] = std::fma(Li[18 * 17 + c], v[17], std::fma(Li[18 * 16 + c], v[16], adm_dot16(col, v)));
    }
    o[16] = std::fma(Li[18 * 17 + 16], v[17], Li[18 * 16 + 16] * v[16]);
    o[17] = Li[18 * 17 + 17] * v[17];
  }
  // (J_k v)_i, i < 12, in the device's order (the q rows' two entries; the v rows by adm_dot16 + u-part)
  double Jrow_dot(int k, int i, const double* v) const {
    if (i < 6) return std::fma(Jkc(k, i, 6 + i), v[6 + i], Jkc(k, i, i) * v[i]);
    const double* Jr = &aJ[216 * k + 18 * i];
    return std::fma(Jr[17], v[17], std::fma(Jr[16], v[16], adm_dot16(Jr, v)));
  }
  // (J_k' u)_j, j < 18, from init: the q row's entry (column j < 12, zero beyond) with u[j % 6], plus
  // rows 6..11 (adm_dot6)
  double Jcol_dot(int k, int j, const double* u, double init) const {
    const double base = j < 12 ? std::fma(Jkc(k, j % 6, j), u[j % 6], init) : init;
    double cf[6];
    for (int r = 0; r < 6; ++r) cf[r] = Jkc(k, 6 + r, j);
    return base + adm_dot6(cf, u + 6);
  }
  // M x = b by the block LDL' above (the device's k_admm_iter solve, without the OSQP steps)
  void admm_solve(const double* b, double* x) const {
    const int N = P.N;
    const double re = 1e3 * rho_cur;
    double h[64][18];
    for (int k = 0; k < N; ++k) {
      const int nk = k < N - 1 ? 18 : 12;
      double g[18], w[18];
      for (int j = 0; j < 18; ++j) g[j] = j < nk ? b[18 * k + j] : 0.0;
      if (k > 0)
        for (int i = 0; i < 12; ++i) g[i] = g[i] - (re * aI[12 * k + i]) * Jrow_dot(k - 1, i, h[k - 1]);
      lmul(k, g, w);
      ltmul(k, w, h[k]);
    }
    double xt[18] = {0.0};
    for (int k = N - 1; k >= 0; --k) {
      const int nk = k < N - 1 ? 18 : 12;
      double cur[18];
      if (k == N - 1) {
        for (int c = 0; c < 18; ++c) cur[c] = h[k][c];
      } else {
        double u[12], t[18], s1[18], s2[18];
        for (int i = 0; i < 12; ++i) u[i] = (re * aI[12 * (k + 1) + i]) * xt[i];
        for (int j = 0; j < 18; ++j) t[j] = Jcol_dot(k, j, u, 0.0);
        lmul(k, t, s1);
        ltmul(k, s1, s2);
        for (int c = 0; c < 18; ++c) cur[c] = h[k][c] - s2[c];
      }
      for (int c = 0; c < nk; ++c) x[18 * k + c] = cur[c];
      for (int c = 0; c < 18; ++c) xt[c] = cur[c];
    }
  }
  void admm_Ax(const double* x, double* o) const {
    for (int i = 0; i < 12; ++i) o[i] = aI[i] * x[i];
    for (int k = 0; k + 1 < P.N; ++k)
      for (int i = 0; i < 12; ++i) o[12 * (k + 1) + i] = Jrow_dot(k, i, x + 18 * k) + aI[12 * (k + 1) + i] * x[18 * (k + 1) + i];
  }
  void admm_Aty(const double* t, double* o) const {
    for (int k = 0; k < P.N; ++k) {
      const int nk = k < P.N - 1 ? 18 : 12;
      for (int j = 0; j < nk; ++j) {
        const double init = j < 12 ? aI[12 * k + j] * t[12 * k + j] : 0.0;
        o[18 * k + j] = k < P.N - 1 ? Jcol_dot(k, j, t + 12 * (k + 1), init) : init;
      }
    }
  }
  void admm_Px(const double* x, double* o) const {
    for (int k = 0; k < P.N; ++k) {
      const int nk = k < P.N - 1 ? 18 : 12;
      for (int i = 0; i < 6; ++i) {
        double acc = 0.0;
        for (int j = 0; j < 6; ++j) acc += aPq[36 * k + 6 * i + j] * x[18 * k + j];
        o[18 * k + i] = acc;
      }
      for (int i = 6; i < nk; ++i) o[18 * k + i] = aPd[18 * k + i] * x[18 * k + i];
    }
  }

  // one QP: setup (scaling with the previous q), the new q, factor, OSQP's iteration from the
  // state's warm start; sol = D x
  void admm(const R* X, const R* xs, AdmmState& st) {
    const int N = P.N, m = 12 * N;
    admm_setup(X, xs, st.qold);
    admm_q(X);
    for (int e = 0; e < T; ++e) { st.qold[e] = aqs[e]; aqs[e] = ac * (aD[e] * aqs[e]); }
    double rho = *st.rho;
    admm_factor(rho);
    double rv = 1e3 * rho, ri = 1.0 / rv;
    std::vector<double> xt(T), zt(m), rhs(T), t(m), Ax(m), Px(T), Aty(T), xp(T);
    double* x = st.x;
    double* z = st.z;
    double* y = st.y;
    const double al = A_.alpha, sg = A_.sigma;
    int it = 0;
    bool checked = false;
    admm_solved = 0;
    for (it = 1; it <= A_.max_iter; ++it) {
      for (int r = 0; r < m; ++r) t[r] = z[r] - ri * y[r];
      for (int r = 0; r < m; ++r) t[r] = rv * t[r];
      admm_Aty(t.data(), rhs.data());
      for (int e = 0; e < T; ++e) rhs[e] = (sg * x[e] - aqs[e]) + rhs[e];
      admm_solve(rhs.data(), xt.data());
      admm_Ax(xt.data(), zt.data());
      for (int e = 0; e < T; ++e) x[e] = al * xt[e] + (1.0 - al) * x[e];
      for (int r = 0; r < m; ++r) {
        const double zr = al * zt[r] + (1.0 - al) * z[r];
        double zn = zr + ri * y[r];
        zn = std::min(std::max(zn, als[r]), als[r]);
        y[r] = y[r] + rv * (zr - zn);
        z[r] = zn;
      }
      checked = A_.check && it % A_.check == 0;
      bool adapt = A_.adapt_interval && it % A_.adapt_interval == 0;
      if (checked || adapt) {
        admm_Ax(x, Ax.data());
        admm_Px(x, Px.data());
        admm_Aty(y, Aty.data());
      }
      if (checked && admm_converged(x, z, y, Ax.data(), Px.data(), Aty.data())) {
        admm_solved = 1;
        break;
      }
      if (adapt) {
        double pri = 0.0, pn = 0.0, dua = 0.0, dn = 0.0;
        for (int r = 0; r < m; ++r) {
          pri = std::max(pri, std::fabs(Ax[r] - z[r]));
          pn = std::max(pn, std::max(std::fabs(z[r]), std::fabs(Ax[r])));
        }
        for (int e = 0; e < T; ++e) {
          dua = std::max(dua, std::fabs(aqs[e] + Px[e] + Aty[e]));
          dn = std::max(dn, std::max(std::fabs(aqs[e]), std::max(std::fabs(Aty[e]), std::fabs(Px[e]))));
        }
        pri = pri / (pn + 1e-30);
        dua = dua / (dn + 1e-30);
        double rn = rho * std::sqrt(pri / (dua + 1e-30));
        rn = std::min(std::max(rn, 1e-6), 1e6);
        if (rn > rho * A_.adapt_tol || rn < rho / A_.adapt_tol) {
          rho = rn;
          rv = 1e3 * rho;
          ri = 1.0 / rv;
          admm_factor(rho);
        }
      }
    }
    admm_it = it > A_.max_iter ? A_.max_iter : it;
    if (!admm_solved) {
      // OSQP after max_iter (oracle/osqp_admm.py OSQP.solve :344-349): the test at the final
      // iterate unless the last iteration ran it, then the approximate one (eps x 10) -> 2
      admm_Ax(x, Ax.data());
      admm_Px(x, Px.data());
      admm_Aty(y, Aty.data());
      if (!checked && admm_converged(x, z, y, Ax.data(), Px.data(), Aty.data()))
        admm_solved = 1;
      else if (admm_converged(x, z, y, Ax.data(), Px.data(), Aty.data(), 10.0))
        admm_solved = 2;
    }
    *st.rho = rho;
    for (int e = 0; e < T; ++e) sol[e] = R(aD[e] * x[e]);
  }
  // OSQP's check_termination on the unscaled residuals, with OSQP 1.x's duality-gap test
  bool admm_converged(const double* x, const double* z, const double* y, const double* Ax, const double* Px,
                      const double* Aty, double es = 1.0) const {
    const double ea = es * A_.eps_abs, er = es * A_.eps_rel;
    const int m = 12 * P.N;
    const double cinv = 1.0 / ac;
    double pr = 0.0, zn = 0.0, an = 0.0;
    for (int r = 0; r < m; ++r) {
      const double ei = 1.0 / aE[r];
      pr = std::max(pr, std::fabs(ei * (Ax[r] - z[r])));
      zn = std::max(zn, std::fabs(ei * z[r]));
      an = std::max(an, std::fabs(ei * Ax[r]));
    }
    double dr = 0.0, qn = 0.0, atn = 0.0, pxn = 0.0, xPx = 0.0, qx = 0.0;
    for (int e = 0; e < T; ++e) {
      const double di = 1.0 / aD[e];
      dr = std::max(dr, std::fabs(di * ((aqs[e] + Px[e]) + Aty[e])));
      qn = std::max(qn, std::fabs(di * aqs[e]));
      atn = std::max(atn, std::fabs(di * Aty[e]));
      pxn = std::max(pxn, std::fabs(di * Px[e]));
      xPx += x[e] * Px[e];
      qx += aqs[e] * x[e];
    }
    dr *= cinv;
    if (!(pr < ea + er * std::max(zn, an))) return false;
    if (!(dr < ea + er * cinv * std::max(qn, std::max(atn, pxn)))) return false;
    if (A_.gap) {
      double sc = 0.0;
      for (int r = 0; r < m; ++r) sc += als[r] * std::max(y[r], 0.0) + als[r] * std::min(y[r], 0.0);
      xPx *= cinv; qx *= cinv; sc *= cinv;
      const double gap = xPx + qx + sc;
      if (!(std::fabs(gap) < ea + er * std::max(std::fabs(xPx), std::max(std::fabs(qx), std::fabs(sc)))))
        return false;
    }
    return true;
  }

  // returns qp_iters; alphas/steps filled
  // box mode: ipm_it[qp] = the interior point's iterations of SQP iteration qp (may be null)
  // ADMM mode (st non-null): admm_it[qp] = OSQP iterations of SQP iteration qp
  int sqp(R* X, const R* xs, const double* goal, const double* f6, double* alphas, double* steps, int* n_alpha,
          int* n_step, int* ipm_it = nullptr, AdmmState* st = nullptr, int* admm_its = nullptr,
          int* admm_st = nullptr) {
    static const double AL[8] = {1.0, 0.5, 0.25, 0.125, 0.0625, 0.03125, 0.015625, 0.0078125};
    std::vector<R> Xn(T);
    *n_alpha = *n_step = 0;
    int qp = 0;
    for (qp = 0; qp < P.max_iters; ++qp) {
      linearize(X, goal, f6);
      if (st) {
        admm(X, xs, *st);
        if (admm_its) admm_its[qp] = admm_it;
        if (admm_st) admm_st[qp] = admm_solved;
      } else {
        riccati(X, xs);
      }
      if (P.box_mask) {
        ipm(X, xs);
        if (ipm_it) ipm_it[qp] = ipm_iters;
      }
      R base = merit(X, X, goal, f6);
      double alpha = 0.0;
      for (int ai = 0; ai < 8; ++ai) {
        for (int e = 0; e < T; ++e) Xn[e] = X[e] + R(AL[ai]) * (sol[e] - X[e]);
        if (merit(Xn.data(), X, goal, f6) <= base) {
          alpha = AL[ai];
          break;
        }
      }
      alphas[(*n_alpha)++] = alpha;
      if (alpha == 0.0) continue;
      R ss = R(0);
      for (int e = 0; e < T; ++e) {
        R stp = R(alpha) * (sol[e] - X[e]);
        X[e] = X[e] + stp;
        ss = ss + stp * stp;
      }
      const double stepsize = val(sqrt(ss));
      steps[(*n_step)++] = stepsize;
      if (stepsize < P.step_tol) break;
    }
    return qp < P.max_iters ? qp + 1 : P.max_iters;
  }
};

Params make_params(int N, const double* cfg, int goal_stride) {
  // cfg: dt, dQ, R, QN, eps, mu, step_tol, regularize, max_iters, fext_world
  Params P;
  P.N = N;
  P.dt = cfg[0]; P.dQ = cfg[1]; P.R = cfg[2]; P.QN = cfg[3]; P.eps = cfg[4]; P.mu = cfg[5]; P.step_tol = cfg[6];
  P.regularize = (int)cfg[7];
  P.max_iters = (int)cfg[8];
  P.fext_world = (int)cfg[9];
  P.goal_stride = goal_stride;
  P.box_mask = 0;
  P.box_max_iters = 30;
  P.box_tol = 1e-8; P.box_theta = 0.2; P.box_eta = 0.99; P.box_z0 = 0.1;
  return P;
}
// box_cfg: mask, max_iters, tol, theta, eta, z0 (BoxParams of i7m_box.h, oracle/box_ipm.py defaults)
void set_box(Params& P, const double* box_cfg) {
  if (!box_cfg) return;
  P.box_mask = (int)box_cfg[0];
  P.box_max_iters = (int)box_cfg[1];
  P.box_tol = box_cfg[2]; P.box_theta = box_cfg[3]; P.box_eta = box_cfg[4]; P.box_z0 = box_cfg[5];
}

}  // namespace

extern "C" {

// Full SQP for B problems (OpenMP over problems when nthreads > 1).  box_cfg non-null with a
// nonzero mask: config 4's box rows (ipm_iters (B, 8) per SQP iteration, and the last QP's
// converged flag and final mu, as i7m_get_box_stats reports them; any may be null).
int i7m_cpu_solve_box(const double* model_packed, int N, const double* cfg, const double* box_cfg, int B,
                      const double* xu_in, const double* xcur, const double* goals, int goal_stride, const double* fext,
                      double* xu_out, int* qp_iters, double* alphas, double* steps, int* ipm_iters, int* ipm_conv,
                      double* ipm_mu, int nthreads) {
  if (N < 2 || N > 64 || B < 0) return -1;
  const Model M = make_model(model_packed);
  Params P = make_params(N, cfg, goal_stride);
  set_box(P, box_cfg);
  const int T = 18 * N - 6;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int b = 0; b < B; ++b) {
    Solver<double> S(M, P);
    double* X = xu_out + (size_t)b * T;
    std::memcpy(X, xu_in + (size_t)b * T, sizeof(double) * T);
    int na, ns;
    qp_iters[b] = S.sqp(X, xcur + 12 * (size_t)b, goals + (size_t)b * N * goal_stride, fext ? fext + 6 * (size_t)b : nullptr,
                        alphas + 8 * (size_t)b, steps + 8 * (size_t)b, &na, &ns,
                        ipm_iters ? ipm_iters + 8 * (size_t)b : nullptr);
    if (ipm_conv) ipm_conv[b] = S.ipm_conv;
    if (ipm_mu) ipm_mu[b] = S.ipm_mu;
  }
  return 0;
}

// ADMM mode (OSQP's algorithm, oracle/osqp_admm.py): admm_cfg = rho0, sigma, alpha, eps_abs,
// eps_rel, max_iter, check_termination, scaling, check_dualgap, adaptive_rho_interval,
// adaptive_rho_tolerance.  The solver state of every problem (scaled x (B, T), z (B, 12N),
// y (B, 12N), the previous QP's q (B, T), rho (B)) is read and written back: it is the
// reference's OSQP object, warm-started from call to call (src/osqp_solver.py:38-40).
// admm_iters (B, 8): OSQP iterations per SQP iteration; admm_status (B, 8): 1 solved, 2 solved
// inaccurate, 0 max_iter reached (as i7m_get_admm_status); either may be null.
int i7m_cpu_solve_admm(const double* model_packed, int N, const double* cfg, const double* admm_cfg, int B,
                       const double* xu_in, const double* xcur, const double* goals, int goal_stride,
                       const double* fext, double* xu_out, int* qp_iters, double* alphas, double* steps,
                       double* st_x, double* st_z, double* st_y, double* st_q, double* st_rho, int* admm_iters,
                       int* admm_status, int nthreads) {
  if (N < 2 || N > 64 || B < 0 || !admm_cfg) return -1;
  const Model M = make_model(model_packed);
  Params P = make_params(N, cfg, goal_stride);
  AdmmParams A;
  A.rho0 = admm_cfg[0]; A.sigma = admm_cfg[1]; A.alpha = admm_cfg[2]; A.eps_abs = admm_cfg[3]; A.eps_rel = admm_cfg[4];
  A.max_iter = (int)admm_cfg[5]; A.check = (int)admm_cfg[6]; A.scaling = (int)admm_cfg[7]; A.gap = (int)admm_cfg[8];
  A.adapt_interval = (int)admm_cfg[9]; A.adapt_tol = admm_cfg[10];
  const int T = 18 * N - 6, m = 12 * N;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int b = 0; b < B; ++b) {
    Solver<double> S(M, P);
    S.A_ = A;
    S.admm_alloc();
    Solver<double>::AdmmState st{st_x + (size_t)b * T, st_z + (size_t)b * m, st_y + (size_t)b * m, st_q + (size_t)b * T,
                                 st_rho + b};
    double* X = xu_out + (size_t)b * T;
    std::memcpy(X, xu_in + (size_t)b * T, sizeof(double) * T);
    int na, ns;
    qp_iters[b] = S.sqp(X, xcur + 12 * (size_t)b, goals + (size_t)b * N * goal_stride, fext ? fext + 6 * (size_t)b : nullptr,
                        alphas + 8 * (size_t)b, steps + 8 * (size_t)b, &na, &ns, nullptr, &st,
                        admm_iters ? admm_iters + 8 * (size_t)b : nullptr,
                        admm_status ? admm_status + 8 * (size_t)b : nullptr);
  }
  return 0;
}

int i7m_cpu_solve(const double* model_packed, int N, const double* cfg, int B, const double* xu_in,
                  const double* xcur, const double* goals, int goal_stride, const double* fext, double* xu_out,
                  int* qp_iters, double* alphas, double* steps, int nthreads) {
  return i7m_cpu_solve_box(model_packed, N, cfg, nullptr, B, xu_in, xcur, goals, goal_stride, fext, xu_out, qp_iters,
                           alphas, steps, nullptr, nullptr, nullptr, nthreads);
}

// Instrumented flop count of one SQP solve, split by stage:
// out[0] linearise, out[1] QP (Riccati; box mode: + the interior point), out[2] line search (all
// merit evals actually run), out[3] step/update; out[4] number of SQP iterations; out[5] merit
// evaluations; box mode (box_cfg): out[6] the interior point's flops (inside out[1]), out[7] its
// iterations over the solve.
int i7m_cpu_count_flops_box(const double* model_packed, int N, const double* cfg, const double* box_cfg,
                            const double* xu_in, const double* xcur, const double* goal, int goal_stride, double* out) {
  const Model M = make_model(model_packed);
  Params P = make_params(N, cfg, goal_stride);
  set_box(P, box_cfg);
  const int T = 18 * N - 6;
  Solver<CountD> S(M, P);
  std::vector<CountD> X(xu_in, xu_in + T), xs(xcur, xcur + 12), Xn(T);
  static const double AL[8] = {1.0, 0.5, 0.25, 0.125, 0.0625, 0.03125, 0.015625, 0.0078125};
  uint64_t f_lin = 0, f_qp = 0, f_ls = 0, f_step = 0, f_ipm = 0;
  int iters = 0, merits = 0, ipm_total = 0;
  for (int qp = 0; qp < P.max_iters; ++qp) {
    ++iters;
    CountD::flops = 0;
    S.linearize(X.data(), goal, nullptr);
    f_lin += CountD::flops;
    CountD::flops = 0;
    S.riccati(X.data(), xs.data());
    if (P.box_mask) {
      const uint64_t f0 = CountD::flops;
      S.ipm(X.data(), xs.data());
      f_ipm += CountD::flops - f0;
      ipm_total += S.ipm_iters;
    }
    f_qp += CountD::flops;
    CountD::flops = 0;
    CountD base = S.merit(X.data(), X.data(), goal, nullptr);
    ++merits;
    double alpha = 0.0;
    for (int ai = 0; ai < 8; ++ai) {
      for (int e = 0; e < T; ++e) Xn[e] = X[e] + CountD(AL[ai]) * (S.sol[e] - X[e]);
      ++merits;
      if (S.merit(Xn.data(), X.data(), goal, nullptr) <= base) {
        alpha = AL[ai];
        break;
      }
    }
    f_ls += CountD::flops;
    if (alpha == 0.0) continue;
    CountD::flops = 0;
    CountD ss(0.0);
    for (int e = 0; e < T; ++e) {
      CountD stp = CountD(alpha) * (S.sol[e] - X[e]);
      X[e] = X[e] + stp;
      ss = ss + stp * stp;
    }
    double stepsize = std::sqrt(ss.v);
    f_step += CountD::flops;
    if (stepsize < P.step_tol) break;
  }
  out[0] = (double)f_lin;
  out[1] = (double)f_qp;
  out[2] = (double)f_ls;
  out[3] = (double)f_step;
  out[4] = iters;
  out[5] = merits;
  if (box_cfg) {
    out[6] = (double)f_ipm;
    out[7] = ipm_total;
  }
  return 0;
}

int i7m_cpu_count_flops(const double* model_packed, int N, const double* cfg, const double* xu_in, const double* xcur,
                        const double* goal, int goal_stride, double* out) {
  return i7m_cpu_count_flops_box(model_packed, N, cfg, nullptr, xu_in, xcur, goal, goal_stride, out);
}

}  // extern "C"
