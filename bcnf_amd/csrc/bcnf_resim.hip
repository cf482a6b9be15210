// Batched re-simulation of ballistic trajectories from posterior draws (psaegert/bcnf
// src/bcnf/simulation/resimulation.py:21-59, which runs physics.py:53-160 once per (draw j, trajectory i) in a
// ProcessPoolExecutor over scipy's LSODA `odeint`).
//
// One thread per (i, j), fp64 throughout:
//   * parameters (physics.py:53-72 order: x0 3, v0 3, g 3, w 3, b, m, rho, r, a 3): column col[q] of the draw
//     y_hat[j][i][:] (resimulation.py:16, ParameterIndexMapping.dictify) or, for a name the model does not predict,
//     the trajectory's fixed value fixed[i][q] (resimulation.py:53);
//   * velocity ODE dv/dt = g - g rho (4/3) pi r^3 / m - (0.5 b / m) (v^2 v / |v| - w^2 w / |w|) + a
//     (physics.py:42, ballistic_ODE, including its elementwise v^2 v / |v| drag and the 0/0 = NaN of a zero wind),
//     integrated between consecutive grid times t[s-1] -> t[s] (t = arange(0, T, dt), physics.py:141) by an adaptive
//     Dormand-Prince 5(4) pair (FSAL, RMS error norm, tolerances far below odeint's default 1.49e-8, so the result is
//     the ODE solution odeint approximates, not a different discretisation);
//   * positions x[0] = x0, x[s] = x[s-1] + v[s] dt (physics.py:149-152); with break_on_impact the first x[s] with
//     z < 0 is replaced by the impact point x[s-1] + v[s] (-x[s-1].z / v[s].z) and repeated to the end
//     (physics.py:154-159).
// Output x[i][j][s][3] = np.array(X_resimulation_list) of resimulation.py:59 (trajectory-major).
// The integration is VALU fp64 work (no MFMA shape: 3-vectors); every thread's state lives in registers and the only
// memory traffic is the parameter gather and the position stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bcnf_amd.h"
#include "bcnf_device.h"

namespace {

constexpr int RWG = 64;        // one wave per workgroup: the chunk barrier costs nothing (533 -> 521 us against 128)

struct ResimArgs {
  int col[BCNF_RESIM_NPARAM];      // y_hat column of each physics parameter, -1 = fixed[i][q]
  const double* fixed;             // [N][19] (may be NULL when every col >= 0)
  const double* tgrid;             // [steps]
  long long M, N;                  // draws, trajectories
  int D, steps, break_on_impact, max_attempts;
  double dt, rtol, atol;
  double* x;                       // [N][M][steps][3]
  int32_t* attempts;               // [N][M] step attempts (accepted + rejected), optional
  int32_t* status;                 // [N][M] BCNF_RESIM_*, optional
};

struct Phys {
  double gb[3], a[3], wt[3], kd;
};

// ballistic_ODE (physics.py:42): (g - buoyancy) - kd (v^2 v / |v| - w^2 w / |w|) + a
__device__ __forceinline__ void rhs(const Phys& P, const double v[3], double d[3]) {
  const double inv = rsqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);     // 1 / |v| (no fp64 division)
#pragma unroll
  for (int c = 0; c < 3; ++c) d[c] = P.gb[c] - P.kd * (v[c] * v[c] * v[c] * inv - P.wt[c]) + P.a[c];
}

// Dormand-Prince 5(4) tableau
constexpr double A21 = 1.0 / 5;
constexpr double A31 = 3.0 / 40, A32 = 9.0 / 40;
constexpr double A41 = 44.0 / 45, A42 = -56.0 / 15, A43 = 32.0 / 9;
constexpr double A51 = 19372.0 / 6561, A52 = -25360.0 / 2187, A53 = 64448.0 / 6561, A54 = -212.0 / 729;
constexpr double A61 = 9017.0 / 3168, A62 = -355.0 / 33, A63 = 46732.0 / 5247, A64 = 49.0 / 176,
                 A65 = -5103.0 / 18656;
constexpr double B1 = 35.0 / 384, B3 = 500.0 / 1113, B4 = 125.0 / 192, B5 = -2187.0 / 6784, B6 = 11.0 / 84;
constexpr double E1 = 71.0 / 57600, E3 = -71.0 / 16695, E4 = 71.0 / 1920, E5 = -17253.0 / 339200, E6 = 22.0 / 525,
                 E7 = -1.0 / 40;

__device__ __forceinline__ bool finite3(const double v[3]) {
  return isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]);
}

// One Dormand-Prince attempt over [t, t + hh] from v (k1 = f(v), FSAL). Returns the squared RMS error norm and
// writes vn and k7 = f(vn).
__device__ __forceinline__ float dp_attempt(const Phys& P, const double v[3], const double k1[3], double hh,
                                            double rtol, double atol, double vn[3], double k7[3]) {
  double y[3], k2[3], k3[3], k4[3], k5[3], k6[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) y[c] = v[c] + hh * (A21 * k1[c]);
  rhs(P, y, k2);
#pragma unroll
  for (int c = 0; c < 3; ++c) y[c] = v[c] + hh * (A31 * k1[c] + A32 * k2[c]);
  rhs(P, y, k3);
#pragma unroll
  for (int c = 0; c < 3; ++c) y[c] = v[c] + hh * (A41 * k1[c] + A42 * k2[c] + A43 * k3[c]);
  rhs(P, y, k4);
#pragma unroll
  for (int c = 0; c < 3; ++c) y[c] = v[c] + hh * (A51 * k1[c] + A52 * k2[c] + A53 * k3[c] + A54 * k4[c]);
  rhs(P, y, k5);
#pragma unroll
  for (int c = 0; c < 3; ++c)
    y[c] = v[c] + hh * (A61 * k1[c] + A62 * k2[c] + A63 * k3[c] + A64 * k4[c] + A65 * k5[c]);
  rhs(P, y, k6);
#pragma unroll
  for (int c = 0; c < 3; ++c) vn[c] = v[c] + hh * (B1 * k1[c] + B3 * k3[c] + B4 * k4[c] + B5 * k5[c] + B6 * k6[c]);
  rhs(P, vn, k7);
  // squared RMS error norm in fp32: it only steers the step size (accept / shrink), so its rounding never reaches the
  // solution beyond the tolerance it enforces; no fp64 division, square root or pow
  float en2 = 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double e = hh * (E1 * k1[c] + E3 * k3[c] + E4 * k4[c] + E5 * k5[c] + E6 * k6[c] + E7 * k7[c]);
    const double sc = atol + rtol * fmax(fabs(v[c]), fabs(vn[c]));
    const float q = (float)e * __builtin_amdgcn_rcpf((float)sc);
    en2 += q * q;
  }
  return en2 * (1.f / 3.f);
}

// Positions go through LDS in chunks of RCH grid points: the workgroup's RWG trajectories are consecutive in x, so a
// chunk is RWG runs of 3 RCH contiguous doubles, copied out by consecutive threads (a thread's own stores would hit
// 64 different lines per wave instruction: 35% of the launch, measured by an experiment build without them).
constexpr int RCH = 6;          // 9.7 KB of LDS per 64-thread workgroup (4 waves / SIMD, as the 107 VGPRs allow; 4 and 3 with
                                // 5 waves / SIMD measured 2-15% slower, tools/ab_resim.sh)
constexpr int RLD = 3 * RCH + 1;       // LDS row (doubles) per trajectory, odd: rows start on different banks

template <typename TY>
__global__ __launch_bounds__(RWG) void k_resim(const ResimArgs a, const TY* __restrict__ yhat) {
  __shared__ double sx[RWG * RLD];
  const long long n = a.M * a.N;
  const long long o0 = (long long)blockIdx.x * RWG, o = o0 + threadIdx.x;
  const bool live = o < n;
  const long long oc = live ? o : n - 1;     // threads past the end compute a copy and store nothing
  const long long i = oc / a.M, j = oc - i * a.M;
  double p[BCNF_RESIM_NPARAM];
#pragma unroll
  for (int q = 0; q < BCNF_RESIM_NPARAM; ++q)
    p[q] = a.col[q] >= 0 ? (double)yhat[(j * a.N + i) * a.D + a.col[q]] : a.fixed[i * BCNF_RESIM_NPARAM + q];
  const double b = p[12], m = p[13], rho = p[14], r = p[15];
  Phys P;
  const double nw = sqrt(p[9] * p[9] + p[10] * p[10] + p[11] * p[11]);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double g = p[6 + c], w = p[9 + c];
    P.gb[c] = g - g * rho * (4.0 / 3.0) * (M_PI * (r * r * r)) / m;
    P.wt[c] = w * w * w / nw;
    P.a[c] = p[16 + c];
  }
  P.kd = 0.5 * b / m;
  double x[3] = {p[0], p[1], p[2]}, v[3] = {p[3], p[4], p[5]};
  double k1[3];
  rhs(P, v, k1);
  // st != OK or `frozen`: the trajectory is finished and x holds what every later grid point repeats (the impact
  // point, or NaN: a non-finite right-hand side, e.g. zero wind's 0/0 in physics.py:42, makes odeint's solution NaN
  // from t[1] on, and a failed step size leaves the rest NaN as well)
  int st = finite3(k1) ? BCNF_RESIM_OK : BCNF_RESIM_NONFINITE;
  bool frozen = false;
  int tries = 0;
  double h = a.steps > 1 ? (a.tgrid[1] - a.tgrid[0]) * 0.25 : 0.0;
  double* row = sx + threadIdx.x * RLD;
  for (int s0 = 0; s0 < a.steps; s0 += RCH) {             // uniform across the workgroup
    const int s1 = s0 + RCH < a.steps ? s0 + RCH : a.steps;
    for (int s = s0; s < s1; ++s) {
      if (s > 0 && st == BCNF_RESIM_OK && !frozen) {
        // integrate v over [t[s-1], t[s]]
        double t = a.tgrid[s - 1];
        const double tend = a.tgrid[s];
        bool reached = !(tend > t);
        while (!reached) {
          if (++tries > a.max_attempts) { st = BCNF_RESIM_STEPS; break; }
          bool last = false;
          double hh = h;
          if (hh >= tend - t) { hh = tend - t; last = true; }
          double vn[3], k7[3];
          const float en2 = dp_attempt(P, v, k1, hh, a.rtol, a.atol, vn, k7);
          const float fac0 = 0.9f * __builtin_amdgcn_exp2f(-0.1f * __builtin_amdgcn_logf(en2));   // 0.9 en^(-1/5)
          if (!(en2 <= 1.f) || !finite3(vn)) {     // reject (a NaN / inf error norm shrinks the step too)
            h = hh * (double)(en2 < INFINITY ? fmaxf(0.2f, fac0) : 0.2f);
            if (!(h > 1e-13 * (fabs(t) + fabs(tend)))) { st = BCNF_RESIM_STEPS; break; }
            continue;
          }
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            v[c] = vn[c];
            k1[c] = k7[c];
          }
          t = last ? tend : t + hh;
          reached = last;
          const double fac = en2 > 0.f ? (double)fminf(5.f, fmaxf(0.2f, fac0)) : 5.0;
          if (!last || fac < 1.0) h = hh * fac;     // a step clipped to the grid keeps the controller's h
        }
        if (st == BCNF_RESIM_OK) {
          double xn[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) xn[c] = x[c] + v[c] * a.dt;
          if (a.break_on_impact && xn[2] < 0.0) {   // physics.py:154-159
            const double ti = -x[2] / v[2];
#pragma unroll
            for (int c = 0; c < 3; ++c) xn[c] = x[c] + v[c] * ti;
            frozen = true;
          }
#pragma unroll
          for (int c = 0; c < 3; ++c) x[c] = xn[c];
        }
      }
      if (s > 0 && st != BCNF_RESIM_OK) x[0] = x[1] = x[2] = __builtin_nan("");
#pragma unroll
      for (int c = 0; c < 3; ++c) row[3 * (s - s0) + c] = x[c];
    }
    __syncthreads();
    const int w = 3 * (s1 - s0);
    for (int e = threadIdx.x; e < RWG * w; e += RWG) {
      const int tt = e / w, q = e - tt * w;
      if (o0 + tt < n) a.x[(o0 + tt) * a.steps * 3 + 3 * s0 + q] = sx[tt * RLD + q];
    }
    __syncthreads();
  }
  if (live && a.attempts) a.attempts[o] = tries;
  if (live && a.status) a.status[o] = st;
}

}  // namespace

extern "C" {

int bcnf_resimulate(const void* y_hat, int32_t y_hat_f64, int64_t n_draws, int64_t n_traj, int32_t dim,
                    const int32_t* param_cols, const double* fixed, const double* tgrid, int32_t steps, double dt,
                    int32_t break_on_impact, double rtol, double atol, int32_t max_attempts, double* x,
                    int32_t* attempts, int32_t* status, void* stream) {
  if (n_draws < 0 || n_traj < 0 || steps < 1 || dim < 0 || !param_cols || !(rtol > 0.0) || !(atol > 0.0) ||
      max_attempts < 1)
    return BCNF_ERR_ARG;
  if (n_draws == 0 || n_traj == 0) return BCNF_OK;
  if (!x || (steps > 1 && !tgrid)) return BCNF_ERR_ARG;
  ResimArgs a;
  bool need_fixed = false, need_y = false;
  for (int q = 0; q < BCNF_RESIM_NPARAM; ++q) {
    if (param_cols[q] >= dim) return BCNF_ERR_ARG;
    a.col[q] = param_cols[q] < 0 ? -1 : param_cols[q];
    need_fixed |= param_cols[q] < 0;
    need_y |= param_cols[q] >= 0;
  }
  if ((need_fixed && !fixed) || (need_y && !y_hat)) return BCNF_ERR_ARG;
  const long long n = n_draws * n_traj;
  const long long nwg = (n + RWG - 1) / RWG;
  if (nwg > 0x7fffffffLL) return BCNF_ERR_UNSUPPORTED;
  a.fixed = fixed;
  a.tgrid = tgrid;
  a.M = n_draws;
  a.N = n_traj;
  a.D = dim;
  a.steps = steps;
  a.break_on_impact = break_on_impact ? 1 : 0;
  a.max_attempts = max_attempts;
  a.dt = dt;
  a.rtol = rtol;
  a.atol = atol;
  a.x = x;
  a.attempts = attempts;
  a.status = status;
  if (y_hat_f64)
    hipLaunchKernelGGL(k_resim<double>, dim3((unsigned)nwg), dim3(RWG), 0, (hipStream_t)stream, a,
                       (const double*)y_hat);
  else
    hipLaunchKernelGGL(k_resim<float>, dim3((unsigned)nwg), dim3(RWG), 0, (hipStream_t)stream, a,
                       (const float*)y_hat);
  return bcnf_rt::launched();
}

}  // extern "C"
