// bcnf_amd: the training-step kernels around the coupling stack (gfx950 / CDNA4).
//
//   k_adam     multi-tensor Adam over the flat parameter buffers (torch.optim.Adam semantics,
//              trainer.py:136 / :270), fused with the per-workgroup sum of squared gradients that
//              clip_grad_norm_ needs (trainer.py:275) and with the device-side step counter bump
//   k_sumsq    per-workgroup sum of squared gradients (standalone clip)
//   k_clip     total norm from the partials (fixed order) + in-place gradient scaling
//   k_gemm     small fp32 MFMA GEMM C = A * op(B) (+ bias) for the feature network's nn.Linear
//              (feature_network.py:114-145): forward and dL/dx
//   k_gemm_wt  split-K dL/dW = dY^T X and dL/db = sum dY partials; k_wt_reduce sums them (fixed order)
//
// Every reduction has a fixed order, so results are bit-reproducible run to run.
#include "bcnf_device.h"
#include "../../include/bcnf_amd.h"

#include <math.h>

namespace {

constexpr int EPT = 4;                          // elements per thread in the elementwise kernels
constexpr int CHUNK = BCNF_WG * EPT;            // elements per workgroup

struct TList {
  float* p[BCNF_MAX_TENSORS];
  float* g[BCNF_MAX_TENSORS];
  float* m[BCNF_MAX_TENSORS];
  float* v[BCNF_MAX_TENSORS];
  long long start[BCNF_MAX_TENSORS + 1];        // prefix offsets of the concatenated index space
  int n;
};

__device__ __forceinline__ int find_tensor(const TList& T, long long i) {
  int t = 0;
#pragma unroll 1
  while (t + 1 < T.n && i >= T.start[t + 1]) ++t;
  return t;
}

// Fixed-order workgroup sum: every thread contributes `v`; thread 0 gets the total.
__device__ __forceinline__ float wg_sum(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int s = BCNF_WG / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  return red[0];
}

// torch.optim.Adam (amsgrad=False, maximize=False), per element (torch/optim/adam.py _single_tensor_adam):
//   g += wd * p;  m = lerp(m, g, 1-b1);  v = b2 v + (1-b2) g g;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// Hyper-parameters arrive as doubles (Python floats) and every scalar is derived in double, then
// rounded once, as torch does (1 - beta2 in fp32 from 0.999f would be off by 1e-5 relative).
// End-of-step bookkeeping carried by the Adam launch (bcnf_adam_step_bookkeep): done by its last workgroup.
struct AdamBook {
  float* step;                  // step count to advance (the kernel's own `step` operand)
  long long* cursor;            // epoch cursor (nullable) and its modulo
  long long n_batches;
  const float* log_values;      // logged values -> log_history[3 * cursor] (nullable)
  float* log_history;
  int* done;                    // workgroups finished; 0 between launches (the last one resets it); NULL: off
};

// G groups of EPT elements per thread (G = BIG_G = 2 for the wide family's ~49M parameters: half the workgroups, so
// half the per-workgroup reductions and launch ramps, and 2x the bytes in flight per thread; G = 1 for small sets,
// where more workgroups cover the chip). Group q of workgroup b starts at b * G * CHUNK + q * CHUNK.
template <int G>
__global__ __launch_bounds__(BCNF_WG) void k_adam(TList T, const float* __restrict__ step, double lr, double b1d,
                                                  double b2d, double epsd, double wdd, float* __restrict__ part,
                                                  const int32_t* __restrict__ guard, AdamBook bk) {
  __shared__ float red[BCNF_WG];
  __shared__ float sc[2];
  // every operand load is issued first: none depends on the guard, the step count or the bias corrections,
  // so their round trip overlaps the scalar loads and thread 0's double pow
  const long long total = T.start[T.n];
  // thread x owns the EPT = 4 consecutive elements i0..i0+3 of each group: one 16-B load / store per array when they
  // lie in one tensor at a 16-B aligned offset (the whole flat coupling buffer), element-wise at tensor seams
  float g[G][EPT], p[G][EPT], m[G][EPT], v[G][EPT];
  int t[G][EPT];
  long long o[G][EPT], i0[G];
  bool vec[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    i0[q] = (long long)blockIdx.x * G * CHUNK + q * CHUNK + EPT * threadIdx.x;
    const int t0 = find_tensor(T, i0[q] < total ? i0[q] : total - 1);
    const long long o0 = i0[q] - T.start[t0];
    vec[q] = i0[q] + EPT <= T.start[t0 + 1] &&
             ((((uintptr_t)(T.p[t0] + o0)) | ((uintptr_t)(T.g[t0] + o0)) | ((uintptr_t)(T.m[t0] + o0)) |
               ((uintptr_t)(T.v[t0] + o0))) & 15) == 0;
    if (vec[q]) {
      const floatx4 g4 = *reinterpret_cast<const floatx4*>(T.g[t0] + o0);
      const floatx4 p4 = *reinterpret_cast<const floatx4*>(T.p[t0] + o0);
      const floatx4 m4 = *reinterpret_cast<const floatx4*>(T.m[t0] + o0);
      const floatx4 v4 = *reinterpret_cast<const floatx4*>(T.v[t0] + o0);
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        g[q][e] = g4[e];
        p[q][e] = p4[e];
        m[q][e] = m4[e];
        v[q][e] = v4[e];
        t[q][e] = t0;
        o[q][e] = o0 + e;
      }
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        long long i = i0[q] + e;
        i = i < total ? i : total - 1;
        t[q][e] = find_tensor(T, i);
        o[q][e] = i - T.start[t[q][e]];
        g[q][e] = T.g[t[q][e]][o[q][e]];
        p[q][e] = T.p[t[q][e]][o[q][e]];
        m[q][e] = T.m[t[q][e]][o[q][e]];
        v[q][e] = T.v[t[q][e]][o[q][e]];
      }
    }
  }
  if (guard && guard[BCNF_GUARD_HALTED]) return;   // a halted step (see nll_finalize) leaves all state
  // bookkeeping: the logged values go out from workgroup 0 at the start (it reads the cursor before its own
  // arrival below, hence before the last workgroup advances it), off the launch's critical path
  if (bk.done && blockIdx.x == 0 && threadIdx.x == 0) store_log(bk.log_values, bk.log_history, bk.cursor);
  const AdamScalars as = adam_scalars(step[0] + 1.0f, lr, b1d, b2d, epsd, wdd, sc);
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < G; ++q) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      if (i0[q] + e < total) {
        ss = fmaf(g[q][e], g[q][e], ss);
        adam_elem(p[q][e], g[q][e], m[q][e], v[q][e], as);
      }
    }
    if (vec[q]) {
      const int t0 = t[q][0];
      const long long o0 = o[q][0];
      *reinterpret_cast<floatx4*>(T.m[t0] + o0) = floatx4{m[q][0], m[q][1], m[q][2], m[q][3]};
      *reinterpret_cast<floatx4*>(T.v[t0] + o0) = floatx4{v[q][0], v[q][1], v[q][2], v[q][3]};
      *reinterpret_cast<floatx4*>(T.p[t0] + o0) = floatx4{p[q][0], p[q][1], p[q][2], p[q][3]};
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e)
        if (i0[q] + e < total) {
          T.m[t[q][e]][o[q][e]] = m[q][e];
          T.v[t[q][e]][o[q][e]] = v[q][e];
          T.p[t[q][e]][o[q][e]] = p[q][e];
        }
    }
  }
  const float s = wg_sum(ss, red);
  if (threadIdx.x == 0 && part) part[blockIdx.x] = s;
  if (bk.done && threadIdx.x == 0) {
    // every thread of this workgroup has consumed its step[0] read (wg_sum synchronised), so the last workgroup
    // to arrive advances the counters after every read of them. Nothing this launch wrote is read by the last
    // workgroup, so a relaxed counter suffices (no release fence: on gfx950 that is an L2 write-back per
    // workgroup); the bookkeeping's own stores reach the next launch through the kernel boundary.
    if (__hip_atomic_fetch_add(bk.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      advance_counters(bk.step, bk.cursor, bk.n_batches);
      __hip_atomic_store(bk.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void k_advance(float* step, long long* cursor, long long n_batches, const int32_t* guard) {
  if (guard && guard[BCNF_GUARD_HALTED]) return;
  if (threadIdx.x == 0) advance_counters(step, cursor, n_batches);
}

template <int G>
__global__ __launch_bounds__(BCNF_WG) void k_sumsq(TList T, float* __restrict__ part) {
  __shared__ float red[BCNF_WG];
  const long long total = T.start[T.n];
  // the same element order and fmaf chain as k_adam<G>'s partials (clip norms bit-identical either way)
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < G; ++q) {
    const long long i0 = (long long)blockIdx.x * G * CHUNK + q * CHUNK + EPT * threadIdx.x;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const long long i = i0 + e;
      if (i < total) {
        const int t = find_tensor(T, i);
        const float g = T.g[t][i - T.start[t]];
        ss = fmaf(g, g, ss);
      }
    }
  }
  const float s = wg_sum(ss, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// torch.nn.utils.clip_grad_norm_: coef = min(max_norm / (||g||_2 + 1e-6), 1); g *= coef.
template <int G>
__global__ __launch_bounds__(BCNF_WG) void k_clip(TList T, const float* __restrict__ part, int nparts, float max_norm,
                                                  float* __restrict__ norm_out, float* step, long long* cursor,
                                                  long long n_batches, const float* __restrict__ log_values,
                                                  float* log_history, const int32_t* __restrict__ guard) {
  __shared__ float red[BCNF_WG];
  // the gradient loads go out first, beside the partials' (the scaling needs the total norm, not the loads). The
  // element layout is k_adam<G>'s: thread x owns EPT = 4 consecutive elements of each group, one 16-B load / store
  // when they lie in one tensor at a 16-B aligned offset (r05: per-element loads and tensor lookups ran FC_large's
  // 49M-gradient clip at 2.3 TB/s)
  const long long total = T.start[T.n];
  float g[G][EPT];
  int t[G][EPT];
  long long o[G][EPT], i0[G];
  bool vec[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    i0[q] = (long long)blockIdx.x * G * CHUNK + q * CHUNK + EPT * threadIdx.x;
    const int t0 = find_tensor(T, i0[q] < total ? i0[q] : total - 1);
    const long long o0 = i0[q] - T.start[t0];
    vec[q] = i0[q] + EPT <= T.start[t0 + 1] && (((uintptr_t)(T.g[t0] + o0)) & 15) == 0;
    if (vec[q]) {
      const floatx4 g4 = *reinterpret_cast<const floatx4*>(T.g[t0] + o0);
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        g[q][e] = g4[e];
        t[q][e] = t0;
        o[q][e] = o0 + e;
      }
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        long long i = i0[q] + e;
        i = i < total ? i : total - 1;
        t[q][e] = find_tensor(T, i);
        o[q][e] = i - T.start[t[q][e]];
        g[q][e] = T.g[t[q][e]][o[q][e]];
      }
    }
  }
  if (guard && guard[BCNF_GUARD_HALTED]) return;
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += BCNF_WG) acc += part[i];
  const float tot = sqrtf(wg_sum(acc, red));
  const float coef = fminf(max_norm / (tot + 1e-6f), 1.0f);
#pragma unroll
  for (int q = 0; q < G; ++q) {
    if (vec[q]) {
      *reinterpret_cast<floatx4*>(T.g[t[q][0]] + o[q][0]) =
          floatx4{g[q][0] * coef, g[q][1] * coef, g[q][2] * coef, g[q][3] * coef};
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e)
        if (i0[q] + e < total) T.g[t[q][e]][o[q][e]] = g[q][e] * coef;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (norm_out) norm_out[0] = tot;
    store_log(log_values, log_history, cursor);   // the step's logged values -> history slot of this batch
    advance_counters(step, cursor, n_batches);
  }
}

// ------------------------------------------------------------------------------------------------
// Small GEMMs for nn.Linear. One wave = one 16x16 output tile, v_mfma_f32_16x16x4f32 over the
// reduction; lane l supplies A[l&15][l>>4] and B[l>>4][l&15] and owns D[4(l>>4)+i][l&15].
// C[M][Nc] = A[M][K] * op(B) + bias; op(B)[k][n] = TB ? B[n*ldb + k] : B[k*ldb + n].
// SA: every A element is multiplied by the same element of sa ([M][lda]) as it is loaded -- the backward of a fused
// GELU + dropout layer, dL/dpre = dL/da * g, never stored.
// ACT (feature MLP layer, feature_network.py:128-134: Linear -> GELU -> Dropout): the epilogue stores
// a = mask GELU(pre) and, when G is given, g = mask GELU'(pre), mask = keep_scale or 0 from Philox4x32-10
// (key = (rng seed ^ salt, (seed >> 32) ^ BCNF_FEATURE_KEY), counter = (column, row / 4, rng offset)) when rng is given,
// else 1. BCNF_FEATURE_KEY keeps every feature layer's key apart from the coupling dropout's (seed, (seed >> 32) ^
// (offset >> 32)), which otherwise coincided with the salt-0 layer's for offsets below 2^32.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t BCNF_FEATURE_KEY = 0x80000000u;
struct ActArgs {
  float* G;
  const uint64_t* rng;
  uint32_t salt, thresh;
  float keep;
};

template <bool TB, bool SA, bool ACT>
__global__ __launch_bounds__(BCNF_WG) void k_gemm(const float* __restrict__ A, int lda, const float* __restrict__ Bm,
                                                  int ldb, const float* __restrict__ bias, float* __restrict__ C,
                                                  int ldc, long long M, int Nc, int K, const float* __restrict__ sa,
                                                  ActArgs act) {
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lq = l >> 4;
  const long long row0 = ((long long)blockIdx.x * 4 + wave) * 16;
  const int col0 = blockIdx.y * 16;
  if (row0 >= M) return;
  const long long ar = row0 + lr < M ? row0 + lr : M - 1;     // clamped rows: loaded, never stored
  const int bc = col0 + lr < Nc ? col0 + lr : Nc - 1;
  const float* a = A + ar * lda;
  const float* as = SA ? sa + ar * lda : nullptr;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  int k0 = 0;
  for (; k0 + 32 <= K; k0 += 32) {              // 8 MFMA steps, all 16 loads issued first
    float av[8], bv[8], sv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int k = k0 + 4 * t + lq;
      av[t] = a[k];
      if (SA) sv[t] = as[k];
      bv[t] = TB ? Bm[(long long)bc * ldb + k] : Bm[(long long)k * ldb + bc];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = mfma4(SA ? av[t] * sv[t] : av[t], bv[t], acc);
  }
  for (; k0 < K; k0 += 4) {
    const int k = k0 + lq;
    const int kc = k < K ? k : K - 1;
    float av = a[kc];
    if (SA) av *= as[kc];
    float bv = TB ? Bm[(long long)bc * ldb + kc] : Bm[(long long)kc * ldb + bc];
    av = k < K ? av : 0.f;
    bv = k < K ? bv : 0.f;
    acc = mfma4(av, bv, acc);
  }
  const int col = col0 + lr;
  if (col < Nc) {
    const float bb = bias ? bias[col] : 0.f;
    if (ACT) {
      float m[4] = {1.f, 1.f, 1.f, 1.f};
      if (act.rng) {
        const uint64_t seed = act.rng[0], off = act.rng[1];
        const uint4 r = philox4x32_10(make_uint4((uint32_t)col, (uint32_t)((row0 >> 2) + lq), (uint32_t)off,
                                                 (uint32_t)(off >> 32)),
                                      make_uint2((uint32_t)seed ^ act.salt, (uint32_t)(seed >> 32) ^ BCNF_FEATURE_KEY));
        m[0] = r.x >= act.thresh ? act.keep : 0.f;
        m[1] = r.y >= act.thresh ? act.keep : 0.f;
        m[2] = r.z >= act.thresh ? act.keep : 0.f;
        m[3] = r.w >= act.thresh ? act.keep : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long rr = row0 + 4 * lq + i;
        float g, dg;
        gelu_fg(acc[i] + bb, g, dg);
        if (rr < M) {
          C[rr * ldc + col] = g * m[i];
          if (act.G) act.G[rr * ldc + col] = dg * m[i];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long r = row0 + 4 * lq + i;
        if (r < M) C[r * ldc + col] = acc[i] + bb;
      }
    }
  }
}

// Feature-MLP GEMMs (nn.Linear forward and dL/dx, e.g. FC_large's 2048 x 310 x 310 layers): C[M][Nc] =
// sum_r A[m][r] Bop[r][n] + bias with the reduction index r contiguous in A's rows (x, or dL/dy), Bop[r][n] =
// TB ? Bm[n][r] (forward: W) : Bm[r][n] (dL/dx: W). A workgroup owns 64 rows x LN_NT * 16 columns: its slab of Bop
// (R x LN_NT * 16 floats, coalesced loads) is staged in LDS once; each wave takes 16 rows, its A operand for 16
// reductions is ONE float4 (lane (q, r) contracts r' = 16 g + 4 q + i at MFMA step i), 4 groups in flight,
// LN_NT output tiles per A load. SA / ACT: as k_gemm. The tile-per-wave k_gemm above re-read every operand from L2
// one scalar per MFMA step (33 us for FC_large's 310 x 310 layer at B = 2048).
constexpr int LN_NT = 2;                 // 16-column MFMA tiles per wave
constexpr int LN_G = 8;                  // 16-reduction groups in flight per wave
constexpr int LN_RMAX = 1024;            // largest reduction staged in LDS (larger: k_gemm)

template <bool TB, bool SA, bool ACT>
__global__ __launch_bounds__(BCNF_WG) void k_lin(const float* __restrict__ A, int lda, const float* __restrict__ Bm,
                                                 int ldb, const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                 long long M, int Nc, int R, const float* __restrict__ sa, ActArgs act) {
  constexpr int NC = LN_NT * 16, BP = NC + 1;          // slab row pitch (odd: conflict-free column reads)
  extern __shared__ float bs[];                          // [R][BP]
  const int col0 = blockIdx.y * NC;
  // stage Bop[r][col0 .. col0 + NC) -> bs[r][c] (zero past Nc)
  constexpr int SU = 20;                                 // staging loads in flight per thread
  const int tot = R * NC;
  for (int i0 = threadIdx.x; i0 < tot; i0 += SU * BCNF_WG) {
    float v[SU];
    int dst[SU];
    bool live[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int i = i0 + u * BCNF_WG;
      const int ic = i < tot ? i : tot - 1;
      int r, c;
      if (TB) { c = ic / R; r = ic - c * R; }            // W rows: consecutive threads walk r (contiguous)
      else { r = ic / NC; c = ic - r * NC; }             // W rows: consecutive threads walk columns
      const int n = col0 + c < Nc ? col0 + c : Nc - 1;
      v[u] = TB ? Bm[(long long)n * ldb + r] : Bm[(long long)r * ldb + n];
      dst[u] = r * BP + c;
      live[u] = col0 + c < Nc;                            // columns past Nc stage zeros
    }
    asm volatile("" ::: "memory");                        // all SU loads issued before the first store
#pragma unroll
    for (int u = 0; u < SU; ++u)
      if (i0 + u * BCNF_WG < tot) bs[dst[u]] = live[u] ? v[u] : 0.f;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lq = l >> 4;
  const long long row0 = ((long long)blockIdx.x * 4 + wave) * 16;
  if (row0 >= M) return;
  const long long ar = row0 + lr < M ? row0 + lr : M - 1;     // clamped rows: loaded, never stored
  const float* a = A + ar * lda;
  const float* as = SA ? sa + ar * lda : nullptr;
  floatx4 acc[LN_NT];
#pragma unroll
  for (int t = 0; t < LN_NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int ng = R / 16;                                  // whole 16-reduction groups
  auto ld4u = [](const float* p) {                         // 4 floats at a 4-byte aligned address
    floatx4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
  };
  auto group = [&](const floatx4& av, const floatx4& sv, int g) {   // reductions 16 g .. 16 g + 15
    const float* b = bs + (16 * g + 4 * lq) * BP + lr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = SA ? av[i] * sv[i] : av[i];
#pragma unroll
      for (int t = 0; t < LN_NT; ++t) acc[t] = mfma4(x, b[i * BP + 16 * t], acc[t]);
    }
  };
  for (int g0 = 0; g0 < ng; g0 += LN_G) {
    floatx4 av[LN_G], sv[LN_G];
#pragma unroll
    for (int u = 0; u < LN_G; ++u) {                      // every load of the step first (clamped: static waits)
      const int g = g0 + u < ng ? g0 + u : ng - 1;
      av[u] = ld4u(a + 16 * g + 4 * lq);
      if (SA) sv[u] = ld4u(as + 16 * g + 4 * lq);
    }
    asm volatile("" ::: "memory");                        // hipcc may not sink them to their first use
#pragma unroll
    for (int u = 0; u < LN_G; ++u)
      if (g0 + u < ng) group(av[u], sv[u], g0 + u);       // uniform
  }
  for (int r0 = 16 * ng; r0 < R; r0 += 4) {               // reduction tail (R % 16)
    const int r = r0 + lq;
    const int rc = r < R ? r : R - 1;
    float x = a[rc];
    if (SA) x *= as[rc];
    x = r < R ? x : 0.f;
#pragma unroll
    for (int t = 0; t < LN_NT; ++t) acc[t] = mfma4(x, r < R ? bs[rc * BP + lr + 16 * t] : 0.f, acc[t]);
  }
#pragma unroll
  for (int t = 0; t < LN_NT; ++t) {
    const int col = col0 + 16 * t + lr;
    if (col >= Nc) continue;
    const float bb = bias ? bias[col] : 0.f;
    if (ACT) {
      float m[4] = {1.f, 1.f, 1.f, 1.f};
      if (act.rng) {
        const uint64_t seed = act.rng[0], off = act.rng[1];
        const uint4 rn = philox4x32_10(make_uint4((uint32_t)col, (uint32_t)((row0 >> 2) + lq), (uint32_t)off,
                                                  (uint32_t)(off >> 32)),
                                       make_uint2((uint32_t)seed ^ act.salt, (uint32_t)(seed >> 32) ^ BCNF_FEATURE_KEY));
        m[0] = rn.x >= act.thresh ? act.keep : 0.f;
        m[1] = rn.y >= act.thresh ? act.keep : 0.f;
        m[2] = rn.z >= act.thresh ? act.keep : 0.f;
        m[3] = rn.w >= act.thresh ? act.keep : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long rr = row0 + 4 * lq + i;
        float g, dg;
        gelu_fg(acc[t][i] + bb, g, dg);
        if (rr < M) {
          C[rr * ldc + col] = g * m[i];
          if (act.G) act.G[rr * ldc + col] = dg * m[i];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long rr = row0 + 4 * lq + i;
        if (rr < M) C[rr * ldc + col] = acc[t][i] + bb;
      }
    }
  }
}

// One feature-MLP GEMM: the LDS-slab kernel when the reduction fits, else the tile-per-wave one.
template <bool TB, bool SA, bool ACT>
int launch_lin(const float* A, int lda, const float* Bm, int ldb, const float* bias, float* C, int ldc, long long M,
               int Nc, int R, const float* sa, const ActArgs& act, hipStream_t st) {
  if (R <= LN_RMAX) {
    constexpr size_t kmax = sizeof(float) * LN_RMAX * (LN_NT * 16 + 1);
    static bool attr = false;                            // first (eager) call, before any capture
    if (!attr) {
      if (const int rc = bcnf_rt::hip_status(hipFuncSetAttribute((const void*)k_lin<TB, SA, ACT>,
                                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kmax)))
        return rc;
      attr = true;
    }
    const size_t lds = sizeof(float) * (size_t)R * (LN_NT * 16 + 1);
    const dim3 grid((unsigned)((M + 63) / 64), (unsigned)((Nc + LN_NT * 16 - 1) / (LN_NT * 16)));
    hipLaunchKernelGGL((k_lin<TB, SA, ACT>), grid, dim3(BCNF_WG), lds, st, A, lda, Bm, ldb, bias, C, ldc, M, Nc, R, sa,
                       act);
  } else {
    const dim3 grid((unsigned)((M + 63) / 64), (unsigned)((Nc + 15) / 16));
    hipLaunchKernelGGL((k_gemm<TB, SA, ACT>), grid, dim3(BCNF_WG), 0, st, A, lda, Bm, ldb, bias, C, ldc, M, Nc, R, sa,
                       act);
  }
  return bcnf_rt::launched();
}

// Split-K weight gradient: work[s][n][k] = sum_{m in split s} dY[m][n] X[m][k],
// bwork[s][n] = sum_{m in split s} dY[m][n]. grid = (tiles_n * tiles_k / 4 rounded up, splits).
template <bool SA>
__global__ __launch_bounds__(BCNF_WG) void k_gemm_wt(const float* __restrict__ X, const float* __restrict__ dY,
                                                     long long M, int N, int K, int rows_per_split,
                                                     float* __restrict__ work, float* __restrict__ bwork,
                                                     const float* __restrict__ sg) {
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, lr = l & 15, lq = l >> 4;
  const int tiles_k = (K + 15) / 16, tiles_n = (N + 15) / 16;
  const int tile = blockIdx.x * 4 + wave;
  if (tile >= tiles_n * tiles_k) return;
  const int n0 = (tile / tiles_k) * 16, k0 = (tile % tiles_k) * 16;
  const int s = blockIdx.y;
  const long long m_begin = (long long)s * rows_per_split;
  long long m_end = m_begin + rows_per_split;
  if (m_end > M) m_end = M;
  const int n = n0 + lr < N ? n0 + lr : N - 1;
  const int k = k0 + lr < K ? k0 + lr : K - 1;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  long long m0 = m_begin;
  for (; m0 + 32 <= m_end; m0 += 32) {
    float av[8], bv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const long long m = m0 + 4 * t + lq;
      av[t] = dY[m * N + n];
      if (SA) av[t] *= sg[m * N + n];     // dL/dpre = dL/da * g of a fused GELU + dropout layer
      bv[t] = X[m * K + k];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      bsum += av[t];
      acc = mfma4(av[t], bv[t], acc);
    }
  }
  for (; m0 < m_end; m0 += 4) {
    const long long m = m0 + lq;
    const long long mc = m < m_end ? m : m_end - 1;
    float av = dY[mc * N + n];          // A[n][m] = dY[m][n]
    if (SA) av *= sg[mc * N + n];
    float bv = X[mc * K + k];           // B[m][k] = X[m][k]
    av = m < m_end ? av : 0.f;
    bv = m < m_end ? bv : 0.f;
    bsum += av;
    acc = mfma4(av, bv, acc);
  }
  float* w = work + (long long)s * N * K;
  const int kk = k0 + lr;
  if (kk < K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nn = n0 + 4 * lq + i;
      if (nn < N) w[(long long)nn * K + kk] = acc[i];
    }
  }
  if (k0 == 0 && bwork) {             // dY column sums of this split: fold the 4 lane quarters
    bsum += __shfl_xor(bsum, 16);
    bsum += __shfl_xor(bsum, 32);
    if (lq == 0 && n0 + lr < N) bwork[(long long)s * N + n0 + lr] = bsum;
  }
}

__global__ __launch_bounds__(BCNF_WG) void k_wt_reduce(const float* __restrict__ work, const float* __restrict__ bwork,
                                                       int splits, int N, int K, float* __restrict__ dW,
                                                       float* __restrict__ db) {
  const long long NK = (long long)N * K;
  const long long i = (long long)blockIdx.x * BCNF_WG + threadIdx.x;
  const float* src;
  long long stride;
  float* dst;
  if (i < NK) {
    src = work + i;
    stride = NK;
    dst = dW + i;
  } else if (db && i < NK + N) {
    src = bwork + (i - NK);
    stride = N;
    dst = db + (i - NK);
  } else {
    return;
  }
  float acc = 0.f;
  int s = 0;
  for (; s + 8 <= splits; s += 8) {              // 8 loads in flight, summed in split order
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = src[(long long)(s + t) * stride];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc += v[t];
  }
  for (; s < splits; ++s) acc += src[(long long)s * stride];
  *dst = acc;
}

using bcnf_rt::launched;

__global__ __launch_bounds__(BCNF_WG) void k_gather2(const int64_t* __restrict__ idx, int n, int rpw,
                                                     const float* __restrict__ s0, int c0, float* __restrict__ d0,
                                                     const float* __restrict__ s1, int c1, float* __restrict__ d1,
                                                     const long long* __restrict__ cursor) {
  gather2_rows(idx, n, rpw, s0, c0, d0, s1, c1, d1, cursor, blockIdx.x);
}

int make_tlist(int n, float* const* p, float* const* g, float* const* m, float* const* v, const int64_t* numel,
               TList* T) {
  if (n < 1 || n > BCNF_MAX_TENSORS || !g || !numel) return BCNF_ERR_ARG;
  T->n = n;
  T->start[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (numel[i] < 0 || !g[i]) return BCNF_ERR_ARG;
    T->p[i] = p ? p[i] : nullptr;
    T->g[i] = g[i];
    T->m[i] = m ? m[i] : nullptr;
    T->v[i] = v ? v[i] : nullptr;
    T->start[i + 1] = T->start[i] + numel[i];
  }
  return BCNF_OK;
}

int split_rows(long long M) {        // rows per split-K chunk of the weight gradient: <= 32 splits
  long long r = (M + 31) / 32;
  if (r < 128) r = 128;
  return (int)((r + 31) & ~31LL);
}

// Element groups per thread of k_adam / k_sumsq / k_clip: BIG_G for large parameter sets (>= 4M), else 1. At
// FC_large's 48.9M parameters (tools/opt_bench.py, profiles/r05x_opt_bench.txt) Adam takes 297 us at 2 groups, 348 at
// 4 (the register arrays of 4 groups cost occupancy), 600 at 8; the clip 131 / 124 / 178 us (103 us at 2 groups once
// k_sum_partials stopped being a serial chain, r05zz3).
constexpr int BIG_G = 2;
inline int adam_groups(int64_t total_numel) { return total_numel >= (1 << 22) ? BIG_G : 1; }
inline int64_t n_partials(int64_t total_numel) {
  const int64_t per = (int64_t)CHUNK * adam_groups(total_numel);
  return total_numel <= 0 ? 1 : (total_numel + per - 1) / per;
}

// Sum of many partials by one workgroup (fixed order), so that every clip workgroup then reads one value
// instead of re-reducing all partials (quadratic in the parameter count otherwise). 1024 threads, 16-B loads, eight in
// flight per thread: FC_large's 23.9k partials are ~6 loads per thread, not a 94-deep chain of dependent ones (the
// 256-thread scalar loop took 18 us at 12k partials, r04zz2).
constexpr int CLIP_DIRECT_PARTIALS = 2048;
constexpr int SP_WG = 1024;
constexpr int SP_U = 8;
__global__ __launch_bounds__(SP_WG) void k_sum_partials(const float* __restrict__ part, int nparts,
                                                       float* __restrict__ out, const int32_t* __restrict__ guard) {
  __shared__ float red[SP_WG / 64];
  if (guard && guard[BCNF_GUARD_HALTED]) return;
  const int n4 = (reinterpret_cast<uintptr_t>(part) & 15) ? 0 : nparts >> 2;    // scalar loop if unaligned
  const floatx4* __restrict__ p4 = reinterpret_cast<const floatx4*>(part);
  float acc[SP_U];
#pragma unroll
  for (int u = 0; u < SP_U; ++u) acc[u] = 0.f;
  for (int b = threadIdx.x; b < n4; b += SP_WG * SP_U) {
    floatx4 v[SP_U];
#pragma unroll
    for (int u = 0; u < SP_U; ++u) v[u] = b + u * SP_WG < n4 ? p4[b + u * SP_WG] : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < SP_U; ++u) acc[u] += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
  }
  float a = 0.f;
#pragma unroll
  for (int u = 0; u < SP_U; ++u) a += acc[u];
  for (int i = 4 * n4 + threadIdx.x; i < nparts; i += SP_WG) a += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < SP_WG / 64; ++w) s += red[w];
    out[0] = s;
  }
}

}  // namespace

extern "C" {

// one partial per workgroup of k_adam / k_sumsq, plus one slot for the pre-reduced total of large sets
int64_t bcnf_grad_partials(int64_t total_numel) { return n_partials(total_numel) + 1; }

int bcnf_adam_step(int32_t n_tensors, float* const* params, float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numel, float* step, double lr, double beta1,
                   double beta2, double eps, double weight_decay, float* grad_partials, int32_t advance_step,
                   const int32_t* guard, void* stream) {
  TList T;
  int rc = make_tlist(n_tensors, params, grads, exp_avg, exp_avg_sq, numel, &T);
  if (rc) return rc;
  if (!params || !exp_avg || !exp_avg_sq || !step) return BCNF_ERR_ARG;
  for (int i = 0; i < n_tensors; ++i)
    if (!T.p[i] || !T.m[i] || !T.v[i]) return BCNF_ERR_ARG;
  const long long total = T.start[T.n];
  const unsigned nwg = (unsigned)n_partials(total);
  if (adam_groups(total) == BIG_G)
    hipLaunchKernelGGL(k_adam<BIG_G>, dim3(nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, T, step, lr, beta1, beta2, eps,
                       weight_decay, grad_partials, guard, AdamBook{});
  else
    hipLaunchKernelGGL(k_adam<1>, dim3(nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, T, step, lr, beta1, beta2, eps,
                       weight_decay, grad_partials, guard, AdamBook{});
  if ((rc = launched()) || !advance_step) return rc;
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, step, (long long*)nullptr, 0LL, guard);
  return launched();
}

int bcnf_adam_step_bookkeep(int32_t n_tensors, float* const* params, float* const* grads, float* const* exp_avg,
                            float* const* exp_avg_sq, const int64_t* numel, float* step, double lr, double beta1,
                            double beta2, double eps, double weight_decay, int64_t* advance_cursor,
                            int64_t cursor_modulo, const float* log_values, float* log_history, int32_t* done_counter,
                            const int32_t* guard, void* stream) {
  TList T;
  int rc = make_tlist(n_tensors, params, grads, exp_avg, exp_avg_sq, numel, &T);
  if (rc) return rc;
  if (!params || !exp_avg || !exp_avg_sq || !step || !done_counter) return BCNF_ERR_ARG;
  if (advance_cursor && cursor_modulo < 1) return BCNF_ERR_ARG;
  for (int i = 0; i < n_tensors; ++i)
    if (!T.p[i] || !T.m[i] || !T.v[i]) return BCNF_ERR_ARG;
  const long long total = T.start[T.n];
  const unsigned nwg = (unsigned)n_partials(total);
  const AdamBook bk{step, (long long*)advance_cursor, (long long)cursor_modulo, log_values, log_history,
                    (int*)done_counter};
  if (adam_groups(total) == BIG_G)
    hipLaunchKernelGGL(k_adam<BIG_G>, dim3(nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, T, step, lr, beta1, beta2, eps,
                       weight_decay, (float*)nullptr, guard, bk);
  else
    hipLaunchKernelGGL(k_adam<1>, dim3(nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, T, step, lr, beta1, beta2, eps,
                       weight_decay, (float*)nullptr, guard, bk);
  return launched();
}

int bcnf_grad_sumsq(int32_t n_tensors, float* const* grads, const int64_t* numel, float* grad_partials, void* stream) {
  TList T;
  int rc = make_tlist(n_tensors, nullptr, grads, nullptr, nullptr, numel, &T);
  if (rc) return rc;
  if (!grad_partials) return BCNF_ERR_ARG;
  const unsigned nwg = (unsigned)n_partials(T.start[T.n]);
  if (adam_groups(T.start[T.n]) == BIG_G)
    hipLaunchKernelGGL(k_sumsq<BIG_G>, dim3(nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, T, grad_partials);
  else
    hipLaunchKernelGGL(k_sumsq<1>, dim3(nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, T, grad_partials);
  return launched();
}

int bcnf_clip_grad_norm(int32_t n_tensors, float* const* grads, const int64_t* numel, const float* grad_partials,
                        float max_norm, float* total_norm, float* advance_step, int64_t* advance_cursor,
                        int64_t cursor_modulo, const float* log_values, float* log_history, const int32_t* guard,
                        void* stream) {
  TList T;
  int rc = make_tlist(n_tensors, nullptr, grads, nullptr, nullptr, numel, &T);
  if (rc) return rc;
  if (!grad_partials) return BCNF_ERR_ARG;
  const long long np = n_partials(T.start[T.n]);
  if (advance_cursor && cursor_modulo < 1) return BCNF_ERR_ARG;
  const float* part = grad_partials;
  int nread = (int)np;
  if (np > CLIP_DIRECT_PARTIALS) {      // pre-reduce into the extra slot
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(SP_WG), 0, (hipStream_t)stream, grad_partials, (int)np,
                       const_cast<float*>(grad_partials) + np, guard);
    part = grad_partials + np;
    nread = 1;
  }
  if (adam_groups(T.start[T.n]) == BIG_G)
    hipLaunchKernelGGL(k_clip<BIG_G>, dim3((unsigned)np), dim3(BCNF_WG), 0, (hipStream_t)stream, T, part, nread,
                       max_norm, total_norm, advance_step, (long long*)advance_cursor, (long long)cursor_modulo,
                       log_values, log_history, guard);
  else
    hipLaunchKernelGGL(k_clip<1>, dim3((unsigned)np), dim3(BCNF_WG), 0, (hipStream_t)stream, T, part, nread,
                       max_norm, total_norm, advance_step, (long long*)advance_cursor, (long long)cursor_modulo,
                       log_values, log_history, guard);
  return launched();
}

namespace {
int gather_launch(const int64_t* idx, int64_t n, const float* src0, int32_t cols0, float* dst0, const float* src1,
                  int32_t cols1, float* dst1, const int64_t* cursor, void* stream) {
  if (n * (int64_t)(cols0 + cols1) >= (1LL << 31)) return BCNF_ERR_UNSUPPORTED;
  int rpw, nwg;
  gather2_plan(n, &rpw, &nwg);
  hipLaunchKernelGGL(k_gather2, dim3((unsigned)nwg), dim3(BCNF_WG), 0, (hipStream_t)stream, idx,
                     (int)n, rpw, src0, cols0, dst0, src1, cols1, dst1, (const long long*)cursor);
  return launched();
}
}  // namespace

int bcnf_gather_rows2(const int64_t* idx, int64_t n, const float* src0, int32_t cols0, float* dst0,
                      const float* src1, int32_t cols1, float* dst1, void* stream) {
  if (n < 0 || cols0 < 1 || cols1 < 1) return BCNF_ERR_ARG;
  if (n == 0) return BCNF_OK;
  if (!idx || !src0 || !dst0 || !src1 || !dst1) return BCNF_ERR_ARG;
  return gather_launch(idx, n, src0, cols0, dst0, src1, cols1, dst1, nullptr, stream);
}

int bcnf_gather_batch(const int64_t* order, const int64_t* cursor, int64_t batch, const float* src0, int32_t cols0,
                      float* dst0, const float* src1, int32_t cols1, float* dst1, void* stream) {
  if (batch < 1 || cols0 < 1 || cols1 < 1) return BCNF_ERR_ARG;
  if (!order || !cursor || !src0 || !dst0 || !src1 || !dst1) return BCNF_ERR_ARG;
  return gather_launch(order, batch, src0, cols0, dst0, src1, cols1, dst1, cursor, stream);
}

int bcnf_advance_counters(float* step, int64_t* cursor, int64_t n_batches, void* stream) {
  if (cursor && n_batches < 1) return BCNF_ERR_ARG;
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, step, (long long*)cursor,
                     (long long)n_batches, (const int32_t*)nullptr);
  return launched();
}

__global__ void k_guard_global(const float* __restrict__ vals, int32_t* guard) {
  if (threadIdx.x != 0 || guard[BCNF_GUARD_HALTED] || !guard[BCNF_GUARD_CHECK_GLOBAL]) return;
  const float loss = vals[0];
  if (loss > 1e5f || isnan(loss)) guard[BCNF_GUARD_DIVERGED] = 1;
}

int bcnf_guard_check_global(const float* global_values, int32_t* guard, void* stream) {
  if (!global_values || !guard) return BCNF_ERR_ARG;
  hipLaunchKernelGGL(k_guard_global, dim3(1), dim3(64), 0, (hipStream_t)stream, global_values, guard);
  return launched();
}

int bcnf_linear_forward(const float* x, const float* weight, const float* bias, int64_t rows, int32_t in_features,
                        int32_t out_features, float* y, void* stream) {
  if (rows < 0 || in_features < 1 || out_features < 1) return BCNF_ERR_ARG;
  if (rows == 0) return BCNF_OK;
  if (!x || !weight || !y) return BCNF_ERR_ARG;
  return launch_lin<true, false, false>(x, in_features, weight, in_features, bias, y, out_features, rows, out_features,
                                        in_features, nullptr, ActArgs{}, (hipStream_t)stream);
}

int bcnf_linear_gelu_forward(const float* x, const float* weight, const float* bias, int64_t rows, int32_t in_features,
                             int32_t out_features, float p, const uint64_t* rng, int32_t salt, float* a, float* g,
                             void* stream) {
  if (rows < 0 || in_features < 1 || out_features < 1 || !(p >= 0.f && p < 1.f)) return BCNF_ERR_ARG;
  if (rows == 0) return BCNF_OK;
  if (!x || !weight || !a) return BCNF_ERR_ARG;
  ActArgs act{g, p > 0.f ? rng : nullptr, (uint32_t)salt * 0x9E3779B9u, 0u, 1.f};
  if (act.rng) {
    act.thresh = (uint32_t)fmin(4294967295.0, floor((double)p * 4294967296.0 + 0.5));   // keep iff u >= thresh
    act.keep = (float)(1.0 / (1.0 - (double)p));
  }
  return launch_lin<true, false, true>(x, in_features, weight, in_features, bias, a, out_features, rows, out_features,
                                       in_features, nullptr, act, (hipStream_t)stream);
}

int64_t bcnf_linear_work_bytes(int64_t rows, int32_t in_features, int32_t out_features) {
  if (rows <= 0) return 0;
  const long long splits = (rows + split_rows(rows) - 1) / split_rows(rows);
  return (int64_t)splits * ((int64_t)out_features * in_features + out_features) * 4;
}

}  // extern "C"

namespace {
// dL/dx, dL/dW, dL/db of y = x W^T + b from dy, or -- sg given -- of a fused GELU + dropout layer from dL/da = dy and
// its saved g (dL/dpre = dy * g, formed as each operand element is loaded).
int linear_backward(const float* x, const float* weight, const float* dy, const float* sg, int64_t rows, int K, int N,
                    float* dx, float* dweight, float* dbias, void* work, hipStream_t st) {
  if (rows == 0) {
    if (dweight)
      if (const int rc = bcnf_rt::hip_status(hipMemsetAsync(dweight, 0, sizeof(float) * (size_t)N * K, st))) return rc;
    if (dbias)
      if (const int rc = bcnf_rt::hip_status(hipMemsetAsync(dbias, 0, sizeof(float) * (size_t)N, st))) return rc;
    return BCNF_OK;
  }
  if (!dy) return BCNF_ERR_ARG;
  if (dx) {   // dX[m][k] = sum_n dY[m][n] W[n][k]
    if (!weight) return BCNF_ERR_ARG;
    int rc = sg ? launch_lin<false, true, false>(dy, N, weight, K, nullptr, dx, K, rows, K, N, sg, ActArgs{}, st)
                : launch_lin<false, false, false>(dy, N, weight, K, nullptr, dx, K, rows, K, N, nullptr, ActArgs{}, st);
    if (rc) return rc;
  }
  if (dweight || dbias) {
    if (!x || !work || !dweight) return BCNF_ERR_ARG;
    const int rps = split_rows(rows);
    const int splits = (int)((rows + rps - 1) / rps);
    const int tiles = ((N + 15) / 16) * ((K + 15) / 16);
    float* w = (float*)work;
    float* bw = w + (long long)splits * N * K;
    const dim3 grid((unsigned)((tiles + 3) / 4), (unsigned)splits);
    if (sg)
      hipLaunchKernelGGL(k_gemm_wt<true>, grid, dim3(BCNF_WG), 0, st, x, dy, (long long)rows, N, K, rps, w,
                         dbias ? bw : nullptr, sg);
    else
      hipLaunchKernelGGL(k_gemm_wt<false>, grid, dim3(BCNF_WG), 0, st, x, dy, (long long)rows, N, K, rps, w,
                         dbias ? bw : nullptr, (const float*)nullptr);
    int rc = launched();
    if (rc) return rc;
    const long long outs = (long long)N * K + (dbias ? N : 0);
    hipLaunchKernelGGL(k_wt_reduce, dim3((unsigned)((outs + BCNF_WG - 1) / BCNF_WG)), dim3(BCNF_WG), 0, st, w, bw,
                       splits, N, K, dweight, dbias);
    return launched();
  }
  return BCNF_OK;
}
}  // namespace

extern "C" {

int bcnf_linear_backward(const float* x, const float* weight, const float* dy, int64_t rows, int32_t in_features,
                         int32_t out_features, float* dx, float* dweight, float* dbias, void* work, void* stream) {
  if (rows < 0 || in_features < 1 || out_features < 1) return BCNF_ERR_ARG;
  return linear_backward(x, weight, dy, nullptr, rows, in_features, out_features, dx, dweight, dbias, work,
                         (hipStream_t)stream);
}

int bcnf_linear_gelu_backward(const float* x, const float* weight, const float* da, const float* g, int64_t rows,
                              int32_t in_features, int32_t out_features, float* dx, float* dweight, float* dbias,
                              void* work, void* stream) {
  if (rows < 0 || in_features < 1 || out_features < 1 || (rows > 0 && !g)) return BCNF_ERR_ARG;
  return linear_backward(x, weight, da, g, rows, in_features, out_features, dx, dweight, dbias, work,
                         (hipStream_t)stream);
}

}  // extern "C"
