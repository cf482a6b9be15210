// bcnf_amd: fused CondRealNVP_v2 coupling stack for MI355X (gfx950 / CDNA4).
//
// Kernels (all fp32):
//   k_pack      canonical nn.Module parameters -> per-lane LDS records (rotation-ready weight rows)
//   k_ldc       ActNorm log|det| constant  sum_k sum_i log|scale_k,i|            (cnf.py:350)
//   k_forward   whole-stack forward, one launch: ActNorm -> nested MLP (GELU, dropout) -> affine
//               coupling -> log-det -> orthonormal mix, for all n_blocks   (cnf.py:476-488)
//   k_inverse   whole-stack inverse, one launch                              (cnf.py:499-506)
//   k_backward  whole-stack backward with per-block recompute, one launch; dW via fp32 MFMA on LDS
//               tiles of the workgroup's 16 samples; per-workgroup slabs
//   k_reduce    deterministic slab sum -> canonical flat gradient
//
// Reference: psaegert/bcnf src/bcnf/models/cnf.py. See DESIGN.md for layouts and rooflines.
#include "bcnf_device.h"
#include "../../include/bcnf_amd.h"

#include <math.h>
#include <string.h>

#include <mutex>

namespace {

constexpr int NT_EXTRA = 7;            // tiles: D_1..D_NH, D_T, D_S, A_0..A_NH, PA, GA, PB, GB
constexpr int TILE = BCNF_ROWS * BCNF_TSTRIDE;   // 272 floats
constexpr int MAXPF = 8;               // max float4 per thread for one staged record set

// ------------------------------------------------------------------------------------------------
// Host-side layout
// ------------------------------------------------------------------------------------------------
int round_rec(int n) {            // multiple of 4 floats with odd quotient (conflict-free ds_read_b128)
  n = (n + 3) & ~3;
  if (((n / 4) & 1) == 0) n += 4;
  return n;
}

int make_layout(const BcnfStackDesc* d, BcnfLayout* L) {
  if (!d || !L) return BCNF_ERR_ARG;
  memset(L, 0, sizeof(*L));
  if (d->size < 2 || d->n_blocks < 1 || d->n_hidden < 0 || d->n_hidden > BCNF_MAX_HIDDEN || d->n_conditions < 0)
    return BCNF_ERR_ARG;
  for (int i = 0; i < d->n_hidden; ++i)
    if (d->hidden[i] < 1) return BCNF_ERR_ARG;
  if (!(d->dropout >= 0.f && d->dropout < 1.f)) return BCNF_ERR_ARG;
  L->D = d->size;
  L->Da = (d->size + 1) / 2;
  L->Db = d->size / 2;
  L->C = d->n_conditions;
  L->Cp = ((d->n_conditions + 15) / 16) * 16;
  if (L->Cp == 0) L->Cp = 16;
  L->NH = d->n_hidden;
  L->nb = d->n_blocks;
  L->act_norm = d->act_norm ? 1 : 0;
  L->H[0] = L->Da;
  for (int i = 0; i < L->NH; ++i) L->H[i + 1] = d->hidden[i];
  L->H[L->NH + 1] = 2 * L->Db;
  int off = 0;
  for (int l = 1; l <= L->NH + 1; ++l) {
    L->lin_in[l] = (l == 1) ? (L->Da + L->C) : L->H[l - 1];
    L->lin_out[l] = L->H[l];
    L->lin_w[l] = off;
    off += L->lin_in[l] * L->lin_out[l];
    L->lin_b[l] = off;
    off += L->lin_out[l];
  }
  L->an_size = L->act_norm ? 2 * L->D : 0;
  L->blk_stride = L->an_size + off;
  L->n_trainable = (L->nb - 1) * L->blk_stride + off;
  L->p = d->dropout;
  L->keep_scale = (d->dropout > 0.f) ? (1.0f / (1.0f - d->dropout)) : 1.0f;
  double t = (double)d->dropout * 65536.0;
  L->thresh16 = (uint32_t)llround(t);
  // forward/inverse record: [sa ba sb bb][b1 pad pad pad][W1y:16][hidden l: 16+1 ...][T:16+1][S:16+1][Q:64]
  L->rf_b1 = 4;
  L->rf_w1 = 8;
  L->rf_hid = 24;
  L->rf_t = L->rf_hid + 17 * (L->NH > 0 ? L->NH - 1 : 0);
  L->rf_s = L->rf_t + 17;
  L->rf_q = (L->rf_s + 17 + 3) & ~3;
  L->RF = round_rec(L->rf_q + 64);
  // backward record: [W1T:16][hidden^T l: 16 ...][Tout^T:16][Sout^T:16][Q^T:64]
  L->rb_w1t = 0;
  L->rb_hid = 16;
  L->rb_tt = 16 + 16 * (L->NH > 0 ? L->NH - 1 : 0);
  L->rb_st = L->rb_tt + 16;
  L->rb_qt = L->rb_st + 16;
  L->RB = round_rec(L->rb_qt + 64);
  long long nbl = L->nb;
  L->pf_off = 0;
  L->pb_off = L->pf_off + nbl * 16 * L->RF;
  L->pi_off = L->pb_off + nbl * 16 * L->RB;
  L->w1t_off = L->pi_off + nbl * 16 * L->RF;
  L->w1h_off = L->w1t_off + nbl * L->Cp * 16;
  L->ldc_off = L->w1h_off + nbl * 16 * L->Cp;
  L->total = L->ldc_off + 4;
  return BCNF_OK;
}

bool layout_supported(const BcnfLayout& L, const BcnfStackDesc* d) {
  if (d->two_way) return false;
  if (L.NH < 1 || L.NH > BCNF_MAX_HIDDEN) return false;
  if (L.Da > 16 || L.Db > 16) return false;
  for (int l = 1; l <= L.NH; ++l)
    if (L.H[l] > 16) return false;
  if (L.C < 1 || L.Cp > 256) return false;
  if (16 * (L.RF + L.RB) > MAXPF * 4 * BCNF_WG) return false;
  return true;
}

// ------------------------------------------------------------------------------------------------
// Packing
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float cW(const BcnfLayout& L, const float* P, int k, int l, int row, int col) {
  return P[coupling_base(L, k) + L.lin_w[l] + row * L.lin_in[l] + col];
}
__device__ __forceinline__ float cB(const BcnfLayout& L, const float* P, int k, int l, int row) {
  return P[coupling_base(L, k) + L.lin_b[l] + row];
}

// PF (inverse=false) / PI (inverse=true) record entry e of lane j in block k.
__device__ float rec_f(const BcnfLayout& L, const float* P, const float* Q, int k, int j, int e, bool inverse) {
  const int Da = L.Da, Db = L.Db, D = L.D, NH = L.NH;
  const bool has_an = L.act_norm && k < L.nb - 1;
  const int anb = k * L.blk_stride;
  if (e < 4) {
    switch (e) {
      case 0: return (j < Da) ? (has_an ? P[anb + j] : 1.f) : 0.f;
      case 1: return (j < Da && has_an) ? P[anb + D + j] : 0.f;
      case 2: return (j < Db) ? (has_an ? P[anb + Da + j] : 1.f) : 0.f;
      default: return (j < Db && has_an) ? P[anb + D + Da + j] : 0.f;
    }
  }
  if (e == L.rf_b1) return (j < L.H[1]) ? cB(L, P, k, 1, j) : 0.f;
  if (e >= L.rf_w1 && e < L.rf_w1 + 16) {
    const int src = (j - (e - L.rf_w1)) & 15;
    return (j < L.H[1] && src < Da) ? cW(L, P, k, 1, j, src) : 0.f;
  }
  if (e >= L.rf_hid && e < L.rf_t) {
    const int l = 2 + (e - L.rf_hid) / 17, r = (e - L.rf_hid) % 17;
    if (r == 16) return (j < L.H[l]) ? cB(L, P, k, l, j) : 0.f;
    const int src = (j - r) & 15;
    return (j < L.H[l] && src < L.H[l - 1]) ? cW(L, P, k, l, j, src) : 0.f;
  }
  if (e >= L.rf_t && e < L.rf_t + 34) {
    const int half = (e - L.rf_t) / 17, r = (e - L.rf_t) % 17;   // half 0: t rows, 1: s rows
    if (r == 16) return (j < Db) ? cB(L, P, k, NH + 1, half * Db + j) : 0.f;
    const int src = (j - r) & 15;
    return (j < Db && src < L.H[NH]) ? cW(L, P, k, NH + 1, half * Db + j, src) : 0.f;
  }
  if (e >= L.rf_q && e < L.rf_q + 64) {
    if (k >= L.nb - 1) return 0.f;
    const float* q = Q + (long long)k * D * D;
    const int qi = (e - L.rf_q) / 16, r = (e - L.rf_q) % 16, src = (j - r) & 15;
    if (!inverse) {  // y_new = y @ Q   (cnf.py:335): [q0 QAA | q1 QBA | q2 QAB | q3 QBB]
      switch (qi) {
        case 0: return (j < Da && src < Da) ? q[src * D + j] : 0.f;
        case 1: return (j < Da && src < Db) ? q[(Da + src) * D + j] : 0.f;
        case 2: return (j < Db && src < Da) ? q[src * D + Da + j] : 0.f;
        default: return (j < Db && src < Db) ? q[(Da + src) * D + Da + j] : 0.f;
      }
    } else {         // z_prev = y @ Q^T (cnf.py:339): [q0 over a->a | q1 over b->a | q2 over a->b | q3 over b->b]
      switch (qi) {
        case 0: return (j < Da && src < Da) ? q[j * D + src] : 0.f;
        case 1: return (j < Da && src < Db) ? q[j * D + Da + src] : 0.f;
        case 2: return (j < Db && src < Da) ? q[(Da + j) * D + src] : 0.f;
        default: return (j < Db && src < Db) ? q[(Da + j) * D + Da + src] : 0.f;
      }
    }
  }
  return 0.f;
}

// PB record entry (transposed weight rows for the backward).
__device__ float rec_b(const BcnfLayout& L, const float* P, const float* Q, int k, int j, int e) {
  const int NH = L.NH, Db = L.Db;
  if (e < 16) {
    const int src = (j - e) & 15;
    return (j < L.Da && src < L.H[1]) ? cW(L, P, k, 1, src, j) : 0.f;
  }
  if (e >= L.rb_hid && e < L.rb_tt) {
    const int l = 2 + (e - L.rb_hid) / 16, r = (e - L.rb_hid) % 16, src = (j - r) & 15;
    return (j < L.H[l - 1] && src < L.H[l]) ? cW(L, P, k, l, src, j) : 0.f;
  }
  if (e >= L.rb_tt && e < L.rb_qt) {
    const int half = (e - L.rb_tt) / 16, r = (e - L.rb_tt) % 16, src = (j - r) & 15;
    return (j < L.H[NH] && src < Db) ? cW(L, P, k, NH + 1, half * Db + src, j) : 0.f;
  }
  if (e >= L.rb_qt && e < L.rb_qt + 64) return rec_f(L, P, Q, k, j, L.rf_q + (e - L.rb_qt), true);
  return 0.f;
}

__global__ void k_pack(BcnfLayout L, const float* __restrict__ P, const float* __restrict__ Q, float* __restrict__ out) {
  const long long n_pf = (long long)L.nb * 16 * L.RF;
  const long long n_pb = (long long)L.nb * 16 * L.RB;
  const long long n_w = (long long)L.nb * L.Cp * 16;
  const long long total = 2 * n_pf + n_pb + 2 * n_w;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    float v;
    long long o;
    if (i < n_pf) {                                   // PF
      const int e = (int)(i % L.RF), j = (int)((i / L.RF) % 16), k = (int)(i / (16LL * L.RF));
      v = rec_f(L, P, Q, k, j, e, false);
      o = L.pf_off + i;
    } else if (i < n_pf + n_pb) {                     // PB
      const long long ii = i - n_pf;
      const int e = (int)(ii % L.RB), j = (int)((ii / L.RB) % 16), k = (int)(ii / (16LL * L.RB));
      v = rec_b(L, P, Q, k, j, e);
      o = L.pb_off + ii;
    } else if (i < 2 * n_pf + n_pb) {                 // PI
      const long long ii = i - n_pf - n_pb;
      const int e = (int)(ii % L.RF), j = (int)((ii / L.RF) % 16), k = (int)(ii / (16LL * L.RF));
      v = rec_f(L, P, Q, k, j, e, true);
      o = L.pi_off + ii;
    } else if (i < 2 * n_pf + n_pb + n_w) {           // W1hT [k][c][j]
      const long long ii = i - 2 * n_pf - n_pb;
      const int j = (int)(ii % 16), c = (int)((ii / 16) % L.Cp), k = (int)(ii / (16LL * L.Cp));
      v = (j < L.H[1] && c < L.C) ? cW(L, P, k, 1, j, L.Da + c) : 0.f;
      o = L.w1t_off + ii;
    } else {                                          // W1h [k][j][c]
      const long long ii = i - 2 * n_pf - n_pb - n_w;
      const int c = (int)(ii % L.Cp), j = (int)((ii / L.Cp) % 16), k = (int)(ii / (16LL * L.Cp));
      v = (j < L.H[1] && c < L.C) ? cW(L, P, k, 1, j, L.Da + c) : 0.f;
      o = L.w1h_off + ii;
    }
    out[o] = v;
  }
}

// sum over ActNorm layers of sum_i log|scale_i| (cnf.py:350); one workgroup, fixed order.
__global__ void k_ldc(BcnfLayout L, const float* __restrict__ P, float* __restrict__ out) {
  __shared__ float part[BCNF_WG];
  float acc = 0.f;
  if (L.act_norm) {
    const int n = (L.nb - 1) * L.D;
    for (int i = threadIdx.x; i < n; i += BCNF_WG) {
      const int k = i / L.D, d = i - k * L.D;
      acc += logf(fabsf(P[k * L.blk_stride + d]));
    }
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = BCNF_WG / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[L.ldc_off] = part[0];
}

// ------------------------------------------------------------------------------------------------
// Shared pieces of the stack kernels
// ------------------------------------------------------------------------------------------------
// Cooperative copy of n floats (multiple of 4) global -> registers (phase 1) -> LDS (phase 2).
// Named members (no array) so the staging registers never become a scratch alloca.
struct Stage {
  floatx4 r0, r1, r2, r3, r4, r5, r6, r7;   // ext_vector (not HIP's float4 struct: that copies via memcpy)
  __device__ __forceinline__ void load(const float* __restrict__ g, int n) {
    const floatx4* g4 = reinterpret_cast<const floatx4*>(g);
    const int n4 = n >> 2, t = (int)threadIdx.x;
#define BCNF_LD(I) { const int idx = t + (I) * BCNF_WG; r##I = g4[idx < n4 ? idx : 0]; }
    BCNF_LD(0) BCNF_LD(1) BCNF_LD(2) BCNF_LD(3) BCNF_LD(4) BCNF_LD(5) BCNF_LD(6) BCNF_LD(7)
#undef BCNF_LD
  }
  __device__ __forceinline__ void store(float* __restrict__ s, int n) const {
    floatx4* s4 = reinterpret_cast<floatx4*>(s);
    const int n4 = n >> 2, t = (int)threadIdx.x;
#define BCNF_ST(I) { const int idx = t + (I) * BCNF_WG; if (idx < n4) s4[idx] = r##I; }
    BCNF_ST(0) BCNF_ST(1) BCNF_ST(2) BCNF_ST(3) BCNF_ST(4) BCNF_ST(5) BCNF_ST(6) BCNF_ST(7)
#undef BCNF_ST
  }
};
static_assert(MAXPF == 8, "Stage holds 8 float4 per thread");

// Stage the workgroup's 16 feature rows h[row] (optionally gathered via cond_index) into
// ht[16][Cp+1], zero-padded to Cp columns.
__device__ __forceinline__ void stage_features(const BcnfLayout& L, const float* __restrict__ h,
                                               const int64_t* __restrict__ cond_index, long long n_rows,
                                               float* __restrict__ ht) {
  const int Cp = L.Cp, hs = Cp + 1;
  for (int i = threadIdx.x; i < 16 * Cp; i += BCNF_WG) {
    const int ss = i / Cp, c = i - ss * Cp;
    long long bb = (long long)blockIdx.x * 16 + ss;
    if (bb > n_rows - 1) bb = n_rows - 1;
    const long long src = cond_index ? (long long)cond_index[bb] : bb;
    ht[ss * hs + c] = (c < L.C) ? h[src * L.C + c] : 0.f;
  }
}

// Per-wave K-quarter of HP_k = H (16 x Cp) @ W1h_k^T (Cp x 16) on fp32 MFMA; partial tile to hpbuf[wave].
__device__ __forceinline__ void hp_quarter(const BcnfLayout& L, const float* __restrict__ w1t,
                                           const float* __restrict__ ht, float* __restrict__ hpbuf, int blk) {
  const int wave = threadIdx.x >> 6, l64 = threadIdx.x & 63, q = l64 >> 4, r = l64 & 15;
  const int nsteps = L.Cp >> 2;
  const int t0 = (wave * nsteps) >> 2, t1 = ((wave + 1) * nsteps) >> 2;
  const float* wb = w1t + (long long)blk * L.Cp * 16;
  const int hs = L.Cp + 1;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t = t0; t < t1; ++t) acc = mfma4(ht[r * hs + 4 * t + q], wb[(4 * t + q) * 16 + r], acc);
  float* o = hpbuf + wave * 256;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[(4 * q + i) * 16 + r] = acc[i];
}

__device__ __forceinline__ float hp_sum(const float* __restrict__ hpbuf, int s, int j) {
  const float* p = hpbuf + s * 16 + j;
  return (p[0] + p[256]) + (p[512] + p[768]);
}

// Nested MLP forward on the row layout (cnf.py:98-107). Input x (layer-1 y-part operand), returns
// t, s' (pre-tanh). Optionally keeps activations / masked GELU derivatives for the backward.
template <int NH, bool KEEP>
__device__ __forceinline__ void mlp_forward(const BcnfLayout& L, const float* __restrict__ R, float x, float hp,
                                            uint32_t bits, bool drop, float& T, float& Sp,
                                            float* act, float* gd) {
  float w[16];
  ld16(w, R + L.rf_w1);
  float pre = rot16(x, w, R[L.rf_b1] + hp);
  float m = drop ? ((bits & 1u) ? L.keep_scale : 0.f) : 1.f;
  float a = gelu_f(pre) * m;
  if (KEEP) { act[0] = a; gd[0] = gelu_grad(pre) * m; }
#pragma unroll
  for (int l = 2; l <= NH; ++l) {
    const float* Rl = R + L.rf_hid + 17 * (l - 2);
    ld16(w, Rl);
    pre = rot16(a, w, Rl[16]);
    m = drop ? (((bits >> (l - 1)) & 1u) ? L.keep_scale : 0.f) : 1.f;
    a = gelu_f(pre) * m;
    if (KEEP) { act[l - 1] = a; gd[l - 1] = gelu_grad(pre) * m; }
  }
  float wt[16], ws[16];
  ld16(wt, R + L.rf_t);
  ld16(ws, R + L.rf_s);
  T = R[L.rf_t + 16];
  Sp = R[L.rf_s + 16];
  rot16x2(a, wt, T, a, ws, Sp);
}

// ------------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------------
template <int NH, bool DROP, bool SAVE>
__global__ __launch_bounds__(BCNF_WG) void k_forward(BcnfLayout L, const float* __restrict__ pk,
                                                     const float* __restrict__ y, const float* __restrict__ h,
                                                     long long B, float* __restrict__ z, float* __restrict__ ldj_out,
                                                     float* __restrict__ logp, const uint64_t* __restrict__ rng,
                                                     float* __restrict__ ysave, uint32_t* __restrict__ msave) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int RFL = 16 * L.RF;
  float* rec = smem;                    // [2][16*RF]
  float* hpb = rec + 2 * RFL;           // [2][4][256]
  float* ht = hpb + 2 * 1024;           // [16][Cp+1]
  const int tid = threadIdx.x, j = tid & 15, s = tid >> 4;
  const long long b = (long long)blockIdx.x * 16 + s;
  const bool valid = b < B;
  const long long bc = valid ? b : B - 1;
  const int D = L.D, Da = L.Da, Db = L.Db, nb = L.nb;

  stage_features(L, h, nullptr, B, ht);
  {
    Stage st;
    st.load(pk + L.pf_off, RFL);
    st.store(rec, RFL);
  }
  __syncthreads();
  hp_quarter(L, pk + L.w1t_off, ht, hpb, 0);
  __syncthreads();

  float ya = (j < Da) ? y[bc * D + j] : 0.f;
  float yb = (j < Db) ? y[bc * D + Da + j] : 0.f;
  float ldj = 0.f;
  uint64_t seed = 0, off = 0;
  if (DROP) { seed = rng[0]; off = rng[1]; }
  uint32_t mword = 0;

  for (int k = 0; k < nb; ++k) {
    const int cur = k & 1;
    Stage st;
    if (k + 1 < nb) {
      st.load(pk + L.pf_off + (long long)(k + 1) * RFL, RFL);
      hp_quarter(L, pk + L.w1t_off, ht, hpb + (cur ^ 1) * 1024, k + 1);
    }
    const float* R = rec + cur * RFL + j * L.RF;
    if (SAVE && valid) {
      float* ys = ysave + ((long long)k * B + b) * 32;
      ys[j] = ya;
      ys[16 + j] = yb;
    }
    const floatx4 an = *reinterpret_cast<const floatx4*>(R);
    const float xa = fmaf(an.x, ya, an.y);           // ActNorm (cnf.py:349)
    const float xb = fmaf(an.z, yb, an.w);
    uint32_t bits = 0xffu;
    if (DROP) bits = dropout_bits(L, seed, off, b, k, j, 0u);
    if (SAVE && DROP) {
      mword |= bits << (8 * (k & 3));
      if ((k & 3) == 3 || k == nb - 1) {
        if (valid) msave[((long long)(k >> 2) * B + b) * 16 + j] = mword;
        mword = 0;
      }
    }
    float T, Sp;
    mlp_forward<NH, false>(L, R, xa, hp_sum(hpb + cur * 1024, s, j), bits, DROP, T, Sp, nullptr, nullptr);
    const float S = tanhf(Sp);                        // cnf.py:107
    const float zb = fmaf(expf(S), xb, T);            // cnf.py:179
    ldj += S;                                          // cnf.py:190
    if (k < nb - 1) {                                  // orthonormal mix y @ Q (cnf.py:335)
      float q0[16], q1[16];
      float na = 0.f, nbv = 0.f;
      ld16(q0, R + L.rf_q);
      ld16(q1, R + L.rf_q + 32);
      rot16x2(xa, q0, na, xa, q1, nbv);
      ld16(q0, R + L.rf_q + 16);
      ld16(q1, R + L.rf_q + 48);
      rot16x2(zb, q0, na, zb, q1, nbv);
      ya = na;
      yb = nbv;
    } else {
      ya = xa;
      yb = zb;
    }
    if (k + 1 < nb) st.store(rec + (cur ^ 1) * RFL, RFL);
    __syncthreads();
  }
  const float ltot = row_sum16(ldj) + pk[L.ldc_off];
  if (valid) {
    if (j < Da) z[b * D + j] = ya;
    if (j < Db) z[b * D + Da + j] = yb;
    if (j == 0 && ldj_out) ldj_out[b] = ltot;
  }
  if (logp) {
    const float q2 = row_sum16(ya * ya + yb * yb);
    if (valid && j == 0) logp[b] = -(0.5f * q2 - ltot) - 0.5f * (float)D * 1.8378770664093454836f;
  }
}

// ------------------------------------------------------------------------------------------------
// Inverse
// ------------------------------------------------------------------------------------------------
template <int NH, bool DROP>
__global__ __launch_bounds__(BCNF_WG) void k_inverse(BcnfLayout L, const float* __restrict__ pk,
                                                     const float* __restrict__ zin, const float* __restrict__ h,
                                                     const int64_t* __restrict__ cond_index, long long N,
                                                     float* __restrict__ yout, const uint64_t* __restrict__ rng) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int RFL = 16 * L.RF;
  float* rec = smem;
  float* hpb = rec + 2 * RFL;
  float* ht = hpb + 2 * 1024;
  const int tid = threadIdx.x, j = tid & 15, s = tid >> 4;
  const long long b = (long long)blockIdx.x * 16 + s;
  const bool valid = b < N;
  const long long bc = valid ? b : N - 1;
  const int D = L.D, Da = L.Da, Db = L.Db, nb = L.nb;

  stage_features(L, h, cond_index, N, ht);
  const int klast = nb - 1;
  {
    Stage st;
    st.load(pk + L.pi_off + (long long)klast * RFL, RFL);
    st.store(rec + (klast & 1) * RFL, RFL);
  }
  __syncthreads();
  hp_quarter(L, pk + L.w1t_off, ht, hpb + (klast & 1) * 1024, klast);
  __syncthreads();

  float ya = (j < Da) ? zin[bc * D + j] : 0.f;
  float yb = (j < Db) ? zin[bc * D + Da + j] : 0.f;
  uint64_t seed = 0, off = 0;
  if (DROP) { seed = rng[0]; off = rng[1]; }

  for (int k = klast; k >= 0; --k) {
    const int cur = k & 1;
    Stage st;
    if (k >= 1) {
      st.load(pk + L.pi_off + (long long)(k - 1) * RFL, RFL);
      hp_quarter(L, pk + L.w1t_off, ht, hpb + (cur ^ 1) * 1024, k - 1);
    }
    const float* R = rec + cur * RFL + j * L.RF;
    float za, zb;
    if (k < nb - 1) {                                  // z @ Q^T (cnf.py:339)
      float q0[16], q1[16];
      za = 0.f;
      zb = 0.f;
      ld16(q0, R + L.rf_q);
      ld16(q1, R + L.rf_q + 32);
      rot16x2(ya, q0, za, ya, q1, zb);
      ld16(q0, R + L.rf_q + 16);
      ld16(q1, R + L.rf_q + 48);
      rot16x2(yb, q0, za, yb, q1, zb);
    } else {
      za = ya;
      zb = yb;
    }
    uint32_t bits = 0xffu;
    if (DROP) bits = dropout_bits(L, seed, off, b, k, j, 0x40000000u);
    float T, Sp;
    mlp_forward<NH, false>(L, R, za, hp_sum(hpb + cur * 1024, s, j), bits, DROP, T, Sp, nullptr, nullptr);
    const float S = tanhf(Sp);
    yb = (zb - T) * expf(-S);                          // cnf.py:205
    ya = za;
    const floatx4 an = *reinterpret_cast<const floatx4*>(R);   // ActNorm inverse (cnf.py:353-354)
    if (L.act_norm && k < nb - 1) {
      ya = (j < Da) ? (ya - an.y) / an.x : 0.f;
      yb = (j < Db) ? (yb - an.w) / an.z : 0.f;
    }
    if (k >= 1) st.store(rec + (cur ^ 1) * RFL, RFL);
    __syncthreads();
  }
  if (valid) {
    if (j < Da) yout[b * D + j] = ya;
    if (j < Db) yout[b * D + Da + j] = yb;
  }
}

// ------------------------------------------------------------------------------------------------
// Backward
// ------------------------------------------------------------------------------------------------
struct BwdTiles {   // tile indices inside one tile buffer
  int NH;
  __device__ __forceinline__ int D(int l) const { return l - 1; }          // l = 1..NH
  __device__ __forceinline__ int DT() const { return NH; }
  __device__ __forceinline__ int DS() const { return NH + 1; }
  __device__ __forceinline__ int A(int l) const { return NH + 2 + l; }     // l = 0..NH
  __device__ __forceinline__ int PA() const { return 2 * NH + 3; }
  __device__ __forceinline__ int GA() const { return 2 * NH + 4; }
  __device__ __forceinline__ int PB() const { return 2 * NH + 5; }
  __device__ __forceinline__ int GB() const { return 2 * NH + 6; }
  __device__ __forceinline__ int count() const { return 2 * NH + NT_EXTRA; }
};

// dW-style chain: out[j][n] = sum_s Dt[s][j] * Bt[s][n] over the 16 samples; B may be ones.
__device__ __forceinline__ floatx4 chain_tt(const float* __restrict__ Dt, const float* __restrict__ Bt, int q, int r) {
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int sidx = (4 * t + q) * BCNF_TSTRIDE + r;
    acc = mfma4(Dt[sidx], Bt ? Bt[sidx] : 1.0f, acc);
  }
  return acc;
}

template <int NH>
__device__ __forceinline__ void bwd_mfma_phase(const BcnfLayout& L, const float* __restrict__ pk, const float* __restrict__ T,
                                               const float* __restrict__ ht, float* __restrict__ slab, int m,
                                               floatx4* dhacc) {
  const BwdTiles TI{NH};
  const int wave = threadIdx.x >> 6, l64 = threadIdx.x & 63, q = l64 >> 4, r = l64 & 15;
  const int NC16 = L.Cp >> 4;
  const int cb = coupling_base(L, m);
  const bool has_an = L.act_norm && m < L.nb - 1;
  const int n_chains = 2 * NH + 8 + NC16;
  for (int c = wave; c < n_chains; c += 4) {
    if (c < NH + 2) {                      // weight gradients of Linear l (or output t / s rows)
      const int l = (c < NH) ? c + 1 : NH + 1;
      const int dtile = (c < NH) ? TI.D(l) : (c == NH ? TI.DT() : TI.DS());
      const int atile = (c < NH) ? TI.A(l - 1) : TI.A(NH);
      const floatx4 acc = chain_tt(T + dtile * TILE, T + atile * TILE, q, r);
      const int in_eff = (l == 1) ? L.Da : L.H[l - 1];
      const int out_l = (c < NH) ? L.H[l] : L.Db;
      const int row0 = (c == NH + 1) ? L.Db : 0;
      if (r < in_eff) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int jr = 4 * q + i;
          if (jr < out_l) slab[cb + L.lin_w[l] + (row0 + jr) * L.lin_in[l] + r] = acc[i];
        }
      }
    } else if (c < 2 * NH + 4) {           // bias gradients
      const int cc = c - (NH + 2);
      const int l = (cc < NH) ? cc + 1 : NH + 1;
      const int dtile = (cc < NH) ? TI.D(l) : (cc == NH ? TI.DT() : TI.DS());
      const floatx4 acc = chain_tt(T + dtile * TILE, nullptr, q, r);
      const int out_l = (cc < NH) ? L.H[l] : L.Db;
      const int row0 = (cc == NH + 1) ? L.Db : 0;
      if (r == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int jr = 4 * q + i;
          if (jr < out_l) slab[cb + L.lin_b[l] + row0 + jr] = acc[i];
        }
      }
    } else if (c < 2 * NH + 8) {           // ActNorm scale / bias
      if (!has_an) continue;
      const int a = c - (2 * NH + 4);      // 0: scale_a 1: bias_a 2: scale_b 3: bias_b
      const int tile = (a == 0) ? TI.PA() : (a == 1 ? TI.GA() : (a == 2 ? TI.PB() : TI.GB()));
      const floatx4 acc = chain_tt(T + tile * TILE, nullptr, q, r);
      const int cnt = (a < 2) ? L.Da : L.Db;
      const int base = m * L.blk_stride + ((a & 1) ? L.D : 0) + ((a < 2) ? 0 : L.Da);
      if (r == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int jr = 4 * q + i;
          if (jr < cnt) slab[base + jr] = acc[i];
        }
      }
    } else {                               // W1 condition part: dW1h[j][c] = sum_s D1[s][j] h[s][c]
      const int n = c - (2 * NH + 8);
      const float* Dt = T + TI.D(1) * TILE;
      const int hs = L.Cp + 1;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc = mfma4(Dt[(4 * t + q) * BCNF_TSTRIDE + r], ht[(4 * t + q) * hs + 16 * n + r], acc);
      const int col = 16 * n + r;
      if (col < L.C) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int jr = 4 * q + i;
          if (jr < L.H[1]) slab[cb + L.lin_w[1] + jr * L.lin_in[1] + L.Da + col] = acc[i];
        }
      }
    }
  }
  // dh[s][c] += sum_j D1[s][j] W1h_m[j][c]   (wave w owns column tiles n = w, w+4, ...)
  const float* D1 = T + TI.D(1) * TILE;
  const float* w1h = pk + L.w1h_off + (long long)m * 16 * L.Cp;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int n = wave + 4 * u;
    if (n < NC16) {
      floatx4 acc = dhacc[u];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc = mfma4(D1[r * BCNF_TSTRIDE + 4 * t + q], w1h[(4 * t + q) * L.Cp + 16 * n + r], acc);
      dhacc[u] = acc;
    }
  }
}

template <int NH>
__global__ __launch_bounds__(BCNF_WG) void k_backward(BcnfLayout L, const float* __restrict__ pk,
                                                      const float* __restrict__ h, const float* __restrict__ dz,
                                                      const float* __restrict__ dldj, long long B,
                                                      const float* __restrict__ ysave, const uint32_t* __restrict__ msave,
                                                      float* __restrict__ dy, float* __restrict__ dh,
                                                      float* __restrict__ slab_all, long long slab_stride) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const BwdTiles TI{NH};
  const int RFL = 16 * L.RF, RBL = 16 * L.RB;
  const int NT = TI.count();
  float* recF = smem;                   // [2][16*RF]
  float* recB = recF + 2 * RFL;         // [2][16*RB]
  float* hpb = recB + 2 * RBL;          // [2][4][256]
  float* tiles = hpb + 2 * 1024;        // [2][NT][272]
  float* ht = tiles + 2 * NT * TILE;    // [16][Cp+1]
  const int tid = threadIdx.x, j = tid & 15, s = tid >> 4;
  const int wave = tid >> 6, l64 = tid & 63, q = l64 >> 4, r = l64 & 15;
  const long long b = (long long)blockIdx.x * 16 + s;
  const bool valid = b < B;
  const long long bc = valid ? b : B - 1;
  const int D = L.D, Da = L.Da, Db = L.Db, nb = L.nb;
  float* slab = slab_all + (long long)blockIdx.x * slab_stride;
  const bool drop = msave != nullptr;

  stage_features(L, h, nullptr, B, ht);
  {
    Stage st;
    const int kl = nb - 1;
    st.load(pk + L.pf_off + (long long)kl * RFL, RFL);
    st.store(recF + (kl & 1) * RFL, RFL);
    st.load(pk + L.pb_off + (long long)kl * RBL, RBL);
    st.store(recB + (kl & 1) * RBL, RBL);
  }
  __syncthreads();
  hp_quarter(L, pk + L.w1t_off, ht, hpb + ((nb - 1) & 1) * 1024, nb - 1);
  __syncthreads();

  float gya = 0.f, gyb = 0.f, dl = 0.f;
  if (valid) {
    if (dz) {
      gya = (j < Da) ? dz[b * D + j] : 0.f;
      gyb = (j < Db) ? dz[b * D + Da + j] : 0.f;
    }
    if (dldj) dl = dldj[b];
  }
  floatx4 dhacc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) dhacc[u] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int k = nb - 1; k >= 0; --k) {
    const int cur = k & 1;
    // (a) prefetch
    const float* ys = ysave + ((long long)k * B + bc) * 32;
    const float ya = ys[j], yb = ys[16 + j];
    uint32_t mword = 0xffffffffu;
    if (drop) mword = msave[((long long)(k >> 2) * B + bc) * 16 + j];
    Stage stF, stB;
    if (k >= 1) {
      stF.load(pk + L.pf_off + (long long)(k - 1) * RFL, RFL);
    }
    // (b) MFMA phase: gradients of block k+1 from its tiles, HP of block k-1
    if (k + 1 < nb) bwd_mfma_phase<NH>(L, pk, tiles + ((k + 1) & 1) * NT * TILE, ht, slab, k + 1, dhacc);
    if (k >= 1) {
      stB.load(pk + L.pb_off + (long long)(k - 1) * RBL, RBL);
      hp_quarter(L, pk + L.w1t_off, ht, hpb + (cur ^ 1) * 1024, k - 1);
    }
    // (c) VALU phase for block k
    const float* RF_ = recF + cur * RFL + j * L.RF;
    const float* RB_ = recB + cur * RBL + j * L.RB;
    float* Tt = tiles + cur * NT * TILE;
    const int tix = s * BCNF_TSTRIDE + j;
    const floatx4 an = *reinterpret_cast<const floatx4*>(RF_);
    const float xa = fmaf(an.x, ya, an.y);
    const float xb = fmaf(an.z, yb, an.w);
    const uint32_t bits = (mword >> (8 * (k & 3))) & 0xffu;
    float act[NH], gd[NH];
    float T, Sp;
    mlp_forward<NH, true>(L, RF_, xa, hp_sum(hpb + cur * 1024, s, j), bits, drop, T, Sp, act, gd);
    const float S = tanhf(Sp);
    const float e = expf(S);
    float gza, gzb;
    if (k < nb - 1) {                                  // grad through y @ Q: g @ Q^T
      float q0[16], q1[16];
      gza = 0.f;
      gzb = 0.f;
      ld16(q0, RB_ + L.rb_qt);
      ld16(q1, RB_ + L.rb_qt + 32);
      rot16x2(gya, q0, gza, gya, q1, gzb);
      ld16(q0, RB_ + L.rb_qt + 16);
      ld16(q1, RB_ + L.rb_qt + 48);
      rot16x2(gyb, q0, gza, gyb, q1, gzb);
    } else {
      gza = gya;
      gzb = gyb;
    }
    const float dT = gzb;                              // z_b = exp(s) y_b + t
    const float dS = (j < Db) ? fmaf(gzb * e, xb, dl) : 0.f;
    const float dSp = dS * (1.f - S * S);
    const float dxb = gzb * e;
    Tt[TI.DT() * TILE + tix] = dT;
    Tt[TI.DS() * TILE + tix] = dSp;
    Tt[TI.A(NH) * TILE + tix] = act[NH - 1];
    float da, da2;
    {
      float w0[16], w1[16];
      da = 0.f;
      da2 = 0.f;
      ld16(w0, RB_ + L.rb_tt);
      ld16(w1, RB_ + L.rb_st);
      rot16x2(dT, w0, da, dSp, w1, da2);
    }
    da += da2;
#pragma unroll
    for (int l = NH; l >= 2; --l) {
      const float dpre = da * gd[l - 1];
      Tt[TI.D(l) * TILE + tix] = dpre;
      Tt[TI.A(l - 1) * TILE + tix] = act[l - 2];
      float w[16];
      ld16(w, RB_ + L.rb_hid + 16 * (l - 2));
      da = rot16(dpre, w, 0.f);
    }
    const float dpre1 = da * gd[0];
    Tt[TI.D(1) * TILE + tix] = dpre1;
    Tt[TI.A(0) * TILE + tix] = xa;
    float dxa;
    {
      float w[16];
      ld16(w, RB_ + L.rb_w1t);
      dxa = rot16(dpre1, w, gza);
    }
    if (L.act_norm && k < nb - 1) {
      const float inv_a = (j < Da) ? 1.f / an.x : 0.f;
      const float inv_b = (j < Db) ? 1.f / an.z : 0.f;
      Tt[TI.PA() * TILE + tix] = fmaf(dxa, ya, dl * inv_a);
      Tt[TI.GA() * TILE + tix] = dxa;
      Tt[TI.PB() * TILE + tix] = fmaf(dxb, yb, dl * inv_b);
      Tt[TI.GB() * TILE + tix] = dxb;
    }
    gya = an.x * dxa;
    gyb = an.z * dxb;
    // (d) commit prefetched records
    if (k >= 1) {
      stF.store(recF + (cur ^ 1) * RFL, RFL);
      stB.store(recB + (cur ^ 1) * RBL, RBL);
    }
    __syncthreads();
  }
  bwd_mfma_phase<NH>(L, pk, tiles, ht, slab, 0, dhacc);
  if (dy && valid) {
    if (j < Da) dy[b * D + j] = gya;
    if (j < Db) dy[b * D + Da + j] = gyb;
  }
  if (dh) {
    const int NC16 = L.Cp >> 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = wave + 4 * u;
      const int col = 16 * n + r;
      if (n < NC16 && col < L.C) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long long bb = (long long)blockIdx.x * 16 + 4 * q + i;
          if (bb < B) dh[bb * L.C + col] = dhacc[u][i];
        }
      }
    }
  }
}

// Deterministic sum of the per-workgroup gradient slabs (fixed order over workgroups).
__global__ __launch_bounds__(BCNF_WG) void k_reduce(const float* __restrict__ slab, long long stride, int nwg,
                                                    long long P, float* __restrict__ out) {
  const long long p = ((long long)blockIdx.x * BCNF_WG + threadIdx.x) * 4;
  if (p >= P) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int w = 0;
  for (; w + 4 <= nwg; w += 4) {
    const float4 v0 = *reinterpret_cast<const float4*>(slab + (long long)(w + 0) * stride + p);
    const float4 v1 = *reinterpret_cast<const float4*>(slab + (long long)(w + 1) * stride + p);
    const float4 v2 = *reinterpret_cast<const float4*>(slab + (long long)(w + 2) * stride + p);
    const float4 v3 = *reinterpret_cast<const float4*>(slab + (long long)(w + 3) * stride + p);
    acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
    acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
    acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
    acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
  }
  for (; w < nwg; ++w) {
    const float4 v = *reinterpret_cast<const float4*>(slab + (long long)w * stride + p);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (p + 3 < P) {
    *reinterpret_cast<float4*>(out + p) = acc;
  } else {
    out[p] = acc.x;
    if (p + 1 < P) out[p + 1] = acc.y;
    if (p + 2 < P) out[p + 2] = acc.z;
  }
}

// ------------------------------------------------------------------------------------------------
// Launch helpers
// ------------------------------------------------------------------------------------------------
thread_local int g_last_hip = 0;

int check_launch() {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return BCNF_ERR_HIP;
  }
  return BCNF_OK;
}

size_t fwd_lds_bytes(const BcnfLayout& L) {
  return sizeof(float) * (size_t)(2 * 16 * L.RF + 2 * 1024 + 16 * (L.Cp + 1));
}
size_t bwd_lds_bytes(const BcnfLayout& L) {
  const int NT = 2 * L.NH + NT_EXTRA;
  return sizeof(float) * (size_t)(2 * 16 * L.RF + 2 * 16 * L.RB + 2 * 1024 + 2 * NT * TILE + 16 * (L.Cp + 1));
}

// Raise a kernel's dynamic-LDS limit once (cached per kernel; safe to call under stream capture
// after the first eager call has set it).
std::mutex g_attr_mu;
const void* g_attr_fn[256];
size_t g_attr_lds[256];
int g_attr_n = 0;

template <typename K>
int launch_lds(K kernel, size_t lds) {
  if (lds > 160 * 1024) return BCNF_ERR_UNSUPPORTED;
  const void* fn = reinterpret_cast<const void*>(kernel);
  std::lock_guard<std::mutex> lk(g_attr_mu);
  for (int i = 0; i < g_attr_n; ++i)
    if (g_attr_fn[i] == fn && g_attr_lds[i] >= lds) return BCNF_OK;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return BCNF_ERR_HIP;
  }
  int slot = -1;
  for (int i = 0; i < g_attr_n; ++i)
    if (g_attr_fn[i] == fn) slot = i;
  if (slot < 0 && g_attr_n < 256) slot = g_attr_n++;
  if (slot >= 0) {
    g_attr_fn[slot] = fn;
    g_attr_lds[slot] = lds;
  }
  return BCNF_OK;
}

template <int NH>
int fwd_dispatch(const BcnfLayout& L, const float* pk, const float* y, const float* h, long long B, float* z,
                 float* ldj, float* logp, bool drop, const uint64_t* rng, float* ysave, uint32_t* msave,
                 hipStream_t st) {
  const dim3 grid((unsigned)((B + 15) / 16));
  const size_t lds = fwd_lds_bytes(L);
  const bool save = ysave != nullptr;
  int rc;
#define BCNF_FWD(DR, SV)                                                                                    \
  rc = launch_lds(k_forward<NH, DR, SV>, lds);                                                    \
  if (rc) return rc;                                                                                        \
  hipLaunchKernelGGL((k_forward<NH, DR, SV>), grid, dim3(BCNF_WG), lds, st, L, pk, y, h, B, z, ldj, logp,   \
                     rng, ysave, msave);
  if (drop) {
    if (save) { BCNF_FWD(true, true) } else { BCNF_FWD(true, false) }
  } else {
    if (save) { BCNF_FWD(false, true) } else { BCNF_FWD(false, false) }
  }
#undef BCNF_FWD
  return check_launch();
}

template <int NH>
int inv_dispatch(const BcnfLayout& L, const float* pk, const float* zin, const float* h, const int64_t* ci,
                 long long N, float* y, bool drop, const uint64_t* rng, hipStream_t st) {
  const dim3 grid((unsigned)((N + 15) / 16));
  const size_t lds = fwd_lds_bytes(L);
  int rc;
  if (drop) {
    rc = launch_lds(k_inverse<NH, true>, lds);
    if (rc) return rc;
    hipLaunchKernelGGL((k_inverse<NH, true>), grid, dim3(BCNF_WG), lds, st, L, pk, zin, h, ci, N, y, rng);
  } else {
    rc = launch_lds(k_inverse<NH, false>, lds);
    if (rc) return rc;
    hipLaunchKernelGGL((k_inverse<NH, false>), grid, dim3(BCNF_WG), lds, st, L, pk, zin, h, ci, N, y, rng);
  }
  return check_launch();
}

template <int NH>
int bwd_dispatch(const BcnfLayout& L, const float* pk, const float* h, const float* dz, const float* dldj,
                 long long B, const float* ysave, const uint32_t* msave, float* dy, float* dh, float* slab,
                 long long stride, hipStream_t st) {
  const dim3 grid((unsigned)((B + 15) / 16));
  const size_t lds = bwd_lds_bytes(L);
  const int rc = launch_lds(k_backward<NH>, lds);
  if (rc) return rc;
  hipLaunchKernelGGL((k_backward<NH>), grid, dim3(BCNF_WG), lds, st, L, pk, h, dz, dldj, B, ysave, msave, dy,
                     dh, slab, stride);
  return check_launch();
}

long long slab_stride_of(const BcnfLayout& L) { return ((long long)L.n_trainable + 3) & ~3LL; }

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

int bcnf_stack_supported(const BcnfStackDesc* desc) {
  BcnfLayout L;
  if (make_layout(desc, &L) != BCNF_OK) return 0;
  return layout_supported(L, desc) ? 1 : 0;
}

int bcnf_param_count(const BcnfStackDesc* desc, int64_t* n_trainable, int64_t* n_frozen) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (n_trainable) *n_trainable = L.n_trainable;
  if (n_frozen) *n_frozen = (int64_t)(L.nb - 1) * L.D * L.D;
  return BCNF_OK;
}

int bcnf_packed_bytes(const BcnfStackDesc* desc, int64_t* bytes) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!bytes) return BCNF_ERR_ARG;
  *bytes = (int64_t)L.total * (int64_t)sizeof(float);
  return BCNF_OK;
}

int bcnf_workspace_bytes(const BcnfStackDesc* desc, int64_t batch, int32_t training, int64_t* bytes) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!bytes || batch < 0) return BCNF_ERR_ARG;
  int64_t n = (int64_t)L.nb * batch * 32 * 4;
  if (training && L.p > 0.f) n += (int64_t)((L.nb + 3) / 4) * batch * 16 * 4;
  *bytes = n;
  return BCNF_OK;
}

int bcnf_slab_bytes(const BcnfStackDesc* desc, int64_t batch, int64_t* bytes) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!bytes || batch < 0) return BCNF_ERR_ARG;
  *bytes = (int64_t)((batch + 15) / 16) * slab_stride_of(L) * 4;
  return BCNF_OK;
}

int bcnf_pack_params(const BcnfStackDesc* desc, const float* params, const float* qmats, void* packed, void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (!params || !packed || (L.nb > 1 && !qmats)) return BCNF_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_pack, dim3(512), dim3(BCNF_WG), 0, st, L, params, qmats, (float*)packed);
  if ((rc = check_launch())) return rc;
  hipLaunchKernelGGL(k_ldc, dim3(1), dim3(BCNF_WG), 0, st, L, params, (float*)packed);
  return check_launch();
}

int bcnf_stack_forward(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h, int64_t batch,
                       float* z, float* ldj, float* log_prob, int32_t training, const uint64_t* rng_state,
                       void* workspace, void* stream) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (batch == 0) return BCNF_OK;
  if (batch < 0 || !packed || !y || !h || !z) return BCNF_ERR_ARG;
  const bool drop = training && L.p > 0.f;
  if (drop && !rng_state) return BCNF_ERR_ARG;
  float* ysave = nullptr;
  uint32_t* msave = nullptr;
  if (workspace) {
    ysave = (float*)workspace;
    if (drop) msave = (uint32_t*)(ysave + (long long)L.nb * batch * 32);
  }
  const float* pk = (const float*)packed;
  hipStream_t st = (hipStream_t)stream;
  switch (L.NH) {
#define BCNF_CASE(N) case N: return fwd_dispatch<N>(L, pk, y, h, batch, z, ldj, log_prob, drop, rng_state, ysave, msave, st);
    BCNF_CASE(1) BCNF_CASE(2) BCNF_CASE(3) BCNF_CASE(4) BCNF_CASE(5) BCNF_CASE(6) BCNF_CASE(7) BCNF_CASE(8)
#undef BCNF_CASE
    default: return BCNF_ERR_UNSUPPORTED;
  }
}

int bcnf_stack_backward(const BcnfStackDesc* desc, const void* packed, const float* h, const float* dz,
                        const float* dldj, int64_t batch, int32_t training, const void* workspace, float* dy,
                        float* dh, float* dparams, void* slab, void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (batch < 0 || !packed || !h || !workspace || !dparams || !slab) return BCNF_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (batch == 0) {
    if (hipMemsetAsync(dparams, 0, sizeof(float) * (size_t)L.n_trainable, st) != hipSuccess) return BCNF_ERR_HIP;
    return BCNF_OK;
  }
  // `training` must match the forward call that filled the workspace: it says whether dropout masks
  // were saved behind the block inputs.
  const float* ysave = (const float*)workspace;
  const uint32_t* msave = nullptr;
  if (training && L.p > 0.f) msave = (const uint32_t*)(ysave + (long long)L.nb * batch * 32);
  const float* pk = (const float*)packed;
  const long long stride = slab_stride_of(L);
  switch (L.NH) {
#define BCNF_CASE(N) case N: rc = bwd_dispatch<N>(L, pk, h, dz, dldj, batch, ysave, msave, dy, dh, (float*)slab, stride, st); break;
    BCNF_CASE(1) BCNF_CASE(2) BCNF_CASE(3) BCNF_CASE(4) BCNF_CASE(5) BCNF_CASE(6) BCNF_CASE(7) BCNF_CASE(8)
#undef BCNF_CASE
    default: return BCNF_ERR_UNSUPPORTED;
  }
  if (rc) return rc;
  const long long P = L.n_trainable;
  const unsigned nblk = (unsigned)((P / 4 + BCNF_WG) / BCNF_WG);
  hipLaunchKernelGGL(k_reduce, dim3(nblk), dim3(BCNF_WG), 0, st, (const float*)slab, stride,
                     (int)((batch + 15) / 16), P, dparams);
  return check_launch();
}

int bcnf_stack_inverse(const BcnfStackDesc* desc, const void* packed, const float* z, const float* h,
                       const int64_t* cond_index, int64_t n_rows, float* y, int32_t training,
                       const uint64_t* rng_state, void* stream) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (n_rows == 0) return BCNF_OK;
  if (n_rows < 0 || !packed || !z || !h || !y) return BCNF_ERR_ARG;
  const bool drop = training && L.p > 0.f;
  if (drop && !rng_state) return BCNF_ERR_ARG;
  const float* pk = (const float*)packed;
  hipStream_t st = (hipStream_t)stream;
  switch (L.NH) {
#define BCNF_CASE(N) case N: return inv_dispatch<N>(L, pk, z, h, cond_index, n_rows, y, drop, rng_state, st);
    BCNF_CASE(1) BCNF_CASE(2) BCNF_CASE(3) BCNF_CASE(4) BCNF_CASE(5) BCNF_CASE(6) BCNF_CASE(7) BCNF_CASE(8)
#undef BCNF_CASE
    default: return BCNF_ERR_UNSUPPORTED;
  }
}

const char* bcnf_status_string(int status) {
  switch (status) {
    case BCNF_OK: return "ok";
    case BCNF_ERR_ARG: return "invalid argument";
    case BCNF_ERR_UNSUPPORTED: return "unsupported stack shape for the fused kernel family";
    case BCNF_ERR_HIP: return "HIP launch error";
    default: return "unknown status";
  }
}

int bcnf_last_hip_error(void) { return g_last_hip; }

}  // extern "C"
