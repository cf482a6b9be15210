// Wide-MLP family of the CondRealNVP_v2 coupling stack on gfx950 (CDNA4): trajectory_FC_large /
// trajectory_LSTM_large shapes (D = 19, C = 1360, nested_sizes = [526] * 5, 26 blocks), i.e. every stack whose
// nested MLP is too wide for the register-resident small family of bcnf_stack.hip.
//
// Reference (psaegert/bcnf, src/bcnf/models/cnf.py): ConditionalNestedNeuralNetwork (:49-107),
// ConditionalAffineCouplingLayer.forward / .inverse (:165-213), OrthonormalTransformation (:312-339), ActNorm
// (:342-354), CondRealNVP_v2.forward / .inverse layer loops (:467-508); autograd backward of all of it.
//
// Shape of the work: per block, the nested MLP is Linear(Da + C -> H), (GELU, Dropout, Linear(H -> H)) x (NH-1),
// GELU, Dropout, Linear(H -> 2 Db). At H = 526 the H x H layers are MFMA-bound GEMMs (fp32 MFMA,
// v_mfma_f32_32x32x2_f32, exact f32, the only fp32 matrix path on gfx950). The kernels:
//
//   k_wgemm<...>   LDS-tiled fp32-MFMA GEMM, three operand layouts (NT forward, NN dX, TN dW), group index in
//                  blockIdx.z, fused epilogues: bias + exact-erf GELU + Philox dropout (writing the activation
//                  and its derivative factor G = mask * GELU'(pre) / (1 - p)), dZ = acc * G, and Linear-gradient
//                  stores straight into the canonical flat gradient (weight rows + bias via a ones column).
//   k_wlink_*      one wavefront per two samples: the end of block k (last Linear, tanh, exp-affine coupling,
//                  log|det J|, orthonormal mix) fused with the start of block k+1 (ActNorm, Linear-1 y-part from
//                  the hoisted condition projection, GELU, dropout); and the mirror image for the backward and
//                  for the inverse.
//   hoisted condition projection: P = h W0h_all^T for ALL blocks in one GEMM (h does not change between
//   blocks); its transposes give dh = dZ0_all W0h_all and dW0h = dZ0_all^T h, again one GEMM each.
//
// Activation rows are padded to HP = round_up(H + 1, 4) floats: column H holds 1.0 (so the dW GEMM emits the
// bias gradient as one more output column) and the padded weight copies are zero beyond H, so every GEMM runs
// with K = HP and no K masks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "bcnf_amd.h"
#include <cstdlib>
#include "bcnf_device.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int WWG = 256;      // threads per workgroup of every wide kernel
constexpr int DM = 32;        // max D of the wide family (register arrays of the link kernels)

__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }
inline long long pad4l(long long x) { return (x + 3) & ~3LL; }

// Virtual blocks: a two_way coupling (cnf.py:176-186) is two half-couplings in sequence -- side a (nn_a: input
// the first Da coordinates, transforms the last Db) then side b (nn_b: input the last Db, transforms the first Da)
// -- so the stack is nv = nb * S half-couplings (S = 2 for two_way, else 1), each with its own nested MLP. Virtual
// block v belongs to real block v / S and has side v % S; ActNorm sits before a block's first half, the orthonormal
// mix after its last half.
struct WideLayout {
  int D, Da, Db, C, Cp, H, NH, nb, an, S, nv;
  int HP, UP, OP, XP, SP, AP;   // row strides: activations, [u_in | 1], dO, block inputs, tanh(s), ActNorm partials
  int nin[2], nout[2], ioff[2], toff[2], in0[2];   // per side: MLP input width / transformed width / their offsets
  long long mlp[2];             // floats of nn_a / nn_b
  long long lin_w[2][BCNF_MAX_HIDDEN + 1], lin_b[2][BCNF_MAX_HIDDEN + 1];   // Linear offsets inside nn_a / nn_b
  long long blk_stride;         // canonical floats per (ActNorm + coupling) block
  long long n_trainable;
  int WY, WL;                   // rows per virtual block of the W0y^T and last-Linear copies (max over sides)
  float p, keep_scale;
  uint32_t thresh;              // drop if philox u32 < thresh
  // packed buffer (floats)
  long long pk_w0h;             // [nv * HP][Cp]    row v*HP + n = W0_v[n][nin_v + c], rows n >= H and c >= C zero
  long long pk_hid;             // [nv][NH-1][HP][HP]  W_l (l = 1..NH-1), zero beyond H
  long long pk_hidT;            // [nv][NH-1][HP][HP]  W_l^T (the backward chain's K-contiguous operand)
  long long pk_w0y;             // [nv][WY][HP]     W0_v[n][j] transposed
  long long pk_wl;              // [nv][WL][HP]     last Linear, zero beyond H
  long long pk_q;               // [nb-1][D][D]
  long long pk_ldc;             // [nb]             sum_i log|scale_k,i| (0 without ActNorm)
  long long pk_b0;              // [nv][HP]         Linear-1 bias, zero beyond H
  long long total;
  int tiling;                   // BcnfStackDesc.gemm_tiling of this call (0 = each GEMM's cost-model tiling)
};

__host__ __device__ inline long long wcb(const WideLayout& L, int k) {
  return (long long)k * L.blk_stride + ((k < L.nb - 1) ? L.an : 0);
}
// first float of virtual block v's nested MLP in the canonical flat parameters
__host__ __device__ inline long long vbase(const WideLayout& L, int v) {
  return wcb(L, v / L.S) + (v % L.S ? L.mlp[0] : 0);
}

int wide_layout(const BcnfStackDesc* d, WideLayout* L) {
  if (!d || !L) return BCNF_ERR_ARG;
  memset(L, 0, sizeof(*L));
  if (d->size < 2 || d->n_blocks < 1 || d->n_hidden < 1 || d->n_hidden > BCNF_MAX_HIDDEN || d->n_conditions < 0)
    return BCNF_ERR_ARG;
  if (!(d->dropout >= 0.f && d->dropout < 1.f)) return BCNF_ERR_ARG;
  for (int i = 0; i < d->n_hidden; ++i)
    if (d->hidden[i] < 1) return BCNF_ERR_ARG;
  for (int i = 1; i < d->n_hidden; ++i)
    if (d->hidden[i] != d->hidden[0]) return BCNF_ERR_UNSUPPORTED;     // equal widths (every shipped config)
  if (d->size > DM || d->n_conditions < 1 || d->hidden[0] > 8192) return BCNF_ERR_UNSUPPORTED;
  if (d->gemm_tiling < 0 || d->gemm_tiling > 11) return BCNF_ERR_ARG;
  L->tiling = d->gemm_tiling;
  L->D = d->size;
  L->Da = (d->size + 1) / 2;
  L->Db = d->size / 2;
  L->C = d->n_conditions;
  L->Cp = pad4(L->C);
  L->H = d->hidden[0];
  L->NH = d->n_hidden;
  L->nb = d->n_blocks;
  L->an = d->act_norm ? 2 * d->size : 0;
  L->S = d->two_way ? 2 : 1;
  L->nv = L->nb * L->S;
  L->nin[0] = L->Da;  L->nout[0] = L->Db;  L->ioff[0] = 0;      L->toff[0] = L->Da;
  L->nin[1] = L->Db;  L->nout[1] = L->Da;  L->ioff[1] = L->Da;  L->toff[1] = 0;
  const int nout_max = L->S == 2 ? L->Da : L->Db;
  L->WY = L->Da;
  L->WL = 2 * nout_max;
  L->HP = pad4(L->H + 1);
  L->UP = pad4(L->Da + 1);
  L->OP = pad4(2 * nout_max);
  L->XP = pad4(L->D);
  L->SP = pad4(nout_max);
  L->AP = pad4(2 * L->D);
  L->blk_stride = L->an;
  for (int sd = 0; sd < L->S; ++sd) {
    L->in0[sd] = L->nin[sd] + L->C;
    long long off = 0;
    for (int l = 0; l <= L->NH; ++l) {
      const long long in = (l == 0) ? L->in0[sd] : L->H;
      const long long out = (l == L->NH) ? 2 * L->nout[sd] : L->H;
      L->lin_w[sd][l] = off;
      off += in * out;
      L->lin_b[sd][l] = off;
      off += out;
    }
    L->mlp[sd] = off;
    L->blk_stride += off;
  }
  L->n_trainable = (long long)L->nb * L->blk_stride - L->an;
  L->p = d->dropout;
  L->keep_scale = 1.0f / (1.0f - d->dropout);
  const double t = (double)d->dropout * 4294967296.0;
  L->thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  long long o = 0;
  L->pk_w0h = o; o += pad4l((long long)L->nv * L->HP * L->Cp);
  L->pk_hid = o; o += pad4l((long long)L->nv * (L->NH - 1) * L->HP * L->HP);
  L->pk_hidT = o; o += pad4l((long long)L->nv * (L->NH - 1) * L->HP * L->HP);
  L->pk_w0y = o; o += pad4l((long long)L->nv * L->WY * L->HP);
  L->pk_wl = o;  o += pad4l((long long)L->nv * L->WL * L->HP);
  L->pk_q = o;   o += pad4l((long long)(L->nb - 1) * L->D * L->D);
  L->pk_ldc = o; o += pad4l(L->nb);
  L->pk_b0 = o;  o += (long long)L->nv * L->HP;
  L->total = o;
  return BCNF_OK;
}

// ------------------------------------------------------------------------------------------------
// Packing: padded, GEMM-friendly copies of the weights, ONE launch per parameter update (k_wpack_all). The
// workgroups of the launch take, in blockIdx order:
//   * the small regions (W0y^T, last Linear, Q, Linear-1 biases, the ActNorm log-det constants);
//   * 64 x 64 tiles of every hidden W_l (l = 1..NH-1): the tile is read once from the flat parameters and written
//     twice, row-major into pk_hid and, through an LDS transpose, into pk_hidT (both sides coalesced);
//   * WP_ROWS rows of W0h_all per workgroup, one per wave.
// Round 5 replaced five launches (209 us alone at FC_large: a row kernel that left most of its threads idle on the
// 528-wide rows, a transpose that re-read pk_hid, three small ones) with this one: 104 us, 4.8 TB/s of written +
// read bytes against 5.4 TB/s for a device copy of the same byte count (tools/pack_bench.py).
// ------------------------------------------------------------------------------------------------
constexpr int WP_T = 64;                // hidden-W tile edge (32: 3% slower)
constexpr int WP_ROWS = WWG / 64;       // W0h_all rows per workgroup (one per wave)
constexpr int WP_SMALL = 256;   // workgroups of the small regions

struct WpackGrid {
  int t;                        // tiles per hidden-W edge
  long long n_tiles, n_rows, n_small;
};
inline WpackGrid wpack_grid(const WideLayout& L) {
  WpackGrid g;
  g.t = (L.HP + WP_T - 1) / WP_T;
  g.n_tiles = L.NH > 1 ? (long long)L.nv * (L.NH - 1) * g.t * g.t : 0;
  g.n_rows = ((long long)L.nv * L.HP + WP_ROWS - 1) / WP_ROWS;
  g.n_small = WP_SMALL;
  return g;
}

__device__ void wpack_small(const WideLayout& L, const float* __restrict__ prm, const float* __restrict__ q,
                            float* __restrict__ pk, int wg, int nwg) {
  const long long stride = (long long)nwg * WWG;
  for (long long e = L.pk_w0y + (long long)wg * WWG + threadIdx.x; e < L.pk_ldc; e += stride) {
    float v = 0.f;
    if (e < L.pk_wl) {
      const long long i = e - L.pk_w0y;
      const long long per = (long long)L.WY * L.HP;
      const int vb = (int)(i / per);
      const long long rem = i - (long long)vb * per;
      const int j = (int)(rem / L.HP), n = (int)(rem - (long long)j * L.HP);
      if (vb < L.nv) {
        const int sd = vb % L.S;
        if (n < L.H && j < L.nin[sd]) v = prm[vbase(L, vb) + L.lin_w[sd][0] + (long long)n * L.in0[sd] + j];
      }
    } else if (e < L.pk_q) {
      const long long i = e - L.pk_wl;
      const long long per = (long long)L.WL * L.HP;
      const int vb = (int)(i / per);
      const long long rem = i - (long long)vb * per;
      const int j = (int)(rem / L.HP), n = (int)(rem - (long long)j * L.HP);
      if (vb < L.nv) {
        const int sd = vb % L.S;
        if (n < L.H && j < 2 * L.nout[sd]) v = prm[vbase(L, vb) + L.lin_w[sd][L.NH] + (long long)j * L.H + n];
      }
    } else {
      const long long i = e - L.pk_q;
      if (i < (long long)(L.nb - 1) * L.D * L.D) v = q[i];
    }
    pk[e] = v;
  }
  // Linear-1 biases (zero beyond H) and the ActNorm log|det J| constant per block (ActNorm.forward,
  // cnf.py:348-351: torch.sum(log|scale|))
  for (long long e = (long long)wg * WWG + threadIdx.x; e < (long long)L.nv * L.HP; e += stride) {
    const int vb = (int)(e / L.HP), n = (int)(e - (long long)vb * L.HP);
    pk[L.pk_b0 + e] = n < L.H ? prm[vbase(L, vb) + L.lin_b[vb % L.S][0] + n] : 0.f;
  }
  for (long long k = (long long)wg * WWG + threadIdx.x; k < L.nb; k += stride) {
    float s = 0.f;
    if (L.an && k < L.nb - 1)
      for (int i = 0; i < L.D; ++i) s += logf(fabsf(prm[k * L.blk_stride + i]));
    pk[L.pk_ldc + k] = s;
  }
}

__global__ __launch_bounds__(WWG) void k_wpack_all(const WideLayout L, const WpackGrid G,
                                                   const float* __restrict__ prm, const float* __restrict__ q,
                                                   float* __restrict__ pk) {
  __shared__ float tile[WP_T][WP_T + 1];
  long long b = blockIdx.x;
  if (b < G.n_small) {          // first in the grid: their grid-stride loops overlap the bulk instead of trailing it
    wpack_small(L, prm, q, pk, (int)b, (int)G.n_small);
    return;
  }
  b -= G.n_small;
  if (b < G.n_tiles) {
    const int tt = G.t * G.t;
    const long long kl = b / tt;                              // hidden matrix index vb * (NH - 1) + (l - 1)
    const int r = (int)(b - kl * tt), n0 = (r / G.t) * WP_T, k0 = (r % G.t) * WP_T;
    const int vb = (int)(kl / (L.NH - 1)), l = (int)(kl % (L.NH - 1)) + 1;
    const float* __restrict__ src = prm + vbase(L, vb) + L.lin_w[vb % L.S][l];    // W_l[n][k] = src[n H + k]
    float* __restrict__ dst = pk + L.pk_hid + kl * L.HP * L.HP;
    float* __restrict__ dstT = pk + L.pk_hidT + kl * L.HP * L.HP;
    const int c = threadIdx.x % WP_T, r0 = threadIdx.x / WP_T;
    const int k = k0 + c;
    constexpr int RPT = WP_T / (WWG / WP_T);                  // rows per thread: every load issued before a store
    float v[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int n = n0 + r0 + j * (WWG / WP_T);
      v[j] = (n < L.H && k < L.H) ? src[(long long)n * L.H + k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int i = r0 + j * (WWG / WP_T), n = n0 + i;
      tile[i][c] = v[j];
      if (n < L.HP && k < L.HP) dst[(long long)n * L.HP + k] = v[j];
    }
    __syncthreads();
    // W^T[k][n] = W[n][k]: row k0 + i of the transposed copy, consecutive lanes on consecutive n
#pragma unroll 4
    for (int i = r0; i < WP_T; i += WWG / WP_T) {
      const int kk = k0 + i, n = n0 + c;
      if (kk < L.HP && n < L.HP) dstT[(long long)kk * L.HP + n] = tile[c][i];
    }
    return;
  }
  b -= G.n_tiles;
  if (b < G.n_rows) {
    // W0h_all row rr = vb * HP + n: W0_vb[n][nin + c], zero beyond H / C. One row per wave, so the row's block,
    // side and source offset are wave-uniform (scalar); batches of WP_EB columns per lane, every load of a batch
    // issued before its stores.
    constexpr int WP_EB = 24;         // 1536 columns: one batch at C = 1360
    const int rows = L.nv * L.HP;
    const int rr = (int)b * WP_ROWS + (int)(threadIdx.x / 64), lane = threadIdx.x % 64;
    if (rr < rows) {
      const int vb = __builtin_amdgcn_readfirstlane(rr / L.HP);
      const int n = __builtin_amdgcn_readfirstlane(rr - vb * L.HP);
      const int sd = vb % L.S;
      const float* __restrict__ src = prm + vbase(L, vb) + L.lin_w[sd][0] + (long long)n * L.in0[sd] + L.nin[sd];
      float* __restrict__ dst = pk + L.pk_w0h + (long long)rr * L.Cp;
      const int cv = n < L.H ? L.C : 0;
      for (int c0 = 0; c0 < L.Cp; c0 += WP_EB * 64) {
        float v[WP_EB];
#pragma unroll
        for (int j = 0; j < WP_EB; ++j) {
          const int c = c0 + j * 64 + lane;
          v[j] = c < cv ? src[c] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < WP_EB; ++j) {
          const int c = c0 + j * 64 + lane;
          if (c < L.Cp) dst[c] = v[j];
        }
      }
    }
  }
}

// out[m][n] = sum_p part[p][m][n] in p order (split-K partials; deterministic)
__global__ __launch_bounds__(WWG) void k_wsum_parts(const float* __restrict__ part, long long pstride, int np, int M,
                                                    int N4, long long ldp, float* __restrict__ out, long long ldo) {
  const long long n = (long long)M * N4;
  for (long long e = (long long)blockIdx.x * WWG + threadIdx.x; e < n; e += (long long)gridDim.x * WWG) {
    const int m = (int)(e / N4), c = 4 * (int)(e - (long long)m * N4);
    floatx4 a = *reinterpret_cast<const floatx4*>(part + (long long)m * ldp + c);
    for (int p = 1; p < np; ++p) {
      const floatx4 b = *reinterpret_cast<const floatx4*>(part + p * pstride + (long long)m * ldp + c);
      a = floatx4{a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]};
    }
    *reinterpret_cast<floatx4*>(out + (long long)m * ldo + c) = a;
  }
}

// rows of C floats -> rows of Cp floats (zero tail), for condition widths that are not a multiple of 4
__global__ __launch_bounds__(WWG) void k_wpad_rows(const float* __restrict__ src, int C, long long rows,
                                                   float* __restrict__ dst, int Cp) {
  const long long n = rows * Cp;
  for (long long e = (long long)blockIdx.x * WWG + threadIdx.x; e < n; e += (long long)gridDim.x * WWG) {
    const long long r = e / Cp;
    const int c = (int)(e - r * Cp);
    dst[e] = c < C ? src[r * C + c] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------------
// fp32-MFMA GEMM  C[m][n] = sum_k A(m, k) B(k, n), v_mfma_f32_32x32x2_f32.
//   A(m, k): AKC ? A[m * lda + k] : A[k * lda + m]      B(k, n): BKC ? B[n * ldb + k] : B[k * ldb + n]
// 256 threads = 2 x 2 waves; each wave owns (BM/2) x (BN/2) as 32x32 accumulators. Tiles are staged global ->
// registers -> LDS (two buffers, one barrier per K tile). K-contiguous operands keep [mn][BK+4] in LDS and are
// read as float4; the others [BK][mn+4] (conflict-free scalar reads). Inside a K tile, lane half h consumes
// k = h*BK/2 + s at MFMA step s (any k order is a valid fp32 sum order; A and B use the same one).
// Requirements (checked by the host): lda, ldb, ldc % 4 == 0, 16-byte aligned bases, K % 4 == 0 when an
// operand is K-contiguous.
// ------------------------------------------------------------------------------------------------
enum { EPI_STORE = 0, EPI_ACT = 1, EPI_GRAD = 2, EPI_LINGRAD = 3, EPI_ROWMAP = 4 };

struct GemmArgs {
  int M, N, K, G0;              // groups: blockIdx.z = g1 * G0 + g0
  const float* A; long long lda, sA1, sA0;
  const float* B; long long ldb, sB1, sB0;
  float* C; long long ldc, sC1, sC0;
  // EPI_ACT: out = dropout(GELU(acc + bias[n])) for n < n_real, 1 at n == n_real, 0 beyond; aux = G factor
  const float* bias;
  float* aux; long long ldaux, saux1, saux0;   // EPI_ACT: G out (nullable); EPI_GRAD: G in
  int n_real;
  const uint64_t* rng; uint32_t thresh; float keep_scale; uint32_t tag, tag_s1;   // tag of group = tag + g1*tag_s1
  // EPI_LINGRAD: row r, col c: c < wcols -> C[r * ldc + c], c == wcols -> C[boff + r]
  int wcols; long long boff;
  // flat-gradient group base (EPI_LINGRAD with use_cb, EPI_ROWMAP) of virtual block v = g1 (real block v / cb_S,
  // side v % cb_S): C + (v / cb_S) * cb_stride + (v / cb_S < cb_nb - 1 ? cb_an : 0) + (v % cb_S) * cb_side + g0 * sC0
  long long cb_stride, cb_side; int cb_an, cb_nb, cb_S, use_cb;
  int cb_v0;                    // virtual block of group g1 = 0 / row 0 (a block range of the backward; else 0)
  // EPI_ROWMAP: row r -> virtual block v = r / rm_hp, n = r % rm_hp (skipped when >= rm_h):
  //   C + cb(v) + rm_off[side] + n * rm_ld[side] + col
  int rm_hp, rm_h; long long rm_off[2], rm_ld[2];
  int tiling;                   // host-side dispatch only: BcnfStackDesc.gemm_tiling of the call (0 = cost model)
  // EPI_ACT on tiling W only (wbr_lp_ok): the block's LAST Linear applied to this tile's activations -- lp[row * lp_ld +
  // 32 tile_x + j] = sum over the tile's columns c of A[row][c] Wl[j][c], j < lp_n (Wl rows of ld HP, lp_w)
  float* lp; long long lp_ld; const float* lp_w; int lp_n, lp_wld;
};

__device__ __forceinline__ floatx4 ld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }
__device__ __forceinline__ void st4(float* p, floatx4 v) { *reinterpret_cast<floatx4*>(p) = v; }

// Global -> register -> LDS staging of one BM x BK (A) and BK x BN (B) tile pair by NT threads, shared by both MFMA
// tilings. FULL: the host has checked that every load of the grid lies inside its operand (K % BK == 0 and the tile
// grid's row / column extent within each leading dimension), so the loads carry no predicates -- no zeroing moves and
// no exec-mask branches in the K loop.
template <int BM, int BN, int BK, bool AKC, bool BKC, int NT = WWG, bool FULL = false>
struct TileIO {
  static constexpr int BKT = BK;
  static constexpr int ASZ = AKC ? BM * (BK + 4) : BK * (BM + 4);
  static constexpr int BSZ = BKC ? BN * (BK + 4) : BK * (BN + 4);
  static constexpr int AV = (BM * BK / 4 + NT - 1) / NT, BV = (BN * BK / 4 + NT - 1) / NT;
  floatx4 ra[AV], rb[BV];

  template <int ROWS, bool KC>
  __device__ __forceinline__ static floatx4 fetch(const float* __restrict__ X, long long ld, int e, int mn0, int k0,
                                                  int MN, int K) {
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    // e = threadIdx.x + NT i over i < AV / BV: in range by construction when NT divides the tile's float4 count
    if ((ROWS * BK / 4) % NT != 0 && e >= ROWS * BK / 4) return v;
    if (KC) {
      const int row = e / (BK / 4), kq = e % (BK / 4);
      const int gm = mn0 + row, gk = k0 + 4 * kq;
      if (FULL || (gm < MN && gk < K)) v = ld4(X + (long long)gm * ld + gk);
    } else {
      // a whole float4 whenever gm < MN: a [K][MN] operand's rows are readable up to roundup4(MN) <= ld (ld % 4 == 0,
      // host-checked), and the values past MN only reach output rows / columns that are never stored. The row offset
      // splits into a loop-invariant part and k0 ld, so the K loop carries no 64-bit multiply and no edge branches.
      const int kr = e / (ROWS / 4), mq = e % (ROWS / 4);
      const int gk = k0 + kr, gm = mn0 + 4 * mq;
      if (FULL || (gk < K && gm < MN)) v = ld4(X + ((long long)kr * ld + gm) + (long long)k0 * ld);
    }
    return v;
  }
  template <int ROWS, bool KC>
  __device__ __forceinline__ static void put(float* S, int e, floatx4 v) {
    if ((ROWS * BK / 4) % NT != 0 && e >= ROWS * BK / 4) return;
    if (KC) st4(S + (e / (BK / 4)) * (BK + 4) + 4 * (e % (BK / 4)), v);
    else st4(S + (e / (ROWS / 4)) * (ROWS + 4) + 4 * (e % (ROWS / 4)), v);
  }
  __device__ __forceinline__ void load(const GemmArgs& g, const float* A, const float* B, int m0, int n0, int k0) {
#pragma unroll
    for (int i = 0; i < AV; ++i) ra[i] = fetch<BM, AKC>(A, g.lda, threadIdx.x + NT * i, m0, k0, g.M, g.K);
#pragma unroll
    for (int i = 0; i < BV; ++i) rb[i] = fetch<BN, BKC>(B, g.ldb, threadIdx.x + NT * i, n0, k0, g.N, g.K);
  }
  __device__ __forceinline__ void store(float* As, float* Bs) const {
#pragma unroll
    for (int i = 0; i < AV; ++i) put<BM, AKC>(As, threadIdx.x + NT * i, ra[i]);
#pragma unroll
    for (int i = 0; i < BV; ++i) put<BN, BKC>(Bs, threadIdx.x + NT * i, rb[i]);
  }
  // four consecutive-k operand values of row / column mn at k offset kb of the staged tile
  template <int ROWS, bool KC>
  __device__ __forceinline__ static floatx4 frag(const float* S, int mn, int kb) {
    if (KC) return ld4(S + mn * (BK + 4) + kb);
    return floatx4{S[(kb + 0) * (ROWS + 4) + mn], S[(kb + 1) * (ROWS + 4) + mn], S[(kb + 2) * (ROWS + 4) + mn],
                   S[(kb + 3) * (ROWS + 4) + mn]};
  }
};

// Epilogue of four consecutive output rows rbase..rbase+3 at column col (both MFMA tilings hold their
// accumulators in such groups). rnd: the group's Philox draw (EPI_ACT with dropout).
// Operands the epilogue of a 4-row group needs from memory (EPI_GRAD: the G factors; EPI_ACT: the column's bias),
// fetched before the K loop so their latency hides behind it.
template <int EPI>
__device__ __forceinline__ void epi_pre(const GemmArgs& g, const float* __restrict__ Xg, int rbase, int col, float pre[4],
                                        int rs = 1) {
  pre[0] = pre[1] = pre[2] = pre[3] = 0.f;
  if (col >= g.N) return;
  if (EPI == EPI_GRAD) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      if (rbase + rs * rr < g.M) pre[rr] = Xg[(long long)(rbase + rs * rr) * g.ldaux + col];
  } else if (EPI == EPI_ACT) {
    if (col < g.n_real) pre[0] = g.bias[col];
  }
}

template <int EPI>
__device__ __forceinline__ void epi4(const GemmArgs& g, float* __restrict__ Cg, float* __restrict__ Xg, int rbase,
                                     int col, const float v[4], uint4 rnd, const float pre[4], int rs = 1,
                                     float* aout = nullptr) {
  const int M = g.M, N = g.N;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = rbase + rs * rr;
    if (aout) aout[rr] = 0.f;
    if (row >= M || col >= N) continue;
    if (EPI == EPI_STORE) {
      Cg[(long long)row * g.ldc + col] = v[rr];
    } else if (EPI == EPI_ACT) {
      // the chain's activations / derivative factors (and EPI_GRAD's dZ, the links' A0 / G0 / dZ) are written through
      // (sc1): nothing stays dirty in the L2s for the kernel boundary (r05: FC_large 7.59 -> 7.43 ms per step,
      // profiles/r05zo_ab_wide_write_through.txt); the Linear-gradient / store / row-map epilogues keep write-back
      // stores (write-through there cost the backward ~80 us)
      float a = 0.f, gd = 0.f;
      if (col < g.n_real) {
        float ge, dg;
        gelu_fg(v[rr] + pre[0], ge, dg);
        if (g.rng) {
          const uint32_t u = rr == 0 ? rnd.x : rr == 1 ? rnd.y : rr == 2 ? rnd.z : rnd.w;
          const float m = u >= g.thresh ? g.keep_scale : 0.f;
          a = ge * m;
          gd = dg * m;
        } else {
          a = ge;
          gd = dg;
        }
      } else if (col == g.n_real) {
        a = 1.f;
      }
      st1_wt(Cg + (long long)row * g.ldc + col, a);
      if (Xg) st1_wt(Xg + (long long)row * g.ldaux + col, gd);
      if (aout) aout[rr] = a;
    } else if (EPI == EPI_GRAD) {
      st1_wt(Cg + (long long)row * g.ldc + col, v[rr] * pre[rr]);
    } else if (EPI == EPI_LINGRAD) {
      if (col < g.wcols) Cg[(long long)row * g.ldc + col] = v[rr];
      else if (col == g.wcols) Cg[g.boff + row] = v[rr];
    } else {   // EPI_ROWMAP
      const int vr = row / g.rm_hp, n = row - vr * g.rm_hp, vb = vr + g.cb_v0;
      if (n < g.rm_h) {
        const int blk = vb / g.cb_S, sd = vb - blk * g.cb_S;
        Cg[(long long)blk * g.cb_stride + ((blk < g.cb_nb - 1) ? g.cb_an : 0) + sd * g.cb_side + g.rm_off[sd] +
           (long long)n * g.rm_ld[sd] + col] = v[rr];
      }
    }
  }
}

// EPI_ROWMAP's destination row (see GemmArgs): the flat-gradient row of output row `row`, nullptr when the row is past
// M or a padding row (n >= rm_h)
__device__ __forceinline__ float* rowmap_ptr(const GemmArgs& g, float* Cg, int row) {
  if (row >= g.M) return nullptr;
  const int vr = row / g.rm_hp, n = row - vr * g.rm_hp, vb = vr + g.cb_v0;
  if (n >= g.rm_h) return nullptr;
  const int blk = vb / g.cb_S, sd = vb - blk * g.cb_S;
  return Cg + (long long)blk * g.cb_stride + ((blk < g.cb_nb - 1) ? g.cb_an : 0) + sd * g.cb_side +
         (sd ? g.rm_off[1] : g.rm_off[0]) + (long long)n * (sd ? g.rm_ld[1] : g.rm_ld[0]);
}

struct EpiCtx {
  float* C;
  float* X;
  uint64_t seed, offs;
  uint32_t tag;
};

template <int EPI>
__device__ __forceinline__ void epi_rng(const GemmArgs& g, EpiCtx& e) {   // the dropout state (EPI_ACT)
  if (EPI == EPI_ACT && g.rng) {
    e.seed = g.rng[0];
    e.offs = g.rng[1];
  }
}

// RNG = false: seed / offs stay 0 here and epi_rng loads them later (just before the epilogue)
template <int EPI, bool RNG = true>
__device__ __forceinline__ EpiCtx epi_ctx(const GemmArgs& g, int g1, int g0) {
  EpiCtx e;
  e.C = g.C;
  if (EPI == EPI_LINGRAD && g.use_cb) {
    const int blk = (g1 + g.cb_v0) / g.cb_S, sd = (g1 + g.cb_v0) - blk * g.cb_S;
    e.C += blk * g.cb_stride + ((blk < g.cb_nb - 1) ? g.cb_an : 0) + sd * g.cb_side + g0 * g.sC0;
  } else if (EPI == EPI_ROWMAP) {
    // the row map carries the whole offset
  } else
    e.C += g1 * g.sC1 + g0 * g.sC0;
  e.X = (EPI == EPI_ACT || EPI == EPI_GRAD) && g.aux ? g.aux + g1 * g.saux1 + g0 * g.saux0 : nullptr;
  e.seed = 0;
  e.offs = 0;
  if (RNG) epi_rng<EPI>(g, e);
  e.tag = g.tag + (uint32_t)g1 * g.tag_s1;
  return e;
}

// Split-K Linear gradient: v = sum_p part[g1][p][r][c] in p order, stored through the EPI_LINGRAD mapping of group g1
// (c < wcols -> the block's dW row r, c == wcols -> its bias entry r). blockIdx.y = group.
__global__ __launch_bounds__(WWG) void k_wsum_lingrad(const GemmArgs g, const float* __restrict__ part, int np,
                                                      long long ldp) {
  const long long e = (long long)blockIdx.x * WWG + threadIdx.x;
  if (e >= (long long)g.M * g.N) return;
  const int g1 = blockIdx.y, r = (int)(e / g.N), c = (int)(e - (long long)r * g.N);
  const long long ps = (long long)g.M * ldp;
  const float* p = part + (long long)g1 * np * ps + (long long)r * ldp + c;
  float v = p[0];
  for (int q = 1; q < np; ++q) v += p[q * ps];
  const EpiCtx x = epi_ctx<EPI_LINGRAD>(g, g1, 0);
  if (c < g.wcols) x.C[(long long)r * g.ldc + c] = v;
  else if (c == g.wcols) x.C[g.boff + r] = v;
}

template <int EPI>
__device__ __forceinline__ uint4 epi_rnd(const GemmArgs& g, const EpiCtx& e, int rbase, int col) {
  if (EPI == EPI_ACT && g.rng)
    return philox4x32_10(make_uint4((uint32_t)rbase, (uint32_t)col, e.tag, (uint32_t)e.offs),
                         make_uint2((uint32_t)e.seed, (uint32_t)(e.seed >> 32) ^ (uint32_t)(e.offs >> 32)));
  return make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup
// dispatch), so linear ids b and b + 8 share an L2. Renumber so that each XCD walks a contiguous run of tiles
// (N fastest, then M, then group): its L2 then holds one band of A rows plus the B columns that band needs, instead
// of every XCD streaming all of A and B. Speed only -- any tile order is correct.
struct TileId {
  int x, y, z;
};
__device__ __forceinline__ TileId tile_id() {
  const unsigned gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const unsigned total = gx * gy * gz;
  unsigned lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  // the dispatcher sends workgroup `lin` to XCD lin % 8: give each XCD one contiguous range of tiles (x fastest, so an
  // XCD's tiles share A row blocks and the whole B in its own L2), also when total is not a multiple of 8 (the
  // 11 x 22 chain grids): XCD x takes q + (x < r) tiles starting at x q + min(x, r)
  if (total >= 16) {
    const unsigned q = total >> 3, r = total & 7u, x = lin & 7u;
    lin = x * q + (x < r ? x : r) + (lin >> 3);
  }
  TileId t;
  t.x = (int)(lin % gx);
  lin /= gx;
  t.y = (int)(lin % gy);
  t.z = (int)(lin / gy);
  return t;
}

// The K loop of both tilings: two LDS buffers and two register staging sets, loads issued TWO K tiles ahead of the
// MFMAs (a tile's global loads have two tiles of MFMA work to land in, not one: at M = 2048, N = K = 528 a tile's
// MFMA phase is ~1.3 us, below one loaded L2/HBM round trip). Hand-unrolled by two so each staging set is a fixed
// register range: the store of set s waits only for s's loads (vmcnt counts the newer set's loads as in flight).
// The prefetch index is clamped instead of predicated (a redundant reload of the last tile) for the same reason.
template <class IO, class F>
__device__ __forceinline__ void k_loop(const GemmArgs& g, const float* __restrict__ A, const float* __restrict__ B,
                                       int m0, int n0, float* lds, F&& tile) {
  constexpr int BK = IO::BKT, STG = IO::ASZ + IO::BSZ;
  const int nk = (g.K + BK - 1) / BK;
  IO s0, s1;
  s0.load(g, A, B, m0, n0, 0);
  s1.load(g, A, B, m0, n0, (nk > 1 ? 1 : 0) * BK);
  s0.store(lds, lds + IO::ASZ);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    s0.load(g, A, B, m0, n0, min(kt + 2, nk - 1) * BK);
    tile(lds);
    s1.store(lds + STG, lds + STG + IO::ASZ);
    __syncthreads();
    if (kt + 1 >= nk) break;
    s1.load(g, A, B, m0, n0, min(kt + 3, nk - 1) * BK);
    tile(lds + STG);
    s0.store(lds, lds + IO::ASZ);
    __syncthreads();
  }
}

// Tiling A: v_mfma_f32_32x32x2_f32, 2 x 2 waves, each (BM/2) x (BN/2) as 32x32 accumulators. Inside a K tile
// lane half h consumes k = h*BK/2 + s at MFMA step s.
template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI>
__global__ __launch_bounds__(WWG, 2) void k_wgemm(const GemmArgs g) {
  using IO = TileIO<BM, BN, BK, AKC, BKC>;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TI = WM / 32, TJ = WN / 32;
  __shared__ __attribute__((aligned(16))) float lds[2 * (IO::ASZ + IO::BSZ)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, c32 = lane & 31, hh = lane >> 5;
  const TileId tl = tile_id();
  const int z = tl.z, g1 = z / g.G0, g0 = z - g1 * g.G0;
  const float* __restrict__ A = g.A + g1 * g.sA1 + g0 * g.sA0;
  const float* __restrict__ B = g.B + g1 * g.sB1 + g0 * g.sB0;
  const int m0 = tl.y * BM, n0 = tl.x * BN;
  const EpiCtx e = epi_ctx<EPI>(g, g1, g0);
  float pre[TI][TJ][4][4];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        epi_pre<EPI>(g, e.X, m0 + wm * WM + 32 * i + 8 * q + 4 * hh, n0 + wn * WN + 32 * j + c32, pre[i][j][q]);
  floatx16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto tile = [&](const float* As) {
    const float* Bs = As + IO::ASZ;
#pragma unroll
    for (int sq = 0; sq < BK / 8; ++sq) {
      const int kb = hh * (BK / 2) + 4 * sq;
      floatx4 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = IO::template frag<BM, AKC>(As, wm * WM + 32 * i + c32, kb);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bf[j] = IO::template frag<BN, BKC>(Bs, wn * WN + 32 * j + c32, kb);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
  };
  // interior tiles (whole K tiles, the tile inside M x N: most of any large grid) stage without load predicates; the
  // edge tiles keep them (a workgroup-uniform branch)
  if (g.K % BK == 0 && m0 + BM <= g.M && n0 + BN <= g.N)
    k_loop<TileIO<BM, BN, BK, AKC, BKC, WWG, true>>(g, A, B, m0, n0, lds, tile);
  else
    k_loop<IO>(g, A, B, m0, n0, lds, tile);
  // accumulator element r of lane (c32, hh): row = (r & 3) + 8 (r >> 2) + 4 hh, col = c32
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + wn * WN + 32 * j + c32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rbase = m0 + wm * WM + 32 * i + 8 * q + 4 * hh;
        const float v[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        epi4<EPI>(g, e.C, e.X, rbase, col, v, epi_rnd<EPI>(g, e, rbase, col), pre[i][j][q]);
      }
    }
}

// Tiling B: v_mfma_f32_16x16x4_f32, NW waves stacked along M, each (BM/NW) x BN as 16x16 accumulators (>= 2
// independent chains cover the 40-cycle dependent latency). Inside a 16-k chunk lane group q = lane >> 4 consumes
// k = 4q + s at MFMA step s. Finer N granularity than tiling A: e.g. BN = 48 tiles N = 528 exactly. NW = 8: two
// waves per SIMD in one workgroup, so a wave's barrier / LDS / staging stalls run under its partner's MFMAs (the
// small-M GEMMs of the wide family leave most CUs with one workgroup).
// Two workgroups per CU only when the two LDS buffers fit twice in the CU's 160 KB (the 128 x 48 tile's 94 KB does
// not: one workgroup per CU, declared as such).
template <int BM, int BN, int BK, bool AKC, bool BKC, int NW>
constexpr int wg16_occ() {
  using IO = TileIO<BM, BN, BK, AKC, BKC, 64 * NW>;
  return (NW == 4 && 2 * (IO::ASZ + IO::BSZ) * 4 <= 80 * 1024) ? 2 : 1;
}
template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI, int NW = 4, bool FULL = false>
__global__ __launch_bounds__(64 * NW, (wg16_occ<BM, BN, BK, AKC, BKC, NW>())) void k_wgemm16(const GemmArgs g) {
  using IO = TileIO<BM, BN, BK, AKC, BKC, 64 * NW, FULL>;
  constexpr int WM = BM / NW;
  constexpr int TI = WM / 16, TJ = BN / 16;
  __shared__ __attribute__((aligned(16))) float lds[2 * (IO::ASZ + IO::BSZ)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, qq = lane >> 4;
  const TileId tl = tile_id();
  const int z = tl.z, g1 = z / g.G0, g0 = z - g1 * g.G0;
  const float* __restrict__ A = g.A + g1 * g.sA1 + g0 * g.sA0;
  const float* __restrict__ B = g.B + g1 * g.sB1 + g0 * g.sB0;
  const int m0 = tl.y * BM, n0 = tl.x * BN;
  const EpiCtx e = epi_ctx<EPI>(g, g1, g0);
  float pre[TI][TJ][4];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) epi_pre<EPI>(g, e.X, m0 + wave * WM + 16 * i + 4 * qq, n0 + 16 * j + c16, pre[i][j]);
  floatx4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto tile = [&](const float* As) {
    const float* Bs = As + IO::ASZ;
#pragma unroll
    for (int kc = 0; kc < BK / 16; ++kc) {
      const int kb = 16 * kc + 4 * qq;
      if constexpr (TI == 1) {
        // one 16-row strip per wave (the 176 x 176 Linear-gradient tile): B columns two at a time, the four k steps of
        // each pair interleaved over the pair's two independent accumulators. With every fragment read first (the
        // order below) hipcc, at its 168-VGPR cap, re-serialised the tile to ds_read2 -> wait -> 2 MFMAs; this order
        // lets it keep several reads in flight: 1180 -> 1153-1162 us per FC_large step
        // (profiles/r05zz7_ab_lingrad_pairs.txt). Same k order per accumulator: bit-identical
        const floatx4 a0 = IO::template frag<BM, AKC>(As, wave * WM + c16, kb);
#pragma unroll
        for (int j = 0; j < TJ; j += 2) {
          const floatx4 b0 = IO::template frag<BN, BKC>(Bs, 16 * j + c16, kb);
          if (j + 1 < TJ) {
            const floatx4 b1 = IO::template frag<BN, BKC>(Bs, 16 * (j + 1) + c16, kb);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b0[s], acc[0][j], 0, 0, 0);
              acc[0][j + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b1[s], acc[0][j + 1], 0, 0, 0);
            }
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
              acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b0[s], acc[0][j], 0, 0, 0);
          }
        }
      } else {
        floatx4 af[TI], bf[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) af[i] = IO::template frag<BM, AKC>(As, wave * WM + 16 * i + c16, kb);
#pragma unroll
        for (int j = 0; j < TJ; ++j) bf[j] = IO::template frag<BN, BKC>(Bs, 16 * j + c16, kb);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
      }
    }
  };
  k_loop<IO>(g, A, B, m0, n0, lds, tile);
  // accumulator element r of lane (c16, qq): row = 4 qq + r, col = c16
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = n0 + 16 * j + c16;
      const int rbase = m0 + wave * WM + 16 * i + 4 * qq;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epi4<EPI>(g, e.C, e.X, rbase, col, v, epi_rnd<EPI>(g, e, rbase, col), pre[i][j]);
    }
}

// ------------------------------------------------------------------------------------------------
// Tiling C: LDS-DMA staging (global_load_lds_dwordx4), the gfx950 GEMM pipeline (cdna_hip_programming.md §5).
// Register-staged tilings A / B serialise each K tile on one global round trip: their staging registers are
// loop-carried, so hipcc drains vmcnt at the loop head (tools: .s of k_wgemm16), and at M = 2048, N = K = 528 the
// chain GEMMs sit at ~23 us for ~8 us of MFMA work per CU. Here a K tile (BK = 64) of both operands is copied
// global -> LDS with no VGPR destination, S stages deep: tile kt + S - 1 is issued right after the barrier that
// retires tile kt, the wait is a counted `s_waitcnt vmcnt(NI x tiles still ahead)` (NI = DMA instructions per wave
// per tile), the barrier is a raw s_barrier (a __syncthreads() fence would drain the in-flight DMA), and all LDS is
// one dynamic array.
//   * K-contiguous operand (KC): image [row][64 floats], 16-B chunk q of row r stored in slot q ^ (r & 15) -- the
//     swizzle is applied to the DMA's per-lane SOURCE address (the LDS side of a DMA is lane-linear) and undone on
//     the read; a fragment is one ds_read_b128 of 4 consecutive k, conflict-free over each 16-lane group.
//   * otherwise: image [64 k][R] linear; lane c reads the float4 of columns 4c..4c+3 at one k, i.e. one k-step's
//     operand for FOUR 16-wide tiles, so such an operand's wave extent is 64 (4 tiles) with tile t holding the
//     rows / columns {4c + t} (undone in the epilogue: row stride 4).
//   * out-of-range rows / columns read clamped (finite, never stored); the K tail beyond K is zeroed in registers.
// Requirements as tilings A / B (checked by the host); rows read as float4 up to roundup4 of their length <= ld.
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, int S, int KS>
struct GlCfg {
  static constexpr int BK = 64, NT = WGM * WGN, NW = NT * KS;   // output-tile waves x K halves
  static constexpr int WM = BM / WGM, WN = BN / WGN, TI = WM / 16, TJ = WN / 16;
  static constexpr int ACH = BM * BK / 4, BCH = BN * BK / 4;   // 16-B chunks of one stage
  static constexpr int NI = (ACH + BCH) / 64 / NW;              // DMA instructions per wave per stage
  static constexpr int STG = (BM + BN) * BK;                    // floats per stage
  static_assert(WM % 16 == 0 && WN % 16 == 0, "16-row MFMA tiles");
  static_assert(AKC || TI == 4, "non-K-contiguous A: 64 rows per wave");
  static_assert(BKC || TJ == 4, "non-K-contiguous B: 64 columns per wave");
  static_assert(ACH % 64 == 0 && BCH % 64 == 0 && (ACH + BCH) % (64 * NW) == 0, "whole DMA instructions per wave");
  static_assert(2 * NI <= 63, "vmcnt range");
};

// per-lane source of 16-B chunk e of an operand stage (KC: R rows x 64 k; else 64 k x R columns)
template <bool KC, int R>
__device__ __forceinline__ const float* gl_src(const float* __restrict__ X, long long ld, int e, int mn0, int k0, int MN,
                                               int K) {
  if (KC) {
    const int r = e >> 4, q = (e & 15) ^ (r & 15);
    const int gm = min(mn0 + r, MN - 1);
    int gk = k0 + 4 * q;
    if (gk >= K) gk = 0;
    return X + (long long)gm * ld + gk;
  } else {
    const int kr = e / (R / 4), c = e - kr * (R / 4);
    int gk = k0 + kr, gm = mn0 + 4 * c;
    if (gk >= K) gk = 0;
    if (gm >= MN) gm = 0;
    return X + (long long)gk * ld + gm;
  }
}

template <class T, bool AKC, bool BKC, int BM, int BN>
__device__ __forceinline__ void gl_issue(const float* __restrict__ A, long long lda, const float* __restrict__ B,
                                         long long ldb, int M, int N, int K, int m0, int n0, int k0, float* buf,
                                         int wave, int lane) {
#pragma unroll
  for (int t = 0; t < T::NI; ++t) {
    const int ins = wave + T::NW * t;                 // wave-uniform
    const int e = ins * 64 + lane;
    const float* src = (ins * 64 < T::ACH) ? gl_src<AKC, BM>(A, lda, e, m0, k0, M, K)
                                           : gl_src<BKC, BN>(B, ldb, e - T::ACH, n0, k0, N, K);
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + ins * 256), 16,
                                     0, 0);
  }
}

// fragments of one 16-deep k chunk: KC -> f[t] = 4 consecutive k of row t; else f[s] = tiles 0..3 at k-step s
template <bool KC, int R, int T4>
__device__ __forceinline__ void gl_frag(const float* __restrict__ Sx, int base, int kc, int c16, int qq, floatx4 f[4]) {
  if (KC) {
#pragma unroll
    for (int t = 0; t < T4; ++t) f[t] = ld4(Sx + (base + 16 * t + c16) * 64 + 4 * ((4 * kc + qq) ^ c16));
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) f[s] = ld4(Sx + (16 * kc + 4 * qq + s) * R + base + 4 * c16);
  }
}

template <class T, bool AKC, bool BKC, int BM, int BN, int KS, bool TAIL>
__device__ __forceinline__ void gl_tile(const float* __restrict__ As, floatx4 (&acc)[T::TI][T::TJ], int am, int bn,
                                        int c16, int qq, int kh, int kvalid) {
  const float* Bs = As + BM * 64;
#pragma unroll
  for (int kq = 0; kq < 4 / KS; ++kq) {
    const int kc = kh * (4 / KS) + kq;
    // a 16-deep chunk wholly past K contributes nothing (K = 528 at BK = 64: 3 of the last tile's 4 chunks); kc and
    // kvalid are wave-uniform, so the skip is a scalar branch
    if (TAIL && 16 * kc >= kvalid) continue;
    floatx4 a[4], b[4];
    gl_frag<AKC, BM, T::TI>(As, am, kc, c16, qq, a);
    gl_frag<BKC, BN, T::TJ>(Bs, bn, kc, c16, qq, b);
    if (TAIL) {   // k >= K: zero (a K-contiguous operand implies K % 4 == 0, so its float4 is all in or all out)
      const floatx4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool out_t = 16 * kc + 4 * qq + t >= kvalid, out_q = 16 * kc + 4 * qq >= kvalid;
        if (AKC ? out_q : out_t) a[t] = zero;
        if (BKC ? out_q : out_t) b[t] = zero;
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < T::TI; ++i)
#pragma unroll
        for (int j = 0; j < T::TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(AKC ? a[i][s] : a[s][i], BKC ? b[j][s] : b[s][j],
                                                           acc[i][j], 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// KS = 2: each output tile's K chunks are split between two waves (k chunks 0-1 / 2-3 of every K tile), whose
// partial accumulators meet in LDS after the loop: twice the waves per SIMD to cover LDS and MFMA latency, and
// tile shapes whose output waves do not divide evenly over the 4 SIMDs (96 x 48 = 6 waves) balance at 12.
template <int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, int EPI, int S, int KS>
__global__ __launch_bounds__(64 * WGM * WGN * KS, (S * (BM + BN) * 64 * 4 <= 80 * 1024) ? 2 : 1) void k_wgl(const GemmArgs g) {
  using T = GlCfg<BM, BN, WGM, WGN, AKC, BKC, S, KS>;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = wave / T::NT, wt = wave - kh * T::NT;
  const int wm = wt / WGN, wn = wt - (wt / WGN) * WGN;
  const int c16 = lane & 15, qq = lane >> 4;
  const TileId tl = tile_id();
  const int z = tl.z, g1 = z / g.G0, g0 = z - g1 * g.G0;
  const float* __restrict__ A = g.A + g1 * g.sA1 + g0 * g.sA0;
  const float* __restrict__ B = g.B + g1 * g.sB1 + g0 * g.sB0;
  const int m0 = tl.y * BM, n0 = tl.x * BN;
  const EpiCtx e = epi_ctx<EPI>(g, g1, g0);
  // output rows / columns of accumulator tile (i, j), element r: KC A -> rows am0 + 16 i + 4 qq + r; else
  // am0 + 16 qq + 4 r + i (row stride 4). KC B -> column bn0 + 16 j + c16; else bn0 + 4 c16 + j.
  const int am0 = m0 + wm * T::WM, bn0 = n0 + wn * T::WN;
  auto rbase = [&](int i) { return AKC ? am0 + 16 * i + 4 * qq : am0 + 16 * qq + i; };
  auto colof = [&](int j) { return BKC ? bn0 + 16 * j + c16 : bn0 + 4 * c16 + j; };
  constexpr int RS = AKC ? 1 : 4;
  // with KS = 2 the two K halves split the epilogue: half 0 finalises accumulator tiles f = i * TJ + j < NF0, half 1
  // the rest (the GELU / Philox / G epilogue is a third of a chain GEMM's time at M = 2048)
  constexpr int NF0 = (T::TI * T::TJ + 1) / 2;
  auto mine = [&](int f) { return KS == 1 || (kh == 0 ? f < NF0 : f >= NF0); };
  float pre[T::TI][T::TJ][4];
#pragma unroll
  for (int i = 0; i < T::TI; ++i)
#pragma unroll
    for (int j = 0; j < T::TJ; ++j)
      if (mine(i * T::TJ + j)) epi_pre<EPI>(g, e.X, rbase(i), colof(j), pre[i][j], RS);
  floatx4 acc[T::TI][T::TJ];
#pragma unroll
  for (int i = 0; i < T::TI; ++i)
#pragma unroll
    for (int j = 0; j < T::TJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = (g.K + T::BK - 1) / T::BK;
#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < nk)
      gl_issue<T, AKC, BKC, BM, BN>(A, g.lda, B, g.ldb, g.M, g.N, g.K, m0, n0, st * T::BK, lds + st * T::STG, wave,
                                    lane);
  int rd = 0, wr = S - 1;       // stage read at kt / stage written by the issue of tile kt + S - 1
  const int am = AKC ? wm * T::WM : wm * 64, bn = BKC ? wn * T::WN : wn * 64;
  auto ktile = [&](int kt) {    // wait for tile kt, issue tile kt + S - 1, return tile kt's stage
    const int ahead = min(nk - 1 - kt, S - 2);
    if (S > 3 && ahead >= 2) vm_wait<2 * T::NI>();
    else if (S > 2 && ahead >= 1) vm_wait<T::NI>();
    else vm_wait<0>();
    raw_barrier();
    if (kt + S - 1 < nk)
      gl_issue<T, AKC, BKC, BM, BN>(A, g.lda, B, g.ldb, g.M, g.N, g.K, m0, n0, (kt + S - 1) * T::BK,
                                    lds + wr * T::STG, wave, lane);
    const float* As = lds + rd * T::STG;
    rd = rd + 1 == S ? 0 : rd + 1;
    wr = wr + 1 == S ? 0 : wr + 1;
    return As;
  };
  // the partial last K tile is peeled off the loop: with the tail variant inside it, hipcc kept two register
  // homes for the accumulators and copied them (a v_mov_b64 per accumulator pair and path) every iteration
  const bool tail = (g.K & (T::BK - 1)) != 0;
  const int nfull = tail ? nk - 1 : nk;
  for (int kt = 0; kt < nfull; ++kt)
    gl_tile<T, AKC, BKC, BM, BN, KS, false>(ktile(kt), acc, am, bn, c16, qq, kh, T::BK);
  if (tail) gl_tile<T, AKC, BKC, BM, BN, KS, true>(ktile(nk - 1), acc, am, bn, c16, qq, kh, g.K - (nk - 1) * T::BK);
  if constexpr (KS > 1) {   // K halves meet: each hands the other the partials of the tiles the other finalises
    static_assert(KS == 2, "two K halves");
    static_assert(T::NT * T::TI * T::TJ * 256 <= S * T::STG, "partials fit the staging ring");
    raw_barrier();
    float* part = lds + (wt * T::TI * T::TJ) * 256 + lane * 4;
#pragma unroll
    for (int i = 0; i < T::TI; ++i)
#pragma unroll
      for (int j = 0; j < T::TJ; ++j)
        if (!mine(i * T::TJ + j)) st4(part + (i * T::TJ + j) * 256, acc[i][j]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
#pragma unroll
    for (int i = 0; i < T::TI; ++i)
#pragma unroll
      for (int j = 0; j < T::TJ; ++j)
        if (mine(i * T::TJ + j)) {
          const floatx4 p = ld4(part + (i * T::TJ + j) * 256);
          acc[i][j] = floatx4{acc[i][j][0] + p[0], acc[i][j][1] + p[1], acc[i][j][2] + p[2], acc[i][j][3] + p[3]};
        }
  }
  if constexpr (EPI == EPI_ROWMAP) {
    // the row map once per output row of the lane (16 rows x TJ columns share it), not once per element: epi4's
    // per-element divisions and selects made this epilogue ~5k instructions (r05: the condition-gradient GEMM ran
    // 183 us against 126 us for the same GEMM with plain stores; backward -8 to -20 us, profiles/r05zv_*)
#pragma unroll
    for (int i = 0; i < T::TI; ++i) {
      float* rowp[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) rowp[rr] = rowmap_ptr(g, e.C, rbase(i) + RS * rr);
#pragma unroll
      for (int j = 0; j < T::TJ; ++j)
        if (mine(i * T::TJ + j) && colof(j) < g.N) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            if (rowp[rr]) rowp[rr][colof(j)] = acc[i][j][rr];
        }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < T::TI; ++i)
#pragma unroll
    for (int j = 0; j < T::TJ; ++j)
      if (mine(i * T::TJ + j)) {
        const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        epi4<EPI>(g, e.C, e.X, rbase(i), colof(j), v, epi_rnd<EPI>(g, e, rbase(i), colof(j)), pre[i][j], RS);
      }
}

// ------------------------------------------------------------------------------------------------
// Tiling W: the workgroup's whole B band resident in LDS (K-contiguous A and B, K <= 768). On the chain shape
// (M = 2048, N = K = 528) tiling C runs ~1.5 us per 64-deep K tile at ANY M (37 rows as at 2048): per-CU issue, not
// bandwidth -- every K tile costs each SIMD 9 LDS-DMA pieces (60-185 issue cycles each beside MFMAs,
// MI355X_MICROARCH.md) and a 12-wave barrier. Here the
// 48-column B band (48 x K floats: 101 KB at K = 528) is copied into LDS ONCE by LDS-DMA at the start, one barrier,
// and each wave then streams only its own 16 A rows straight into a P-deep register ring (one float4 per lane per
// 16-deep K chunk; A rows are never shared between waves): inside the K loop there is no barrier, no DMA, and per
// chunk one global load + 3 ds_read_b128 per 12 MFMAs. Band layout [column][S], S = K16 + 4 floats (S / 4 odd: the
// 16 columns of a fragment read start on 16 distinct 4-bank groups, conflict-free). KS = 2 waves per output wave tile
// split the chunks (contiguous halves) and meet in LDS after the loop as in tiling R (fixed order).
// ------------------------------------------------------------------------------------------------
#ifndef WB_P
#define WB_P 2          // A-operand register ring depth of tiling W (chunks in flight per wave)
#endif
constexpr int WB_KMAX = 768;   // K of the resident B band (48 x 772 floats = 148 KB of LDS)
template <int WGM, int KS, int P, int KQ, int TI = 1>
struct WbCfg {
  // KQ float4 per lane per chunk: a chunk is CK = 16 KQ deep and lane group q holds its k = 4 KQ q .. 4 KQ q + 4 KQ - 1
  // (KQ = 2: each row's 128-B line is fetched by ONE load instruction instead of half a line per load, twice)
  static constexpr int BM = 16 * TI * WGM, BN = 48, TJ = 3, NF = TI * TJ, NT = WGM, NW = NT * KS, CK = 16 * KQ;
  static constexpr int KMAX = WB_KMAX;
  __host__ __device__ static constexpr int stride(int K) { return ((K + CK - 1) / CK) * CK + 4; }
  __host__ __device__ static constexpr int band_floats(int K) { return (BN * stride(K) + 255) & ~255; }
  // after the K loop the band is dead: KS-merge partials at 0, then (EPI_ACT with lp) a [16][17] transpose tile per
  // wave and the owner waves' last-Linear partials [NT][KS][2][64 lanes][4]
  // and the tile's slice of the last Linear's weights [32 rows][52] (row stride 52: the B-operand reads of 16 rows x 4
  // columns hit 64 distinct banks)
  static constexpr int LP_T = NT * NF * KS * 256, LP_M = LP_T + NW * 272, LP_W = LP_M + NT * KS * 2 * 256,
                       LP_END = LP_W + 32 * 52;
  __host__ __device__ static constexpr int lds_floats(int K) {
    return band_floats(K) > LP_END ? band_floats(K) : LP_END;
  }
};

// Phase stamps of tiling W (diagnostic build only, -DBCNF_PHASE_STAMPS): wave 0 of each of the first 256 tiles of the
// latest launch -> g_wbr_st[tile][8] = cycles to (A + band issued, band landed, K loop done, KS merge done, epilogue
// done), 100 MHz ticks over the whole wave, its total cycles, the dispatch order (bcnf_wide_debug_wbr).
#ifdef BCNF_PHASE_STAMPS
__device__ unsigned long long g_wbr_st[256 * 8];
#define WBR_ST(i) do { if (threadIdx.x == 0) wst_[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define WBR_ST(i) do {} while (0)
#endif

// KT: K has a partial last chunk (K % CK != 0). Without one (the chain GEMMs: K = 528) the A loads are a pointer plus
// a chunk offset and nothing is zeroed: no per-chunk index selects or masks on the VALU.
template <int WGM, int KS, int P, int KQ, int TI, int EPI, bool KT = true>
__global__ __launch_bounds__(64 * WGM * KS, (WGM * KS + 3) / 4) void k_wbr(const GemmArgs g) {
#ifdef BCNF_PHASE_STAMPS
  unsigned long long wst_[6] = {0, 0, 0, 0, 0, 0};
  const unsigned long long wrt0_ = __builtin_amdgcn_s_memrealtime();
  WBR_ST(0);
#endif
  using T = WbCfg<WGM, KS, P, KQ, TI>;
  constexpr int CK = T::CK;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kh = wave / T::NT, wm = wave - kh * T::NT;
  const int c16 = lane & 15, qq = lane >> 4;
  const TileId tl = tile_id();
  const int z = tl.z, g1 = z / g.G0, g0 = z - g1 * g.G0;
  const float* __restrict__ A = g.A + g1 * g.sA1 + g0 * g.sA0;
  const float* __restrict__ B = g.B + g1 * g.sB1 + g0 * g.sB0;
  const int am0 = tl.y * T::BM + wm * 16 * TI, n0 = tl.x * T::BN;
  const int K = g.K, S = T::stride(K);
  // 1. A: this wave's 16 rows, its contiguous share of the chunks, the first P chunks issued now -- before anything
  //    else, from the first batch of kernel arguments (r05: behind the epilogue's context they waited for four
  //    dependent scalar-load round trips, ~2k cycles). A float4 wholly past K (K % 4 == 0) reads the row start
  //    instead and is zeroed before use.
  const float* pa[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i) pa[i] = A + (long long)min(am0 + 16 * i + c16, g.M - 1) * g.lda + 4 * KQ * qq;
  const int nchunk = (K + CK - 1) / CK;
  const int c_lo = kh * nchunk / KS, n = (kh + 1) * nchunk / KS - c_lo;
  const int clast = min(c_lo + (n > 0 ? n - 1 : 0), nchunk - 1);
  floatx4 buf[P][TI][KQ];
  auto load = [&](int u, int c) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int h = 0; h < KQ; ++h)
        buf[u][i][h] = ld4(pa[i] + (!KT || CK * c + 4 * KQ * qq + 4 * h < K ? CK * c + 4 * h : 4 * h - 4 * KQ * qq));
  };
#pragma unroll
  for (int u = 0; u < P; ++u) load(u, min(c_lo + u, clast));
  // the epilogue's context and operands (bias / G), its dropout state only at the epilogue (a pointer round trip)
  EpiCtx e = epi_ctx<EPI, false>(g, g1, g0);
  auto mine = [&](int f) { return KS == 1 || f % KS == kh; };     // accumulator tile f = i * TJ + j
  float pre[T::NF][4];
#pragma unroll
  for (int f = 0; f < T::NF; ++f)
    if (mine(f)) epi_pre<EPI>(g, e.X, am0 + 16 * (f / T::TJ) + 4 * qq, n0 + 16 * (f % T::TJ) + c16, pre[f]);
  // the last Linear's weights for the epilogue (EPI_ACT with lp, the block's last hidden layer): the tile's slice
  // Wl[j][n0 .. n0 + 47], j < 32, one coalesced float4 per thread (in flight with the band, stored to LDS at the merge)
  floatx4 wl4 = {0.f, 0.f, 0.f, 0.f};
  const int wlr = threadIdx.x / 12, wlc = 4 * (threadIdx.x % 12);
  if constexpr (EPI == EPI_ACT) {
    static_assert(TI == 1 && KS > 1, "last-Linear partials: one 16-row tile per wave, a KS merge");
    static_assert(64 * T::NW >= 32 * 12, "one float4 of the weight slice per thread");
    if (g.lp && wlr < g.lp_n && n0 + wlc < g.N) wl4 = ld4(g.lp_w + (long long)wlr * g.lp_wld + n0 + wlc);
  }
  // 2. the B band: piece p (1 KB) = LDS floats [256 p, 256 p + 256); lane l's float4 is column f / S, k = f % S
  //    (k >= K: padding, any valid source). (col, k) advance by a constant step per piece: one division per lane,
  //    not one per piece (r05)
  {
    const int np = T::band_floats(K) / 256;
    constexpr int STEP = 256 * T::NW;              // floats between a wave's consecutive pieces
    const int f0 = 256 * wave + 4 * lane;
    int col = f0 / S, k = f0 - col * S;
    const int dcol = STEP / S, dk = STEP - dcol * S, nlast = g.N - 1;
    const unsigned ldb = (unsigned)g.ldb;
    for (int p = wave; p < np; p += T::NW) {     // wave-uniform trip count
      const float* src = B + ((unsigned long long)(unsigned)min(n0 + col, nlast) * ldb + (unsigned)(k < K ? k : 0));
      k += dk;
      col += dcol;
      if (k >= S) {
        k -= S;
        ++col;
      }
      // the DMA as inline asm: hipcc's wait pass, seeing an LDS-DMA builtin before the K loop, puts a vmcnt(0) at
      // the loop head (it cannot bound the DMA against the band reads there), draining the A ring every iteration;
      // the explicit vmcnt(0) below retires these copies before anything reads the band
      const uint32_t dst = (uint32_t)(uintptr_t)(lds + 256 * p);
      uint32_t m0_saved;                          // m0 is reserved to the compiler: restored after the copy
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                   "s_mov_b32 m0, %0" : "=&s"(m0_saved) : "v"(src), "s"(dst) : "memory");
    }
  }
  floatx4 acc[T::NF];
#pragma unroll
  for (int f = 0; f < T::NF; ++f) acc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
  WBR_ST(1);
  // everything landed (every other wave's pieces too after the barrier)
  __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)
  raw_barrier();
  WBR_ST(2);
  const float* bs = lds + c16 * S + 4 * KQ * qq;  // column 16 j + c16 at k = CK c + 4 KQ q: bs + 16 j S + CK c
  // B fragments one chunk ahead (bq): a chunk's MFMAs never wait for their own ds_reads
  static_assert(KQ == 1, "the B prefetch holds one float4 per fragment and chunk");
  floatx4 bq[T::TJ];
#pragma unroll
  for (int j = 0; j < T::TJ; ++j) bq[j] = ld4(bs + 16 * j * S + CK * c_lo);
  for (int c = 0; c < n; c += P) {
#pragma unroll
    for (int u = 0; u < P; ++u) {
      if (c + u < n) {
        const int ck = c_lo + c + u;
#pragma unroll
        for (int h = 0; h < KQ; ++h) {
          floatx4 a[TI], b[T::TJ];
          const int cn = ck + 1 < c_lo + n ? ck + 1 : ck;
#pragma unroll
          for (int j = 0; j < T::TJ; ++j) {
            b[j] = bq[j];
            bq[j] = ld4(bs + 16 * j * S + CK * cn);
          }
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            a[i] = buf[u][i][h];
            if (KT && ck == nchunk - 1 && CK * ck + 4 * KQ * qq + 4 * h >= K) a[i] = floatx4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
              for (int j = 0; j < T::TJ; ++j)
                acc[i * T::TJ + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i * T::TJ + j], 0, 0, 0);
        }
      }
      load(u, min(c_lo + c + u + P, clast));
    }
  }
  WBR_ST(3);
  if constexpr (KS > 1) {    // the band is dead once every wave has finished its MFMAs: partials reuse its LDS
    raw_barrier();
    float* part = lds + (wm * T::NF) * KS * 256 + lane * 4;      // [wave tile][f][slice][64 lanes][4]
#pragma unroll
    for (int f = 0; f < T::NF; ++f)
      if (!mine(f)) st4(part + (f * KS + kh) * 256, acc[f]);
    if constexpr (EPI == EPI_ACT)
      if (g.lp && wlr < 32) st4(lds + T::LP_W + wlr * 52 + wlc, wl4);
    __syncthreads();
#pragma unroll
    for (int f = 0; f < T::NF; ++f)
      if (mine(f)) {
        floatx4 s = kh == 0 ? acc[f] : ld4(part + (f * KS) * 256);
#pragma unroll
        for (int h = 1; h < KS; ++h) {
          const floatx4 p = h == kh ? acc[f] : ld4(part + (f * KS + h) * 256);
          s = floatx4{s[0] + p[0], s[1] + p[1], s[2] + p[2], s[3] + p[3]};
        }
        acc[f] = s;
      }
  }
  WBR_ST(4);
  epi_rng<EPI>(g, e);
  float act[T::NF][4];
#pragma unroll
  for (int f = 0; f < T::NF; ++f)
    if (mine(f)) {
      const float v[4] = {acc[f][0], acc[f][1], acc[f][2], acc[f][3]};
      const int rb = am0 + 16 * (f / T::TJ) + 4 * qq, col = n0 + 16 * (f % T::TJ) + c16;
      epi4<EPI>(g, e.C, e.X, rb, col, v, epi_rnd<EPI>(g, e, rb, col), pre[f], 1, act[f]);
    }
  if constexpr (EPI == EPI_ACT && KS > 1) {
    if (g.lp) {
      // the block's last Linear over this tile's 48 columns on the matrix cores: each owner wave transposes its
      // sub-tiles' activations through LDS into A operands (A[m = lane & 15][k = lane >> 4]) and accumulates
      // rows x (32 outputs); the owner waves of a row strip are then summed in K-slice order, and one partial per
      // (row, column tile) goes out -- the link sums the column tiles' partials in order instead of 528-long dots
      float* Tt = lds + T::LP_T + wave * 272;
      floatx4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int f = 0; f < T::NF; ++f)
        if (mine(f)) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) Tt[(4 * qq + rr) * 17 + c16] = act[f][rr];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            // A[m = lane & 15][k = lane >> 4] = activation (row m, column 16 f + 4 s + k);
            // B[k][n = lane & 15] = Wl[16 h + n][16 f + 4 s + k]
            const float a = Tt[c16 * 17 + 4 * s4 + qq];
            const float* wb = lds + T::LP_W + c16 * 52 + 16 * f + 4 * s4 + qq;
            d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, wb[0], d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, wb[16 * 52], d1, 0, 0, 0);
          }
        }
      float* Mm = lds + T::LP_M + (wm * KS + kh) * 512 + lane * 4;
      st4(Mm, d0);
      st4(Mm + 256, d1);
      __syncthreads();
      if (kh == 0) {
        const float* M0 = lds + T::LP_M + wm * KS * 512 + lane * 4;
        floatx4 s0 = ld4(M0), s1 = ld4(M0 + 256);
#pragma unroll
        for (int h = 1; h < KS; ++h) {
          const floatx4 p0 = ld4(M0 + h * 512), p1 = ld4(M0 + h * 512 + 256);
          s0 = floatx4{s0[0] + p0[0], s0[1] + p0[1], s0[2] + p0[2], s0[3] + p0[3]};
          s1 = floatx4{s1[0] + p1[0], s1[1] + p1[1], s1[2] + p1[2], s1[3] + p1[3]};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = am0 + 4 * qq + i;
          if (row < g.M) {
            float* o = g.lp + (long long)row * g.lp_ld + 32 * tl.x;
            o[c16] = s0[i];
            o[16 + c16] = s1[i];
          }
        }
      }
    }
  }
#ifdef BCNF_PHASE_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  WBR_ST(5);
  const int tix_ = tl.x + gridDim.x * (tl.y + gridDim.y * tl.z);
  if (threadIdx.x == 0 && tix_ < 256) {
    unsigned long long* o = g_wbr_st + 8 * tix_;
    for (int i = 1; i < 6; ++i) o[i - 1] = wst_[i] - wst_[0];
    o[5] = __builtin_amdgcn_s_memrealtime() - wrt0_;
    o[6] = wst_[5] - wst_[0];
    o[7] = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);   // dispatch order
  }
#endif
}

// ------------------------------------------------------------------------------------------------
// Link kernels: one 32-lane half-wavefront per sample, 8 samples per 256-thread workgroup.
//   * The sample's D-vector is lane-distributed (lane i < D holds element i); vectors every lane needs (u_in, v,
//     dO) go through LDS, so no register array is ever indexed by a runtime value.
//   * The long dot products (last Linear: 2 nout outputs over HP inputs; Linear-1 input-part backward: nin outputs)
//     are lane-split over float4 chunks, then reduced through an LDS transpose: lane j sums the 32 partials of j.
//   * TS / HS: side of the virtual block whose tail / head the launch runs (0 = nn_a, 1 = nn_b of a two_way
//     coupling; always 0 for one-way stacks), so every per-side width is a compile-time constant when DD is.
// ------------------------------------------------------------------------------------------------
constexpr int LR = 8;          // samples per link workgroup
constexpr int MQ = 5;          // float4 chunks per lane prefetched into registers (rows of up to 640 floats)
constexpr int LP_MAX = 16;     // column-tile partials of the last Linear (tiling W: ceil(HP / 48) <= 16 at K <= 768)

// Global -> LDS copy of n4 float4 by the whole workgroup with 8 loads in flight per thread (a plain copy loop
// serialises one L2 round trip per iteration).
__device__ __forceinline__ void stage4(float* __restrict__ dst, const float* __restrict__ src, int n4) {
  for (int e0 = 0; e0 < n4; e0 += 8 * WWG) {
    floatx4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * WWG + (int)threadIdx.x;
      if (e < n4) v[u] = ld4(src + 4 * e);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * WWG + (int)threadIdx.x;
      if (e < n4) st4(dst + 4 * e, v[u]);
    }
  }
}

// Two regions staged with every load in flight at once (one memory round trip for up to 16 float4 per thread). Every
// workgroup of a link launch stages the SAME weights: the copy starts at a per-workgroup offset (whole 128-B lines,
// spread over the XCD's 32 concurrent workgroups, b >> 3) so that they do not all request the same L2 lines in the
// same order.
__device__ __forceinline__ void stage4x2(float* __restrict__ d1, const float* __restrict__ s1, int n1,
                                         float* __restrict__ d2, const float* __restrict__ s2, int n2) {
  const int n = n1 + n2;
  // (b >> 3) & 31 < 32, so rot <= 31 * (n >> 5) < n at any grid size (a launch of more than 256 workgroups, B > 2048
  // rows, wraps back to offset 0 instead of stepping past the end of the staged regions).
  const int rot = (int)(((blockIdx.x >> 3) & 31u) * (unsigned)(n >> 5)) & ~7;
  for (int e0 = 0; e0 < n; e0 += 16 * WWG) {
    floatx4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = e0 + u * WWG + (int)threadIdx.x;
      const int f = e + rot < n ? e + rot : e + rot - n;
      if (e < n) v[u] = f < n1 ? ld4(s1 + 4 * f) : ld4(s2 + 4 * (f - n1));
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = e0 + u * WWG + (int)threadIdx.x;
      const int f = e + rot < n ? e + rot : e + rot - n;
      if (e < n) {
        if (f < n1) st4(d1 + 4 * f, v[u]);
        else st4(d2 + 4 * (f - n1), v[u]);
      }
    }
  }
}

__device__ __forceinline__ float half_sum(float v) {      // sum over the 32 lanes of a half-wavefront
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, true));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, true));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, true));  // row_ror:2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, true));  // row_ror:1
  return v + __shfl_xor(v, 16);
}

struct LinkArgs {
  long long B;
  int vt, vh;                   // virtual block of the tail / of the head (-1: none)
  const float* prm;             // canonical flat parameters
  const float* pk;              // packed
  // tail
  const float* Alast;           // [B][HP] last hidden activation of block vt
  const float* Opart;           // nullable: the last Linear's per-column-tile partials of block vt (GemmArgs.lp),
  long long ldo; int nop;       //   Opart[row * ldo + 32 p + j], p < nop -- replaces the dot products over Alast
  const float* Xt;              // block vt's saved input rows (forward: pre-ActNorm x or mid-coupling state; inverse: v)
  float* S;                     // forward save: tanh(s) of block vt [B][SP] (nullable)
  float* z;                     // last block: z / inverse output y [B][D] (ld D)
  float* ldj;                   // [B]
  float* nllp;                  // last block: 0.5 |z|^2 - ldj per row (nullable)
  // head
  const float* xin;             // head-only launch: input rows (ld D): y (forward) or z (inverse)
  float* Xh;                    // block vh's saved input rows [B][XP]
  const float* P; long long ldP; const int64_t* cidx;   // hoisted projection rows (row r uses cidx[r])
  float* A0; float* G0;         // [B][HP] first hidden activation and its derivative factor (G0 nullable)
  float* U;                     // forward save: [u_in | 1 | 0] of block vh [B][UP] (nullable)
  const uint64_t* rng;          // dropout (nullable = off)
  unsigned long long* dbg;      // phase timestamps of workgroup 0 (bcnf_wide_debug_phases), nullable
};

// Phase stamps of the forward link: diagnostic build only (-DBCNF_PHASE_STAMPS, tools/exp_variants.sh).
#ifdef BCNF_PHASE_STAMPS
#define LINK_STAMP(i)                                                                          \
  do {                                                                                         \
    if (a.dbg && a.vt >= 0 && a.vh >= 0 && blockIdx.x == 0 && threadIdx.x == 0)                \
      a.dbg[i] = __builtin_amdgcn_s_memtime();                                                 \
  } while (0)
#else
#define LINK_STAMP(i) do {} while (0)
#endif

// Dropout mask for a float4 group (4 consecutive columns n..n+3 of one row).
__device__ __forceinline__ uint4 drop4(uint64_t seed, uint64_t offs, long long row, int n, uint32_t tag) {
  return philox4x32_10(make_uint4((uint32_t)row, (uint32_t)n | 0x80000000u, tag, (uint32_t)offs),
                       make_uint2((uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(offs >> 32)));
}

__host__ __device__ inline int link_ps(const WideLayout& L) { return (L.WL > L.WY ? L.WL : L.WY) + 1; }

// LDS floats of a link launch: [last-Linear rows][W0y^T rows][Q][partials][8 x 3 x 32 vectors]
__host__ __device__ inline int link_lds_floats(const WideLayout& L, bool w_last, bool w_first) {
  return (w_last ? L.WL * L.HP : 0) + (w_first ? L.WY * L.HP : 0) + pad4(L.D * L.D) + pad4(LR * 32 * link_ps(L)) +
         LR * 96;
}

// Forward (INV = false): tail(vt) = last Linear, t / tanh(s), x_T = exp(s) x_T + t on the half's transformed part,
//                        ldj += sum s, x Q after a block's last half;
//                        head(vh) = ActNorm before a block's first half, Linear-1 from P + u_in W0y^T + b0, GELU,
//                        dropout.   (cnf.py:165-196, 333-335, 348-351)
// Inverse (INV = true):  head(vh) = v = x Q^T before a block's first processed half; tail(vt) =
//                        x_T = (x_T - t) exp(-s), ActNorm^-1 after its last half. The reference's two_way inverse
//                        (cnf.py:198-213) runs nn_a then nn_b, both on the current state -- not the true inverse; the
//                        processing order of the host loop reproduces exactly that.   (cnf.py:337-339, 353-354)
// DD > 0: the sample dimension D as a compile-time constant (every loop over D and the per-side widths fully
// unrolled); DD = 0: runtime D (any D <= 32).
template <bool INV, int DD, int TS, int HS>
__global__ __launch_bounds__(WWG) void k_wlink(const WideLayout L, const LinkArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, ln = tid & 31, r = tid >> 5;
  const int HP = L.HP, H = L.H;
  const int D = DD ? DD : L.D, Da = DD ? (DD + 1) / 2 : L.Da, Db = DD ? DD / 2 : L.Db;
  const int nout_t = TS ? Da : Db, toff_t = TS ? 0 : Da, O2 = 2 * nout_t;
  const int nin_h = HS ? Db : Da, ioff_h = HS ? Da : 0;
  const int PS = link_ps(L);
  const int nq = HP / 4;
  const int vt = a.vt, vh = a.vh;
  const int kt = vt >= 0 ? vt / L.S : -1, kh = vh >= 0 ? vh / L.S : -1;
  const bool t_first = vt >= 0 && vt % L.S == 0, t_last = vt >= 0 && vt % L.S == L.S - 1;
  const bool h_first = vh >= 0 && vh % L.S == 0;
  LINK_STAMP(0);
  float* Wl = sm;
  float* W0 = Wl + (vt >= 0 ? L.WL * HP : 0);
  float* Qs = W0 + (vh >= 0 ? L.WY * HP : 0);
  float* part = Qs + pad4(D * D);
  float* Os = part + pad4(LR * 32 * PS) + r * 96;
  float* vs = Os + 32;
  float* us = vs + 32;
  // the orthonormal matrix this launch applies: forward after the tail block's last half, inverse before the head
  // block's first processed half
  const int kq = INV ? (h_first ? kh : -1) : (t_last ? kt : -1);
  const long long row = (long long)blockIdx.x * LR + r;
  const bool valid = row < a.B;
  const bool lv = valid && ln < D;
  // The sample's HBM rows (last activation of block vt, projection row of block vh, saved input) are requested
  // first, so their latency overlaps the weight staging instead of serialising inside the dot-product loops.
  floatx4 ach[MQ], pch[MQ];
  const bool dots = vt >= 0 && !a.Opart;          // the last Linear here (else its partials come with the tail)
  const float* arow = dots ? a.Alast + row * HP : nullptr;
  const float* Pr = nullptr;
  if (vh >= 0) Pr = a.P + (a.cidx && valid ? a.cidx[row] : row) * a.ldP + (long long)vh * HP;
#pragma unroll
  for (int t = 0; t < MQ; ++t) {
    const int q = ln + 32 * t;
    if (valid && q < nq) {
      if (dots) ach[t] = ld4(arow + 4 * q);
      if (vh >= 0) pch[t] = ld4(Pr + 4 * q);
    }
  }
  float opv[LP_MAX];
  if (vt >= 0 && !dots) {
#pragma unroll
    for (int p = 0; p < LP_MAX; ++p)
      opv[p] = (valid && ln < O2 && p < a.nop) ? a.Opart[row * a.ldo + 32 * p + ln] : 0.f;
  }
  float xpre = 0.f;
  if (lv) xpre = vt >= 0 ? a.Xt[row * L.XP + ln] : a.xin[row * D + ln];
  // every other global operand of the launch, also up front (a load behind a global store in a loop cannot be
  // hoisted by the compiler, and each one left in the body is a full memory round trip on the critical path)
  floatx4 bch[MQ];
  if (vh >= 0) {
    const float* b0 = a.pk + L.pk_b0 + (long long)vh * HP;
#pragma unroll
    for (int t = 0; t < MQ; ++t)
      if (valid && ln + 32 * t < nq) bch[t] = ld4(b0 + 4 * (ln + 32 * t));
  }
  const bool has_q = kq >= 0 && kq < L.nb - 1;
  float qv[4] = {0.f, 0.f, 0.f, 0.f};       // D * D <= 1024 = 4 per thread
  if (has_q)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (tid + u * WWG < D * D) qv[u] = a.pk[L.pk_q + (long long)kq * D * D + tid + u * WWG];
  const float blast = (vt >= 0 && ln < O2) ? a.prm[vbase(L, vt) + L.lin_b[vt % L.S][L.NH] + ln] : 0.f;
  float sct = 1.f, bct = 0.f, sch = 1.f, bch_an = 0.f, ldj0 = 0.f, ldc_h = 0.f;
  if (ln < D) {
    if (vt >= 0 && L.an && kt < L.nb - 1) {
      sct = a.prm[(long long)kt * L.blk_stride + ln];
      bct = a.prm[(long long)kt * L.blk_stride + D + ln];
    }
    if (vh >= 0 && L.an && kh < L.nb - 1) {
      sch = a.prm[(long long)kh * L.blk_stride + ln];
      bch_an = a.prm[(long long)kh * L.blk_stride + D + ln];
    }
  }
  if (!INV && valid && ln == 0) {
    if (vt >= 0) ldj0 = a.ldj[row];
    if (vh >= 0 && L.an && kh < L.nb - 1) ldc_h = a.pk[L.pk_ldc + kh];
  }
  stage4x2(Wl, a.pk + L.pk_wl + (long long)(vt >= 0 ? vt : 0) * L.WL * HP, dots ? O2 * HP / 4 : 0,
           W0, a.pk + L.pk_w0y + (long long)(vh >= 0 ? vh : 0) * L.WY * HP, vh >= 0 ? nin_h * HP / 4 : 0);
  if (has_q)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (tid + u * WWG < D * D) Qs[tid + u * WWG] = qv[u];
  __syncthreads();
  LINK_STAMP(1);
  uint64_t seed = 0, offs = 0;
  if (a.rng) {
    seed = a.rng[0];
    offs = a.rng[1];
  }
  float xi = 0.f;                                   // element ln of the sample's D-vector
  // ------------------------------------------------------------ tail of virtual block vt
  if (vt >= 0 && !dots) {                          // the partials of the chain's last GEMM, summed in column order
    if (ln < O2) {
      float sp = opv[0];
#pragma unroll
      for (int p = 1; p < LP_MAX; ++p) sp += opv[p];  // zero past nop
      Os[ln] = sp + blast;
    }
    __syncthreads();
  }
  if (vt >= 0) {
    const int st = vt % L.S;
    float acc[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) acc[j] = 0.f;
    if (dots) {
      if (valid) {
        auto chunk = [&](int q, floatx4 av) {
#pragma unroll
          for (int j = 0; j < DM; ++j) {
            if (j < O2) {
              const floatx4 w = ld4(Wl + j * HP + 4 * q);
              acc[j] = fmaf(av.x, w.x, fmaf(av.y, w.y, fmaf(av.z, w.z, fmaf(av.w, w.w, acc[j]))));
            }
          }
        };
#pragma unroll
        for (int t = 0; t < MQ; ++t)
          if (ln + 32 * t < nq) chunk(ln + 32 * t, ach[t]);
        for (int q = ln + 32 * MQ; q < nq; q += 32) chunk(q, ld4(arow + 4 * q));
      }
#pragma unroll
      for (int j = 0; j < DM; ++j)
        if (j < O2) part[(r * 32 + ln) * PS + j] = acc[j];
      LINK_STAMP(2);
      __syncthreads();
      if (ln < O2) {
        float s = 0.f;
#pragma unroll
        for (int l = 0; l < 32; ++l) s += part[(r * 32 + l) * PS + ln];
        Os[ln] = s + blast;
      }
      __syncthreads();
    }
    LINK_STAMP(3);
    float sj = 0.f;
    const int jt = ln - toff_t;
    const bool tl = lv && jt >= 0 && jt < nout_t;             // lane in the transformed part
    if (lv) {
      xi = xpre;
      if (!INV) {
        if (t_first && L.an && kt < L.nb - 1) xi = sct * xi + bct;                 // ActNorm (cnf.py:350)
        if (tl) {
          sj = tanh_bf(Os[nout_t + jt]);
          xi = fmaf(exp_fast(sj), xi, Os[jt]);                    // x_T = exp(s) x_T + t (cnf.py:179, 184)
          if (a.S) a.S[row * L.SP + jt] = sj;
        }
      } else {
        if (tl) xi = (xi - Os[jt]) * exp_fast(-tanh_bf(Os[nout_t + jt]));   // (x_T - t) exp(-s) (cnf.py:201, 208)
        if (t_last && L.an && kt < L.nb - 1) xi = (xi - bct) / sct;            // ActNorm inverse (cnf.py:354)
      }
    }
    if (!INV) {
      const float ssum = half_sum(sj);
      if (vt < L.nv - 1) {
        if (t_last) {                                             // x Q_k (cnf.py:333-335)
          vs[ln] = xi;
          __syncthreads();
          float c = 0.f;
          if (ln < D) {
#pragma unroll
            for (int i = 0; i < DM; ++i)
              if (i < D) c = fmaf(vs[i], Qs[i * D + ln], c);
          }
          xi = c;
        }
        ldj0 += ssum;
      } else {
        const float zz = half_sum(xi * xi);
        if (lv) a.z[row * D + ln] = xi;
        if (valid && ln == 0) {
          const float lj = ldj0 + ssum;
          a.ldj[row] = lj;
          if (a.nllp) a.nllp[row] = 0.5f * zz - lj;               // per-sample inn_nll_loss (utils.py:49-53)
        }
      }
    } else if (t_last && kt == 0 && lv) {
      a.z[row * D + ln] = xi;
    }
  } else {
    xi = xpre;
    ldj0 = 0.f;
  }
  // ------------------------------------------------------------ head of virtual block vh
  if (vh >= 0) {
    if (!INV) {
      if (lv) a.Xh[row * L.XP + ln] = xi;                         // saved input (pre-ActNorm for a first half)
      if (h_first && L.an && kh < L.nb - 1) {
        if (ln < D) xi = sch * xi + bch_an;
        ldj0 += ldc_h;                                            // ActNorm log|det J| (cnf.py:349)
      }
    } else {
      if (h_first && kh < L.nb - 1) {                             // v = x Q_k^T (cnf.py:337-339)
        vs[ln] = xi;
        __syncthreads();
        float c = 0.f;
        if (ln < D) {
#pragma unroll
          for (int j = 0; j < DM; ++j)
            if (j < D) c = fmaf(vs[j], Qs[ln * D + j], c);
        }
        xi = c;
      }
      if (lv) a.Xh[row * L.XP + ln] = xi;                         // read back by this half's tail
    }
    if (!INV && valid && ln == 0) a.ldj[row] = ldj0;             // the running log|det J| of the sample
    LINK_STAMP(4);
    us[ln] = xi;
    __syncthreads();
    LINK_STAMP(5);
    float ua[DM / 2];
#pragma unroll
    for (int j = 0; j < DM / 2; ++j) ua[j] = j < nin_h ? us[ioff_h + j] : 0.f;
    if (a.U && valid && ln < L.UP) a.U[row * L.UP + ln] = ln < nin_h ? us[ioff_h + ln] : (ln == nin_h ? 1.f : 0.f);
    if (valid) {
      const float* b0 = a.pk + L.pk_b0 + (long long)vh * HP;
      const uint32_t tag = (uint32_t)vh * 16u;
      auto chunk = [&](int q, floatx4 pv4, floatx4 bv4) {
        const int n = 4 * q;
        floatx4 pre = pv4 + bv4;
#pragma unroll
        for (int j = 0; j < DM / 2; ++j) {
          if (j < nin_h) {
            const floatx4 w = ld4(W0 + j * HP + n);
            pre.x = fmaf(ua[j], w.x, pre.x);
            pre.y = fmaf(ua[j], w.y, pre.y);
            pre.z = fmaf(ua[j], w.z, pre.z);
            pre.w = fmaf(ua[j], w.w, pre.w);
          }
        }
        uint4 rnd = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
        if (a.rng) rnd = drop4(seed, offs, row, n, tag);
        float av[4], gv[4];
        const float pv[4] = {pre.x, pre.y, pre.z, pre.w};
        const uint32_t rv[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = n + e;
          float ge, dg;
          gelu_fg(pv[e], ge, dg);
          const float m = (c < H) ? (a.rng ? (rv[e] >= L.thresh ? L.keep_scale : 0.f) : 1.f) : 0.f;
          av[e] = c == H ? 1.f : ge * m;
          gv[e] = dg * m;
        }
        st4_wt_ordered(a.A0 + row * HP + n, floatx4{av[0], av[1], av[2], av[3]});   // may alias Alast (eval, NH odd)
        if (a.G0) st4_wt(a.G0 + row * HP + n, floatx4{gv[0], gv[1], gv[2], gv[3]});
      };
#pragma unroll
      for (int t = 0; t < MQ; ++t)
        if (ln + 32 * t < nq) chunk(ln + 32 * t, pch[t], bch[t]);
      for (int q = ln + 32 * MQ; q < nq; q += 32) chunk(q, ld4(Pr + 4 * q), ld4(b0 + 4 * q));
    }
  }
  LINK_STAMP(6);
}

// Backward links (forward order reversed, one virtual block = one half-coupling).
//   head-B(v): dv = dX Q_k^T after a block's last half (k < nb-1), or dX = dz (final half); half-coupling backward on
//              the transformed part -> dO = [dt, ds'] (stored), d x_T and the untouched input part (stored in DV);
//              dZ_{NH-1} = (dO W_NH) * G_{NH-1} (stored).
//   tail-B(v): d x_in = DV_in + dZ_0 W0y on the input part; ActNorm backward before a block's first half (per-row
//              partials of dscale, dbias) -> dX of the previous half.
// One launch = tail-B(vt) then head-B(vt - 1) (vt = -1: head-B(nv-1) only).
struct LinkBArgs {
  long long B;
  int vt, vh;
  const float* prm; const float* pk;
  const float* X;  long long sX;      // saved half inputs, virtual block v at X + v * sX
  const float* S;  long long sS;      // saved tanh(s)
  const float* dz; const float* dldj; // head-B(nv-1) input (dz nullable in NLL mode), dldj nullable
  const float* zn; const float* dvals; int nll;   // NLL mode: dz = z g / B, dldj = -g / B, g = dvals[0] + dvals[1]
  // tail-B(vt)
  const float* dZ0; long long ldZ0;   // dZ_0 of block vt (row stride ldZ0)
  float* DV;                          // [B][XP]: d(input part) | d(transformed part)  (head-B -> tail-B)
  float* ANP;                         // [B][AP] ActNorm partials of real block vt / S (du*x | du)
  float* dy;                          // vt == 0: dL/dy (nullable)
  // head-B(vh)
  float* Ob;                          // [B][OP] dO of block vh
  const float* Gl;                    // [B][HP] G_{NH-1} of block vh
  float* dZl;  long long ldZl;        // dZ_{NH-1} of block vh
};

template <int DD, int TS, int HS>
__global__ __launch_bounds__(WWG) void k_wlink_bwd(const WideLayout L, const LinkBArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, ln = tid & 31, r = tid >> 5;
  const int HP = L.HP;
  const int D = DD ? DD : L.D, Da = DD ? (DD + 1) / 2 : L.Da, Db = DD ? DD / 2 : L.Db;
  const int nin_t = TS ? Db : Da, ioff_t = TS ? Da : 0;
  const int nout_h = HS ? Da : Db, toff_h = HS ? 0 : Da, O2 = 2 * nout_h;
  const int PS = link_ps(L);
  const int nq = HP / 4;
  const int vt = a.vt, vh = a.vh;
  const int kt = vt >= 0 ? vt / L.S : -1, kh = vh >= 0 ? vh / L.S : -1;
  const bool t_first = vt >= 0 && vt % L.S == 0;
  const bool h_first = vh >= 0 && vh % L.S == 0, h_last = vh >= 0 && vh % L.S == L.S - 1;
  float* Wl = sm;                                   // [2 nout][HP] last Linear of block vh
  float* W0 = Wl + (vh >= 0 ? L.WL * HP : 0);       // [nin][HP] W0y^T of block vt
  float* Qs = W0 + (vt >= 0 ? L.WY * HP : 0);
  float* part = Qs + pad4(D * D);
  float* Os = part + pad4(LR * 32 * PS) + r * 96;
  float* vs = Os + 32;
  const long long row = (long long)blockIdx.x * LR + r;
  const bool valid = row < a.B;
  const bool lv = valid && ln < D;
  // HBM rows first (dZ_0 of block vt, G of block vh, per-sample vectors), then the weight staging
  floatx4 zch[MQ], gch[MQ];
  const float* zr = vt >= 0 ? a.dZ0 + row * a.ldZ0 : nullptr;
  const float* gr = vh >= 0 ? a.Gl + row * HP : nullptr;
#pragma unroll
  for (int t = 0; t < MQ; ++t) {
    const int q = ln + 32 * t;
    if (valid && q < nq) {
      if (vt >= 0) zch[t] = ld4(zr + 4 * q);
      if (vh >= 0) gch[t] = ld4(gr + 4 * q);
    }
  }
  const int jh = ln - toff_h;
  const bool hl = lv && vh >= 0 && jh >= 0 && jh < nout_h;  // lane in head block's transformed part
  float dvp = 0.f, xkt = 0.f, xkh = 0.f, skh = 0.f;
  if (lv) {
    if (vt >= 0) {
      dvp = a.DV[row * L.XP + ln];
      xkt = a.X[vt * a.sX + row * L.XP + ln];
    }
    if (vh >= 0) {
      xkh = a.X[vh * a.sX + row * L.XP + ln];
      if (hl) skh = a.S[vh * a.sS + row * L.SP + jh];
    }
  }
  // the remaining global operands, up front as well
  const bool has_q = vh >= 0 && h_last && kh < L.nb - 1;
  float qv[4] = {0.f, 0.f, 0.f, 0.f};       // D * D <= 1024 = 4 per thread
  if (has_q)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (tid + u * WWG < D * D) qv[u] = a.pk[L.pk_q + (long long)kh * D * D + tid + u * WWG];
  float sct = 1.f, sch = 1.f, bch_an = 0.f, dlp = 0.f;
  if (ln < D) {
    if (vt >= 0 && L.an && kt < L.nb - 1) sct = a.prm[(long long)kt * L.blk_stride + ln];
    if (vh >= 0 && L.an && kh < L.nb - 1) {
      sch = a.prm[(long long)kh * L.blk_stride + ln];
      bch_an = a.prm[(long long)kh * L.blk_stride + D + ln];
    }
  }
  const float gscale = a.nll ? (a.dvals ? a.dvals[0] + a.dvals[1] : 1.f) / (float)a.B : 0.f;
  if (hl && !a.nll && a.dldj) dlp = a.dldj[row];
  stage4x2(W0, a.pk + L.pk_w0y + (long long)(vt >= 0 ? vt : 0) * L.WY * HP, vt >= 0 ? nin_t * HP / 4 : 0,
           Wl, a.pk + L.pk_wl + (long long)(vh >= 0 ? vh : 0) * L.WL * HP, vh >= 0 ? O2 * HP / 4 : 0);
  if (has_q)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (tid + u * WWG < D * D) Qs[tid + u * WWG] = qv[u];
  __syncthreads();
  float dxi = 0.f;                                  // element ln of the gradient w.r.t. the current D-vector
  // ------------------------------------------------------------ tail-B of virtual block vt
  if (vt >= 0) {
    float acc[DM / 2];
#pragma unroll
    for (int j = 0; j < DM / 2; ++j) acc[j] = 0.f;
    if (valid) {
      auto chunk = [&](int q, floatx4 dzv) {
#pragma unroll
        for (int j = 0; j < DM / 2; ++j) {
          if (j < nin_t) {
            const floatx4 w = ld4(W0 + j * HP + 4 * q);
            acc[j] = fmaf(dzv.x, w.x, fmaf(dzv.y, w.y, fmaf(dzv.z, w.z, fmaf(dzv.w, w.w, acc[j]))));
          }
        }
      };
#pragma unroll
      for (int t = 0; t < MQ; ++t)
        if (ln + 32 * t < nq) chunk(ln + 32 * t, zch[t]);
      for (int q = ln + 32 * MQ; q < nq; q += 32) chunk(q, ld4(zr + 4 * q));
    }
#pragma unroll
    for (int j = 0; j < DM / 2; ++j)
      if (j < nin_t) part[(r * 32 + ln) * PS + j] = acc[j];
    __syncthreads();
    if (lv) {
      float du = dvp;
      const int ji = ln - ioff_t;
      if (ji >= 0 && ji < nin_t) {
        float t = 0.f;
#pragma unroll
        for (int l = 0; l < 32; ++l) t += part[(r * 32 + l) * PS + ji];
        du += t;                                                  // d x_in = dv_in + dZ_0 W0y
      }
      if (t_first && L.an && kt < L.nb - 1) {
        a.ANP[row * L.AP + ln] = du * xkt;                       // dscale partial
        a.ANP[row * L.AP + D + ln] = du;                         // dbias partial
        du *= sct;
      }
      dxi = du;
      if (vt == 0 && a.dy) a.dy[row * D + ln] = dxi;
    }
  } else if (lv) {
    dxi = a.nll ? a.zn[row * D + ln] * gscale : (a.dz ? a.dz[row * D + ln] : 0.f);
  }
  // ------------------------------------------------------------ head-B of virtual block vh
  if (vh >= 0) {
    if (h_last && kh < L.nb - 1) {                                // dv = dX Q_k^T
      vs[ln] = dxi;
      __syncthreads();
      float c = 0.f;
      if (ln < D) {
#pragma unroll
        for (int j = 0; j < DM; ++j)
          if (j < D) c = fmaf(vs[j], Qs[ln * D + j], c);
      }
      dxi = c;
    }
    float dvo = dxi;
    if (hl) {
      const float dl = a.nll ? -gscale : dlp;
      float ub = xkh;
      if (h_first && L.an && kh < L.nb - 1) ub = sch * ub + bch_an;
      const float s = skh;
      const float es = exp_fast(s);
      dvo = dxi * es;                                             // d x_T before the affine
      Os[jh] = dxi;                                               // dt
      Os[nout_h + jh] = fmaf(dxi * ub, es, dl) * (1.f - s * s);   // d s' (through tanh and the log-det)
    }
    if (valid && ln < L.XP) a.DV[row * L.XP + ln] = ln < D ? dvo : 0.f;
    __syncthreads();
    if (valid) {
      if (ln < L.OP) a.Ob[row * L.OP + ln] = ln < O2 ? Os[ln] : 0.f;
      float dO[DM];
#pragma unroll
      for (int j = 0; j < DM; ++j) dO[j] = j < O2 ? Os[j] : 0.f;
      float* out = a.dZl + row * a.ldZl;
      auto chunk = [&](int q, floatx4 gv) {
        const int n = 4 * q;
        floatx4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < DM; ++j) {
          if (j < O2) {
            const floatx4 w = ld4(Wl + j * HP + n);
            s4.x = fmaf(dO[j], w.x, s4.x);
            s4.y = fmaf(dO[j], w.y, s4.y);
            s4.z = fmaf(dO[j], w.z, s4.z);
            s4.w = fmaf(dO[j], w.w, s4.w);
          }
        }
        st4_wt(out + n, s4 * gv);
      };
#pragma unroll
      for (int t = 0; t < MQ; ++t)
        if (ln + 32 * t < nq) chunk(ln + 32 * t, gch[t]);
      for (int q = ln + 32 * MQ; q < nq; q += 32) chunk(q, ld4(gr + 4 * q));
    }
  }
}

// ActNorm gradients of every block: dscale_i = sum_b du_i x_i + (sum_b dldj_b) / scale_i  (the log|scale| term of
// ActNorm.log_det_J, cnf.py:349), dbias_i = sum_b du_i. Fixed-order reduction, one workgroup per block.
__global__ __launch_bounds__(WWG) void k_wactnorm_grad(const WideLayout L, const float* __restrict__ ANP, long long B,
                                                       const float* __restrict__ dldj, const float* __restrict__ zn,
                                                       const float* __restrict__ dvals, int nll,
                                                       const float* __restrict__ prm, float* __restrict__ dprm, int k0) {
  __shared__ float red[WWG];
  __shared__ float dsum_s;
  const int k = k0 + (int)blockIdx.x, tid = threadIdx.x;
  const int ncol = 2 * L.D;
  const float* P = ANP + (long long)k * B * L.AP;
  // sum of dldj over the batch
  float acc = 0.f;
  if (nll) {
    if (tid == 0) acc = -(dvals ? dvals[0] + dvals[1] : 1.f);
  } else if (dldj) {
    for (long long r = tid; r < B; r += WWG) acc += dldj[r];
  }
  red[tid] = acc;
  __syncthreads();
  for (int w = WWG / 2; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) dsum_s = red[0];
  __syncthreads();
  const float dsum = dsum_s;
  // columns: 4 row phases x 64 columns
  const int c = tid & 63, ph = tid >> 6;
  float s = 0.f;
  if (c < ncol) {                      // 8 independent chains per thread keep 8 loads in flight
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    long long r = ph;
    for (; r + 28 < B; r += 32)
#pragma unroll
      for (int u = 0; u < 8; ++u) s8[u] += P[(r + 4 * u) * L.AP + c];
    for (; r < B; r += 4) s8[0] += P[r * L.AP + c];
    s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  }
  __syncthreads();
  red[tid] = s;
  __syncthreads();
  if (ph == 0 && c < ncol) {
    float t = (red[c] + red[64 + c]) + (red[128 + c] + red[192 + c]);
    const long long base = (long long)k * L.blk_stride;
    if (c < L.D) t += dsum / prm[base + c];
    dprm[base + c] = t;
  }
  (void)zn;
}

// Mean of the per-sample NLL terms -> [loss, nll, mse = 0] (trainer.py:260-266) plus the dropout RNG advance and
// the divergence guard, exactly as bcnf_stack.hip's nll_finalize (include/bcnf_amd.h, BCNF_GUARD_*).
__global__ __launch_bounds__(WWG) void k_wnll_finalize(const float* __restrict__ part, long long B, float* __restrict__ out,
                                                       uint64_t* rng, int32_t* guard) {
  __shared__ float red[WWG];
  float acc = 0.f;
  for (long long i = threadIdx.x; i < B; i += WWG) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = WWG / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float nll = red[0] / (float)B;
    out[0] = nll;
    out[1] = nll;
    out[2] = 0.f;
    bool halt = false;
    if (guard) {
      if (guard[BCNF_GUARD_DIVERGED]) {
        guard[BCNF_GUARD_HALTED] = 1;
        halt = true;
      } else if (guard[BCNF_GUARD_CHECK] && (nll > 1e5f || isnan(nll))) {
        guard[BCNF_GUARD_DIVERGED] = 1;
      }
    }
    if (rng && !halt) rng[1] += 1;
  }
}

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------
bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

GemmArgs gemm_args(int tiling, int M, int N, int K, const float* A, long long lda, const float* B, long long ldb,
                   float* C, long long ldc) {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.tiling = tiling;
  g.M = M;
  g.N = N;
  g.K = K;
  g.G0 = 1;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.keep_scale = 1.f;
  g.cb_S = 1;
  return g;
}

template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI>
int launch_cfg(const GemmArgs& g, int groups, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, groups);
  hipLaunchKernelGGL((k_wgemm<BM, BN, BK, AKC, BKC, EPI>), grid, dim3(WWG), 0, st, g);
  return bcnf_rt::launched();
}

template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI, int NW = 4, bool FULL = false>
int launch_cfg16(const GemmArgs& g, int groups, hipStream_t st) {
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, groups);
  hipLaunchKernelGGL((k_wgemm16<BM, BN, BK, AKC, BKC, EPI, NW, FULL>), grid, dim3(64 * NW), 0, st, g);
  return bcnf_rt::launched();
}

template <int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, int EPI, int S, int KS = 2>
int launch_gl(const GemmArgs& g, int groups, hipStream_t st) {
  using T = GlCfg<BM, BN, WGM, WGN, AKC, BKC, S, KS>;
  constexpr int bytes = S * T::STG * 4;
  static bool attr = false;
  if (!attr) {
    if (const int rc = bcnf_rt::hip_status(hipFuncSetAttribute((const void*)k_wgl<BM, BN, WGM, WGN, AKC, BKC, EPI, S, KS>,
                                                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes)))
      return rc;
    attr = true;
  }
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, groups);
  hipLaunchKernelGGL((k_wgl<BM, BN, WGM, WGN, AKC, BKC, EPI, S, KS>), grid, dim3(64 * T::NW), bytes, st, g);
  return bcnf_rt::launched();
}

// Set by launch_wb when an EPI_ACT launch on tiling W carries GemmArgs.lp (only tiling W's epilogue writes the
// last-Linear partials): hidden_fwd reports the partials as written from this, not from a copy of the dispatch rule.
thread_local bool g_lp_written = false;

template <int WGM, int KS, int P, int KQ, int EPI, int TI = 1>
int launch_wb(const GemmArgs& g, int groups, hipStream_t st) {
  using T = WbCfg<WGM, KS, P, KQ, TI>;
  if (EPI == EPI_ACT && g.lp) g_lp_written = true;
  const int bytes = T::lds_floats(g.K) * 4;
  static bool attr = false;
  if (!attr) {
    if (const int rc = bcnf_rt::hip_status(hipFuncSetAttribute((const void*)k_wbr<WGM, KS, P, KQ, TI, EPI>,
                                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                                               T::lds_floats(T::KMAX) * 4)))
      return rc;
    attr = true;
  }
  dim3 grid((g.N + T::BN - 1) / T::BN, (g.M + T::BM - 1) / T::BM, groups);
  if (g.K % T::CK == 0) {
    static bool attr2 = false;
    if (!attr2) {
      if (const int rc = bcnf_rt::hip_status(hipFuncSetAttribute((const void*)k_wbr<WGM, KS, P, KQ, TI, EPI, false>,
                                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                                 T::lds_floats(T::KMAX) * 4)))
        return rc;
      attr2 = true;
    }
    hipLaunchKernelGGL((k_wbr<WGM, KS, P, KQ, TI, EPI, false>), grid, dim3(64 * T::NW), bytes, st, g);
    return bcnf_rt::launched();
  }
  hipLaunchKernelGGL((k_wbr<WGM, KS, P, KQ, TI, EPI>), grid, dim3(64 * T::NW), bytes, st, g);
  return bcnf_rt::launched();
}

// LDS-DMA tilings per operand layout (tiling C): 5 = auto, 6 = the large-tile variant forced
template <bool AKC, bool BKC, int EPI>
int gemm_gl(const GemmArgs& g, int groups, hipStream_t st, bool large);

constexpr int N_CU = 256;
// Modelled time of a tiling: rounds of one workgroup per CU (MI355X: 256 CUs) x tile area / relative efficiency.
double tile_cost(const GemmArgs& g, int groups, int BM, int BN, double eff) {
  const long long wgs = (long long)((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN) * groups;
  return (double)((wgs + N_CU - 1) / N_CU) * BM * BN / eff;
}

// Forced tilings (GemmArgs.tiling = t + 1, from BcnfStackDesc.gemm_tiling; 0 = the cost model): 0 = 128x128,
// 1 = 64x64, 2 = 128x48 (16x16 MFMA), 3 = 128x48 on 8 waves, 4 = 96x48 on 6 waves, 5 = LDS-DMA (tiling C, the default;
// 96 x 48 for K-contiguous operands), 6 = tiling C large tiles, 7 = tiling C 48 x 48, 8 = 176 x 176 on 11 waves
// (strided x strided operands only; the dispatcher's choice otherwise), 9 = tiling W 96 x 48, 10 = tiling W 48 x 48
// (K-contiguous x K-contiguous, K <= 768; the dispatcher's choice otherwise). Auto: tiling W for K-contiguous
// operands with K <= 768 unless the grid is large enough for tiling C's 128 x 128 tiles.

template <bool AKC, bool BKC, int EPI>
int gemm(const GemmArgs& g, int groups, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0 || groups <= 0) return BCNF_OK;
  if ((g.lda & 3) || (g.ldb & 3) || (!aligned16(g.A)) || (!aligned16(g.B))) return BCNF_ERR_ARG;
  if ((AKC || BKC) && (g.K & 3)) return BCNF_ERR_ARG;
  int pick = g.tiling - 1;
  // LDS-DMA tiling C for K-contiguous x K-contiguous operands (the chain GEMMs, the projections, the row-mapped
  // condition gradient); the register-staged tilings keep the strided layouts, where tiling C's permuted
  // 64-wide wave tiles measured slower (tools/gemm_bench.py t6 / t7, profiles/r02t_gemm_tilings.txt)
  if (pick < 0 && AKC && BKC) pick = 5;
  if (pick >= 5 && pick <= 7) return gemm_gl<AKC, BKC, EPI>(g, groups, st, pick == 6);
  if constexpr (AKC && BKC) {   // tiling W forced
    if (pick == 9 && g.K >= 4 && g.K <= WB_KMAX) return launch_wb<6, 2, WB_P, 1, EPI>(g, groups, st);
    if (pick == 10 && g.K >= 4 && g.K <= WB_KMAX) return launch_wb<3, 4, WB_P, 1, EPI>(g, groups, st);
  }
  // strided x strided (the grouped Linear gradients, M = H + 1, N = H at H = 526): 176 x 176 tiles cover 528 x 528
  // exactly (the 64 x 64 / 128 x 128 grids compute 1.19x / 1.47x the area) and re-read each operand 3 times instead
  // of 9; 11 waves of 16 x 176
  if constexpr (!AKC && !BKC) {
    if (pick == 8 || (pick < 0 && g.M > 352 && g.M <= 528 && g.N > 352 && g.N <= 528)) {
      // unpredicated loads when no load of the grid can leave its operand: whole K tiles, and the tile grid's M / N
      // extent within the [K][M] / [K][N] rows (the Linear gradients: M = 526, N = 527 in rows of HP = 528)
      const bool full = g.K % 32 == 0 && (g.M + 175) / 176 * 176 <= g.lda && (g.N + 175) / 176 * 176 <= g.ldb;
      return full ? launch_cfg16<176, 176, 32, AKC, BKC, EPI, 11, true>(g, groups, st)
                  : launch_cfg16<176, 176, 32, AKC, BKC, EPI, 11>(g, groups, st);
    }
  }
  if (pick == 8) pick = -1;
  if (pick < 0) {
    // relative efficiencies per operand layout, measured at 4096^3 on MI355X (tools/gemm_bench.py)
    const double e1 = AKC ? (BKC ? 1.06 : 0.88) : 0.78, e2 = AKC ? (BKC ? 0.86 : 0.70) : 0.60;
    const double c0 = tile_cost(g, groups, 128, 128, 1.0);
    const double c1 = tile_cost(g, groups, 64, 64, e1);
    const double c2 = tile_cost(g, groups, 128, 48, e2);
    pick = (c0 <= c1 && c0 <= c2) ? 0 : (c2 <= c1 ? 2 : 1);
    // two waves per SIMD inside the workgroup pay off once the 16x16 tiling's grid covers most CUs
    // (tools/gemm_bench.py, M = 2048, N = K = 528: 128x48 on 4 waves 23.4-27.9 us, 96x48 on 6 waves 21.0-25.2,
    // 128x48 on 8 waves 21.6-23.5; at M = 1024 the 4-wave tile stays fastest)
    if (pick == 2 && (long long)((g.M + 127) / 128) * ((g.N + 47) / 48) * groups >= N_CU / 2)
      pick = (AKC && !BKC) || !AKC ? 3 : 4;
  }
  if (pick == 0) return launch_cfg<128, 128, 16, AKC, BKC, EPI>(g, groups, st);
  if (pick == 2) return launch_cfg16<128, 48, 64, AKC, BKC, EPI>(g, groups, st);
  if (pick == 3) return launch_cfg16<128, 48, 64, AKC, BKC, EPI, 8>(g, groups, st);
  if (pick == 4) return launch_cfg16<96, 48, 64, AKC, BKC, EPI, 6>(g, groups, st);
  return launch_cfg<64, 64, 64, AKC, BKC, EPI>(g, groups, st);
}

template <bool AKC, bool BKC, int EPI>
int gemm_gl(const GemmArgs& g, int groups, hipStream_t st, bool large) {
  const long long t128 = (long long)((g.M + 127) / 128) * ((g.N + 127) / 128) * groups;
  if (AKC && BKC) {
    if (large || t128 >= 2 * N_CU) return launch_gl<128, 128, 2, 2, true, true, EPI, 2>(g, groups, st);
    // tiling W (B band resident in LDS, one workgroup per CU) unless tiling C is forced: 48 x 48 tiles on 12 waves
    // (K in 4 slices) while that grid fits one round of the CUs (M = 1024, the LSTM_large chain: 13.2 -> 10.9 us),
    // else 96 x 48 on 12 waves (K halves; M = 2048, the FC_large chain: 17.9 -> 17.3 us; tools/gemm_rd.py,
    // profiles/r03n_gemm_wbti.txt)
    const int forced = g.tiling - 1;
    const bool wb = g.K >= 4 && g.K <= WB_KMAX && forced != 5 && forced != 7;
    const long long t48 = (long long)((g.M + 47) / 48) * ((g.N + 47) / 48) * groups;
    // A ring 2 chunks deep (3: -0.8%, 4: -1.1%, 6: -2.3% on FC_large; tools/ab_wide.sh, profiles/r03zh_*)
    if (wb && t48 <= N_CU) return launch_wb<3, 4, WB_P, 1, EPI>(g, groups, st);
    if (wb) return launch_wb<6, 2, WB_P, 1, EPI>(g, groups, st);
    // tiling C: 96 x 48 on one workgroup per CU while that grid covers most CUs (M = 2048, N = 528: 242 tiles); below,
    // 48 x 48 workgroups two per CU (M = 1024: 13.3 vs 17.6 us, tools/gemm_bench.py)
    const long long t96 = (long long)((g.M + 95) / 96) * ((g.N + 47) / 48) * groups;
    if (forced == 7 || (forced != 5 && t96 < 3 * N_CU / 4))
      return launch_gl<48, 48, 3, 1, true, true, EPI, 3>(g, groups, st);
    return launch_gl<96, 48, 6, 1, true, true, EPI, 4>(g, groups, st);
  }
  if (!AKC && !BKC) return launch_gl<128, 128, 2, 2, false, false, EPI, 2>(g, groups, st);
  if (AKC) return launch_gl<64, 128, 2, 2, true, false, EPI, 3>(g, groups, st);
  return launch_gl<128, 64, 2, 2, false, true, EPI, 3>(g, groups, st);
}

// C = A B with K split into np equal chunks (grouped launch into `part`, then a fixed-order sum): tall-K GEMMs whose
// M x N grid alone cannot fill the chip (the folded condition gradients, K = nv * HP). Falls back to one GEMM when
// K does not split evenly or the scratch is too small.
template <bool AKC, bool BKC>
int gemm_splitk(const GemmArgs& g, int np, float* part, long long part_floats, hipStream_t st) {
  const int kc = np > 0 ? g.K / np : 0;
  const long long ldp = (g.N + 3) & ~3LL;
  if (np < 2 || kc * np != g.K || ((AKC || BKC) && (kc & 3)) || (g.N & 3) || (g.ldc & 3) || !aligned16(g.C) ||
      (long long)np * g.M * ldp > part_floats)
    return gemm<AKC, BKC, EPI_STORE>(g, 1, st);
  GemmArgs p = g;
  p.K = kc;
  p.C = part;
  p.ldc = ldp;
  p.G0 = 1;
  p.sA1 = AKC ? kc : (long long)kc * g.lda;
  p.sB1 = BKC ? kc : (long long)kc * g.ldb;
  p.sC1 = (long long)g.M * ldp;
  const int rc = gemm<AKC, BKC, EPI_STORE>(p, np, st);
  if (rc) return rc;
  const long long n4 = (long long)g.M * (g.N / 4);
  const int grid = (int)std::min<long long>((n4 + WWG - 1) / WWG, 2048);
  hipLaunchKernelGGL(k_wsum_parts, dim3(grid), dim3(WWG), 0, st, part, p.sC1, np, g.M, g.N / 4, ldp, g.C, g.ldc);
  return bcnf_rt::launched();
}

// Skinny split-K Linear-gradient partials: part[g1][s][m][n] = sum_{k in split s} A[k][m] B[k][n] with one operand
// "wide" (W = 526 / 527 columns: the activation rows A_{NH-1} of the last Linear's gradient, or dZ_0 of Linear 1's
// input columns) and the other narrow (Q <= 36: the last Linear's 2 nout outputs, or Linear 1's nin + 1 inputs).
// HBM-bound: the wide operand is 111 MB per call at FC_large B = 2048, streamed once. Each thread owns 4 wide columns
// (float4 loads, 8 rows in flight), the split's narrow rows sit in LDS (broadcast b128 reads), every (q, column)
// accumulates in registers on packed FMAs; the four waves take quarters of the split's rows and meet in LDS in a fixed
// order (deterministic). The 64 x 64 register-staged tile this replaces kept ~1.5 TB/s (r03: 59-258 us per call).
typedef float f32x2w __attribute__((ext_vector_type(2)));
constexpr int SK_COLS = 4 * 64;      // wide columns per workgroup
constexpr int SK_ROWS = 8;           // rows in flight per thread

// acc + a * (w[H], w[H]): one v_pk_fma_f32 reading one half of the w pair for both lanes (op_sel), so the column value
// needs no broadcast copy
template <int H>
__device__ __forceinline__ f32x2w pk_fma_bc(f32x2w a, f32x2w w, f32x2w acc) {
  if (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(a), "v"(w));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(a), "v"(w));
  return acc;
}

template <int QT, bool WIDE_A>
__global__ __launch_bounds__(WWG) void k_skinny(const GemmArgs g, int np, float* __restrict__ part, long long ldp) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int g1 = blockIdx.z, sp = blockIdx.y;
  const int W = WIDE_A ? g.M : g.N, Q = WIDE_A ? g.N : g.M;
  const float* __restrict__ wb = WIDE_A ? g.A + g1 * g.sA1 : g.B + g1 * g.sB1;
  const float* __restrict__ nb = WIDE_A ? g.B + g1 * g.sB1 : g.A + g1 * g.sA1;
  const long long ldw = WIDE_A ? g.lda : g.ldb, ldn = WIDE_A ? g.ldb : g.lda;
  const int KS = g.K / np;                       // rows of this split (the dispatch checks KS % (8 SK_ROWS) == 0)
  const long long k0 = (long long)sp * KS;
  for (int i = threadIdx.x; i < KS * QT; i += WWG) {   // the split's narrow rows, zero beyond Q
    const int r = i / QT, q = i - r * QT;
    sm[i] = q < Q ? nb[(k0 + r) * ldn + q] : 0.f;
  }
  __syncthreads();
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c0 = blockIdx.x * SK_COLS + 4 * l;
  const int cl = c0 < W ? c0 : 0;                // columns past W read column 0 (inside the row), never stored
  const int rq = KS / 4, r0 = wv * rq;
  f32x2w acc[QT / 2][4];                         // acc[p][c] = (out[2p][c], out[2p + 1][c]) of column c0 + c
#pragma unroll
  for (int p = 0; p < QT / 2; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[p][c] = f32x2w{0.f, 0.f};
  const float* wrow = wb + (k0 + r0) * ldw + cl;
  // two register sets of SK_ROWS rows, the next set's loads issued before the current set is consumed; the empty
  // asm statements with a memory clobber keep hipcc from sinking each load to its first use (one round trip per row)
  auto load = [&](floatx4 (&v)[SK_ROWS], int r) {       // rows past the wave's range re-read its last row
#pragma unroll
    for (int t = 0; t < SK_ROWS; ++t) v[t] = ld4(wrow + (long long)(r + t < rq ? r + t : rq - 1) * ldw);
    asm volatile("" ::: "memory");
  };
  auto consume = [&](const floatx4 (&v)[SK_ROWS], int r) {
#pragma unroll
    for (int t = 0; t < SK_ROWS; ++t) {
      const float* nr = sm + (r0 + r + t) * QT;
#pragma unroll
      for (int q4 = 0; q4 < QT / 4; ++q4) {
        const floatx4 n4 = *reinterpret_cast<const floatx4*>(nr + 4 * q4);   // same address in every lane
        const f32x2w n01 = __builtin_shufflevector(n4, n4, 0, 1), n23 = __builtin_shufflevector(n4, n4, 2, 3);
        const f32x2w w01 = __builtin_shufflevector(v[t], v[t], 0, 1), w23 = __builtin_shufflevector(v[t], v[t], 2, 3);
        acc[2 * q4][0] = pk_fma_bc<0>(n01, w01, acc[2 * q4][0]);
        acc[2 * q4 + 1][0] = pk_fma_bc<0>(n23, w01, acc[2 * q4 + 1][0]);
        acc[2 * q4][1] = pk_fma_bc<1>(n01, w01, acc[2 * q4][1]);
        acc[2 * q4 + 1][1] = pk_fma_bc<1>(n23, w01, acc[2 * q4 + 1][1]);
        acc[2 * q4][2] = pk_fma_bc<0>(n01, w23, acc[2 * q4][2]);
        acc[2 * q4 + 1][2] = pk_fma_bc<0>(n23, w23, acc[2 * q4 + 1][2]);
        acc[2 * q4][3] = pk_fma_bc<1>(n01, w23, acc[2 * q4][3]);
        acc[2 * q4 + 1][3] = pk_fma_bc<1>(n23, w23, acc[2 * q4 + 1][3]);
      }
    }
  };
  floatx4 va[SK_ROWS], vb[SK_ROWS];
  load(va, 0);
  for (int r = 0; r < rq; r += 2 * SK_ROWS) {    // rq % (2 SK_ROWS) == 0 (try_skinny)
    load(vb, r + SK_ROWS);
    consume(va, r);
    load(va, r + 2 * SK_ROWS);                   // unconditional (clamped): static wait counts
    consume(vb, r + SK_ROWS);
  }
  __syncthreads();                               // narrow rows consumed: the LDS now holds waves 1..3's partials
  floatx4* red = reinterpret_cast<floatx4*>(sm);   // [3][QT][64 lanes]: (q, columns c0..c0+3)
  auto row_q = [&](int q) {
    const int p = q >> 1, h = q & 1;
    return floatx4{acc[p][0][h], acc[p][1][h], acc[p][2][h], acc[p][3][h]};
  };
  if (wv > 0) {
#pragma unroll
    for (int q = 0; q < QT; ++q) red[((wv - 1) * QT + q) * 64 + l] = row_q(q);
  }
  __syncthreads();
  if (wv != 0 || c0 >= W) return;
  float* out = part + ((long long)g1 * np + sp) * ((long long)g.M * ldp);
#pragma unroll
  for (int q = 0; q < QT; ++q) {
    floatx4 t = row_q(q);
#pragma unroll
    for (int w = 0; w < 3; ++w) t += red[(w * QT + q) * 64 + l];      // wave order 0, 1, 2, 3
    if (q >= Q) continue;
    if (!WIDE_A) {
      *reinterpret_cast<floatx4*>(out + (long long)q * ldp + c0) = t;   // row q, columns c0..c0+3 (< ldp)
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (c0 + u < W) out[(long long)(c0 + u) * ldp + q] = t[u];
    }
  }
}

template <int QT, bool WIDE_A>
int launch_skinny(const GemmArgs& g, int groups, int np, float* part, long long ldp, hipStream_t st) {
  const int W = WIDE_A ? g.M : g.N;
  const size_t rows = (size_t)(g.K / np);
  const size_t bytes = 4 * std::max(rows * QT, (size_t)3 * QT * 64 * 4);
  static bool attr = false;
  if (!attr) {
    if (const int rc = bcnf_rt::hip_status(hipFuncSetAttribute((const void*)k_skinny<QT, WIDE_A>,
                                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)))
      return rc;
    attr = true;
  }
  if (bytes > 160 * 1024) return BCNF_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)((W + SK_COLS - 1) / SK_COLS), (unsigned)np, (unsigned)groups);
  hipLaunchKernelGGL((k_skinny<QT, WIDE_A>), grid, dim3(WWG), bytes, st, g, np, part, ldp);
  return bcnf_rt::launched();
}

// The skinny kernel when it applies (cost-model dispatch only; a forced tiling keeps the tiled GEMM): -1 otherwise.
int try_skinny(const GemmArgs& g, int groups, int np, float* part, long long ldp, hipStream_t st) {
  if (g.tiling != 0 || np < 1 || g.K % np != 0 || (g.K / np) % (8 * SK_ROWS) != 0) return -1;
  const bool wide_a = g.N <= 36 && g.M >= 64, wide_b = g.M <= 36 && g.N >= 64;
  if (!wide_a && !wide_b) return -1;
  const long long ldw = wide_a ? g.lda : g.ldb, sw = wide_a ? g.sA1 : g.sB1;
  const int W = wide_a ? g.M : g.N;
  if ((ldw & 3) || (sw & 3) || ldw < ((W + 3) & ~3) || !aligned16(wide_a ? g.A : g.B) || (!wide_a && (ldp & 3)))
    return -1;
  if ((long long)(g.K / np) * 36 * 4 > 160 * 1024) return -1;
  const int Q = wide_a ? g.N : g.M;
  if (wide_a) {
    if (Q <= 12) return launch_skinny<12, true>(g, groups, np, part, ldp, st);
    if (Q <= 20) return launch_skinny<20, true>(g, groups, np, part, ldp, st);
    return launch_skinny<36, true>(g, groups, np, part, ldp, st);
  }
  if (Q <= 12) return launch_skinny<12, false>(g, groups, np, part, ldp, st);
  if (Q <= 20) return launch_skinny<20, false>(g, groups, np, part, ldp, st);
  return launch_skinny<36, false>(g, groups, np, part, ldp, st);
}

// Grouped strided x strided EPI_LINGRAD GEMM with K (= the batch) split into np parts: partials in `part`, then a
// fixed-order sum through the LINGRAD mapping. The last-Linear and Linear-1 input-column gradients have M or N <= 36,
// so unsplit their grid is ~one 64 x 64 workgroup per block and column tile, each streaming the whole batch
// (FC_large B = 2048: 85 us each at 7-12 TFLOP/s). Falls back to the direct launch for small or ragged batches.
int lingrad_splitk(const GemmArgs& g, int groups, float* part, long long part_floats, hipStream_t st) {
  const int np = (g.K >= 256 && g.K % 8 == 0) ? 8 : (g.K >= 256 && g.K % 4 == 0) ? 4 : 1;
  const long long ldp = (g.N + 3) & ~3LL;
  if (np < 2 || !part || g.G0 != 1 || (long long)groups * np * g.M * ldp > part_floats)
    return gemm<false, false, EPI_LINGRAD>(g, groups, st);
  GemmArgs p = g;
  p.K = g.K / np;
  p.G0 = np;
  p.sA0 = (long long)p.K * g.lda;
  p.sB0 = (long long)p.K * g.ldb;
  p.C = part;
  p.ldc = ldp;
  p.sC0 = (long long)g.M * ldp;
  p.sC1 = (long long)np * p.sC0;
  p.use_cb = 0;
  int rc = try_skinny(g, groups, np, part, ldp, st);       // the HBM-streaming kernel for the skinny shapes
  if (rc < 0) rc = gemm<false, false, EPI_STORE>(p, groups * np, st);
  if (rc) return rc;
  hipLaunchKernelGGL(k_wsum_lingrad, dim3((unsigned)(((long long)g.M * g.N + WWG - 1) / WWG), groups), dim3(WWG), 0, st,
                     g, part, np, ldp);
  return bcnf_rt::launched();
}

struct WideWs {       // workspace carve-up (floats)
  float *P, *A, *G, *dZ, *dZ0, *X, *S, *U, *O, *DV, *ANP, *nllp, *Hp;
  float* LP;          // [B][32 * ceil(HP / 48)] last-Linear partials of the current block (tiling W epilogue)
  long long total;
  long long g_off;    // offset of G (floats; bcnf_wide_backward_plan)
};

inline int lp_tiles(const WideLayout& L) { return (L.HP + 47) / 48; }

WideWs carve(const WideLayout& L, long long B, bool train, float* base) {
  WideWs w;
  memset(&w, 0, sizeof(w));
  long long o = 0;
  auto take = [&](long long n) {
    float* p = base ? base + o : nullptr;
    o += pad4l(n) + 64;     // keep every region 16-B aligned (and apart)
    return p;
  };
  const long long slab = B * L.HP;
  w.P = take(B * (long long)L.nv * L.HP);
  w.nllp = take(B);
  if (train) {
    w.A = take((long long)L.nv * L.NH * slab);
    w.g_off = o;
    w.G = take((long long)L.nv * L.NH * slab);
    w.dZ = take((long long)L.nv * (L.NH - 1) * slab);
    w.dZ0 = take(B * (long long)L.nv * L.HP);
    w.X = take((long long)(L.nv + 1) * B * L.XP);
    w.S = take((long long)L.nv * B * L.SP);
    w.U = take((long long)L.nv * B * L.UP);
    w.O = take((long long)L.nv * B * L.OP);
    w.DV = take(B * (long long)L.XP);
    w.ANP = take((long long)L.nb * B * L.AP);
  } else {
    w.A = take(2 * slab);     // ping-pong
    w.X = take(B * (long long)L.XP);
  }
  if (L.Cp != L.C) w.Hp = take(B * (long long)L.Cp);   // h re-laid to rows of Cp floats
  w.LP = take(B * 32LL * lp_tiles(L));
  w.total = o;
  return w;
}

// (tail side, head side) of a link launch -> kernel instantiation; the unused side of a head-only / tail-only
// launch is free, so every launch maps onto (0,0) [one-way], (0,1) or (1,0) [two_way].
template <bool INV, int DD>
void link_dispatch(int ts, int hs, dim3 grid, size_t lds, hipStream_t st, const WideLayout& L, const LinkArgs& a) {
  if (L.S == 1) hipLaunchKernelGGL((k_wlink<INV, DD, 0, 0>), grid, dim3(WWG), lds, st, L, a);
  else if (ts == 0 && hs == 1) hipLaunchKernelGGL((k_wlink<INV, DD, 0, 1>), grid, dim3(WWG), lds, st, L, a);
  else hipLaunchKernelGGL((k_wlink<INV, DD, 1, 0>), grid, dim3(WWG), lds, st, L, a);
}

#ifdef BCNF_PHASE_STAMPS
unsigned long long* g_link_dbg = nullptr;   // bcnf_wide_debug_phases (diagnostic build)
#endif

int link_launch(const WideLayout& L, const LinkArgs& a_in, bool inv, hipStream_t st) {
  LinkArgs a = a_in;
#ifdef BCNF_PHASE_STAMPS
  a.dbg = g_link_dbg;
#else
  a.dbg = nullptr;
#endif
  dim3 grid((unsigned)((a.B + LR - 1) / LR));
  const size_t lds = (size_t)link_lds_floats(L, a.vt >= 0, a.vh >= 0) * sizeof(float);
  const int ts = a.vt >= 0 ? a.vt % L.S : 1 - (a.vh % L.S);
  const int hs = a.vh >= 0 ? a.vh % L.S : 1 - ts;
  if (L.D == 19) {                       // every shipped trajectory config (19 physical parameters)
    if (inv) link_dispatch<true, 19>(ts, hs, grid, lds, st, L, a);
    else link_dispatch<false, 19>(ts, hs, grid, lds, st, L, a);
  } else {
    if (inv) link_dispatch<true, 0>(ts, hs, grid, lds, st, L, a);
    else link_dispatch<false, 0>(ts, hs, grid, lds, st, L, a);
  }
  return bcnf_rt::launched();
}

template <int DD>
void linkb_dispatch(int ts, int hs, dim3 grid, size_t lds, hipStream_t st, const WideLayout& L, const LinkBArgs& a) {
  if (L.S == 1) hipLaunchKernelGGL((k_wlink_bwd<DD, 0, 0>), grid, dim3(WWG), lds, st, L, a);
  else if (ts == 0 && hs == 1) hipLaunchKernelGGL((k_wlink_bwd<DD, 0, 1>), grid, dim3(WWG), lds, st, L, a);
  else hipLaunchKernelGGL((k_wlink_bwd<DD, 1, 0>), grid, dim3(WWG), lds, st, L, a);
}

int linkb_launch(const WideLayout& L, const LinkBArgs& a, hipStream_t st) {
  dim3 grid((unsigned)((a.B + LR - 1) / LR));
  const size_t lds = (size_t)link_lds_floats(L, a.vh >= 0, a.vt >= 0) * sizeof(float);
  const int ts = a.vt >= 0 ? a.vt % L.S : 1 - (a.vh % L.S);
  const int hs = a.vh >= 0 ? a.vh % L.S : 1 - ts;
  if (L.D == 19) linkb_dispatch<19>(ts, hs, grid, lds, st, L, a);
  else linkb_dispatch<0>(ts, hs, grid, lds, st, L, a);
  return bcnf_rt::launched();
}

bool lds_attr_done = false;
void ensure_lds_attrs() {
  if (lds_attr_done) return;
  const void* fns[] = {
      (const void*)k_wlink<true, 0, 0, 0>,  (const void*)k_wlink<true, 0, 0, 1>,  (const void*)k_wlink<true, 0, 1, 0>,
      (const void*)k_wlink<false, 0, 0, 0>, (const void*)k_wlink<false, 0, 0, 1>, (const void*)k_wlink<false, 0, 1, 0>,
      (const void*)k_wlink<true, 19, 0, 0>, (const void*)k_wlink<true, 19, 0, 1>, (const void*)k_wlink<true, 19, 1, 0>,
      (const void*)k_wlink<false, 19, 0, 0>, (const void*)k_wlink<false, 19, 0, 1>,
      (const void*)k_wlink<false, 19, 1, 0>, (const void*)k_wlink_bwd<0, 0, 0>, (const void*)k_wlink_bwd<0, 0, 1>,
      (const void*)k_wlink_bwd<0, 1, 0>,    (const void*)k_wlink_bwd<19, 0, 0>, (const void*)k_wlink_bwd<19, 0, 1>,
      (const void*)k_wlink_bwd<19, 1, 0>};
  for (const void* f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  lds_attr_done = true;
}

#define WCHK(x)            \
  do {                     \
    const int _rc = (x);   \
    if (_rc) return _rc;   \
  } while (0)

// h (rows x C) as rows of Cp floats: h itself when C % 4 == 0, else a padded copy in `pad`
const float* padded_h(const WideLayout& L, const float* h, long long rows, float* pad, hipStream_t st, int* rc) {
  *rc = BCNF_OK;
  if (L.Cp == L.C || rows == 0) return h;
  const long long n = rows * L.Cp;
  const int grid = (int)std::min<long long>((n + WWG - 1) / WWG, 4096);
  hipLaunchKernelGGL(k_wpad_rows, dim3(grid), dim3(WWG), 0, st, h, L.C, rows, pad, L.Cp);
  *rc = bcnf_rt::launched();
  return pad;
}

// P = h W0h_all^T  (rows x nv*HP), h with row stride Cp
int projection(const WideLayout& L, const float* pk, const float* hp, long long rows, float* P, hipStream_t st) {
  GemmArgs g = gemm_args(L.tiling, (int)rows, L.nv * L.HP, L.Cp, hp, L.Cp, pk + L.pk_w0h, L.Cp, P, (long long)L.nv * L.HP);
  return gemm<true, true, EPI_STORE>(g, 1, st);
}

// Can gemm<true, true, EPI_ACT> run this GEMM on tiling W (k_wbr, whose epilogue can apply the block's last Linear)?
// A pre-filter only (the partials' column-tile count fits LP_MAX, K in tiling W's range): whether the partials were
// written is what launch_wb reports (g_lp_written), so a dispatch change cannot leave the link summing stale ones.
bool wbr_lp_ok(const GemmArgs& g, int groups) {
  if (g.K < 4 || g.K > WB_KMAX || g.M <= 0 || (g.N + 47) / 48 > LP_MAX) return false;
  const int forced = g.tiling - 1;
  if (forced == 9 || forced == 10) return true;
  if (forced >= 0) return false;
  const long long t128 = (long long)((g.M + 127) / 128) * ((g.N + 127) / 128) * groups;
  return t128 < 2 * N_CU;
}

// hidden Linear l (1..NH-1) of virtual block v: A_l = dropout(GELU(A_{l-1} W_l^T + b_l)), G_l. With `lp` and the
// last hidden layer on tiling W, the epilogue also writes the block's last-Linear partials (returned through *lp_on).
int hidden_fwd(const WideLayout& L, const float* prm, const float* pk, int v, int l, long long B, const float* Ain,
               float* Aout, float* Gout, const uint64_t* rng, hipStream_t st, float* lp = nullptr,
               bool* lp_on = nullptr) {
  GemmArgs g = gemm_args(L.tiling, (int)B, L.HP, L.HP, Ain, L.HP, pk + L.pk_hid + ((long long)v * (L.NH - 1) + (l - 1)) * L.HP * L.HP,
                         L.HP, Aout, L.HP);
  g.bias = prm + vbase(L, v) + L.lin_b[v % L.S][l];
  g.aux = Gout;
  g.ldaux = L.HP;
  g.n_real = L.H;
  g.rng = rng;
  g.thresh = L.thresh;
  g.keep_scale = L.keep_scale;
  g.tag = (uint32_t)v * 16u + (uint32_t)l;
  if (lp_on) *lp_on = false;
  if (lp && l == L.NH - 1 && wbr_lp_ok(g, 1)) {
    const int sd = v % L.S;
    g.lp = lp;
    g.lp_ld = 32LL * lp_tiles(L);
    g.lp_w = pk + L.pk_wl + (long long)v * L.WL * L.HP;
    g.lp_wld = L.HP;
    g.lp_n = 2 * L.nout[sd];
  }
  g_lp_written = false;
  const int rc = gemm<true, true, EPI_ACT>(g, 1, st);
  if (lp_on) *lp_on = rc == BCNF_OK && g.lp && g_lp_written;
  return rc;
}

// Folded last feature Linear (h = x Wf^T + bf, the wide analogue of bcnf_stack.hip's FC_small fold): with
// x1 = [x | 1 | 0] (B x Xp), wfb = [Wf | bf | 0] (C x Xp) and Wcb = W0h_all wfb (nv*HP x Xp):
//   P = x1 Wcb^T;   Gx = dZ0_all^T x1;   dW0h_all = Gx wfb^T;   [dWf | dbf] = W0h_all^T Gx;   dL/dx = dZ0_all Wcb
// The projection's K drops from C to Xp and dL/dh is never formed (FC_large: 235 -> 87 GFLOP of condition GEMMs).
struct WideFold {
  const float* x1;     // [B][Xp]
  const float* wfb;    // [C][Xp]
  const float* wcb;    // [nv*HP][Xp]
  float* gx;           // [nv*HP][Xp] scratch
  float* dwfb;         // [C][Xp] out (nullable)
  float* dx;           // [B][Xp] out, columns < X meaningful (nullable)
  int Xp;
};

int fold_prepare(const WideLayout& L, const float* pk, const float* wfb, int Xp, float* wcb, hipStream_t st) {
  GemmArgs g = gemm_args(L.tiling, L.nv * L.HP, Xp, L.C, pk + L.pk_w0h, L.Cp, wfb, Xp, wcb, Xp);
  return gemm<true, false, EPI_STORE>(g, 1, st);
}

int wide_forward(const WideLayout& L, const float* prm, const float* pk, const float* y, const float* h, long long B,
                 float* z, float* ldj, bool training, const uint64_t* rng, float* ws, bool save, hipStream_t st,
                 const WideFold* fold = nullptr) {
  if (B == 0) return BCNF_OK;
  ensure_lds_attrs();
  const bool drop = training && L.p > 0.f && rng;
  const WideWs w = carve(L, B, save, ws);
  const long long slab = B * L.HP;
  int rc;
  if (fold) {
    GemmArgs g = gemm_args(L.tiling, (int)B, L.nv * L.HP, fold->Xp, fold->x1, fold->Xp, fold->wcb, fold->Xp, w.P,
                           (long long)L.nv * L.HP);
    WCHK((gemm<true, true, EPI_STORE>(g, 1, st)));
  } else {
    const float* hp = padded_h(L, h, B, w.Hp, st, &rc);
    WCHK(rc);
    WCHK(projection(L, pk, hp, B, w.P, st));
  }
  auto Aptr = [&](int v, int l) -> float* { return save ? w.A + ((long long)v * L.NH + l) * slab : w.A + (l & 1) * slab; };
  auto Gptr = [&](int v, int l) -> float* { return save ? w.G + ((long long)v * L.NH + l) * slab : nullptr; };
  for (int v = -1; v < L.nv; ++v) {
    bool lp_on = false;
    if (v >= 0)
      for (int l = 1; l < L.NH; ++l)
        WCHK(hidden_fwd(L, prm, pk, v, l, B, Aptr(v, l - 1), Aptr(v, l), Gptr(v, l), drop ? rng : nullptr, st, w.LP,
                        &lp_on));
    LinkArgs a;
    memset(&a, 0, sizeof(a));
    if (lp_on) {
      a.Opart = w.LP;
      a.ldo = 32LL * lp_tiles(L);
      a.nop = lp_tiles(L);
    }
    a.B = B;
    a.vt = v;
    a.vh = (v + 1 < L.nv) ? v + 1 : -1;
    a.prm = prm;
    a.pk = pk;
    if (v >= 0) {
      a.Alast = Aptr(v, L.NH - 1);
      a.Xt = save ? w.X + (long long)v * B * L.XP : w.X;
      a.S = save ? w.S + (long long)v * B * L.SP : nullptr;
    }
    a.z = z;
    a.ldj = ldj;
    a.nllp = w.nllp;
    a.xin = y;
    if (a.vh >= 0) {
      a.Xh = save ? w.X + (long long)a.vh * B * L.XP : w.X;
      a.P = w.P;
      a.ldP = (long long)L.nv * L.HP;
      a.A0 = Aptr(a.vh, 0);
      a.G0 = Gptr(a.vh, 0);
      a.U = save ? w.U + (long long)a.vh * B * L.UP : nullptr;
    }
    a.rng = drop ? rng : nullptr;
    WCHK(link_launch(L, a, false, st));
  }
  return BCNF_OK;
}

// The G region's split-K scratch plan of one wide_backward call (host arithmetic only; bcnf_wide_backward_plan
// exposes it to the CPU tests and the ASan run, tools/asan_host.sh). The G region holds nv * NH slabs of B * HP
// floats. The last range's dL/dx and [dWf | dbf] put their split-K partials at its END (`tail` floats), the parameter
// gradients of the range use the range's own G slots from its head (`gsc_off`, `gsc_floats`), so phase 1 and phase 2
// may run on two streams. A need larger than the whole region reserves nothing (that GEMM runs unsplit), and the
// head region is clamped to what the tail leaves.
struct GPlan {
  long long gfl_all, dx_need, dwfb_need, tail, gsc_off, gsc_floats;
};
GPlan g_plan(const WideLayout& L, long long B, bool dx, bool dwfb, int Xp, int blo, int bhi) {
  GPlan p;
  p.gfl_all = (long long)L.nv * L.NH * B * L.HP;
  p.dx_need = (dx && blo == 0) ? (long long)L.nv * B * ((Xp + 3) & ~3) : 0;
  p.dwfb_need = (dwfb && blo == 0) ? (long long)L.nv * L.C * ((Xp + 3) & ~3) : 0;
  if (p.dx_need > p.gfl_all) p.dx_need = 0;
  if (p.dwfb_need > p.gfl_all) p.dwfb_need = 0;
  p.tail = std::max(p.dx_need, p.dwfb_need);
  const int vlo = blo * L.S, nvr = (bhi - blo) * L.S;
  p.gsc_off = (long long)vlo * L.NH * B * L.HP;
  p.gsc_floats = std::max(0LL, std::min((long long)nvr * L.NH * B * L.HP, p.gfl_all - p.tail - p.gsc_off));
  return p;
}

// Real blocks [blo, bhi) of the backward: the chain iterations that complete them, then their parameter gradients
// (canonical flat, every element written exactly once). The whole backward is [0, nb). A data-parallel caller may
// split it into descending contiguous ranges, the first with bhi = nb, and reduce each range's gradient slice while
// the next range runs (bcnf_wide_fold_backward_range); the range with blo = 0 also runs what needs every block (fold:
// the feature-Linear gradients and dL/dx; else dL/dh). The chain iteration v finishes virtual block v (tail-B: dZ_0)
// and starts v - 1 (head-B, then its hidden-layer chain), so a range runs v = (vhi == nv ? nv : vhi - 1) .. vlo.
// Per-element results do not depend on the split: every GEMM keeps its K order, the split-K partials of the small
// Linear gradients go to the finished range's G slots (dead once its chain has run).
// phase (whole range only): bit 1 = what the caller's next layers wait for (the chain, then Gx, dL/dx, [dWf | dbf] /
// dL/dh), bit 2 = the coupling parameter gradients. Bit 2 reads only the workspace, Gx and the operands and puts its
// split-K partials at the head of the G region, bit 1's at its tail, so a caller may run bit 2 on a second stream
// (after bit 1's chain in stream order) while its own backward continues on the first.
int wide_backward(const WideLayout& L, const float* prm, const float* pk, const float* h, const float* zn,
                  const float* dz, const float* dldj, const float* dvals, int nll, long long B, float* ws, float* dy,
                  float* dh, float* dprm, hipStream_t st, const WideFold* fold = nullptr, int blo = 0, int bhi = -1,
                  int phase = 3) {
  if (B == 0) return BCNF_OK;
  if (bhi < 0) bhi = L.nb;
  if (blo < 0 || bhi > L.nb || blo >= bhi) return BCNF_ERR_ARG;
  ensure_lds_attrs();
  const WideWs w = carve(L, B, true, ws);
  const GPlan gp = g_plan(L, B, fold && fold->dx, fold && fold->dwfb, fold ? fold->Xp : 0, blo, bhi);
  const long long gfl_all = gp.gfl_all, tail = gp.tail;
  const long long slab = B * L.HP;
  const long long ld0 = (long long)L.nv * L.HP;
  const int vlo = blo * L.S, vhi = bhi * L.S, nvr = vhi - vlo;
  auto Gptr = [&](int v, int l) -> float* { return w.G + ((long long)v * L.NH + l) * slab; };
  // dZ_l (l = 1..NH-1) of virtual block v; dZ_0 of v is the column slice v*HP of dZ0_all
  auto dZptr = [&](int v, int l, long long* ld) -> float* {
    if (l == 0) {
      *ld = ld0;
      return w.dZ0 + (long long)v * L.HP;
    }
    *ld = L.HP;
    return w.dZ + ((long long)v * (L.NH - 1) + (l - 1)) * slab;
  };
  if (phase & 1) {
  for (int v = vhi == L.nv ? L.nv : vhi - 1; v >= vlo; --v) {
    // link: tail-B(v) (v < nv), head-B(v-1)
    LinkBArgs a;
    memset(&a, 0, sizeof(a));
    a.B = B;
    a.vt = (v < L.nv) ? v : -1;
    a.vh = v - 1;
    a.prm = prm;
    a.pk = pk;
    a.X = w.X;
    a.sX = B * L.XP;
    a.S = w.S;
    a.sS = B * L.SP;
    a.dz = dz;
    a.dldj = dldj;
    a.zn = zn;
    a.dvals = dvals;
    a.nll = nll;
    a.DV = w.DV;
    a.dy = dy;
    if (a.vt >= 0) {
      a.dZ0 = dZptr(v, 0, &a.ldZ0);
      a.ANP = w.ANP + (long long)(v / L.S) * B * L.AP;
    }
    if (a.vh >= 0) {
      a.Ob = w.O + (long long)a.vh * B * L.OP;
      a.Gl = Gptr(a.vh, L.NH - 1);
      a.dZl = dZptr(a.vh, L.NH - 1, &a.ldZl);
    }
    WCHK(linkb_launch(L, a, st));
    if (a.vh < 0) break;
    const int vb = a.vh;
    // dZ_{l-1} = (dZ_l W_l) * G_{l-1}, l = NH-1 .. 1
    for (int l = L.NH - 1; l >= 1; --l) {
      long long ldi, ldo;
      const float* din = dZptr(vb, l, &ldi);
      float* dout = dZptr(vb, l - 1, &ldo);
      GemmArgs g = gemm_args(L.tiling, (int)B, L.HP, L.HP, din, ldi,
                             pk + L.pk_hidT + ((long long)vb * (L.NH - 1) + (l - 1)) * L.HP * L.HP, L.HP, dout, ldo);
      g.aux = Gptr(vb, l - 1);
      g.ldaux = L.HP;
      WCHK((gemm<true, true, EPI_GRAD>(g, 1, st)));
    }
  }
  if (fold) {   // Gx rows of the range = dZ0_all[:, range]^T x1 (the condition-side gradients go through it)
    GemmArgs g = gemm_args(L.tiling, nvr * L.HP, fold->Xp, (int)B, w.dZ0 + (long long)vlo * L.HP, ld0, fold->x1,
                           fold->Xp, fold->gx + (long long)vlo * L.HP * fold->Xp, fold->Xp);
    WCHK((gemm<false, false, EPI_STORE>(g, 1, st)));
  }
  // what needs every block (the last range): the feature side's gradients, split K = nv * HP per virtual block,
  // partials in the tail of the G region (dead once the chain has run)
  if (fold && fold->dx && blo == 0) {     // dL/dx = dZ0_all Wcb
    GemmArgs g = gemm_args(L.tiling, (int)B, fold->Xp, L.nv * L.HP, w.dZ0, ld0, fold->wcb, fold->Xp, fold->dx, fold->Xp);
    WCHK((gemm_splitk<true, false>(g, L.nv, w.G + gfl_all - tail, tail, st)));
  }
  if (fold && fold->dwfb && blo == 0) {   // [dWf | dbf] = W0h_all^T Gx
    GemmArgs g = gemm_args(L.tiling, L.C, fold->Xp, L.nv * L.HP, pk + L.pk_w0h, L.Cp, fold->gx, fold->Xp, fold->dwfb, fold->Xp);
    WCHK((gemm_splitk<false, false>(g, L.nv, w.G + gfl_all - tail, tail, st)));
  }
  if (!fold && dh && blo == 0) {   // dh = dZ0_all W0h_all
    GemmArgs g = gemm_args(L.tiling, (int)B, L.C, L.nv * L.HP, w.dZ0, ld0, pk + L.pk_w0h, L.Cp, dh, L.C);
    WCHK((gemm<true, false, EPI_STORE>(g, 1, st)));
  }
  }
  if (!(phase & 2)) return BCNF_OK;
  int rc = BCNF_OK;
  const float* hp = fold ? nullptr : padded_h(L, h, B, w.Hp, st, &rc);
  WCHK(rc);
  float* const gsc = w.G + gp.gsc_off;               // the range's G slots: split-K scratch once its chain has run
  const long long gsc_floats = gp.gsc_floats;
  // ---- parameter gradients of the range (canonical flat, every element written exactly once) ----
  if (dprm) {
    auto flat_groups = [&](GemmArgs& g) {   // group g1 = virtual block (or real block with S = 1 semantics)
      g.use_cb = 1;
      g.cb_stride = L.blk_stride;
      g.cb_an = L.an;
      g.cb_nb = L.nb;
    };
    if (L.NH > 1) {   // hidden Linears of every virtual block in one grouped launch: [dW_l | db_l] = dZ_l^T [A_{l-1} | 1]
      GemmArgs g = gemm_args(L.tiling, L.H, L.H + 1, (int)B, w.dZ + (long long)vlo * (L.NH - 1) * slab, L.HP,
                             w.A + (long long)vlo * L.NH * slab, L.HP, dprm + L.lin_w[0][1], L.H);
      g.G0 = L.NH - 1;
      g.sA1 = (long long)(L.NH - 1) * slab;
      g.sA0 = slab;
      g.sB1 = (long long)L.NH * slab;
      g.sB0 = slab;
      flat_groups(g);
      g.cb_S = L.S;
      g.cb_v0 = vlo;
      g.cb_side = L.mlp[0] + (L.S == 2 ? L.lin_w[1][1] - L.lin_w[0][1] : 0);
      g.sC0 = (L.NH > 2) ? (L.lin_w[0][2] - L.lin_w[0][1]) : 0;
      g.wcols = L.H;
      g.boff = (long long)L.H * L.H;
      WCHK((gemm<false, false, EPI_LINGRAD>(g, nvr * (L.NH - 1), st)));
    }
    for (int sd = 0; sd < L.S; ++sd) {
      {   // last Linear of every block's side-sd half: [dW | db] = dO^T [A_{NH-1} | 1]
        GemmArgs g = gemm_args(L.tiling, 2 * L.nout[sd], L.H + 1, (int)B,
                               w.O + ((long long)blo * L.S + sd) * B * L.OP, L.OP,
                               w.A + (((long long)blo * L.S + sd) * L.NH + L.NH - 1) * slab, L.HP,
                               dprm + (sd ? L.mlp[0] : 0) + L.lin_w[sd][L.NH], L.H);
        g.sA1 = (long long)L.S * B * L.OP;
        g.sB1 = (long long)L.S * L.NH * slab;
        flat_groups(g);
        g.cb_v0 = blo;
        g.wcols = L.H;
        g.boff = (long long)2 * L.nout[sd] * L.H;
        WCHK(lingrad_splitk(g, bhi - blo, gsc, gsc_floats, st));
      }
      {   // Linear-1, input columns + bias: [dW0[:, :nin] | db0] = dZ_0^T [u_in | 1]
        GemmArgs g = gemm_args(L.tiling, L.H, L.nin[sd] + 1, (int)B, w.dZ0 + ((long long)blo * L.S + sd) * L.HP, ld0,
                               w.U + ((long long)blo * L.S + sd) * B * L.UP, L.UP,
                               dprm + (sd ? L.mlp[0] : 0) + L.lin_w[sd][0], L.in0[sd]);
        g.sA1 = (long long)L.S * L.HP;
        g.sB1 = (long long)L.S * B * L.UP;
        flat_groups(g);
        g.cb_v0 = blo;
        g.wcols = L.nin[sd];
        g.boff = (long long)L.H * L.in0[sd];
        WCHK(lingrad_splitk(g, bhi - blo, gsc, gsc_floats, st));
      }
    }
    {   // Linear-1, condition columns of the range's virtual blocks in one GEMM: dW0h = dZ0^T h (folded: Gx wfb^T)
      GemmArgs g = fold ? gemm_args(L.tiling, nvr * L.HP, L.C, fold->Xp, fold->gx + (long long)vlo * L.HP * fold->Xp,
                                    fold->Xp, fold->wfb, fold->Xp, dprm, 0)
                        : gemm_args(L.tiling, nvr * L.HP, L.C, (int)B, w.dZ0 + (long long)vlo * L.HP, ld0, hp, L.Cp,
                                    dprm, 0);
      g.cb_stride = L.blk_stride;
      g.cb_an = L.an;
      g.cb_nb = L.nb;
      g.cb_S = L.S;
      g.cb_v0 = vlo;
      g.cb_side = L.mlp[0];
      g.rm_hp = L.HP;
      g.rm_h = L.H;
      for (int sd = 0; sd < 2; ++sd) {
        const int ss = sd < L.S ? sd : 0;
        g.rm_off[sd] = L.lin_w[ss][0] + L.nin[ss];
        g.rm_ld[sd] = L.in0[ss];
      }
      if (fold)
        WCHK((gemm<true, true, EPI_ROWMAP>(g, 1, st)));
      else
        WCHK((gemm<false, false, EPI_ROWMAP>(g, 1, st)));
    }
    const int an_hi = bhi < L.nb - 1 ? bhi : L.nb - 1;   // ActNorm k sits in real block k (the last block has none)
    if (L.an && an_hi > blo) {
      hipLaunchKernelGGL(k_wactnorm_grad, dim3(an_hi - blo), dim3(WWG), 0, st, L, w.ANP, B, dldj, zn, dvals, nll, prm,
                         dprm, blo);
      WCHK(bcnf_rt::launched());
    }
  }
  return BCNF_OK;
}

long long inverse_scratch_floats(const WideLayout& L, long long hrows, long long n) {
  return pad4l(hrows * (long long)L.nv * L.HP) + 64 + pad4l(2 * n * (long long)L.HP) + 64 + pad4l(n * (long long)L.XP) +
         64 + (L.Cp != L.C ? pad4l(hrows * (long long)L.Cp) + 64 : 0);
}

int wide_inverse(const WideLayout& L, const float* prm, const float* pk, const float* z, const float* h, long long hrows,
                 const int64_t* cidx, long long n, float* y, bool training, const uint64_t* rng, float* scratch,
                 hipStream_t st) {
  if (n == 0) return BCNF_OK;
  ensure_lds_attrs();
  const bool drop = training && L.p > 0.f && rng;
  // scratch: P (hrows x nv*HP) | A ping-pong (2 x n x HP) | X (n x XP) | padded h
  float* P = scratch;
  float* A = P + pad4l(hrows * (long long)L.nv * L.HP) + 64;
  float* X = A + pad4l(2 * n * (long long)L.HP) + 64;
  float* Hp = X + pad4l(n * (long long)L.XP) + 64;
  const long long slab = n * L.HP;
  int rc;
  const float* hp = padded_h(L, h, hrows, Hp, st, &rc);
  WCHK(rc);
  WCHK(projection(L, pk, hp, hrows, P, st));
  auto Ap = [&](int l) { return A + (l & 1) * slab; };
  // processing order (cnf.py:499-506 with the coupling inverse cnf.py:198-213): real blocks in reverse, and inside a
  // two_way block nn_a's half before nn_b's (the reference's order)
  auto order = [&](int i) { return i < 0 ? -1 : (L.nb - 1 - i / L.S) * L.S + i % L.S; };
  for (int i = -1; i < L.nv; ++i) {
    const int vt = order(i), vh = (i + 1 < L.nv) ? order(i + 1) : -1;
    if (vt >= 0)
      for (int l = 1; l < L.NH; ++l)
        WCHK(hidden_fwd(L, prm, pk, vt, l, n, Ap(l - 1), Ap(l), nullptr, drop ? rng : nullptr, st));
    LinkArgs a;
    memset(&a, 0, sizeof(a));
    a.B = n;
    a.vt = vt;
    a.vh = vh;
    a.prm = prm;
    a.pk = pk;
    a.Alast = Ap(L.NH - 1);
    a.Xt = X;
    a.z = y;
    a.xin = z;
    a.Xh = X;
    a.P = P;
    a.ldP = (long long)L.nv * L.HP;
    a.cidx = cidx;
    a.A0 = Ap(0);
    a.rng = drop ? rng : nullptr;
    WCHK(link_launch(L, a, true, st));
  }
  return BCNF_OK;
}

}  // namespace

// ================================================================================================
// C-ABI (include/bcnf_amd.h)
// ================================================================================================
extern "C" {

int bcnf_wide_supported(const BcnfStackDesc* desc) {
  WideLayout L;
  return wide_layout(desc, &L) == BCNF_OK ? 1 : 0;
}

int bcnf_wide_param_count(const BcnfStackDesc* desc, int64_t* n_trainable, int64_t* n_frozen) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (n_trainable) *n_trainable = L.n_trainable;
  if (n_frozen) *n_frozen = (int64_t)(L.nb - 1) * L.D * L.D;
  return BCNF_OK;
}

int bcnf_wide_packed_bytes(const BcnfStackDesc* desc, int64_t* bytes) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!bytes) return BCNF_ERR_ARG;
  *bytes = L.total * 4;
  return BCNF_OK;
}

int bcnf_wide_workspace_bytes(const BcnfStackDesc* desc, int64_t batch, int32_t save, int64_t* bytes) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!bytes || batch < 0) return BCNF_ERR_ARG;
  *bytes = carve(L, batch, save != 0, nullptr).total * 4;
  return BCNF_OK;
}

int bcnf_wide_inverse_scratch_bytes(const BcnfStackDesc* desc, int64_t h_rows, int64_t n_rows, int64_t* bytes) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!bytes || h_rows < 0 || n_rows < 0) return BCNF_ERR_ARG;
  *bytes = inverse_scratch_floats(L, h_rows, n_rows) * 4;
  return BCNF_OK;
}

int bcnf_wide_pack(const BcnfStackDesc* desc, const float* params, const float* qmats, void* packed, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!params || !packed || (L.nb > 1 && !qmats) || !aligned16(packed)) return BCNF_ERR_ARG;
  const WpackGrid g = wpack_grid(L);
  const long long nwg = g.n_tiles + g.n_rows + g.n_small;
  if (nwg > 0x7fffffffLL) return BCNF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_wpack_all, dim3((unsigned)nwg), dim3(WWG), 0, (hipStream_t)stream, L, g, params, qmats,
                     (float*)packed);
  return bcnf_rt::launched();
}

int bcnf_wide_forward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* y,
                      const float* h, int64_t batch, float* z, float* ldj, float* nll_part, int32_t training,
                      const uint64_t* rng_state, void* workspace, int32_t save, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch < 0) return BCNF_ERR_ARG;
  if (batch == 0) return BCNF_OK;
  if (!params || !packed || !y || !h || !z || !ldj || !workspace || !aligned16(workspace) ||
      (L.Cp == L.C && !aligned16(h)))
    return BCNF_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  WCHK(wide_forward(L, params, (const float*)packed, y, h, batch, z, ldj, training != 0, rng_state, (float*)workspace,
                    save != 0, st));
  if (nll_part) {
    const WideWs w = carve(L, batch, save != 0, (float*)workspace);
    return bcnf_rt::hip_status(hipMemcpyAsync(nll_part, w.nllp, batch * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  return BCNF_OK;
}

int bcnf_wide_nll_finalize(const BcnfStackDesc* desc, const void* workspace, int64_t batch, int32_t save,
                           float* loss_out, uint64_t* rng_state, int32_t* guard, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch <= 0 || !workspace || !loss_out) return BCNF_ERR_ARG;
  const WideWs w = carve(L, batch, save != 0, (float*)workspace);
  hipLaunchKernelGGL(k_wnll_finalize, dim3(1), dim3(WWG), 0, (hipStream_t)stream, w.nllp, (long long)batch, loss_out,
                     rng_state, guard);
  return bcnf_rt::launched();
}

int bcnf_wide_proj_rows(const BcnfStackDesc* desc, int64_t* rows) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!rows) return BCNF_ERR_ARG;
  *rows = (int64_t)L.nv * L.HP;
  return BCNF_OK;
}

int bcnf_wide_fold_prepare(const BcnfStackDesc* desc, const void* packed, const float* wfb, int32_t xp, float* wcb,
                           void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!packed || !wfb || !wcb || xp < 4 || (xp & 3) || !aligned16(wfb) || !aligned16(wcb)) return BCNF_ERR_ARG;
  return fold_prepare(L, (const float*)packed, wfb, xp, wcb, (hipStream_t)stream);
}

int bcnf_wide_fold_forward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* y,
                           const float* x1, int32_t xp, const float* wcb, int64_t batch, float* z, float* ldj,
                           int32_t training, const uint64_t* rng_state, void* workspace, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch < 1 || !params || !packed || !y || !x1 || !wcb || !z || !ldj || !workspace || !aligned16(workspace) ||
      xp < 4 || (xp & 3) || !aligned16(x1) || !aligned16(wcb))
    return BCNF_ERR_ARG;
  WideFold f = {x1, nullptr, wcb, nullptr, nullptr, nullptr, (int)xp};
  return wide_forward(L, params, (const float*)packed, y, nullptr, batch, z, ldj, training != 0, rng_state,
                      (float*)workspace, true, (hipStream_t)stream, &f);
}

int bcnf_wide_fold_backward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* x1,
                            int32_t xp, const float* wfb, const float* wcb, const float* z, const float* dloss,
                            int64_t batch, void* workspace, float* gx_scratch, float* dparams, float* dwfb, float* dx,
                            void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch < 1 || !params || !packed || !x1 || !wfb || !wcb || !z || !workspace || !gx_scratch || !dparams ||
      xp < 4 || (xp & 3) || !aligned16(x1) || !aligned16(wfb) || !aligned16(wcb) || !aligned16(gx_scratch) ||
      (dwfb && !aligned16(dwfb)) || (dx && !aligned16(dx)))
    return BCNF_ERR_ARG;
  WideFold f = {x1, wfb, wcb, gx_scratch, dwfb, dx, (int)xp};
  return wide_backward(L, params, (const float*)packed, nullptr, z, nullptr, nullptr, dloss, 1, batch,
                       (float*)workspace, nullptr, nullptr, dparams, (hipStream_t)stream, &f);
}

int bcnf_wide_fold_backward_phase(const BcnfStackDesc* desc, const float* params, const void* packed, const float* x1,
                                  int32_t xp, const float* wfb, const float* wcb, const float* z, const float* dloss,
                                  int64_t batch, void* workspace, float* gx_scratch, float* dparams, float* dwfb,
                                  float* dx, int32_t phase, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch < 1 || !params || !packed || !x1 || !wfb || !wcb || !z || !workspace || !gx_scratch || !dparams ||
      xp < 4 || (xp & 3) || !aligned16(x1) || !aligned16(wfb) || !aligned16(wcb) || !aligned16(gx_scratch) ||
      (dwfb && !aligned16(dwfb)) || (dx && !aligned16(dx)) || phase < 1 || phase > 3)
    return BCNF_ERR_ARG;
  WideFold f = {x1, wfb, wcb, gx_scratch, dwfb, dx, (int)xp};
  return wide_backward(L, params, (const float*)packed, nullptr, z, nullptr, nullptr, dloss, 1, batch,
                       (float*)workspace, nullptr, nullptr, dparams, (hipStream_t)stream, &f, 0, -1, phase);
}

int bcnf_wide_fold_backward_range(const BcnfStackDesc* desc, const float* params, const void* packed, const float* x1,
                                  int32_t xp, const float* wfb, const float* wcb, const float* z, const float* dloss,
                                  int64_t batch, void* workspace, float* gx_scratch, float* dparams, float* dwfb,
                                  float* dx, int32_t block_lo, int32_t block_hi, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch < 1 || !params || !packed || !x1 || !wfb || !wcb || !z || !workspace || !gx_scratch || !dparams ||
      xp < 4 || (xp & 3) || !aligned16(x1) || !aligned16(wfb) || !aligned16(wcb) || !aligned16(gx_scratch) ||
      (dwfb && !aligned16(dwfb)) || (dx && !aligned16(dx)) || block_lo < 0 || block_hi > L.nb || block_lo >= block_hi)
    return BCNF_ERR_ARG;
  WideFold f = {x1, wfb, wcb, gx_scratch, dwfb, dx, (int)xp};
  return wide_backward(L, params, (const float*)packed, nullptr, z, nullptr, nullptr, dloss, 1, batch,
                       (float*)workspace, nullptr, nullptr, dparams, (hipStream_t)stream, &f, block_lo, block_hi);
}

int bcnf_wide_backward_plan(const BcnfStackDesc* desc, int64_t batch, int32_t xp, int32_t want_dx, int32_t want_dwfb,
                            int32_t block_lo, int32_t block_hi, int64_t* out) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!out || batch < 0 || block_lo < 0 || block_hi > L.nb || block_lo >= block_hi || xp < 0) return BCNF_ERR_ARG;
  const WideWs w = carve(L, batch, true, nullptr);
  const GPlan p = g_plan(L, batch, want_dx != 0, want_dwfb != 0, (int)xp, block_lo, block_hi);
  out[0] = w.total;
  out[1] = w.g_off;
  out[2] = p.gfl_all;
  out[3] = p.tail;
  out[4] = p.gsc_off;
  out[5] = p.gsc_floats;
  out[6] = p.dx_need;
  out[7] = p.dwfb_need;
  return BCNF_OK;
}

int bcnf_wide_block_offset(const BcnfStackDesc* desc, int32_t block, int64_t* offset) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (!offset || block < 0 || block > L.nb) return BCNF_ERR_ARG;
  *offset = block == L.nb ? (int64_t)L.n_trainable : (int64_t)block * L.blk_stride;
  return BCNF_OK;
}

int bcnf_wide_backward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* h,
                       const float* z, const float* dz, const float* dldj, const float* dloss, int32_t nll,
                       int64_t batch, void* workspace, float* dy, float* dh, float* dparams, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (batch < 0) return BCNF_ERR_ARG;
  if (!params || !packed || !h || !workspace || (nll && !z)) return BCNF_ERR_ARG;
  if (batch == 0) {
    if (dparams) return bcnf_rt::hip_status(hipMemsetAsync(dparams, 0, L.n_trainable * 4, (hipStream_t)stream));
    return BCNF_OK;
  }
  return wide_backward(L, params, (const float*)packed, h, z, dz, dldj, dloss, nll, batch, (float*)workspace, dy, dh,
                       dparams, (hipStream_t)stream);
}

int bcnf_wide_inverse(const BcnfStackDesc* desc, const float* params, const void* packed, const float* z,
                      const float* h, int64_t h_rows, const int64_t* cond_index, int64_t n_rows, float* y,
                      int32_t training, const uint64_t* rng_state, void* scratch, void* stream) {
  WideLayout L;
  WCHK(wide_layout(desc, &L));
  if (n_rows < 0 || h_rows < 0) return BCNF_ERR_ARG;
  if (n_rows == 0) return BCNF_OK;
  if (!params || !packed || !z || !h || !y || !scratch || !aligned16(scratch) || (L.Cp == L.C && !aligned16(h)))
    return BCNF_ERR_ARG;
  if (!cond_index && h_rows != n_rows) return BCNF_ERR_ARG;
  return wide_inverse(L, params, (const float*)packed, z, h, h_rows, cond_index, n_rows, y, training != 0, rng_state,
                      (float*)scratch, (hipStream_t)stream);
}

#ifdef BCNF_PHASE_STAMPS
// Diagnostic build only: phase timestamps (s_memtime) of workgroup 0 of every forward link launch into dbg[0..6].
int bcnf_wide_debug_phases(unsigned long long* dbg) {
  g_link_dbg = dbg;
  return BCNF_OK;
}
int bcnf_wide_debug_wbr(unsigned long long* out) {   // g_wbr_st of the latest tiling-W launch -> host [256][8]
  return bcnf_rt::hip_status(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wbr_st), sizeof(g_wbr_st)));
}
#endif

// Test hook: one plain GEMM through the tile machinery. layout: 0 = NT (A[m][k], B[n][k]), 1 = NN (A[m][k], B[k][n]),
// 2 = TN (A[k][m], B[k][n]), 3 = TT (A[k][m], B[n][k]).
int bcnf_wide_gemm_test(int32_t layout, int32_t M, int32_t N, int32_t K, const float* A, int64_t lda, const float* B,
                        int64_t ldb, float* C, int64_t ldc, void* stream) {
  GemmArgs g = gemm_args(layout >> 4, M, N, K, A, lda, B, ldb, C, ldc);
  layout &= 15;
  hipStream_t st = (hipStream_t)stream;
  if (layout == 0) return gemm<true, true, EPI_STORE>(g, 1, st);
  if (layout == 1) return gemm<true, false, EPI_STORE>(g, 1, st);
  if (layout == 2) return gemm<false, false, EPI_STORE>(g, 1, st);
  if (layout == 3) return gemm<false, true, EPI_STORE>(g, 1, st);
  return BCNF_ERR_ARG;
}

}  // extern "C"
