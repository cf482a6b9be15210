// bcnf_amd: fused CondRealNVP_v2 coupling stack for MI355X (gfx950 / CDNA4).
//
// Kernels (all fp32):
//   k_pack      canonical nn.Module parameters -> per-lane LDS records (rotation-ready weight rows),
//               plus the ActNorm log|det| constant  sum_k sum_i log|scale_k,i|   (cnf.py:350)
//   k_forward   whole-stack forward, one launch: ActNorm -> nested MLP (GELU, dropout) -> affine
//               coupling -> log-det -> orthonormal mix, for all n_blocks   (cnf.py:476-488)
//   k_inverse   whole-stack inverse, one launch                              (cnf.py:499-506)
//   k_backward  whole-stack backward with per-block recompute, one launch; dW via fp32 MFMA on LDS
//               tiles of the workgroup's 16 samples; per-workgroup slabs
//   k_bwd_tail  deterministic slab sum -> canonical flat gradient
//
// Reference: psaegert/bcnf src/bcnf/models/cnf.py. See DESIGN.md for layouts and rooflines.
#include "bcnf_device.h"
#include "../../include/bcnf_amd.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>


// Phase stamps (s_memtime per phase of workgroup 0's first compute and helper waves) exist only in a diagnostic
// build with -DBCNF_PHASE_STAMPS (tools/exp_variants.sh); the shipped library has no stamp code, no debug globals
// and no debug exports.
#ifdef BCNF_PHASE_STAMPS
#define BCNF_STAMPS 1
#else
#define BCNF_STAMPS 0
#endif

namespace {

constexpr int NC16_MAX = 16;           // C <= 256: register-resident column tiles of k_hp / k_dh / k_dw1h            // tiles: D_1..D_NH, D_T, D_S, A_0..A_NH, PA, GA, PB, GB
// Backward LDS tile of [16 samples s][16 columns r], unpadded: the four samples 4 t + q (t = 0..3) of column r sit in
// the 16-B slot tile_slot(r, q) = 4 r + ((q + (r >> 1)) & 3), so the MFMA operand of lane (q, r) for the four K-steps t
// is ONE 16-B read at 4 tile_slot(r, q), and each ds_read_b128 lane group covers all 16 slot banks (conflict-free). The
// rotation by r >> 1 also spreads the element stores: a compute / helper wave holds samples w + 4 i (sample_of) --
// one q per wave, t = i -- so a 32-lane half stores to 16 distinct banks (2-way, which costs a ds_write_b32 nothing;
// the padded pitch-24 rows were 4-way: 4.13M conflict cycles per k_backward launch).
constexpr int TILE = 256;
__host__ __device__ constexpr int tile_slot(int r, int q) { return 4 * r + ((q + (r >> 1)) & 3); }
__host__ __device__ constexpr int tile_ix(int s, int r) { return 4 * tile_slot(r, s & 3) + (s >> 2); }
// Sample (0..15) a forward / backward thread t8 (role-relative, 256 per role) works on: wave w = t8 >> 6 holds the
// samples w + 4 i of its four 16-lane rows i (the activation records and the derivative slots are per t8, so both
// kernels use the same map).
__host__ __device__ constexpr int sample_of(int t8) { return (t8 >> 6) + 4 * ((t8 >> 4) & 3); }
constexpr int STAGE_REC = 4;   // 16 * RF (RB) floats  <= 4 float4 per thread (RF, RB <= 256)
constexpr int RING = STAGE_REC * BCNF_WG * 4;    // floats per record-ring slot: a Stage stores all of it
constexpr int RAW_KP = 100;   // pack-free forward: LDS row pitch of the staged Wf / x rows (X <= 96), = 4 mod 32
// floats per lane of a block's activation record (ActRec); the AR1 single floats follow all the float4 parts
__host__ __device__ constexpr int act_rec_floats(int NH) { return 2 * NH + 3; }
__host__ __device__ constexpr long long ar1_off(int nb, long long nwg, int ar4) { return (long long)nb * nwg * ar4 * 4 * 256; }
// floats per block of a backward workgroup's gradient slab: NH + 2 MFMA tiles + NH + 6 column sums (BwdJobs)
__host__ __device__ constexpr int slab_blk_floats(int NH) { return (NH + 2) * 256 + (NH + 6) * 16; }

// ------------------------------------------------------------------------------------------------
// Host-side layout
// ------------------------------------------------------------------------------------------------
int round_rec(int n) {            // multiple of 4 floats with odd quotient (conflict-free ds_read_b128)
  n = (n + 3) & ~3;
  if (((n / 4) & 1) == 0) n += 4;
  return n;
}

// Broadcast-form sections (row_newbcast DPP, D_a = 10 / D_b = 9 stacks only): QBC_W1 Linear 1 (forward), QBC_MIX
// the mix Q / Q^T (forward, inverse, backward), QBC_HEAD the T / S heads' transposes (backward).
#ifndef BCNF_QBC_MASK
#define BCNF_QBC_MASK 7
#endif
constexpr int QBC_W1 = 1, QBC_MIX = 2, QBC_HEAD = 4;
// the kernels' test of a section's form (BCNF_QBC_CONST: a compile-time answer, for layout-specific A/B builds)
#ifdef BCNF_QBC_CONST
#define QBC_DEV(L, bit) (BCNF_QBC_CONST != 0)
#else
#define QBC_DEV(L, bit) (((L).qbc & (bit)) != 0)
#endif

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
  L->ldh = d->n_conditions;
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
  L->cblk = L->blk_stride - L->H[1] * L->C;
  L->blk_pad = (L->cblk + 3) & ~3;
  L->sblk = slab_blk_floats(L->NH);
  L->qbc = (L->Da == 10 && L->Db == 9) ? BCNF_QBC_MASK : 0;
  L->p = d->dropout;
  L->keep_scale = (d->dropout > 0.f) ? (1.0f / (1.0f - d->dropout)) : 1.0f;
  const double t32 = std::min(4294967295.0, floor((double)d->dropout * 4294967296.0 + 0.5));   // dropout_bits
  L->thr_hi = (uint32_t)t32 >> 16;
  L->thr_lo = (uint32_t)t32 & 0xffffu;
  // forward/inverse record: [sa ba sb bb][b1 pad pad pad][W1y:16][hidden l: 16+1 ...][T:16+1][S:16+1][Q:64]
  L->rf_b1 = 4;
  L->rf_w1 = 8;
  L->rf_hid = 24;
  L->rf_t = L->rf_hid + 17 * (L->NH > 0 ? L->NH - 1 : 0);
  L->rf_s = L->rf_t + 17;
  L->rf_q = (L->rf_s + 17 + 3) & ~3;
  L->RF = round_rec(L->rf_q + 64);
  // backward record, in the order the backward consumes it (so its LDS reads are waited for piecewise, not all at
  // once): [ActNorm sa ba sb bb][Q^T:64][Tout^T:16][Sout^T:16][hidden^T l = NH .. 2: 16 each][W1T:16]
  L->rb_an = 0;
  L->rb_qt = 4;
  L->rb_tt = 68;
  L->rb_st = 84;
  L->rb_hid = 100;                             // hidden layer l at rb_hid + 16 (NH - l)
  L->rb_w1t = 100 + 16 * (L->NH > 0 ? L->NH - 1 : 0);
  L->RB = round_rec(L->rb_w1t + 16);
  long long nbl = L->nb;
  L->pf_off = 0;
  L->pb_off = L->pf_off + nbl * 16 * L->RF;
  L->pi_off = L->pb_off + nbl * 16 * L->RB;
  L->NKp = ((L->nb * 16 + 63) / 64) * 64;
  L->w1c_off = L->pi_off + nbl * 16 * L->RF;
  L->w1r_off = L->w1c_off + (long long)L->Cp * L->NKp;
  L->b1c_off = L->w1r_off + (long long)L->NKp * L->Cp;
  L->ldc_off = L->b1c_off + L->NKp;
  // matrix-core inverse record in MFMA A-operand order (k_inverse_mfma, inv_mo_*): NH + 6 matrices x 64 lanes x 4
  // steps, hidden / T / S biases as [4 q][4 r], ActNorm inverse [4 q][4 r][4]
  L->PMB = (L->NH + 6) * 256 + (L->NH - 1) * 16 + 32 + 64;
  L->pm_off = L->ldc_off + 4;
  L->total = L->pm_off + nbl * L->PMB;
  return BCNF_OK;
}

size_t fwd_lds_bytes(const BcnfLayout& L) {   // forward / inverse record ring (2 blocks)
  return sizeof(float) * (size_t)(2 * RING);
}
size_t fwd2_lds_bytes(const BcnfLayout& L, bool raw = false) {  // k_forward: record ring, projection partials,
  return sizeof(float) * (size_t)(3 * RING + 3 * 4 * 256 + 3 * 8 * 256 +   // dropout masks (3 slots)
                                  (raw ? 4 + 16 * (128 + 4) + (L.C + 16) * RAW_KP : 0));   // RAW: log-det
                                                                           // partials, h tile, staged Wf / x
}
size_t bwd_lds_bytes(const BcnfLayout& L) {   // backward record ring, delta tiles (2), activation tiles (3), derivative slots (2)
  return sizeof(float) * (size_t)(2 * RING + 2 * (L.NH + 6) * TILE + 3 * (L.NH + 1) * TILE + 2 * 3 * 4 * 256);
}
constexpr size_t LDS_MAX = 160 * 1024;

bool layout_supported(const BcnfLayout& L, const BcnfStackDesc* d) {
  if (d->two_way) return false;
  if (L.NH < 1 || L.NH > BCNF_MAX_HIDDEN) return false;
  if (L.Da > 16 || L.Db > 16) return false;
  for (int l = 1; l <= L.NH; ++l)
    if (L.H[l] > 16) return false;
  if (L.C < 1 || L.Cp > 16 * NC16_MAX) return false;
  if (sizeof(float) * (size_t)(64 * 132 + 128 * (L.Cp + 32)) > LDS_MAX) return false;   // k_dw1h staging
  if (16 * L.RF > 4 * 4 * BCNF_WG || 16 * L.RB > 4 * 4 * BCNF_WG) return false;
  if (fwd_lds_bytes(L) > LDS_MAX || bwd_lds_bytes(L) > LDS_MAX) return false;
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

// Input index of record entry r of lane j in a matvec section: rotation form (r-th rotation: input (j - r) & 15) or,
// with L.qbc's bit for the section (QBC_*), broadcast form (entry r = input r; bc10 / bc9x2 / mix_bc).
__host__ __device__ inline int rec_src(const BcnfLayout& L, int j, int r, int bit) {
  return (L.qbc & bit) ? r : ((j - r) & 15);
}

// Entry c (0..63) of lane j of a mix section -> (quadrant qi: 0 a->a, 1 b->a, 2 a->b, 3 b->b, input src of the
// quadrant's input half); false: a padding entry. Rotation form: 16 entries per quadrant; broadcast form (mix_bc):
// entries [0, D) feed output half a, [D, 2D) half b, each over the D inputs (a's Da first, then b's Db).
__host__ __device__ inline bool q_entry(const BcnfLayout& L, int j, int c, int* qi, int* src) {
  if (!(L.qbc & QBC_MIX)) {
    *qi = c / 16;
    *src = (j - c % 16) & 15;
    return true;
  }
  const int D = L.D;
  if (c >= 2 * D) return false;
  const int oh = c / D, gi = c % D;
  *qi = 2 * oh + (gi < L.Da ? 0 : 1);
  *src = gi < L.Da ? gi : gi - L.Da;
  return true;
}

// The mix weight of quadrant qi from input src (of its input half) to output lane j (of its output half) in block k:
// y_new = y @ Q (cnf.py:335) or, inverse, z_prev = y @ Q^T (cnf.py:339); the identity after the last block (no mix),
// so the kernels need no branch.
__device__ float q_quad(const BcnfLayout& L, const float* Q, int k, int j, int qi, int src, bool inverse) {
  const int Da = L.Da, Db = L.Db, D = L.D;
  const int no = (qi < 2) ? Da : Db, ni = (qi & 1) ? Db : Da;   // output / input half widths
  if (j >= no || src >= ni) return 0.f;
  if (k >= L.nb - 1) return ((qi == 0 || qi == 3) && src == j) ? 1.f : 0.f;
  const float* q = Q + (long long)k * D * D;
  const int gi = (qi & 1) ? Da + src : src, go = (qi < 2) ? j : Da + j;   // global input / output index
  return inverse ? q[go * D + gi] : q[gi * D + go];
}

// PF (inverse=false) / PI (inverse=true) record entry e of lane j in block k.
__device__ float rec_f(const BcnfLayout& L, const float* P, const float* Q, int k, int j, int e, bool inverse) {
  const int Da = L.Da, Db = L.Db, D = L.D, NH = L.NH;
  const bool has_an = L.act_norm && k < L.nb - 1;
  const int anb = k * L.blk_stride;
  if (e < 4) {   // ActNorm scale / bias; the inverse record holds 1 / scale (the inverse multiplies, no fp32 divide)
    switch (e) {
      case 0: return (j < Da) ? (has_an ? (inverse ? 1.f / P[anb + j] : P[anb + j]) : 1.f) : 0.f;
      case 1: return (j < Da && has_an) ? P[anb + D + j] : 0.f;
      case 2: return (j < Db) ? (has_an ? (inverse ? 1.f / P[anb + Da + j] : P[anb + Da + j]) : 1.f) : 0.f;
      default: return (j < Db && has_an) ? P[anb + D + Da + j] : 0.f;
    }
  }
  if (e == L.rf_b1) return (j < L.H[1]) ? cB(L, P, k, 1, j) : 0.f;
  if (e >= L.rf_w1 && e < L.rf_w1 + 16) {
    const int src = rec_src(L, j, e - L.rf_w1, QBC_W1);
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
    int qi, src;
    if (!q_entry(L, j, e - L.rf_q, &qi, &src)) return 0.f;
    return q_quad(L, Q, k, j, qi, src, inverse);
  }
  return 0.f;
}

// PB record entry (transposed weight rows for the backward).
__device__ float rec_b(const BcnfLayout& L, const float* P, const float* Q, int k, int j, int e) {
  const int NH = L.NH, Db = L.Db;
  if (e >= L.rb_w1t && e < L.rb_w1t + 16) {
    const int src = (j - (e - L.rb_w1t)) & 15;
    return (j < L.Da && src < L.H[1]) ? cW(L, P, k, 1, src, j) : 0.f;
  }
  if (e >= L.rb_hid && e < L.rb_w1t) {
    const int l = NH - (e - L.rb_hid) / 16, r = (e - L.rb_hid) % 16, src = (j - r) & 15;
    return (j < L.H[l - 1] && src < L.H[l]) ? cW(L, P, k, l, src, j) : 0.f;
  }
  if (e >= L.rb_tt && e < L.rb_tt + 32) {
    const int half = (e - L.rb_tt) / 16, src = rec_src(L, j, (e - L.rb_tt) % 16, QBC_HEAD);
    return (j < L.H[NH] && src < Db) ? cW(L, P, k, NH + 1, half * Db + src, j) : 0.f;
  }
  if (e >= L.rb_qt && e < L.rb_qt + 64) return rec_f(L, P, Q, k, j, L.rf_q + (e - L.rb_qt), true);
  if (e >= L.rb_an && e < L.rb_an + 4) return rec_f(L, P, Q, k, j, e - L.rb_an, false);
  return 0.f;
}

// Matrix-core inverse record of block k in MFMA A-operand order, entry e (k_inverse_mfma): matrix m's lane l = (q, s)
// reads ONE float4 at m * 256 + 4 l -- its A operands of the layer's 4 K-steps t -- instead of 4 scalar reads of the
// row-layout inverse record at lane-dependent offsets (bank conflicts: DESIGN 3e). Values are PI-record entries
// (rec_f, inverse = true): m = 0..3 the mix quadrants qi (half -> half), 4 Linear 1 (half -> hidden), 5 .. NH + 3
// the hidden layers, NH + 4 / NH + 5 the T / S heads (hidden -> half). PERM (D_a, D_b <= 12): half-vector feature
// 3q + r in register r < 3; rows with no feature read lane 15's zero entry.
__device__ float rec_pm(const BcnfLayout& L, const float* P, const float* Q, int k, int e) {
  const int NH = L.NH, nm = NH + 6;
  const bool perm = L.Da <= 12 && L.Db <= 12;
  auto feat = [&](int q, int r) { return perm ? (r < 3 ? 3 * q + r : 15) : 4 * q + r; };
  if (e < nm * 256) {
    const int m = e >> 8, l = (e >> 2) & 63, t = e & 3, q = l >> 4, s = l & 15;
    const bool none = perm && (s & 3) == 3;
    const int fo = perm ? 3 * (s >> 2) + (s & 3) : s;
    const int ch = perm ? 3 * q + t : 4 * q + t, cu = 4 * q + t;
    if (m < 4) {                                                           // mix quadrant qi = m
      if (perm && t == 3) return 0.f;
      return none ? 0.f : q_quad(L, Q, k, fo, m, ch, true);
    }
    if (m == 4) {                                                          // Linear 1, y-part
      if (perm && t == 3) return 0.f;
      return (s < L.H[1] && ch < L.Da) ? cW(L, P, k, 1, s, ch) : 0.f;
    }
    if (m < NH + 4) return rec_f(L, P, Q, k, s, L.rf_hid + 17 * (m - 5) + ((s - cu) & 15), true);
    const int off = (m == NH + 4) ? L.rf_t : L.rf_s;
    return none ? rec_f(L, P, Q, k, 15, off, true) : rec_f(L, P, Q, k, fo, off + ((fo - cu) & 15), true);
  }
  e -= nm * 256;
  if (e < (NH - 1) * 16) {                                                 // hidden biases, row 4q + r
    const int h = e >> 4, q = (e >> 2) & 3, r = e & 3;
    return rec_f(L, P, Q, k, 4 * q + r, L.rf_hid + 17 * h + 16, true);
  }
  e -= (NH - 1) * 16;
  if (e < 32) {                                                            // T / S biases, row feat(q, r)
    const int half = e >> 4, q = (e >> 2) & 3, r = e & 3;
    return rec_f(L, P, Q, k, feat(q, r), (half ? L.rf_s : L.rf_t) + 16, true);
  }
  e -= 32;                                                                 // ActNorm inverse [1/sa ba 1/sb bb]
  const int q = e >> 4, r = (e >> 2) & 3, i = e & 3;
  return rec_f(L, P, Q, k, feat(q, r), i, true);
}

// ------------------------------------------------------------------------------------------------
// Pack-free training forward (bcnf_fold_train_forward, round 4): the forward's helper waves build each block's
// forward record straight from the canonical parameters instead of reading a packed copy, so the folded training
// step needs no pack launch. The record entries of a block k < nb - 1 that are not structurally zero are each one
// parameter at a block-independent offset from k * blk_stride (ActNorm, coupling Linears) or from k * D * D
// (the orthonormal mix); RawTable lists them once per layout, split into P-sourced and Q-sourced slots of RAW_NP /
// RAW_NQ entries per helper thread (padding entries copy parameter 0 into an unused word of the ring slot), so a
// helper thread gathers its entries with block-uniform base pointers and never branches. The zero entries stay zero
// in the LDS ring (zeroed once); the last block (no ActNorm, identity mix) goes through rec_f itself.
// ------------------------------------------------------------------------------------------------
constexpr int RAW_NP = 10, RAW_NQ = 2, RAW_NZ = 6;   // slots per helper thread (FC_small: 2152 P-sourced, 361
                                                     // Q-sourced and 1071 zero entries)
constexpr int RAW_NS = RAW_NP + RAW_NQ + RAW_NZ;
constexpr int RAW_NSP = (RAW_NS + 3) & ~3;   // a thread's entries, contiguous: RAW_NSP / 4 16-byte loads
constexpr int RAW_DUMMY = RING - 1;       // an unused float of a ring slot (16 RF <= RING - 1)
constexpr int RAW_SRC_MAX = 1 << 20;

// A table entry: destination float of the ring slot (j * RF + e, < 4096) | source offset << 12.
__host__ __device__ constexpr uint32_t raw_entry(int dst, int src) { return (uint32_t)dst | ((uint32_t)src << 12); }

// Source of mix-section entry c of lane j (q_entry / q_quad): kind 2 (qmats at k * D * D + off) or 0 (zero).
int q_quad_source(const BcnfLayout& L, int j, int c, bool inverse, int* off) {
  int qi, src;
  if (!q_entry(L, j, c, &qi, &src)) return 0;
  const int Da = L.Da, Db = L.Db, D = L.D;
  const int no = (qi < 2) ? Da : Db, ni = (qi & 1) ? Db : Da;
  if (j >= no || src >= ni) return 0;
  const int gi = (qi & 1) ? Da + src : src, go = (qi < 2) ? j : Da + j;
  *off = inverse ? go * D + gi : gi * D + go;
  return 2;
}

// Source of forward-record entry e of lane j for a block k < nb - 1: kind 0 = structurally zero, 1 = params at
// k * blk_stride + off, 2 = qmats at k * D * D + off; -1 = a constant the table cannot express (no ActNorm: 1.0).
// Mirrors rec_f (inverse = false) entry by entry.
int rec_f_source(const BcnfLayout& L, int j, int e, int* off) {
  const int Da = L.Da, Db = L.Db, D = L.D, NH = L.NH, an = L.an_size;
  auto lin_w = [&](int l, int row, int col) { return an + L.lin_w[l] + row * L.lin_in[l] + col; };
  *off = 0;
  if (e < 4) {
    if (!L.act_norm) return ((e == 0 && j < Da) || (e == 2 && j < Db)) ? -1 : 0;
    switch (e) {
      case 0: return j < Da ? (*off = j, 1) : 0;
      case 1: return j < Da ? (*off = D + j, 1) : 0;
      case 2: return j < Db ? (*off = Da + j, 1) : 0;
      default: return j < Db ? (*off = D + Da + j, 1) : 0;
    }
  }
  if (e == L.rf_b1) return j < L.H[1] ? (*off = an + L.lin_b[1] + j, 1) : 0;
  if (e >= L.rf_w1 && e < L.rf_w1 + 16) {
    const int src = rec_src(L, j, e - L.rf_w1, QBC_W1);
    return (j < L.H[1] && src < Da) ? (*off = lin_w(1, j, src), 1) : 0;
  }
  if (e >= L.rf_hid && e < L.rf_t) {
    const int l = 2 + (e - L.rf_hid) / 17, r = (e - L.rf_hid) % 17;
    if (r == 16) return j < L.H[l] ? (*off = an + L.lin_b[l] + j, 1) : 0;
    const int src = (j - r) & 15;
    return (j < L.H[l] && src < L.H[l - 1]) ? (*off = lin_w(l, j, src), 1) : 0;
  }
  if (e >= L.rf_t && e < L.rf_t + 34) {
    const int half = (e - L.rf_t) / 17, r = (e - L.rf_t) % 17;
    if (r == 16) return j < Db ? (*off = an + L.lin_b[NH + 1] + half * Db + j, 1) : 0;
    const int src = (j - r) & 15;
    return (j < Db && src < L.H[NH]) ? (*off = lin_w(NH + 1, half * Db + j, src), 1) : 0;
  }
  if (e >= L.rf_q && e < L.rf_q + 64) return q_quad_source(L, j, e - L.rf_q, false, off);
  return 0;
}

// Source of backward-record entry e of lane j for a block k < nb - 1 (mirrors rec_b): kinds as rec_f_source.
int rec_b_source(const BcnfLayout& L, int j, int e, int* off) {
  const int NH = L.NH, Da = L.Da, Db = L.Db, D = L.D, an = L.an_size;
  auto lin_w = [&](int l, int row, int col) { return an + L.lin_w[l] + row * L.lin_in[l] + col; };
  *off = 0;
  if (e >= L.rb_w1t && e < L.rb_w1t + 16) {
    const int src = (j - (e - L.rb_w1t)) & 15;
    return (j < Da && src < L.H[1]) ? (*off = lin_w(1, src, j), 1) : 0;
  }
  if (e >= L.rb_hid && e < L.rb_w1t) {
    const int l = NH - (e - L.rb_hid) / 16, r = (e - L.rb_hid) % 16, src = (j - r) & 15;
    return (j < L.H[l - 1] && src < L.H[l]) ? (*off = lin_w(l, src, j), 1) : 0;
  }
  if (e >= L.rb_tt && e < L.rb_tt + 32) {
    const int half = (e - L.rb_tt) / 16, src = rec_src(L, j, (e - L.rb_tt) % 16, QBC_HEAD);
    return (j < L.H[NH] && src < Db) ? (*off = lin_w(NH + 1, half * Db + src, j), 1) : 0;
  }
  if (e >= L.rb_qt && e < L.rb_qt + 64) return q_quad_source(L, j, e - L.rb_qt, true, off);   // Q^T
  if (e >= L.rb_an && e < L.rb_an + 4) return rec_f_source(L, j, e - L.rb_an, off);
  return 0;
}

// Words of the pack-free forward's table: the forward slots [256 threads][RAW_NSP] (a thread's slots contiguous, so
// it loads them with RAW_NSP / 4 16-byte loads), then one block's backward record [16 RB] as (source << 2 | kind)
// with kind 0 params, 1 qmats, 2 zero.
long long raw_table_words(const BcnfLayout& L) { return (long long)RAW_NSP * BCNF_WG + 16LL * L.RB; }

// The table [RAW_NS][BCNF_WG] (P slots, then Q slots, then zero slots) for layout L: every float of a ring slot's
// 16 RF record floats belongs to exactly one (thread, slot), so a helper thread writes its own words and no two
// threads race. Within a kind the entries go in SOURCE order, entry n to slot n / 256, thread n % 256: a wave's
// gather then reads 64 consecutive parameters (the P entries are exactly a block's parameters minus the W1
// condition columns, the Q entries all of Q_k) -- a few cache lines per load instead of one per lane -- and the
// scattered side is the LDS write. Padding entries name RAW_DUMMY. False if the raw path does not apply (no
// ActNorm: constant entries; or more entries of a kind than slots).
bool build_raw_table(const BcnfLayout& L, uint32_t* out) {
  if (L.nb < 2 || 16 * L.RF > RAW_DUMMY || L.blk_stride >= RAW_SRC_MAX) return false;
  std::vector<std::pair<int, int>> ent[3];                  // (src, dst) per kind: P, Q, zero
  for (int j = 0; j < 16; ++j)
    for (int e = 0; e < L.RF; ++e) {
      int off;
      const int kind = rec_f_source(L, j, e, &off);
      if (kind < 0) return false;
      ent[kind == 1 ? 0 : kind == 2 ? 1 : 2].emplace_back(off, j * L.RF + e);
    }
  const int cap[3] = {RAW_NP, RAW_NQ, RAW_NZ}, first[3] = {0, RAW_NP, RAW_NP + RAW_NQ};
  for (int i = 0; i < RAW_NSP * BCNF_WG; ++i) out[i] = raw_entry(RAW_DUMMY, 0);
  if (L.an_size > BCNF_WG) return false;                     // the ActNorm words (smallest sources) in P slot 0
  for (int g = 0; g < 3; ++g) {
    if ((int)ent[g].size() > cap[g] * BCNF_WG) return false;
    std::sort(ent[g].begin(), ent[g].end());
    for (int n = 0; n < (int)ent[g].size(); ++n)
      out[(n % BCNF_WG) * RAW_NSP + first[g] + n / BCNF_WG] = raw_entry(ent[g][n].second, ent[g][n].first);
  }
  uint32_t* pb = out + (long long)RAW_NSP * BCNF_WG;
  for (int j = 0; j < 16; ++j)
    for (int e = 0; e < L.RB; ++e) {
      int off;
      const int kind = rec_b_source(L, j, e, &off);
      if (kind < 0 || off >= (1 << 29)) return false;
      pb[j * L.RB + e] = ((uint32_t)off << 2) | (uint32_t)(kind == 1 ? 0 : kind == 2 ? 1 : 2);
    }
  return true;
}

// Grid: 1 workgroup that computes the ActNorm log|det| constant  sum_k sum_i log|scale_k,i|  (cnf.py:350) in a
// fixed order, then npw record workgroups (grid-stride over every packed float; pack_wgs gives every thread about
// one element, so the launch is one load round trip, not a chain of them).
constexpr int PACK_WG_MAX = 4096;

// train_only (the folded training step, bcnf_pack_params_fold): only what its forward, backward and tail read --
// PF, PB, W1hR and the log-det constant -- not the inverse records PI / PM (the costliest entries: rec_pm calls
// rec_f per element) nor the unfolded projection's W1hC / b1c: about half the elements of a full pack.
__device__ __forceinline__ void pack_body(const BcnfLayout& L, const float* __restrict__ P,
                                          const float* __restrict__ Q, float* __restrict__ out, int bx, int npw,
                                          float* __restrict__ part, bool train_only = false) {
  if (bx == 0) {
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
    return;
  }
  // every packed section is < 2^31 floats (layout_supported bounds the shapes), so 32-bit index math
  const int n_pf = L.nb * 16 * L.RF;
  const int n_pb = L.nb * 16 * L.RB;
  const int n_w = L.Cp * L.NKp;                       // each of W1hC, W1hR
  const int n_pm = L.nb * L.PMB;
  const int total = train_only ? n_pf + n_pb + n_w : 2 * n_pf + n_pb + 2 * n_w + L.NKp + n_pm;
  for (int ii0 = (bx - 1) * BCNF_WG + threadIdx.x; ii0 < total; ii0 += npw * BCNF_WG) {
    float v;
    long long o;
    // train_only: [PF | PB | W1hR] mapped onto the full pack's index space (PI and W1hC skipped)
    const int i = (train_only && ii0 >= n_pf + n_pb) ? ii0 + n_pf + n_w : ii0;
    if (i < n_pf) {                                   // PF
      const int kj = i / L.RF, e = i - kj * L.RF;
      v = rec_f(L, P, Q, kj >> 4, kj & 15, e, false);
      o = L.pf_off + i;
    } else if (i < n_pf + n_pb) {                     // PB
      const int ii = i - n_pf;
      const int kj = ii / L.RB, e = ii - kj * L.RB;
      v = rec_b(L, P, Q, kj >> 4, kj & 15, e);
      o = L.pb_off + ii;
    } else if (i < 2 * n_pf + n_pb) {                 // PI
      const int ii = i - n_pf - n_pb;
      const int kj = ii / L.RF, e = ii - kj * L.RF;
      v = rec_f(L, P, Q, kj >> 4, kj & 15, e, true);
      o = L.pi_off + ii;
    } else if (i < 2 * n_pf + n_pb + n_w) {           // W1hC [c][kj]
      const int ii = i - 2 * n_pf - n_pb;
      const int c = ii / L.NKp, kj = ii - c * L.NKp, k = kj >> 4, j = kj & 15;
      v = (k < L.nb && j < L.H[1] && c < L.C) ? cW(L, P, k, 1, j, L.Da + c) : 0.f;
      o = L.w1c_off + ii;
    } else if (i < 2 * n_pf + n_pb + 2 * n_w) {       // W1hR [kj][c]
      const int ii = i - 2 * n_pf - n_pb - n_w;
      const int kj = ii / L.Cp, c = ii - kj * L.Cp, k = kj >> 4, j = kj & 15;
      v = (k < L.nb && j < L.H[1] && c < L.C) ? cW(L, P, k, 1, j, L.Da + c) : 0.f;
      o = L.w1r_off + ii;
    } else if (i < 2 * n_pf + n_pb + 2 * n_w + L.NKp) {   // b1c [kj]
      const int kj = i - 2 * n_pf - n_pb - 2 * n_w, k = kj >> 4, j = kj & 15;
      v = (k < L.nb && j < L.H[1]) ? cB(L, P, k, 1, j) : 0.f;
      o = L.b1c_off + kj;
    } else {                                          // PM (matrix-core inverse, operand order)
      const int ii = i - 2 * n_pf - n_pb - 2 * n_w - L.NKp;
      const int k = ii / L.PMB, e = ii - k * L.PMB;
      v = rec_pm(L, P, Q, k, e);
      o = L.pm_off + ii;
    }
    out[o] = v;
  }
}

__global__ __launch_bounds__(BCNF_WG) void k_pack(BcnfLayout L, const float* __restrict__ P,
                                                  const float* __restrict__ Q, float* __restrict__ out, int npw) {
  __shared__ float part[BCNF_WG];
  pack_body(L, P, Q, out, blockIdx.x, npw, part);
}

// Record workgroups of a pack launch (the log-det workgroup not included).
int pack_wgs(const BcnfLayout& L, bool train_only = false) {
  const long long total = train_only ? (long long)L.nb * 16 * (L.RF + L.RB) + (long long)L.Cp * L.NKp
                                     : 2LL * L.nb * 16 * L.RF + (long long)L.nb * 16 * L.RB + 2LL * L.Cp * L.NKp +
                                           L.NKp + (long long)L.nb * L.PMB;
  const long long w = (total + BCNF_WG - 1) / BCNF_WG;
  return (int)(w < PACK_WG_MAX ? (w > 0 ? w : 1) : PACK_WG_MAX);
}

// ------------------------------------------------------------------------------------------------
// Folded linear feature network (training fast path when the feature stack is ONE nn.Linear,
// feature_network.py:114-145 with sizes [X, C] — trajectory_FC_small). h = x Wf^T + bf reaches the stack
// only through the condition projection, so with kj = k*16 + j and W1h_k[j][c] = W1_k[j][Da + c]:
//   HP[k][r][j] = sum_xc x[r][xc] Wc[xc][kj] + bc[kj],  Wc[xc][kj] = sum_c W1h_k[j][c] Wf[c][xc],
//                                                       bc[kj]     = b1_k[j] + sum_c W1h_k[j][c] bf[c]
// and with Gx[kj][xc] = sum_b D1[k][b][j] x1[b][xc]  (x1 = [x | 1], D1 = dL/d pre-activation of Linear 1):
//   dW1h_k[j][c] = sum_{xc<X} Gx[kj][xc] Wf[c][xc] + Gx[kj][X] bf[c]
//   dWf[c][xc]   = sum_kj W1h_k[j][c] Gx[kj][xc],       dbf[c] = sum_kj W1h_k[j][c] Gx[kj][X]
// h and dL/dh are never formed: the feature Linear's forward GEMM, the dL/dh GEMM and the feature dW split-K
// disappear from the step (same sums, reassociated: fp32 rounding differs from the unfolded path at ~1e-6).
// The fold buffer: Wc [Xp][NKp] then bc [NKp], Xp = 16-multiple > X (row X, the ones column, is zero).
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline int fold_xp(int X) { return ((X + 1 + 15) / 16) * 16; }

// Layout seen by the projection kernels (k_hp, the split-K dW1h body) when they run on x instead of h.
BcnfLayout fold_layout(const BcnfLayout& L, int X, int ldx) {
  BcnfLayout F = L;
  F.C = X;
  F.ldh = ldx;
  F.Cp = fold_xp(X);
  F.w1c_off = 0;
  F.b1c_off = (long long)F.Cp * L.NKp;
  return F;
}

// Fold workgroup f: block k = f / 4, rows j0 = 4 (f % 4) .. j0 + 3; thread xc < Xp computes column xc of
// W1h_k[j0:j0+4] [Wf | bf | 0]: Wc[xc][kj] for xc < X, the bias dot for xc == X, zero rows X..Xp-1. One staging
// round trip (the 4 W1h rows, [c][4] in LDS, read as broadcast float4), then C independent L2-resident loads of Wf
// per thread, coalesced across the lanes.
constexpr int FOLD_SPLIT = 4;

__device__ __forceinline__ void fold_body(const BcnfLayout& L, const float* __restrict__ P,
                                          const float* __restrict__ wf, const float* __restrict__ bf, int X,
                                          float* __restrict__ fold, int f, float* __restrict__ w1s) {
  const int Xp = fold_xp(X), k = f / FOLD_SPLIT, j0 = (f % FOLD_SPLIT) * 4, tid = threadIdx.x;
  const bool kval = k < L.nb;
  for (int i = tid; i < 4 * L.C; i += BCNF_WG) {
    const int c = i >> 2, jj = i & 3, j = j0 + jj;
    w1s[i] = (kval && j < L.H[1]) ? cW(L, P, k, 1, j, L.Da + c) : 0.f;
  }
  __syncthreads();
  if (tid >= Xp) return;
  const int xc = tid;
  const bool isw = xc < X, live = isw || (xc == X && bf != nullptr);
  const float* src = isw ? wf + xc : bf;
  const int stride = isw ? X : 1;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int c = 0; c < L.C; ++c) {
    const float v = live ? src[(long long)c * stride] : 0.f;
    const floatx4 w = *reinterpret_cast<const floatx4*>(w1s + 4 * c);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[jj] = fmaf(w[jj], v, acc[jj]);
  }
  const int kj = k * 16 + j0;
  if (xc == X) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = j0 + jj;
      fold[(long long)Xp * L.NKp + kj + jj] = (kval && j < L.H[1]) ? cB(L, P, k, 1, j) + acc[jj] : 0.f;
    }
    acc = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  *reinterpret_cast<floatx4*>(fold + (long long)xc * L.NKp + kj) = acc;
}

// NKp / 4 fold workgroups first (they start before the record workgroups), then the optional batch gather's
// workgroups (the step's batch feed: independent of the pack), then k_pack's grid. The fold reads the canonical
// parameters, not k_pack's output.
__global__ __launch_bounds__(BCNF_WG) void k_pack_fold(BcnfLayout L, const float* __restrict__ P,
                                                       const float* __restrict__ Q, float* __restrict__ out,
                                                       const float* __restrict__ wf, const float* __restrict__ bf,
                                                       int X, float* __restrict__ fold, BcnfGatherArgs ga, int npw) {
  __shared__ __attribute__((aligned(16))) float smem[4 * 16 * NC16_MAX];
  const int n_fold = L.NKp / 16 * FOLD_SPLIT;
  int bx = blockIdx.x;
  if (bx < n_fold) {
    fold_body(L, P, wf, bf, X, fold, bx, smem);
    return;
  }
  bx -= n_fold;
  if (bx < ga.nwg) {
    gather2_rows(ga.idx, ga.n, ga.rpw, ga.s0, ga.c0, ga.d0, ga.s1, ga.c1, ga.d1, ga.cursor, bx);
    return;
  }
  pack_body(L, P, Q, out, bx - ga.nwg, npw, smem, true);
}

// ------------------------------------------------------------------------------------------------
// Shared pieces of the stack kernels
// ------------------------------------------------------------------------------------------------
// Cooperative copy of n floats (multiple of 4) global -> registers (phase 1) -> LDS (phase 2), so the
// global latency of the NEXT block's data hides under the current block's compute.
template <int N>
struct Stage {
  floatx4 r[N];
  __device__ __forceinline__ void load(const float* __restrict__ g, int n) {
    const floatx4* g4 = reinterpret_cast<const floatx4*>(g);
    const int n4 = n >> 2, t = (int)threadIdx.x;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = t + i * BCNF_WG;
      r[i] = g4[idx < n4 ? idx : 0];   // unconditional (clamped) so r[] stays in VGPRs
    }
  }
  // all N float4 per thread, no bounds branch: the destination is a RING-sized slot
  __device__ __forceinline__ void store(float* __restrict__ s) const { store_t(s, (int)threadIdx.x); }
  // the same for thread t of a 256-thread role inside a larger workgroup
  __device__ __forceinline__ void load_t(const float* __restrict__ g, int n, int t) {
    const floatx4* g4 = reinterpret_cast<const floatx4*>(g);
    const int n4 = n >> 2;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = t + i * BCNF_WG;
      r[i] = g4[idx < n4 ? idx : 0];
    }
  }
  __device__ __forceinline__ void store_t(float* __restrict__ s, int t) const {
    floatx4* s4 = reinterpret_cast<floatx4*>(s);
#pragma unroll
    for (int i = 0; i < N; ++i) s4[t + i * BCNF_WG] = r[i];
  }
};

// ------------------------------------------------------------------------------------------------
// Condition projection, hoisted out of the stack kernels (one fp32 MFMA GEMM per direction):
//   HP[k][r][j] = sum_c h[r][c] W1_k[j][Da + c] + b1_k[j]     (the y-independent part of Linear 1)
//   dh[b][c]   = sum_k sum_j D1[k][b][j] W1_k[j][Da + c]      (dL/dh, all blocks)
//   dW1_k[j][Da + c] = sum_b D1[k][b][j] h[b][c]               (split-K, then fixed-order reduce)
// W1h^T comes from the packed buffer ([k][Cp][17], zero-padded); D1 = dL/d pre-activation of Linear 1.
// MFMA lane roles: A[l&15][l>>4], B[l>>4][l&15], D[4(l>>4)+i][l&15].
// ------------------------------------------------------------------------------------------------
// The three projection GEMMs (FC_small: 4096 x 512 x 80, 4096 x 80 x 512, 512 x 80 x 4096). They are
// bound by load issue / round trips rather than MFMA, so: operands come from contiguous packed copies
// (W1hC, W1hR) with float4 loads, a workgroup stages a K-chunk of up to 128 of both operands in LDS per
// round trip (next chunk in flight), and the K loops issue all LDS reads of 4-8 steps before their MFMAs.
// VEC: float4 row loads (vec_rows: the row stride ld and the base are 16-byte aligned).
constexpr int KC = 128;                // K-chunk
// LDS strides for the MFMA operand reads: [row = lane&15][k = 4t + lane>>4] wants stride = 4 (mod 32),
// [k = 4t + lane>>4][col = lane&15] wants stride = 16 (mod 32): 64 lanes then hit every bank exactly twice.
constexpr int KCP = KC + 4;            // A tiles [64][KC]
constexpr int BNS = 80;                // k_hp B tile [KC][64]
__host__ __device__ constexpr int bstride16(int n) { return n + ((16 - (n & 31)) & 31); }   // >= n, = 16 mod 32

// Stage rows [r0, r0 + 64) x cols [c0, c0 + KC) of a row-major (nrows x ncols, ld) matrix into regs
// (8 float4 per thread: row = i4 / 32, col = 4 (i4 % 32)), zero outside; column `ones` (>= ncols, or -1 for
// none) of every valid row reads 1.0 (the bias column of the folded feature Linear).
template <bool VEC>
__device__ __forceinline__ void load_rows64(const float* __restrict__ M, long long nrows, int ncols, long long ld,
                                            long long r0, int c0, floatx4* reg, int ones = -1) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int i4 = threadIdx.x + 256 * e, row = i4 >> 5, col = c0 + (i4 & 31) * 4;
    const long long r = r0 + row < nrows ? r0 + row : nrows - 1;
    if (VEC) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(M + r * ld + (col < ncols ? col : 0));
#pragma unroll
      for (int q = 0; q < 4; ++q) reg[e][q] = (r0 + row < nrows && col + q < ncols) ? v[q] : 0.f;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cq = col + q;
        const float v = M[r * ld + (cq < ncols ? cq : ncols - 1)];
        reg[e][q] = (r0 + row < nrows && cq < ncols) ? v : 0.f;
      }
    }
    if (ones >= 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (col + q == ones && r0 + row < nrows) reg[e][q] = 1.f;
    }
  }
}

// HP tile: 64 rows x 64 columns kj. grid = (ceil(R/64), NKp/64)
template <bool VEC>
__global__ __launch_bounds__(BCNF_WG) void k_hp(BcnfLayout L, const float* __restrict__ pk,
                                                const float* __restrict__ h, long long R, float* __restrict__ hp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                    // [64][KCP]  (row, c)
  float* Bs = smem + 64 * KCP;         // [KC][BNS]  (c, kj)
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lq = l >> 4;
  const long long b0 = (long long)blockIdx.x * 64;
  const int n0 = blockIdx.y * 64;
  const int Cp = L.Cp, NKp = L.NKp;
  const float* w1c = pk + L.w1c_off;
  floatx4 ra[8], rb[8];
  auto load = [&](int c0) {
    load_rows64<VEC>(h, R, L.C, L.ldh, b0, c0, ra);
#pragma unroll
    for (int e = 0; e < 8; ++e) {                    // B: [KC rows c][64 cols]: row = i4 / 16, col4
      const int i4 = tid + 256 * e, row = c0 + (i4 >> 4), col = n0 + (i4 & 15) * 4;
      const floatx4 v = *reinterpret_cast<const floatx4*>(w1c + (long long)(row < Cp ? row : Cp - 1) * NKp + col);
      rb[e] = v * (row < Cp ? 1.f : 0.f);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i4 = tid + 256 * e;
      *reinterpret_cast<floatx4*>(As + (i4 >> 5) * KCP + (i4 & 31) * 4) = ra[e];
      *reinterpret_cast<floatx4*>(Bs + (i4 >> 4) * BNS + (i4 & 15) * 4) = rb[e];
    }
  };
  floatx4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = floatx4{0.f, 0.f, 0.f, 0.f};
  load(0);
  float b1v[4];                                        // the epilogue's biases, fetched with the first chunk
#pragma unroll
  for (int u = 0; u < 4; ++u) b1v[u] = pk[L.b1c_off + n0 + 16 * u + lr];
  for (int c0 = 0; c0 < Cp; c0 += KC) {
    store();
    __syncthreads();
    if (c0 + KC < Cp) load(c0 + KC);
    const int ks = (Cp - c0 < KC ? Cp - c0 : KC) >> 2;   // multiple of 4
    for (int t0 = 0; t0 < ks; t0 += 4) {
      float a[4], bv[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = As[(16 * wave + lr) * KCP + 4 * (t0 + t) + lq];
#pragma unroll
        for (int u = 0; u < 4; ++u) bv[t][u] = Bs[(4 * (t0 + t) + lq) * BNS + 16 * u + lr];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = mfma4(a[t], bv[t][u], acc[u]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int kj = n0 + 16 * u + lr, k = kj >> 4;
    if (k < L.nb) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long r = b0 + 16 * wave + 4 * lq + i;
        if (r < R) hp[((long long)k * R + r) * 16 + lr] = acc[u][i] + b1v[u];
      }
    }
  }
}

// dh tile: 64 rows x 16 columns; K = nb * 16 (kj) in chunks of 128 (8 blocks). grid = (ceil(B/64), Cp/16)
__device__ __forceinline__ void dh_body(const BcnfLayout& L, const float* __restrict__ pk, const float* __restrict__ d1,
                                        long long B, float* __restrict__ dh, int bx, int by, float* __restrict__ smem) {
  float* As = smem;                    // [64][KCP] (row b, kj)
  float* Bs = smem + 64 * KCP;         // [KC][16]  (kj, c)
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lq = l >> 4;
  const long long b0 = (long long)bx * 64;
  const int n = by;
  const int K = L.nb * 16, Cp = L.Cp;
  const float* w1r = pk + L.w1r_off + 16 * n;
  floatx4 ra[8], rb[2];
  const int arow = tid >> 2, aj4 = (tid & 3) * 4;
  const long long ab = b0 + arow < B ? b0 + arow : B - 1;
  auto load = [&](int kj0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {                    // A: block (kj0 / 16 + e), rows [b0, b0 + 64) x 16
      const int k = (kj0 >> 4) + e;
      const floatx4 v = *reinterpret_cast<const floatx4*>(d1 + ((long long)(k < L.nb ? k : L.nb - 1) * B + ab) * 16 + aj4);
      ra[e] = v * (k < L.nb ? 1.f : 0.f);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {                    // B: [128 kj][16 c]: row = i4 / 4, col4
      const int i4 = tid + 256 * e, kj = kj0 + (i4 >> 2);
      const floatx4 v = *reinterpret_cast<const floatx4*>(w1r + (long long)(kj < K ? kj : K - 1) * Cp + (i4 & 3) * 4);
      rb[e] = v * (kj < K ? 1.f : 0.f);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < 8; ++e) *reinterpret_cast<floatx4*>(As + arow * KCP + 16 * e + aj4) = ra[e];
#pragma unroll
    for (int e = 0; e < 2; ++e) *reinterpret_cast<floatx4*>(Bs + (tid + 256 * e) * 4) = rb[e];
  };
  floatx4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int kj0 = 0; kj0 < K; kj0 += KC) {
    store();
    __syncthreads();
    if (kj0 + KC < K) load(kj0 + KC);
    const int ks = (K - kj0 < KC ? K - kj0 : KC) >> 2;   // multiple of 4
    for (int t0 = 0; t0 < ks; t0 += 4) {
      float a[4], bv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = As[(16 * wave + lr) * KCP + 4 * (t0 + t) + lq];
        bv[t] = Bs[(4 * (t0 + t) + lq) * 16 + lr];
      }
      acc = mfma4(a[0], bv[0], acc);
      acc1 = mfma4(a[1], bv[1], acc1);
      acc = mfma4(a[2], bv[2], acc);
      acc1 = mfma4(a[3], bv[3], acc1);
    }
    __syncthreads();
  }
  acc += acc1;
  const int col = 16 * n + lr;
  if (col < L.C) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long r = b0 + 16 * wave + 4 * lq + i;
      if (r < B) dh[r * L.C + col] = acc[i];
    }
  }
}

__global__ __launch_bounds__(BCNF_WG) void k_dh(BcnfLayout L, const float* __restrict__ pk,
                                                const float* __restrict__ d1, long long B, float* __restrict__ dh) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  dh_body(L, pk, d1, B, dh, blockIdx.x, blockIdx.y, smem);
}

// dW1h split-K partials: 64 kj (4 blocks, one per wave) x all columns over one split of KC rows.
// grid = (ceil(nb/4), splits); work[s][k][16][Cp]
template <bool VEC, int BPW = 4>
__device__ __forceinline__ void dw1h_body(const BcnfLayout& L, const float* __restrict__ d1, const float* __restrict__ h,
                                          long long B, int rows_per_split, float* __restrict__ work, int bx, int by,
                                          float* __restrict__ smem, int ones = -1) {
  const int hs = bstride16(L.Cp);
  // BPW blocks per workgroup: 4 (one per wave, every column tile) or 2 (two waves per block, half the column
  // tiles each: twice the workgroups, LDS for two resident per CU)
  float* As = smem;                    // [16 BPW][KCP] (kj, b)
  float* Bs = smem + 16 * BPW * KCP;   // [KC][hs]  (b, c)
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lq = l >> 4;
  const int k0 = bx * BPW, s = by;
  const long long m0 = (long long)s * rows_per_split;
  long long m1 = m0 + rows_per_split;
  if (m1 > B) m1 = B;
  const int NC16 = L.Cp >> 4;
  {
    // every global load of the tile goes out before the first LDS store (one round trip, not three): A = the 4
    // blocks' D1 rows [KC][16] (transposed into [kj][b]), B = the split's h rows [KC][Cp] in 64-row halves (a
    // second K-chunk of columns only when Cp > KC)
    const int row = tid >> 1, j8 = (tid & 1) * 8;
    const long long b = m0 + row;
    const bool ok = b < m1;
    const long long bb = ok ? b : m1 - 1;
    floatx4 va[2 * BPW];
#pragma unroll
    for (int kk = 0; kk < BPW; ++kk) {
      const int k = k0 + kk < L.nb ? k0 + kk : L.nb - 1;
      const floatx4* src = reinterpret_cast<const floatx4*>(d1 + ((long long)k * B + bb) * 16 + j8);
      va[2 * kk] = src[0];
      va[2 * kk + 1] = src[1];
    }
    floatx4 rv[2][8];
#pragma unroll
    for (int half = 0; half < 2; ++half) load_rows64<VEC>(h, m1, L.C, L.ldh, m0 + 64 * half, 0, rv[half], ones);
#pragma unroll
    for (int kk = 0; kk < BPW; ++kk) {
      const float m = (ok && k0 + kk < L.nb) ? 1.f : 0.f;
      const floatx4 v0 = va[2 * kk] * m, v1 = va[2 * kk + 1] * m;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        As[(kk * 16 + j8 + q) * KCP + row] = v0[q];
        As[(kk * 16 + j8 + 4 + q) * KCP + row] = v1[q];
      }
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i4 = tid + 256 * e, r = 64 * half + (i4 >> 5), col = (i4 & 31) * 4;
        if (col < L.Cp) *reinterpret_cast<floatx4*>(Bs + r * hs + col) = rv[half][e];
      }
    }
    for (int c0 = KC; c0 < L.Cp; c0 += KC) {           // Cp > 128 only
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        load_rows64<VEC>(h, m1, L.C, L.ldh, m0 + 64 * half, c0, rv[half], ones);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i4 = tid + 256 * e, r = 64 * half + (i4 >> 5), col = c0 + (i4 & 31) * 4;
          if (col < L.Cp) *reinterpret_cast<floatx4*>(Bs + r * hs + col) = rv[half][e];
        }
      }
    }
  }
  __syncthreads();
  const int kw = BPW == 4 ? wave : wave >> 1;
  const int k = k0 + kw;
  const int nh = BPW == 4 ? NC16 : (NC16 + 1) >> 1;
  const int n_lo = BPW == 4 ? 0 : (wave & 1) * nh, n_hi = min(NC16, n_lo + nh);
  float* o = work + (((long long)s * L.nb + (k < L.nb ? k : 0)) * 16) * L.Cp;
  for (int n = n_lo; n < n_hi; ++n) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int t0 = 0; t0 < KC / 4; t0 += 8) {            // LDS reads of 8 steps, then 8 MFMAs (2 chains)
      float a[8], bv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        a[t] = As[(16 * kw + lr) * KCP + 4 * (t0 + t) + lq];
        bv[t] = Bs[(4 * (t0 + t) + lq) * hs + 16 * n + lr];
      }
#pragma unroll
      for (int t = 0; t < 8; t += 2) {
        acc = mfma4(a[t], bv[t], acc);
        acc1 = mfma4(a[t + 1], bv[t + 1], acc1);
      }
    }
    acc += acc1;
    if (k < L.nb) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[(long long)(4 * lq + i) * L.Cp + 16 * n + lr] = acc[i];
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(BCNF_WG) void k_dw1h(BcnfLayout L, const float* __restrict__ d1,
                                                  const float* __restrict__ h, long long B, int rows_per_split,
                                                  float* __restrict__ work) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  dw1h_body<VEC>(L, d1, h, B, rows_per_split, work, blockIdx.x, blockIdx.y, smem);
}

size_t hp_lds_bytes() { return sizeof(float) * (size_t)(64 * KCP + KC * BNS); }
size_t dh_lds_bytes() { return sizeof(float) * (size_t)(64 * KCP + KC * 16); }
size_t dw1h_lds_bytes(const BcnfLayout& L, int bpw = 4) {
  return sizeof(float) * (size_t)(16 * bpw * KCP + KC * bstride16(L.Cp));
}

// Folded path, first launch of the backward tail: the split-K D1^T [x | 1] alone, two blocks per workgroup.
template <bool VEC>
__global__ __launch_bounds__(BCNF_WG) void k_fold_splitk(BcnfLayout F, const float* __restrict__ d1,
                                                         const float* __restrict__ x, long long B, int rows_per_split,
                                                         float* __restrict__ work, int gx_dw, int ones,
                                                         FoldAdamArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (A.on && blockIdx.x == gridDim.x - 1) {       // one extra workgroup: the Adam scalars for k_red_gx / finish
    if (threadIdx.x == 0) adam_scalars_publish(A);
    return;
  }
  dw1h_body<VEC, 2>(F, d1, x, B, rows_per_split, work, blockIdx.x % gx_dw, blockIdx.x / gx_dw, smem, ones);
}

__global__ __launch_bounds__(BCNF_WG) void k_dw1h_reduce(BcnfLayout L, const float* __restrict__ work, int splits,
                                                         float* __restrict__ dparams) {
  const long long per = 16LL * L.Cp, total = (long long)L.nb * per;
  const long long i = (long long)blockIdx.x * BCNF_WG + threadIdx.x;
  if (i >= total) return;
  const int k = (int)(i / per);
  const int rem = (int)(i - (long long)k * per);
  const int j = rem / L.Cp, c = rem - j * L.Cp;
  if (j >= L.H[1] || c >= L.C) return;
  float acc = 0.f;
  int s = 0;
  for (; s + 8 <= splits; s += 8) {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = work[(long long)(s + t) * total + i];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc += v[t];
  }
  for (; s < splits; ++s) acc += work[(long long)s * total + i];
  dparams[coupling_base(L, k) + L.lin_w[1] + j * L.lin_in[1] + L.Da + c] = acc;
}

// Folded path: Gx[kj][xc] = sum of the split-K partials work[s][kj][xc] (fixed order), dense [nb*16][Xp].
__device__ __forceinline__ void gx_reduce_body(long long total, const float* __restrict__ work, int splits,
                                               float* __restrict__ gx, long long i) {
  if (i >= total) return;
  float acc = 0.f;
  int s = 0;
  for (; s + 16 <= splits; s += 16) {               // 16 loads in flight per lane (32 splits at B = 4096)
    float v[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) v[t] = work[(long long)(s + t) * total + i];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc += v[t];
  }
  for (; s < splits; ++s) acc += work[(long long)s * total + i];
  gx[i] = acc;
}

// Folded path, last launch of the backward: two small GEMMs as 16 x 16 output tiles, each operand K-chunk staged
// in LDS as [k][16] in one memory round trip (every load of a chunk issued together: the operands were written by
// other XCDs, so each access is an L2 miss and a streaming K loop of dependent round trips is what costs).
//   role a, workgroups [0, nb * nct): dW1h_k[j][c] = sum_{xc<=X} Gx[k*16+j][xc] Wf1[c][xc]   (Wf1 = [Wf | bf])
//   role b, the rest:               [dWf | dbf][c][xc] = sum_kj W1hR[kj][c] Gx[kj][xc], K = nb*16
// Tile product: thread (ks = lane & 15, rb = lane >> 4, cb = wave) accumulates the 4 x 4 block rows 4rb.., cols
// 4cb.. over k = ks + 16 i (conflict-free ds_read_b128: 16 consecutive rows x 4 float4 per wave), then the 16
// k-slices are summed in a fixed order through LDS.
__device__ __forceinline__ int c0_of_finish(int bx, int nct) { return (bx % nct) * 16; }

constexpr int FIN_KC = 512;                           // K chunk: role a (Xp <= 256) and role b at nb <= 32
                                                      // (K = 16 nb) each load their operands in ONE round trip
constexpr int FIN_SMEM = 2 * FIN_KC * 16;             // As + Bs; the 16 x 256 reduction aliases them

__device__ __forceinline__ void tile16_accum(const float* __restrict__ As, const float* __restrict__ Bs, int kn,
                                             floatx4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, ks = lane & 15, rb = lane >> 4, cb = threadIdx.x >> 6;
#pragma unroll 4
  for (int k = ks; k < kn; k += 16) {
    const floatx4 a = *reinterpret_cast<const floatx4*>(As + k * 16 + 4 * rb);
    const floatx4 b = *reinterpret_cast<const floatx4*>(Bs + k * 16 + 4 * cb);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(a[r], b[c], acc[r][c]);
  }
}

// Fixed-order sum of the 16 k-slices; returns element (row = tid / 16, col = tid % 16) of the tile.
__device__ __forceinline__ float tile16_reduce(float* __restrict__ red, const floatx4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, ks = lane & 15, rb = lane >> 4, cb = threadIdx.x >> 6;
  __syncthreads();                                    // the staging buffers are reused
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[ks * 256 + (4 * rb + r) * 16 + 4 * cb + c] = acc[r][c];
  __syncthreads();
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) v += red[q * 256 + threadIdx.x];
  return v;
}

__global__ __launch_bounds__(BCNF_WG) void k_fold_finish(BcnfLayout L, const float* __restrict__ pk,
                                                         const float* __restrict__ gx, const float* __restrict__ wf,
                                                         const float* __restrict__ bf, int X,
                                                         float* __restrict__ dparams, float* __restrict__ dwf,
                                                         float* __restrict__ dbf, FoldAdamArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];   // FIN_SMEM floats (64 KB: dynamic)
  float* As = smem;
  float* Bs = smem + FIN_KC * 16;
  const int Xp = fold_xp(X), tid = threadIdx.x, nct = L.Cp >> 4;
  floatx4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
  // fused Adam (FoldAdamArgs): this thread's output is one parameter whose gradient it computes; its parameter and
  // moments are fetched now, the update follows the tile product. The launch's last workgroup does the step's
  // bookkeeping (bcnf_adam_step_bookkeep semantics), workgroup 0 stores the logged values.
  // The scalars come from k_fold_splitk (adam_scalars_publish); workgroup 0's log row index is loaded now and its
  // system-scope stores issued once the operands are staged, their fence at the end (no round trip up front).
  const bool adam = A.on && !(A.guard && A.guard[BCNF_GUARD_HALTED]);
  AdamScalars as{};
  // Workgroup 0's thread 0 keeps the step's books (bcnf_adam_step_bookkeep semantics): it alone reads the step count
  // and the cursor in this launch (the scalars came from k_fold_splitk), so it advances both itself at its end --
  // no arrival counter, no last-workgroup round trip.
  const bool keeper = adam && blockIdx.x == 0 && tid == 0;
  const bool logger = keeper && A.log_values && A.log_history;
  long long log_row = 0;
  float step0 = 0.f, log_v[3];
  if (adam) {
    as = adam_scalars_of(A, A.asc[0], A.asc[1]);
    if (keeper) {
      log_row = A.cursor ? A.cursor[0] : 0LL;
      step0 = A.step[0];
    }
    if (logger) {
#pragma unroll
      for (int i = 0; i < 3; ++i) log_v[i] = A.log_values[i];
    }
  }
  int slot = -1;                                       // which parameter tensor / element this thread updates
  long long idx = 0;
  float ap = 0.f, am = 0.f, av = 0.f;
  if ((int)blockIdx.x < L.nb * nct) {
    const int j = tid >> 4, c = c0_of_finish(blockIdx.x, nct) + (tid & 15), k = blockIdx.x / nct;
    if (j < L.H[1] && c < L.C) {
      slot = 0;
      idx = coupling_base(L, k) + L.lin_w[1] + j * L.lin_in[1] + L.Da + c;
    }
  } else {
    const int tile = blockIdx.x - L.nb * nct, c = (tile % nct) * 16 + (tid >> 4), x = (tile / nct) * 16 + (tid & 15);
    if (c < L.C) {
      if (x < X) {
        slot = 1;
        idx = (long long)c * X + x;
      } else if (x == X && dbf) {
        slot = 2;
        idx = c;
      }
    }
  }
  // the slot's tensors picked with constant indices (scalar argument loads + a per-lane select): indexed by the
  // per-lane slot they were per-lane loads of the kernel arguments, a round trip in front of the p / m / v loads
  float *sp = nullptr, *sm = nullptr, *sv = nullptr;
  if (adam) {
    if (slot == 0) {
      sp = A.p[0]; sm = A.m[0]; sv = A.v[0];
    } else if (slot == 1) {
      sp = A.p[1]; sm = A.m[1]; sv = A.v[1];
    } else if (slot == 2) {
      sp = A.p[2]; sm = A.m[2]; sv = A.v[2];
    }
  }
  if (sp) {
    ap = sp[idx];
    am = sm[idx];
    av = sv[idx];
  }
  auto finish_elem = [&](float gval) {
    if (!sp) return;
    adam_elem(ap, gval, am, av, as);
    sp[idx] = ap;
    sm[idx] = am;
    sv[idx] = av;
  };
  auto arrive = [&]() {
    if (!keeper) return;
    if (logger) __threadfence_system();                // the log row's stores (system scope)
    A.step[0] = step0 + 1.0f;                          // advance_counters on the values read at the start
    if (A.cursor) {
      const long long c = log_row + 1;
      A.cursor[0] = c < A.n_batches ? c : 0;
    }
  };
  if ((int)blockIdx.x < L.nb * nct) {
    const int k = blockIdx.x / nct, c0 = (blockIdx.x % nct) * 16;
    const float* g = gx + (long long)k * 16 * Xp;     // [16][Xp], contiguous
    float va[16], vb[16];                             // every load issued before the first LDS store
#pragma unroll
    for (int e = 0; e < 16; ++e) {                    // 16 Xp <= 16 * 256: at most 16 elements per thread
      const int i = tid + BCNF_WG * e;
      const int j = i / Xp, xc = i - j * Xp, c = c0 + j;   // (row, xc) of Gx_k and of Wf1[c0 + row]
      const bool in = i < 16 * Xp;
      va[e] = in ? g[i] : 0.f;
      float v = 0.f;
      if (in && c < L.C) v = xc < X ? wf[(long long)c * X + xc] : ((xc == X && bf) ? bf[c] : 0.f);
      vb[e] = v;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int i = tid + BCNF_WG * e;
      if (i < 16 * Xp) {
        const int j = i / Xp, xc = i - j * Xp;
        As[xc * 16 + j] = va[e];
        Bs[xc * 16 + j] = vb[e];
      }
    }
    __syncthreads();
    if (logger) {                                     // the step's logged values -> history row of this batch
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __hip_atomic_store(A.log_history + 3 * log_row + i, log_v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    tile16_accum(As, Bs, Xp, acc);
    const float v = tile16_reduce(smem, acc);
    const int j = tid >> 4, c = c0 + (tid & 15);
    if (j < L.H[1] && c < L.C) dparams[coupling_base(L, k) + L.lin_w[1] + j * L.lin_in[1] + L.Da + c] = v;
    finish_elem(v);
    __syncthreads();
    arrive();
    return;
  }
  const int tile = blockIdx.x - L.nb * nct, c0 = (tile % nct) * 16, x0 = (tile / nct) * 16;
  const int K = L.nb * 16;
  const float* w1r = pk + L.w1r_off + c0;             // W1hR [NKp][Cp], zero beyond C
  for (int k0 = 0; k0 < K; k0 += FIN_KC) {
    const int kn = min(FIN_KC, K - k0);
    if (k0) __syncthreads();
    floatx4 va[FIN_KC * 4 / BCNF_WG], vb[FIN_KC * 4 / BCNF_WG];
#pragma unroll
    for (int e = 0; e < FIN_KC * 4 / BCNF_WG; ++e) {   // row = i4 / 4, float4 q = i4 % 4
      const int i4 = tid + BCNF_WG * e, r = i4 >> 2, q = i4 & 3, kj = k0 + (r < kn ? r : 0);
      va[e] = *reinterpret_cast<const floatx4*>(w1r + (long long)kj * L.Cp + 4 * q);
      vb[e] = *reinterpret_cast<const floatx4*>(gx + (long long)kj * Xp + x0 + 4 * q);
    }
#pragma unroll
    for (int e = 0; e < FIN_KC * 4 / BCNF_WG; ++e) {
      const int i4 = tid + BCNF_WG * e;
      reinterpret_cast<floatx4*>(As)[i4] = va[e];
      reinterpret_cast<floatx4*>(Bs)[i4] = vb[e];
    }
    __syncthreads();
    tile16_accum(As, Bs, kn, acc);
  }
  const float v = tile16_reduce(smem, acc);
  const int c = c0 + (tid >> 4), x = x0 + (tid & 15);
  if (c < L.C) {
    if (x < X) {
      if (dwf) dwf[(long long)c * X + x] = v;
    } else if (x == X && dbf) {
      dbf[c] = v;
    }
  }
  finish_elem(v);
  __syncthreads();
  arrive();
}

// Compile-time mirror of the forward / backward record layouts of make_layout (checked on the host).
template <int NH>
struct RecF {
  static constexpr int B1 = 4, W1 = 8, HID = 24, T = 24 + 17 * (NH - 1), S = T + 17;
  static constexpr int Q = (S + 17 + 3) & ~3, MLP_END = (S + 17 + 3) & ~3, USED = Q + 64;
};
template <int NH>
struct RecB {   // consumption order (make_layout): ActNorm, Q^T, T / S heads, hidden l = NH .. 2, W1^T
  static constexpr int AN = 0, QT = 4, TT = 68, ST = 84, HID = 100, W1T = 100 + 16 * (NH - 1);
  static constexpr int USED = W1T + 16;
};
// Activation record a training forward saves per (block, sample, lane) for the backward, so the backward never
// recomputes the MLP: masked activations, masked GELU derivatives, tanh(s) and the block input, 2 NH + 3 floats
// stored as AR4 float4 [k][workgroup][AR4][256 threads] plus AR1 floats [k][workgroup][AR1][256] (no padding).
// Order (r05): (activation, derivative) of hidden layer 1, 2, ..., then y_a, y_b, tanh(s) -- a float4 is complete
// every two layers and the forward stores it there (ready_layer), spread over the block. Measured: the
// record writes cost k_forward ~7 us (an ablation without them: 57 -> 50 us), the same whether the stores go out in
// one burst after the coupling, spread like this, or from the helper waves through LDS -- the cost is the 132 MB of
// writes in the memory system, not the issuing wave.
template <int NH>
struct ActRec {
  static constexpr int YA = 2 * NH, YB = 2 * NH + 1, S = 2 * NH + 2;
  static constexpr int AR = 2 * NH + 3, AR4 = AR / 4, AR1 = AR - 4 * AR4;
  __host__ __device__ static constexpr int act(int l) { return 2 * l; }   // hidden layer l + 1
  __host__ __device__ static constexpr int gd(int l) { return 2 * l + 1; }
  // the hidden layer (1-based) after which float4 q is complete; NH + 1: only after tanh(s)
  __host__ __device__ static constexpr int ready_layer(int q) {
    int r = 0;
    for (int i = 4 * q; i < 4 * q + 4; ++i) {
      const int li = i < 2 * NH ? i / 2 + 1 : (i == S ? NH + 1 : 0);
      r = li > r ? li : r;
    }
    return r;
  }
};

// Burst-load floats [lo, hi) of this lane's LDS record into registers (compile-time indices, so the
// array lives in VGPRs): one LDS wait per block instead of one per layer.
template <int LO, int HI>
__device__ __forceinline__ void ld_rec(float* __restrict__ rr, const float* __restrict__ R) {
  static_assert(LO % 4 == 0 && HI % 4 == 0, "record slices are 16-B aligned");
  const floatx4* R4 = reinterpret_cast<const floatx4*>(R + LO);
#pragma unroll
  for (int i = 0; i < (HI - LO) / 4; ++i) {
    const floatx4 v = R4[i];
    rr[LO + 4 * i + 0] = v.x;
    rr[LO + 4 * i + 1] = v.y;
    rr[LO + 4 * i + 2] = v.z;
    rr[LO + 4 * i + 3] = v.w;
  }
}

// Nested MLP forward on the row layout (cnf.py:98-107) from a register-resident forward record.
// Input x (layer-1 y-part operand) and hp (its condition part + bias, from k_hp); returns t and s'
// (pre-tanh). KEEP: also the masked activations and masked GELU derivatives for the backward's record.
template <int NH, bool KEEP>
__device__ __forceinline__ void mlp_forward(const BcnfLayout& L, const float* __restrict__ rr, float x, float hp,
                                            uint32_t bits, bool drop, float& T, float& Sp, float* act, float* gd) {
  using F = RecF<NH>;
  float a = x;
#pragma unroll
  for (int l = 1; l <= NH; ++l) {
    const float* w = (l == 1) ? rr + F::W1 : rr + F::HID + 17 * (l - 2);
    const float bias = (l == 1) ? hp : w[16];            // hp = h W1h^T + b1 (k_hp)
    const float pre = (l == 1 && QBC_DEV(L, QBC_W1)) ? bc10(a, w, bias) : rot16(a, w, bias);   // (uniform)
    const float m = drop ? (((bits >> (l - 1)) & 1u) ? L.keep_scale : 0.f) : 1.f;
    if (KEEP) {
      float g, dg;
      gelu_fg(pre, g, dg);
      a = g * m;
      act[l - 1] = a;
      gd[l - 1] = dg * m;
    } else {
      a = gelu_f(pre) * m;
    }
  }
  T = rr[F::T + 16];
  Sp = rr[F::S + 16];
  rot16x2(a, rr + F::T, T, a, rr + F::S, Sp);
}

// The same with the dropout multipliers as floats (msk[l - 1] = keep_scale or 0 for hidden layer l, drawn by
// k_forward's helper waves): no bit extraction on the compute wave's chain.
template <int NH, bool KEEP, bool DROP>
__device__ __forceinline__ void mlp_forward_m(const float* __restrict__ rr, float x, float hp,
                                              const float* __restrict__ msk, float& T, float& Sp, float* act, float* gd) {
  using F = RecF<NH>;
  float a = x;
#pragma unroll
  for (int l = 1; l <= NH; ++l) {
    const float* w = (l == 1) ? rr + F::W1 : rr + F::HID + 17 * (l - 2);
    const float pre = rot16(a, w, (l == 1) ? hp : w[16]);
    if (KEEP) {
      float g, dg;
      gelu_fg(pre, g, dg);
      a = DROP ? g * msk[l - 1] : g;
      act[l - 1] = a;
      gd[l - 1] = DROP ? dg * msk[l - 1] : dg;
    } else {
      a = DROP ? gelu_f(pre) * msk[l - 1] : gelu_f(pre);
    }
  }
  T = rr[F::T + 16];
  Sp = rr[F::S + 16];
  rot16x2(a, rr + F::T, T, a, rr + F::S, Sp);
}

// Streamed form for k_forward's compute waves (r05). The record is read in consumption order: before stage l (hidden
// layer l = 1..NH, then NH + 1 = the T / S heads, NH + 2 = the mix) the wave issues the quads stage l + FWD_AHEAD
// ends in, behind a scheduling barrier, so each lgkmcnt wait covers reads issued two layers earlier. (r04's
// burst form ld_rec<FWD_HEAD, USED> let hipcc issue 17 reads after layer 1 and wait for all of them at once, then
// 4 and 8 more each with a wait one GELU later: five exposed LDS round trips per block under four waves' load.)
constexpr int FWD_AHEAD = 2;
template <int NH>
__host__ __device__ constexpr int rf_stage_end(int l) {   // exclusive end (floats) of what stage l reads
  return l <= NH ? 24 + 17 * (l - 1) : (l == NH + 1 ? RecF<NH>::S + 17 : RecF<NH>::USED);
}
template <int NH>
__host__ __device__ constexpr int rf_stage_q(int l) {     // quads issued once stage l's reads are out
  // at most 8 new quads per stage (lgkmcnt tracks 15 outstanding: a 16-read burst at the last layer made hipcc wait
  // for its oldest reads at once); whatever the cap defers goes out with the next stage, all of it by the mix
  int q = 6;
  for (int i = 1; i <= l; ++i) {
    const int want = (rf_stage_end<NH>(i + FWD_AHEAD < NH + 2 ? i + FWD_AHEAD : NH + 2) + 3) / 4;
    q = i >= NH + 2 ? want : (want < q + 8 ? want : q + 8);
  }
  return q;
}
template <int NH>
__device__ __forceinline__ void rf_issue(float* __restrict__ rr, const float* __restrict__ R, int l) {
  const floatx4* R4 = reinterpret_cast<const floatx4*>(R);
#pragma unroll
  for (int q = rf_stage_q<NH>(l - 1); q < rf_stage_q<NH>(l); ++q) {
    const floatx4 v = R4[q];
    rr[4 * q] = v.x;
    rr[4 * q + 1] = v.y;
    rr[4 * q + 2] = v.z;
    rr[4 * q + 3] = v.w;
  }
  __builtin_amdgcn_sched_barrier(0);
}
// KEEP: the activation record goes to ar (ActRec order), and emit(q) is called right after float4 q is complete.
template <int NH, bool KEEP, bool DROP, typename Emit>
__device__ __forceinline__ void mlp_forward_s(float* __restrict__ rr, const float* __restrict__ R, float x, float hp,
                                              const float* __restrict__ msk, float& T, float& Sp, float* ar,
                                              Emit&& emit, bool qbc) {
  static_assert(RecF<NH>::HID == 24, "stage 1 reads only the prefetched head (FWD_HEAD = 24)");
  using F = RecF<NH>;
  using AR = ActRec<NH>;
  float a = x;
#pragma unroll
  for (int l = 1; l <= NH; ++l) {
    rf_issue<NH>(rr, R, l);
    const float* w = (l == 1) ? rr + F::W1 : rr + F::HID + 17 * (l - 2);
    const float pre = (l == 1 && qbc) ? bc10(a, w, hp) : rot16(a, w, (l == 1) ? hp : w[16]);   // (uniform)
    if (KEEP) {
      float g, dg;
      gelu_fg(pre, g, dg);
      a = DROP ? g * msk[l - 1] : g;
      ar[AR::act(l - 1)] = a;
      ar[AR::gd(l - 1)] = DROP ? dg * msk[l - 1] : dg;
#pragma unroll
      for (int q = 0; q < AR::AR4; ++q)
        if (AR::ready_layer(q) == l) emit(q);
    } else {
      a = DROP ? gelu_f(pre) * msk[l - 1] : gelu_f(pre);
    }
  }
  rf_issue<NH>(rr, R, NH + 1);
  T = rr[F::T + 16];
  Sp = rr[F::S + 16];
  rot16x2(a, rr + F::T, T, a, rr + F::S, Sp);
  rf_issue<NH>(rr, R, NH + 2);   // (empty: the mix's quads went out with stage NH)
}

// Row-layout orthonormal mix: (na, nb) = (a, b) @ M with the four pre-rotated quadrants at rq
// (register-resident): [a->a | b->a | a->b | b->b].
__device__ __forceinline__ void mix(const float* __restrict__ rq, float a, float b, float& na, float& nbv) {
  na = 0.f;
  nbv = 0.f;
  rot16x2(a, rq, na, a, rq + 32, nbv);
  rot16x2(b, rq + 16, na, b, rq + 48, nbv);
}

// ------------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------------
#if BCNF_STAMPS
__device__ unsigned long long g_phase[32];   // phase stamps (bcnf_debug_phases), diagnostic build only
#endif

// Condition projection operands of the forward (the y-independent part of Linear 1, cnf.py:98-107 with the
// condition columns): HP[b][16k + j] = sum_c h[b][c] W1hC[c][16k + j] + b1c[16k + j]; on the folded path h = x and
// W1hC / b1c are the folded Wc / bc (fold_layout).
struct ProjArgs {
  const float* h;
  const float* w1c;      // [Cp][NKp], rows >= C zero
  const float* b1c;      // [NKp]
  long long ldh;
  int C, Cp, NKp;
};
// RAW (bcnf_fold_train_forward): the pack-free folded training forward, so the folded training step needs no pack
// launch. Differences from the packed forward, all in the prologue and the helper waves:
//  * records: each helper thread owns RAW_NS words of a ring slot (build_raw_table) and gathers block k's record
//    straight from the parameters -- RAW_NP loads at k * blk_stride + src, RAW_NQ at k * D * D + src, zero words
//    written once; the last block (no ActNorm, identity mix) through rec_f on the same words;
//  * projection: helper wave hw computes h^T = Wf x^T + bf for its 16-column tiles ct = hw, hw + 4, .. of the
//    workgroup's 16 samples on fp32 MFMA (once), and that output layout IS the projection's A operand with the K
//    order (ct, r) -> column 16 ct + 4 lq + r, so no LDS round trip: per block the B operand is W1_k[j][Da + that
//    column] read from the parameters. The sums are the unfolded ones (h first), not the folded Wc;
//  * batch rows: with idx the rows come from the pools (the captured step's batch gather), and the forward writes
//    the gathered y and x rows for the backward;
//  * side outputs for the backward kernels, spread over the grid in the helpers' first interval: the backward
//    records PB and W1hR into `pk`; the compute waves sum the ActNorm log-det constant themselves.
struct RawArgs {
  const float* P;          // canonical flat parameters
  const float* Q;          // orthonormal matrices [nb - 1][D][D]
  const uint32_t* table;   // [RAW_NS][256] (build_raw_table)
  const float* wf;         // feature Linear weight [C][X]
  const float* bf;         // its bias [C] (nullable)
  const float* ypool;      // y rows [*][D]
  float* ydst;             // gathered y rows [B][D] (nullable: no copy)
  const float* xpool;      // x rows [*][ldx]
  float* xdst;             // gathered x rows [B][ldx] (nullable: no copy)
  const int64_t* idx;      // batch row b -> pool row idx[(cursor ? cursor[0] * B : 0) + b]; NULL: row b
  const long long* cursor;
  float* pk;               // packed buffer: PB and W1hR are written here
  int X, ldx;
};
constexpr int RAW_WQ = 8;              // Wf quads per thread in flight while staging (C * ceil(X / 4) <= 2048 in one go)
constexpr int RAW_TPW = 2;             // h column tiles per helper wave: C <= 128
constexpr int RAW_SIDE_Q = 4;          // side units per workgroup done in the idle interval
__host__ __device__ constexpr int raw_hs_pitch(int C) { return 16 * ((C + 15) / 16) + 4; }
__device__ __forceinline__ long long raw_row(const RawArgs& R, long long B, long long b) {
  return R.idx ? (long long)R.idx[(R.cursor ? R.cursor[0] * B : 0) + b] : b;
}

constexpr int FWD_WG = 2 * BCNF_WG;
constexpr int HP_SMAX = 16;            // K-steps of 4 per helper wave: Cp / 16 <= 16 (Cp <= 256)
constexpr int FWD_SLOTS = 3;           // ring depth: the helpers prepare block k + 2 while block k runs
constexpr int FWD_HP = FWD_SLOTS * 4 * 256;   // LDS: [slot][4 helper waves][16 samples][16] partial HP tiles
constexpr int FWD_HEAD = 24;           // record floats the compute waves prefetch one block ahead (ActNorm, b1, W1y)

// Whole-stack forward, one launch, 512 threads = two roles per SIMD (waves w and w + 4 share a SIMD):
//  * compute waves 0..3 (4 samples each, row layout): ActNorm -> nested MLP (GELU, dropout) -> affine coupling ->
//    log-det -> orthonormal mix of block k, reading its record, condition projection and dropout multipliers from
//    LDS;
//  * helper waves 4..7 prepare block k + 2 in the same interval (a 3-slot ring): stage its forward record into LDS,
//    compute its condition projection for the workgroup's 16 samples on fp32 MFMA (one K-quarter per helper wave;
//    the compute lanes add the four partials in a fixed order), and draw its dropout multipliers (Philox -> floats).
// With the ring one block deeper, the compute waves read block k + 1's record head, projection partials and
// multipliers at the end of block k (its slot is complete since the previous barrier), so a block starts without
// an LDS round trip: a lone wave per SIMD is issue-bound on its own stream (tools/probe_issue.py, recalibrated in
// r05: ~5 cycles per plain VALU, 6-8 per DPP FMA), and the old block start waited for 27 record reads of
// all four compute waves. The rest of the record streams in two stages ahead (mlp_forward_s).
// The projection needs no separate GEMM launch and no HBM round trip, and the compute waves' loop issues no global
// loads (the record stores of SAVE are its only VMEM traffic).
template <int NH, bool DROP, bool SAVE, bool RAW = false>
__global__ __launch_bounds__(2 * BCNF_WG) void k_forward(BcnfLayout L, const float* __restrict__ pk,
                                                    const float* __restrict__ y, ProjArgs P,
                                                    long long B, float* __restrict__ z, float* __restrict__ ldj_out,
                                                    float* __restrict__ logp, const uint64_t* rng,
                                                    float* __restrict__ arec, float* __restrict__ nll_part,
                                                    RawArgs R) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int RFL = 16 * L.RF;
  float* rec = smem;                          // [3][16*RF]
  float* hpb = rec + FWD_SLOTS * RING;        // [3][4][16][16]
  floatx4* mkb = reinterpret_cast<floatx4*>(hpb + FWD_HP);   // [3][2][256] dropout multipliers of layers 1..8
  float* lps = hpb + FWD_HP + FWD_SLOTS * 8 * 256;            // RAW: the helpers' log-det constant partials [4]
  float* hs = lps + 4;                                        // RAW: h of the 16 rows [16][raw_hs_pitch(C)]
  using AR = ActRec<NH>;
  static_assert(NH <= 8, "two float4 of dropout multipliers");
  const int nb = L.nb;
  const float* pf = pk + L.pf_off;
  const bool helper = threadIdx.x >= BCNF_WG;
  const int t8 = (int)threadIdx.x & (BCNF_WG - 1);              // thread index within the role
  const int j = t8 & 15, s = sample_of(t8);                     // (sample, lane) of a compute / Philox thread
  const long long b = (long long)blockIdx.x * 16 + s;
  const long long bc = b < B ? b : B - 1;                       // rows past the batch replay the last sample
  uint64_t seed = 0, off = 0;
  if (DROP) { seed = rng[0]; off = rng[1]; }
  // diagnostic build: per-phase cycles of workgroup 0's wave 0 (compute) and wave 4 (helper) -> g_phase[8..]
  unsigned long long ph_t = BCNF_STAMPS ? __builtin_amdgcn_s_memtime() : 0ULL, ph_acc[3] = {0, 0, 0};
  const unsigned long long ph_t0 = ph_t;
  const unsigned long long ph_r0 = BCNF_STAMPS ? __builtin_amdgcn_s_memrealtime() : 0ULL;   // 100 MHz
  unsigned long long ph_b[2] = {0, 0};   // RAW prologue: cycles from the start to barrier #0 / #1 arrival
#define PHB(i)                                                 \
  if (BCNF_STAMPS) ph_b[i] = __builtin_amdgcn_s_memtime() - ph_t0;
  unsigned long long ph_p[4] = {0, 0, 0, 0};   // RAW prologue points (each after an explicit wait: stamped build only)
#define PHP(i)                                                                           \
  if (BCNF_STAMPS) {                                                                     \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                          \
    ph_p[i] = __builtin_amdgcn_s_memtime() - ph_t0;                                      \
  }
#define PHF(i)                                                                                   \
  if (BCNF_STAMPS) {                                                                             \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                                  \
    ph_acc[i] += _t - ph_t;                                                                      \
    ph_t = _t;                                                                                   \
  }

  if (helper) {
    const int hw = __builtin_amdgcn_readfirstlane(t8 >> 6);
    const int l64 = t8 & 63, lr = l64 & 15, lq = l64 >> 4;
    if constexpr (RAW) {
      const int Da = L.Da, C = L.C, X = R.X, H1 = L.H[1], D = L.D, an = L.an_size;
      const int nt = (C + 15) >> 4;                               // 16-column tiles of h (<= 4 RAW_TPW)
      const long long row = (long long)blockIdx.x * 16 + lr;
      const float* xrow = R.xpool + raw_row(R, B, row < B ? row : B - 1) * R.ldx;
      // ---- prologue loads, all issued before any of them is consumed ----
      // this thread's table slots: RAW_NSP / 4 16-byte loads, all issued before any is used (decoded one at a time,
      // the compiler waited for each load before issuing the next)
      uint32_t tw[RAW_NSP];
#pragma unroll
      for (int i = 0; i < RAW_NSP / 4; ++i) {
        const uint4 v = reinterpret_cast<const uint4*>(R.table + t8 * RAW_NSP)[i];
        tw[4 * i] = v.x;
        tw[4 * i + 1] = v.y;
        tw[4 * i + 2] = v.z;
        tw[4 * i + 3] = v.w;
      }
      // side units of this workgroup (RawSide): backward-record chunks u < nb * ch, then W1hR rows
      const int rb16 = 16 * L.RB, ch = (rb16 + BCNF_WG - 1) / BCNF_WG, n_units = nb * ch + L.NKp;
      const uint32_t* tpb = R.table + RAW_NSP * BCNF_WG;
      uint32_t pbe[RAW_SIDE_Q];                                   // (the unit checks happen at the use)
#pragma unroll
      for (int q = 0; q < RAW_SIDE_Q; ++q) {
        const int u = blockIdx.x + q * gridDim.x, n = (u % ch) * BCNF_WG + t8;
        pbe[q] = tpb[n < rb16 ? n : 0];
      }
      asm volatile("" ::: "memory");                              // the table loads above are all in flight
      uint32_t srcb[RAW_NP + RAW_NQ], dstb[RAW_NP + RAW_NQ];      // byte offsets: source, word of the ring slot
#pragma unroll
      for (int i = 0; i < RAW_NP + RAW_NQ; ++i) {
        srcb[i] = (tw[i] >> 12) * 4u;
        dstb[i] = (tw[i] & 4095u) * 4u;
      }
      uint32_t zw[RAW_NZ];
#pragma unroll
      for (int i = 0; i < RAW_NZ; ++i) zw[i] = tw[RAW_NP + RAW_NQ + i] & 4095u;
      PHP(0)
      // projection B operand of block k: W1_k[lr][Da + 16 ct + 4 lq + r], r = 0..3 one (dword-aligned) 16-byte load
      // per tile (at most 3 floats past the row end: still inside the block's parameters), zero past C or H[1]
      int wo[RAW_TPW];
      uint32_t wok = 0;
#pragma unroll
      for (int i = 0; i < RAW_TPW; ++i) {
        const int c0 = 16 * (hw + 4 * i) + 4 * lq;
        wo[i] = (c0 < C && lr < H1) ? L.lin_w[1] + lr * L.lin_in[1] + Da + c0 : 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) wok |= (c0 + r < C && lr < H1) ? 1u << (4 * i + r) : 0u;
      }
      const bool bias_lane = hw == 0 && lr < H1;
      struct Pre {                                                // one block's loaded operands
        float v[RAW_NP + RAW_NQ];
        floatx4 w4[RAW_TPW];
        float bias;
      };
      // buffer loads: the block base goes in the scalar offset, the table's byte offset in the vector offset (no
      // per-lane 64-bit address arithmetic, which otherwise stays live across the loop)
      const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(R.P), (short)0,
                                                                         (int)(L.n_trainable * 4), 0x00020000);
      const __amdgpu_buffer_rsrc_t rQ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(R.Q), (short)0,
                                                                         (nb - 1) * D * D * 4, 0x00020000);
      // The last block (rec_f with k = nb - 1) goes through the same branch-free loads: its coupling sits an_size
      // floats earlier in its block (no ActNorm), so the P base shifts by -an_size and only the ActNorm words --
      // the an_size smallest sources, slot 0 of threads < an_size -- take constants (scale 1, bias 0); its Q base
      // lies past the end of qmats, where the buffer range check returns 0, and the diagonal words take 1
      // (identity mix). Those fix-ups happen at the use (finish_rec), so no load is waited for early.
      const bool an_word = (int)(srcb[0] >> 2) < an;
      const float an_val = (int)(srcb[0] >> 2) < D ? 1.f : 0.f;
      bool q_diag[RAW_NQ];
#pragma unroll
      for (int i = 0; i < RAW_NQ; ++i) q_diag[i] = ((srcb[RAW_NP + i] >> 2) % (uint32_t)(D + 1)) == 0;
      auto load = [&](int k, Pre& g) {
        const int cb = coupling_base(L, k);
        const int sp = (k < nb - 1 ? k * L.blk_stride : k * L.blk_stride - an) * 4, sq = k * D * D * 4;
#pragma unroll
        for (int i = 0; i < RAW_NP; ++i)
          g.v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rP, srcb[i], sp, 0));
#pragma unroll
        for (int i = RAW_NP; i < RAW_NP + RAW_NQ; ++i)
          g.v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rQ, srcb[i], sq, 0));
#pragma unroll
        for (int i = 0; i < RAW_TPW; ++i) {   // unconditional (wo = 0 for an absent tile, whose MFMAs are skipped)
          const auto w = __builtin_amdgcn_raw_buffer_load_b128(rP, wo[i] * 4, cb * 4, 0);
          g.w4[i] = floatx4{__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]), __uint_as_float(w[3])};
        }
        // raw: the select waits for the load, so it happens at the use (finish_proj), not here
        g.bias = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rP, (L.lin_b[1] + lr) * 4, cb * 4, 0));
      };
      float xa[RAW_TPW][4];                                       // h[row lr][16 (hw + 4 i) + 4 lq + r]
      // block k -> slot sl (a constant after unrolling): dropout multipliers and record (no h needed), then the
      // projection partial
      auto finish_rec = [&](int k, int sl, const Pre& g) {
        if (DROP) {
          const uint32_t bits = dropout_bits<NH>(L, seed, off, bc, k, j, 0u);
          float m[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) m[i] = ((bits >> i) & 1u) ? L.keep_scale : 0.f;
          mkb[(2 * sl) * BCNF_WG + t8] = floatx4{m[0], m[1], m[2], m[3]};
          mkb[(2 * sl + 1) * BCNF_WG + t8] = floatx4{m[4], m[5], m[6], m[7]};
        }
        char* slot = reinterpret_cast<char*>(rec + sl * RING);
        float v0 = g.v[0], vq[RAW_NQ];
#pragma unroll
        for (int i = 0; i < RAW_NQ; ++i) vq[i] = g.v[RAW_NP + i];
        if (k == nb - 1) {                                        // uniform
          v0 = an_word ? an_val : v0;
#pragma unroll
          for (int i = 0; i < RAW_NQ; ++i) vq[i] = q_diag[i] ? 1.f : vq[i];
        }
        *reinterpret_cast<float*>(slot + dstb[0]) = v0;
#pragma unroll
        for (int i = 1; i < RAW_NP; ++i) *reinterpret_cast<float*>(slot + dstb[i]) = g.v[i];
#pragma unroll
        for (int i = 0; i < RAW_NQ; ++i) *reinterpret_cast<float*>(slot + dstb[RAW_NP + i]) = vq[i];
      };
      auto finish_proj = [&](int sl, const Pre& g) {
        const float bias = bias_lane ? g.bias : 0.f;
        floatx4 acc = {bias, bias, bias, bias};
#pragma unroll
        for (int i = 0; i < RAW_TPW; ++i)
          if (hw + 4 * i < nt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc = mfma4(xa[i][r], ((wok >> (4 * i + r)) & 1u) ? g.w4[i][r] : 0.f, acc);
        float* hd = hpb + sl * 1024 + hw * 256 + 64 * lq + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r) hd[16 * r] = acc[r];
      };
      auto finish = [&](int k, int sl, const Pre& g) {
        finish_rec(k, sl, g);
        finish_proj(sl, g);
      };
      Pre gb[FWD_SLOTS];                                          // block b's operands in gb[b % 3] (interval())
      load(0, gb[0]);
      load(1, gb[1]);                                             // nb >= 2 (build_raw_table)
      load(nb > 2 ? 2 : 1, gb[2]);
      asm volatile("" ::: "memory");                              // all three blocks' loads issued here, not sunk
      PHP(1)
#pragma unroll
      for (int i = 0; i < RAW_NZ; ++i)                            // this thread's zero words, in all three slots
#pragma unroll
        for (int sl = 0; sl < FWD_SLOTS; ++sl) rec[sl * RING + zw[i]] = 0.f;
      finish_rec(0, 0, gb[0]);
      finish_rec(1, 1, gb[1]);
      PHP(2)
      __syncthreads();                                            // barrier A (the compute waves' operand staging)
      PHB(0)
      __syncthreads();                                            // barrier B: the compute waves' h tile is in hs
#pragma unroll
      for (int i = 0; i < RAW_TPW; ++i) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(hs + lr * raw_hs_pitch(C) + 16 * (hw + 4 * i) + 4 * lq);
#pragma unroll
        for (int r = 0; r < 4; ++r) xa[i][r] = v[r];
      }
      finish_proj(0, gb[0]);
      finish_proj(1, gb[1]);
      // ---- side work: the backward kernels' inputs, one unit per workgroup and q (coalesced rows) ----
      auto side_unit = [&](int u, uint32_t e) {
        if (u < nb * ch) {
          const int k = u / ch, n = (u - k * ch) * BCNF_WG + t8;
          if (n >= rb16) return;
          const uint32_t kind = e & 3u, src = e >> 2;
          float v = 0.f;
          if (k < nb - 1) {
            if (kind == 0) v = R.P[(long long)k * L.blk_stride + src];
            else if (kind == 1) v = R.Q[(long long)k * D * D + src];
          } else if (kind == 0) {
            v = (int)src < an ? ((int)src < D ? 1.f : 0.f) : R.P[(long long)k * L.blk_stride - an + src];
          } else if (kind == 1) {
            v = (src % (uint32_t)(D + 1)) == 0 ? 1.f : 0.f;
          }
          R.pk[L.pb_off + (long long)k * rb16 + n] = v;
        } else if (u < n_units) {
          const int kj = u - nb * ch, k = kj >> 4, jj = kj & 15;
          const bool live = k < nb && jj < H1;
          const float* w = live ? R.P + coupling_base(L, k) + L.lin_w[1] + jj * L.lin_in[1] + Da : R.P;
          for (int c = t8; c < L.Cp; c += BCNF_WG) R.pk[L.w1r_off + (long long)kj * L.Cp + c] = (live && c < C) ? w[c] : 0.f;
        }
      };
      // intervals k < nb - 2 prepare block k + 2 into slot (k + 2) % 3 (unrolled by 3: constant LDS offsets); the
      // last two intervals have no block to prepare and take the side work: this workgroup's units (k = nb - 2) and
      // the log-det constant into lps for the compute epilogue (k = nb - 1)
      // software-pipelined: block k + 3's operands are loaded in interval k and consumed in interval k + 1, so an
      // interval never waits for its own loads; with the loop unrolled by 3 every buffer index is a constant
      PHB(1)
      auto interval = [&](int k, int sl) {
        // unconditional (block nb - 1 again past the end, unused): a load on one path only would make the wait
        // counts conservative -- the consumers would wait for this interval's loads too
        load(k + 3 < nb ? k + 3 : nb - 1, gb[sl == FWD_SLOTS - 1 ? 0 : sl + 1]);
        asm volatile("" ::: "memory");                            // issued here, consumed next interval
        finish(k + 2, sl, gb[sl]);
        PHF(1)
        // LDS writes complete, then a bare barrier: __syncthreads' release fence would also wait for the loads of
        // block k + 3 still in flight (vmcnt counts them too)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        PHF(2)
      };
      __syncthreads();
      PHF(0)
      for (int k = 0; k < nb - 2; k += FWD_SLOTS) {
        interval(k, 2);
        if (k + 1 < nb - 2) interval(k + 1, 0);
        if (k + 2 < nb - 2) interval(k + 2, 1);
      }
#pragma unroll
      for (int q = 0; q < RAW_SIDE_Q; ++q) side_unit(blockIdx.x + q * gridDim.x, pbe[q]);
      {  // the ActNorm log-det constant  sum_k sum_i log|scale_k,i|  (cnf.py:350): strided partials (loads issued
         // together), a fixed-order butterfly per wave, lps[hw] for the compute epilogue after the last barrier
        constexpr int LU = 4;
        float acc = 0.f;
        const int n = (nb - 1) * D;
        for (int i0 = t8; i0 < n; i0 += LU * BCNF_WG) {
          float v[LU];
#pragma unroll
          for (int u = 0; u < LU; ++u) {
            const int i = i0 + u * BCNF_WG, ii = i < n ? i : 0, kb = ii / D;
            v[u] = R.P[(long long)kb * L.blk_stride + (ii - kb * D)];
          }
#pragma unroll
          for (int u = 0; u < LU; ++u)
            if (i0 + u * BCNF_WG < n) acc += logf(fabsf(v[u]));
        }
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
        if (l64 == 0) lps[hw] = acc;
      }
      __syncthreads();                                            // interval nb - 2
      __syncthreads();                                            // interval nb - 1
      for (int u = blockIdx.x + RAW_SIDE_Q * gridDim.x; u < n_units; u += gridDim.x)   // small grids only
        side_unit(u, u < nb * ch ? tpb[(u % ch) * BCNF_WG + t8 < rb16 ? (u % ch) * BCNF_WG + t8 : 0] : 0u);
    } else {
    const int S = P.Cp >> 4;                                     // K-steps per helper wave
    const long long row = (long long)blockIdx.x * 16 + lr;
    const float* hrow = P.h + (row < B ? row : B - 1) * P.ldh;
    float xa[HP_SMAX];                                           // A operand: this wave's K-quarter of h / x
#pragma unroll
    for (int t = 0; t < HP_SMAX; ++t) {
      const int kk = 4 * (hw * S + t) + lq;
      xa[t] = (t < S && kk < P.C) ? hrow[kk < P.C ? kk : 0] : 0.f;
    }
    const float* wcol = P.w1c + (long long)(4 * hw * S + lq) * P.NKp + lr;   // + 4 t NKp + 16 k
    // block k's projection partial, dropout multipliers and record -> slot sl
    auto prepare = [&](int k, int sl) {
      Stage<STAGE_REC> sr;
      sr.load_t(pf + (long long)k * RFL, RFL, t8);
      float wb[HP_SMAX];
#pragma unroll
      for (int t = 0; t < HP_SMAX; ++t) wb[t] = (t < S) ? wcol[(long long)4 * t * P.NKp + 16 * k] : 0.f;
      if (DROP) {
        const uint32_t bits = dropout_bits<NH>(L, seed, off, bc, k, j, 0u);
        float m[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = ((bits >> i) & 1u) ? L.keep_scale : 0.f;
        mkb[(2 * sl) * BCNF_WG + t8] = floatx4{m[0], m[1], m[2], m[3]};
        mkb[(2 * sl + 1) * BCNF_WG + t8] = floatx4{m[4], m[5], m[6], m[7]};
      }
      const float bias = (hw == 0) ? P.b1c[16 * k + lr] : 0.f;
      floatx4 acc = {bias, bias, bias, bias};
#pragma unroll
      for (int t = 0; t < HP_SMAX; ++t)
        if (t < S) acc = mfma4(xa[t], wb[t], acc);
      float* hd = hpb + sl * 1024 + hw * 256 + 64 * lq + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) hd[16 * r] = acc[r];
      sr.store_t(rec + sl * RING, t8);
    };
    prepare(0, 0);
    if (nb > 1) prepare(1, 1);
    __syncthreads();
    PHF(0)
    int sl = 2;
    for (int k = 0; k < nb; ++k) {
      if (k + 2 < nb) prepare(k + 2, sl);
      sl = sl == FWD_SLOTS - 1 ? 0 : sl + 1;
      PHF(1)
      __syncthreads();
      PHF(2)
    }
    }
  } else {
    const int tid = t8;
    // the compute waves issue ahead of the helper wave on their SIMD whenever both are ready (r06: k_forward
    // -1.1 us same box, profiles/r06b_rawab.txt; the helpers have slack at every block's barrier)
    __builtin_amdgcn_s_setprio(3);
    const int D = L.D, Da = L.Da, Db = L.Db;
    float ya, yb, ldc = 0.f;
    if constexpr (RAW) {
      // h^T = Wf x^T + bf of the workgroup's 16 rows on the matrix cores. Wf (C x X) and the 16 x rows are staged
      // into LDS by coalesced 16-byte loads of all four compute waves (per-lane strided operand loads made ~1.2M
      // cache-line requests per launch and queued everyone's first loads behind them), then compute wave
      // cw takes the column tiles ct = cw + 4 i. K order: MFMA step (u, r) of lane (lr, lq) is column
      // 16 u + 4 lq + r, so each operand quad is one conflict-free ds_read_b128 (row pitch RAW_KP = 4 mod 32), and
      // the output layout (h[row lr][16 ct + 4 lq + r] at lane (lr, lq)) is helper wave cw's projection A operand.
      // ldc: the helpers' wave sums of the ActNorm log-det constant (lps), read after the last barrier.
      const long long src = raw_row(R, B, bc);
      ya = (j < Da) ? R.ypool[src * D + j] : 0.f;
      yb = (j < Db) ? R.ypool[src * D + Da + j] : 0.f;
      // float4 quads per row (<= RAW_KP / 4 - 1): XQ hold columns; the h GEMM's K steps run to XQP, so Wf's quads
      // XQ .. XQP - 1 are stored as zeros -- LDS holds whatever the previous kernel left there, and a 0 x NaN residue
      // made the loss NaN
      const int C = L.C, X = R.X, XQ = (X + 3) >> 2, XQP = ((X + 15) >> 4) * 4;
      float* ws = hs + 16 * raw_hs_pitch(C);                      // Wf [C][RAW_KP]
      float* xs = ws + C * RAW_KP;                                // x rows [16][RAW_KP]
      const int cw = __builtin_amdgcn_readfirstlane(tid >> 6), l64 = tid & 63, lr = l64 & 15, lq = l64 >> 4;
      const float* bfp = R.bf ? R.bf : R.wf;
      float hb[RAW_TPW][4];                                       // bf of the columns this lane ends with
#pragma unroll
      for (int i = 0; i < RAW_TPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cc = 16 * (cw + 4 * i) + 4 * lq + r;
          hb[i][r] = bfp[cc < C ? cc : 0];
        }
      {
        // every staging load in flight at once (one round trip): Wf quad (c, q) = columns 4q .. 4q + 3 of row c,
        // read past the row end into the next row (zeroed below) and past the tensor's end through a range-checked
        // buffer load (0); the x quads of the 16 rows (gathered through idx when given), the row's last partial
        // quad element by element
        const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(R.wf), (short)0,
                                                                           C * X * 4, 0x00020000);
        // the K padding quads first: their stores need no load and go out before the staging round trip
        for (int i = tid; i < C * (XQP - XQ); i += BCNF_WG) {
          const int c = i / (XQP - XQ), q = XQ + (i - c * (XQP - XQ));
          *reinterpret_cast<floatx4*>(ws + c * RAW_KP + 4 * q) = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        const int nq = C * XQ;
        uint32_t v[RAW_WQ][4];
#pragma unroll
        for (int u = 0; u < RAW_WQ; ++u) {
          const int i = tid + u * BCNF_WG, ii = i < nq ? i : 0, c = ii / XQ, q = ii - c * XQ;
          const auto w = __builtin_amdgcn_raw_buffer_load_b128(rW, (c * X + 4 * q) * 4, 0, 0);
          v[u][0] = w[0]; v[u][1] = w[1]; v[u][2] = w[2]; v[u][3] = w[3];
        }
        constexpr int NXQ = (16 * (RAW_KP / 4) + BCNF_WG - 1) / BCNF_WG;
        floatx4 xo[NXQ];
#pragma unroll
        for (int u = 0; u < NXQ; ++u) {
          const int i = tid + u * BCNF_WG, ii = i < 16 * (RAW_KP / 4) ? i : 0;
          const int rr = ii / (RAW_KP / 4), q = ii - rr * (RAW_KP / 4);
          const long long bb = (long long)blockIdx.x * 16 + rr;
          const float* xr = R.xpool + raw_row(R, B, bb < B ? bb : B - 1) * R.ldx + 4 * q;
          xo[u] = floatx4{0.f, 0.f, 0.f, 0.f};
          if (4 * q + 3 < X) {
            __builtin_memcpy(&xo[u], xr, sizeof(floatx4));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (4 * q + r < X) xo[u][r] = xr[r];
          }
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < RAW_WQ; ++u) {
          const int i = tid + u * BCNF_WG, c = i / XQ, q = i - c * XQ;
          if (i < nq) {
            floatx4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = 4 * q + r < X ? __uint_as_float(v[u][r]) : 0.f;
            *reinterpret_cast<floatx4*>(ws + c * RAW_KP + 4 * q) = o;
          }
        }
        for (int i = nq > RAW_WQ * BCNF_WG ? tid + RAW_WQ * BCNF_WG : nq; i < nq; i += BCNF_WG) {   // C X > 7680
          const int c = i / XQ, q = i - c * XQ;
          const auto w = __builtin_amdgcn_raw_buffer_load_b128(rW, (c * X + 4 * q) * 4, 0, 0);
          floatx4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = 4 * q + r < X ? __uint_as_float(w[r]) : 0.f;
          *reinterpret_cast<floatx4*>(ws + c * RAW_KP + 4 * q) = o;
        }
#pragma unroll
        for (int u = 0; u < NXQ; ++u) {
          const int i = tid + u * BCNF_WG;
          if (i < 16 * (RAW_KP / 4)) {
            const int rr = i / (RAW_KP / 4), q = i - rr * (RAW_KP / 4);
            *reinterpret_cast<floatx4*>(xs + rr * RAW_KP + 4 * q) = xo[u];
            const long long bb = (long long)blockIdx.x * 16 + rr;
            if (R.xdst && bb < B && 4 * q < X) {                  // the backward tail's x rows
              float* xd = R.xdst + bb * R.ldx + 4 * q;
              if (4 * q + 3 < X) {
                __builtin_memcpy(xd, &xo[u], sizeof(floatx4));
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  if (4 * q + r < X) xd[r] = xo[u][r];
              }
            }
          }
        }
      }
      PHP(0)
      __syncthreads();                                            // ws / xs complete (barrier A)
      // independent accumulation chains (tile i, parity of r), summed in a fixed order
      floatx4 acc[RAW_TPW][2];
#pragma unroll
      for (int i = 0; i < RAW_TPW; ++i) acc[i][0] = acc[i][1] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < RAW_KP / 16; ++u) {
        if (16 * u >= X) break;                                   // uniform
        const floatx4 xv = *reinterpret_cast<const floatx4*>(xs + lr * RAW_KP + 16 * u + 4 * lq);
#pragma unroll
        for (int i = 0; i < RAW_TPW; ++i) {
          const int ct = cw + 4 * i;
          if (16 * ct < C) {
            const int c = 16 * ct + lr;
            const floatx4 wv = *reinterpret_cast<const floatx4*>(ws + (c < C ? c : 0) * RAW_KP + 16 * u + 4 * lq);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][r & 1] = mfma4(wv[r], xv[r], acc[i][r & 1]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < RAW_TPW; ++i) {
        const int ct = cw + 4 * i;
        if (16 * ct < C) {                                        // uniform
          floatx4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cc = 16 * ct + 4 * lq + r;
            o[r] = cc < C ? (acc[i][0][r] + acc[i][1][r]) + (R.bf ? hb[i][r] : 0.f) : 0.f;
          }
          *reinterpret_cast<floatx4*>(hs + lr * raw_hs_pitch(C) + 16 * ct + 4 * lq) = o;
        }
      }
      PHB(0)
      __syncthreads();                                            // hs complete (barrier B)
      PHB(1)
      if (R.ydst && b < B) {                                      // the gathered y rows for the backward
        if (j < Da) R.ydst[b * D + j] = ya;
        if (j < Db) R.ydst[b * D + Da + j] = yb;
      }
    } else {
      ya = (j < Da) ? y[bc * D + j] : 0.f;
      yb = (j < Db) ? y[bc * D + Da + j] : 0.f;
      ldc = pk[L.ldc_off];
    }
    __syncthreads();
    // block k + 1's head: record floats [0, FWD_HEAD), the four projection partials, the dropout multipliers
    float hd[FWD_HEAD], hq4[4];
    floatx4 mk0 = {1.f, 1.f, 1.f, 1.f}, mk1 = {1.f, 1.f, 1.f, 1.f};
    auto fetch_head = [&](int sl) {
      ld_rec<0, FWD_HEAD>(hd, rec + sl * RING + j * L.RF);
      const float* hq = hpb + sl * 1024 + 16 * s + j;            // [sample][neuron] partial tiles
#pragma unroll
      for (int i = 0; i < 4; ++i) hq4[i] = hq[256 * i];
      if (DROP) {
        mk0 = mkb[(2 * sl) * BCNF_WG + tid];
        mk1 = mkb[(2 * sl + 1) * BCNF_WG + tid];
      }
    };
    fetch_head(0);
    float ldj = 0.f;
    int cur = 0;
    // activation-record destinations, advanced per block: nothing in the loop reads the grid size (hipcc reloaded
    // it from the kernarg segment after every barrier's memory clobber, and that scalar load in flight turned the
    // next LDS wait into lgkmcnt(0))
    int gdim = gridDim.x;
    asm volatile("" : "+s"(gdim));
    floatx4* d4 = reinterpret_cast<floatx4*>(arec) + (long long)blockIdx.x * AR::AR4 * BCNF_WG + tid;
    float* d1p = arec + ar1_off(nb, gdim, AR::AR4) + (long long)blockIdx.x * AR::AR1 * BCNF_WG + tid;
    const long long d4s = (long long)gdim * AR::AR4 * BCNF_WG, d1s = (long long)gdim * AR::AR1 * BCNF_WG;
    for (int k = 0; k < nb; ++k) {
      const int nxt = cur == FWD_SLOTS - 1 ? 0 : cur + 1;
      float rr[RecF<NH>::USED];
#pragma unroll
      for (int i = 0; i < FWD_HEAD; ++i) rr[i] = hd[i];
      const float hpk = ((hq4[0] + hq4[1]) + hq4[2]) + hq4[3];
      const float msk[8] = {mk0[0], mk0[1], mk0[2], mk0[3], mk1[0], mk1[1], mk1[2], mk1[3]};
      const float xa = fmaf(rr[0], ya, rr[1]);          // ActNorm (cnf.py:349)
      const float xb = fmaf(rr[2], yb, rr[3]);
      float T, Sp;
      float ar[AR::AR];                                   // activation record of this block (SAVE)
      ar[AR::YA] = ya;
      ar[AR::YB] = yb;
      // each float4 of the record is stored as soon as it is complete (coalesced across the wave), written through
      // (sc1): the 132 MB of records never sit dirty in the L2s, whose write-back the kernel's end would otherwise
      // wait for (r05: k_forward 55.3 -> 51.5 us, step -1.7 %, profiles/r05zl_ab_write_through_records.txt)
      auto emit = [&](int q) {
        if (SAVE) st4_wt(d4 + q * BCNF_WG, floatx4{ar[4 * q], ar[4 * q + 1], ar[4 * q + 2], ar[4 * q + 3]});
      };
      mlp_forward_s<NH, SAVE, DROP>(rr, rec + cur * RING + j * L.RF, xa, hpk, msk, T, Sp, ar, emit, QBC_DEV(L, QBC_W1));
      const float Sv = tanh_bf(Sp);                      // cnf.py:107
      const float zb = fmaf(exp_fast(Sv), xb, T);        // cnf.py:179
      ldj += Sv;                                         // cnf.py:190
      if (SAVE) {
        ar[AR::S] = Sv;
#pragma unroll
        for (int q = 0; q < AR::AR4; ++q)
          if (AR::ready_layer(q) == NH + 1) emit(q);
#pragma unroll
        for (int i = 0; i < AR::AR1; ++i) st1_wt(d1p + i * BCNF_WG, ar[4 * AR::AR4 + i]);
        d4 += d4s;
        d1p += d1s;
      }
      fetch_head(nxt);     // slot nxt is complete since the previous barrier (after the last block: unused, no
                           // branch); the reads land while the mix runs
      if (QBC_DEV(L, QBC_MIX)) mix_bc(rr + RecF<NH>::Q, xa, zb, ya, yb);   // y @ Q (cnf.py:335); identity after the last block
      else mix(rr + RecF<NH>::Q, xa, zb, ya, yb);
      cur = nxt;
      PHF(1)
      // a bare barrier: the head reads stay in flight across it (nobody writes slot nxt in the next interval; the
      // helpers write slot k % 3, whose reads this block's compute has consumed), so the wait for them lands on
      // their first use in block k + 1, not here
      asm volatile("s_barrier" ::: "memory");
      PHF(2)
    }
    if constexpr (RAW) ldc = ((lps[0] + lps[1]) + lps[2]) + lps[3];
    const float ltot = row_sum16(ldj) + ldc;
    const float q2 = row_sum16(ya * ya + yb * yb);
    if (j < Da) z[bc * D + j] = ya;
    if (j < Db) z[bc * D + Da + j] = yb;
    if (j == 0 && ldj_out) ldj_out[bc] = ltot;
    if (logp && j == 0) logp[bc] = -(0.5f * q2 - ltot) - 0.5f * (float)D * 1.8378770664093454836f;
    if (nll_part && j == 0) rec[s] = (b < B) ? 0.5f * q2 - ltot : 0.f;   // rec: free after the last barrier
  }
#if BCNF_STAMPS
  if (SAVE && blockIdx.x == 0 && (threadIdx.x == 0 || threadIdx.x == BCNF_WG))
  {
    for (int i = 0; i < 3; ++i) g_phase[8 + (helper ? 4 : 0) + i] = ph_acc[i];
    g_phase[helper ? 15 : 11] = (ph_b[1] << 32) | (ph_b[0] & 0xffffffffULL);   // slots 3 / 7 belong to the backward
    for (int i = 0; i < 4; ++i) g_phase[16 + (helper ? 4 : 0) + i] = ph_p[i];
    // the wave's whole life in shader cycles and in 100 MHz ticks: the clock it ran at (MI355X_MICROARCH note 6)
    g_phase[24 + (helper ? 2 : 0)] = __builtin_amdgcn_s_memtime() - ph_t0;
    g_phase[25 + (helper ? 2 : 0)] = __builtin_amdgcn_s_memrealtime() - ph_r0;
  }
#endif
#undef PHF
#undef PHB
#undef PHP
  if (nll_part) {   // per-workgroup partial of inn_nll_loss (utils.py:40-46); reduced by nll_finalize
    __syncthreads();
    if (threadIdx.x == 0) {
      float acc = 0.f;
      for (int i = 0; i < 16; ++i) acc += rec[i];
      nll_part[blockIdx.x] = acc;
    }
  }
}

// Mean of the forward's per-workgroup NLL partials -> loss_out = [loss, nll, mse = 0] (trainer.py:260-266)
// and the dropout RNG offset advance, by ONE workgroup that runs strictly after the forward (a separate
// launch, or workgroup 0 of the backward): no cross-workgroup synchronisation inside any kernel.
// Divergence guard (int32[4], BCNF_GUARD_*): a step whose loss exceeds 1e5 or is NaN while checking is
// enabled raises `diverged` (trainer.py:168 raises after that step's update); the NEXT step's finalize
// then raises `halted`, which turns that step's RNG advance, Adam update, clip and counter advances into
// no-ops -- so an epoch replayed without host syncs stops with the state the reference raises in.
template <int NTH = BCNF_WG>
__device__ void nll_finalize(const float* __restrict__ part, int nparts, long long B, float* __restrict__ loss_out,
                             uint64_t* rng_w, int32_t* guard, float* __restrict__ red) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += NTH) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = NTH / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float nll = red[0] / (float)B;
    loss_out[0] = nll;                                 // (nll + mse * 0) / (1 + 0)   (trainer.py:264)
    loss_out[1] = nll;
    loss_out[2] = 0.f;
    bool halt = false;
    if (guard) {
      if (guard[BCNF_GUARD_DIVERGED]) {
        guard[BCNF_GUARD_HALTED] = 1;
        halt = true;
      } else if (guard[BCNF_GUARD_CHECK] && (nll > 1e5f || isnan(nll))) {
        guard[BCNF_GUARD_DIVERGED] = 1;
      }
    }
    if (rng_w && !halt) rng_w[1] += 1;                 // the forward has read the offset
  }
}

__global__ __launch_bounds__(BCNF_WG) void k_nll_finalize(const float* __restrict__ part, int nparts, long long B,
                                                          float* __restrict__ loss_out, uint64_t* rng_w,
                                                          int32_t* guard) {
  __shared__ float red[BCNF_WG];
  nll_finalize(part, nparts, B, loss_out, rng_w, guard, red);
}

// ------------------------------------------------------------------------------------------------
// Inverse
// ------------------------------------------------------------------------------------------------
template <int NH, bool DROP>
__global__ __launch_bounds__(BCNF_WG) void k_inverse(BcnfLayout L, const float* __restrict__ pk,
                                                     const float* __restrict__ zin, const float* __restrict__ hp,
                                                     long long R, const int64_t* __restrict__ cond_index, long long N,
                                                     float* __restrict__ yout, const uint64_t* __restrict__ rng) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int RFL = 16 * L.RF;
  float* rec = smem;
  const int tid = threadIdx.x, j = tid & 15, s = tid >> 4;
  const long long b = (long long)blockIdx.x * 16 + s;
  const long long bc = b < N ? b : N - 1;
  const int D = L.D, Da = L.Da, Db = L.Db, nb = L.nb;
  const float* pi = pk + L.pi_off;
  const long long hr = cond_index ? (long long)cond_index[bc] : bc;   // projection row of this sample
  const float* hpl = hp + hr * 16 + j;                                // HP[k][hr][j] = hpl[k * R * 16]
  const long long hps = R * 16;

  float ya = (j < Da) ? zin[bc * D + j] : 0.f;
  float yb = (j < Db) ? zin[bc * D + Da + j] : 0.f;
  uint64_t seed = 0, off = 0;
  if (DROP) { seed = rng[0]; off = rng[1]; }
  const int kl = nb - 1;
  float hp_n = hpl[kl * hps];
  {
    Stage<STAGE_REC> sr;
    sr.load(pi + (long long)kl * RFL, RFL);
    sr.store(rec + (kl & 1) * RING);
  }
  __syncthreads();

  for (int k = kl; k >= 0; --k) {
    const int cur = k & 1;
    const int k1 = k >= 1 ? k - 1 : 0;                // clamped: no branches
    Stage<STAGE_REC> sr;
    sr.load(pi + (long long)k1 * RFL, RFL);
    const float hpk = hp_n;
    hp_n = hpl[k1 * hps];
    __builtin_amdgcn_sched_barrier(0);
    float rr[RecF<NH>::USED];
    ld_rec<0, RecF<NH>::USED>(rr, rec + cur * RING + j * L.RF);
    float za, zb;
    if (QBC_DEV(L, QBC_MIX)) mix_bc(rr + RecF<NH>::Q, ya, yb, za, zb);   // z @ Q^T (cnf.py:339); identity for the last block
    else mix(rr + RecF<NH>::Q, ya, yb, za, zb);
    uint32_t bits = 0xffu;
    if (DROP) bits = dropout_bits<NH>(L, seed, off, bc, k, j, 0x40000000u);
    float T, Sp;
    mlp_forward<NH, false>(L, rr, za, hpk, bits, DROP, T, Sp, nullptr, nullptr);
    const float S = tanh_bf(Sp);
    const float ybn = (zb - T) * exp_fast(-S);         // cnf.py:205
    ya = (j < Da) ? (za - rr[1]) * rr[0] : 0.f;        // ActNorm inverse (cnf.py:353-354), rr[0] = 1 / scale;
    yb = (j < Db) ? (ybn - rr[3]) * rr[2] : 0.f;       // identity where none
    sr.store(rec + (cur ^ 1) * RING);
    __syncthreads();
  }
  if (b < N) {
    if (j < Da) yout[b * D + j] = ya;
    if (j < Db) yout[b * D + Da + j] = yb;
  }
}

// Whole-stack inverse on the matrix cores (eval / no dropout: sampling, cnf.py:499-506 via _sample), 16 samples
// per wave. A feature vector of the wave's samples is 4 registers per lane: lane (q = l >> 4, s = l & 15) holds
// features 4q .. 4q+3 of sample s -- exactly the v_mfma_f32_16x16x4f32 output layout D[4q + r][s] of out = W x
// (rows = out features, columns = samples). Contracting the 16 inputs in 4 MFMA steps with input feature 4q + t
// in K-slot q of step t makes the B operand of step t the lane's own register t, so a dense 16 x 16 layer is 4
// MFMAs with no data movement; the A operand (W[s][4q + t]) is one LDS read per step from the same pre-rotated
// inverse record k_inverse uses (entry (o - c) & 15 of out-row o). Mix, Linear 1 (condition part + bias from k_hp
// as the accumulator), hidden layers and the T / S heads run on the matrix pipe; the VALU keeps GELU, tanh, exp
// and the coupling / ActNorm inverse (row-layout k_inverse: ~380 VALU instructions per block per 4 samples, 95% of
// VALU issue in profiles/r02y_k_inverse_pmc_insts.csv). Same sums as k_inverse in a different association order.
// G independent 16-sample groups per wave interleaving their MFMA chains and GELUs (G = 2 measured neutral, DESIGN 3e;
// again with the r04 GELU: 1.304 against 1.295 ms per 512k draws, profiles/r04zc_ab_sample.txt).
constexpr int INV_M_G = 1;
constexpr int INV_M_SPW = 16 * INV_M_G;              // samples per wave
constexpr int INV_M_WG = 512;                       // 8 waves share one record ring (2 x 16 KB): 4 workgroups per CU
constexpr int INV_M_SPB = INV_M_SPW * (INV_M_WG / 64);
template <int NH>
constexpr int inv_m_rf() {                          // L.RF of this NH (round_rec of the record end), compile-time so
  int n = (RecF<NH>::Q + 64 + 3) & ~3;              // every LDS address is a lane base + an immediate offset
  if (((n / 4) & 1) == 0) n += 4;
  return n;
}

// gelu_f's approximation on a pair of values with packed fp32 arithmetic (v_pk_fma_f32 / v_pk_mul_f32: two lanes'
// worth per instruction); the same erfc fit, combined as max(x, 0) - |x| h (one rounding fewer than x (1 - h)).
typedef float f32x2 __attribute__((ext_vector_type(2)));
// max(x, 0) as ONE v_max_f32 (fmaxf under IEEE mode adds a canonicalising max per operand). hipcc pads no hazard
// inside an asm string, and x is usually an MFMA result (its D needs 12 wait states before any VALU read,
// cdna_hip_programming.md, inline-asm rule 2): `after` is a value hipcc computed from x with the pad in front of it,
// so the dependency places this read behind that pad.
__device__ __forceinline__ float relu_f(float x, float after) {
  float r;
  asm("v_max_f32_e32 %0, 0, %1" : "=v"(r) : "v"(x), "v"(after));
  return r;
}
__device__ __forceinline__ f32x2 gelu_f2(f32x2 x) {
  // scalar FMAs here: VOP3 takes |x| as a free source modifier (VOP3P has none)
  const f32x2 den = {fmaf(2.616295218e-01f, fabsf(x.x), 1.0f), fmaf(2.616295218e-01f, fabsf(x.y), 1.0f)};
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 q = {-7.295463979e-02f, -7.295463979e-02f};
  q = __builtin_elementwise_fma(q, t, f32x2{2.239411026e-01f, 2.239411026e-01f});
  q = __builtin_elementwise_fma(q, t, f32x2{-1.021702215e-01f, -1.021702215e-01f});
  q = __builtin_elementwise_fma(q, t, f32x2{1.654430181e-01f, 1.654430181e-01f});
  q = __builtin_elementwise_fma(q, t, f32x2{7.358670980e-02f, 7.358670980e-02f});
  q = __builtin_elementwise_fma(q, t, f32x2{1.080111340e-01f, 1.080111340e-01f});
  q = __builtin_elementwise_fma(q, t, f32x2{1.041427255e-01f, 1.041427255e-01f});
  const f32x2 e = (x * x) * f32x2{-0.72134752044448170368f, -0.72134752044448170368f};
  const f32x2 ez = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
  // x Phi(x) = max(x, 0) - |x| h with h = erfc(|x| / sqrt 2) / 2 = t Q(t) e^{-x^2/2}: one VOP3 FMA per element
  // (|x| as a free source modifier) instead of the sign select, 1 - h and the product x cdf
  const f32x2 h = (t * q) * ez;
  return f32x2{fmaf(-fabsf(x.x), h.x, relu_f(x.x, den.x)), fmaf(-fabsf(x.y), h.y, relu_f(x.y, den.y))};
}
// GELU for the forward-only kernels (sampling): x Phi(x) = max(x, 0) - |x| h(|x|) with log2 h fitted as ONE degree-6
// polynomial in a = min(|x|, 6.5) (the -x^2/2 of erfc's decay is quadratic in a, so it is inside the fit): one exp2
// and no reciprocal per element, 14 instructions per pair against gelu_f2's 20 (two of them transcendental instead
// of four). The pair form of bcnf_device.h gelu_h / gelu_f (same coefficients): fp32 error <= 1 ulp of the result
// above 0, <= 1e-7 below (tools/fit_erf.py: fit_log2h); past |x| = 6.5, |x| h < 3e-10.
__device__ __forceinline__ f32x2 gelu_p2(f32x2 x) {
  // med3(|x|, 0, 6.5): ONE v_med3_f32 with the |x| source modifier (fminf under IEEE mode adds a canonicalising
  // v_max first)
  const f32x2 a = {__builtin_amdgcn_fmed3f(fabsf(x.x), 0.f, 6.5f), __builtin_amdgcn_fmed3f(fabsf(x.y), 0.f, 6.5f)};
  f32x2 p = {3.3094816899392754e-05f, 3.3094816899392754e-05f};
  p = __builtin_elementwise_fma(p, a, f32x2{-7.692371727898717e-04f, -7.692371727898717e-04f});
  p = __builtin_elementwise_fma(p, a, f32x2{8.080773986876011e-03f, 8.080773986876011e-03f});
  p = __builtin_elementwise_fma(p, a, f32x2{-5.3412191569805145e-02f, -5.3412191569805145e-02f});
  p = __builtin_elementwise_fma(p, a, f32x2{-4.5877090096473694e-01f, -4.5877090096473694e-01f});
  p = __builtin_elementwise_fma(p, a, f32x2{-1.1512017250061035e+00f, -1.1512017250061035e+00f});
  p = __builtin_elementwise_fma(p, a, f32x2{-9.99993085861206e-01f, -9.99993085861206e-01f});
  const f32x2 h = {__builtin_amdgcn_exp2f(p.x), __builtin_amdgcn_exp2f(p.y)};
  return f32x2{fmaf(-fabsf(x.x), h.x, relu_f(x.x, a.x)), fmaf(-fabsf(x.y), h.y, relu_f(x.y, a.y))};
}
__device__ __forceinline__ void gelu4(floatx4& a) {
  const f32x2 lo = gelu_p2(f32x2{a[0], a[1]}), hi = gelu_p2(f32x2{a[2], a[3]});
  a[0] = lo.x;
  a[1] = lo.y;
  a[2] = hi.x;
  a[3] = hi.y;
}

template <int NH>
__device__ __forceinline__ floatx4 inv_mv(floatx4 acc, const float* __restrict__ slot, const int (&aoff)[4], int off,
                                          const floatx4& x) {
#pragma unroll
  for (int t = 0; t < 4; ++t) acc = mfma4(slot[aoff[t] + off], x[t], acc);
  return acc;
}
constexpr int INV_M_OCC = 6;   // min waves per SIMD (80 VGPRs, no spills; 5 and 8 measured slower)


// One dense layer on the matrix cores: the lane's A operands of the KS K-steps are ONE float4 of the operand-ordered
// record (rec_pm: matrix mat, lane l), conflict-free ds_read_b128.
template <int G, int KS>
__device__ __forceinline__ void inv_mv_mo(floatx4 (&acc)[G], const float* __restrict__ mat, int l,
                                          const floatx4 (&x)[G]) {
  const floatx4 w = *reinterpret_cast<const floatx4*>(mat + 4 * l);
#pragma unroll
  for (int t = 0; t < KS; ++t) {
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = mfma4(w[t], x[g][t], acc[g]);
  }
}

// PERM (D_a, D_b <= 12): the y / z half-vectors hold feature 3q + r in register r < 3 of lane (q, s) (register 3
// stays 0), so every product with a half-vector input contracts in 3 MFMA steps instead of 4 (mix 16 -> 12 and
// Linear 1 4 -> 3 MFMAs per block) and the coupling / ActNorm inverse runs on 3 registers. Rows of a permuted
// output with no feature read entry 0 of lane record 15, which is zero in the mix, T and S rows when D_a, D_b < 15.
template <int NH, bool PERM>
__global__ __launch_bounds__(INV_M_WG, PERM ? INV_M_OCC - 1 : INV_M_OCC) void k_inverse_mfma(BcnfLayout L, const float* __restrict__ pk,
                                                          const float* __restrict__ zin, const float* __restrict__ hp,
                                                          long long R, const int64_t* __restrict__ cond_index,
                                                          long long N, float* __restrict__ yout) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using F = RecF<NH>;
  constexpr int G = INV_M_G;
  constexpr int KA = PERM ? 3 : 4;                  // MFMA steps over a half-vector input
  constexpr int NM = NH + 6;                         // matrices of the operand-ordered record (rec_pm)
  constexpr int PMB = NM * 256 + (NH - 1) * 16 + 32 + 64;   // == L.PMB (checked by the dispatch)
  constexpr int BIAS = NM * 256, TSB = BIAS + (NH - 1) * 16, ANB = TSB + 32;
  static_assert(PMB <= RING, "operand-ordered record fits a ring slot");
  float* rec = smem;
  const int l = threadIdx.x & 63, q = l >> 4, s = l & 15;
  const int D = L.D, Da = L.Da, Db = L.Db, nb = L.nb;
  const float* pm = pk + L.pm_off;
  long long b[G];
  const floatx4* hpl[G];
  const long long hps4 = R * 4;
  // half-vector feature of register r (15: none -- a zero row of the mix / T / S records)
  auto feat = [&](int r) { return PERM ? (r < 3 ? 3 * q + r : 15) : 4 * q + r; };
  floatx4 ya[G], yb[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    b[g] = (long long)blockIdx.x * INV_M_SPB + (threadIdx.x >> 6) * INV_M_SPW + 16 * g + s;
    const long long bc = b[g] < N ? b[g] : N - 1;
    const long long hr = cond_index ? (long long)cond_index[bc] : bc;
    hpl[g] = reinterpret_cast<const floatx4*>(hp + hr * 16 + 4 * q);   // HP[k][hr][4q..4q+3]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = feat(r);
      ya[g][r] = (f < Da) ? zin[bc * D + f] : 0.f;
      yb[g][r] = (f < Db) ? zin[bc * D + Da + f] : 0.f;
    }
  }

  const int kl = nb - 1;
  floatx4 hp_n[G];
#pragma unroll
  for (int g = 0; g < G; ++g) hp_n[g] = hpl[g][kl * hps4];
  // record staging by LDS-DMA (global_load_lds_dwordx4, no staging registers): wave w copies 1 KB chunks
  // w, w + 8 of block k's record into a ring slot; chunks past the record re-read its start (slot slack)
  const int wv = threadIdx.x >> 6;
  static_assert(RING % (INV_M_WG * 4) == 0, "ring chunks per wave");
  auto stage = [&](int k, float* dst) {
#pragma unroll
    for (int c = 0; c < RING / (INV_M_WG * 4); ++c) {
      const int ch = wv + (INV_M_WG / 64) * c, e = ch * 256 + 4 * l;
      const float* src = pm + (long long)k * PMB + (e < PMB ? e : 0);
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + ch * 256), 16,
                                       0, 0);
    }
  };
  stage(kl, rec + (kl & 1) * RING);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int k = kl; k >= 0; --k) {
    const int cur = k & 1;
    const int k1 = k >= 1 ? k - 1 : 0;
    stage(k1, rec + (cur ^ 1) * RING);               // slot cur ^ 1 was last read before the previous barrier
    floatx4 a[G], za[G], zb[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      a[g] = hp_n[g];                                // Linear 1 accumulator: condition projection + b1 (k_hp)
      hp_n[g] = hpl[g][k1 * hps4];
      za[g] = floatx4{0.f, 0.f, 0.f, 0.f};
      zb[g] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    const float* slot = rec + cur * RING;
    // z @ Q^T (cnf.py:339): quadrants [a->a | b->a | a->b | b->b]; identity for the last block
    inv_mv_mo<G, KA>(za, slot, l, ya);                // quadrant 0: a -> a
    inv_mv_mo<G, KA>(zb, slot + 2 * 256, l, ya);      // quadrant 2: a -> b
    inv_mv_mo<G, KA>(za, slot + 1 * 256, l, yb);      // quadrant 1: b -> a
    inv_mv_mo<G, KA>(zb, slot + 3 * 256, l, yb);      // quadrant 3: b -> b
    // nested MLP (cnf.py:98-107): Linear 1 on za, then the hidden layers
    inv_mv_mo<G, KA>(a, slot + 4 * 256, l, za);
#pragma unroll
    for (int g = 0; g < G; ++g) gelu4(a[g]);
#pragma unroll
    for (int h = 2; h <= NH; ++h) {
      const floatx4 bias = *reinterpret_cast<const floatx4*>(slot + BIAS + 16 * (h - 2) + 4 * q);
      floatx4 x[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        x[g] = a[g];
        a[g] = bias;
      }
      inv_mv_mo<G, 4>(a, slot + (5 + h - 2) * 256, l, x);
#pragma unroll
      for (int g = 0; g < G; ++g) gelu4(a[g]);
    }
    floatx4 T[G], Sp[G];
    const floatx4 tb = *reinterpret_cast<const floatx4*>(slot + TSB + 4 * q);
    const floatx4 sb = *reinterpret_cast<const floatx4*>(slot + TSB + 16 + 4 * q);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      T[g] = tb;
      Sp[g] = sb;
    }
    inv_mv_mo<G, 4>(T, slot + (NH + 4) * 256, l, a);
    inv_mv_mo<G, 4>(Sp, slot + (NH + 5) * 256, l, a);
#pragma unroll
    for (int r = 0; r < (PERM ? 3 : 4); ++r) {
      const int f = feat(r);
      const floatx4 an = *reinterpret_cast<const floatx4*>(slot + ANB + 16 * q + 4 * r);   // [1/sa ba 1/sb bb]
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float S = tanh_bf(Sp[g][r]);
        const float ybn = (zb[g][r] - T[g][r]) * exp_fast(-S);                    // cnf.py:205
        ya[g][r] = (f < Da) ? (za[g][r] - an[1]) * an[0] : 0.f;                    // ActNorm inverse (cnf.py:353-354)
        yb[g][r] = (f < Db) ? (ybn - an[3]) * an[2] : 0.f;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next record has landed in LDS
    __syncthreads();
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (b[g] < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = feat(r);
        if (f < Da) yout[b[g] * D + f] = ya[g][r];
        if (f < Db) yout[b[g] * D + Da + f] = yb[g][r];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Backward
// ------------------------------------------------------------------------------------------------
// Backward LDS tiles ([16 samples][17] each): the compute waves' delta tiles of a block, [D_1 .. D_NH, D_T, D_S, PA,
// GA, PB, GB] (2 slots), and the helper waves' activation tiles A_0 .. A_NH (A_0 = ActNorm output of the y-part,
// A_l = masked GELU output of hidden layer l; 3 slots, since they are built one block ahead of the compute waves).
template <int NH>
struct BwdJobs {
  static constexpr int ND = NH + 6, NA = NH + 1;
  static constexpr int NW = NH + 2, NS = NH + 6;
  static constexpr int SUM_OFF = NW * 256;                 // slab block: [NW][64 lanes][4] then [NS][16]
  static constexpr int BLK = NW * 256 + NS * 16;
  // W job c = dW of Linear c + 1 (c = NH, NH + 1: the last Linear's t / s row halves): delta tile c x act tile wb(c)
  __device__ static constexpr int wb(int c) { return c < NH ? c : NH; }
  // sum job c = column sum of delta tile c (biases of Linear 1 .. NH, t / s halves, then ActNorm PA, GA, PB, GB)
};

// Sum of v over the 4 rows (16-lane groups) of the wave, returned in every lane (gfx950 permlane swaps:
// the two results of each swap are the row pairs, so adding them is the pairwise sum whatever the order).
__device__ __forceinline__ float sum_rows4(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto p2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p2[0]) + __uint_as_float(p2[1]);
}

// Helper-wave gradient jobs of block m, from its delta tiles Td and activation tiles Ta, straight to slab block m
// (no LDS gradient block):
//   W job c: 16 x 16 fp32-MFMA tile over the workgroup's 16 samples, out[i][j] = sum_s delta[s][i] act[s][j]; lane l
//            holds D[4(l>>4) + r][l & 15], r = 0..3, stored as ONE float4 at [c][l] (1 KB per wave, coalesced)
//            (Linear 1: only its y-part columns; the condition part is the split-K GEMM of the tail)
//   sum job c: 16 column sums at SUM_OFF + 16 c (lanes 0..15)
// The slab layout is decoded by slab_to_canonical. The MFMA tiles are written through (sc1), like the forward's
// records: k_red_gx reads them from memory anyway.
template <int NH>
__device__ __forceinline__ void bwd_grad_jobs(const float* __restrict__ Td, const float* __restrict__ Ta,
                                              float* __restrict__ out, int hw) {
  using J = BwdJobs<NH>;
  const int l64 = threadIdx.x & 63, q = l64 >> 4, r = l64 & 15;
  constexpr int UW = (J::NW + 3) / 4, US = (J::NS + 3) / 4;
  floatx4 a[UW], bv[UW], v[US];                            // lane (q, r): samples 4 t + q of column r, t = 0..3
  const int o = 4 * tile_slot(r, q);
#pragma unroll
  for (int u = 0; u < UW; ++u) {                           // all operand reads first
    const int c = hw + 4 * u < J::NW ? hw + 4 * u : J::NW - 1;
    a[u] = *reinterpret_cast<const floatx4*>(Td + c * TILE + o);
    bv[u] = *reinterpret_cast<const floatx4*>(Ta + J::wb(c) * TILE + o);
  }
#pragma unroll
  for (int u = 0; u < US; ++u) {
    const int c = hw + 4 * u < J::NS ? hw + 4 * u : J::NS - 1;
    v[u] = *reinterpret_cast<const floatx4*>(Td + c * TILE + o);
  }
  floatx4 acc[UW];
#pragma unroll
  for (int u = 0; u < UW; ++u) acc[u] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t)                              // independent chains interleaved
#pragma unroll
    for (int u = 0; u < UW; ++u) acc[u] = mfma4(a[u][t], bv[u][t], acc[u]);
#pragma unroll
  for (int u = 0; u < US; ++u) {
    const float tot = sum_rows4((v[u][0] + v[u][1]) + (v[u][2] + v[u][3]));
    if (hw + 4 * u < J::NS && q == 0) out[J::SUM_OFF + 16 * (hw + 4 * u) + r] = tot;
  }
#pragma unroll
  for (int u = 0; u < UW; ++u)
    if (hw + 4 * u < J::NW) st4_wt_mfma(reinterpret_cast<floatx4*>(out + 256 * (hw + 4 * u)) + l64, acc[u]);
}

// Whole-stack backward, one launch, 512 threads = two roles per SIMD (waves w and w + 4 share a SIMD):
//  * compute waves 0..3 (4 samples each, row layout): back-propagate block k (VALU, DPP rotations) from its
//    backward record and its masked GELU derivatives (LDS), writing block k's delta tiles;
//  * helper waves 4..7, in the same interval: the MFMA / column-sum gradient jobs of block k+1 (tiles of the
//    previous interval) straight to the slab, and block k-1's inputs -- its activation record (loaded one interval
//    earlier) split into activation tiles and the compute waves' derivative slot, its backward record staged into
//    the LDS ring.
// One barrier per block; the compute waves issue no global loads.
constexpr int BWD_WG = 2 * BCNF_WG;
constexpr int BWD_G4 = 3;                // float4 per thread of the derivative slot: gd[NH], S, ya, yb (NH <= 9)

template <int NH>
__global__ __launch_bounds__(BWD_WG) void k_backward(BcnfLayout L, const float* __restrict__ pk,
                                                     const float* __restrict__ dz, const float* __restrict__ dldj,
                                                     const float* __restrict__ dloss, int nll, long long B,
                                                     const float* __restrict__ arec,
                                                     float* __restrict__ dy, float* __restrict__ d1,
                                                     float* __restrict__ slab_all, long long slab_stride,
                                                     const float* __restrict__ nll_part, float* __restrict__ loss_out,
                                                     uint64_t* rng_w, int32_t* guard) {
  static_assert(NH + 3 <= 4 * BWD_G4, "derivative slot");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using AR = ActRec<NH>;
  using RBk = RecB<NH>;
  using J = BwdJobs<NH>;
  const int RBL = 16 * L.RB;
  float* recB = smem;                                   // [2][16*RB]
  float* dT = recB + 2 * RING;                          // [2][ND][TILE]
  float* aT = dT + 2 * J::ND * TILE;                    // [3][NA][TILE]
  floatx4* gsl = reinterpret_cast<floatx4*>(aT + 3 * J::NA * TILE);   // [2][BWD_G4][256]
  const int nb = L.nb;
  const float* pbk = pk + L.pb_off;
  const bool helper = threadIdx.x >= BCNF_WG;
  const int t8 = (int)threadIdx.x & (BCNF_WG - 1);
  const int j = t8 & 15, s = sample_of(t8);
  const int tix = tile_ix(s, j);
  // diagnostic build: per-phase cycles of workgroup 0's wave 0 (compute) and wave 4 (helper) -> g_phase
  unsigned long long ph_t = BCNF_STAMPS ? __builtin_amdgcn_s_memtime() : 0ULL, ph_acc[4] = {0, 0, 0, 0};
#define PHS(i)                                                                                   \
  if (BCNF_STAMPS) {                                                                             \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                                  \
    ph_acc[i] += _t - ph_t;                                                                      \
    ph_t = _t;                                                                                   \
  }

  if (helper) {
    const int hw = __builtin_amdgcn_readfirstlane(t8 >> 6);
    float* slab = slab_all + (long long)blockIdx.x * slab_stride;
    // activation records [k][workgroup][AR/4][256 threads] float4 (k_forward)
    const floatx4* arl = reinterpret_cast<const floatx4*>(arec) + (long long)blockIdx.x * AR::AR4 * BCNF_WG + t8;
    const long long ars = (long long)gridDim.x * AR::AR4 * BCNF_WG;
    struct Prep {
      Stage<STAGE_REC> sr;
      floatx4 rec[AR::AR4];
      float rec1[AR::AR1 > 0 ? AR::AR1 : 1];
      float sa, ba;
    };
    const float* ar1l = arec + ar1_off(nb, gridDim.x, AR::AR4) + (long long)blockIdx.x * AR::AR1 * BCNF_WG + t8;
    const long long ar1s = (long long)gridDim.x * AR::AR1 * BCNF_WG;
    auto prep_load = [&](Prep& P, int k) {                  // block k's inputs: HBM / L2 -> registers
      P.sr.load_t(pbk + (long long)k * RBL, RBL, t8);
#pragma unroll
      for (int i = 0; i < AR::AR4; ++i) P.rec[i] = arl[(long long)k * ars + i * BCNF_WG];
#pragma unroll
      for (int i = 0; i < AR::AR1; ++i) P.rec1[i] = ar1l[(long long)k * ar1s + i * BCNF_WG];
      const float* an = pbk + (long long)k * RBL + j * L.RB + RBk::AN;
      P.sa = an[0];
      P.ba = an[1];
    };
    auto prep_store = [&](Prep& P, int k) {                 // registers -> LDS slots of block k
      // every loaded register stays live until here: a register the compiler reallocated while its load is in
      // flight would cost a wait for that load
#pragma unroll
      for (int i = 0; i < AR::AR4; ++i) asm volatile("" : "+v"(P.rec[i]));
#pragma unroll
      for (int i = 0; i < AR::AR1; ++i) asm volatile("" : "+v"(P.rec1[i]));
      asm volatile("" : "+v"(P.sa), "+v"(P.ba));
      float ar[4 * AR::AR4 + AR::AR1];
#pragma unroll
      for (int i = 0; i < AR::AR4; ++i) {
        ar[4 * i] = P.rec[i][0];
        ar[4 * i + 1] = P.rec[i][1];
        ar[4 * i + 2] = P.rec[i][2];
        ar[4 * i + 3] = P.rec[i][3];
      }
#pragma unroll
      for (int i = 0; i < AR::AR1; ++i) ar[4 * AR::AR4 + i] = P.rec1[i];
      float* ta = aT + (k % 3) * J::NA * TILE + tix;
#pragma unroll
      for (int l = 1; l <= NH; ++l) ta[l * TILE] = ar[AR::act(l - 1)];
      ta[0] = fmaf(P.sa, ar[AR::YA], P.ba);                // A_0: ActNorm output of the y-part (cnf.py:349)
      float gs[4 * BWD_G4];
#pragma unroll
      for (int l = 0; l < NH; ++l) gs[l] = ar[AR::gd(l)];
      gs[NH] = ar[AR::S];
      gs[NH + 1] = ar[AR::YA];
      gs[NH + 2] = ar[AR::YB];
#pragma unroll
      for (int i = NH + 3; i < 4 * BWD_G4; ++i) gs[i] = 0.f;
      floatx4* gd = gsl + (k & 1) * BWD_G4 * BCNF_WG + t8;
#pragma unroll
      for (int i = 0; i < BWD_G4; ++i) gd[i * BCNF_WG] = floatx4{gs[4 * i], gs[4 * i + 1], gs[4 * i + 2], gs[4 * i + 3]};
      P.sr.store_t(recB + (k & 1) * RING, t8);
    };
    // two-deep pipeline: block k-1 is rebuilt from registers loaded one interval earlier, while block k-2's
    // loads are in flight (an HBM round trip under load is longer than one interval)
    // (the two register sets alternate by hand-unrolling: a copy of in-flight loads would wait for them)
    Prep Pa, Pb;
    prep_load(Pa, nb - 1);
    prep_load(Pb, nb >= 2 ? nb - 2 : 0);
    prep_store(Pa, nb - 1);
    __syncthreads();
    auto step = [&](int k, Prep& Pc, Prep& Pnext) {  // interval k: Pc holds block k-1's loads
      PHS(0)
      prep_load(Pnext, k >= 2 ? k - 2 : 0);             // unconditional (clamped): no branch around loads in flight
      PHS(1)
      if (k + 1 < nb)
        bwd_grad_jobs<NH>(dT + ((k + 1) & 1) * J::ND * TILE, aT + ((k + 1) % 3) * J::NA * TILE,
                          slab + (long long)(k + 1) * J::BLK, hw);
      PHS(2)
      if (k >= 1) prep_store(Pc, k - 1);
      PHS(3)
      __syncthreads();
    };
    for (int k = nb - 1; k >= 0; k -= 2) {
      step(k, Pb, Pa);
      if (k == 0) break;
      step(k - 1, Pa, Pb);
    }
    bwd_grad_jobs<NH>(dT, aT, slab, hw);                     // block 0 (tiles of the last interval)
  } else {
    const int tid = t8;
#ifdef BCNF_BWD_PRIO
    __builtin_amdgcn_s_setprio(BCNF_BWD_PRIO);
#endif
    const long long b = (long long)blockIdx.x * 16 + s;
    const bool valid = b < B;
    const long long bc = valid ? b : B - 1;
    const int D = L.D, Da = L.Da, Db = L.Db;
    float* d1l = d1 + bc * 16 + j;                    // D1[k][b][j]  = d1l[k * B * 16]
    float* d1_dummy = d1 + (long long)nb * B * 16 + j; // rows past the batch (workspace slack)
    const long long hps = B * 16;

    float gya = 0.f, gyb = 0.f, dl = 0.f;
    if (valid) {                                      // padded rows carry zero gradient
      if (nll) {    // d/dz, d/dldj of mean_b(0.5 |z_b|^2 - ldj_b); dz holds z here
        const float sc = (dloss ? dloss[0] + dloss[1] : 1.f) / (float)B;   // d loss/d nll = d nll/d nll = 1
        gya = (j < Da) ? dz[b * D + j] * sc : 0.f;
        gyb = (j < Db) ? dz[b * D + Da + j] * sc : 0.f;
        dl = -sc;
      } else {
        if (dz) {
          gya = (j < Da) ? dz[b * D + j] : 0.f;
          gyb = (j < Db) ? dz[b * D + Da + j] : 0.f;
        }
        if (dldj) dl = dldj[b];
      }
    }
    __syncthreads();
    PHS(0)
    for (int k = nb - 1; k >= 0; --k) {
      const int cur = k & 1;
      float gs[4 * BWD_G4];
      {
        const floatx4* gd4 = gsl + cur * BWD_G4 * BCNF_WG + tid;
#pragma unroll
        for (int i = 0; i < BWD_G4; ++i) {
          const floatx4 v = gd4[i * BCNF_WG];
          gs[4 * i] = v[0];
          gs[4 * i + 1] = v[1];
          gs[4 * i + 2] = v[2];
          gs[4 * i + 3] = v[3];
        }
      }
      float* Tt = dT + cur * J::ND * TILE + tix;
      // the record streams in consumption order (RecB): ActNorm + Q^T + the heads now, then each stage issues the
      // reads of a later one behind a scheduling barrier, so every wait covers a few reads, not the whole record
      // (lgkmcnt counts at most 15 outstanding: a block-wide burst of 53 reads made the mix wait for ~40 of them)
      const float* R = recB + cur * RING + j * L.RB;
      float rb[RBk::USED];
      ld_rec<0, RBk::HID>(rb, R);                        // ActNorm, Q^T, T / S heads
      __builtin_amdgcn_sched_barrier(0);
      const float* gd = gs;
      const float S = gs[NH], ya = gs[NH + 1], yb = gs[NH + 2];
      const float an_sa = rb[RBk::AN], an_sb = rb[RBk::AN + 2], an_bb = rb[RBk::AN + 3];
      const float xb = fmaf(an_sb, yb, an_bb);
      const float e = exp_fast(S);
      float gza, gzb;
      if (QBC_DEV(L, QBC_MIX)) mix_bc(rb + RBk::QT, gya, gyb, gza, gzb);   // g @ Q^T (identity for the last block)
      else mix(rb + RBk::QT, gya, gyb, gza, gzb);
      ld16(rb + RBk::HID, R + RBk::HID);                 // hidden layer NH
      __builtin_amdgcn_sched_barrier(0);
      const float dT_ = gzb;                             // z_b = exp(s) y_b + t
      const float dS = (j < Db) ? fmaf(gzb * e, xb, dl) : 0.f;
      const float dSp = dS * (1.f - S * S);
      const float dxb = gzb * e;
      Tt[NH * TILE] = dT_;
      Tt[(NH + 1) * TILE] = dSp;
      float da = 0.f, da2 = 0.f;
      if (QBC_DEV(L, QBC_HEAD)) bc9x2(dT_, rb + RBk::TT, da, dSp, rb + RBk::ST, da2);   // (uniform)
      else rot16x2(dT_, rb + RBk::TT, da, dSp, rb + RBk::ST, da2);
      da += da2;
#pragma unroll
      for (int l = NH; l >= 2; --l) {
        ld16(rb + RBk::HID + 16 * (NH - l + 1), R + RBk::HID + 16 * (NH - l + 1));   // next layer (last: W1^T)
        __builtin_amdgcn_sched_barrier(0);
        const float dpre = da * gd[l - 1];
        Tt[(l - 1) * TILE] = dpre;
        da = rot16(dpre, rb + RBk::HID + 16 * (NH - l), 0.f);
      }
      const float dpre1 = da * gd[0];
      Tt[0] = dpre1;
      *(valid ? d1l + k * hps : d1_dummy) = dpre1;      // dL/d pre-activation of Linear 1 (split-K, dh)
      const float dxa = rot16(dpre1, rb + RBk::W1T, gza);
      {   // ActNorm tiles (consumed only for blocks that have an ActNorm)
        const float inv_a = (j < Da) ? __builtin_amdgcn_rcpf(an_sa) : 0.f;
        const float inv_b = (j < Db) ? __builtin_amdgcn_rcpf(an_sb) : 0.f;
        Tt[(NH + 2) * TILE] = fmaf(dxa, ya, dl * inv_a);
        Tt[(NH + 3) * TILE] = dxa;
        Tt[(NH + 4) * TILE] = fmaf(dxb, yb, dl * inv_b);
        Tt[(NH + 5) * TILE] = dxb;
      }
      gya = an_sa * dxa;
      gyb = an_sb * dxb;
      PHS(1)
      __syncthreads();
      PHS(2)
    }
    if (dy && valid) {
      if (j < Da) dy[b * D + j] = gya;
      if (j < Db) dy[b * D + Da + j] = gyb;
    }
  }
#if BCNF_STAMPS
  if (blockIdx.x == 0 && (threadIdx.x == 0 || threadIdx.x == BCNF_WG))
    for (int i = 0; i < 4; ++i) g_phase[(helper ? 4 : 0) + i] = ph_acc[i];
#endif
#undef PHS
  if (loss_out && blockIdx.x == 0) {                 // deferred NLL reduction of the forward
    __syncthreads();                                  // (the helpers' last jobs have read the tiles)
    nll_finalize<BWD_WG>(nll_part, (int)gridDim.x, B, loss_out, rng_w, guard, dT);
  }
}

// Deterministic sum of the per-workgroup gradient slabs (fixed order over workgroups). Slab block m (slab_blk_floats
// floats at m * L.sblk) is what the backward's helper waves wrote (BwdJobs): NH + 2 MFMA tiles in lane order, then
// NH + 6 column sums; this maps each element back to its canonical position, or -1 for tile padding (rows / columns
// past a Linear's shape, ActNorm sums of the last block). W1's condition columns come from the split-K GEMM.
// a[i] for a per-lane i through constant indices (scalar argument loads and selects): indexed directly, every such
// read was a per-lane load of the kernel arguments in front of the reduce's first dependent load
template <int N>
__device__ __forceinline__ int lpick(const int (&a)[N], int i) {
  int r = a[0];
#pragma unroll
  for (int t = 1; t < N; ++t) r = (i == t) ? a[t] : r;
  return r;
}

__device__ __forceinline__ long long slab_to_canonical(const BcnfLayout& L, int m, int o) {
  const int NH = L.NH, NW = NH + 2;
  const int cb = m * L.blk_stride + ((m < L.nb - 1) ? L.an_size : 0);      // coupling base
  if (o < NW * 256) {
    const int c = o >> 8, e = o & 255, lane = e >> 2;
    const int row = 4 * (lane >> 4) + (e & 3), col = lane & 15;
    const int l = c < NH ? c + 1 : NH + 1;
    const int nrows = c < NH ? lpick(L.H, l) : L.Db, ncols = (l == 1) ? L.Da : lpick(L.H, l - 1);
    if (row >= nrows || col >= ncols) return -1;
    const int row0 = (c == NH + 1) ? L.Db : 0;
    return (long long)cb + lpick(L.lin_w, l) + (row0 + row) * lpick(L.lin_in, l) + col;
  }
  const int o2 = o - NW * 256, c = o2 >> 4, r = o2 & 15;
  if (c < NH) return r < lpick(L.H, c + 1) ? (long long)cb + lpick(L.lin_b, c + 1) + r : -1;
  if (c < NH + 2) return r < L.Db ? (long long)cb + lpick(L.lin_b, NH + 1) + ((c == NH + 1) ? L.Db : 0) + r : -1;
  const int a = c - NH - 2;
  if (a >= 4 || !L.act_norm || m >= L.nb - 1 || r >= ((a < 2) ? L.Da : L.Db)) return -1;
  return (long long)m * L.blk_stride + ((a & 1) ? L.D : 0) + ((a < 2) ? 0 : L.Da) + r;
}

// RED_O4 output float4 per workgroup x RED_G slab groups (group g sums workgroups g, g+RED_G, ...; RED_T loads
// in flight per lane), combined in a fixed order through LDS. The slab stream is latency-bound on bytes in
// flight: 32 lanes x 16 B x 16 loads per group keeps ~35 MB in flight over the ~580-workgroup grid at B=4096.
constexpr int RED_G = 8, RED_O4 = 32, RED_T = 16;

// With `A` (folded training step inside a multi-step graph, FoldAdamArgs): the reduced gradient of each output also
// takes its Adam update here; the parameters / moments are fetched before the slab stream, the scalars are `as`.
__device__ __forceinline__ void reduce_body(const BcnfLayout& L, const float* __restrict__ slab, long long stride,
                                            int nwg, float* __restrict__ out, int bx, float* __restrict__ smem,
                                            const FoldAdamArgs* A = nullptr, const AdamScalars* as = nullptr) {
  floatx4 (*part)[RED_O4] = reinterpret_cast<floatx4 (*)[RED_O4]>(smem);   // [RED_G][RED_O4]
  const int g = threadIdx.x / RED_O4, o4 = threadIdx.x % RED_O4;
  const long long i = ((long long)bx * RED_O4 + o4) * 4;
  const bool live = i < stride;
  const long long ic = live ? i : 0;
  const int m = (int)(ic / L.sblk), o = (int)(ic - (long long)m * L.sblk);
  long long ci[4];
  float ap[4], am[4], av[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ci[e] = slab_to_canonical(L, m, o + e);
    if (A && g == 0) {
      const long long c = ci[e] >= 0 ? ci[e] : 0;
      ap[e] = A->p[0][c];
      am[e] = A->m[0][c];
      av[e] = A->v[0][c];
    }
  }
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  int w = g;
  for (; w + RED_G * (RED_T - 1) < nwg; w += RED_G * RED_T) {
    floatx4 v[RED_T];
#pragma unroll
    for (int t = 0; t < RED_T; ++t)
      v[t] = *reinterpret_cast<const floatx4*>(slab + (long long)(w + RED_G * t) * stride + ic);
#pragma unroll
    for (int t = 0; t < RED_T; ++t) acc += v[t];
  }
  for (; w < nwg; w += RED_G) acc += *reinterpret_cast<const floatx4*>(slab + (long long)w * stride + ic);
  part[g][o4] = acc;
  __syncthreads();
  if (g != 0 || !live) return;
  floatx4 tot = part[0][o4];
#pragma unroll
  for (int q = 1; q < RED_G; ++q) tot += part[q][o4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (ci[e] < 0) continue;
    out[ci[e]] = tot[e];
    if (A) {
      adam_elem(ap[e], tot[e], am[e], av[e], *as);
      A->p[0][ci[e]] = ap[e];
      A->m[0][ci[e]] = am[e];
      A->v[0][ci[e]] = av[e];
    }
  }
}

// The backward's tail in ONE launch: dL/dh tiles, the slab reduction and the W1 condition-part split-K
// partials are independent, so their workgroups share a grid (role by block index) and run
// concurrently instead of paying three launch floors back to back.
struct TailGrid {
  int n_dh, gx_dh;      // dh tiles: (gx_dh x Cp/16), 0 if dh is not requested
  int n_red;            // slab-reduce workgroups
  int gx_dw;            // dW1h: (gx_dw x splits)
  int ones;             // folded path: the split-K runs on x1 = [x | 1] (ones column index), else -1
};

// Lw: the split-K role's layout (L itself, or fold_layout(L, X) with h = x on the folded path).
template <bool VEC>
__global__ __launch_bounds__(BCNF_WG) void k_bwd_tail(BcnfLayout L, BcnfLayout Lw, TailGrid G, const float* __restrict__ pk,
                                                      const float* __restrict__ d1, const float* __restrict__ h,
                                                      long long B, float* __restrict__ dh,
                                                      const float* __restrict__ slab, long long stride, int nwg,
                                                      float* __restrict__ dparams, int rows_per_split,
                                                      float* __restrict__ work) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int i = blockIdx.x;
  if (i < G.n_dh) {
    dh_body(L, pk, d1, B, dh, i % G.gx_dh, i / G.gx_dh, smem);
    return;
  }
  i -= G.n_dh;
  if (i < G.n_red) {
    reduce_body(L, slab, stride, nwg, dparams, i, smem);
    return;
  }
  i -= G.n_red;
  dw1h_body<VEC>(Lw, d1, h, B, rows_per_split, work, i % G.gx_dw, i / G.gx_dw, smem, G.ones);
}

// Folded path, second launch of the backward tail: the Gx reduce (latency-bound, 6 MB) placed first, then the
// slab reduce (HBM-bound, 75 MB at B = 4096), so the former hides under the latter; the split-K that produces
// the Gx partials ran alone in the launch before (the two roles in one launch did not overlap: 28 us vs 13 + 10).
__global__ __launch_bounds__(BCNF_WG) void k_red_gx(BcnfLayout L, long long total, const float* __restrict__ work,
                                                    int splits, float* __restrict__ gx, int n_gx,
                                                    const float* __restrict__ slab, long long stride, int nwg,
                                                    float* __restrict__ dparams, FoldAdamArgs A) {
  __shared__ __attribute__((aligned(16))) float smem[RED_G * RED_O4 * 4];
  const int bx = blockIdx.x;
  if (bx < n_gx) {
    gx_reduce_body(total, work, splits, gx, (long long)bx * BCNF_WG + threadIdx.x);
    return;
  }
  if (A.on && !(A.guard && A.guard[BCNF_GUARD_HALTED])) {      // (a halted step updates nothing)
    const AdamScalars as = adam_scalars_of(A, A.asc[0], A.asc[1]);   // (k_fold_splitk published them)
    reduce_body(L, slab, stride, nwg, dparams, bx - n_gx, smem, &A, &as);
    return;
  }
  reduce_body(L, slab, stride, nwg, dparams, bx - n_gx, smem);
}

// Test hook: the whole dynamic LDS of the workgroup set to `value` (bcnf_lds_fill).
__global__ __launch_bounds__(BCNF_WG) void k_fill_lds(float value) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  for (int i = threadIdx.x; i < (int)(LDS_MAX / 16); i += BCNF_WG)
    reinterpret_cast<floatx4*>(smem)[i] = floatx4{value, value, value, value};
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// Launch helpers
// ------------------------------------------------------------------------------------------------
int check_launch() { return bcnf_rt::launched(); }



// Raise a kernel's dynamic-LDS limit once (cached per kernel; safe to call under stream capture
// after the first eager call has set it).
std::mutex g_attr_mu;
const void* g_attr_fn[256];
size_t g_attr_lds[256];
int g_attr_n = 0;

template <typename K>
int launch_lds(K kernel, size_t& lds) {
  if (lds > LDS_MAX) return BCNF_ERR_UNSUPPORTED;
  const void* fn = reinterpret_cast<const void*>(kernel);
  std::lock_guard<std::mutex> lk(g_attr_mu);
  for (int i = 0; i < g_attr_n; ++i)
    if (g_attr_fn[i] == fn && g_attr_lds[i] >= lds) return BCNF_OK;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return bcnf_rt::hip_status(e);
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
bool layout_matches(const BcnfLayout& L) {
  return L.rf_b1 == RecF<NH>::B1 && L.rf_w1 == RecF<NH>::W1 && L.rf_hid == RecF<NH>::HID && L.rf_t == RecF<NH>::T &&
         L.rf_s == RecF<NH>::S && L.rf_q == RecF<NH>::Q && L.RF >= RecF<NH>::USED && L.rb_w1t == RecB<NH>::W1T &&
         L.rb_hid == RecB<NH>::HID && L.rb_tt == RecB<NH>::TT && L.rb_st == RecB<NH>::ST && L.rb_qt == RecB<NH>::QT &&
         L.rb_an == RecB<NH>::AN && L.RB >= RecB<NH>::USED;
}

struct NllOut {
  float* part = nullptr;
};

// float4 row loads: the row stride and the base are 16-byte aligned (columns >= C of a loaded float4 are
// discarded by select, so a padded row's tail may hold anything).
bool vec_rows(const BcnfLayout& L, const float* h) { return L.ldh % 4 == 0 && ((uintptr_t)h & 15) == 0; }

int launch_hp(const BcnfLayout& L, const float* pk, const float* h, long long R, float* hp, hipStream_t st) {
  size_t lds = hp_lds_bytes();
  const dim3 grid((unsigned)((R + 63) / 64), (unsigned)(L.NKp / 64));
  int rc;
  if (vec_rows(L, h)) {
    if ((rc = launch_lds(k_hp<true>, lds))) return rc;
    hipLaunchKernelGGL(k_hp<true>, grid, dim3(BCNF_WG), lds, st, L, pk, h, R, hp);
  } else {
    if ((rc = launch_lds(k_hp<false>, lds))) return rc;
    hipLaunchKernelGGL(k_hp<false>, grid, dim3(BCNF_WG), lds, st, L, pk, h, R, hp);
  }
  return check_launch();
}

template <int NH>
int fwd_dispatch(const BcnfLayout& L, const float* pk, const float* y, const ProjArgs& P, long long B, float* z,
                 float* ldj, float* logp, bool drop, const uint64_t* rng, float* arec, const NllOut& no,
                 hipStream_t st, const RawArgs* raw = nullptr) {
  if (!layout_matches<NH>(L)) return BCNF_ERR_ARG;
  if (P.Cp % 16 != 0 || P.Cp / 16 > HP_SMAX || P.C > P.Cp) return BCNF_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)((B + 15) / 16));
  size_t lds = fwd2_lds_bytes(L, raw != nullptr);
  const bool save = arec != nullptr;
  const RawArgs R = raw ? *raw : RawArgs{};
  int rc;
#define BCNF_FWD(DR, SV, RW)                                                                                   \
  rc = launch_lds(k_forward<NH, DR, SV, RW>, lds);                                                             \
  if (rc) return rc;                                                                                           \
  hipLaunchKernelGGL((k_forward<NH, DR, SV, RW>), grid, dim3(2 * BCNF_WG), lds, st, L, pk, y, P, B, z, ldj, logp, \
                     rng, arec, no.part, R);
  if (raw) {
    if (!save) return BCNF_ERR_ARG;
    if (drop) { BCNF_FWD(true, true, true) } else { BCNF_FWD(false, true, true) }
  } else if (drop) {
    if (save) { BCNF_FWD(true, true, false) } else { BCNF_FWD(true, false, false) }
  } else {
    if (save) { BCNF_FWD(false, true, false) } else { BCNF_FWD(false, false, false) }
  }
#undef BCNF_FWD
  return check_launch();
}

template <int NH>
int inv_dispatch(const BcnfLayout& L, const float* pk, const float* zin, const float* hp, long long R,
                 const int64_t* ci, long long N, float* y, bool drop, const uint64_t* rng, hipStream_t st) {
  if (!layout_matches<NH>(L)) return BCNF_ERR_ARG;
  int rc;
  if (!drop && L.RF == inv_m_rf<NH>() && L.PMB == (NH + 6) * 256 + (NH - 1) * 16 + 96) {   // eval: matrix cores
    size_t lds_m = sizeof(float) * (size_t)(2 * RING);
    const dim3 grid_m((unsigned)((N + INV_M_SPB - 1) / INV_M_SPB));
    if (L.Da <= 12 && L.Db <= 12) {
      if ((rc = launch_lds(k_inverse_mfma<NH, true>, lds_m))) return rc;
      hipLaunchKernelGGL((k_inverse_mfma<NH, true>), grid_m, dim3(INV_M_WG), lds_m, st, L, pk, zin, hp, R, ci, N, y);
    } else {
      if ((rc = launch_lds(k_inverse_mfma<NH, false>, lds_m))) return rc;
      hipLaunchKernelGGL((k_inverse_mfma<NH, false>), grid_m, dim3(INV_M_WG), lds_m, st, L, pk, zin, hp, R, ci, N, y);
    }
    return check_launch();
  }
  const dim3 grid((unsigned)((N + 15) / 16));
  size_t lds = fwd_lds_bytes(L);
  if (drop) {
    rc = launch_lds(k_inverse<NH, true>, lds);
    if (rc) return rc;
    hipLaunchKernelGGL((k_inverse<NH, true>), grid, dim3(BCNF_WG), lds, st, L, pk, zin, hp, R, ci, N, y, rng);
  } else {
    rc = launch_lds(k_inverse<NH, false>, lds);
    if (rc) return rc;
    hipLaunchKernelGGL((k_inverse<NH, false>), grid, dim3(BCNF_WG), lds, st, L, pk, zin, hp, R, ci, N, y, rng);
  }
  return check_launch();
}

long long slab_stride_of(const BcnfLayout& L) { return (long long)L.nb * L.sblk; }

template <int NH>
int bwd_dispatch(const BcnfLayout& L, const float* pk, const float* dz, const float* dldj, const float* dloss,
                 int nll, long long B, const float* arec, float* dy, float* d1, float* slab, long long stride,
                 const float* part, float* loss_out, uint64_t* rng_w, int32_t* guard, hipStream_t st) {
  if (!layout_matches<NH>(L)) return BCNF_ERR_ARG;
  const dim3 grid((unsigned)((B + 15) / 16));
  size_t lds = bwd_lds_bytes(L);
  const int rc = launch_lds(k_backward<NH>, lds);
  if (rc) return rc;
  hipLaunchKernelGGL((k_backward<NH>), grid, dim3(BWD_WG), lds, st, L, pk, dz, dldj, dloss, nll, B, arec, dy,
                     d1, slab, stride, part, loss_out, rng_w, guard);
  return check_launch();
}

// split-K geometry of the W1 condition-part gradient
int w1h_rows_per_split(long long) { return KC; }   // one LDS chunk of rows per split
long long w1h_splits(long long B) { return (B + w1h_rows_per_split(B) - 1) / w1h_rows_per_split(B); }
long long w1h_work_floats(const BcnfLayout& L, long long B) { return w1h_splits(B) * L.nb * 16LL * L.Cp; }

// Workspace (floats): [activation records nb*B*16*AR][loss partials][HP nb*B*16][D1 nb*B*16]
// (`drop` no longer changes the layout: the records hold the masked activations)
long long ws_part_off(const BcnfLayout& L, long long B, bool) {
  return (long long)L.nb * ((B + 15) / 16) * BCNF_WG * act_rec_floats(L.NH);   // padded rows own slots
}
long long ws_hp_off(const BcnfLayout& L, long long B, bool drop) {
  return ws_part_off(L, B, drop) + (((B + 15) / 16 + 3) & ~3LL);
}
long long ws_d1_off(const BcnfLayout& L, long long B, bool drop) { return ws_hp_off(L, B, drop) + (long long)L.nb * B * 16; }
long long ws_floats(const BcnfLayout& L, long long B, bool drop) {
  return ws_d1_off(L, B, drop) + (long long)L.nb * B * 16 + 16;   // + D1 dummy row
}

int forward_impl(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h, int64_t batch,
                 float* z, float* ldj, float* log_prob, int32_t training, const uint64_t* rng_state, void* workspace,
                 bool save, bool nll, bool finalize, float* loss_out, int32_t* guard, void* stream,
                 const float* fold = nullptr, int X = 0, int ldx = 0, const RawArgs* raw = nullptr) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (batch < 0) return BCNF_ERR_ARG;
  if (batch == 0) return nll ? BCNF_ERR_ARG : BCNF_OK;      // the mean over an empty batch is undefined
  if (!packed || !y || !h || !z || !workspace) return BCNF_ERR_ARG;
  if (nll && finalize && !loss_out) return BCNF_ERR_ARG;
  const bool drop = training && L.p > 0.f;
  if (drop && !rng_state) return BCNF_ERR_ARG;
  float* ws = (float*)workspace;
  float* arec = (save || nll) ? ws : nullptr;
  NllOut no;
  if (nll) no.part = ws + ws_part_off(L, batch, drop);
  const float* pk = (const float*)packed;
  hipStream_t st = (hipStream_t)stream;
  // the condition projection runs inside k_forward: h, or x with the folded feature Linear (fold_layout: Wc / bc
  // instead of W1h^T / b1)
  const BcnfLayout Lp = fold ? fold_layout(L, X, ldx) : L;
  const float* pbase = fold ? fold : pk;
  const ProjArgs P{h, pbase + Lp.w1c_off, pbase + Lp.b1c_off, (long long)Lp.ldh, Lp.C, Lp.Cp, Lp.NKp};
  switch (L.NH) {
#define BCNF_CASE(N) case N: rc = fwd_dispatch<N>(L, pk, y, P, batch, z, ldj, log_prob, drop, rng_state, arec, no, st, raw); break;
    BCNF_CASE(1) BCNF_CASE(2) BCNF_CASE(3) BCNF_CASE(4) BCNF_CASE(5) BCNF_CASE(6) BCNF_CASE(7) BCNF_CASE(8)
#undef BCNF_CASE
    default: return BCNF_ERR_UNSUPPORTED;
  }
  if (rc || !nll || !finalize) return rc;
  hipLaunchKernelGGL(k_nll_finalize, dim3(1), dim3(BCNF_WG), 0, st, (const float*)no.part, (int)((batch + 15) / 16),
                     (long long)batch, loss_out, drop ? const_cast<uint64_t*>(rng_state) : nullptr, guard);
  return check_launch();
}

int backward_impl(const BcnfStackDesc* desc, const void* packed, const float* h, const float* dz, const float* dldj,
                  const float* dloss, int nll, int64_t batch, int32_t training, void* workspace, float* dy,
                  float* dh, float* dparams, void* slab, float* loss_out, uint64_t* rng_state, int32_t* guard,
                  void* stream);

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
  *bytes = ws_floats(L, batch, training && L.p > 0.f) * 4;
  return BCNF_OK;
}

int bcnf_slab_bytes(const BcnfStackDesc* desc, int64_t batch, int64_t* bytes) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!bytes || batch < 0) return BCNF_ERR_ARG;
  *bytes = ((int64_t)((batch + 15) / 16) * slab_stride_of(L) + w1h_work_floats(L, batch)) * 4;
  return BCNF_OK;
}

int bcnf_inverse_scratch_bytes(const BcnfStackDesc* desc, int64_t h_rows, int64_t* bytes) {
  BcnfLayout L;
  const int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!bytes || h_rows < 0) return BCNF_ERR_ARG;
  *bytes = (int64_t)L.nb * h_rows * 16 * 4;
  return BCNF_OK;
}

int bcnf_pack_params(const BcnfStackDesc* desc, const float* params, const float* qmats, void* packed, void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (!params || !packed || (L.nb > 1 && !qmats)) return BCNF_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int npw = pack_wgs(L);
  hipLaunchKernelGGL(k_pack, dim3(npw + 1), dim3(BCNF_WG), 0, st, L, params, qmats, (float*)packed, npw);
  return check_launch();
}

int bcnf_stack_forward(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h, int64_t batch,
                       float* z, float* ldj, float* log_prob, int32_t training, const uint64_t* rng_state,
                       void* workspace, int32_t save, void* stream) {
  return forward_impl(desc, packed, y, h, batch, z, ldj, log_prob, training, rng_state, workspace, save != 0, false,
                      false, nullptr, nullptr, stream);
}

int bcnf_nll_forward(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h, int64_t batch,
                     float* z, float* ldj, int32_t training, uint64_t* rng_state, void* workspace, int32_t finalize,
                     float* loss_out, int32_t* guard, void* stream) {
  return forward_impl(desc, packed, y, h, batch, z, ldj, nullptr, training, rng_state, workspace, true, true,
                      finalize != 0, loss_out, guard, stream);
}

int bcnf_stack_backward(const BcnfStackDesc* desc, const void* packed, const float* h, const float* dz,
                        const float* dldj, int64_t batch, int32_t training, void* workspace, float* dy,
                        float* dh, float* dparams, void* slab, void* stream) {
  return backward_impl(desc, packed, h, dz, dldj, nullptr, 0, batch, training, workspace, dy, dh, dparams, slab,
                       nullptr, nullptr, nullptr, stream);
}

int bcnf_nll_backward(const BcnfStackDesc* desc, const void* packed, const float* h, const float* z,
                      const float* dloss, int64_t batch, int32_t training, void* workspace, float* dy,
                      float* dh, float* dparams, void* slab, float* loss_out, uint64_t* rng_state, int32_t* guard,
                      void* stream) {
  if (!z && batch > 0) return BCNF_ERR_ARG;
  return backward_impl(desc, packed, h, z, nullptr, dloss, 1, batch, training, workspace, dy, dh, dparams, slab,
                       loss_out, rng_state, guard, stream);
}

int bcnf_backward_tail(const BcnfStackDesc* desc, const void* packed, const void* slab, const float* h,
                       const void* workspace, int64_t batch, int32_t training, float* dh, float* dparams,
                       void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (!packed || !slab || !h || !workspace || !dparams || batch < 1) return BCNF_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const long long S = slab_stride_of(L);
  const int nwg = (int)((batch + 15) / 16);
  const bool drop = training && L.p > 0.f;
  const float* d1 = (const float*)workspace + ws_d1_off(L, batch, drop);
  float* work = (float*)slab + (long long)nwg * S;
  const int rps = w1h_rows_per_split(batch);
  const long long splits = w1h_splits(batch);
  TailGrid G;
  G.gx_dh = (int)((batch + 63) / 64);
  G.n_dh = dh ? G.gx_dh * (L.Cp >> 4) : 0;
  G.n_red = (int)((S / 4 + RED_O4 - 1) / RED_O4);
  G.gx_dw = (L.nb + 3) / 4;
  G.ones = -1;
  const long long n_dw = (long long)G.gx_dw * splits;
  size_t lds = dw1h_lds_bytes(L);
  if (dh_lds_bytes() > lds) lds = dh_lds_bytes();
  const dim3 grid((unsigned)(G.n_dh + G.n_red + n_dw));
  if (vec_rows(L, h)) {
    if ((rc = launch_lds(k_bwd_tail<true>, lds))) return rc;
    hipLaunchKernelGGL(k_bwd_tail<true>, grid, dim3(BCNF_WG), lds, st, L, L, G, (const float*)packed, d1, h,
                       (long long)batch, dh, (const float*)slab, S, nwg, dparams, rps, work);
  } else {
    if ((rc = launch_lds(k_bwd_tail<false>, lds))) return rc;
    hipLaunchKernelGGL(k_bwd_tail<false>, grid, dim3(BCNF_WG), lds, st, L, L, G, (const float*)packed, d1, h,
                       (long long)batch, dh, (const float*)slab, S, nwg, dparams, rps, work);
  }
  if ((rc = check_launch())) return rc;
  const long long outs = (long long)L.nb * 16 * L.Cp;
  hipLaunchKernelGGL(k_dw1h_reduce, dim3((unsigned)((outs + BCNF_WG - 1) / BCNF_WG)), dim3(BCNF_WG), 0, st, L,
                     (const float*)work, (int)splits, dparams);
  return check_launch();
}

// ---- folded linear feature network (see fold_body) ----
namespace {
int fold_setup(const BcnfStackDesc* desc, int32_t X, BcnfLayout* L) {
  int rc = make_layout(desc, L);
  if (rc) return rc;
  if (!layout_supported(*L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (X < 1 || fold_xp(X) > 16 * NC16_MAX) return BCNF_ERR_UNSUPPORTED;
  if (dw1h_lds_bytes(fold_layout(*L, X, X)) > LDS_MAX) return BCNF_ERR_UNSUPPORTED;
  return BCNF_OK;
}
long long fold_floats(const BcnfLayout& L, int X) { return (long long)(fold_xp(X) + 1) * L.NKp; }
// The pack-free forward's shape limits (its table must also build: build_raw_table).
bool raw_applicable(const BcnfLayout& L, int X) {
  return X <= RAW_KP - 4 && L.C <= 64 * RAW_TPW && L.nb >= 2 && L.act_norm;
}
}  // namespace

int bcnf_fold_bytes(const BcnfStackDesc* desc, int32_t in_features, int64_t* bytes) {
  BcnfLayout L;
  const int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!bytes) return BCNF_ERR_ARG;
  *bytes = fold_floats(L, in_features) * 4;
  return BCNF_OK;
}

int bcnf_fold_slab_bytes(const BcnfStackDesc* desc, int32_t in_features, int64_t batch, int64_t* bytes) {
  BcnfLayout L;
  const int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!bytes || batch < 0) return BCNF_ERR_ARG;
  const BcnfLayout F = fold_layout(L, in_features, in_features);
  *bytes = ((int64_t)((batch + 15) / 16) * slab_stride_of(L) + w1h_work_floats(F, batch) +
            (int64_t)L.nb * 16 * F.Cp + 4) * 4;                // + the fused Adam's two scalars (FoldAdamArgs::asc)
  return BCNF_OK;
}

int bcnf_pack_params_fold(const BcnfStackDesc* desc, const float* params, const float* qmats,
                          const float* feat_weight, const float* feat_bias, int32_t in_features, void* packed,
                          float* fold, const BcnfGather2* gather, void* stream) {
  BcnfLayout L;
  int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!params || !packed || !fold || !feat_weight || (L.nb > 1 && !qmats)) return BCNF_ERR_ARG;
  BcnfGatherArgs ga = {};
  if (gather) {
    const BcnfGather2& g = *gather;
    if (g.n < 1 || g.cols0 < 1 || g.cols1 < 1 || !g.idx || !g.src0 || !g.dst0 || !g.src1 || !g.dst1)
      return BCNF_ERR_ARG;
    if (g.n * (int64_t)(g.cols0 + g.cols1) >= (1LL << 31)) return BCNF_ERR_UNSUPPORTED;
    ga = BcnfGatherArgs{g.idx, (const long long*)g.cursor, g.src0, g.dst0, g.src1, g.dst1, (int)g.n, 0, g.cols0,
                        g.cols1, 0};
    gather2_plan(g.n, &ga.rpw, &ga.nwg);
  }
  const int npw = pack_wgs(L, true);
  const unsigned grid = (unsigned)(L.NKp / 16 * FOLD_SPLIT + ga.nwg + npw + 1);
  hipLaunchKernelGGL(k_pack_fold, dim3(grid), dim3(BCNF_WG), 0, (hipStream_t)stream, L, params, qmats, (float*)packed,
                     feat_weight, feat_bias, (int)in_features, fold, ga, npw);
  return check_launch();
}

int bcnf_fold_nll_forward(const BcnfStackDesc* desc, const void* packed, const float* fold, int32_t in_features,
                          const float* y, const float* x, int32_t ldx, int64_t batch, float* z, float* ldj, int32_t training,
                          uint64_t* rng_state, void* workspace, int32_t finalize, float* loss_out, int32_t* guard,
                          void* stream) {
  BcnfLayout L;
  const int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!fold || ldx < in_features) return BCNF_ERR_ARG;
  return forward_impl(desc, packed, y, x, batch, z, ldj, nullptr, training, rng_state, workspace, true, true,
                      finalize != 0, loss_out, guard, stream, fold, in_features, ldx);
}

int bcnf_lds_fill(float value, void* stream) {
  size_t lds = LDS_MAX;
  const int rc = launch_lds(k_fill_lds, lds);
  if (rc) return rc;
  hipLaunchKernelGGL(k_fill_lds, dim3(4 * 256), dim3(BCNF_WG), LDS_MAX, (hipStream_t)stream, value);
  return check_launch();
}

int bcnf_fold_raw_table_bytes(const BcnfStackDesc* desc, int32_t in_features, int64_t* bytes) {
  BcnfLayout L;
  const int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!bytes) return BCNF_ERR_ARG;
  if (!raw_applicable(L, in_features)) return BCNF_ERR_UNSUPPORTED;
  std::vector<uint32_t> t((size_t)raw_table_words(L));
  if (!build_raw_table(L, t.data())) return BCNF_ERR_UNSUPPORTED;
  *bytes = (int64_t)t.size() * (int64_t)sizeof(uint32_t);
  return BCNF_OK;
}

int bcnf_fold_raw_table(const BcnfStackDesc* desc, int32_t in_features, void* host_table) {
  BcnfLayout L;
  const int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!host_table) return BCNF_ERR_ARG;
  if (!raw_applicable(L, in_features)) return BCNF_ERR_UNSUPPORTED;
  return build_raw_table(L, (uint32_t*)host_table) ? BCNF_OK : BCNF_ERR_UNSUPPORTED;
}

int bcnf_fold_train_forward(const BcnfStackDesc* desc, const float* params, const float* qmats, const void* table,
                            const float* feat_weight, const float* feat_bias, int32_t in_features,
                            const BcnfGather2* gather, const float* y, const float* x, int32_t ldx, int64_t batch,
                            void* packed, float* z, float* ldj, int32_t training, uint64_t* rng_state,
                            void* workspace, int32_t finalize, float* loss_out, int32_t* guard, void* stream) {
  BcnfLayout L;
  const int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!raw_applicable(L, in_features)) return BCNF_ERR_UNSUPPORTED;
  if (!params || !qmats || !table || !feat_weight || !packed || batch < 1) return BCNF_ERR_ARG;
  RawArgs R = {};
  R.P = params;
  R.Q = qmats;
  R.table = (const uint32_t*)table;
  R.wf = feat_weight;
  R.bf = feat_bias;
  R.pk = (float*)packed;
  R.X = in_features;
  if (gather) {
    const BcnfGather2& g = *gather;
    if (g.n != batch || g.cols0 != L.D || g.cols1 < in_features || !g.idx || !g.src0 || !g.src1 || !g.dst0 ||
        !g.dst1)
      return BCNF_ERR_ARG;
    R.idx = g.idx;
    R.cursor = (const long long*)g.cursor;
    R.ypool = g.src0;
    R.ydst = g.dst0;
    R.xpool = g.src1;
    R.xdst = g.dst1;
    R.ldx = g.cols1;
  } else {
    if (!y || !x || ldx < in_features) return BCNF_ERR_ARG;
    R.ypool = y;
    R.xpool = x;
    R.ldx = ldx;
  }
  return forward_impl(desc, packed, R.ypool, R.xpool, batch, z, ldj, nullptr, training, rng_state, workspace, true,
                      true, finalize != 0, loss_out, guard, stream, nullptr, 0, 0, &R);
}

int bcnf_fold_backward_tail(const BcnfStackDesc* desc, const void* packed, const void* slab, const float* x,
                            int32_t ldx, int32_t in_features, const float* feat_weight, const float* feat_bias,
                            const void* workspace, int64_t batch, int32_t training, float* dparams,
                            float* dfeat_weight, float* dfeat_bias, const BcnfFoldAdam* adam, void* stream) {
  BcnfLayout L;
  int rc = fold_setup(desc, in_features, &L);
  if (rc) return rc;
  if (!packed || !slab || !x || !feat_weight || !workspace || !dparams || batch < 1 || ldx < in_features)
    return BCNF_ERR_ARG;
  FoldAdamArgs A = {};
  if (adam) {
    const BcnfFoldAdam& a = *adam;
    if (!a.params[0] || !a.exp_avg[0] || !a.exp_avg_sq[0] || !a.params[1] || !a.exp_avg[1] || !a.exp_avg_sq[1] ||
        !a.step || !a.done_counter || (feat_bias && (!a.params[2] || !a.exp_avg[2] || !a.exp_avg_sq[2])) ||
        (a.advance_cursor && a.cursor_modulo < 1))
      return BCNF_ERR_ARG;
    for (int t = 0; t < 3; ++t) {
      A.p[t] = a.params[t];
      A.m[t] = a.exp_avg[t];
      A.v[t] = a.exp_avg_sq[t];
    }
    if (!feat_bias) A.p[2] = A.m[2] = A.v[2] = nullptr;
    A.step = a.step;
    A.lr = a.lr;
    A.b1 = a.beta1;
    A.b2 = a.beta2;
    A.eps = a.eps;
    A.wd = a.weight_decay;
    A.cursor = (long long*)a.advance_cursor;
    A.n_batches = (long long)a.cursor_modulo;
    A.log_values = a.log_values;
    A.log_history = a.log_history;
    A.done = (int*)a.done_counter;
    A.guard = (const int*)a.guard;
    A.on = 1;
  }
  const BcnfLayout F = fold_layout(L, in_features, ldx);
  hipStream_t st = (hipStream_t)stream;
  const long long S = slab_stride_of(L);
  const int nwg = (int)((batch + 15) / 16);
  const bool drop = training && L.p > 0.f;
  const float* d1 = (const float*)workspace + ws_d1_off(L, batch, drop);
  float* work = (float*)slab + (long long)nwg * S;
  float* gx = work + w1h_work_floats(F, batch);
  A.asc = gx + (long long)L.nb * 16 * F.Cp;
  const int rps = w1h_rows_per_split(batch);
  const long long splits = w1h_splits(batch);
  const int n_red = (int)((S / 4 + RED_O4 - 1) / RED_O4);
  const int gx_dw = (L.nb + 1) / 2;
  const dim3 grid((unsigned)((long long)gx_dw * splits + (A.on ? 1 : 0)));
  size_t lds = dw1h_lds_bytes(F, 2);
  if (vec_rows(F, x)) {
    if ((rc = launch_lds(k_fold_splitk<true>, lds))) return rc;
    hipLaunchKernelGGL(k_fold_splitk<true>, grid, dim3(BCNF_WG), lds, st, F, d1, x, (long long)batch, rps, work, gx_dw,
                       (int)in_features, A);
  } else {
    if ((rc = launch_lds(k_fold_splitk<false>, lds))) return rc;
    hipLaunchKernelGGL(k_fold_splitk<false>, grid, dim3(BCNF_WG), lds, st, F, d1, x, (long long)batch, rps, work, gx_dw,
                       (int)in_features, A);
  }
  if ((rc = check_launch())) return rc;
  const long long total = (long long)L.nb * 16 * F.Cp;
  const int n_gx = (int)((total + BCNF_WG - 1) / BCNF_WG);
  hipLaunchKernelGGL(k_red_gx, dim3((unsigned)(n_gx + n_red)), dim3(BCNF_WG), 0, st, L, total, (const float*)work,
                     (int)splits, gx, n_gx, (const float*)slab, S, nwg, dparams, A);
  if ((rc = check_launch())) return rc;
  const int n_fin = (L.nb + (F.Cp >> 4)) * (L.Cp >> 4);
  size_t fin_lds = sizeof(float) * FIN_SMEM;
  if ((rc = launch_lds(k_fold_finish, fin_lds))) return rc;
  hipLaunchKernelGGL(k_fold_finish, dim3((unsigned)n_fin), dim3(BCNF_WG), fin_lds, st, L, (const float*)packed,
                     (const float*)gx, feat_weight, feat_bias, (int)in_features, dparams, dfeat_weight, dfeat_bias, A);
  return check_launch();
}

int bcnf_grad_reduce(const BcnfStackDesc* desc, const void* slab, const float* h, const void* workspace,
                     int64_t batch, int32_t training, float* dparams, void* stream) {
  // (packed is only read by the dh role, which is off here)
  return bcnf_backward_tail(desc, slab, slab, h, workspace, batch, training, nullptr, dparams, stream);
}

int bcnf_stack_dh(const BcnfStackDesc* desc, const void* packed, const void* workspace, int64_t batch, int32_t training,
                  float* dh, void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (batch < 0 || !packed || !workspace || !dh) return BCNF_ERR_ARG;
  if (batch == 0) return BCNF_OK;
  const float* d1 = (const float*)workspace + ws_d1_off(L, batch, training && L.p > 0.f);
  size_t lds = dh_lds_bytes();
  if ((rc = launch_lds(k_dh, lds))) return rc;
  hipLaunchKernelGGL(k_dh, dim3((unsigned)((batch + 63) / 64), (unsigned)(L.Cp >> 4)), dim3(BCNF_WG), lds,
                     (hipStream_t)stream, L, (const float*)packed, d1, (long long)batch, dh);
  return check_launch();
}

int bcnf_stack_inverse(const BcnfStackDesc* desc, const void* packed, const float* z, const float* h, int64_t h_rows,
                       const int64_t* cond_index, int64_t n_rows, float* y, int32_t training,
                       const uint64_t* rng_state, void* scratch, void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (n_rows == 0) return BCNF_OK;
  if (n_rows < 0 || h_rows < 1 || !packed || !z || !h || !y || !scratch) return BCNF_ERR_ARG;
  if (!cond_index && h_rows != n_rows) return BCNF_ERR_ARG;
  const bool drop = training && L.p > 0.f;
  if (drop && !rng_state) return BCNF_ERR_ARG;
  const float* pk = (const float*)packed;
  hipStream_t st = (hipStream_t)stream;
  float* hp = (float*)scratch;
  if ((rc = launch_hp(L, pk, h, h_rows, hp, st))) return rc;
  switch (L.NH) {
#define BCNF_CASE(N) case N: return inv_dispatch<N>(L, pk, z, hp, h_rows, cond_index, n_rows, y, drop, rng_state, st);
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
    default: return status >= BCNF_ERR_HIP_BASE ? hipGetErrorString((hipError_t)(status - BCNF_ERR_HIP_BASE))
                                                 : "unknown status";
  }
}

#if BCNF_STAMPS
int bcnf_debug_phases(unsigned long long* out) {   // diagnostic build only (not in include/bcnf_amd.h)
  return bcnf_rt::hip_status(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(g_phase)));
}
#endif


}  // extern "C"

namespace {

int backward_impl(const BcnfStackDesc* desc, const void* packed, const float* h, const float* dz, const float* dldj,
                  const float* dloss, int nll, int64_t batch, int32_t training, void* workspace, float* dy,
                  float* dh, float* dparams, void* slab, float* loss_out, uint64_t* rng_state, int32_t* guard,
                  void* stream) {
  BcnfLayout L;
  int rc = make_layout(desc, &L);
  if (rc) return rc;
  if (!layout_supported(L, desc)) return BCNF_ERR_UNSUPPORTED;
  if (batch < 0 || !packed || !h || !workspace || !slab) return BCNF_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (batch == 0) {
    if (dparams) return bcnf_rt::hip_status(hipMemsetAsync(dparams, 0, sizeof(float) * (size_t)L.n_trainable, st));
    return BCNF_OK;
  }
  // `training` must match the forward call that filled the workspace: it says whether dropout masks
  // were saved behind the block inputs.
  const bool drop = training && L.p > 0.f;
  float* ws = (float*)workspace;
  const float* arec = ws;
  float* d1 = ws + ws_d1_off(L, batch, drop);
  const float* pk = (const float*)packed;
  const long long stride = slab_stride_of(L);
  const float* part = ws + ws_part_off(L, batch, drop);
  uint64_t* rng_w = (loss_out && drop) ? rng_state : nullptr;
  switch (L.NH) {
#define BCNF_CASE(N) case N: rc = bwd_dispatch<N>(L, pk, dz, dldj, dloss, nll, batch, arec, dy, d1, (float*)slab, stride, part, loss_out, rng_w, guard, st); break;
    BCNF_CASE(1) BCNF_CASE(2) BCNF_CASE(3) BCNF_CASE(4) BCNF_CASE(5) BCNF_CASE(6) BCNF_CASE(7) BCNF_CASE(8)
#undef BCNF_CASE
    default: return BCNF_ERR_UNSUPPORTED;
  }
  if (rc) return rc;
  if (dparams) return bcnf_backward_tail(desc, packed, slab, h, workspace, batch, training, dh, dparams, stream);
  if (dh) return bcnf_stack_dh(desc, packed, workspace, batch, training, dh, stream);
  return BCNF_OK;   // caller finishes with bcnf_backward_tail / bcnf_grad_reduce
}

}  // namespace
