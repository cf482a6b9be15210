// Device-side building blocks for the fused CondRealNVP_v2 coupling stack (gfx950 / CDNA4).
//
// Execution layout ("row layout"): one sample per 16-lane DPP row, lane j of the row = neuron j.
// A 64-wide wavefront therefore carries 4 samples and a 256-thread workgroup 16 samples. Every
// dense layer of width <= 16 is a 16-step rotation: out_j = sum_r x[(j - r) & 15] * w_j[r], where the
// rotated operand comes from `row_ror:r` DPP folded into `v_fmac_f32_dpp` (one VALU op per MAC step,
// no LDS round trip), and w_j[r] is the lane's pre-rotated weight row staged in LDS by the pack kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bcnf_amd.h"

#define BCNF_WG 256
#define BCNF_ROWS 16           // samples per workgroup
#define BCNF_TSTRIDE 17        // padded row stride of the [16 samples][16] LDS tiles (bank spread)

typedef float floatx4 __attribute__((ext_vector_type(4)));

// HIP failures travel in the status code only (BCNF_ERR_HIP_BASE + the hipError_t, include/bcnf_amd.h): the library
// keeps no error state between calls.
namespace bcnf_rt {
inline int hip_status(hipError_t e) { return e == hipSuccess ? 0 : BCNF_ERR_HIP_BASE + (int)e; }
inline int launched() { return hip_status(hipGetLastError()); }
}  // namespace bcnf_rt

// dst0[r] = src0[idx[r]] (cols0 floats), dst1[r] = src1[idx[r]] (cols1 floats), one launch for both;
// workgroup w copies rows [w * rpw, (w + 1) * rpw) (32-bit index math: n * (cols0 + cols1) < 2^31), each
// thread BCNF_GU elements per round with every index and data load issued before the stores. With
// `cursor` != NULL the rows are idx[cursor[0] * n + r] (the cursor is advanced by a later launch).
constexpr int BCNF_GU = 8;
__device__ __forceinline__ void gather2_rows(const int64_t* __restrict__ idx, int n, int rpw,
                                             const float* __restrict__ s0, int c0, float* __restrict__ d0,
                                             const float* __restrict__ s1, int c1, float* __restrict__ d1,
                                             const long long* __restrict__ cursor, int bx) {
  if (cursor) idx += cursor[0] * n;
  const int r0 = bx * rpw, r1 = r0 + rpw < n ? r0 + rpw : n;
  const int cw = c0 + c1, total = (r1 - r0) * cw;
  for (int e0 = 0; e0 < total; e0 += BCNF_GU * BCNF_WG) {
    int r[BCNF_GU], col[BCNF_GU];
    long long src[BCNF_GU];
    float v[BCNF_GU];
#pragma unroll
    for (int u = 0; u < BCNF_GU; ++u) {
      int e = e0 + u * BCNF_WG + threadIdx.x;
      e = e < total ? e : total - 1;
      const int rr = e / cw;
      r[u] = r0 + rr;
      col[u] = e - rr * cw;
      src[u] = idx[r[u]];
    }
#pragma unroll
    for (int u = 0; u < BCNF_GU; ++u)
      v[u] = col[u] < c0 ? s0[src[u] * c0 + col[u]] : s1[src[u] * c1 + (col[u] - c0)];
#pragma unroll
    for (int u = 0; u < BCNF_GU; ++u) {
      if (e0 + u * BCNF_WG + (int)threadIdx.x >= total) continue;
      if (col[u] < c0)
        d0[r[u] * c0 + col[u]] = v[u];
      else
        d1[r[u] * c1 + (col[u] - c0)] = v[u];
    }
  }
}

// Kernel-argument form of a two-tensor gather (k_gather2, or extra workgroups of another launch).
struct BcnfGatherArgs {
  const int64_t* idx;
  const long long* cursor;
  const float* s0;
  float* d0;
  const float* s1;
  float* d1;
  int n, rpw, c0, c1, nwg;     // nwg = 0: no gather
};

// Rows per workgroup and workgroup count of a gather of n rows (at most 512 workgroups).
inline void gather2_plan(long long n, int* rpw, int* nwg) {
  const int w = n < 512 ? (int)n : 512;
  *rpw = w > 0 ? (int)((n + w - 1) / w) : 1;
  *nwg = w > 0 ? (int)((n + *rpw - 1) / *rpw) : 0;
}

// torch.optim.Adam (amsgrad=False, maximize=False) per element -- the one definition every Adam kernel uses, so the
// standalone update (k_adam) and the ones fused into the backward tail round identically:
//   g += wd p;  m = lerp(m, g, 1 - b1);  v = b2 v + (1 - b2) g g;  p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)
struct AdamScalars {
  float step_size, bc2s, omb1, omb2, b2, eps, wd;
};

// Contraction off: every caller (k_adam's vector / element paths, the fused Adam of the folded backward tail)
// rounds each operation exactly like this, whatever fma shapes the surrounding code lets hipcc pick -- the
// run_epoch == per-step-loop bit-equality rests on it.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamScalars& a) {
#pragma clang fp contract(off)
  if (a.wd != 0.f) g = fmaf(a.wd, p, g);
  m = m + a.omb1 * (g - m);                          // lerp, |weight| < 0.5 branch
  v = v * a.b2 + a.omb2 * (g * g);
  const float denom = sqrtf(v) / a.bc2s + a.eps;
  p = p + (-a.step_size) * (m / denom);
}

// Hyper-parameters arrive as doubles (Python floats); every scalar is derived in double and rounded once, as
// torch does. `sc` is 2 floats of LDS; the two pows run on two waves; ends with a __syncthreads.
__device__ __forceinline__ AdamScalars adam_scalars(float step_next, double lr, double b1d, double b2d, double epsd,
                                                    double wdd, float* sc) {
  if (threadIdx.x == 0) sc[0] = (float)(lr / (1.0 - pow(b1d, (double)step_next)));
  if (threadIdx.x == 64) sc[1] = (float)sqrt(1.0 - pow(b2d, (double)step_next));
  __syncthreads();
  return AdamScalars{sc[0], sc[1], (float)(1.0 - b1d), (float)(1.0 - b2d), (float)b2d, (float)epsd, (float)wdd};
}

__device__ __forceinline__ void store_log(const float* log_values, float* log_history, const long long* cursor) {
  if (!log_values || !log_history) return;   // host memory: system-scope stores, read after a sync
  float* dst = log_history + 3 * (cursor ? cursor[0] : 0LL);
#pragma unroll
  for (int i = 0; i < 3; ++i) __hip_atomic_store(dst + i, log_values[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
}

// End-of-step bookkeeping by one thread of a LATER launch (every reader of these counters is done):
// the Adam step count (torch keeps it as a float tensor) and an epoch cursor.
__device__ __forceinline__ void advance_counters(float* step, long long* cursor, long long n_batches) {
  if (step) step[0] += 1.0f;
  if (cursor) {
    const long long c = cursor[0] + 1;
    cursor[0] = c < n_batches ? c : 0;
  }
}

// Kernel-side form of BcnfFoldAdam (include/bcnf_amd.h): Adam applied inside the folded backward tail.
struct FoldAdamArgs {
  float* p[3];                  // 0: the coupling stack's flat parameters, 1: feature W, 2: feature b (nullable)
  float* m[3];
  float* v[3];
  float* step;
  double lr, b1, b2, eps, wd;
  long long* cursor;
  long long n_batches;
  const float* log_values;
  float* log_history;
  int* done;
  const int* guard;
  int on;
  float* asc;                   // [step_size, bc2s] of this step, written by an earlier launch of the tail
};

// The folded tail's Adam scalars, once per step: one thread of the tail's first launch derives step_size and bc2s
// exactly as adam_scalars does (double, rounded once) and stores them; the later launches load the two floats with
// their other operands instead of a step-count round trip, two double pows and a barrier per workgroup.
__device__ __forceinline__ void adam_scalars_publish(const FoldAdamArgs& A) {
  const double t = (double)(A.step[0] + 1.0f);
  A.asc[0] = (float)(A.lr / (1.0 - pow(A.b1, t)));
  A.asc[1] = (float)sqrt(1.0 - pow(A.b2, t));
}
__device__ __forceinline__ AdamScalars adam_scalars_of(const FoldAdamArgs& A, float step_size, float bc2s) {
  return AdamScalars{step_size, bc2s, (float)(1.0 - A.b1), (float)(1.0 - A.b2), (float)A.b2, (float)A.eps,
                     (float)A.wd};
}

// Host-computed layout of one stack (passed by value to every kernel).
struct BcnfLayout {
  int D, Da, Db, C, Cp, NH, nb, act_norm;
  int H[10];            // H[0] = Da (y-part width of layer 1), H[1..NH] hidden, H[NH+1] = 2*Db
  int lin_w[10], lin_b[10], lin_in[10], lin_out[10];   // Linear l = 1..NH+1 inside a coupling
  int an_size;          // 2*D if act_norm else 0
  int blk_stride;       // canonical floats per (ActNorm + coupling) block
  int cblk;             // slab floats per block: blk_stride without the W1 condition columns (H1 x C)
  int blk_pad;          // cblk rounded up to 4
  int sblk;             // floats per block of a workgroup's gradient slab (slab_blk_floats: MFMA tiles + column sums)
  int n_trainable;
  int qbc;              // QBC_* bits (Da = 10, Db = 9: every D = 19 stack): Linear 1's y-part, the mix and the
                        // backward's T / S head transposes in broadcast form (record entry c of lane j = weight of
                        // input c to output j; bc10, mix_bc, bc9x2), else rotation form (input (j - r) & 15)
  float p, keep_scale;
  uint32_t thr_hi, thr_lo;   // thresh32 = round(p 2^32) = thr_hi 2^16 + thr_lo: drop if a unit's u32 < thresh32
  int RF, RB;           // per-lane record floats (forward/inverse, backward)
  int PMB;              // floats per block of the matrix-core inverse's operand-ordered record (k_inverse_mfma)
  // record offsets (floats, per lane)
  int rf_b1, rf_w1, rf_hid, rf_t, rf_s, rf_q;
  int rb_w1t, rb_hid, rb_tt, rb_st, rb_qt, rb_an;
  // packed buffer offsets (floats)
  // W1 condition part, two contiguous copies for the projection GEMMs (NKp = nb*16 rounded up to 64):
  //   W1hC [Cp][NKp]  (c, k*16+j)   W1hR [NKp][Cp]  (k*16+j, c)   b1c [NKp]
  int NKp;
  long long pf_off, pb_off, pi_off, w1c_off, w1r_off, b1c_off, ldc_off, pm_off, total;
  int ldh;              // row stride (floats) of the projection input: C for h, ldx for the folded path's x
};

__device__ __forceinline__ int coupling_base(const BcnfLayout& L, int k) {
  return k * L.blk_stride + ((k < L.nb - 1) ? L.an_size : 0);
}

// 16-B store written through to memory (sc1): nothing of it stays dirty in the XCD's L2 for the kernel boundary's
// write-back. Inline asm: the wait pass does not count it, which only makes the compiler's own vmcnt waits stricter;
// the trailing s_nop 1 is the store-data hazard of a > 8-byte store (a VALU must not overwrite its data VGPRs in the
// next cycles), which the compiler's hazard pass covers for its own stores only (cdna_hip_programming.md §5.7).
// Only for data that later launches read: the asm carries no memory clobber, so the compiler may move this launch's
// own loads across it (every st4_wt / st1_wt call site stores records / activations / partials its kernel never
// reads back; where it may, st4_wt_ordered).
__device__ __forceinline__ void st4_wt(void* p, floatx4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v));
}
// st4_wt of an MFMA result: the compiler's hazard pass does not see the asm store read the accumulator, so the
// XDL-write -> VMEM-read wait states (11 for an 8-pass v_mfma_f32_16x16x4_f32, 19 for 16 passes) are inserted here,
// tied to the value so the nops sit between the MFMA and the store (r06: a tile stored right behind its last MFMA
// had element 2 of lanes 0-3 of each row group stale, profiles/r06j_gx_mode.patch.txt).
__device__ __forceinline__ void st4_wt_mfma(void* p, floatx4 v) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(v));
  st4_wt(p, v);
}
// The same with a "memory" clobber, for a destination the launch may also have read: k_wlink's A0 rows are the
// slab its dots path read as Alast in a non-save forward with NH odd (eval ping-pong), so no load of Alast may move
// below the store.
__device__ __forceinline__ void st4_wt_ordered(void* p, floatx4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st1_wt(void* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" : : "v"(p), "v"(v));
}

// ---------------------------------------------------------------------------------------------
// Rotation dot product over a 16-lane row: acc + sum_r x[(j-r)&15] * w[r].
// The 15 DPP steps sit in ONE asm statement: the leading `s_nop 1` covers the VALU-write -> DPP-read
// hazard on x (2 wait states) for whatever the compiler scheduled right before, and no compiler
// copy of x can land between two DPP reads.
// ---------------------------------------------------------------------------------------------
#define BCNF_DPP(R, A, X, W) "v_fmac_f32_dpp " A ", " X ", " W " row_ror:" #R " row_mask:0xf bank_mask:0xf\n\t"

__device__ __forceinline__ float rot16(float x, const float* __restrict__ w, float acc) {
  // two interleaved partial sums (even / odd rotations) halve the dependent fmac chain
  float acc1;
  acc = fmaf(x, w[0], acc);
  asm("s_nop 1\n\t"
      "v_mul_f32_dpp %1, %2, %3 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      BCNF_DPP(2, "%0", "%2", "%4") BCNF_DPP(3, "%1", "%2", "%5") BCNF_DPP(4, "%0", "%2", "%6")
      BCNF_DPP(5, "%1", "%2", "%7") BCNF_DPP(6, "%0", "%2", "%8") BCNF_DPP(7, "%1", "%2", "%9")
      BCNF_DPP(8, "%0", "%2", "%10") BCNF_DPP(9, "%1", "%2", "%11") BCNF_DPP(10, "%0", "%2", "%12")
      BCNF_DPP(11, "%1", "%2", "%13") BCNF_DPP(12, "%0", "%2", "%14") BCNF_DPP(13, "%1", "%2", "%15")
      BCNF_DPP(14, "%0", "%2", "%16") BCNF_DPP(15, "%1", "%2", "%17")
      : "+v"(acc), "=&v"(acc1)
      : "v"(x), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]),
        "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15]));
  return acc + acc1;
}

// Two independent rotation chains interleaved in one asm block (hides the fmac dependency latency).
__device__ __forceinline__ void rot16x2(float x0, const float* __restrict__ w0, float& a0,
                                        float x1, const float* __restrict__ w1, float& a1) {
  a0 = fmaf(x0, w0[0], a0);
  a1 = fmaf(x1, w1[0], a1);
  asm("s_nop 1\n\t"
      BCNF_DPP(1, "%0", "%2", "%4") BCNF_DPP(1, "%1", "%3", "%19")
      BCNF_DPP(2, "%0", "%2", "%5") BCNF_DPP(2, "%1", "%3", "%20")
      BCNF_DPP(3, "%0", "%2", "%6") BCNF_DPP(3, "%1", "%3", "%21")
      BCNF_DPP(4, "%0", "%2", "%7") BCNF_DPP(4, "%1", "%3", "%22")
      BCNF_DPP(5, "%0", "%2", "%8") BCNF_DPP(5, "%1", "%3", "%23")
      BCNF_DPP(6, "%0", "%2", "%9") BCNF_DPP(6, "%1", "%3", "%24")
      BCNF_DPP(7, "%0", "%2", "%10") BCNF_DPP(7, "%1", "%3", "%25")
      BCNF_DPP(8, "%0", "%2", "%11") BCNF_DPP(8, "%1", "%3", "%26")
      BCNF_DPP(9, "%0", "%2", "%12") BCNF_DPP(9, "%1", "%3", "%27")
      BCNF_DPP(10, "%0", "%2", "%13") BCNF_DPP(10, "%1", "%3", "%28")
      BCNF_DPP(11, "%0", "%2", "%14") BCNF_DPP(11, "%1", "%3", "%29")
      BCNF_DPP(12, "%0", "%2", "%15") BCNF_DPP(12, "%1", "%3", "%30")
      BCNF_DPP(13, "%0", "%2", "%16") BCNF_DPP(13, "%1", "%3", "%31")
      BCNF_DPP(14, "%0", "%2", "%17") BCNF_DPP(14, "%1", "%3", "%32")
      BCNF_DPP(15, "%0", "%2", "%18") BCNF_DPP(15, "%1", "%3", "%33")
      : "+v"(a0), "+v"(a1)
      : "v"(x0), "v"(x1),
        "v"(w0[1]), "v"(w0[2]), "v"(w0[3]), "v"(w0[4]), "v"(w0[5]), "v"(w0[6]), "v"(w0[7]), "v"(w0[8]),
        "v"(w0[9]), "v"(w0[10]), "v"(w0[11]), "v"(w0[12]), "v"(w0[13]), "v"(w0[14]), "v"(w0[15]),
        "v"(w1[1]), "v"(w1[2]), "v"(w1[3]), "v"(w1[4]), "v"(w1[5]), "v"(w1[6]), "v"(w1[7]), "v"(w1[8]),
        "v"(w1[9]), "v"(w1[10]), "v"(w1[11]), "v"(w1[12]), "v"(w1[13]), "v"(w1[14]), "v"(w1[15]));
}

// Broadcast forms (round 6) for the D = 19 stacks' half-vectors (Da = 10, Db = 9 inputs in lanes 0 .. 9 / 0 .. 8):
// `row_newbcast:c` reads lane c of the lane's own 16-lane row, so acc_j + sum_{c < N} x[c] w_j[c] costs N DPP FMAs
// where a rotation matvec costs 16 (record entry c of lane j = the weight from input c to output j). Two interleaved
// accumulators hide the fmac latency; the leading s_nop 1 covers a VALU write of x right before (as in rot16).
#define BCNF_BC(C, A, X, W) "v_fmac_f32_dpp " A ", " X ", " W " row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t"
#define BCNF_BCM(C, A, X, W) "v_mul_f32_dpp " A ", " X ", " W " row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t"

// acc + sum_{c < 10} x[c] w[c]  (Linear 1's y-part: Da = 10 inputs -> 16 hidden)
__device__ __forceinline__ float bc10(float x, const float* __restrict__ w, float acc) {
  float acc1;
  asm("s_nop 1\n\t"
      BCNF_BC(0, "%0", "%2", "%3") BCNF_BCM(1, "%1", "%2", "%4") BCNF_BC(2, "%0", "%2", "%5")
      BCNF_BC(3, "%1", "%2", "%6") BCNF_BC(4, "%0", "%2", "%7") BCNF_BC(5, "%1", "%2", "%8")
      BCNF_BC(6, "%0", "%2", "%9") BCNF_BC(7, "%1", "%2", "%10") BCNF_BC(8, "%0", "%2", "%11")
      BCNF_BC(9, "%1", "%2", "%12")
      : "+v"(acc), "=&v"(acc1)
      : "v"(x), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]), "v"(w[8]), "v"(w[9]));
  return acc + acc1;
}

// (a0, a1) = (sum_{c < 9} x0[c] w0[c], sum_{c < 9} x1[c] w1[c])  (the backward's T / S heads: Db = 9 inputs each)
__device__ __forceinline__ void bc9x2(float x0, const float* __restrict__ w0, float& a0,
                                      float x1, const float* __restrict__ w1, float& a1) {
  asm("s_nop 1\n\t"
      BCNF_BCM(0, "%0", "%2", "%4") BCNF_BCM(0, "%1", "%3", "%13")
      BCNF_BC(1, "%0", "%2", "%5") BCNF_BC(1, "%1", "%3", "%14")
      BCNF_BC(2, "%0", "%2", "%6") BCNF_BC(2, "%1", "%3", "%15")
      BCNF_BC(3, "%0", "%2", "%7") BCNF_BC(3, "%1", "%3", "%16")
      BCNF_BC(4, "%0", "%2", "%8") BCNF_BC(4, "%1", "%3", "%17")
      BCNF_BC(5, "%0", "%2", "%9") BCNF_BC(5, "%1", "%3", "%18")
      BCNF_BC(6, "%0", "%2", "%10") BCNF_BC(6, "%1", "%3", "%19")
      BCNF_BC(7, "%0", "%2", "%11") BCNF_BC(7, "%1", "%3", "%20")
      BCNF_BC(8, "%0", "%2", "%12") BCNF_BC(8, "%1", "%3", "%21")
      : "=&v"(a0), "=&v"(a1)
      : "v"(x0), "v"(x1), "v"(w0[0]), "v"(w0[1]), "v"(w0[2]), "v"(w0[3]), "v"(w0[4]), "v"(w0[5]), "v"(w0[6]), "v"(w0[7]), "v"(w0[8]),
        "v"(w1[0]), "v"(w1[1]), "v"(w1[2]), "v"(w1[3]), "v"(w1[4]), "v"(w1[5]), "v"(w1[6]), "v"(w1[7]), "v"(w1[8]));
}

// The orthonormal mix of a D = 19 state (a: 10 lanes, b: 9 lanes) in broadcast form: na = sum_c a[c] rq[c] +
// sum_c b[c] rq[10 + c], nb = sum_c a[c] rq[19 + c] + sum_c b[c] rq[29 + c]: 38 DPP FMAs instead of 4 rotations (64).
__device__ __forceinline__ void mix_bc(const float* __restrict__ rq, float a, float b, float& na, float& nbv) {
  asm("s_nop 1\n\t"
      BCNF_BCM(0, "%0", "%2", "%4") BCNF_BCM(0, "%1", "%2", "%23")
      BCNF_BC(1, "%0", "%2", "%5") BCNF_BC(1, "%1", "%2", "%24")
      BCNF_BC(2, "%0", "%2", "%6") BCNF_BC(2, "%1", "%2", "%25")
      BCNF_BC(3, "%0", "%2", "%7") BCNF_BC(3, "%1", "%2", "%26")
      BCNF_BC(4, "%0", "%2", "%8") BCNF_BC(4, "%1", "%2", "%27")
      BCNF_BC(5, "%0", "%2", "%9") BCNF_BC(5, "%1", "%2", "%28")
      BCNF_BC(6, "%0", "%2", "%10") BCNF_BC(6, "%1", "%2", "%29")
      BCNF_BC(7, "%0", "%2", "%11") BCNF_BC(7, "%1", "%2", "%30")
      BCNF_BC(8, "%0", "%2", "%12") BCNF_BC(8, "%1", "%2", "%31")
      BCNF_BC(9, "%0", "%2", "%13") BCNF_BC(9, "%1", "%2", "%32")
      BCNF_BC(0, "%0", "%3", "%14") BCNF_BC(0, "%1", "%3", "%33")
      BCNF_BC(1, "%0", "%3", "%15") BCNF_BC(1, "%1", "%3", "%34")
      BCNF_BC(2, "%0", "%3", "%16") BCNF_BC(2, "%1", "%3", "%35")
      BCNF_BC(3, "%0", "%3", "%17") BCNF_BC(3, "%1", "%3", "%36")
      BCNF_BC(4, "%0", "%3", "%18") BCNF_BC(4, "%1", "%3", "%37")
      BCNF_BC(5, "%0", "%3", "%19") BCNF_BC(5, "%1", "%3", "%38")
      BCNF_BC(6, "%0", "%3", "%20") BCNF_BC(6, "%1", "%3", "%39")
      BCNF_BC(7, "%0", "%3", "%21") BCNF_BC(7, "%1", "%3", "%40")
      BCNF_BC(8, "%0", "%3", "%22") BCNF_BC(8, "%1", "%3", "%41")
      : "=&v"(na), "=&v"(nbv)
      : "v"(a), "v"(b), "v"(rq[0]), "v"(rq[1]), "v"(rq[2]), "v"(rq[3]), "v"(rq[4]), "v"(rq[5]), "v"(rq[6]), "v"(rq[7]), "v"(rq[8]), "v"(rq[9]), "v"(rq[10]), "v"(rq[11]), "v"(rq[12]), "v"(rq[13]), "v"(rq[14]), "v"(rq[15]), "v"(rq[16]), "v"(rq[17]), "v"(rq[18]), "v"(rq[19]), "v"(rq[20]), "v"(rq[21]), "v"(rq[22]), "v"(rq[23]), "v"(rq[24]), "v"(rq[25]), "v"(rq[26]), "v"(rq[27]), "v"(rq[28]), "v"(rq[29]), "v"(rq[30]), "v"(rq[31]), "v"(rq[32]), "v"(rq[33]), "v"(rq[34]), "v"(rq[35]), "v"(rq[36]), "v"(rq[37]));
}

// Sum over the 16 lanes of a row, result in every lane of the row.
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, true));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, true));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, true));  // row_ror:2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, true));  // row_ror:1
  return v;
}

// Load 16 consecutive floats (16-B aligned LDS) into registers.
__device__ __forceinline__ void ld16(float* __restrict__ w, const float* __restrict__ p) {
  const floatx4* q = reinterpret_cast<const floatx4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const floatx4 v = q[i];
    w[4 * i + 0] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}

// ---------------------------------------------------------------------------------------------
// Branch-free fp32 transcendentals for the block bodies (no divergent basic blocks, unlike ocml's
// erff / expf range checks). tanh: both regions evaluated and selected (coefficients fitted and
// verified in emulated fp32 by tools/fit_erf.py, <= 1.3 ulp).
// ---------------------------------------------------------------------------------------------
// exp(x) as one v_exp_f32 (2^x, 1 ulp) of x log2(e): relative error < 1 ulp + |x| 2^-24, no range
// checks (overflow -> inf, underflow -> 0, which every caller tolerates).
__device__ __forceinline__ float exp_fast(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896340736f); }

// tanh(a) = 1 - 2 / (exp(2a) + 1): one v_exp_f32, one v_rcp_f32, branch-free, saturating to +-1 through inf / 0
// (r04: replaces a two-region form -- odd polynomial below |a| = 0.625, this expression above, both evaluated and
// selected -- that cost ~16 VALU instead of 5). Absolute error <= 1.9e-7 on [-12, 12] against float64 tanh
// (emulated fp32, tools/fit_erf.py tanh_check); S = tanh(s') enters the coupling as exp(S) and the log-det as S, both
// of which see absolute, not relative, error.
__device__ __forceinline__ float tanh_bf(float a) {
  const float e = __builtin_amdgcn_exp2f(a * 2.88539008177792681472f);   // exp(2a)
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

// Exact-erf GELU as nn.GELU(approximate='none') (cnf.py:81 via LayerFactory): x Phi(x), with the normal
// CDF from the complementary error function, Phi(-|x|) = erfc(z) / 2, z = |x| / sqrt2, and
//   erfc(z) = t exp(-z^2) Q(t),  t = 1 / (1 + p z),  p = 0.37,  Q of degree 6
// (weighted least-squares minimax fit on z in [0, 7], |relative error| < 3.8e-7; tools/fit_erf.py gelu_fit).
// One exp -- exp(-x^2/2), shared with phi(x) in the derivative -- and one rcp; the 1/2 is folded into Q.
// Branch-free; no cancellation for x < 0. In fp32: |GELU error| < 3.9e-7, |GELU' error| < 3.6e-7 against the
// double-precision function (the fp32 0.5 x (1 + erf(x/sqrt2)) of the reference: < 4.5e-7). Replaces (r02x) the
// Numerical Recipes erfcc form t exp(-z^2 + P9(t)), which took a second exp and three more FMAs per call: the
// GELUs are ~18% of the FC_small forward's compute chain (an r02 experiment build with GELU replaced by x/2: 64.4 -> 52.5 us).
// r04: the 1/2 and 1/sqrt(2 pi) live in the constants: the exponential is phi(x) = exp(-x^2/2) / sqrt(2 pi) itself
// (exp2(x^2 (-log2(e)/2) + log2(1/sqrt(2 pi))): the derivative's phi costs nothing extra) and Q carries sqrt(2 pi)/2,
// so h = Phi(-|x|) = t Q(t) phi(x).
__device__ __forceinline__ float gelu_tq(float x, float& phi) {   // t Q(t); phi = phi(x)
  const float t = __builtin_amdgcn_rcpf(fmaf(2.616295218e-01f, fabsf(x), 1.0f));   // p / sqrt2
  float q = -1.828701629e-01f;                                                      // Q x sqrt(2 pi)
  q = fmaf(q, t, 5.613370996e-01f);
  q = fmaf(q, t, -2.561027660e-01f);
  q = fmaf(q, t, 4.147041470e-01f);
  q = fmaf(q, t, 1.844545274e-01f);
  q = fmaf(q, t, 2.707437625e-01f);
  q = fmaf(q, t, 2.610471003e-01f);
  phi = __builtin_amdgcn_exp2f(fmaf(x * x, -0.72134752044448170368f, -1.32574806473615920f));
  return t * q;
}
// Forward-only GELU (no derivative needed): x Phi(x) = max(x, 0) - |x| h, h = Phi(-|x|) = exp2(P6(min(|x|, 6.5))) --
// erfc's e^{-x^2/2} decay is quadratic in |x|, so log2 h is ONE polynomial (tools/fit_erf.py fit_log2h: fp32 GELU error
// 2.8e-7 = the result's rounding; 8.7e-8 for x < 0): one exp2 and no reciprocal.
__device__ __forceinline__ float gelu_h(float x) {
  const float a = __builtin_amdgcn_fmed3f(fabsf(x), 0.f, 6.5f);   // one v_med3 (fminf adds a canonicalising v_max)
  float p = 3.309481690e-05f;
  p = fmaf(p, a, -7.692371728e-04f);
  p = fmaf(p, a, 8.080773987e-03f);
  p = fmaf(p, a, -5.341219157e-02f);
  p = fmaf(p, a, -4.587709010e-01f);
  p = fmaf(p, a, -1.151201725e+00f);
  p = fmaf(p, a, -9.999930859e-01f);
  return __builtin_amdgcn_exp2f(p);
}
__device__ __forceinline__ float gelu_f(float x) {          // x Phi(x) = max(x, 0) - |x| Phi(-|x|)
  const float h = gelu_h(x);
  // max(x, 0) as ONE v_max_f32 (fmaxf under IEEE mode canonicalises an operand that comes out of inline asm); it reads
  // x after h, whose computation from x carries any wait states an MFMA-produced x needs
  float r;
  asm("v_max_f32_e32 %0, 0, %1" : "=v"(r) : "v"(x), "v"(h));
  return fmaf(-fabsf(x), h, r);
}
// GELU and its derivative Phi(x) + x phi(x): Phi(x) = 1/2 + sign(x) (1/2 - Phi(-|x|)), the sign moved by one bit
// and-or (v_and_or_b32) instead of a compare and a select.
__device__ __forceinline__ void gelu_fg(float x, float& g, float& dg) {
  float phi;
  const float hm = fmaf(-gelu_tq(x, phi), phi, 0.5f);                      // 1/2 - Phi(-|x|) >= 0
  const float cdf = 0.5f + __uint_as_float(__float_as_uint(hm) | (__float_as_uint(x) & 0x80000000u));
  g = x * cdf;
  dg = fmaf(x, phi, cdf);
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al. 2011) for in-register dropout masks.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {     // one 32x32->64 multiply (v_mad_u64_u32) per product
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Keep bits (bit l = keep decision for hidden layer l+1) for (sample, block, lane) of a stack with NU <= 8 hidden
// layers. Unit i keeps iff its 32-bit uniform u_i >= thresh32 = round(p 2^32): nn.Dropout's p to 2^-32, the rule of
// the wide family and k_lin (round 5 compared 16-bit draws with round(p 2^16): p = 0.383 ran as 0.38299561, and any
// p < 2^-17 as no dropout at all). u_i = (high half: one 16-bit half of a Philox4x32-10 draw, low half L):
//  * NU < 8 (FC_small: 7): L is the draw's unused eighth half, shared by the units of one call -- each u_i is then
//    exactly uniform on 32 bits (so each unit drops with probability thresh32 / 2^32), and two units of one call
//    are dependent only through ties of BOTH high halves with thr_hi (probability < 2^-32 per call). As L is shared,
//    u_i >= thresh32 <=> h_i >= thr_hi + [L < thr_lo]: one compare per unit, the cost of the 16-bit rule;
//  * NU == 8: each unit's own L from a second draw of the same counter with tag bit 29, which a wave runs only when
//    one of its lanes ties (probability 2^-16 per unit) and thr_lo != 0.
template <int NU>
__device__ __forceinline__ uint32_t dropout_bits(const BcnfLayout& L, uint64_t seed, uint64_t offset,
                                                 long long sample, int block, int lane, uint32_t tag) {
  static_assert(NU >= 1 && NU <= 8, "8 units per draw");
  const uint4 ctr = make_uint4((uint32_t)sample,
                               (uint32_t)((unsigned long long)sample >> 32) ^ ((uint32_t)block << 8) ^ tag,
                               (uint32_t)lane, (uint32_t)offset);
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(offset >> 32));
  const uint4 r = philox4x32_10(ctr, key);
  uint32_t bits = 0;
  if constexpr (NU < 8) {
    // u_i = (h_i, L) >= (thr_hi, thr_lo)  <=>  h_i >= thr_hi + [L < thr_lo]: with L shared, one 16-bit threshold per
    // call, and each unit costs the one compare of a 16-bit rule (a compare of a word half)
    const uint32_t t = L.thr_hi + ((r.w >> 16) < L.thr_lo ? 1u : 0u);
    const uint32_t h[7] = {r.x & 0xffffu, r.x >> 16, r.y & 0xffffu, r.y >> 16, r.z & 0xffffu, r.z >> 16, r.w & 0xffffu};
#pragma unroll
    for (int i = 0; i < NU; ++i) bits |= (h[i] >= t ? 1u : 0u) << i;
  } else {
    const uint32_t th = L.thr_hi;
    const uint32_t h[8] = {r.x & 0xffffu, r.x >> 16, r.y & 0xffffu, r.y >> 16,
                           r.z & 0xffffu, r.z >> 16, r.w & 0xffffu, r.w >> 16};
    uint32_t tie = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bits |= (h[i] > th ? 1u : 0u) << i;
      tie |= (h[i] == th ? 1u : 0u) << i;
    }
    if (tie) {
      const uint32_t tl = L.thr_lo;
      if (tl == 0) {
        bits |= tie;
      } else {
        const uint4 r2 = philox4x32_10(make_uint4(ctr.x, ctr.y ^ 0x20000000u, ctr.z, ctr.w), key);
        const uint32_t lo[8] = {r2.x & 0xffffu, r2.x >> 16, r2.y & 0xffffu, r2.y >> 16,
                                r2.z & 0xffffu, r2.z >> 16, r2.w & 0xffffu, r2.w >> 16};
#pragma unroll
        for (int i = 0; i < 8; ++i) bits |= (((tie >> i) & 1u) && lo[i] >= tl ? 1u : 0u) << i;
      }
    }
  }
  return bits;
}

// ---------------------------------------------------------------------------------------------
// fp32-in MFMA 16x16x4 (v_mfma_f32_16x16x4_f32; exact f32 fma chain).
// Lane l: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15], D[row = 4*(l>>4) + r][col = l&15].
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
