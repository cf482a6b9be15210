// Issue-rate probe (gfx950): cycles per instruction of the forward chain's instruction kinds, one wave per SIMD
// and two waves per SIMD. Each wave runs REP x a body (32 instructions unless the driver says otherwise) between
// two (s_memtime, s_memrealtime) stamp pairs; the host divides by the instruction count. s_memrealtime ticks at a
// constant 100 MHz, so ns per instruction and the shader clock (MI355X_MICROARCH.md note (6): d memtime / d realtime
// x 100 MHz) come out of the same run. Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe_issue.hip
//   -o tools/probe_issue.so ; run: python tools/probe_issue.py
#include <hip/hip_runtime.h>
#include <stdint.h>

#define REP 4096

#define FMA4(a, b, c, d) "v_fmac_f32 " a ", %4, %5\n\tv_fmac_f32 " b ", %4, %5\n\tv_fmac_f32 " c ", %4, %5\n\tv_fmac_f32 " d ", %4, %5\n\t"
#define DPP2(r) "v_fmac_f32_dpp %0, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %1, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"
#define DPP4(r) "v_fmac_f32_dpp %0, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %1, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %3, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"
#define DEP1 "v_fmac_f32 %0, %4, %5\n\t"
#define PK2 "v_pk_fma_f32 %0, %4, %5, %0\n\tv_pk_fma_f32 %2, %4, %5, %2\n\t"
#define EXP4 "v_exp_f32 %0, %4\n\tv_exp_f32 %1, %4\n\tv_exp_f32 %2, %4\n\tv_exp_f32 %3, %4\n\t"

template <int KIND>
__device__ __forceinline__ void body(float& a, float& b, float& c, float& d, float x, float w) {
  if (KIND == 0) {          // 32 independent v_fmac_f32 (4 accumulators)
    asm volatile(FMA4("%0", "%1", "%2", "%3") FMA4("%0", "%1", "%2", "%3") FMA4("%0", "%1", "%2", "%3")
                 FMA4("%0", "%1", "%2", "%3") FMA4("%0", "%1", "%2", "%3") FMA4("%0", "%1", "%2", "%3")
                 FMA4("%0", "%1", "%2", "%3") FMA4("%0", "%1", "%2", "%3")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 1) {   // 32 v_fmac_f32_dpp, 2 interleaved accumulators (the rot16 shape)
    asm volatile("s_nop 1\n\t" DPP2(1) DPP2(2) DPP2(3) DPP2(4) DPP2(5) DPP2(6) DPP2(7) DPP2(8) DPP2(9) DPP2(10)
                 DPP2(11) DPP2(12) DPP2(13) DPP2(14) DPP2(15) DPP2(1)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 2) {   // 32 v_fmac_f32_dpp, 4 interleaved accumulators
    asm volatile("s_nop 1\n\t" DPP4(1) DPP4(2) DPP4(3) DPP4(4) DPP4(5) DPP4(6) DPP4(7) DPP4(8)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 3) {   // 32 dependent v_fmac_f32 (one accumulator)
    asm volatile(DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1
                 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1 DEP1
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 5) {   // 32 v_pk_fma_f32 (independent, 2 packed accumulators)
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p = {a, b}, q = {c, d};
    const f2 xx = {x, x}, ww = {w, w};
    asm volatile(PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2 PK2
                 : "+v"(p), "+v"(b), "+v"(q), "+v"(d) : "v"(xx), "v"(ww));
    a = p[0] + p[1];
    c = q[0] + q[1];
  } else if (KIND == 6) {   // 32 v_mul_f32_dpp row_newbcast-free form: v_add_f32_dpp row_ror (2 acc)
    asm volatile("s_nop 1\n\t"
#define ADPP2(r) "v_add_f32_dpp %0, %4, %0 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %1, %4, %1 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"
                 ADPP2(1) ADPP2(2) ADPP2(3) ADPP2(4) ADPP2(5) ADPP2(6) ADPP2(7) ADPP2(8) ADPP2(9) ADPP2(10)
                 ADPP2(11) ADPP2(12) ADPP2(13) ADPP2(14) ADPP2(15) ADPP2(1)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 7) {   // 32 v_permlane16_swap_b32 (4 independent register pairs)
#define PL4 "v_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\tv_permlane16_swap_b32 %1, %0\n\tv_permlane16_swap_b32 %3, %2\n\t"
    asm volatile(PL4 PL4 PL4 PL4 PL4 PL4 PL4 PL4 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 8) {   // the split-row combine, dependent: 8 x (2 add, nop, permlane16_swap, nop, add_dpp) = 32 VALU
#define CMB "v_add_f32 %1, %0, %2\n\tv_add_f32 %3, %2, %0\n\ts_nop 1\n\tv_permlane16_swap_b32 %1, %3\n\ts_nop 1\n\tv_add_f32_dpp %0, %3, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
    asm volatile(CMB CMB CMB CMB CMB CMB CMB CMB : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 9) {   // the forward's GELU, 17 dependent VALU (2 transcendental) x 2 = 34 instructions
#define GELU "v_fma_f32 %1, |%0|, %5, 1.0\n\tv_rcp_f32 %1, %1\n\tv_mul_f32 %2, %0, %0\n\tv_fmamk_f32 %2, %2, 0xbf38aa3b, %4\n\t" \
             "v_exp_f32 %3, %2\n\tv_fmamk_f32 %2, %1, 0xbe3b4251, %4\n\tv_fmaak_f32 %2, %2, %1, 0xbe831fe7\n\t"         \
             "v_fmaak_f32 %2, %2, %1, 0x3ed4541a\n\tv_fmaak_f32 %2, %2, %1, 0x3e3ce1a6\n\tv_fmaak_f32 %2, %2, %1, 0x3e8a9eed\n\t" \
             "v_fmaak_f32 %2, %2, %1, 0x3e85a7f7\n\tv_mul_f32 %1, %1, -%2\n\tv_fma_f32 %1, %1, %3, 0.5\n\t"               \
             "v_and_or_b32 %1, %0, %5, %1\n\tv_add_f32 %1, 0.5, %1\n\tv_mul_f32 %1, %0, %1\n\tv_mul_f32 %0, %1, %5\n\t"
    asm volatile(GELU GELU : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 10) {  // one row-layout dense layer as in k_forward: fma + mul_dpp + 14 fmac_dpp (2 acc) + add,
                            // the layer output feeding the next layer's DPP source (s_nop 1 hazard) x 2 = 38
#define LAYER "v_fma_f32 %1, %0, %5, %4\n\ts_nop 1\n\tv_mul_f32_dpp %2, %0, %5 row_ror:1 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:2 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:3 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:4 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:5 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:6 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:7 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:8 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:9 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:10 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:11 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:12 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:13 row_mask:0xf bank_mask:0xf\n\t" \
              "v_fmac_f32_dpp %1, %0, %5 row_ror:14 row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %2, %0, %5 row_ror:15 row_mask:0xf bank_mask:0xf\n\t" \
              "v_add_f32 %0, %1, %2\n\tv_mul_f32 %0, %0, %5\n\t"
    asm volatile(LAYER LAYER : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 11) {  // 32 v_fmac_f32_dpp, 2 acc, the rotation changing every instruction (rot16's order)
#define D1(A, r) "v_fmac_f32_dpp " A ", %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"
    asm volatile("s_nop 1\n\t" D1("%0", 1) D1("%1", 2) D1("%0", 3) D1("%1", 4) D1("%0", 5) D1("%1", 6) D1("%0", 7) D1("%1", 8)
                 D1("%0", 9) D1("%1", 10) D1("%0", 11) D1("%1", 12) D1("%0", 13) D1("%1", 14) D1("%0", 15) D1("%1", 1)
                 D1("%0", 2) D1("%1", 3) D1("%0", 4) D1("%1", 5) D1("%0", 6) D1("%1", 7) D1("%0", 8) D1("%1", 9)
                 D1("%0", 10) D1("%1", 11) D1("%0", 12) D1("%1", 13) D1("%0", 14) D1("%1", 15) D1("%0", 1) D1("%1", 2)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 12) {  // rot16x2's shape: 2 acc, 2 DPP sources, each rotation twice in a row
#define D2(r) "v_fmac_f32_dpp %0, %4, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\tv_fmac_f32_dpp %1, %2, %5 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"
    asm volatile("s_nop 1\n\t" D2(1) D2(2) D2(3) D2(4) D2(5) D2(6) D2(7) D2(8) D2(9) D2(10) D2(11) D2(12) D2(13) D2(14) D2(15) D2(1)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 13) {  // one accumulator, 32 dependent v_fmac_f32_dpp, rotation changing every instruction
    asm volatile("s_nop 1\n\t" D1("%0", 1) D1("%0", 2) D1("%0", 3) D1("%0", 4) D1("%0", 5) D1("%0", 6) D1("%0", 7) D1("%0", 8)
                 D1("%0", 9) D1("%0", 10) D1("%0", 11) D1("%0", 12) D1("%0", 13) D1("%0", 14) D1("%0", 15) D1("%0", 1)
                 D1("%0", 2) D1("%0", 3) D1("%0", 4) D1("%0", 5) D1("%0", 6) D1("%0", 7) D1("%0", 8) D1("%0", 9)
                 D1("%0", 10) D1("%0", 11) D1("%0", 12) D1("%0", 13) D1("%0", 14) D1("%0", 15) D1("%0", 1) D1("%0", 2)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 14) {  // 4 acc, rotation changing every instruction
    asm volatile("s_nop 1\n\t" D1("%0", 1) D1("%1", 2) D1("%2", 3) D1("%3", 4) D1("%0", 5) D1("%1", 6) D1("%2", 7) D1("%3", 8)
                 D1("%0", 9) D1("%1", 10) D1("%2", 11) D1("%3", 12) D1("%0", 13) D1("%1", 14) D1("%2", 15) D1("%3", 1)
                 D1("%0", 2) D1("%1", 3) D1("%2", 4) D1("%3", 5) D1("%0", 6) D1("%1", 7) D1("%2", 8) D1("%3", 9)
                 D1("%0", 10) D1("%1", 11) D1("%2", 12) D1("%3", 13) D1("%0", 14) D1("%1", 15) D1("%2", 1) D1("%3", 2)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 15) {  // 2 acc, the same rotation (row_ror:1) throughout
    asm volatile("s_nop 1\n\t" D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1)
                 D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1)
                 D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1)
                 D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1) D1("%0", 1) D1("%1", 1)
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 16) {  // plain v_fmac_f32, 2 acc (the DPP-free twin of 11)
    asm volatile(FMA4("%0", "%1", "%0", "%1") FMA4("%0", "%1", "%0", "%1") FMA4("%0", "%1", "%0", "%1") FMA4("%0", "%1", "%0", "%1")
                 FMA4("%0", "%1", "%0", "%1") FMA4("%0", "%1", "%0", "%1") FMA4("%0", "%1", "%0", "%1") FMA4("%0", "%1", "%0", "%1")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  } else if (KIND == 4) {   // 32 v_exp_f32 (independent)
    asm volatile(EXP4 EXP4 EXP4 EXP4 EXP4 EXP4 EXP4 EXP4 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  }
}


// Explicit-register DPP probes (r05): one asm statement holds the whole REP loop, so the VGPR banks (v mod 4) of the
// accumulators, the DPP source and the weight are fixed: "A0 A1 S W" name the registers.
#define XD(A, S, W, r) "v_fmac_f32_dpp " A ", " S ", " W " row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t"
#define XB(A0, A1, S, W) XD(A0, S, W, 1) XD(A1, S, W, 2) XD(A0, S, W, 3) XD(A1, S, W, 4) XD(A0, S, W, 5) XD(A1, S, W, 6) \
  XD(A0, S, W, 7) XD(A1, S, W, 8) XD(A0, S, W, 9) XD(A1, S, W, 10) XD(A0, S, W, 11) XD(A1, S, W, 12) XD(A0, S, W, 13)  \
  XD(A1, S, W, 14) XD(A0, S, W, 15) XD(A1, S, W, 1) XD(A0, S, W, 2) XD(A1, S, W, 3) XD(A0, S, W, 4) XD(A1, S, W, 5)     \
  XD(A0, S, W, 6) XD(A1, S, W, 7) XD(A0, S, W, 8) XD(A1, S, W, 9) XD(A0, S, W, 10) XD(A1, S, W, 11) XD(A0, S, W, 12)   \
  XD(A1, S, W, 13) XD(A0, S, W, 14) XD(A1, S, W, 15) XD(A0, S, W, 1) XD(A1, S, W, 2)
#define XP(A, S, W) "v_fmac_f32 " A ", " S ", " W "\n\t"
#define XBP(A0, A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) \
  XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W)                          \
  XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W)                          \
  XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W) XP(A0, S, W) XP(A1, S, W)
#define XLOOP(BODY, A0, A1, S, W)                                                                              \
  asm volatile("v_mov_b32 " A0 ", %1\n\tv_mov_b32 " A1 ", %1\n\tv_mov_b32 " S ", %2\n\tv_mov_b32 " W ", %3\n\t" \
               "s_mov_b32 s40, 4096\n\ts_nop 4\n"                                                            \
               "1:\n\t" BODY "s_sub_u32 s40, s40, 1\n\ts_cmp_lg_u32 s40, 0\n\ts_cbranch_scc1 1b\n\t"     \
               "v_add_f32 %0, " A0 ", " A1 "\n\t"                                                            \
               : "=v"(a) : "v"(a), "v"(x), "v"(w) : "v10", "v11", "v13", "v14", "v21", "v22", "v29", "v32", "v33", "v34", "s40", "scc")

template <int KIND>
__device__ __forceinline__ void xbody(float& a, float x, float w) {
  if (KIND == 17) XLOOP(XB("v10", "v11", "v21", "v32"), "v10", "v11", "v21", "v32");        // banks 2 3 | 1 | 0
  else if (KIND == 18) XLOOP(XB("v10", "v14", "v22", "v33"), "v10", "v14", "v22", "v33");   // acc = src bank (2)
  else if (KIND == 19) XLOOP(XB("v10", "v11", "v21", "v29"), "v10", "v11", "v21", "v29");   // w = src bank (1)
  else if (KIND == 20) XLOOP(XB("v10", "v14", "v21", "v34"), "v10", "v14", "v21", "v34");   // acc = w bank (2)
  else if (KIND == 21) XLOOP(XB("v10", "v14", "v22", "v34"), "v10", "v14", "v22", "v34");   // all bank 2
  else if (KIND == 22) XLOOP(XBP("v10", "v14", "v22", "v34"), "v10", "v14", "v22", "v34");  // plain fmac, all bank 2
  else if (KIND == 23) XLOOP(XBP("v10", "v11", "v21", "v32"), "v10", "v11", "v21", "v32");  // plain fmac, distinct
}

template <int KIND>
__global__ void k_xprobe(const float* in, unsigned long long* cyc, float* out, int active_waves) {
  const int wave = threadIdx.x >> 6;
  float a = in[threadIdx.x & 63];
  const float x = in[64 + (threadIdx.x & 63)], w = 0.999f;
  if (wave < active_waves) {
    __builtin_amdgcn_s_barrier();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    xbody<KIND>(a, x, w);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
      cyc[(blockIdx.x * 16 + wave) * 2] = t1 - t0;
      cyc[(blockIdx.x * 16 + wave) * 2 + 1] = r1 - r0;
    }
  } else {
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

template <int KIND>
__global__ void k_probe(const float* in, unsigned long long* cyc, float* out, int active_waves) {
  // cyc[(block * 16 + wave) * 2 + {0, 1}] = (d s_memtime, d s_memrealtime)
  const int wave = threadIdx.x >> 6;
  float a = in[threadIdx.x & 63], b = a + 1.f, c = a + 2.f, d = a + 3.f;
  const float x = in[64 + (threadIdx.x & 63)], w = 0.999f;
  if (wave < active_waves) {
    __builtin_amdgcn_s_barrier();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < REP; ++i) body<KIND>(a, b, c, d, x, w);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
      cyc[(blockIdx.x * 16 + wave) * 2] = t1 - t0;
      cyc[(blockIdx.x * 16 + wave) * 2 + 1] = r1 - r0;
    }
  } else {
    __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

extern "C" int probe_run(int kind, int threads, int active, const float* in, unsigned long long* cyc, float* out,
                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (kind) {
    case 0: hipLaunchKernelGGL(k_probe<0>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 1: hipLaunchKernelGGL(k_probe<1>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 2: hipLaunchKernelGGL(k_probe<2>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 3: hipLaunchKernelGGL(k_probe<3>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 4: hipLaunchKernelGGL(k_probe<4>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 5: hipLaunchKernelGGL(k_probe<5>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 6: hipLaunchKernelGGL(k_probe<6>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 7: hipLaunchKernelGGL(k_probe<7>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 8: hipLaunchKernelGGL(k_probe<8>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 9: hipLaunchKernelGGL(k_probe<9>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 10: hipLaunchKernelGGL(k_probe<10>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 11: hipLaunchKernelGGL(k_probe<11>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 12: hipLaunchKernelGGL(k_probe<12>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 13: hipLaunchKernelGGL(k_probe<13>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 14: hipLaunchKernelGGL(k_probe<14>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 15: hipLaunchKernelGGL(k_probe<15>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 16: hipLaunchKernelGGL(k_probe<16>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 17: hipLaunchKernelGGL(k_xprobe<17>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 18: hipLaunchKernelGGL(k_xprobe<18>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 19: hipLaunchKernelGGL(k_xprobe<19>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 20: hipLaunchKernelGGL(k_xprobe<20>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 21: hipLaunchKernelGGL(k_xprobe<21>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 22: hipLaunchKernelGGL(k_xprobe<22>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    case 23: hipLaunchKernelGGL(k_xprobe<23>, dim3(256), dim3(threads), 0, s, in, cyc, out, active); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
