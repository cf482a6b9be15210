// Issue-rate probe (gfx950): cycles per instruction of the forward chain's instruction kinds, one wave per SIMD
// and two waves per SIMD. Each wave runs REP x a 32-instruction body between two s_memtime stamps; the host
// divides by the instruction count. Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe_issue.hip
//   -o tools/probe_issue.so ; run: python tools/probe_issue.py
#include <hip/hip_runtime.h>
#include <stdint.h>

#define REP 64

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
  } else if (KIND == 4) {   // 32 v_exp_f32 (independent)
    asm volatile(EXP4 EXP4 EXP4 EXP4 EXP4 EXP4 EXP4 EXP4 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(w));
  }
}

template <int KIND>
__global__ void k_probe(const float* in, unsigned long long* cyc, float* out, int active_waves) {
  const int wave = threadIdx.x >> 6;
  float a = in[threadIdx.x & 63], b = a + 1.f, c = a + 2.f, d = a + 3.f;
  const float x = in[64 + (threadIdx.x & 63)], w = 0.999f;
  if (wave < active_waves) {
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < REP; ++i) body<KIND>(a, b, c, d, x, w);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + wave] = t1 - t0;
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
    default: return -1;
  }
  return (int)hipGetLastError();
}
