// Probe: DPP row_ror / row_newbcast / permlane semantics on gfx950 and ctypes+torch runtime interop.
#include <hip/hip_runtime.h>
__global__ void probe(const float* in, float* out) {
  int l = threadIdx.x;
  float v = in[l];
  out[0*64 + l] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  out[1*64 + l] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x12F, 0xf, 0xf, false));
  out[2*64 + l] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x153, 0xf, 0xf, false));
  out[3*64 + l] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false));
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  out[4*64 + l] = __int_as_float(p[0]);
  out[5*64 + l] = __int_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  out[6*64 + l] = __int_as_float(q[0]);
  out[7*64 + l] = __int_as_float(q[1]);
  float acc = 0.f;
  asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_ror:3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(1.0f));
  out[8*64 + l] = acc;
}
extern "C" int probe_launch(const float* in, float* out, void* stream) {
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, (hipStream_t)stream, in, out);
  return (int)hipGetLastError();
}
