// Slab layout probe (round 6): does the FC_small gradient slab reduce read faster when the 256 workgroups' partials
// of one output chunk are contiguous? Two layouts of the same 256 x S floats (S = 32 blocks x 2560):
//   0 = workgroup-major  slab[w][i]                          (k_backward today: each workgroup's slab contiguous)
//   1 = chunk-major      slab[i / 64][w][i % 64]             (64-float pieces of every workgroup side by side)
// k_fill writes the slab the way the backward's helpers do (16-B write-through stores, 1 KB per wave instruction);
// k_red sums over w with k_red_gx's shape (8 groups x 32 float4, 16 loads in flight per lane, fixed order).
// Built and driven by tools/slab_layout_probe.py; timing only.
#include <hip/hip_runtime.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr int NW = 256, CH = 64, RG = 8, RO4 = 32, RT = 16;

__device__ __forceinline__ long long addr(int layout, int w, long long i, long long S) {
  return layout == 0 ? (long long)w * S + i : (i / CH) * (NW * CH) + (long long)w * CH + (i % CH);
}

__global__ __launch_bounds__(256) void k_fill(float* slab, long long S, int layout) {
  const int w = blockIdx.y;
  for (long long i4 = (long long)blockIdx.x * 256 + threadIdx.x; i4 < S / 4; i4 += (long long)gridDim.x * 256) {
    const long long i = 4 * i4;
    const floatx4 v = {(float)(w & 7), 1.f, 0.5f, (float)(i & 3)};
    floatx4* p = reinterpret_cast<floatx4*>(slab + addr(layout, w, i, S));
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v));
  }
}

__global__ __launch_bounds__(256) void k_red(const float* slab, long long S, int layout, float* out) {
  __shared__ floatx4 part[RG][RO4];
  const int g = threadIdx.x / RO4, o4 = threadIdx.x % RO4;
  const long long i = ((long long)blockIdx.x * RO4 + o4) * 4;
  const bool live = i < S;
  const long long ic = live ? i : 0;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  int w = g;
  for (; w + RG * (RT - 1) < NW; w += RG * RT) {
    floatx4 v[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) v[t] = *reinterpret_cast<const floatx4*>(slab + addr(layout, w + RG * t, ic, S));
#pragma unroll
    for (int t = 0; t < RT; ++t) acc += v[t];
  }
  for (; w < NW; w += RG) acc += *reinterpret_cast<const floatx4*>(slab + addr(layout, w, ic, S));
  part[g][o4] = acc;
  __syncthreads();
  if (g != 0 || !live) return;
  floatx4 tot = part[0][o4];
#pragma unroll
  for (int q = 1; q < RG; ++q) tot += part[q][o4];
  *reinterpret_cast<floatx4*>(out + i) = tot;
}

extern "C" int probe_slab(int layout, int what, float* slab, long long S, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (what == 0)
    hipLaunchKernelGGL(k_fill, dim3(8, NW), dim3(256), 0, st, slab, S, layout);
  else
    hipLaunchKernelGGL(k_red, dim3((unsigned)((S / 4 + RO4 - 1) / RO4)), dim3(256), 0, st, slab, S, layout, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
