// Calibration rank counting on the GPU (psaegert/bcnf src/bcnf/eval/calibration.py:20-48, compute_y_hat_ranks):
//   ranks[i][d] = sum_s [ y_hat[s][i][d] < y[i][d] ]
// over posterior draws y_hat (M x N x D, the (n, N, D) layout of CondRealNVP_v2.sample(outer=True)); the reference
// appends y itself as draw M, which never counts (y < y is false). Counts accumulate (+=) so draws can arrive in
// chunks without ever holding all M x N x D draws. Integer atomics: exact and order-independent (deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bcnf_amd.h"
#include "bcnf_device.h"

namespace {

constexpr int EWG = 256;
constexpr int S_PER_WG = 64;     // draws per workgroup along the draw axis

__global__ __launch_bounds__(EWG) void k_rank_count(const float* __restrict__ yhat, const float* __restrict__ y,
                                                    long long M, long long ND, uint32_t* __restrict__ counts) {
  const long long e = (long long)blockIdx.x * EWG + threadIdx.x;
  if (e >= ND) return;
  const float ref = y[e];
  const long long s0 = (long long)blockIdx.y * S_PER_WG;
  const long long s1 = s0 + S_PER_WG < M ? s0 + S_PER_WG : M;
  uint32_t c = 0;
#pragma unroll 8
  for (long long s = s0; s < s1; ++s) c += yhat[s * ND + e] < ref ? 1u : 0u;
  if (c) atomicAdd(counts + e, c);
}

}  // namespace

extern "C" {

int bcnf_abi_version(void) { return BCNF_AMD_ABI_VERSION; }


int bcnf_rank_count(const float* y_hat, const float* y, int64_t n_draws, int64_t n_rows, int32_t dim, uint32_t* counts,
                    void* stream) {
  if (n_draws < 0 || n_rows < 0 || dim < 1) return BCNF_ERR_ARG;
  if (n_draws == 0 || n_rows == 0) return BCNF_OK;
  if (!y_hat || !y || !counts) return BCNF_ERR_ARG;
  const long long ND = n_rows * (long long)dim;
  dim3 grid((unsigned)((ND + EWG - 1) / EWG), (unsigned)((n_draws + S_PER_WG - 1) / S_PER_WG));
  if (grid.y > 65535) return BCNF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(k_rank_count, grid, dim3(EWG), 0, (hipStream_t)stream, y_hat, y, (long long)n_draws, ND, counts);
  return bcnf_rt::launched();
}

}  // extern "C"
