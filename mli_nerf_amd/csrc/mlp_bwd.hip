// Heads backward dX chain (the shared heads machinery: mlp_core.h).
#include "mlp_core.h"

namespace {

__global__ __launch_bounds__(GBwd::THREADS) void rgb_bwd_kernel(mli_rgb_bwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= GBwd::NW / 2) rgb_bwd_body<GBwd, STORE>(a, lds);
  else rgb_bwd_body<GBwd, DMA>(a, lds);
}


}  // namespace

extern "C" int mli_rgb_bwd(const mli_rgb_bwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S % 256 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rgb_bwd_kernel, dim3(S / GBwd::SAMPLES), dim3(GBwd::THREADS), GBwd::LDS_BWD, (hipStream_t)s,
                     *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_rgb_bwd_workspace(const mli_rgb_bwd_args* a, int64_t* bytes) {
  const int64_t S = (int64_t)a->R * a->N;
  if (S <= 0 || S % 256 != 0) return (int)hipErrorInvalidValue;
  bytes[0] = 3 * 4 * 256 * S * 2;  // dzT
  bytes[1] = 3 * S * 16 * 2;       // dz4T (one-k-step fragment images)
  return 0;
}

