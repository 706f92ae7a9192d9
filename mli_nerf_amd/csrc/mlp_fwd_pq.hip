// Heads training forward, PQ mode kernel (its own translation unit: the PF schedule of chunk_mma is slow to compile) (the shared heads machinery: mlp_core.h).
#include "mlp_core.h"

static_assert(GFwdT::LDS_FWD_PQF <= 163840, "LDS per workgroup");

int mli_launch_rgb_fwd_pq(const mli_rgb_fwd_args* a, hipStream_t s) {
  hipLaunchKernelGGL((rgb_fwd_kernel<true, true>), dim3(a->R * a->N / GFwd::SAMPLES), dim3(GFwd::THREADS), GFwdT::LDS_FWD_PQF, s, *a);
  MLI_LAUNCH_CHECK();
}
