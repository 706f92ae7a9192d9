// Heads training forward kernel (its own translation unit: the PF schedule of chunk_mma is slow to compile) (the shared heads machinery: mlp_core.h).
#include "mlp_core.h"

int mli_launch_rgb_fwd_train(const mli_rgb_fwd_args* a, hipStream_t s) {
  hipLaunchKernelGGL((rgb_fwd_kernel<true, false>), dim3(a->R * a->N / GFwd::SAMPLES), dim3(GFwd::THREADS), GFwd::LDS_FWD, s, *a);
  MLI_LAUNCH_CHECK();
}
