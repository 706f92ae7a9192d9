// Heads forward: the C entry points and the eval kernel (the shared heads machinery: mlp_core.h).
#include "mlp_core.h"

extern "C" int mli_rgb_fwd(const mli_rgb_fwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S % 256 != 0) return (int)hipErrorInvalidValue;
  const bool train = a->xT != nullptr;
  if (a->feat_frag == nullptr || (train && a->masks == nullptr)) return (int)hipErrorInvalidValue;
  if (a->n_heads != 1 && a->n_heads != 3) return (int)hipErrorInvalidValue;
  // output-layer partials: training only, one ray per 32-sample tile, both pointers or none
  const bool pq = a->weights != nullptr;
  if (pq && (!train || a->q4 == nullptr || a->N % 32 != 0)) return (int)hipErrorInvalidValue;
  if (!pq && a->q4 != nullptr) return (int)hipErrorInvalidValue;
  const dim3 grid(S / GFwd::SAMPLES), block(GFwd::THREADS);
  if (pq) return mli_launch_rgb_fwd_pq(a, (hipStream_t)s);
  if (train) return mli_launch_rgb_fwd_train(a, (hipStream_t)s);
  static_assert(GFwd::LDS_FWD_F <= 163840, "LDS per workgroup");
  hipLaunchKernelGGL((rgb_fwd_kernel<false, false>), grid, block, GFwd::LDS_FWD_F, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_rgb_fwd_workspace(const mli_rgb_fwd_args* a, int64_t* bytes) {
  const int64_t S = (int64_t)a->R * a->N;
  if (S <= 0 || S % 256 != 0 || (a->n_heads != 1 && a->n_heads != 3)) return (int)hipErrorInvalidValue;
  const bool pq = a->weights != nullptr;
  if (pq && a->N % 32 != 0) return (int)hipErrorInvalidValue;
  bytes[0] = S * 8 * 4;                                   // y
  bytes[1] = (int64_t)MLI_HEAD_K0 * S * 2;                // feat_frag = the x0 image (ABI 15)
  bytes[2] = 0;                                           // (x0T: gone, ABI 15)
  bytes[3] = (int64_t)a->n_heads * (pq ? 3 : 4) * 256 * S * 2;  // xT (training)
  bytes[4] = (int64_t)a->n_heads * 4 * (S / 32) * 64 * 16;  // masks (training)
  bytes[5] = pq ? (S / 256) * MLI_Q4_SEGS(a->N) * a->n_heads * 257 * 4 * 4 : 0;  // q4 (PQ)
  return 0;
}

