// Stage-b losses and their gradients w.r.t. the composited outputs, fused.
//
// Replaces _compute_loss (projects/NeuralLumen/trainer.py:133-149) with
//   render     3 * L1(rgb, gt)                                   (trainer.py:135)
//   eikonal    mean((|grad| - 1)^2 * !outside)                   (neuralangelo/utils/misc.py:74-81)
//   curvature  mean(|sum(hess)| * !outside)                      (misc.py:83-90)
//   intrinsic  mean(|o_r - ref| w_ref) + mean(|o_s - sha| w_sha) with w = global min/max
//              rescaled maps, w_ref = min(w_vis, w_sha)          (NeuralLumen/utils/utils.py:142-162)
//   regularize_re  f_neg mean(|min(o_re, 0)|) + f_pos mean(max(o_re, 0)^e)  (utils.py:165-174)
//   total = sum w_k loss_k (imaginaire/trainers/base.py:534-544), PSNR = -10 log10 mse
// and the autograd of total w.r.t. rgb / o_r / o_s / o_re (L1: sign; abs'(0) = 0 as torch),
// which feed mli_composite_bwd.  In stage b eikonal/curvature carry no gradient (frozen SDF).
//
// Three launches: min/max of the pseudo maps (one block), per-element terms + gradients with
// one partial sum per workgroup and accumulator, and a finalize that sums the partials in
// workgroup order (no atomics: values and gradients are bit-reproducible).
//
// scratch layout (floats): [0, 4) min/max of sha and cert, [4, 4 + ACC_N * workgroups) partials.
#include "loss.h"

namespace {

using namespace mli_loss;

MLI_FI float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(1024) void minmax_kernel(mli_loss_args a) {
  __shared__ float red[4 * 16];
  __shared__ float mm[4];
  block_minmax<1024>(a, red, mm);
  if (threadIdx.x < 4) a.scratch[threadIdx.x] = mm[threadIdx.x];
}

// blocks [0, nb_ray) handle rays, the rest the R*N samples (eikonal / curvature)
__global__ __launch_bounds__(256) void terms_kernel(mli_loss_args a, int nb_ray) {
  __shared__ float redw[4];
  const int R = a.R;
  float acc[ACC_N];
#pragma unroll
  for (int i = 0; i < ACC_N; ++i) acc[i] = 0.f;
  if ((int)blockIdx.x < nb_ray) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) {
      float d_rgb[3], d_o_r[3], d_o_s, d_o_re[3];
      ray_terms(a, r, a.scratch, a.rgb + 3 * r, a.o_r + 3 * r, a.o_s[r], a.o_re + 3 * r, acc, d_rgb, d_o_r, d_o_s,
                d_o_re);
      for (int i = 0; i < 3; ++i) {
        a.d_rgb[3 * r + i] = d_rgb[i];
        a.d_o_r[3 * r + i] = d_o_r[i];
        a.d_o_re[3 * r + i] = d_o_re[i];
      }
      a.d_o_s[r] = d_o_s;
    }
  } else {
    const size_t S = (size_t)R * a.N;
    for (size_t s = (size_t)(blockIdx.x - nb_ray) * blockDim.x + threadIdx.x; s < S;
         s += (size_t)(gridDim.x - nb_ray) * blockDim.x) {
      const int r = (int)(s % (size_t)R);
      if (a.outside[r]) continue;
      sample_terms(a, s, acc);
    }
  }
#pragma unroll
  for (int i = 0; i < ACC_N; ++i) {
    const float v = block_sum(acc[i], redw);
    if (threadIdx.x == 0) a.scratch[4 + (size_t)blockIdx.x * ACC_N + i] = v;
  }
}

// thread i sums accumulator i over the workgroups, in workgroup order.  The partials come into
// LDS by one coalesced pass of all threads first (a single thread walking them in global memory
// paid one dependent load per workgroup: 30-125 us per step); the order of the adds is unchanged.
constexpr int FIN_THREADS = 256;
constexpr int FIN_MAX = 1024;  // workgroups whose partials fit the LDS copy (32 KiB)

__global__ __launch_bounds__(FIN_THREADS) void finalize_kernel(mli_loss_args a, int n_blocks) {
  __shared__ float part[FIN_MAX * ACC_N];
  __shared__ float acc[ACC_N];
  const int n = n_blocks * ACC_N;
  const bool staged = n_blocks <= FIN_MAX;
  if (staged)
    for (int e = threadIdx.x; e < n; e += FIN_THREADS) part[e] = a.scratch[4 + e];
  __syncthreads();
  if (threadIdx.x < ACC_N) {
    float t = 0.f;
    if (staged) {
      for (int b = 0; b < n_blocks; ++b) t += part[b * ACC_N + threadIdx.x];
    } else {
      for (int b = 0; b < n_blocks; ++b) t += a.scratch[4 + (size_t)b * ACC_N + threadIdx.x];
    }
    acc[threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) finalize(a, acc);
}

constexpr int NB_SMP = 256;  // workgroups over the R*N samples (eikonal / curvature)
inline int n_blocks(int R) { return (R + 255) / 256 + NB_SMP; }

}  // namespace

extern "C" int mli_stage_b_loss(const mli_loss_args* a, mli_stream_t s) {
  if (a->R <= 0 || a->N <= 0) return (int)hipErrorInvalidValue;
  if (a->w_intrinsic != 0.f && (a->sha == nullptr || a->cert == nullptr || a->ref == nullptr))
    return (int)hipErrorInvalidValue;
  if (a->scratch == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(minmax_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, *a);
  const int nb_ray = (a->R + 255) / 256;
  hipLaunchKernelGGL(terms_kernel, dim3(nb_ray + NB_SMP), dim3(256), 0, (hipStream_t)s, *a, nb_ray);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(FIN_THREADS), 0, (hipStream_t)s, *a, n_blocks(a->R));
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_stage_b_loss_workspace(const mli_loss_args* a, int64_t* bytes) {
  if (a->R <= 0 || a->N <= 0) return (int)hipErrorInvalidValue;
  bytes[0] = (4 + (int64_t)ACC_N * n_blocks(a->R)) * 4;
  bytes[1] = (int64_t)a->R * 3 * 4;
  bytes[2] = (int64_t)a->R * 3 * 4;
  bytes[3] = (int64_t)a->R * 4;
  bytes[4] = (int64_t)a->R * 3 * 4;
  return 0;
}
