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
#include "common.h"

namespace {

constexpr int ACC_N = 8;  // render_l1, mse, eik, curv, intr_r, intr_s, re_neg, re_pos

MLI_FI float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

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
  __shared__ float red[4][16];
  float mn_s = INFINITY, mx_s = -INFINITY, mn_c = INFINITY, mx_c = -INFINITY;
  for (int r = threadIdx.x; r < a.R; r += blockDim.x) {
    if (a.sha) { const float v = a.sha[r]; mn_s = fminf(mn_s, v); mx_s = fmaxf(mx_s, v); }
    if (a.cert) { const float v = a.cert[r]; mn_c = fminf(mn_c, v); mx_c = fmaxf(mx_c, v); }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn_s = fminf(mn_s, __shfl_xor(mn_s, o)); mx_s = fmaxf(mx_s, __shfl_xor(mx_s, o));
    mn_c = fminf(mn_c, __shfl_xor(mn_c, o)); mx_c = fmaxf(mx_c, __shfl_xor(mx_c, o));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red[0][wave] = mn_s; red[1][wave] = mx_s; red[2][wave] = mn_c; red[3][wave] = mx_c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      mn_s = fminf(mn_s, red[0][w]); mx_s = fmaxf(mx_s, red[1][w]);
      mn_c = fminf(mn_c, red[2][w]); mx_c = fmaxf(mx_c, red[3][w]);
    }
    a.scratch[0] = mn_s; a.scratch[1] = mx_s;
    a.scratch[2] = mn_c; a.scratch[3] = mx_c;
  }
}

// rescale(x, lo, hi) = lo + (x - min) / clamp(max - min, 1e-6) * (hi - lo)
MLI_FI float rescale(float x, float mn, float mx, float lo, float hi) {
  return lo + (x - mn) / fmaxf(mx - mn, 1e-6f) * (hi - lo);
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
      const float inv3r = 1.0f / (3.0f * R), invr = 1.0f / R;
      // render: 3 * mean |rgb - gt|; d/drgb = w * 3 * sgn / (3R); mse for PSNR
      for (int i = 0; i < 3; ++i) {
        const float d = a.rgb[3 * r + i] - a.gt[3 * r + i];
        acc[0] += fabsf(d);
        acc[1] += d * d;
        float g = a.w_render * 3.0f * sgn(d) * inv3r;
        a.d_rgb[3 * r + i] = g;
      }
      // intrinsic
      float w_sha = 0.f, w_ref = 0.f;
      if (a.w_intrinsic != 0.f) {
        const float* st = a.scratch;
        w_sha = rescale(a.sha[r], st[0], st[1], a.range_sha_lo, a.range_sha_hi);
        const float w_vis = rescale(a.cert[r], st[2], st[3], a.range_vis_lo, a.range_vis_hi);
        w_ref = fminf(w_vis, w_sha);
      }
      for (int i = 0; i < 3; ++i) {
        const float d = a.o_r[3 * r + i] - (a.ref ? a.ref[3 * r + i] : 0.f);
        acc[4] += fabsf(d) * w_ref;
        a.d_o_r[3 * r + i] = a.w_intrinsic * a.f_ref * sgn(d) * w_ref * inv3r;
      }
      {
        const float d = a.o_s[r] - (a.sha ? a.sha[r] : 0.f);
        acc[5] += fabsf(d) * w_sha;
        a.d_o_s[r] = a.w_intrinsic * a.f_sha * sgn(d) * w_sha * invr;
      }
      // regularize_re
      for (int i = 0; i < 3; ++i) {
        const float x = a.o_re[3 * r + i];
        float g;
        if (x < 0.f) {
          acc[6] += -x;
          g = -a.f_neg;
        } else {
          acc[7] += powf(x, a.e_pos);
          g = a.f_pos * a.e_pos * powf(x, a.e_pos - 1.0f);
        }
        a.d_o_re[3 * r + i] = a.w_re * g * inv3r;
      }
    }
  } else {
    const size_t S = (size_t)R * a.N;
    for (size_t s = (size_t)(blockIdx.x - nb_ray) * blockDim.x + threadIdx.x; s < S;
         s += (size_t)(gridDim.x - nb_ray) * blockDim.x) {
      const int r = (int)(s % (size_t)R);
      if (a.outside[r]) continue;
      if (a.grad) {
        const float g0 = a.grad[3 * s], g1 = a.grad[3 * s + 1], g2 = a.grad[3 * s + 2];
        const float n = sqrtf((g0 * g0 + g1 * g1) + g2 * g2);
        const float e = (n - 1.0f) * (n - 1.0f);
        acc[2] += isfinite(e) ? e : 0.f;  // nan_to_num(nan=0, posinf=0, neginf=0)
      }
      if (a.hess) {
        const float l = fabsf((a.hess[3 * s] + a.hess[3 * s + 1]) + a.hess[3 * s + 2]);
        acc[3] += isfinite(l) ? l : 0.f;
      }
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
  if (threadIdx.x != 0) return;
  const float R3 = 3.0f * a.R, SN = (float)a.R * a.N;
  const float render = acc[0] / R3 * 3.0f;
  const float mse = acc[1] / R3;
  const float eik = acc[2] / SN, curv = acc[3] / SN;
  const float intr = acc[4] / R3 * a.f_ref + acc[5] / a.R * a.f_sha;
  const float re = acc[6] / R3 * a.f_neg + acc[7] / R3 * a.f_pos;
  float* o = a.losses;
  o[0] = render; o[1] = eik; o[2] = curv; o[3] = intr; o[4] = re;
  o[5] = a.w_render * render + a.w_eikonal * eik + a.w_curvature * curv + a.w_intrinsic * intr + a.w_re * re;
  o[6] = -10.0f * log10f(mse);
  o[7] = mse;
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
