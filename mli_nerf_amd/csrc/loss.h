// Stage-b loss arithmetic shared by the three-launch mli_stage_b_loss (loss.hip) and the fused
// composite + loss + composite-backward launch mli_composite_loss (rays.hip): one definition, so
// both produce the same gradients bit for bit.  Formulas and citations: loss.hip.
#pragma once
#include "common.h"

namespace mli_loss {

constexpr int ACC_N = 8;  // render_l1, mse, eik, curv, intr_r, intr_s, re_neg, re_pos

MLI_FI float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// rescale(x, lo, hi) = lo + (x - min) / clamp(max - min, 1e-6) * (hi - lo)
MLI_FI float rescale(float x, float mn, float mx, float lo, float hi) {
  return lo + (x - mn) / fmaxf(mx - mn, 1e-6f) * (hi - lo);
}

// Per-ray terms of ray r (adds into acc[0, 1, 4..7]) and d total / d (rgb, o_r, o_s, o_re).
// mm = min/max of sha and cert over the batch (read only when the intrinsic weight is on).
MLI_FI void ray_terms(const mli_loss_args& a, int r, const float* mm, const float* rgb, const float* o_r, float o_s,
                      const float* o_re, float* acc, float* d_rgb, float* d_o_r, float& d_o_s, float* d_o_re) {
  const int R = a.R;
  const float inv3r = 1.0f / (3.0f * R), invr = 1.0f / R;
  // render: 3 * mean |rgb - gt|; d/drgb = w * 3 * sgn / (3R); mse for PSNR
  for (int i = 0; i < 3; ++i) {
    const float d = rgb[i] - a.gt[3 * r + i];
    acc[0] += fabsf(d);
    acc[1] += d * d;
    d_rgb[i] = a.w_render * 3.0f * sgn(d) * inv3r;
  }
  // intrinsic
  float w_sha = 0.f, w_ref = 0.f;
  if (a.w_intrinsic != 0.f) {
    w_sha = rescale(a.sha[r], mm[0], mm[1], a.range_sha_lo, a.range_sha_hi);
    const float w_vis = rescale(a.cert[r], mm[2], mm[3], a.range_vis_lo, a.range_vis_hi);
    w_ref = fminf(w_vis, w_sha);
  }
  for (int i = 0; i < 3; ++i) {
    const float d = o_r[i] - (a.ref ? a.ref[3 * r + i] : 0.f);
    acc[4] += fabsf(d) * w_ref;
    d_o_r[i] = a.w_intrinsic * a.f_ref * sgn(d) * w_ref * inv3r;
  }
  {
    const float d = o_s - (a.sha ? a.sha[r] : 0.f);
    acc[5] += fabsf(d) * w_sha;
    d_o_s = a.w_intrinsic * a.f_sha * sgn(d) * w_sha * invr;
  }
  // regularize_re
  for (int i = 0; i < 3; ++i) {
    const float x = o_re[i];
    float g;
    if (x < 0.f) {
      acc[6] += -x;
      g = -a.f_neg;
    } else {
      acc[7] += powf(x, a.e_pos);
      g = a.f_pos * a.e_pos * powf(x, a.e_pos - 1.0f);
    }
    d_o_re[i] = a.w_re * g * inv3r;
  }
}

// eikonal / curvature terms of sample s (adds into acc[2], acc[3]); the caller skips outside rays
MLI_FI void sample_terms(const mli_loss_args& a, size_t s, float* acc) {
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

// The loss values from the summed accumulators: losses[8] = render, eikonal, curvature,
// intrinsic, regularize_re, total, psnr, mse.
MLI_FI void finalize(const mli_loss_args& a, const float* acc) {
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

// min/max of sha and cert over the R rays, by every thread of a block of NT threads; the result
// lands in mm[4] (LDS) for the whole block.  red: LDS [4][NT / 64].
template <int NT>
MLI_FI void block_minmax(const mli_loss_args& a, float* red, float* mm) {
  float mn_s = INFINITY, mx_s = -INFINITY, mn_c = INFINITY, mx_c = -INFINITY;
  for (int r = threadIdx.x; r < a.R; r += NT) {
    if (a.sha) { const float v = a.sha[r]; mn_s = fminf(mn_s, v); mx_s = fmaxf(mx_s, v); }
    if (a.cert) { const float v = a.cert[r]; mn_c = fminf(mn_c, v); mx_c = fmaxf(mx_c, v); }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn_s = fminf(mn_s, __shfl_xor(mn_s, o)); mx_s = fmaxf(mx_s, __shfl_xor(mx_s, o));
    mn_c = fminf(mn_c, __shfl_xor(mn_c, o)); mx_c = fmaxf(mx_c, __shfl_xor(mx_c, o));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NWV = NT / 64;
  if (lane == 0) {
    red[0 * NWV + wave] = mn_s; red[1 * NWV + wave] = mx_s;
    red[2 * NWV + wave] = mn_c; red[3 * NWV + wave] = mx_c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NWV; ++w) {
      mn_s = fminf(mn_s, red[0 * NWV + w]); mx_s = fmaxf(mx_s, red[1 * NWV + w]);
      mn_c = fminf(mn_c, red[2 * NWV + w]); mx_c = fmaxf(mx_c, red[3 * NWV + w]);
    }
    mm[0] = mn_s; mm[1] = mx_s; mm[2] = mn_c; mm[3] = mx_c;
  }
  __syncthreads();
}

}  // namespace mli_loss
