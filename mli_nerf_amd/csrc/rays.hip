// Per-ray kernels: ray generation + bounds, coarse / hierarchical sampling, NeuS alpha
// compositing (forward) and its backward into the head outputs.
//
// Per-sample arrays are sample-major [N][R] so that one thread per ray walking its
// samples in order reads coalesced across the wave, and the sequential scans
// (cumprod / cumsum) keep the reference's left-to-right accumulation order.
// Compiled with -ffp-contract=off: products and sums round like the reference's torch ops.
#include "common.h"

namespace {

// --------------------------------------------------------------------------- rays
__global__ __launch_bounds__(256) void rays_kernel(mli_rays_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const int64_t pix = a.ray_idx ? a.ray_idx[r] : a.first_pixel + r;
  const float py = (float)(pix / a.W) + 0.5f;
  const float px = (float)(pix % a.W) + 0.5f;
  const float* K = a.intr_inv;
  const float* T = a.c2w;
  // img2cam: [px, py, 1] @ Kinv^T   (camera.py:259-260)
  float cam[3];
  for (int i = 0; i < 3; ++i) cam[i] = (px * K[3 * i + 0] + py * K[3 * i + 1]) + K[3 * i + 2];
  // cam2world: [cam, 1] @ c2w^T     (camera.py:263-266)
  float world[3], ray[3];
  for (int i = 0; i < 3; ++i) {
    world[i] = ((cam[0] * T[4 * i + 0] + cam[1] * T[4 * i + 1]) + cam[2] * T[4 * i + 2]) + T[4 * i + 3];
    ray[i] = world[i] - T[4 * i + 3];
  }
  const float nrm = sqrtf((ray[0] * ray[0] + ray[1] * ray[1]) + ray[2] * ray[2]);
  const float den = fmaxf(nrm, 1e-12f);  // F.normalize
  float v[3], c[3];
  for (int i = 0; i < 3; ++i) {
    v[i] = ray[i] / den;
    c[i] = T[4 * i + 3];
    a.center[3 * r + i] = c[i];
    a.ray_unit[3 * r + i] = v[i];
    a.pts_light[3 * r + i] = a.c2w_light[4 * i + 3];
  }
  a.ray_norm[r] = nrm;
  float nr, fr;
  bool out;
  if (a.bounding == 0) {  // nerf_util.py:199-205, neuralangelo/model.py:426-429
    const float ctc = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
    const float ctv = (c[0] * v[0] + c[1] * v[1]) + c[2] * v[2];
    const float disc = ctv * ctv - (ctc - 1.0f);
    const float sq = sqrtf(disc);
    const float n0 = -ctv - sq;
    out = isnan(n0);
    nr = out ? 1.0f : fmaxf(n0, 0.0f);
    fr = out ? 1.2f : -ctv + sq;
  } else {  // NeuralLumen/utils/utils.py:86-123
    float tmin = -INFINITY, tmax = INFINITY;
    for (int i = 0; i < 3; ++i) {
      const float t0 = (a.aabb[i] - c[i]) / v[i];
      const float t1 = (a.aabb[3 + i] - c[i]) / v[i];
      tmin = fmaxf(tmin, fminf(t0, t1));
      tmax = fminf(tmax, fmaxf(t0, t1));
    }
    tmin = fminf(fmaxf(tmin, 0.0f), 1e10f);
    tmax = fminf(fmaxf(tmax, 0.0f), 1e10f);
    out = tmax <= tmin;
    nr = out ? 1.0f : tmin;
    fr = out ? 1.2f : tmax;
  }
  a.near_[r] = nr;
  a.far_[r] = fr;
  a.outside[r] = out ? 1 : 0;
}

// --------------------------------------------------------------------------- sampling
__global__ __launch_bounds__(256) void sample_coarse_kernel(mli_sample_coarse_args a) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= a.R * a.Nc) return;
  const int k = gid / a.R, r = gid - k * a.R;
  const float u = a.u ? a.u[(size_t)r * a.Nc + k] : 0.5f;
  const float near = a.near_[r], far = a.far_[r];
  // ((u + k) / Nc) * (far - near) + near   (nerf_util.py:33-37)
  a.dists[gid] = ((u + (float)k) / (float)a.Nc) * (far - near) + near;
}

struct FineArgs {
  mli_sample_fine_args a;
  float u[64];
};

// Section alpha of NeuS sampling (neuralangelo/model.py:467-482), robust cos.
MLI_FI float section_alpha(float d0, float d1, float s0, float s1, float& prev_cos, float inv_s) {
  const float mid = (s0 + s1) * 0.5f;
  float cosv = (s1 - s0) / ((d1 - d0) + 1e-5f);
  cosv = fminf(prev_cos, cosv);
  prev_cos = (s1 - s0) / ((d1 - d0) + 1e-5f);
  const float iv = d1 - d0;
  const float ep = mid - (cosv * iv) * 0.5f;
  const float en = mid + (cosv * iv) * 0.5f;
  const float cp = 1.0f / (1.0f + expf(-(ep * inv_s)));
  const float cn = 1.0f / (1.0f + expf(-(en * inv_s)));
  const float al = (cp - cn) / (cp + 1e-5f);
  return fminf(fmaxf(al, 0.0f), 1.0f);
}

// One thread per ray: merge the two sorted lists (torch.sort of cat, ties irrelevant:
// equal dists are the same point, hence the same sdf), then draw Nf fine dists by the
// section pdf's inverse CDF (nerf_util.py:41-68), walking the cdf once.
__global__ __launch_bounds__(128) void sample_fine_kernel(FineArgs fa) {
  const mli_sample_fine_args& a = fa.a;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const int R = a.R;
  const int Nh = a.Na + a.Nb;
  {
    int i = 0, j = 0;
    for (int o = 0; o < Nh; ++o) {
      const float da = i < a.Na ? a.dists_a[(size_t)i * R + r] : INFINITY;
      const float db = j < a.Nb ? a.dists_b[(size_t)j * R + r] : INFINITY;
      const bool take_a = (j >= a.Nb) || (i < a.Na && da <= db);
      float dv, sv = 0.f;
      if (take_a) {
        dv = da;
        if (a.sdf_out) sv = a.sdf_a[(size_t)i * R + r];
        ++i;
      } else {
        dv = db;
        if (a.sdf_out) sv = a.sdf_b[(size_t)j * R + r];
        ++j;
      }
      a.dists_out[(size_t)o * R + r] = dv;
      if (a.sdf_out) a.sdf_out[(size_t)o * R + r] = sv;
    }
  }
  if (a.Nf == 0) return;
  const float* D = a.dists_out;
  const float* S = a.sdf_out;
  // pass 1: L1 norm of the section weights (F.normalize p=1, eps 1e-12)
  float l1 = 0.f;
  {
    float T = 1.f, pc = 0.f;
    float d0 = D[r], s0 = S[r];
    for (int i = 0; i + 1 < Nh; ++i) {
      const float d1 = D[(size_t)(i + 1) * R + r], s1 = S[(size_t)(i + 1) * R + r];
      const float al = section_alpha(d0, d1, s0, s1, pc, a.inv_s);
      l1 += fabsf(al * T);
      T = T * (1.0f - al);
      d0 = d1; s0 = s1;
    }
  }
  const float den = fmaxf(l1, 1e-12f);
  // pass 2: cdf walk; idx_j = #{k : cdf_k <= u_j} (searchsorted right)
  int j = 0;
  float T = 1.f, pc = 0.f, cdf = 0.f;
  float d0 = D[r], s0 = S[r];
  float cprev = 0.f, dprev = d0;
  // k = 0: cdf_0 = 0 (never > u)
  for (int i = 0; i + 1 < Nh && j < a.Nf; ++i) {
    const float d1 = D[(size_t)(i + 1) * R + r], s1 = S[(size_t)(i + 1) * R + r];
    const float al = section_alpha(d0, d1, s0, s1, pc, a.inv_s);
    const float pdf = (al * T) / den;
    T = T * (1.0f - al);
    cprev = cdf;
    dprev = d0;
    cdf = cdf + pdf;  // cdf_{i+1}
    while (j < a.Nf && cdf > fa.u[j]) {  // idx = i+1: low = i, high = i+1
      const float u = fa.u[j];
      const float t = (u - cprev) / ((cdf - cprev) + 1e-8f);
      a.fine_out[(size_t)j * R + r] = dprev + t * (d1 - dprev);
      ++j;
    }
    d0 = d1; s0 = s1;
  }
  // idx = Nh: low = high = Nh-1 -> the last dist
  const float dl = D[(size_t)(Nh - 1) * R + r];
  for (; j < a.Nf; ++j) a.fine_out[(size_t)j * R + r] = dl + ((fa.u[j] - cdf) / (0.f + 1e-8f)) * (dl - dl);
}

// --------------------------------------------------------------------------- composite
__global__ __launch_bounds__(128) void composite_fwd_kernel(mli_composite_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const int R = a.R, N = a.N;
  const float inv_s = expf(a.s_var[0]);
  const float an = a.anneal;
  const float v0 = a.ray_unit[3 * r], v1 = a.ray_unit[3 * r + 1], v2 = a.ray_unit[3 * r + 2];
  const float far = a.far_[r];
  float T = 1.f;
  float rgb[3] = {0, 0, 0}, orr[3] = {0, 0, 0}, os = 0.f, op = 0.f, gr[3] = {0, 0, 0}, dep = 0.f;
  float dk = a.dists[r];
  for (int k = 0; k < N; ++k) {
    const size_t s = (size_t)k * R + r;
    const float dn = (k + 1 < N) ? a.dists[s + R] : far;
    const float step = dn - dk;
    const float g0 = a.grad[3 * s], g1 = a.grad[3 * s + 1], g2 = a.grad[3 * s + 2];
    const float cosv = (v0 * g0 + v1 * g1) + v2 * g2;
    // _get_iter_cos (neuralangelo/model.py:511-515)
    const float ic = -(fmaxf(-cosv * 0.5f + 0.5f, 0.f) * (1.0f - an) + fmaxf(-cosv, 0.f) * an);
    const float sd = a.sdf[s];
    const float ep = sd - (ic * step) * 0.5f;
    const float en = sd + (ic * step) * 0.5f;
    const float cp = 1.0f / (1.0f + expf(-(ep * inv_s)));
    const float cn = 1.0f / (1.0f + expf(-(en * inv_s)));
    float al = (cp - cn) / (cp + 1e-5f);
    al = fminf(fmaxf(al, 0.f), 1.f);
    const float w = al * T;
    T = T * (1.0f - al);
    a.weights[s] = w;
    const float* y = a.y + 8 * s;
    for (int i = 0; i < 3; ++i) {
      rgb[i] += y[i] * w;
      orr[i] += y[3 + i] * w;
    }
    os += y[6] * w;
    op += w;
    gr[0] += g0 * w; gr[1] += g1 * w; gr[2] += g2 * w;
    dep += dk * w;
    dk = dn;
  }
  if (a.white_bg) {
    for (int i = 0; i < 3; ++i) {
      rgb[i] = rgb[i] + (1.f - op);
      orr[i] = orr[i] + (1.f - op);
    }
    os = os + (1.f - op);
  }
  for (int i = 0; i < 3; ++i) {
    a.rgb[3 * r + i] = rgb[i];
    a.o_r[3 * r + i] = orr[i];
    a.o_re[3 * r + i] = rgb[i] - orr[i] * os;
  }
  a.o_s[r] = os;
  if (a.opacity) a.opacity[r] = op;
  if (a.gradient) for (int i = 0; i < 3; ++i) a.gradient[3 * r + i] = gr[i];
  if (a.depth) a.depth[r] = dep / a.ray_norm[r];
}

__global__ __launch_bounds__(128) void composite_bwd_kernel(mli_composite_bwd_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const int R = a.R, N = a.N;
  float dr[3], dor[3], dos;
  const float os = a.o_s[r];
  float sre = 0.f;
  for (int i = 0; i < 3; ++i) {
    const float dre = a.d_o_re ? a.d_o_re[3 * r + i] : 0.f;
    dr[i] = (a.d_rgb ? a.d_rgb[3 * r + i] : 0.f) + dre;
    dor[i] = (a.d_o_r ? a.d_o_r[3 * r + i] : 0.f) - dre * os;
    sre += dre * a.o_r[3 * r + i];
  }
  dos = (a.d_o_s ? a.d_o_s[r] : 0.f) - sre;
  const float sc = a.grad_scale;
  for (int k = 0; k < N; ++k) {
    const size_t s = (size_t)k * R + r;
    const float w = a.weights[s] * sc;
    const float* y = a.y + 8 * s;
    float* o = a.dz4 + 8 * s;
    for (int i = 0; i < 3; ++i) {
      o[i] = w * dr[i] * (y[i] * (1.f - y[i]));
      o[3 + i] = w * dor[i] * (y[3 + i] * (1.f - y[3 + i]));
    }
    o[6] = w * dos * (y[6] * (1.f - y[6]));
    o[7] = 0.f;
  }
}

}  // namespace

extern "C" int mli_rays(const mli_rays_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  hipLaunchKernelGGL(rays_kernel, dim3((a->R + 255) / 256), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_sample_coarse(const mli_sample_coarse_args* a, mli_stream_t s) {
  const int n = a->R * a->Nc;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sample_coarse_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_sample_fine(const mli_sample_fine_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  if (a->Nf > 64) return (int)hipErrorInvalidValue;
  if (a->Nf > 0 && a->sdf_out == nullptr) return (int)hipErrorInvalidValue;
  FineArgs fa;
  fa.a = *a;
  for (int j = 0; j < 64; ++j) fa.u[j] = (j < a->Nf && a->u_fine) ? a->u_fine[j] : 2.0f;
  hipLaunchKernelGGL(sample_fine_kernel, dim3((a->R + 127) / 128), dim3(128), 0, (hipStream_t)s, fa);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_fwd(const mli_composite_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  hipLaunchKernelGGL(composite_fwd_kernel, dim3((a->R + 127) / 128), dim3(128), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_bwd(const mli_composite_bwd_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  hipLaunchKernelGGL(composite_bwd_kernel, dim3((a->R + 127) / 128), dim3(128), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}
