// Per-ray kernels: ray generation + bounds, coarse / hierarchical sampling, NeuS alpha
// compositing (forward) and its backward into the head outputs.
//
// Per-sample arrays are sample-major [N][R] so that one thread per ray walking its
// samples in order reads coalesced across the wave, and the sequential scans
// (cumprod / cumsum) keep the reference's left-to-right accumulation order.
// Compiled with -ffp-contract=off: products and sums round like the reference's torch ops.
#include "common.h"
#include "loss.h"

namespace {

// --------------------------------------------------------------------------- rays
__global__ __launch_bounds__(256) void rays_kernel(mli_rays_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const int64_t pix = a.ray_idx ? a.ray_idx[r] : a.first_pixel + r;
  const float py = (float)(pix / a.W) + 0.5f;
  const float px = (float)(pix % a.W) + 0.5f;
  // intr.inverse() (camera.py:259) by the adjugate, and Pose.invert (camera.py:46-52):
  // c2w = [R^T | -R^T t], recomputed per thread (a few dozen flops, no host round trip)
  float K[9], T[12], TL[3];
  {
    const float* M = a.intr;
    const float c00 = M[4] * M[8] - M[5] * M[7], c01 = M[5] * M[6] - M[3] * M[8], c02 = M[3] * M[7] - M[4] * M[6];
    const float det = (M[0] * c00 + M[1] * c01) + M[2] * c02;
    const float id = 1.0f / det;
    K[0] = c00 * id; K[1] = (M[2] * M[7] - M[1] * M[8]) * id; K[2] = (M[1] * M[5] - M[2] * M[4]) * id;
    K[3] = c01 * id; K[4] = (M[0] * M[8] - M[2] * M[6]) * id; K[5] = (M[2] * M[3] - M[0] * M[5]) * id;
    K[6] = c02 * id; K[7] = (M[1] * M[6] - M[0] * M[7]) * id; K[8] = (M[0] * M[4] - M[1] * M[3]) * id;
    const float* P = a.pose;  // w2c [R | t]
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) T[4 * i + j] = P[4 * j + i];
      T[4 * i + 3] = -((P[4 * 0 + i] * P[3] + P[4 * 1 + i] * P[7]) + P[4 * 2 + i] * P[11]);
    }
    const float* Q = a.pose_light;
    for (int i = 0; i < 3; ++i) TL[i] = -((Q[4 * 0 + i] * Q[3] + Q[4 * 1 + i] * Q[7]) + Q[4 * 2 + i] * Q[11]);
  }
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
    a.pts_light[3 * r + i] = TL[i];
  }
  a.ray_norm[r] = nrm;
  float nr, fr;
  bool out;
  ray_bounds(c, v, a.bounding, 1.0f, a.aabb, nr, fr, out);
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

// Wave-level scans over 64 lanes (Hillis-Steele through ds_bpermute).
MLI_FI float wave_excl_prod(float x, int lane) {
  float v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(v, o);
    if (lane >= o) v *= y;
  }
  const float e = __shfl_up(v, 1);
  return lane == 0 ? 1.0f : e;
}
MLI_FI float wave_excl_sum(float x, int lane) {
  float v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  const float e = __shfl_up(v, 1);
  return lane == 0 ? 0.0f : e;
}
MLI_FI float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// One wave per ray (FW rays per block), the ray's lists staged in LDS:
//  1. merge = torch.sort(cat(a, b)) (neuralangelo/model.py:461): every element's output
//     slot is its rank under (dist, list a first, index) -- a upper-bound binary search in
//     the sorted list a for b's elements, a linear count over b (<= 64) for a's -- so the
//     scatter is a permutation even if b is not exactly sorted;
//  2. section alphas (robust cos, model.py:467-482), exclusive transmittance
//     (render.py:87-99) and the L1-normalised pdf / cdf (nerf_util.py:41-57) by wave scans,
//     each lane owning 4 consecutive sections;
//  3. inverse CDF at the midpoint quantiles: searchsorted(cdf, u, right) by binary search
//     (nerf_util.py:58-68), one lane per fine sample.
constexpr int FW = 4;
constexpr int FMAX = 256;  // Na + Nb
constexpr int FBMAX = 64;  // Nb, Nf
__global__ __launch_bounds__(FW * 64) void sample_fine_kernel(FineArgs fa) {
  const mli_sample_fine_args& a = fa.a;
  __shared__ float s_ad[FW][FMAX], s_bd[FW][FBMAX], s_md[FW][FMAX], s_ms[FW][FMAX], s_cd[FW][FMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int R = a.R, Na = a.Na, Nb = a.Nb, Nh = Na + Nb;
  const int r = min((int)(blockIdx.x * FW + w), R - 1);  // tail waves redo the last ray (same values)
  float* ad = s_ad[w];
  float* bd = s_bd[w];
  float* md = s_md[w];
  float* ms = s_ms[w];
  float* cd = s_cd[w];
  const bool with_sdf = a.sdf_out != nullptr;
  // ---- 1. merge
  float av[FMAX / 64], as[FMAX / 64];
#pragma unroll
  for (int e = 0; e < FMAX / 64; ++e) {
    const int i = lane + 64 * e;
    av[e] = i < Na ? a.dists_a[(size_t)i * R + r] : 0.f;
    as[e] = (i < Na && with_sdf) ? a.sdf_a[(size_t)i * R + r] : 0.f;
    if (i < Na) ad[i] = av[e];
  }
  const float bv = lane < Nb ? a.dists_b[(size_t)lane * R + r] : 0.f;
  const float bs = (lane < Nb && with_sdf) ? a.sdf_b[(size_t)lane * R + r] : 0.f;
  if (lane < Nb) bd[lane] = bv;
  __syncthreads();
  int apos[FMAX / 64];
#pragma unroll
  for (int e = 0; e < FMAX / 64; ++e) apos[e] = lane + 64 * e;
  int bpos = 0;
  for (int j = 0; j < Nb; ++j) {
    const float y = bd[j];
#pragma unroll
    for (int e = 0; e < FMAX / 64; ++e) apos[e] += (y < av[e]) ? 1 : 0;
    bpos += (y < bv || (y == bv && j < lane)) ? 1 : 0;
  }
  if (lane < Nb) {  // + #{i : a_i <= bv}
    int lo = 0, hi = Na;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ad[mid] <= bv) lo = mid + 1; else hi = mid;
    }
    bpos += lo;
  }
  const bool store = blockIdx.x * FW + w < R;
#pragma unroll
  for (int e = 0; e < FMAX / 64; ++e) {
    if (lane + 64 * e < Na) {
      md[apos[e]] = av[e];
      ms[apos[e]] = as[e];
    }
  }
  if (lane < Nb) {
    md[bpos] = bv;
    ms[bpos] = bs;
  }
  __syncthreads();
  for (int i = lane; i < Nh; i += 64) {
    if (store) {
      a.dists_out[(size_t)i * R + r] = md[i];
      if (with_sdf) a.sdf_out[(size_t)i * R + r] = ms[i];
    }
  }
  if (a.Nf == 0) return;
  // ---- 2. sections i = 4*lane + e (i + 1 < Nh)
  constexpr int E = FMAX / 64;
  float al[E], q[E];
  {
    const int i0 = E * lane;
    float prev_raw = 0.f;
    if (i0 >= 1 && i0 < Nh) {
      const float dm = md[i0 - 1], sm = ms[i0 - 1];
      prev_raw = (ms[i0] - sm) / ((md[i0] - dm) + 1e-5f);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = i0 + e;
      al[e] = 0.f;
      if (i + 1 < Nh) {
        float pc = prev_raw;
        al[e] = section_alpha(md[i], md[i + 1], ms[i], ms[i + 1], pc, a.inv_s);
        prev_raw = pc;
      }
      q[e] = 1.0f - al[e];
    }
  }
  float lp = 1.f;
#pragma unroll
  for (int e = 0; e < E; ++e) lp *= q[e];
  float T = wave_excl_prod(lp, lane);
  float wv[E], l1 = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    wv[e] = al[e] * T;
    T = T * q[e];
    l1 += fabsf(wv[e]);
  }
  const float den = fmaxf(wave_sum(l1), 1e-12f);
  float c[E], run = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    run += wv[e] / den;
    c[e] = run;
  }
  const float base = wave_excl_sum(run, lane);
  if (lane == 0) cd[0] = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (E * lane + e + 1 < Nh) cd[E * lane + e + 1] = base + c[e];
  __syncthreads();
  // ---- 3. inverse CDF, lane j -> fine sample j
  if (lane < a.Nf && store) {
    const float u = fa.u[lane];
    int lo = 0, hi = Nh;  // idx = #{k : cdf_k <= u}
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cd[mid] <= u) lo = mid + 1; else hi = mid;
    }
    const int i_lo = max(lo - 1, 0), i_hi = min(lo, Nh - 1);
    const float d0 = md[i_lo], d1 = md[i_hi], c0 = cd[i_lo], c1 = cd[i_hi];
    const float t = (u - c0) / ((c1 - c0) + 1e-8f);
    a.fine_out[(size_t)lane * R + r] = d0 + t * (d1 - d0);
  }
}

// --------------------------------------------------------------------------- composite
// One wave per ray, lane l owning samples 4l..4l+3 (N <= 256): NeuS alphas
// (neuralangelo/model.py:492-515), exclusive transmittance by a wave product scan
// (render.py:87-99), the composited sums by wave reductions (NeuralLumen/model.py:266-305).
constexpr int CW = 4;  // rays per block
constexpr int CE = 4;  // samples per lane

// Scans / sums over the L lanes of one ray (L = 64: the whole wave; L = 32: two rays per wave).
// For a ray of N <= 32 * CE samples the L = 32 forms give bit-identical results to L = 64: the
// lanes 32..63 of a 64-lane ray hold the identities (1 for the product, 0 for the sums), and
// every step the lanes below 32 take is the same in both.
template <int L>
MLI_FI float seg_excl_prod(float x, int sub) {
  float v = x;
#pragma unroll
  for (int o = 1; o < L; o <<= 1) {
    const float y = __shfl_up(v, o, L);
    if (sub >= o) v *= y;
  }
  const float e = __shfl_up(v, 1, L);
  return sub == 0 ? 1.0f : e;
}
template <int L>
MLI_FI float seg_sum0(float x) {  // the segment's sum as its lane 0 forms it, in every lane
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, L);
  return __shfl(x, 0, L);
}

// The ray's NeuS alphas, weights (stored) and the reduced composited sums acc[12] (rgb 3, o_r 3,
// o_s, opacity, gradient 3, sum w d), every lane of the ray holding its lane 0's values; the ray
// owns L lanes, lane `sub` of them samples CE*sub .. CE*sub + CE-1.
// yk: the head outputs each lane read for its samples (kept for the fused backward).
template <int L>
MLI_FI void composite_ray(const mli_composite_args& a, int r, int lane, float (&wv)[CE], float (&yk)[CE][7],
                          float (&acc)[12]) {
  const int R = a.R, N = a.N;
  const float inv_s = expf(a.s_var[0]);
  const float an = a.anneal;
  const float v0 = a.ray_unit[3 * r], v1 = a.ray_unit[3 * r + 1], v2 = a.ray_unit[3 * r + 2];
  const float far = a.far_[r];
  float al[CE], dk[CE], g[CE][3];
  float lp = 1.f;
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const int k = CE * lane + e;
    al[e] = 0.f; dk[e] = 0.f; g[e][0] = g[e][1] = g[e][2] = 0.f;
    if (k < N) {
      const size_t s = (size_t)k * R + r;
      dk[e] = a.dists[s];
      const float dn = (k + 1 < N) ? a.dists[s + R] : far;
      const float step = dn - dk[e];
      g[e][0] = a.grad[3 * s]; g[e][1] = a.grad[3 * s + 1]; g[e][2] = a.grad[3 * s + 2];
      const float cosv = (v0 * g[e][0] + v1 * g[e][1]) + v2 * g[e][2];
      // _get_iter_cos (neuralangelo/model.py:511-515)
      const float ic = -(fmaxf(-cosv * 0.5f + 0.5f, 0.f) * (1.0f - an) + fmaxf(-cosv, 0.f) * an);
      const float sd = a.sdf[s];
      const float ep = sd - (ic * step) * 0.5f;
      const float en = sd + (ic * step) * 0.5f;
      const float cp = 1.0f / (1.0f + expf(-(ep * inv_s)));
      const float cn = 1.0f / (1.0f + expf(-(en * inv_s)));
      const float x = (cp - cn) / (cp + 1e-5f);
      al[e] = fminf(fmaxf(x, 0.f), 1.f);
    }
    lp *= 1.0f - al[e];
  }
  float T = seg_excl_prod<L>(lp, lane);
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = 0.f;
#pragma unroll
  for (int e = 0; e < CE; ++e) {
    const int k = CE * lane + e;
    wv[e] = al[e] * T;
    T = T * (1.0f - al[e]);
#pragma unroll
    for (int i = 0; i < 7; ++i) yk[e][i] = 0.f;
    if (k < N) {
      const size_t s = (size_t)k * R + r;
      a.weights[s] = wv[e];
      if (a.y == nullptr) continue;  // weights only (mli_composite_fwd, PQ heads)
      const f32x4 y0 = *reinterpret_cast<const f32x4*>(a.y + 8 * s);
      const f32x4 y1 = *reinterpret_cast<const f32x4*>(a.y + 8 * s + 4);
      yk[e][0] = y0[0]; yk[e][1] = y0[1]; yk[e][2] = y0[2]; yk[e][3] = y0[3];
      yk[e][4] = y1[0]; yk[e][5] = y1[1]; yk[e][6] = y1[2];
      acc[0] += y0[0] * wv[e]; acc[1] += y0[1] * wv[e]; acc[2] += y0[2] * wv[e];
      acc[3] += y0[3] * wv[e]; acc[4] += y1[0] * wv[e]; acc[5] += y1[1] * wv[e];
      acc[6] += y1[2] * wv[e];
      acc[7] += wv[e];
      acc[8] += g[e][0] * wv[e]; acc[9] += g[e][1] * wv[e]; acc[10] += g[e][2] * wv[e];
      acc[11] += dk[e] * wv[e];
    }
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = seg_sum0<L>(acc[i]);
}

// Composited outputs with the white background and o_re (NeuralLumen/model.py:266-305).
MLI_FI void composite_outputs(const mli_composite_args& a, const float (&acc)[12], float (&rgb)[3], float (&orr)[3],
                              float& os, float (&ore)[3]) {
  rgb[0] = acc[0]; rgb[1] = acc[1]; rgb[2] = acc[2];
  orr[0] = acc[3]; orr[1] = acc[4]; orr[2] = acc[5];
  os = acc[6];
  const float op = acc[7];
  if (a.white_bg) {
    for (int i = 0; i < 3; ++i) {
      rgb[i] = rgb[i] + (1.f - op);
      orr[i] = orr[i] + (1.f - op);
    }
    os = os + (1.f - op);
  }
  for (int i = 0; i < 3; ++i) ore[i] = rgb[i] - orr[i] * os;
}

// L lanes per ray: 64 / L rays per wave, CW waves per block
template <int L>
__global__ __launch_bounds__(CW * 64) void composite_fwd_kernel(mli_composite_args a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane % L;
  const int r = (blockIdx.x * CW + w) * (64 / L) + lane / L;
  if (r >= a.R) return;  // the ray's lanes exit together (no block barriers below)
  float wv[CE], yk[CE][7], acc[12];
  composite_ray<L>(a, r, sub, wv, yk, acc);
  if (sub != 0 || a.y == nullptr) return;
  float rgb[3], orr[3], os, ore[3];
  composite_outputs(a, acc, rgb, orr, os, ore);
  for (int i = 0; i < 3; ++i) {
    a.rgb[3 * r + i] = rgb[i];
    a.o_r[3 * r + i] = orr[i];
    a.o_re[3 * r + i] = ore[i];
  }
  a.o_s[r] = os;
  if (a.opacity) a.opacity[r] = acc[7];
  if (a.gradient) for (int i = 0; i < 3; ++i) a.gradient[3 * r + i] = acc[8 + i];
  if (a.depth) a.depth[r] = acc[11] / a.ray_norm[r];
  if (a.blend_dist) a.blend_dist[r] = acc[11];  // render.composite(dists, weights)
}

// d total / d (rgb, o_r, o_s, o_re) of one ray -> d total / d composited rgb, o_r, o_s once the
// o_re = rgb - o_r * o_s chain is folded in (NeuralLumen/model.py:305): the per-ray factor D of
// every sample's pre-sigmoid gradient (written as `dray` for mli_dw4).
MLI_FI void ray_dz(const float (&dr_in)[3], const float (&dor_in)[3], float d_o_s, const float (&d_o_re)[3],
                   const float (&orr)[3], float os, float (&D)[7]) {
  float sre = 0.f;
  for (int i = 0; i < 3; ++i) {
    const float dre = d_o_re[i];
    D[i] = dr_in[i] + dre;
    D[3 + i] = dor_in[i] - dre * os;
    sre += dre * orr[i];
  }
  D[6] = d_o_s - sre;
}

// The per-sample pre-sigmoid gradients (scaled) of a ray's samples from its D: the composite +
// sigmoid backward (one definition for both paths).
MLI_FI void composite_bwd_sample(const float (&D)[7], float w, const float (&y)[7], f32x4& o0, f32x4& o1) {
  o0[0] = w * D[0] * (y[0] * (1.f - y[0]));
  o0[1] = w * D[1] * (y[1] * (1.f - y[1]));
  o0[2] = w * D[2] * (y[2] * (1.f - y[2]));
  o0[3] = w * D[3] * (y[3] * (1.f - y[3]));
  o1[0] = w * D[4] * (y[4] * (1.f - y[4]));
  o1[1] = w * D[5] * (y[5] * (1.f - y[5]));
  o1[2] = w * D[6] * (y[6] * (1.f - y[6]));
  o1[3] = 0.f;
}

MLI_FI void store_dray(float* dray, int r, const float (&D)[7]) {
  *reinterpret_cast<f32x4*>(dray + 8 * r) = f32x4{D[0], D[1], D[2], D[3]};
  *reinterpret_cast<f32x4*>(dray + 8 * r + 4) = f32x4{D[4], D[5], D[6], 0.f};
}

// Fused stage-b training tail, one wave per ray: composite (as composite_fwd_kernel), the loss
// terms and d total / d outputs of the ray (mli_loss::ray_terms, as terms_kernel), its samples'
// eikonal / curvature terms, and the composite backward of its samples (as composite_bwd_kernel)
// -- the composited outputs and the loss gradients never leave registers.  Loss values: one
// partial sum per workgroup and accumulator; composite_loss_finalize adds them up.  (A
// last-workgroup-done counter in this kernel instead cost 80 us per launch: each workgroup's
// agent-scope release writes back its XCD's whole L2.)
template <int LN>
__global__ __launch_bounds__(CW * 64) void composite_loss_kernel(mli_composite_loss_args A) {
  using namespace mli_loss;
  const mli_composite_args& a = A.comp;
  const mli_loss_args& L = A.loss;
  __shared__ float red[4 * CW], mm[4], part[CW][ACC_N];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (L.w_intrinsic != 0.f) block_minmax<CW * 64>(L, red, mm);
  const int R = a.R, N = a.N;
  const int sub = lane % LN;
  const int r = (blockIdx.x * CW + w) * (64 / LN) + lane / LN;
  float acc[ACC_N];
#pragma unroll
  for (int i = 0; i < ACC_N; ++i) acc[i] = 0.f;
  if (r < R) {
    float wv[CE], yk[CE][7], cs[12];
    composite_ray<LN>(a, r, sub, wv, yk, cs);
    float rgb[3], orr[3], os, ore[3];
    composite_outputs(a, cs, rgb, orr, os, ore);
    if (sub == 0) {
      for (int i = 0; i < 3; ++i) {
        a.rgb[3 * r + i] = rgb[i];
        a.o_r[3 * r + i] = orr[i];
        a.o_re[3 * r + i] = ore[i];
      }
      a.o_s[r] = os;
    }
    // every lane forms the ray's gradients (same inputs, same arithmetic); lane 0 counts its terms
    float ra[ACC_N] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float d_rgb[3], d_o_r[3], d_o_s, d_o_re[3];
    ray_terms(L, r, mm, rgb, orr, os, ore, ra, d_rgb, d_o_r, d_o_s, d_o_re);
    if (sub == 0) {
      acc[0] = ra[0]; acc[1] = ra[1]; acc[4] = ra[4]; acc[5] = ra[5]; acc[6] = ra[6]; acc[7] = ra[7];
    }
    const bool outside = L.outside[r] != 0;
    float D[7];
    ray_dz(d_rgb, d_o_r, d_o_s, d_o_re, orr, os, D);
    if (A.dray && sub == 0) store_dray(A.dray, r, D);
#pragma unroll
    for (int e = 0; e < CE; ++e) {
      const int k = CE * sub + e;
      if (k < N) {
        const size_t s = (size_t)k * R + r;
        if (!outside) sample_terms(L, s, acc);
        f32x4 o0, o1;
        composite_bwd_sample(D, wv[e] * A.grad_scale, yk[e], o0, o1);
        *reinterpret_cast<f32x4*>(A.dz4 + 8 * s) = o0;
        *reinterpret_cast<f32x4*>(A.dz4 + 8 * s + 4) = o1;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < ACC_N; ++i) acc[i] = wave_sum(acc[i]);  // the wave's rays and samples
  if (lane == 0)
    for (int i = 0; i < ACC_N; ++i) part[w][i] = acc[i];
  __syncthreads();
  if (threadIdx.x < ACC_N) {
    float t = 0.f;
    for (int v = 0; v < CW; ++v) t += part[v][threadIdx.x];
    L.scratch[(size_t)blockIdx.x * ACC_N + threadIdx.x] = t;
  }
}

// The loss values from the workgroup partials: accumulator i = threadIdx.x / 32; lane j of its 32
// adds workgroups j, j + 32, ... in order, then a fixed xor tree over the 32 lanes (bit-reproducible).
__global__ __launch_bounds__(256) void composite_loss_finalize(mli_loss_args L, int nb) {
  __shared__ float fin[mli_loss::ACC_N];
  const int i = threadIdx.x >> 5, j = threadIdx.x & 31;
  float t = 0.f;
  int b = j;
  for (; b + 7 * 32 < nb; b += 8 * 32) {  // 8 independent loads in flight, then the adds in order
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = L.scratch[(size_t)(b + 32 * u) * mli_loss::ACC_N + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  for (; b < nb; b += 32) t += L.scratch[(size_t)b * mli_loss::ACC_N + i];
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) t += __shfl_xor(t, o);
  if (j == 0) fin[i] = t;
  __syncthreads();
  if (threadIdx.x == 0) mli_loss::finalize(L, fin);
}

// Backward of the composite + heads' output sigmoids: one thread per sample (no scan: the
// gradient w.r.t. y only needs the forward weights), scaled by the power-of-two grad scale.
__global__ __launch_bounds__(256) void composite_bwd_kernel(mli_composite_bwd_args a) {
  const int R = a.R;
  const size_t S = (size_t)R * a.N;
  const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= S) return;
  const int r = (int)(s % (size_t)R);
  float dr[3], dor[3], dre[3], orr[3];
  for (int i = 0; i < 3; ++i) {
    dre[i] = a.d_o_re ? a.d_o_re[3 * r + i] : 0.f;
    dr[i] = a.d_rgb ? a.d_rgb[3 * r + i] : 0.f;
    dor[i] = a.d_o_r ? a.d_o_r[3 * r + i] : 0.f;
    orr[i] = a.o_r[3 * r + i];
  }
  const float dos = a.d_o_s ? a.d_o_s[r] : 0.f;
  const f32x4 y0 = *reinterpret_cast<const f32x4*>(a.y + 8 * s);
  const f32x4 y1 = *reinterpret_cast<const f32x4*>(a.y + 8 * s + 4);
  const float y[7] = {y0[0], y0[1], y0[2], y0[3], y1[0], y1[1], y1[2]};
  float D[7];
  ray_dz(dr, dor, dos, dre, orr, a.o_s[r], D);
  if (a.dray && s < (size_t)R) store_dray(a.dray, r, D);  // sample k = 0 of each ray
  f32x4 o0, o1;
  composite_bwd_sample(D, a.weights[s] * a.grad_scale, y, o0, o1);
  *reinterpret_cast<f32x4*>(a.dz4 + 8 * s) = o0;
  *reinterpret_cast<f32x4*>(a.dz4 + 8 * s + 4) = o1;
}


// Stage-a composite backward (geometry terms), one wave per ray, lane l owning samples
// 4l..4l+3.  The forward alphas are recomputed with the forward kernel's arithmetic; the
// transmittance backward uses the suffix recurrence
//   B_k = sum_{j>k} dw_j a_j prod_{k<m<j} (1 - a_m) = dw_{k+1} a_{k+1} + (1 - a_{k+1}) B_{k+1},
//   d a_k = T_k (dw_k - B_k)
// (division-free, exact where 1 - a = 0), evaluated as a wave suffix scan of affine maps.
// Then clamp (torch: inclusive bounds), the NeuS ratio, the two sigmoids, the section
// endpoints (d sdf, d iter_cos, d inv_s) and _get_iter_cos (relu' = [x > 0]) -> d grad.
__global__ __launch_bounds__(CW * 64) void composite_bwd_geo_kernel(mli_composite_bwd_geo_args a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int R = a.R, N = a.N;
  const int r = blockIdx.x * CW + w;
  if (r >= R) return;
  const float inv_s = expf(a.s_var[0]);
  const float an = a.anneal;
  const float v0 = a.ray_unit[3 * r], v1 = a.ray_unit[3 * r + 1], v2 = a.ray_unit[3 * r + 2];
  const float far = a.far_[r];
  const float dr0 = a.d_rgb[3 * r], dr1 = a.d_rgb[3 * r + 1], dr2 = a.d_rgb[3 * r + 2];
  const float bg = a.white_bg ? (dr0 + dr1) + dr2 : 0.f;  // rgb += 1 - sum(w)
  constexpr int E = 4;
  float al[E], x[E], cp[E], cn[E], ep[E], en[E], st[E], cs[E], dw[E], yv[E][3];
  float lp = 1.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int k = E * lane + e;
    al[e] = 0.f; x[e] = 0.f; cp[e] = cn[e] = 0.5f; ep[e] = en[e] = 0.f; st[e] = 0.f; cs[e] = 0.f; dw[e] = 0.f;
    yv[e][0] = yv[e][1] = yv[e][2] = 0.f;
    if (k < N) {
      const size_t s = (size_t)k * R + r;
      const float dk = a.dists[s];
      const float dn = (k + 1 < N) ? a.dists[s + R] : far;
      st[e] = dn - dk;
      const float g0 = a.grad[3 * s], g1 = a.grad[3 * s + 1], g2 = a.grad[3 * s + 2];
      cs[e] = (v0 * g0 + v1 * g1) + v2 * g2;
      const float ic = -(fmaxf(-cs[e] * 0.5f + 0.5f, 0.f) * (1.0f - an) + fmaxf(-cs[e], 0.f) * an);
      const float sd = a.sdf[s];
      ep[e] = sd - (ic * st[e]) * 0.5f;
      en[e] = sd + (ic * st[e]) * 0.5f;
      cp[e] = 1.0f / (1.0f + expf(-(ep[e] * inv_s)));
      cn[e] = 1.0f / (1.0f + expf(-(en[e] * inv_s)));
      x[e] = (cp[e] - cn[e]) / (cp[e] + 1e-5f);
      al[e] = fminf(fmaxf(x[e], 0.f), 1.f);
      const f32x4 y0 = *reinterpret_cast<const f32x4*>(a.y + 8 * s);
      yv[e][0] = y0[0]; yv[e][1] = y0[1]; yv[e][2] = y0[2];
      dw[e] = ((dr0 * y0[0] + dr1 * y0[1]) + dr2 * y0[2]) - bg;
    }
    lp *= 1.0f - al[e];
  }
  float T[E];
  T[0] = wave_excl_prod(lp, lane);
#pragma unroll
  for (int e = 1; e < E; ++e) T[e] = T[e - 1] * (1.0f - al[e - 1]);
  // this lane's map B_in -> B_{4l-1}: f_{4l} o ... o f_{4l+3}, f_j(x) = (1 - a_j) x + dw_j a_j
  float ma = 1.f, mb = 0.f;
#pragma unroll
  for (int e = E - 1; e >= 0; --e) {
    mb = (1.0f - al[e]) * mb + dw[e] * al[e];
    ma = (1.0f - al[e]) * ma;
  }
  // suffix scan: G_l = F_l o F_{l+1} o ... o F_63
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float na = __shfl_down(ma, o), nb = __shfl_down(mb, o);
    if (lane + o < 64) { mb = ma * nb + mb; ma = ma * na; }
  }
  float B = __shfl_down(mb, 1);
  if (lane == 63) B = 0.f;
  float dinv = 0.f;
#pragma unroll
  for (int e = E - 1; e >= 0; --e) {
    const int k = E * lane + e;
    const float da = T[e] * (dw[e] - B);
    B = (1.0f - al[e]) * B + dw[e] * al[e];
    if (k >= N) continue;
    const size_t s = (size_t)k * R + r;
    const float dx = (x[e] >= 0.f && x[e] <= 1.f) ? da : 0.f;
    const float den_ = cp[e] + 1e-5f;
    const float dcp = dx * (1.0f - x[e]) / den_, dcn = -dx / den_;
    const float dtp = dcp * (cp[e] * (1.0f - cp[e])), dtn = dcn * (cn[e] * (1.0f - cn[e]));
    const float dep = dtp * inv_s, den = dtn * inv_s;
    dinv += dtp * ep[e] + dtn * en[e];
    a.d_sdf[s] = dep + den;
    const float dic = (den - dep) * 0.5f * st[e];
    const float dcos = dic * ((-cs[e] * 0.5f + 0.5f > 0.f ? 0.5f * (1.0f - an) : 0.f) + (-cs[e] > 0.f ? an : 0.f));
    a.d_grad[3 * s] = v0 * dcos;
    a.d_grad[3 * s + 1] = v1 * dcos;
    a.d_grad[3 * s + 2] = v2 * dcos;
    const float wsc = al[e] * T[e] * a.grad_scale;
    f32x4 o0, o1;
    o0[0] = wsc * dr0 * (yv[e][0] * (1.f - yv[e][0]));
    o0[1] = wsc * dr1 * (yv[e][1] * (1.f - yv[e][1]));
    o0[2] = wsc * dr2 * (yv[e][2] * (1.f - yv[e][2]));
    o0[3] = 0.f;
    o1[0] = o1[1] = o1[2] = o1[3] = 0.f;
    *reinterpret_cast<f32x4*>(a.dz4 + 8 * s) = o0;
    *reinterpret_cast<f32x4*>(a.dz4 + 8 * s + 4) = o1;
  }
  dinv = wave_sum(dinv);
  if (lane == 0) a.d_inv_s_part[r] = dinv;
}

// d s_var = exp(s_var) * sum_r d inv_s_r (inv_s = exp(s_var)); the per-ray partials summed in a
// fixed order (strided per thread, then a fixed tree): bit-reproducible
__global__ __launch_bounds__(256) void svar_grad_kernel(mli_composite_bwd_geo_args a) {
  __shared__ float red[256];
  float t = 0.f;
  for (int r = threadIdx.x; r < a.R; r += 256) t += a.d_inv_s_part[r];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.d_s_var[0] = expf(a.s_var[0]) * red[0];
}


// --------------------------------------------------------------------------- ray batch
MLI_FI uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// Bijection of [0, 2^bits) (balanced-ish Feistel, 4 rounds keyed by the seed).
MLI_FI uint64_t feistel(uint64_t x, int bits, uint64_t seed) {
  const int lb = bits >> 1, hb = bits - lb;
  const uint64_t lmask = (1ull << lb) - 1ull, hmask = (1ull << hb) - 1ull;
  uint64_t L = x >> lb, Rr = x & lmask;  // L: hb bits, Rr: lb bits
  for (int k = 0; k < 4; ++k) {
    // alternate which half is mixed so both widths stay valid
    const uint32_t f = mix32((uint32_t)Rr ^ mix32((uint32_t)(seed >> (8 * k)) + 0x9e3779b9u * (k + 1)) ^
                             (uint32_t)(seed >> 32));
    const uint64_t nL = Rr, nR = (L ^ f) & hmask;
    // swap roles: after a round the widths swap, so re-split the combined value
    const uint64_t comb = (nL << hb) | nR;  // lb + hb bits
    L = comb >> lb;
    Rr = comb & lmask;
  }
  return (L << lb) | Rr;
}

__global__ __launch_bounds__(256) void ray_batch_kernel(mli_ray_batch_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  int bits = 1;
  while ((1ll << bits) < a.n_pixels) ++bits;
  uint64_t x = (uint64_t)r;
  do {  // cycle walking: the bijection of [0, 2^bits) restricted to [0, n_pixels)
    x = feistel(x, bits, a.seed);
  } while (x >= (uint64_t)a.n_pixels);
  const int64_t p = (int64_t)x, n = a.n_pixels;
  a.ray_idx[r] = p;
  if (a.image)
    for (int c = 0; c < 3; ++c) a.image_sampled[3 * r + c] = a.image[c * n + p];
  if (a.ref)
    for (int c = 0; c < 3; ++c) a.ref_sampled[3 * r + c] = a.ref[c * n + p];
  if (a.sha) a.sha_sampled[r] = a.sha[p];
  if (a.cert) a.cert_sampled[r] = a.cert[p];
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
  if (a->Nf > FBMAX || a->Nb > FBMAX || a->Na < 1 || a->Na + a->Nb > FMAX) return (int)hipErrorInvalidValue;
  if (a->Nf > 0 && a->sdf_out == nullptr) return (int)hipErrorInvalidValue;
  FineArgs fa;
  fa.a = *a;
  for (int j = 0; j < 64; ++j) fa.u[j] = (j < a->Nf && a->u_fine) ? a->u_fine[j] : 2.0f;
  hipLaunchKernelGGL(sample_fine_kernel, dim3((a->R + FW - 1) / FW), dim3(FW * 64), 0, (hipStream_t)s, fa);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_fwd(const mli_composite_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  if (a->N > 256) return (int)hipErrorInvalidValue;
  if (a->N <= 32 * CE)  // two rays per wave (bit-identical to one, see seg_excl_prod)
    hipLaunchKernelGGL(composite_fwd_kernel<32>, dim3((a->R + 2 * CW - 1) / (2 * CW)), dim3(CW * 64), 0,
                       (hipStream_t)s, *a);
  else
    hipLaunchKernelGGL(composite_fwd_kernel<64>, dim3((a->R + CW - 1) / CW), dim3(CW * 64), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_bwd(const mli_composite_bwd_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  const size_t S = (size_t)a->R * a->N;
  hipLaunchKernelGGL(composite_bwd_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_bwd_geo(const mli_composite_bwd_geo_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  if (a->N > 256) return (int)hipErrorInvalidValue;
  if (a->d_inv_s_part == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(composite_bwd_geo_kernel, dim3((a->R + CW - 1) / CW), dim3(CW * 64), 0, (hipStream_t)s, *a);
  hipLaunchKernelGGL(svar_grad_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_bwd_geo_workspace(const mli_composite_bwd_geo_args* a, int64_t* bytes) {
  if (a->R <= 0 || a->N <= 0) return (int)hipErrorInvalidValue;
  const int64_t S = (int64_t)a->R * a->N;
  bytes[0] = S * 8 * 4;   // dz4
  bytes[1] = S * 4;       // d_sdf
  bytes[2] = S * 3 * 4;   // d_grad
  bytes[3] = (int64_t)a->R * 4;
  return 0;
}

extern "C" int mli_ray_batch(const mli_ray_batch_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  if (a->n_pixels < a->R || a->n_pixels > (1ll << 40) || !a->ray_idx) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ray_batch_kernel, dim3((a->R + 255) / 256), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

// mli_composite_loss geometry, shared by the launch, the finalize and the workspace query: rays
// per workgroup (two per wave for N <= 128) and workgroups; the partials the finalize sums.
struct CLGeo {
  int rpb, nb;
};
static CLGeo cl_geo(int R, int N) {
  const int rpb = N <= 32 * CE ? 2 * CW : CW;
  return CLGeo{rpb, (R + rpb - 1) / rpb};
}
static bool cl_valid(const mli_composite_loss_args* a) {
  const mli_composite_args& c = a->comp;
  const mli_loss_args& l = a->loss;
  if (c.R <= 0 || c.N <= 0 || c.N > 256 || l.R != c.R || l.N != c.N) return false;
  if (!c.weights || !c.rgb || !c.o_r || !c.o_s || !c.o_re || !a->dz4 || !l.scratch || !l.losses || !l.gt ||
      !l.outside || !c.y)
    return false;
  return !(l.w_intrinsic != 0.f && (l.sha == nullptr || l.cert == nullptr || l.ref == nullptr));
}

extern "C" int mli_composite_loss(const mli_composite_loss_args* a, mli_stream_t s) {
  if (!cl_valid(a)) return (int)hipErrorInvalidValue;
  const CLGeo g = cl_geo(a->comp.R, a->comp.N);
  if (g.rpb == 2 * CW)
    hipLaunchKernelGGL(composite_loss_kernel<32>, dim3(g.nb), dim3(CW * 64), 0, (hipStream_t)s, *a);
  else
    hipLaunchKernelGGL(composite_loss_kernel<64>, dim3(g.nb), dim3(CW * 64), 0, (hipStream_t)s, *a);
  if (!a->defer_finalize)
    hipLaunchKernelGGL(composite_loss_finalize, dim3(1), dim3(256), 0, (hipStream_t)s, a->loss, g.nb);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_loss_finalize(const mli_composite_loss_args* a, mli_stream_t s) {
  if (!cl_valid(a)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(composite_loss_finalize, dim3(1), dim3(256), 0, (hipStream_t)s, a->loss,
                     cl_geo(a->comp.R, a->comp.N).nb);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_composite_loss_workspace(const mli_composite_loss_args* a, int64_t* bytes) {
  const int R = a->comp.R;
  if (R <= 0 || a->comp.N <= 0) return (int)hipErrorInvalidValue;
  bytes[0] = (int64_t)mli_loss::ACC_N * cl_geo(R, a->comp.N).nb * 4;  // workgroup partials
  bytes[1] = (int64_t)R * a->comp.N * 8 * 4;                            // dz4
  return 0;
}
