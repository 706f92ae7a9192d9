// Fused neural-SDF evaluation on gfx950.
//
// Replaces NeuralSDF.encode + tcnn HashGrid + MLPforNeuralSDF layer 0 + sdf head
// (projects/neuralangelo/utils/modules.py:68-95, mlp.py:55-69) and, in FIELD mode, the
// 4-tap numerical gradient / diagonal hessian (modules.py:157-175) with the outside
// overwrite (NeuralLumen/model.py:343).
//
// One wave = 32 samples (lane c = sample, lane half h picks rows of the MFMA tiles).
// Per point:  X0^T (16 enc rows per k-step, level 2q+h in half h, NAT order) is built by
// the hash lookup in registers; pre = W0_enc (fp16 fragments from LDS) x X0^T on
// v_mfma_f32_32x32x16_f16, accumulator initialised in fp32 with b0 + W0[:, :3] . p (the
// point coordinates never go through fp16: a 1-ulp fp16 rounding of p is ~eps of the taps);
// softplus(beta=100) and the 256-wide sdf dot stay fp32; lane halves combine with a
// cross-half shuffle.  FIELD mode evaluates center + 4 taps and stores the center's
// softplus activations h0 as an fp16 frag image for layer 1 (mli_rgb_fwd).
#include "hashgrid.h"

namespace {

constexpr int SDF_WAVES = 4;
constexpr int FRAG_BYTES = 65536;          // 8 n-tiles x 8 k-steps x 1 KiB
constexpr int ROWC_OFF = FRAG_BYTES;        // 5 arrays [8 t][2 h][16 i] fp32 in acc order
constexpr int ROWC_ARRAY = 1024;            // bytes per array
constexpr int BSDF_OFF = FRAG_BYTES + 5 * ROWC_ARRAY;
static_assert(BSDF_OFF + 16 == MLI_SDF_PACK_BYTES, "pack layout");

struct SdfKArgs {
  mli_sdf_args a;
};

// Row constants of n-tile t for this lane half: 16 floats of array `arr`.
MLI_FI void load_rowc(const uint8_t* lds, int arr, int t, int h, float (&v)[16]) {
  const f32x4* p = reinterpret_cast<const f32x4*>(lds + ROWC_OFF + arr * ROWC_ARRAY + (t * 2 + h) * 64);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f32x4 q = p[u];
    v[4 * u] = q[0]; v[4 * u + 1] = q[1]; v[4 * u + 2] = q[2]; v[4 * u + 3] = q[3];
  }
}

// Evaluate the SDF at one point per lane (both lane halves see the same point).
// Returns the full sdf (after the cross-half reduction).  If h0_out != nullptr the fp16
// softplus activations are stored as the frag image of this tile.
MLI_FI float sdf_point(const uint8_t* lds, const uint16_t* __restrict__ table,
                       const mli_grid_levels& L, int lane, float px, float py, float pz,
                       uint16_t* __restrict__ h0_tile) {
  const int h = lane >> 5;
  // x01 = (p - (-2)) / (2 - (-2))  (modules.py:82-83)
  const float x0 = (px + 2.0f) * 0.25f, x1 = (py + 2.0f) * 0.25f, x2 = (pz + 2.0f) * 0.25f;
  half8 enc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float acc[8];
    hash_level_pair(table, L, 2 * q, 2 * q + 1, h, x0, x1, x2, acc);
#pragma unroll
    for (int f = 0; f < 8; ++f) enc[q][f] = (f16)acc[f];
    // at most two levels (16 x 16 B gathers) in flight per lane
    if (q & 1) __builtin_amdgcn_sched_barrier(0);
  }
  float part = 0.0f;
#pragma unroll 1
  for (int t = 0; t < 8; ++t) {
    float b0[16], wx[16], wy[16], wz[16];
    load_rowc(lds, 0, t, h, b0);
    load_rowc(lds, 1, t, h, wx);
    load_rowc(lds, 2, t, h, wy);
    load_rowc(lds, 3, t, h, wz);
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = b0[i] + (wx[i] * px + wy[i] * py + wz[i] * pz);
    const half8* frag = reinterpret_cast<const half8*>(lds + t * 8 * 1024) + lane;
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = mfma32(frag[q * 64], enc[q], acc);
    float ws[16];
    load_rowc(lds, 4, t, h, ws);
    f32x16 sp;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      sp[i] = softplus100(acc[i]);
      part = fmaf(ws[i], sp[i], part);
    }
    if (h0_tile) {
      half8* dst = reinterpret_cast<half8*>(h0_tile) + (2 * t) * 64 + lane;
      dst[0] = acc_to_frag(sp, 0);
      dst[64] = acc_to_frag(sp, 1);
    }
  }
  part += __shfl_xor(part, 32);
  return part + *reinterpret_cast<const float*>(lds + BSDF_OFF);
}

template <int MODE>
__global__ __launch_bounds__(256) void sdf_kernel(mli_sdf_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(a.wsdf);
    u32x4* dst = reinterpret_cast<u32x4*>(lds);
    for (int o = threadIdx.x; o < MLI_SDF_PACK_BYTES / 16; o += blockDim.x) dst[o] = src[o];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int n_total = a.R * a.n_per_ray;
  const int n_tiles = (n_total + 31) >> 5;
  for (int tile = blockIdx.x * SDF_WAVES + wave; tile < n_tiles; tile += gridDim.x * SDF_WAVES) {
    // opaque LDS base: keeps the 64 weight fragments / row constants from being hoisted
    // out of the tile loop (they would pin ~700 registers)
    const uint8_t* lds_t = lds + opaque_v(0);
    const int m = tile * 32 + c;
    const bool valid = m < n_total;
    const int mm = valid ? m : n_total - 1;
    const int r = mm / a.n_per_ray, k = mm - r * a.n_per_ray;
    const int slot = k * a.R + r;
    const float d = a.dists[slot];
    // p = c + v * d  (camera.py:314-320; two roundings, no fma)
    const float px = __fadd_rn(a.center[3 * r + 0], __fmul_rn(a.ray_unit[3 * r + 0], d));
    const float py = __fadd_rn(a.center[3 * r + 1], __fmul_rn(a.ray_unit[3 * r + 1], d));
    const float pz = __fadd_rn(a.center[3 * r + 2], __fmul_rn(a.ray_unit[3 * r + 2], d));
    if (MODE == MLI_SDF_MODE_SDF) {
      const float s = sdf_point(lds_t, a.table, a.levels, lane, px, py, pz, nullptr);
      if (valid && h == 0) a.sdf[slot] = s;
    } else {
      uint16_t* h0_tile = a.h0 + (size_t)tile * (16 * 64 * 8);
      const float e = a.eps;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
      // point 0 = center (stores h0), taps k1=(1,-1,-1) k2=(-1,-1,1) k3=(-1,1,-1) k4=(1,1,1)
      // (modules.py:159-166): x + k * eps in fp32
#pragma unroll 1
      for (int pi = 0; pi < 5; ++pi) {
        const float ex = (pi == 1 || pi == 4) ? e : -e;
        const float ey = (pi == 3 || pi == 4) ? e : -e;
        const float ez = (pi == 2 || pi == 4) ? e : -e;
        const float qx = pi ? __fadd_rn(px, ex) : px;
        const float qy = pi ? __fadd_rn(py, ey) : py;
        const float qz = pi ? __fadd_rn(pz, ez) : pz;
        const float v = sdf_point(lds_t, a.table, a.levels, lane, qx, qy, qz, pi == 0 ? h0_tile : nullptr);
        s0 = pi == 0 ? v : s0;
        s1 = pi == 1 ? v : s1;
        s2 = pi == 2 ? v : s2;
        s3 = pi == 3 ? v : s3;
        s4 = pi == 4 ? v : s4;
      }
      if (a.outside[r]) s0 = a.outside_val;
      if (valid && h == 0) {
        a.sdf[slot] = s0;
        // (k1*s1 + k2*s2 + k3*s3 + k4*s4) / (4 eps), summed left to right per component.
        const float gx = __fadd_rn(__fadd_rn(__fadd_rn(s1, -s2), -s3), s4);
        const float gy = __fadd_rn(__fadd_rn(__fadd_rn(-s1, -s2), s3), s4);
        const float gz = __fadd_rn(__fadd_rn(__fadd_rn(-s1, s2), -s3), s4);
        a.grad[3 * slot + 0] = gx / a.grad_den;
        a.grad[3 * slot + 1] = gy / a.grad_den;
        a.grad[3 * slot + 2] = gz / a.grad_den;
        if (a.with_hessian) {
          const float sum = __fadd_rn(__fadd_rn(__fadd_rn(s1, s2), s3), s4);
          const float hxx = __fadd_rn(sum / 2.0f, -__fmul_rn(2.0f, s0)) / a.hess_den;
          const float hv = hxx / 3.0f;
          a.hess[3 * slot + 0] = hv;
          a.hess[3 * slot + 1] = hv;
          a.hess[3 * slot + 2] = hv;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void hashgrid_kernel(mli_hashgrid_args a) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int p = gid >> 4, level = gid & 15;
  if (p >= a.n) return;
  float acc[8];
  hash_level<2>(a.table, level_params(a.levels, level), a.x01[3 * p], a.x01[3 * p + 1],
                a.x01[3 * p + 2], acc);
#pragma unroll
  for (int f = 0; f < 8; ++f) a.out[(size_t)p * 128 + level * 8 + f] = acc[f];
}

// ---------------------------------------------------------------- SDF layer-0 packing
// W0 = g0 * v0 / ||v0||_row (torch weight_norm dim=0); fp16 fragments of the 128 encoding
// columns (NAT order, k = 16q + 8h + j -> input column 3 + k) and fp32 row constants in
// accumulator order: b0, W0[:,0], W0[:,1], W0[:,2], w_sdf.
__global__ __launch_bounds__(256) void pack_sdf_kernel(mli_pack_sdf_args a) {
  const int n = blockIdx.x;  // output row 0..255
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const float* vrow = a.v0 + n * 131;
  float ss = 0.f;
  for (int k = tid; k < 131; k += 256) ss += vrow[k] * vrow[k];
  red[tid] = ss;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const float scale = a.g0[n] / sqrtf(red[0]);
  const int t = n >> 5, r = n & 31;
  // fragments: thread k-index over 128 enc columns
  if (tid < 128) {
    const int k = tid, q = k >> 4, hh = (k >> 3) & 1, j = k & 7;
    const int lanei = hh * 32 + r;
    f16* dst = reinterpret_cast<f16*>(a.dst + (t * 8 + q) * 1024 + lanei * 16) + j;
    *dst = (f16)(vrow[3 + k] * scale);
  }
  if (tid == 0) {
    // locate (h, i) with acc_row(i, h) == r
    for (int hh = 0; hh < 2; ++hh)
      for (int i = 0; i < 16; ++i)
        if (acc_row(i, hh) == r) {
          float* base = reinterpret_cast<float*>(a.dst + ROWC_OFF) + (t * 2 + hh) * 16 + i;
          base[0 * 256] = a.b0[n];
          base[1 * 256] = vrow[0] * scale;
          base[2 * 256] = vrow[1] * scale;
          base[3 * 256] = vrow[2] * scale;
          base[4 * 256] = a.w_sdf[n];
        }
    if (n == 0) *reinterpret_cast<float*>(a.dst + BSDF_OFF) = a.b_sdf[0];
  }
}

}  // namespace

extern "C" int mli_sdf(const mli_sdf_args* a, mli_stream_t s) {
  const int n_total = a->R * a->n_per_ray;
  const int tiles = (n_total + 31) / 32;
  int blocks = (tiles + SDF_WAVES - 1) / SDF_WAVES;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) return 0;
  if (a->mode == MLI_SDF_MODE_SDF)
    hipLaunchKernelGGL(sdf_kernel<MLI_SDF_MODE_SDF>, dim3(blocks), dim3(256), MLI_SDF_PACK_BYTES,
                       (hipStream_t)s, *a);
  else
    hipLaunchKernelGGL(sdf_kernel<MLI_SDF_MODE_FIELD>, dim3(blocks), dim3(256), MLI_SDF_PACK_BYTES,
                       (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_hashgrid_fwd(const mli_hashgrid_args* a, mli_stream_t s) {
  const int total = a->n * 16;
  if (total == 0) return 0;
  hipLaunchKernelGGL(hashgrid_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_pack_sdf(const mli_pack_sdf_args* a, mli_stream_t s) {
  hipLaunchKernelGGL(pack_sdf_kernel, dim3(256), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}
