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
// cross-half shuffle.
//
// SDF mode (sampling rounds) fuses encode + MLP per point.  FIELD mode (center + 4 taps,
// h0 frag image of the center for layer 1 / mli_rgb_fwd) runs in two phases per chunk of
// tiles: encode5_kernel gathers the hash grid level-outer for the 5 points (taps in the
// center's cell reuse its corners; high occupancy for the gather latency) into fp16
// B-fragment images, then field_mlp_kernel streams them through layer 0 + softplus + sdf
// head.  Chunks keep the encodings Infinity-Cache resident between the two.
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

// The packed SDF block (70 KiB) -> LDS by LDS-DMA: every 16 B piece issued back to back,
// one wait (a load -> store loop would pay one global round trip per 4 KiB).  The DMA lands
// lane-linearly in whole 1 KiB wave pieces, so the kernels allocate LDS_SDF (rounded up):
// the tail lanes repeat the last piece into the padding.
constexpr int PIECES = MLI_SDF_PACK_BYTES / 16;  // 4481 (the last one: b_sdf)
constexpr int LDS_SDF = ((PIECES + 63) / 64) * 64 * 16;
MLI_FI void load_weights(uint8_t* lds, const void* wsdf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(wsdf);
  for (int base = wave * 64; base < PIECES; base += nw * 64) {
    const int piece = min(base + lane, PIECES - 1);  // the tail lanes repeat the last piece
    glds16(src + piece * 16, lds + base * 16);
  }
  vm_wait(0);
  __syncthreads();
}

// Row constants of n-tile t for this lane half: 16 floats of array `arr`.
MLI_FI void load_rowc(const uint8_t* lds, int arr, int t, int h, float (&v)[16]) {
  const f32x4* p = reinterpret_cast<const f32x4*>(lds + ROWC_OFF + arr * ROWC_ARRAY + (t * 2 + h) * 64);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f32x4 q = p[u];
    v[4 * u] = q[0]; v[4 * u + 1] = q[1]; v[4 * u + 2] = q[2]; v[4 * u + 3] = q[3];
  }
}

// Hash encoding of one point per lane (both lane halves see the same point; half h holds
// level 2q+h of k-step q): the B-fragment image X0^T of layer 0, NAT order.
MLI_FI void hash_encode(const uint16_t* __restrict__ table, const mli_grid_levels& L, int lane, float px,
                        float py, float pz, half8 (&enc)[8]) {
  const int h = lane >> 5;
  // x01 = (p - (-2)) / (2 - (-2))  (modules.py:82-83)
  const float x0 = (px + 2.0f) * 0.25f, x1 = (py + 2.0f) * 0.25f, x2 = (pz + 2.0f) * 0.25f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float acc[8];
    hash_level_pair(table, L, 2 * q, 2 * q + 1, h, x0, x1, x2, acc);
#pragma unroll
    for (int f = 0; f < 8; ++f) enc[q][f] = (f16)acc[f];
    // at most two levels (16 x 16 B gathers) in flight per lane
    if (q & 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// Layer 0 + softplus + sdf head from the encoding fragments.  Returns the full sdf (after
// the cross-half reduction).  If h0_tile != nullptr the fp16 softplus activations are stored
// as the frag image of this tile.
MLI_FI float sdf_from_enc(const uint8_t* lds, const half8 (&enc)[8], int lane, float px, float py, float pz,
                          uint16_t* __restrict__ h0_tile) {
  const int h = lane >> 5;
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
    if (h0_tile) {  // read by the next kernel only: non-temporal
      half8* dst = reinterpret_cast<half8*>(h0_tile) + (2 * t) * 64 + lane;
      __builtin_nontemporal_store(acc_to_frag(sp, 0), dst);
      __builtin_nontemporal_store(acc_to_frag(sp, 1), dst + 64);
    }
  }
  part += __shfl_xor(part, 32);
  return part + *reinterpret_cast<const float*>(lds + BSDF_OFF);
}

MLI_FI float sdf_point(const uint8_t* lds, const uint16_t* __restrict__ table, const mli_grid_levels& L,
                       int lane, float px, float py, float pz, uint16_t* __restrict__ h0_tile) {
  half8 enc[8];
  hash_encode(table, L, lane, px, py, pz, enc);
  return sdf_from_enc(lds, enc, lane, px, py, pz, h0_tile);
}

// ---------------------------------------------------------------- FIELD mode, phase A
// Hash encodings of the center and the 4 taps, level-outer: the center's 8 corners are
// gathered once per level and every tap that falls in the same grid cell (most of them:
// the taps are eps = 1/2048/sqrt(3) away, <= 0.14 cells even at the finest level) reuses
// them with its own trilinear weights; only the other lanes gather.  Same arithmetic as
// hash_level (bit-identical encodings), written as B-fragment images for phase B.
constexpr int TAPS = 5;

template <int KIND>
MLI_FI void level5(const uint16_t* __restrict__ table, const LevelP& P, const float (&x)[TAPS][3],
                   uint16_t* __restrict__ dst /* enc + (tile*5*8 + q)*512 + lane*8 */) {
  const uint32_t r2 = P.res * P.res;
  const bool dense_lane = (uint64_t)P.res * P.res * P.res <= (uint64_t)P.size;
  auto index_of = [&](uint32_t cx, uint32_t cy, uint32_t cz, bool skip_mod) MLI_LAMBDA_FI {
    const uint32_t lin = cx + cy * P.res + cz * r2;
    const uint32_t hsh = (cx ^ (cy * 2654435761u) ^ (cz * 805459861u)) & (P.size - 1u);
    if (KIND == 1) return hsh;
    const uint32_t dn = skip_mod ? lin : fastmod_u32(lin, P.magic, P.size);
    return KIND == 0 ? dn : (dense_lane ? dn : hsh);
  };
  auto cell = [&](const float (&xp)[3], uint32_t (&g)[3], float (&pos)[3]) MLI_LAMBDA_FI {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float p = fmaf(P.scale, xp[d], 0.5f);  // tcnn pos_fract
      const float fl = floorf(p);
      g[d] = (uint32_t)(int)fl;
      pos[d] = p - fl;
    }
  };
  auto interp_store = [&](const u32x4 (&cv)[8], const float (&pos)[3], uint16_t* out) MLI_LAMBDA_FI {
    float acc[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) acc[f] = 0.0f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float w = 1.0f;
      w *= (c & 1) ? pos[0] : 1.0f - pos[0];
      w *= ((c >> 1) & 1) ? pos[1] : 1.0f - pos[1];
      w *= ((c >> 2) & 1) ? pos[2] : 1.0f - pos[2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f16 lo = __builtin_bit_cast(f16, (uint16_t)(cv[c][q] & 0xFFFFu));
        const f16 hi = __builtin_bit_cast(f16, (uint16_t)(cv[c][q] >> 16));
        acc[2 * q] = fmaf(w, (float)lo, acc[2 * q]);
        acc[2 * q + 1] = fmaf(w, (float)hi, acc[2 * q + 1]);
      }
    }
    half8 e;
#pragma unroll
    for (int f = 0; f < 8; ++f) e[f] = (f16)acc[f];
    *reinterpret_cast<half8*>(out) = e;
  };
  // center
  uint32_t g0[3];
  float pos0[3];
  cell(x[0], g0, pos0);
  const bool in_grid = g0[0] + 1 < P.res && g0[1] + 1 < P.res && g0[2] + 1 < P.res;
  const bool skip_mod = KIND == 0 && __all(in_grid);
  u32x4 cc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint32_t idx = index_of(g0[0] + (c & 1), g0[1] + ((c >> 1) & 1), g0[2] + ((c >> 2) & 1), skip_mod);
    cc[c] = *reinterpret_cast<const u32x4*>(table + (size_t)(P.offset + idx) * 8);
  }
  interp_store(cc, pos0, dst);
  // taps
#pragma unroll
  for (int p = 1; p < TAPS; ++p) {
    uint32_t g[3];
    float pos[3];
    cell(x[p], g, pos);
    const bool same = g[0] == g0[0] && g[1] == g0[1] && g[2] == g0[2];
    u32x4 tc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) tc[c] = cc[c];
    if (!same) {  // divergent: only the lanes whose tap left the center's cell gather
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t idx = index_of(g[0] + (c & 1), g[1] + ((c >> 1) & 1), g[2] + ((c >> 2) & 1), false);
        tc[c] = *reinterpret_cast<const u32x4*>(table + (size_t)(P.offset + idx) * 8);
      }
    }
    interp_store(tc, pos, dst + (size_t)p * 8 * 512);
  }
}

// The 5 points of a sample: center p = c + v d, taps p + k_i eps, k1=(1,-1,-1) k2=(-1,-1,1)
// k3=(-1,1,-1) k4=(1,1,1) (modules.py:159-166), fp32 adds.
MLI_FI void field_points(const mli_sdf_args& a, int slot, int r, float (&q)[TAPS][3]) {
  const float d = a.dists[slot];
  // p = c + v * d  (camera.py:314-320; two roundings, no fma)
  const float px = __fadd_rn(a.center[3 * r + 0], __fmul_rn(a.ray_unit[3 * r + 0], d));
  const float py = __fadd_rn(a.center[3 * r + 1], __fmul_rn(a.ray_unit[3 * r + 1], d));
  const float pz = __fadd_rn(a.center[3 * r + 2], __fmul_rn(a.ray_unit[3 * r + 2], d));
  const float e = a.eps;
#pragma unroll
  for (int pi = 0; pi < TAPS; ++pi) {
    const float ex = (pi == 1 || pi == 4) ? e : -e;
    const float ey = (pi == 3 || pi == 4) ? e : -e;
    const float ez = (pi == 2 || pi == 4) ? e : -e;
    q[pi][0] = pi ? __fadd_rn(px, ex) : px;
    q[pi][1] = pi ? __fadd_rn(py, ey) : py;
    q[pi][2] = pi ? __fadd_rn(pz, ez) : pz;
  }
}

__global__ __launch_bounds__(256) void encode5_kernel(mli_sdf_args a, int tile0, int tile1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int n_total = a.R * a.n_per_ray;
  const int tile = tile0 + blockIdx.x * 4 + wave;
  if (tile >= tile1) return;
  const int m = min(tile * 32 + c, n_total - 1);
  const int r = m / a.n_per_ray, k = m - r * a.n_per_ray;
  float q[TAPS][3];
  field_points(a, k * a.R + r, r, q);
  float x[TAPS][3];
#pragma unroll
  for (int p = 0; p < TAPS; ++p)
#pragma unroll
    for (int d = 0; d < 3; ++d) x[p][d] = (q[p][d] + 2.0f) * 0.25f;  // modules.py:82-83
  uint16_t* base = a.enc + ((size_t)tile * TAPS * 8) * 512 + lane * 8;
  const mli_grid_levels& L = a.levels;
#pragma unroll 1
  for (int qq = 0; qq < 8; ++qq) {
    const int lv0 = 2 * qq, lv1 = 2 * qq + 1;
    const LevelP P0 = level_params(L, lv0), P1 = level_params(L, lv1);
    const LevelP P{h ? P1.scale : P0.scale, h ? P1.res : P0.res, h ? P1.size : P0.size,
                   h ? P1.offset : P0.offset, h ? P1.magic : P0.magic};
    const bool d0 = level_dense(L, lv0), d1 = level_dense(L, lv1);
    uint16_t* dst = base + (size_t)qq * 512;
    if (d0 && d1)
      level5<0>(a.table, P, x, dst);
    else if (!d0 && !d1)
      level5<1>(a.table, P, x, dst);
    else
      level5<2>(a.table, P, x, dst);
  }
}

// ---------------------------------------------------------------- FIELD mode, phase B
constexpr int MLP_WAVES = 8;  // 8 waves share the 70 KiB LDS weight block: 2 blocks = 16 waves per CU

__global__ __launch_bounds__(MLP_WAVES * 64) void field_mlp_kernel(mli_sdf_args a, int tile0, int tile1) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_weights(lds, a.wsdf);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int n_total = a.R * a.n_per_ray;
  for (int tile = tile0 + blockIdx.x * MLP_WAVES + wave; tile < tile1; tile += gridDim.x * MLP_WAVES) {
    const uint8_t* lds_t = lds + opaque_v(0);  // keep LDS fragments from being hoisted (registers)
    const int m = tile * 32 + c;
    const bool valid = m < n_total;
    const int mm = valid ? m : n_total - 1;
    const int r = mm / a.n_per_ray, k = mm - r * a.n_per_ray;
    const int slot = k * a.R + r;
    float q[TAPS][3];
    field_points(a, slot, r, q);
    uint16_t* h0_tile = a.h0 + (size_t)tile * (16 * 64 * 8);
    const half8* encp = reinterpret_cast<const half8*>(a.enc + (size_t)tile * TAPS * 8 * 512) + opaque_v(lane);
    float s[TAPS];
#pragma unroll 1
    for (int pi = 0; pi < TAPS; ++pi) {
      half8 enc[8];
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) enc[qq] = encp[(pi * 8 + qq) * 64];
      // point pi by bitwise selects (a runtime index into q[][] would go to scratch)
      float px = q[0][0], py = q[0][1], pz = q[0][2];
#pragma unroll
      for (int j = 1; j < TAPS; ++j) {
        const uint32_t mk = pi == j ? ~0u : 0u;
        px = sel_mask(mk, q[j][0], px);
        py = sel_mask(mk, q[j][1], py);
        pz = sel_mask(mk, q[j][2], pz);
      }
      const float v = sdf_from_enc(lds_t, enc, lane, px, py, pz, pi == 0 ? h0_tile : nullptr);
#pragma unroll
      for (int j = 0; j < TAPS; ++j) s[j] = pi == j ? v : s[j];
    }
    float s0 = s[0];
    const float s1 = s[1], s2 = s[2], s3 = s[3], s4 = s[4];
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

// SDF only (sampling rounds): one point per lane, encode + layer 0 + sdf head fused.
__global__ __launch_bounds__(256) void sdf_kernel(mli_sdf_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_weights(lds, a.wsdf);
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
    const float s = sdf_point(lds_t, a.table, a.levels, lane, px, py, pz, nullptr);
    if (valid && h == 0) a.sdf[slot] = s;
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
  if (tiles < 1) return 0;
  if (a->mode == MLI_SDF_MODE_SDF) {
    int blocks = (tiles + SDF_WAVES - 1) / SDF_WAVES;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(sdf_kernel, dim3(blocks), dim3(256), LDS_SDF, (hipStream_t)s, *a);
    MLI_LAUNCH_CHECK();
  }
  if (a->enc == nullptr || a->h0 == nullptr || a->grad == nullptr) return (int)hipErrorInvalidValue;
  // FIELD: phase A (encodings of the 5 points) then phase B (layer 0 + softplus + sdf head),
  // in chunks of tiles so a chunk's encodings (chunk * 40 KiB) are re-read from the
  // Infinity Cache instead of HBM
  constexpr int CHUNK_TILES = 4096;  // 131072 samples, 160 MiB of encodings
  for (int t0 = 0; t0 < tiles; t0 += CHUNK_TILES) {
    const int t1 = t0 + CHUNK_TILES < tiles ? t0 + CHUNK_TILES : tiles;
    hipLaunchKernelGGL(encode5_kernel, dim3((t1 - t0 + 3) / 4), dim3(256), 0, (hipStream_t)s, *a, t0, t1);
    int blocks = (t1 - t0 + MLP_WAVES - 1) / MLP_WAVES;
    if (blocks > 512) blocks = 512;
    hipLaunchKernelGGL(field_mlp_kernel, dim3(blocks), dim3(MLP_WAVES * 64), LDS_SDF, (hipStream_t)s,
                       *a, t0, t1);
    const int e = (int)hipGetLastError();
    if (e) return e;
  }
  return 0;
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
