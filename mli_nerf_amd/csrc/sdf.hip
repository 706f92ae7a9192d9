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

#include <type_traits>

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

#ifndef MLI_PTERM_MFMA
#define MLI_PTERM_MFMA 1
#endif
// b0 + W0[:, 0:3] . p of n-tile t on the (otherwise idle) fp32 MFMA pipe: two
// v_mfma_f32_32x32x2_f32 with K = (x, y) and (z, 1), A = the tile's rows of (wx, wy) / (wz, b0)
// read from the row-constant arrays (acc order: row r of the tile is element
// ((r >> 3) << 2) | (r & 3) of lane half (r >> 2) & 1), B = the lane's point.  Exact fp32
// products and fp32 sums, in the MFMA's order instead of the fma chain's (the point
// coordinates still never go through fp16); the accumulator comes out in the 32x32 layout the
// fp16 chain continues.
MLI_FI f32x16 pterm_mfma(const uint8_t* lds, int t, int lane, float px, float py, float pz) {
  const int r = lane & 31, k = lane >> 5;
  const uint8_t* base = lds + ROWC_OFF + (t * 2 + ((r >> 2) & 1)) * 64 + ((((r >> 3) << 2) | (r & 3)) * 4);
  const float a1 = *reinterpret_cast<const float*>(base + (1 + k) * ROWC_ARRAY);   // wx | wy
  const float a2 = *reinterpret_cast<const float*>(base + (k ? 0 : 3) * ROWC_ARRAY);  // wz | b0
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, k ? py : px, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a2, k ? 1.0f : pz, acc, 0, 0, 0);
}

// Hash encoding of one point per lane (both lane halves see the same point; half h holds
// level 2q+h of k-step q): the B-fragment image X0^T of layer 0, NAT order.
MLI_FI void hash_encode(const uint16_t* __restrict__ table, const mli_grid_levels& L, int active, int lane,
                        float px, float py, float pz, half8 (&enc)[8]) {
  const int h = lane >> 5;
  // x01 = (p - (-2)) / (2 - (-2))  (modules.py:82-83)
  const float x0 = (px + 2.0f) * 0.25f, x1 = (py + 2.0f) * 0.25f, x2 = (pz + 2.0f) * 0.25f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    // coarse-to-fine mask (modules.py:91-93): levels >= active encode to 0 (uniform branch)
    if (2 * q >= active) {
#pragma unroll
      for (int f = 0; f < 8; ++f) enc[q][f] = (f16)0.0f;
      continue;
    }
    float acc[8];
    hash_level_pair(table, L, 2 * q, 2 * q + 1, h, x0, x1, x2, acc);
    const bool keep = 2 * q + h < active;
#pragma unroll
    for (int f = 0; f < 8; ++f) enc[q][f] = (f16)(keep ? acc[f] : 0.0f);
    // at most two levels (16 x 16 B gathers) in flight per lane
    if (q & 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// Layer 0 + softplus + sdf head from the encoding fragments.  Returns the full sdf (after
// the cross-half reduction).  If h0_tile != nullptr the fp16 softplus activations are stored
// as the frag image of this tile.  The row constants are read four at a time (fewer live
// registers); the pre-activation, softplus and sdf dot run on element pairs (packed fp32:
// common.h softplus100x2 / pterm_x2).
MLI_FI float sdf_from_enc(const uint8_t* lds, const half8 (&enc)[8], int lane, float px, float py, float pz,
                          uint16_t* __restrict__ h0_tile) {
  const int h = lane >> 5;
  f32x2 part2 = {0.0f, 0.0f};
#pragma unroll 1
  for (int t = 0; t < 8; ++t) {
    const f32x4* rc = reinterpret_cast<const f32x4*>(lds + ROWC_OFF + (t * 2 + h) * 64);
    constexpr int A4 = ROWC_ARRAY / 16;  // f32x4 per array
    f32x16 acc;
#if MLI_PTERM_MFMA
    acc = pterm_mfma(lds, t, lane, px, py, pz);
#else
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 b0 = rc[u], wx = rc[A4 + u], wy = rc[2 * A4 + u], wz = rc[3 * A4 + u];
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const f32x2 v = pterm_x2((f32x2){b0[j], b0[j + 1]}, (f32x2){wx[j], wx[j + 1]}, (f32x2){wy[j], wy[j + 1]},
                                 (f32x2){wz[j], wz[j + 1]}, px, py, pz);
        acc[4 * u + j] = v.x;
        acc[4 * u + j + 1] = v.y;
      }
    }
#endif
    const half8* frag = reinterpret_cast<const half8*>(lds + t * 8 * 1024) + lane;
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = mfma32(frag[q * 64], enc[q], acc);
    f32x16 sp;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4 ws = rc[4 * A4 + u];
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const f32x2 v = softplus100x2((f32x2){acc[4 * u + j], acc[4 * u + j + 1]});
        sp[4 * u + j] = v.x;
        sp[4 * u + j + 1] = v.y;
        part2 = fma_x2((f32x2){ws[j], ws[j + 1]}, v, part2);
      }
    }
    if (h0_tile) {  // read by the next kernel only: non-temporal
      half8* dst = reinterpret_cast<half8*>(h0_tile) + (2 * t) * 64 + lane;
      __builtin_nontemporal_store(acc_to_frag(sp, 0), dst);
      __builtin_nontemporal_store(acc_to_frag(sp, 1), dst + 64);
    }
  }
  float part = part2.x + part2.y;
  part += __shfl_xor(part, 32);
  return part + *reinterpret_cast<const float*>(lds + BSDF_OFF);
}

MLI_FI float sdf_point(const uint8_t* lds, const uint16_t* __restrict__ table, const mli_grid_levels& L,
                       int active, int lane, float px, float py, float pz, uint16_t* __restrict__ h0_tile) {
  half8 enc[8];
  hash_encode(table, L, active, lane, px, py, pz, enc);
  return sdf_from_enc(lds, enc, lane, px, py, pz, h0_tile);
}

// ---------------------------------------------------------------- FIELD mode, phase A
// Hash encodings of the center and the 4 taps, level-outer: the center's 8 corners are
// gathered once per level and every tap that falls in the same grid cell (most of them:
// the taps are eps = 1/2048/sqrt(3) away, <= 0.14 cells even at the finest level) reuses
// them with its own trilinear weights; only the other lanes gather.  Same arithmetic as
// hash_level (bit-identical encodings), written as B-fragment images for phase B.
constexpr int TAPS = 5;

// The 5 points' encodings at one level pair (lane half h = level 2qq+h), taps' own gathers
// compacted across the wave.  The center's 8 corners are gathered once and every tap in the
// center's cell interpolates them with its own weights.  A per-tap gather on the lanes whose tap
// left the cell (the straightforward form) costs up to 5 dependent gather rounds of mostly idle
// lanes per level pair at the fine levels (SQ counters: 213 gather instructions per 32-sample
// tile, waves parked 82 % of their cycles).  Instead every (tap, lane) whose cell differs from
// the center's becomes a job: its tap position goes to a wave-private LDS list (ballot + mbcnt
// slots, taps in order, lanes ascending) and the wave runs the jobs 64 at a time, one per lane,
// with the job's own level (the source lane's half) -- 8 fully used gathers per job round,
// issued beside the center's.  FIELD -4 % (0.832 -> 0.798 ms): the gather request count is
// unchanged, and that, not the round trips, is most of the bound.  The interpolation of every
// (point, level) is one function (interp8) on the same inputs whichever lane runs it.
// sink(p, src_lane, e) stores point p of lane src_lane.
struct TapJob {
  float x0, x1, x2;
  uint32_t tag;  // (p << 8) | source lane
};

template <int KIND>
MLI_FI uint32_t corner_index(const LevelP& P, uint32_t cx, uint32_t cy, uint32_t cz, bool skip_mod) {
  const uint32_t lin = cx + cy * P.res + cz * (P.res * P.res);
  const uint32_t hsh = (cx ^ (cy * 2654435761u) ^ (cz * 805459861u)) & (P.size - 1u);
  if (KIND == 1) return hsh;
  const uint32_t dn = skip_mod ? lin : fastmod_u32(lin, P.magic, P.size);
  if (KIND == 0) return dn;
  return (uint64_t)P.res * P.res * P.res <= (uint64_t)P.size ? dn : hsh;
}

MLI_FI void grid_cell(const LevelP& P, const float (&xp)[3], uint32_t (&g)[3], float (&pos)[3]) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float q = fmaf(P.scale, xp[d], 0.5f);  // tcnn pos_fract
    const float fl = floorf(q);
    g[d] = (uint32_t)(int)fl;
    pos[d] = q - fl;
  }
}

MLI_FI half8 interp8(const u32x4 (&cv)[8], const float (&pos)[3], bool keep) {
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
  for (int f = 0; f < 8; ++f) e[f] = (f16)(keep ? acc[f] : 0.0f);  // c2f mask
  return e;
}

template <int KIND>
MLI_FI void gather8(const uint16_t* __restrict__ table, const LevelP& P, const uint32_t (&g)[3], bool skip_mod,
                    u32x4 (&cv)[8]) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint32_t idx = corner_index<KIND>(P, g[0] + (c & 1), g[1] + ((c >> 1) & 1), g[2] + ((c >> 2) & 1), skip_mod);
    cv[c] = *reinterpret_cast<const u32x4*>(table + (size_t)(P.offset + idx) * 8);
  }
}

// P: this lane's level (half h); P0 / P1: the pair's two levels (a job takes its source's);
// keep0 / keep1: the coarse-to-fine masks of the two levels; jobs: this wave's LDS list.
template <int KIND, class Sink>
MLI_FI void level5(const uint16_t* __restrict__ table, const LevelP& P0, const LevelP& P1, int lane,
                    const float (&x)[TAPS][3], bool keep0, bool keep1, TapJob* jobs, Sink&& sink) {
  const int h = lane >> 5;
  const LevelP P{h ? P1.scale : P0.scale, h ? P1.res : P0.res, h ? P1.size : P0.size, h ? P1.offset : P0.offset,
                 h ? P1.magic : P0.magic};
  const bool keep = h ? keep1 : keep0;
  uint32_t g0[3];
  float pos0[3];
  grid_cell(P, x[0], g0, pos0);
  // the job list: taps whose cell is not the center's
  int n_jobs = 0;
#pragma unroll
  for (int p = 1; p < TAPS; ++p) {
    uint32_t g[3];
    float pos[3];
    grid_cell(P, x[p], g, pos);
    const bool div = g[0] != g0[0] || g[1] != g0[1] || g[2] != g0[2];
    const uint64_t mask = __ballot(div);
    if (div) {
      const int slot = n_jobs + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
      jobs[slot] = TapJob{x[p][0], x[p][1], x[p][2], (uint32_t)((p << 8) | lane)};
    }
    n_jobs += __popcll(mask);
  }
  const bool in_grid = g0[0] + 1 < P.res && g0[1] + 1 < P.res && g0[2] + 1 < P.res;
  const bool skip_mod = KIND == 0 && __all(in_grid);
  u32x4 cc[8];
  gather8<KIND>(table, P, g0, skip_mod, cc);
  // job rounds: lane j runs job j0 + j with its source lane's level
  for (int j0 = 0; j0 < n_jobs; j0 += 64) {
    const int j = j0 + lane;
    if (j < n_jobs) {
      const TapJob jb = jobs[j];
      const int src = (int)(jb.tag & 255u), p = (int)(jb.tag >> 8);
      const int hs = src >> 5;
      const LevelP Q{hs ? P1.scale : P0.scale, hs ? P1.res : P0.res, hs ? P1.size : P0.size,
                     hs ? P1.offset : P0.offset, hs ? P1.magic : P0.magic};
      const float xj[3] = {jb.x0, jb.x1, jb.x2};
      uint32_t g[3];
      float pos[3];
      grid_cell(Q, xj, g, pos);
      u32x4 tc[8];
      gather8<KIND>(table, Q, g, false, tc);
      sink(p, src, interp8(tc, pos, hs ? keep1 : keep0));
    }
  }
  // the center, and every tap in the center's cell, from the center's corners
  sink(0, lane, interp8(cc, pos0, keep));
#pragma unroll
  for (int p = 1; p < TAPS; ++p) {
    uint32_t g[3];
    float pos[3];
    grid_cell(P, x[p], g, pos);
    if (g[0] == g0[0] && g[1] == g0[1] && g[2] == g0[2]) sink(p, lane, interp8(cc, pos, keep));
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
  __shared__ TapJob job_lists[4][4 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31;
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
  uint16_t* base = a.enc + ((size_t)tile * TAPS * 8) * 512;
  const mli_grid_levels& L = a.levels;
  TapJob* jobs = job_lists[wave];
#pragma unroll 1
  for (int qq = 0; qq < 8; ++qq) {
    const int lv0 = 2 * qq, lv1 = 2 * qq + 1;
    uint16_t* dst = base + (size_t)qq * 512;
    if (lv0 >= a.active_levels) {  // coarse-to-fine: the whole level pair encodes to 0
#pragma unroll
      for (int p = 0; p < TAPS; ++p)
        *reinterpret_cast<u32x4*>(dst + (size_t)p * 8 * 512 + lane * 8) = u32x4{0, 0, 0, 0};
      continue;
    }
    const LevelP P0 = level_params(L, lv0), P1 = level_params(L, lv1);
    const bool keep0 = lv0 < a.active_levels, keep1 = lv1 < a.active_levels;
    const bool d0 = level_dense(L, lv0), d1 = level_dense(L, lv1);
    auto sink = [&](int p, int src, const half8& e) MLI_LAMBDA_FI {
      *reinterpret_cast<half8*>(dst + (size_t)p * 8 * 512 + src * 8) = e;
    };
    if (d0 && d1)
      level5<0>(a.table, P0, P1, lane, x, keep0, keep1, jobs, sink);
    else if (!d0 && !d1)
      level5<1>(a.table, P0, P1, lane, x, keep0, keep1, jobs, sink);
    else
      level5<2>(a.table, P0, P1, lane, x, keep0, keep1, jobs, sink);
  }
}

// ---------------------------------------------------------------- FIELD mode, phase B
template <int MLP_WAVES>
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
    const float s = sdf_point(lds_t, a.table, a.levels, a.active_levels, lane, px, py, pz, nullptr);
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


// ================================================================ stage a: backward
// W0_enc^T block: 4 n-tiles x 16 k-steps of A fragments.  Row r of n-tile u holds the
// layer-0 weights of encoding feature (level 2q'+h, feature f) with h = (r>>2)&1,
// i = (r&3) + 4(r>>3), q' = 2u + (i>>3), f = i&7, so accumulator register i of lane half h is
// that feature; k = h0 index in ACC order (the dZ0 fragments come from acc_to_frag).
constexpr int SDFT_PIECES = MLI_SDF_T_PACK_BYTES / 16;
__global__ __launch_bounds__(256) void pack_sdf_t_kernel(mli_pack_sdf_t_args a) {
  // blockIdx.x = (u*16 + q); thread = lane*8 + j (512 elements per k-step)... 64 lanes x 8
  const int uq = blockIdx.x, u = uq >> 4, q = uq & 15;
  for (int e = threadIdx.x; e < 512; e += blockDim.x) {
    const int lane = e >> 3, j = e & 7;
    const int rl = lane & 31, hh = lane >> 5;
    const int hr = (rl >> 2) & 1, i = (rl & 3) + 4 * (rl >> 3);
    const int qp = 2 * u + (i >> 3), level = 2 * qp + hr, f = i & 7;
    const int col = 3 + level * 8 + f;
    const int n = k_acc(q, hh, j);  // h0 index = output row of W0
    const float* vrow = a.v0 + n * 131;
    float ss = 0.f;
    for (int kk = 0; kk < 131; ++kk) ss += vrow[kk] * vrow[kk];
    const float w = vrow[col] * (a.g0[n] / sqrtf(ss));
    reinterpret_cast<f16*>(a.dst + uq * 1024 + lane * 16)[j] = (f16)w;
  }
}

MLI_FI void load_block(uint8_t* lds, const void* src_v, int pieces) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(src_v);
  for (int base = wave * 64; base < pieces; base += nw * 64) {
    const int piece = min(base + lane, pieces - 1);
    glds16(src + piece * 16, lds + base * 16);
  }
}

// Sum of v[0..15] over the 32 lanes of each lane half (samples), by recursive halving: lane c
// ends with the total of register i = (c >> 1) & 15 (lanes c, c^1 both hold it).
#ifndef MLI_HR_DPP
#define MLI_HR_DPP 1
#endif
// v from lane (lane xor M) within each 32-lane half, without LDS: quad_perm for M = 1, 2; the
// row_shl:4 / row_shr:4 pair with bank masks for M = 4; row_ror:8 for M = 8
template <int M>
MLI_FI float xor_lanes(float v) {
  const int x = __builtin_bit_cast(int, v);
  if (M == 1) return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
  if (M == 2) return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
  if (M == 4) {
    const int t = __builtin_amdgcn_update_dpp(0, x, 0x104, 0xF, 0x5, false);  // banks 0, 2 <- p + 4
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(t, x, 0x114, 0xF, 0xA, false));  // 1, 3 <- p - 4
  }
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false));  // M = 8
}

MLI_FI float half_reduce16(const float (&v)[16], int c) {
  float p8[8], p4[4], p2[2];
#if MLI_HR_DPP
  // the same pairwise sums as the __shfl_xor form below (a + b == b + a exactly): the xor-16 step
  // by v_permlane16_swap (lane p of row 0 / 1 ends with both halves' own / partner values), the
  // rest by DPP -- no LDS instructions
  const uint32_t b3 = (c & 8) ? ~0u : 0u, b2 = (c & 4) ? ~0u : 0u, b1 = (c & 2) ? ~0u : 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[j]),
                                                     __builtin_bit_cast(uint32_t, v[j + 8]), false, false);
    p8[j] = __builtin_bit_cast(float, (uint32_t)sw[0]) + __builtin_bit_cast(float, (uint32_t)sw[1]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) p4[j] = sel_mask(b3, p8[j + 4], p8[j]) + xor_lanes<8>(sel_mask(b3, p8[j], p8[j + 4]));
#pragma unroll
  for (int j = 0; j < 2; ++j) p2[j] = sel_mask(b2, p4[j + 2], p4[j]) + xor_lanes<4>(sel_mask(b2, p4[j], p4[j + 2]));
  const float p1 = sel_mask(b1, p2[1], p2[0]) + xor_lanes<2>(sel_mask(b1, p2[0], p2[1]));
  return p1 + xor_lanes<1>(p1);
#else
  // bitwise selects (a ternary on the arrays becomes a dynamically indexed scratch load)
  const uint32_t b4 = (c & 16) ? ~0u : 0u, b3 = (c & 8) ? ~0u : 0u, b2 = (c & 4) ? ~0u : 0u,
                 b1 = (c & 2) ? ~0u : 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    p8[j] = sel_mask(b4, v[j + 8], v[j]) + __shfl_xor(sel_mask(b4, v[j], v[j + 8]), 16);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    p4[j] = sel_mask(b3, p8[j + 4], p8[j]) + __shfl_xor(sel_mask(b3, p8[j], p8[j + 4]), 8);
#pragma unroll
  for (int j = 0; j < 2; ++j)
    p2[j] = sel_mask(b2, p4[j + 2], p4[j]) + __shfl_xor(sel_mask(b2, p4[j], p4[j + 2]), 4);
  const float p1 = sel_mask(b1, p2[1], p2[0]) + __shfl_xor(sel_mask(b1, p2[0], p2[1]), 2);
  return p1 + __shfl_xor(p1, 1);
#endif
}

MLI_FI void field_points5(const float* center, const float* ray_unit, float d, int r, float e,
                          float (&q)[TAPS][3]) {
  const float px = __fadd_rn(center[3 * r + 0], __fmul_rn(ray_unit[3 * r + 0], d));
  const float py = __fadd_rn(center[3 * r + 1], __fmul_rn(ray_unit[3 * r + 1], d));
  const float pz = __fadd_rn(center[3 * r + 2], __fmul_rn(ray_unit[3 * r + 2], d));
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

constexpr int BWD_WAVES = 8;  // stage-a sdf_bwd_kernel: waves per workgroup
constexpr int LDS_SDFT_OFF = LDS_SDF;
constexpr int LDS_DWS_OFF = LDS_SDF + MLI_SDF_T_PACK_BYTES;
constexpr int LDS_SDF_BWD = LDS_DWS_OFF + BWD_WAVES * 260 * 4;  // one dW/db slice per wave
static_assert(LDS_SDF_BWD <= 160 * 1024, "sdf_bwd LDS");

// Per sample: d sdf_i of the 5 points, then per point: layer 0 recomputed from the FIELD
// encoding (as field_mlp_kernel), dZ0 = (w_sdf ds_i [+ W1^T dZ1 for the center]) *
// softplus'(z0), d enc = W0_enc^T dZ0 (MFMA), dW/db of linear_sdf by lane reductions into the
// wave's own LDS slice (plain adds: distinct lanes, distinct addresses), then the slices in
// wave order into the workgroup's partial row and sdf_bwd_reduce_kernel over the workgroups in
// order: no atomics, bit-reproducible.
__global__ __launch_bounds__(BWD_WAVES * 64) void sdf_bwd_kernel(mli_sdf_bwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_block(lds, a.wsdf, PIECES);
  load_block(lds + LDS_SDFT_OFF, a.wsdf_t, SDFT_PIECES);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* dws_all = reinterpret_cast<float*>(lds + LDS_DWS_OFF);
  float* dws = dws_all + wave * 260;
  for (int i = lane; i < 260; i += 64) dws[i] = 0.f;
  vm_wait(0);
  __syncthreads();
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tiles = S / 32;
  const float inv_scale = 1.0f / a.grad_scale;
  const float inv_rn = 1.0f / (float)S;
  for (int tile = blockIdx.x * BWD_WAVES + wave; tile < tiles; tile += gridDim.x * BWD_WAVES) {
    const uint8_t* lds_t = lds + opaque_v(0);
    const int m = tile * 32 + c;
    const int r = m / a.N, k = m - r * a.N;
    const size_t slot = (size_t)k * a.R + r;
    float q[TAPS][3];
    field_points5(a.center, a.ray_unit, a.dists[slot], r, a.eps, q);
    // ---- d sdf of the 5 points (modules.py:157-175, model.py:343-347, misc.py:74-90)
    const bool out = a.outside[r] != 0;
    const float g0 = a.grad[3 * slot], g1 = a.grad[3 * slot + 1], g2 = a.grad[3 * slot + 2];
    float dg0 = a.d_grad[3 * slot], dg1 = a.d_grad[3 * slot + 1], dg2 = a.d_grad[3 * slot + 2];
    if (a.d_grad_ext) {  // autograd: d loss / d gradients of the caller's own loss terms
      dg0 += a.d_grad_ext[3 * slot]; dg1 += a.d_grad_ext[3 * slot + 1]; dg2 += a.d_grad_ext[3 * slot + 2];
    }
    const float gn = sqrtf((g0 * g0 + g1 * g1) + g2 * g2);
    if (!out && gn > 0.f) {  // eikonal: mean((|g| - 1)^2 * !outside)
      const float e = (gn - 1.0f) * (gn - 1.0f);
      if (isfinite(e)) {
        const float f = a.w_eikonal * inv_rn * 2.0f * (gn - 1.0f) / gn;
        dg0 += f * g0; dg1 += f * g1; dg2 += f * g2;
      }
    }
    {  // F.normalize(g) backward, denominator max(|g|, 1e-12)
      const float n0 = a.d_nrm[4 * slot] * inv_scale, n1 = a.d_nrm[4 * slot + 1] * inv_scale,
                  n2 = a.d_nrm[4 * slot + 2] * inv_scale;
      if (gn > 1e-12f) {
        const float dot = (g0 * n0 + g1 * n1) + g2 * n2;
        const float i1 = 1.0f / gn, i3 = dot / (gn * gn * gn);
        dg0 += n0 * i1 - g0 * i3; dg1 += n1 * i1 - g1 * i3; dg2 += n2 * i1 - g2 * i3;
      } else {
        dg0 += n0 * 1e12f; dg1 += n1 * 1e12f; dg2 += n2 * 1e12f;
      }
    }
    float dH = 0.f;  // d hxx: curvature mean(|sum(hess)| * !outside)
    if (!out && a.hess) {
      const float lap = (a.hess[3 * slot] + a.hess[3 * slot + 1]) + a.hess[3 * slot + 2];
      if (isfinite(lap) && lap != 0.f) dH = a.w_curvature * inv_rn * (lap > 0.f ? 1.f : -1.f);
    }
    if (a.d_hess_ext)  // hessians = [h, h, h] / 3 (modules.py:172-174): d h = sum_c d hess_c / 3
      dH += ((a.d_hess_ext[3 * slot] + a.d_hess_ext[3 * slot + 1]) + a.d_hess_ext[3 * slot + 2]) / 3.0f;
    float ds[TAPS];
    {
      const float gd = 1.0f / a.grad_den, hh = 0.5f * dH / a.hess_den;
      // grad = (k1 s1 + k2 s2 + k3 s3 + k4 s4) / (4 eps), k1=(1,-1,-1) k2=(-1,-1,1) k3=(-1,1,-1) k4=(1,1,1)
      ds[1] = (dg0 - dg1 - dg2) * gd + hh;
      ds[2] = (-dg0 - dg1 + dg2) * gd + hh;
      ds[3] = (-dg0 + dg1 - dg2) * gd + hh;
      ds[4] = (dg0 + dg1 + dg2) * gd + hh;
      ds[0] = out ? 0.f : a.d_sdf[slot] - 2.0f * dH / a.hess_den;
#pragma unroll
      for (int i = 0; i < TAPS; ++i) ds[i] *= a.grad_scale;
    }
    if (h == 0) {  // db_sdf partial
      float t = (((ds[0] + ds[1]) + ds[2]) + ds[3]) + ds[4];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (c == 0) dws[256] += t;
    }
    const half8* encp = reinterpret_cast<const half8*>(a.enc + (size_t)tile * TAPS * 8 * 512) + opaque_v(lane);
    const half8* dh0p = reinterpret_cast<const half8*>(a.dh0_frag + (size_t)tile * (16 * 64 * 8)) + lane;
#pragma unroll 1
    for (int pi = 0; pi < TAPS; ++pi) {
      half8 E[8];
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) E[qq] = encp[(pi * 8 + qq) * 64];
      float px = q[0][0], py = q[0][1], pz = q[0][2], dsp = ds[0];
#pragma unroll
      for (int j = 1; j < TAPS; ++j) {
        const uint32_t mk = pi == j ? ~0u : 0u;
        px = sel_mask(mk, q[j][0], px);
        py = sel_mask(mk, q[j][1], py);
        pz = sel_mask(mk, q[j][2], pz);
        dsp = sel_mask(mk, ds[j], dsp);
      }
      // the layer-0 weight gradient's operands (ABI 16): 32-sample tile `tile` of point pi is
      // tile 5 tile + pi of the enc image, and of the dZ0 and p images written here
      const size_t vt = (size_t)tile * TAPS + pi;
      {  // p as a one-k-step NAT frag image: features 0..2 in lane half 0, the rest 0
        half8 pv;
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = (f16)0.f;
        if (h == 0) {
          pv[0] = (f16)px;
          pv[1] = (f16)py;
          pv[2] = (f16)pz;
        }
        __builtin_nontemporal_store(pv, reinterpret_cast<half8*>(a.p_frag + vt * 512) + lane);
      }
      // d enc = W0_enc^T dZ0 (4 n-tiles x 16 k-steps), accumulated as dZ0's k-steps 2t, 2t+1
      // come out of tile t (no 16-fragment dZ0 array: it would need a runtime index)
      f32x16 de[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) de[u][i] = 0.f;
      half8* ztile = reinterpret_cast<half8*>(a.dz0_frag + vt * (16 * 512)) + lane;  // 16 k-steps per tile
#pragma unroll 1
      for (int t = 0; t < 8; ++t) {
        const uint8_t* lt = lds + opaque_v(0);
        // layer 0 recomputed exactly as the forward (sdf_from_enc: row constants four at a time)
        const f32x4* rc = reinterpret_cast<const f32x4*>(lt + ROWC_OFF + (t * 2 + h) * 64);
        constexpr int A4 = ROWC_ARRAY / 16;  // f32x4 per array
        f32x16 acc;
#if MLI_PTERM_MFMA
        acc = pterm_mfma(lt, t, lane, px, py, pz);
#else
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4 b0 = rc[u], wx = rc[A4 + u], wy = rc[2 * A4 + u], wz = rc[3 * A4 + u];
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            const f32x2 v = pterm_x2((f32x2){b0[j], b0[j + 1]}, (f32x2){wx[j], wx[j + 1]},
                                     (f32x2){wy[j], wy[j + 1]}, (f32x2){wz[j], wz[j + 1]}, px, py, pz);
            acc[4 * u + j] = v.x;
            acc[4 * u + j + 1] = v.y;
          }
        }
#endif
        const half8* frag = reinterpret_cast<const half8*>(lt + t * 8 * 1024) + lane;
#pragma unroll
        for (int qq = 0; qq < 8; ++qq) acc = mfma32(frag[qq * 64], E[qq], acc);
        half8 c0, c1;
        if (pi == 0) { c0 = dh0p[(2 * t) * 64]; c1 = dh0p[(2 * t + 1) * 64]; }
        f32x16 dz;
        float part[16];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4 ws = rc[4 * A4 + u];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * u + j;
            // one exp for softplus and its derivative: with q = e^{-|100 x|} (base 2, as
            // softplus100), softplus = max(x, 0) + log(1 + q) / 100 (bit-identical to
            // softplus100) and torch's backward sigmoid(100 x) = 1 / (1 + q) for x >= 0, else
            // q / (1 + q) (within an ulp of its z / (z + 1), without the overflow guard)
            const float x = acc[i];
            const float q = __builtin_amdgcn_exp2f(-fabsf(x * 144.26950408889634f));
            const float r = __builtin_amdgcn_rcpf(1.0f + q);
            const float dsig = x >= 0.0f ? r : q * r;
            const float sp = fmaf(__builtin_amdgcn_logf(q + 1.0f), 0.0069314718055994531f, relu_f(x));
            float dh = ws[j] * dsp;
            if (pi == 0) dh += (float)((i < 8) ? c0[i] : c1[i - 8]);
            dz[i] = dh * dsig;
            part[i] = dsp * sp;
          }
        }
        const half8 z0 = acc_to_frag(dz, 0), z1 = acc_to_frag(dz, 1);
        // k-steps 2t, 2t + 1 of the tile's dZ0 image, straight from the registers (streaming: read
        // back only by mli_wgrad)
        __builtin_nontemporal_store(z0, ztile + (2 * t) * 64);
        __builtin_nontemporal_store(z1, ztile + (2 * t + 1) * 64);
        const half8* fr = reinterpret_cast<const half8*>(lt + LDS_SDFT_OFF + (2 * t) * 1024) + lane;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          de[u] = mfma32(fr[(u * 16) * 64], z0, de[u]);
          de[u] = mfma32(fr[(u * 16 + 1) * 64], z1, de[u]);
        }
        const float tot = half_reduce16(part, c);
        if ((c & 1) == 0) dws[32 * t + acc_row((c >> 1) & 15, h)] += tot;
      }
      float* dst = a.d_enc + ((size_t)(tile * TAPS + pi) * 8) * 512 + lane * 8;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          f32x4* o = reinterpret_cast<f32x4*>(dst + (size_t)(2 * u + s2) * 512);
          const f32x16& v = de[u];
          __builtin_nontemporal_store(f32x4{v[8 * s2] * inv_scale, v[8 * s2 + 1] * inv_scale,
                                            v[8 * s2 + 2] * inv_scale, v[8 * s2 + 3] * inv_scale}, o);
          __builtin_nontemporal_store(f32x4{v[8 * s2 + 4] * inv_scale, v[8 * s2 + 5] * inv_scale,
                                            v[8 * s2 + 6] * inv_scale, v[8 * s2 + 7] * inv_scale}, o + 1);
        }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 257; i += blockDim.x) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < BWD_WAVES; ++w) v += dws_all[w * 260 + i];
    a.partials[(size_t)blockIdx.x * 257 + i] = v;
  }
}

// One workgroup per output (256 dW + db): strided partial sums, then an LDS tree -- a fixed
// order, so bit-reproducible (one thread looping over the 1024 partials took 330 us: a chain
// of dependent loads).
__global__ __launch_bounds__(256) void sdf_bwd_reduce_kernel(mli_sdf_bwd_args a, int blocks) {
  __shared__ float red[256];
  const int i = blockIdx.x, t = threadIdx.x;
  float v = 0.f;
  for (int b = t; b < blocks; b += 256) v += a.partials[(size_t)b * 257 + i];
  red[t] = v;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) {
    if (i < 256) a.dw_sdf[i] = red[0];
    else a.db_sdf[0] = red[0];
  }
}

// Hash-grid backward, level-outer like encode5_kernel: lane (c, h) = sample c, level 2qq+h.
// The center's 8 corners take the weighted d enc of every point in the center's cell (one
// fp32 atomic per corner feature); a tap in another cell scatters its own 64.  (A level-major
// variant, one level per launch so the atomic working set is Infinity-Cache sized, measured
// slower in round 1: 17.8 vs 15.7 ms before the coalesced scatter.)
#ifndef MLI_HB_VROW
#define MLI_HB_VROW 68
#endif
#ifndef MLI_HB_DPP
#define MLI_HB_DPP 1
#endif
#ifndef MLI_HB_FMAC
#define MLI_HB_FMAC 1
#endif
// One step of hash_bwd's segmented run scan: V += (take ? V of the DPP source lane : 0) for all
// 64 corner-feature sums (CTRL: row_shr:n = 0x110 + n, row_bcast:15 = 0x142; rows outside RMASK
// and out-of-row sources read 0).
template <int CTRL, int RMASK>
MLI_FI uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RMASK, 0xF, true);
}
template <int CTRL, int RMASK>
MLI_FI void hb_scan_step(float (&V)[8][8], bool take) {
#if MLI_HB_FMAC
  // V + take * o as one fma (exact: o * 1 + V rounds once as the add did, o * 0 + V = V for finite
  // o): a DPP move and a v_fmac per value and step instead of a move, a select and an add (an
  // inline v_fmac_f32_dpp form raised the kernel to 284 VGPRs)
  const float tf = take ? 1.0f : 0.0f;
#endif
#pragma unroll
  for (int cc = 0; cc < 8; ++cc)
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      const float o = __builtin_bit_cast(
          float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, V[cc][f]), CTRL, RMASK, 0xF, true));
#if MLI_HB_FMAC
      V[cc][f] = __builtin_fmaf(o, tf, V[cc][f]);
#else
      V[cc][f] += take ? o : 0.0f;
#endif
    }
}
#ifndef MLI_HB_SROW
#define MLI_HB_SROW 9
#endif
__global__ __launch_bounds__(256) void hash_bwd_kernel(mli_hash_bwd_args a) {
  // per wave: up to 64 run totals (64 floats) + their 8 corner slots, for the coalesced scatter.
  // Rows padded (VROW = 68 floats, SROW = 9 slots) so that the tail lanes' row writes fall in
  // distinct banks: at 64 / 8 the rows of consecutive ranks shared banks (SQ_LDS_BANK_CONFLICT
  // 50 M cycles per launch, profiles/r6/trio_a)
  constexpr int VROW = MLI_HB_VROW, SROW = MLI_HB_SROW;
  __shared__ __attribute__((aligned(16))) float s_vals[4][64 * VROW];
  __shared__ uint32_t s_slot[4][64 * SROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* tvals = s_vals[wave];
  uint32_t* tslot = s_slot[wave];
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tile = blockIdx.x * 4 + wave;
  if (tile >= S / 32) return;
  const int m = tile * 32 + c;
  const int r = m / a.N, k = m - r * a.N;
  float q[TAPS][3];
  field_points5(a.center, a.ray_unit, a.dists[(size_t)k * a.R + r], r, a.eps, q);
  float x[TAPS][3];
#pragma unroll
  for (int p = 0; p < TAPS; ++p)
#pragma unroll
    for (int d = 0; d < 3; ++d) x[p][d] = (q[p][d] + 2.0f) * 0.25f;
  const float* src = a.d_enc + ((size_t)tile * TAPS * 8) * 512 + lane * 8;
#pragma unroll 1
  for (int qq = 0; qq < 8; ++qq) {
    if (2 * qq >= a.active_levels) break;
    const int lv = 2 * qq + h;
    // a masked level stays in the loop with zero contributions: the coalesced scatter needs
    // every lane of the wave (lane j adds corner j/8 of a run)
    const bool lv_on = lv < a.active_levels;
    if (!__any(lv_on)) continue;
    const LevelP P = level_params(a.levels, lv);
    const bool dense = level_dense(a.levels, lv);
    const uint32_t r2 = P.res * P.res;
    auto index_of = [&](uint32_t cx, uint32_t cy, uint32_t cz) MLI_LAMBDA_FI {
      return dense ? fastmod_u32(cx + cy * P.res + cz * r2, P.magic, P.size)
                   : ((cx ^ (cy * 2654435761u) ^ (cz * 805459861u)) & (P.size - 1u));
    };
    auto cell = [&](const float (&xp)[3], uint32_t (&g)[3], float (&pos)[3]) MLI_LAMBDA_FI {
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float p = fmaf(P.scale, xp[d], 0.5f);
        const float fl = floorf(p);
        g[d] = (uint32_t)(int)fl;
        pos[d] = p - fl;
      }
    };
    auto weight = [&](const float (&pos)[3], int cc) MLI_LAMBDA_FI {
      float w = 1.0f;
      w *= (cc & 1) ? pos[0] : 1.0f - pos[0];
      w *= ((cc >> 1) & 1) ? pos[1] : 1.0f - pos[1];
      w *= ((cc >> 2) & 1) ? pos[2] : 1.0f - pos[2];
      return w;
    };
    uint32_t g0[3];
    float pos0[3];
    cell(x[0], g0, pos0);
    float G[8][8];
    {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src + (size_t)qq * 512);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + (size_t)qq * 512 + 4);
      const float on = lv_on ? 1.0f : 0.0f;
      const float d[8] = {lo[0] * on, lo[1] * on, lo[2] * on, lo[3] * on, hi[0] * on, hi[1] * on, hi[2] * on, hi[3] * on};
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) {
        const float w = weight(pos0, cc);
#pragma unroll
        for (int f = 0; f < 8; ++f) G[cc][f] = w * d[f];
      }
    }
    // Run-segmented reduction (see below) over the 32 consecutive samples of the lane half:
    // lanes sharing `key` cell form contiguous runs along the ray; the run's last lane holds
    // the run total of V and (if the run carries any contribution) scatters it.
    const int c0 = lane & 31;
    auto run_scatter = [&](const uint32_t (&cellk)[3], float (&V)[8][8], bool mine) MLI_LAMBDA_FI {
      // lanes without a contribution get a lane-unique key: singleton runs that never scatter
      // and never lengthen the scan
      const uint32_t key[3] = {mine ? cellk[0] : 0xFFFFFFFFu, mine ? cellk[1] : (uint32_t)lane,
                               mine ? cellk[2] : 0xFFFFFFFFu};
#if MLI_HB_DPP
      // neighbour keys by DPP wave_shr:1 / wave_shl:1 (lane 0 / 63 read 0: c0 == 0 / 31 decide)
      const uint32_t px = dpp_u32<0x138, 0xF>(key[0]), py = dpp_u32<0x138, 0xF>(key[1]),
                     pz = dpp_u32<0x138, 0xF>(key[2]);
#else
      const uint32_t px = __shfl_up(key[0], 1), py = __shfl_up(key[1], 1), pz = __shfl_up(key[2], 1);
#endif
      const bool head = c0 == 0 || px != key[0] || py != key[1] || pz != key[2];
      int start = head ? c0 : 0;  // first lane of this lane's run: max-scan of the heads
#if MLI_HB_DPP
      // (max is exact: the same values as the bpermute scan) in-row row_shr steps, then rows 1 / 3
      // take lane 15 / 47's running max (start is 0 / a head index of the same half, so a row-0
      // value is a valid lower bound for row 1)
      start = max(start, (int)dpp_u32<0x111, 0xF>((uint32_t)start));
      start = max(start, (int)dpp_u32<0x112, 0xF>((uint32_t)start));
      start = max(start, (int)dpp_u32<0x114, 0xF>((uint32_t)start));
      start = max(start, (int)dpp_u32<0x118, 0xF>((uint32_t)start));
      start = max(start, (int)dpp_u32<0x142, 0xA>((uint32_t)start));
#else
#pragma unroll
      for (int d = 1; d < 32; d <<= 1) {
        const int o = __shfl_up(start, d);
        if (c0 >= d) start = max(start, o);
      }
#endif
      // any lane of the run contributing (runs without contributions issue nothing)
      const uint64_t bal = __ballot(mine);
      const uint32_t hb = (uint32_t)(bal >> (32 * h));
      const uint32_t upto = c0 == 31 ? 0xFFFFFFFFu : ((2u << c0) - 1u);
      const uint32_t from = ~((1u << start) - 1u);
      const bool any = (hb & upto & from) != 0u;
      if (!__any(any)) return;
      // scan steps only up to the longest run of the wave (fine levels: mostly 1-sample runs)
      int span = c0 - start;
#if MLI_HB_DPP
      // the wave's longest run: in-row max, then rows 1 / 3 with lane 15 / 47 and rows 2 / 3 with
      // lane 31 (row_bcast:31 = 0x143): lane 63 holds the maximum
      span = max(span, (int)dpp_u32<0x111, 0xF>((uint32_t)span));
      span = max(span, (int)dpp_u32<0x112, 0xF>((uint32_t)span));
      span = max(span, (int)dpp_u32<0x114, 0xF>((uint32_t)span));
      span = max(span, (int)dpp_u32<0x118, 0xF>((uint32_t)span));
      span = max(span, (int)dpp_u32<0x142, 0xA>((uint32_t)span));
      span = max(span, (int)dpp_u32<0x143, 0xC>((uint32_t)span));
      span = __builtin_amdgcn_readlane(span, 63);
#else
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) span = max(span, __shfl_xor(span, o));
#endif
#if MLI_HB_DPP
      // the segmented scan on DPP moves (VALU) instead of ds_bpermute (LDS): row_shr 1, 2, 4, 8
      // within each 16-lane row, then row 1 / row 3 take lane 15 / 47's run prefix (row_bcast15)
      // if their run started in the row before -- per lane [start, c0] as the bpermute form, the
      // cross-row terms added in another order
      if (span >= 1) hb_scan_step<0x111, 0xF>(V, c0 - 1 >= start);
      if (span >= 2) hb_scan_step<0x112, 0xF>(V, c0 - 2 >= start);
      if (span >= 4) hb_scan_step<0x114, 0xF>(V, c0 - 4 >= start);
      if (span >= 8) hb_scan_step<0x118, 0xF>(V, c0 - 8 >= start);
      if (__any(c0 >= 16 && start <= 15)) hb_scan_step<0x142, 0xA>(V, c0 >= 16 && start <= 15);
#else
#pragma unroll 1
      for (int d = 1; d <= span; d <<= 1) {
        const bool take = c0 - d >= start;
#pragma unroll
        for (int cc = 0; cc < 8; ++cc)
#pragma unroll
          for (int f = 0; f < 8; ++f) {
            const float o = __shfl_up(V[cc][f], d);
            V[cc][f] += take ? o : 0.0f;
          }
      }
#endif
#if MLI_HB_DPP
      const uint32_t nx = dpp_u32<0x130, 0xF>(key[0]), ny = dpp_u32<0x130, 0xF>(key[1]),
                     nz = dpp_u32<0x130, 0xF>(key[2]);
#else
      const uint32_t nx = __shfl_down(key[0], 1), ny = __shfl_down(key[1], 1), nz = __shfl_down(key[2], 1);
#endif
      const bool tail = (c0 == 31 || nx != key[0] || ny != key[1] || nz != key[2]) && any;
      // Coalesced scatter: the run totals go through LDS so one atomic instruction adds one
      // run's 8 corners x 8 features with 8 consecutive lanes per corner (one 32 B L2 request
      // per corner instead of 8 -- atomics here are request-rate bound, tools/atomic_bench.hip)
      const uint64_t tb = __ballot(tail);
      const int rank = __popcll(tb & ((1ull << lane) - 1ull));
      const int ntail = __popcll(tb);
      if (tail) {
        f32x4* vd = reinterpret_cast<f32x4*>(tvals + rank * VROW);
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          vd[2 * cc] = f32x4{V[cc][0], V[cc][1], V[cc][2], V[cc][3]};
          vd[2 * cc + 1] = f32x4{V[cc][4], V[cc][5], V[cc][6], V[cc][7]};
          tslot[rank * SROW + cc] =
              P.offset + index_of(cellk[0] + (cc & 1), cellk[1] + ((cc >> 1) & 1), cellk[2] + ((cc >> 2) & 1));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // 4 runs per round: their LDS reads issue together (latency overlapped)
#pragma unroll 1
      for (int i0 = 0; i0 < ntail; i0 += 4) {
        float v[4];
        uint32_t slot[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = min(i0 + u, 63);
          v[u] = tvals[i * VROW + lane];
          slot[u] = tslot[i * SROW + (lane >> 3)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (i0 + u >= ntail) break;
          if (v[u] != 0.0f) {
            if (a.deterministic)  // fixed point: integer sums are order-independent
              atomicAdd(reinterpret_cast<unsigned long long*>(a.workspace) + (size_t)slot[u] * 8 + (lane & 7),
                        (unsigned long long)__double2ll_rn((double)v[u] * 1099511627776.0));
            else
              unsafeAtomicAdd(a.d_table + (size_t)slot[u] * 8 + (lane & 7), v[u]);
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#pragma unroll 1
    for (int p = 1; p < TAPS; ++p) {
      const float* sp = src + ((size_t)p * 8 + qq) * 512;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(sp);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(sp + 4);
      const float on = lv_on ? 1.0f : 0.0f;
      const float d[8] = {lo[0] * on, lo[1] * on, lo[2] * on, lo[3] * on, hi[0] * on, hi[1] * on, hi[2] * on, hi[3] * on};
      float xp[3] = {x[0][0], x[0][1], x[0][2]};
#pragma unroll
      for (int j = 1; j < TAPS; ++j) {
        const uint32_t mk = p == j ? ~0u : 0u;
        xp[0] = sel_mask(mk, x[j][0], xp[0]);
        xp[1] = sel_mask(mk, x[j][1], xp[1]);
        xp[2] = sel_mask(mk, x[j][2], xp[2]);
      }
      uint32_t g[3];
      float pos[3];
      cell(xp, g, pos);
      const bool same = g[0] == g0[0] && g[1] == g0[1] && g[2] == g0[2];
      float T[8][8];
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) {
        const float w = weight(pos, cc);
#if MLI_HB_FMAC
        // the weight split by the branch once per corner: G += w_in d (w_in = 0 off the center's
        // cell: G + 0 d = G), T = w_out d -- an fma and a mul per element, no selects (equal values
        // up to the sign of zeros, which the scatter skips)
        const float w_in = same ? w : 0.0f, w_out = same ? 0.0f : w;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          G[cc][f] = fmaf(w_in, d[f], G[cc][f]);
          T[cc][f] = w_out * d[f];
        }
#else
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          if (same) {
            G[cc][f] = fmaf(w, d[f], G[cc][f]);
            T[cc][f] = 0.0f;
          } else {
            T[cc][f] = w * d[f];
          }
        }
#endif
      }
      // a tap outside the center's cell: reduced over the runs of its own cell
      if (__any(!same && lv_on)) run_scatter(g, T, !same && lv_on);
    }
    // Samples of a wave are 32 consecutive depths of one ray: lanes sharing the center cell
    // form contiguous runs (a ray crosses a cell once).  Segmented inclusive scan of the 64
    // corner-feature sums over each run (within the lane half = one level), then only the
    // run's last lane issues the atomics -- coarse levels and the clustered fine samples
    // collapse to a few atomics per cell instead of one per sample.
    run_scatter(g0, G, lv_on);
  }
}


// deterministic hash_bwd: d_table = float(fixed * 2^-40)
__global__ __launch_bounds__(256) void fixed_to_float_kernel(const int64_t* w, float* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = (float)((double)w[i] * 9.094947017729282e-13);
}

// ================================================================ light visibility
struct TraceArgs {
  int R, iters, active;
  const float* origin; const float* dir;  // [R,3]
  const float* near_; const float* far_;  // [R]
  const float* start;                     // [R] or NULL (= near)
  const uint16_t* table;
  mli_grid_levels levels;
  const void* wsdf;
  float* dist; uint8_t* mask; float* pts;  // outputs ([R], [R], [R,3] or NULL)
};

// sphere_tracing_intersection (neuralangelo/model.py:298-325): one wave = 32 rays (the lane
// halves split the hash levels, as sdf_kernel), `iters` SDF evaluations of the moving point;
// dist += sdf while the ray is live, a ray dies once dist leaves [near, far]; finally
// dist = clamp(dist, near, far) (torch.clamp: NaN propagates) and pts = o + v dist.
__global__ __launch_bounds__(256) void trace_kernel(TraceArgs t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  load_weights(lds, t.wsdf);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int tiles = (t.R + 31) >> 5;
  for (int tile = blockIdx.x * SDF_WAVES + wave; tile < tiles; tile += gridDim.x * SDF_WAVES) {
    const int r = tile * 32 + c;
    const bool valid = r < t.R;
    const int rr = valid ? r : t.R - 1;
    const float o0 = t.origin[3 * rr], o1 = t.origin[3 * rr + 1], o2 = t.origin[3 * rr + 2];
    const float v0 = t.dir[3 * rr], v1 = t.dir[3 * rr + 1], v2 = t.dir[3 * rr + 2];
    const float nr = t.near_[rr], fr = t.far_[rr];
    float d = t.start ? t.start[rr] : nr;
    bool live = true;
#pragma unroll 1
    for (int it = 0; it < t.iters; ++it) {
      const uint8_t* lds_t = lds + opaque_v(0);
      const float px = __fadd_rn(o0, __fmul_rn(v0, d));
      const float py = __fadd_rn(o1, __fmul_rn(v1, d));
      const float pz = __fadd_rn(o2, __fmul_rn(v2, d));
      const float s = sdf_point(lds_t, t.table, t.levels, t.active, lane, px, py, pz, nullptr);
      if (live) d = d + s;
      if (d > fr) live = false;
      if (d < nr) live = false;
    }
    d = d < nr ? nr : (d > fr ? fr : d);
    if (valid && h == 0) {
      t.dist[r] = d;
      t.mask[r] = live ? 1 : 0;
      if (t.pts) {
        t.pts[3 * r] = __fadd_rn(o0, __fmul_rn(v0, d));
        t.pts[3 * r + 1] = __fadd_rn(o1, __fmul_rn(v1, d));
        t.pts[3 * r + 2] = __fadd_rn(o2, __fmul_rn(v2, d));
      }
    }
  }
}

// camera_ray_type blend_z: the composited depth is the intersection (model.py:143-146)
__global__ __launch_bounds__(256) void blend_z_kernel(mli_light_visibility_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const float d = a.blend_dist[r];
  a.inter_dist[r] = d;
  a.inter_mask[r] = d > 0.0f ? 1 : 0;
  for (int i = 0; i < 3; ++i) a.inter_pts[3 * r + i] = __fadd_rn(a.center[3 * r + i], __fmul_rn(a.ray_unit[3 * r + i], d));
}

// light ray from the light position to the camera-ray intersection (model.py:149-173)
__global__ __launch_bounds__(256) void light_prep_kernel(mli_light_visibility_args a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  float lr[3], c[3], v[3];
  for (int i = 0; i < 3; ++i) {
    c[i] = a.pts_light[3 * r + i];
    lr[i] = a.inter_pts[3 * r + i] - c[i];
  }
  const float n = sqrtf((lr[0] * lr[0] + lr[1] * lr[1]) + lr[2] * lr[2]);
  const float den = fmaxf(n, 1e-12f);  // F.normalize
  for (int i = 0; i < 3; ++i) {
    v[i] = lr[i] / den;
    a.light_unit[3 * r + i] = v[i];
  }
  float nl, fl;
  bool out;
  ray_bounds(c, v, a.vis_box, a.vis_r2, a.aabb, nl, fl, out);
  const float ft = n - 1e-3f;
  a.near_l[r] = nl;
  a.far_t[r] = ft;
  a.inside[r] = (nl < ft && ft < fl && !out) ? 1 : 0;
}

// visibility, normal x light, pseudo shading (model.py:169-184, :330-334)
__global__ __launch_bounds__(256) void light_finalize_kernel(mli_light_visibility_args a, const uint8_t* hit) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const bool vis = !hit[r] || !a.inside[r];
  const float g0 = -a.gradient[3 * r], g1 = -a.gradient[3 * r + 1], g2 = -a.gradient[3 * r + 2];
  const float gn = fmaxf(sqrtf((g0 * g0 + g1 * g1) + g2 * g2), 1e-12f);
  const float dot = ((g0 / gn) * a.light_unit[3 * r] + (g1 / gn) * a.light_unit[3 * r + 1]) +
                    (g2 / gn) * a.light_unit[3 * r + 2];
  const float nxl = fmaxf(dot, 0.0f);
  float sh = nxl * (vis ? 1.0f : 0.0f);
  if (a.gamma != 0.0f) sh = powf(sh, 1.0f / a.gamma);
  a.visibility[r] = vis ? 1 : 0;
  a.normal_x_light[r] = nxl;
  a.pseudo_shading[r] = sh;
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
  if (a->h0 == nullptr || a->grad == nullptr) return (int)hipErrorInvalidValue;
  if (a->enc == nullptr) return (int)hipErrorInvalidValue;
  // FIELD: phase A (encodings of the 5 points) then phase B (layer 0 + softplus + sdf head),
  // in chunks of tiles (a chunk's encodings: tiles x 40 KiB).  Measured at 4096 x 128 samples
  // with the geometry prefetched beside the heads: 1024 / 2048 / 4096 / 8192 /
  // 16384 tiles per chunk give FIELD 1.55 / 1.01 / 0.88 / 0.81 / 0.77 ms and steps of 5.49 /
  // 4.90 / 4.60 / 4.53 / 4.66 ms: each chunk pays a launch tail, and one chunk of 640 MiB
  // crowds the heads; 8192 (320 MiB, half of it re-read from the Infinity Cache) is kept.
  constexpr int CHUNK_TILES = 8192;
  for (int t0 = 0; t0 < tiles; t0 += CHUNK_TILES) {
    const int t1 = t0 + CHUNK_TILES < tiles ? t0 + CHUNK_TILES : tiles;
    hipLaunchKernelGGL(encode5_kernel, dim3((t1 - t0 + 3) / 4), dim3(256), 0, (hipStream_t)s, *a, t0, t1);
    int blocks = (t1 - t0 + 7) / 8;
    if (blocks > 512) blocks = 512;  // workgroups loop over the chunk's tiles (256 / 1024: DESIGN 9.0)
    hipLaunchKernelGGL(field_mlp_kernel<8>, dim3(blocks), dim3(8 * 64), LDS_SDF, (hipStream_t)s, *a, t0, t1);
    const int e = (int)hipGetLastError();
    if (e) return e;
  }
  return 0;
}

extern "C" int mli_sdf_workspace(const mli_sdf_args* a, int64_t* bytes) {
  const int64_t tiles = ((int64_t)a->R * a->n_per_ray + 31) / 32;
  bytes[0] = a->mode == MLI_SDF_MODE_FIELD ? tiles * 32 * 640 * 2 : 0;  // enc
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

extern "C" int mli_pack_sdf_t(const mli_pack_sdf_t_args* a, mli_stream_t s) {
  hipLaunchKernelGGL(pack_sdf_t_kernel, dim3(64), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

inline int sdf_bwd_blocks(int S) { return S / 256 > 1024 ? 1024 : S / 256; }

extern "C" int mli_sdf_bwd(const mli_sdf_bwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S <= 0) return 0;
  if (S % 256 != 0 || !a->enc || !a->wsdf || !a->wsdf_t || !a->d_enc || !a->dz0_frag || !a->p_frag ||
      !a->dw_sdf || !a->db_sdf || !a->dh0_frag || !a->d_nrm || !a->d_sdf || !a->d_grad)
    return (int)hipErrorInvalidValue;
  if (!a->partials) return (int)hipErrorInvalidValue;
  const int blocks = sdf_bwd_blocks(S);
  hipLaunchKernelGGL(sdf_bwd_kernel, dim3(blocks), dim3(BWD_WAVES * 64), LDS_SDF_BWD, (hipStream_t)s, *a);
  hipLaunchKernelGGL(sdf_bwd_reduce_kernel, dim3(257), dim3(256), 0, (hipStream_t)s, *a, blocks);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_sdf_bwd_workspace(const mli_sdf_bwd_args* a, int64_t* bytes) {
  const int64_t S = (int64_t)a->R * a->N;
  if (S <= 0 || S % 256 != 0) return (int)hipErrorInvalidValue;
  bytes[0] = S * 640 * 4;                         // d_enc
  bytes[1] = 5 * S * 256 * 2;                     // dz0_frag
  bytes[2] = 5 * S * 16 * 2;                      // p_frag
  bytes[3] = (int64_t)sdf_bwd_blocks((int)S) * 257 * 4;             // partials
  return 0;
}

extern "C" int mli_hash_bwd(const mli_hash_bwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S <= 0) return 0;
  if (S % 64 != 0 || !a->d_enc || !a->d_table) return (int)hipErrorInvalidValue;
  if (a->deterministic && (!a->workspace || a->n_params <= 0)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hash_bwd_kernel, dim3((S / 32 + 3) / 4), dim3(256), 0, (hipStream_t)s, *a);
  if (a->deterministic)
    hipLaunchKernelGGL(fixed_to_float_kernel, dim3(2048), dim3(256), 0, (hipStream_t)s, a->workspace, a->d_table,
                       a->n_params);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_hash_bwd_workspace(const mli_hash_bwd_args* a, int64_t* bytes) {
  bytes[0] = a->deterministic ? a->n_params * 8 : 0;
  return 0;
}

extern "C" int mli_light_visibility(const mli_light_visibility_args* a, mli_stream_t s) {
  if (a->R <= 0) return 0;
  if (a->camera_ray_type < 0 || a->camera_ray_type > 2 || a->iters < 0) return (int)hipErrorInvalidValue;
  const hipStream_t st = (hipStream_t)s;
  const int rb = (a->R + 255) / 256;
  int tb = (a->R + 32 * SDF_WAVES - 1) / (32 * SDF_WAVES);
  if (tb > 2048) tb = 2048;
  TraceArgs t{a->R, a->iters, a->active_levels, a->center, a->ray_unit, a->near_, a->far_,
              a->camera_ray_type == 0 ? a->blend_dist : nullptr, a->table, a->levels, a->wsdf,
              a->inter_dist, a->inter_mask, a->inter_pts};
  if (a->camera_ray_type == 1)
    hipLaunchKernelGGL(blend_z_kernel, dim3(rb), dim3(256), 0, st, *a);
  else
    hipLaunchKernelGGL(trace_kernel, dim3(tb), dim3(256), LDS_SDF, st, t);
  hipLaunchKernelGGL(light_prep_kernel, dim3(rb), dim3(256), 0, st, *a);
  // light ray: from the light position over [near_l, far_t]; its hit flag goes into `visibility`
  // (scratch until the finalize overwrites it) and its distance into pseudo_shading (scratch)
  TraceArgs tl{a->R, a->iters, a->active_levels, a->pts_light, a->light_unit, a->near_l, a->far_t, nullptr,
               a->table, a->levels, a->wsdf, a->pseudo_shading, a->visibility, nullptr};
  hipLaunchKernelGGL(trace_kernel, dim3(tb), dim3(256), LDS_SDF, st, tl);
  hipLaunchKernelGGL(light_finalize_kernel, dim3(rb), dim3(256), 0, st, *a, (const uint8_t*)a->visibility);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_light_visibility_workspace(const mli_light_visibility_args* a, int64_t* bytes) {
  const int64_t R = a->R;
  bytes[0] = R * 3 * 4;  // light_unit
  bytes[1] = R * 4;      // near_l
  bytes[2] = R * 4;      // far_t
  bytes[3] = R;          // inside
  bytes[4] = R * 3 * 4;  // inter_pts
  return 0;
}
