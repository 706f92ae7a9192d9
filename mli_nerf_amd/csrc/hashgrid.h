// Multires hash-grid trilinear lookup (replaces tiny-cuda-nn HashGrid forward,
// projects/neuralangelo/utils/modules.py:42-50,83-86; semantics: oracle/hashgrid.py).
#pragma once
#include "common.h"

// Exact n % d for 32-bit n, d via Lemire's fastmod with M = floor(2^64 / d) + 1.
MLI_FI uint32_t fastmod_u32(uint32_t n, uint64_t M, uint32_t d) {
  const uint64_t low = M * (uint64_t)n;
  return (uint32_t)__umul64hi(low, (uint64_t)d);
}

// Level parameters resolved for one lane.
struct LevelP {
  float scale;
  uint32_t res, size, offset;
  uint64_t magic;
};

// One level for one point: 8 corner gathers of 16 B (8 fp16 features), trilinear weights
// in fp32, fp32 accumulation (tcnn accumulates in fp16; we are at least as accurate).
// KIND 0: dense index (gx + gy*res + gz*res^2) % size, 1: coherent prime hash & (size-1),
// 2: per-lane choice (only for configurations where a lane pair mixes both kinds).
template <int KIND>
MLI_FI void hash_level(const uint16_t* __restrict__ table, const LevelP& P, float x0, float x1,
                       float x2, float (&acc)[8]) {
  float pos[3];
  const float xin[3] = {x0, x1, x2};
  uint32_t g[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const float p = fmaf(P.scale, xin[d], 0.5f);  // tcnn pos_fract
    const float fl = floorf(p);
    g[d] = (uint32_t)(int)fl;
    pos[d] = p - fl;
  }
  const uint32_t r2 = P.res * P.res;
  const bool dense_lane = (uint64_t)P.res * P.res * P.res <= (uint64_t)P.size;
#pragma unroll
  for (int f = 0; f < 8; ++f) acc[f] = 0.0f;
  auto corners = [&](auto index_of) MLI_LAMBDA_FI {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint32_t cx = g[0] + (c & 1), cy = g[1] + ((c >> 1) & 1), cz = g[2] + ((c >> 2) & 1);
      float w = 1.0f;
      w *= (c & 1) ? pos[0] : 1.0f - pos[0];
      w *= ((c >> 1) & 1) ? pos[1] : 1.0f - pos[1];
      w *= ((c >> 2) & 1) ? pos[2] : 1.0f - pos[2];
      const uint32_t idx = index_of(cx, cy, cz);
      const u32x4 raw = *reinterpret_cast<const u32x4*>(table + (size_t)(P.offset + idx) * 8);
      const uint32_t words[4] = {raw[0], raw[1], raw[2], raw[3]};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f16 lo = __builtin_bit_cast(f16, (uint16_t)(words[q] & 0xFFFFu));
        const f16 hi = __builtin_bit_cast(f16, (uint16_t)(words[q] >> 16));
        acc[2 * q] = fmaf(w, (float)lo, acc[2 * q]);
        acc[2 * q + 1] = fmaf(w, (float)hi, acc[2 * q + 1]);
      }
    }
  };
  auto dense_mod = [&](uint32_t cx, uint32_t cy, uint32_t cz) MLI_LAMBDA_FI {
    return fastmod_u32(cx + cy * P.res + cz * r2, P.magic, P.size);
  };
  auto hashed = [&](uint32_t cx, uint32_t cy, uint32_t cz) MLI_LAMBDA_FI {
    return (cx ^ (cy * 2654435761u) ^ (cz * 805459861u)) & (P.size - 1u);
  };
  if (KIND == 0) {
    // whole cell inside the dense grid (every corner index < res^3 <= size): the modulo is
    // the identity -- a uniform branch skips the 64-bit fastmod when the whole wave qualifies
    const bool in_grid = g[0] + 1 < P.res && g[1] + 1 < P.res && g[2] + 1 < P.res;
    if (__all(in_grid))
      corners([&](uint32_t cx, uint32_t cy, uint32_t cz) MLI_LAMBDA_FI { return cx + cy * P.res + cz * r2; });
    else
      corners(dense_mod);
  } else if (KIND == 1) {
    corners(hashed);
  } else {
    corners([&](uint32_t cx, uint32_t cy, uint32_t cz) MLI_LAMBDA_FI {
      return dense_lane ? dense_mod(cx, cy, cz) : hashed(cx, cy, cz);
    });
  }
}

MLI_FI LevelP level_params(const mli_grid_levels& L, int lv) {
  return LevelP{L.scale[lv], L.res[lv], L.size[lv], L.offset[lv], L.modmagic[lv]};
}

MLI_FI bool level_dense(const mli_grid_levels& L, int lv) {
  return (uint64_t)L.res[lv] * L.res[lv] * L.res[lv] <= (uint64_t)L.size[lv];
}

// Levels lv0 (lane half 0) and lv1 (lane half 1) for this lane's point, uniform branch on
// the pair's kinds (scalar values from the kernel arguments).
MLI_FI void hash_level_pair(const uint16_t* __restrict__ table, const mli_grid_levels& L, int lv0,
                            int lv1, int h, float x0, float x1, float x2, float (&acc)[8]) {
  const LevelP P0 = level_params(L, lv0), P1 = level_params(L, lv1);
  const LevelP P{h ? P1.scale : P0.scale, h ? P1.res : P0.res, h ? P1.size : P0.size,
                 h ? P1.offset : P0.offset, h ? P1.magic : P0.magic};
  const bool d0 = level_dense(L, lv0), d1 = level_dense(L, lv1);
  if (d0 && d1) {
    hash_level<0>(table, P, x0, x1, x2, acc);
  } else if (!d0 && !d1) {
    hash_level<1>(table, P, x0, x1, x2, acc);
  } else {
    hash_level<2>(table, P, x0, x1, x2, acc);
  }
}
