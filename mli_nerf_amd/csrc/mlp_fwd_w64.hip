// EXPERIMENT (round 4): heads forward with 64 samples per wave, one wave per SIMD.
// Each weight fragment read from the LDS ring feeds two MFMAs (two 32-sample column tiles), so
// the ring's LDS reads per MFMA halve and the two accumulation chains are independent.
// DEFER: the epilogue of tile t runs after the MFMA chain of tile t+1 has been issued (its
// accumulators carried across the barrier), so the wave's own VALU fills its MFMA gaps.
#include "mlp_core.h"

#ifdef MLI_EXP_W64
namespace {

struct G64 {
  static constexpr int NW = 4, ND = 4, THREADS = 256, SAMPLES = 256, PF = 4;
  static constexpr int RND = 5;                  // 20 pieces of 1 KiB per chunk / 4 waves
  static constexpr int SLOT = RND * ND * 1024;   // 20 KiB
  static constexpr int SROW = SAMPLES * 2 + 16;
  static constexpr int STAGE = 32 * SROW;
  static constexpr int STAGE_OFF = NSLOT * SLOT;
  static constexpr int TPR = SAMPLES / 8;
  static constexpr int FL = 32 * TPR / THREADS;  // flush stores per thread and staged tile
  static constexpr int PQ_WAVE = 2048 + 256;
  static constexpr int PQ_OFF = STAGE_OFF + 2 * STAGE;
  // feat k-steps of each column kept in LDS, and where: eval (no stager / PQ blocks), training
  static constexpr int FKS_EVAL = 12, FOFF_EVAL = STAGE_OFF;
  static constexpr int FKS_TRAIN = 6, FOFF_TRAIN = PQ_OFF + NW * PQ_WAVE;
  static constexpr int LDS_EVAL = FOFF_EVAL + NW * 2 * FKS_EVAL * 1024;
  static constexpr int LDS_TRAIN = FOFF_TRAIN + NW * 2 * FKS_TRAIN * 1024;
  template <int ROLE> static constexpr int ring_ops() { return RND; }
};
static_assert(G64::LDS_EVAL <= 163840 && G64::LDS_TRAIN <= 163840, "LDS");
static_assert(8 * Q4_SLOT <= 2 * G64::STAGE, "Q slots in the staging area");

template <int KS, int PF>
MLI_FI void chunk_mma2(const uint8_t* chunk, const half8* X0, const half8* X1, int lane, f32x16& acc0,
                       f32x16& acc1) {
  const int h = lane >> 5;
  const f32x4* bias = reinterpret_cast<const f32x4*>(chunk + KS * 1024 + h * 64);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 b = bias[u];
    acc0[4 * u] = b[0]; acc0[4 * u + 1] = b[1]; acc0[4 * u + 2] = b[2]; acc0[4 * u + 3] = b[3];
  }
  acc1 = acc0;
  const half8* w = reinterpret_cast<const half8*>(chunk) + lane;
  constexpr int D = PF < KS ? PF : KS;
  half8 wr[D];
#pragma unroll
  for (int q = 0; q < D; ++q) wr[q] = w[q * 64];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    acc0 = mfma32(wr[q % D], X0[q], acc0);
    acc1 = mfma32(wr[q % D], X1[q], acc1);
    if (q + D < KS) wr[q % D] = w[(q + D) * 64];
  }
#pragma unroll
  for (int q = 0; q < D; ++q) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    if (q + D < KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
}

// ---------------------------------------------------------------------- staging (2 columns)
struct Stager64 {
  uint16_t* pend;
  int buf, pbuf;
};

// column block j (= 2 wave + col) of the tile: element i of the accumulator tile goes to row
// acc_row(i, h), column 32 j + c
MLI_FI void stage_col(uint8_t* sb, half8 f0, half8 f1, int j, int lane) {
  const int c = lane & 31, h = lane >> 5;
  uint8_t* p = sb + (4 * h) * G64::SROW + (j * 32 + c) * 2;
  const u32x4 w[2] = {__builtin_bit_cast(u32x4, f0), __builtin_bit_cast(u32x4, f1)};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t word = w[i >> 3][(i & 7) >> 1];
    *reinterpret_cast<uint16_t*>(p + ((i & 3) + 8 * (i >> 2)) * G64::SROW) = (uint16_t)((i & 1) ? (word >> 16) : word);
  }
}

MLI_FI void stage2(Stager64& sg, uint8_t* lds, const half8* o0, const half8* o1, int t, uint16_t* dst, int lane) {
  const int wave = threadIdx.x >> 6;
  uint8_t* sb = lds + G64::STAGE_OFF + sg.buf * G64::STAGE;
  stage_col(sb, o0[2 * t], o0[2 * t + 1], 2 * wave, lane);
  stage_col(sb, o1[2 * t], o1[2 * t + 1], 2 * wave + 1, lane);
  sg.pend = dst;
  sg.pbuf = sg.buf;
  sg.buf ^= 1;
}

MLI_FI void flush64(Stager64& sg, const uint8_t* lds, int S) {
  constexpr int RSTEP = G64::THREADS / G64::TPR;
  const int t = threadIdx.x, row = t / G64::TPR, col = t % G64::TPR;
  const uint8_t* sb = lds + G64::STAGE_OFF + sg.pbuf * G64::STAGE + row * G64::SROW + col * 16;
  uint16_t* g = sg.pend + (size_t)row * S + col * 8;
  const size_t step = (size_t)RSTEP * S;
#pragma unroll
  for (int u = 0; u < G64::FL; ++u) {
    const u32x4 x = *reinterpret_cast<const u32x4*>(sb + RSTEP * u * G64::SROW);
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(g + u * step));
  }
  sg.pend = nullptr;
}

// One layer of NT n-tiles over both columns.  Stores counted for the vmcnt waits (undercounts are
// safe: they only wait for more): STAGED flushes, EPI direct stores per epilogue, MASKN mask stores
// at the last tile.  DEFER: epi(t - 1) after the chain of tile t; the last tile's epilogue is the
// caller's (the next layer's `prev`, which runs before that layer's first chain: it produces the
// chain's last k-steps).  prev: the previous layer's pending epilogue (or nothing).
struct NoPre64 {
  MLI_FI int count(int) const { return 0; }
  MLI_FI void issue(int) const {}
};

template <int KS, int NT, bool STAGED, int EPI, int MASKN, bool DEFER, class Bytes, class Prev, class Epi,
          class Pre = NoPre64>
MLI_FI void run_layer64(Ring& rg, uint8_t* lds, Stager64& sg, int S, const half8* X0, const half8* X1, int lane,
                        Bytes&& bytes, Prev&& prev, Epi&& epi, f32x16& p0, f32x16& p1, Pre pre = Pre{}) {
  auto stores = [](int t) MLI_LAMBDA_FI {
    if (t < 0) return 0;
    if (DEFER) return (STAGED && t >= 2 ? G64::FL : 0) + (t >= 1 ? EPI : 0);
    return (STAGED && t >= 1 ? G64::FL : 0) + EPI + (t == NT - 1 ? MASKN : 0);
  };
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    pre.issue(t);
    ring_issue<G64, ALL>(rg, lds, bytes);
    if (sg.pend) flush64(sg, lds, S);
    if (t == 0) prev(p0, p1);
    f32x16 acc0, acc1;
    chunk_mma2<KS, G64::PF>(lds + (rg.cur % NSLOT) * G64::SLOT, X0, X1, lane, acc0, acc1);
    if (DEFER) {
      if (t > 0) epi(t - 1, p0, p1);
      p0 = acc0;
      p1 = acc1;
    } else {
      epi(t, acc0, acc1);
    }
    vm_wait((DIST - 1) * G64::RND + pre.count(t) + stores(t) + stores(t - 1));
    block_sync();
    rg.cur++;
  }
}

MLI_FI void extras64(const mli_rgb_fwd_args& a, int r, size_t slot, int h, half8 (&B)[19], bool train, int S, int m) {
  const float d = a.dists[slot];
  const float* cr = a.center + 3 * r;
  const float* vr = a.ray_unit + 3 * r;
  float p[3], nrm[3], g[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    p[i] = __fadd_rn(cr[i], __fmul_rn(vr[i], d));
    g[i] = a.grad[3 * slot + i];
  }
  const float gn = fmaxf(sqrtf((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2]), 1e-12f);
#pragma unroll
  for (int i = 0; i < 3; ++i) nrm[i] = g[i] / gn;
  float shl[16], shv[16];
  sh16(a.pts_light[3 * r], a.pts_light[3 * r + 1], a.pts_light[3 * r + 2], shl);
  sh16(vr[0], vr[1], vr[2], shv);
  const float e16[8] = {p[0], p[1], p[2], nrm[0], nrm[1], nrm[2], 0.f, 0.f};
  const uint32_t hm = opaque_v(h) ? ~0u : 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v16 = sel_mask(hm, 0.f, e16[j]);
    const float v17 = sel_mask(hm, shl[8 + j], shl[j]);
    const float v18 = sel_mask(hm, shv[8 + j], shv[j]);
    B[16][j] = (f16)v16;
    B[17][j] = (f16)v17;
    B[18][j] = (f16)v18;
    if (train) {
      a.x0T[(size_t)k_nat(16, h, j) * S + m] = __builtin_bit_cast(uint16_t, (f16)v16);
      a.x0T[(size_t)k_nat(17, h, j) * S + m] = __builtin_bit_cast(uint16_t, (f16)v17);
      a.x0T[(size_t)k_nat(18, h, j) * S + m] = __builtin_bit_cast(uint16_t, (f16)v18);
    }
  }
}

// Output-layer partials of one column tile j of the workgroup (q4_tile of mlp_core.h, per column):
// Q of tile j parks in slot j of the staging area; q4_sum64 then sums the tiles of each ray segment
// in tile order (the same order as the 8-wave kernel's wave order: bit-identical q4).
MLI_FI void q4_col64(uint8_t* lds, const half8 (&X)[19], const float (&gq)[3], int j, int lane) {
  const int wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  uint8_t* xr = lds + G64::PQ_OFF + wave * G64::PQ_WAVE;
  uint8_t* gr = xr + 2048;
  uint8_t* qs = lds + G64::STAGE_OFF + j * Q4_SLOT;
  if (h == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<f16*>(gr + i * 64 + c * 2) = (f16)(i < 3 ? gq[i] : 0.f);
  }
  asm volatile("" ::: "memory");
  half8 gf[2];
  {
    const int gi = min(c, 3);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) gf[ks] = *reinterpret_cast<const half8*>(gr + gi * 64 + (16 * ks + 8 * h) * 2);
  }
  const int g16 = (lane >> 4) & 3, q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = 4 * (g16 & 1) + p;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const u32x4 w = __builtin_bit_cast(u32x4, X[2 * b + u]);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ch = (4 * u + 2 * jj + h) ^ ((c >> 1) & 7);
        uint32_t* dst = reinterpret_cast<uint32_t*>(xr + c * 64 + ch * 8);
        *reinterpret_cast<uint2*>(dst) = make_uint2(w[2 * jj], w[2 * jj + 1]);
      }
    }
    asm volatile("" ::: "memory");
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int s0 = 16 * ks + 8 * h + q, s1 = s0 + 4;
      const half4 lo = ds_read_tr16(xr + s0 * 64 + (chunk ^ ((s0 >> 1) & 7)) * 8);
      const half4 hi = ds_read_tr16(xr + s1 * 64 + (chunk ^ ((s1 >> 1) & 7)) * 8);
      half8 xf;
      xf[0] = lo[0]; xf[1] = lo[1]; xf[2] = lo[2]; xf[3] = lo[3];
      xf[4] = hi[0]; xf[5] = hi[1]; xf[6] = hi[2]; xf[7] = hi[3];
      acc = mfma32(gf[ks], xf, acc);
    }
    asm volatile("" ::: "memory");
    if (h == 0) *reinterpret_cast<f32x4*>(qs + (32 * b + c) * 16) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  }
  float sb[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float v = gq[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    sb[i] = v;
  }
  if (lane == 0) *reinterpret_cast<f32x4*>(qs + 256 * 16) = f32x4{sb[0], sb[1], sb[2], 0.f};
  asm volatile("" ::: "memory");
}

MLI_FI void q4_sum64(const mli_rgb_fwd_args& a, const uint8_t* lds, int hd) {
  block_sync();
  const int N = a.N, t0 = blockIdx.x * 8;
  const int r_first = t0 * 32 / N;
  const int nseg = ((t0 + 8) * 32 - 1) / N - r_first + 1;
  const int segs = MLI_Q4_SEGS(N);
  f32x4* qo = reinterpret_cast<f32x4*>(a.q4) + (size_t)blockIdx.x * segs * a.n_heads * 257;
  for (int it = threadIdx.x; it < nseg * 257; it += G64::THREADS) {
    const int seg = it / 257, row = it - seg * 257;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 8; ++w)
      if ((t0 + w) * 32 / N - r_first == seg) v += *reinterpret_cast<const f32x4*>(lds + G64::STAGE_OFF + w * Q4_SLOT + row * 16);
    __builtin_nontemporal_store(v, qo + ((size_t)seg * a.n_heads + hd) * 257 + row);
  }
  block_sync();
}

template <bool TRAIN, bool PQ, bool DEFER>
__global__ __launch_bounds__(256, 1) void rgb_fwd64_kernel(mli_rgb_fwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tile0 = blockIdx.x * 8 + 2 * wave;
  constexpr int XL = PQ ? 3 : 4;
  constexpr int FKS = TRAIN ? G64::FKS_TRAIN : G64::FKS_EVAL;
  constexpr int FOFF = TRAIN ? G64::FOFF_TRAIN : G64::FOFF_EVAL;
  int mc[2], rc[2];
  size_t sc[2];
  float wgt[2];
#pragma unroll
  for (int col = 0; col < 2; ++col) {
    const int m = (tile0 + col) * 32 + c;
    const int r = m / a.N, k = m - r * a.N;
    mc[col] = m;
    rc[col] = r;
    sc[col] = (size_t)k * a.R + r;
    wgt[col] = PQ ? a.weights[sc[col]] : 0.f;
  }
  auto bytes = [](int cc) MLI_LAMBDA_FI { return fwd_bytes(cc); };
  Ring rg;
  ring_start(rg, a.wfwd, 8 + a.n_heads * 33, bytes);
  half8 A0[16], A1[16], B0[19], B1[19];
  {
    const half8* s0 = reinterpret_cast<const half8*>(a.h0 + (size_t)tile0 * FRAG_TILE) + lane;
    const half8* s1 = reinterpret_cast<const half8*>(a.h0 + (size_t)(tile0 + 1) * FRAG_TILE) + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      B0[q] = s0[q * 64];
      B1[q] = s1[q * 64];
    }
  }
  extras64(a, rc[0], sc[0], h, B0, TRAIN, S, mc[0]);
  extras64(a, rc[1], sc[1], h, B1, TRAIN, S, mc[1]);
#pragma unroll
  for (int d = 0; d < DIST; ++d) ring_issue<G64, ALL>(rg, lds, bytes);
  vm_wait((DIST - 1) * G64::RND);
  block_sync();

  Stager64 sg{nullptr, 0, 0};
  const size_t col0 = (size_t)blockIdx.x * G64::SAMPLES;
  uint8_t* fl = lds + FOFF + wave * 2 * FKS * 1024;
  uint16_t* ft0 = a.feat_frag + (size_t)tile0 * FRAG_TILE;
  uint16_t* ft1 = a.feat_frag + (size_t)(tile0 + 1) * FRAG_TILE;
  f32x16 p0, p1;
  auto none = [](f32x16&, f32x16&) MLI_LAMBDA_FI {};

  // SDF layer 1: feat = softplus(W1 h0 + b1) -> A; frag image (every k-step: static store counts;
  // eval: only the k-steps not in LDS) + LDS block (+ x0T rows 0..255 in training)
  auto feat_epi = [&](int t, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
    f32x16 v0, v1;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const f32x2 s0 = softplus100x2((f32x2){acc0[i], acc0[i + 1]});
      const f32x2 s1 = softplus100x2((f32x2){acc1[i], acc1[i + 1]});
      v0[i] = s0.x; v0[i + 1] = s0.y; v1[i] = s1.x; v1[i + 1] = s1.y;
    }
    A0[2 * t] = acc_to_frag(v0, 0); A0[2 * t + 1] = acc_to_frag(v0, 1);
    A1[2 * t] = acc_to_frag(v1, 0); A1[2 * t + 1] = acc_to_frag(v1, 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = 2 * t + s;
      if (TRAIN || q >= FKS) {
        reinterpret_cast<half8*>(ft0)[q * 64 + lane] = A0[q];
        reinterpret_cast<half8*>(ft1)[q * 64 + lane] = A1[q];
      }
      if (q < FKS) {
        *reinterpret_cast<half8*>(fl + q * 1024 + lane * 16) = A0[q];
        *reinterpret_cast<half8*>(fl + (FKS + q) * 1024 + lane * 16) = A1[q];
      }
    }
    if (TRAIN) stage2(sg, lds, A0, A1, t, a.x0T + (size_t)(32 * t) * S + col0, lane);
  };
  run_layer64<16, 8, TRAIN, TRAIN ? 4 : 0, 0, DEFER>(rg, lds, sg, S, B0, B1, lane, bytes, none, feat_epi, p0, p1);
  if (DEFER) {
    // the last feat tile (the heads reload feat next): tile 6's staged rows leave first
    if (sg.pend) flush64(sg, lds, S);
    feat_epi(7, p0, p1);
    block_sync();
    vm_wait(0);
  }

  for (int hd = 0; hd < a.n_heads; ++hd) {
    const int S = opaque_s(a.R * a.N);
    {
      const half8* i0 = reinterpret_cast<const half8*>(ft0) + opaque_v(lane);
      const half8* i1 = reinterpret_cast<const half8*>(ft1) + opaque_v(lane);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q < FKS) {
          B0[q] = *reinterpret_cast<const half8*>(fl + q * 1024 + lane * 16);
          B1[q] = *reinterpret_cast<const half8*>(fl + (FKS + q) * 1024 + lane * 16);
        } else {
          B0[q] = i0[q * 64];
          B1[q] = i1[q * 64];
        }
      }
    }
    uint32_t mb0[4], mb1[4];
    auto relu_epi = [&](half8* o0, half8* o1, int layer, bool stg) MLI_LAMBDA_FI {
      return [&, o0, o1, layer, stg](int t, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
        f32x16 v0, v1;
#pragma unroll
        for (int i = 0; i < 16; ++i) { v0[i] = relu1(acc0[i]); v1[i] = relu1(acc1[i]); }
        o0[2 * t] = acc_to_frag(v0, 0); o0[2 * t + 1] = acc_to_frag(v0, 1);
        o1[2 * t] = acc_to_frag(v1, 0); o1[2 * t + 1] = acc_to_frag(v1, 1);
        if (TRAIN) {
          const uint32_t b0 = relu_bits16(v0), b1 = relu_bits16(v1);
          if (t & 1) { mb0[t >> 1] |= b0 << 16; mb1[t >> 1] |= b1 << 16; }
          else { mb0[t >> 1] = b0; mb1[t >> 1] = b1; }
          if (stg) stage2(sg, lds, o0, o1, t, a.xT + ((size_t)(hd * XL + layer) * 256 + 32 * t) * S + col0, lane);
          if (t == 7) {
            u32x4* mp = reinterpret_cast<u32x4*>(a.masks) + ((size_t)(hd * 4 + layer) * (S / 32) + tile0) * 64 + lane;
            __builtin_nontemporal_store(u32x4{mb0[0], mb0[1], mb0[2], mb0[3]}, mp);
            __builtin_nontemporal_store(u32x4{mb1[0], mb1[1], mb1[2], mb1[3]}, mp + 64);
          }
        }
      };
    };
    auto e0 = relu_epi(A0, A1, 0, true);
    auto e1 = relu_epi(B0, B1, 1, true);
    auto e2 = relu_epi(A0, A1, 2, true);
    auto e3 = relu_epi(B0, B1, 3, !PQ);
    auto fin = [&](auto& e) MLI_LAMBDA_FI { return [&](f32x16& q0, f32x16& q1) MLI_LAMBDA_FI { e(7, q0, q1); }; };
    constexpr int MN = TRAIN ? 2 : 0;
    run_layer64<19, 8, TRAIN, 0, MN, DEFER>(rg, lds, sg, S, B0, B1, lane, bytes, none, e0, p0, p1);
    if (DEFER) {
      run_layer64<16, 8, TRAIN, 0, MN, true>(rg, lds, sg, S, A0, A1, lane, bytes, fin(e0), e1, p0, p1);
      run_layer64<16, 8, TRAIN, 0, MN, true>(rg, lds, sg, S, B0, B1, lane, bytes, fin(e1), e2, p0, p1);
      run_layer64<16, 8, TRAIN && !PQ, 0, MN, true>(rg, lds, sg, S, A0, A1, lane, bytes, fin(e2), e3, p0, p1);
    } else {
      run_layer64<16, 8, TRAIN, 0, MN, false>(rg, lds, sg, S, A0, A1, lane, bytes, none, e1, p0, p1);
      run_layer64<16, 8, TRAIN, 0, MN, false>(rg, lds, sg, S, B0, B1, lane, bytes, none, e2, p0, p1);
      run_layer64<16, 8, TRAIN && !PQ, 0, MN, false>(rg, lds, sg, S, A0, A1, lane, bytes, none, e3, p0, p1);
    }
    const int no = hd == 2 ? 1 : 3;
    const int off = hd * 3;
    float gq0[3] = {0.f, 0.f, 0.f}, gq1[3] = {0.f, 0.f, 0.f};
    auto out_epi = [&](int, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
      if (h == 0) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (i < no) {
            const float y0 = sigmoidf_acc(acc0[i]), y1 = sigmoidf_acc(acc1[i]);
            a.y[8 * sc[0] + off + i] = y0;
            a.y[8 * sc[1] + off + i] = y1;
            if (PQ) {
              gq0[i] = Q4_SCALE * wgt[0] * (y0 * (1.0f - y0));
              gq1[i] = Q4_SCALE * wgt[1] * (y1 * (1.0f - y1));
            }
          }
      }
    };
    if (DEFER)
      run_layer64<16, 1, false, 0, 0, false>(rg, lds, sg, S, B0, B1, lane, bytes, fin(e3), out_epi, p0, p1);
    else
      run_layer64<16, 1, false, 0, 0, false>(rg, lds, sg, S, B0, B1, lane, bytes, none, out_epi, p0, p1);
    if (PQ) {
      if (sg.pend) flush64(sg, lds, S);  // (PQ: X3 is not staged; nothing is pending here)
      q4_col64(lds, B0, gq0, 2 * wave, lane);
      q4_col64(lds, B1, gq1, 2 * wave + 1, lane);
      q4_sum64(a, lds, hd);
    }
  }
  if (sg.pend) flush64(sg, lds, opaque_s(a.R * a.N));
  vm_wait(0);
}


// ---------------------------------------------------------------------- backward dX chain, W64
// rgb_bwd_body (mlp_core.h) with two column tiles per wave: per head W4^T (KS 1), W3^T, W2^T,
// W1^T, each tile masked by the forward's ReLU bits (DMA'd per layer into a double-buffered LDS
// block: the workgroup's 8 tiles x 1 KiB) and staged to dzT.
constexpr int MASK_OFF64 = G64::PQ_OFF;          // after the ring and the stager
constexpr int MASKB64 = 8 * 1024;
constexpr int LDS_BWD64 = MASK_OFF64 + 2 * MASKB64;

template <bool DEFER>
__global__ __launch_bounds__(256, 1) void rgb_bwd64_kernel(mli_rgb_bwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tiles = S / 32;
  const int tile0 = blockIdx.x * 8 + 2 * wave;
  size_t sc[2];
#pragma unroll
  for (int col = 0; col < 2; ++col) {
    const int m = (tile0 + col) * 32 + c;
    const int r = m / a.N, k = m - r * a.N;
    sc[col] = (size_t)k * a.R + r;
  }
  auto bytes = [](int cc) MLI_LAMBDA_FI { return bwd_bytes(cc); };
  auto mask_dma = [&](int L) MLI_LAMBDA_FI {
    const int Lc = min(L, 11);
    const int hd = Lc >> 2, ml = 3 - (Lc & 3);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.masks) + (((size_t)(hd * 4 + ml) * tiles + (size_t)blockIdx.x * 8) * 64) * 16;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      glds16(src + u * (MASKB64 / 2) + threadIdx.x * 16, lds + MASK_OFF64 + (L & 1) * MASKB64 + u * (MASKB64 / 2) + wave * 1024);
  };
  Ring rg;
  ring_start(rg, a.wbwd, BWD_CHUNKS, bytes);
  mask_dma(0);
#pragma unroll
  for (int d = 0; d < DIST; ++d) ring_issue<G64, ALL>(rg, lds, bytes);
  vm_wait((DIST - 1) * G64::RND);
  block_sync();

  half8 A0[16], A1[16], B0[16], B1[16];
  Stager64 sg{nullptr, 0, 0};
  const size_t col0 = (size_t)blockIdx.x * G64::SAMPLES;
  f32x16 p0, p1;
  auto none = [](f32x16&, f32x16&) MLI_LAMBDA_FI {};
  for (int hd = 0; hd < 3; ++hd) {
    const int S = opaque_s(a.R * a.N);
    const int no = hd == 2 ? 1 : 3;
    half8 z40, z41;
#pragma unroll
    for (int j = 0; j < 8; ++j) { z40[j] = (f16)0.f; z41[j] = (f16)0.f; }
    if (h == 0) {
      const float* d0 = a.dz4 + 8 * sc[0] + 3 * hd;
      const float* d1 = a.dz4 + 8 * sc[1] + 3 * hd;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (j < no) {
          const f16 u0 = (f16)d0[j], u1 = (f16)d1[j];
          z40[j] = u0;
          z41[j] = u1;
          if (a.dz4T) {
            a.dz4T[((size_t)hd * 4 + j) * S + (tile0 * 32 + c)] = __builtin_bit_cast(uint16_t, u0);
            a.dz4T[((size_t)hd * 4 + j) * S + ((tile0 + 1) * 32 + c)] = __builtin_bit_cast(uint16_t, u1);
          }
        }
    }
    struct MaskPre {
      decltype(mask_dma)& dma;
      int next_layer;
      MLI_FI int count(int t) const { return t == 8 - DIST ? 2 : 0; }
      MLI_FI void issue(int t) const {
        if (t == 8 - DIST) dma(next_layer);
      }
    };
    auto pre = [&](int li) MLI_LAMBDA_FI { return MaskPre{mask_dma, hd * 4 + li + 1}; };
    auto mask_epi = [&](half8* o0, half8* o1, int layer, int li) MLI_LAMBDA_FI {
      return [&, o0, o1, layer, li](int t, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
        const uint8_t* mb = lds + MASK_OFF64 + (li & 1) * MASKB64 + lane * 16;
        const u32x4 m0 = *reinterpret_cast<const u32x4*>(mb + (2 * wave) * 1024);
        const u32x4 m1 = *reinterpret_cast<const u32x4*>(mb + (2 * wave + 1) * 1024);
        const int wi = t >> 1;
        const uint32_t w0 = wi == 0 ? m0[0] : wi == 1 ? m0[1] : wi == 2 ? m0[2] : m0[3];
        const uint32_t w1 = wi == 0 ? m1[0] : wi == 1 ? m1[1] : wi == 2 ? m1[2] : m1[3];
        f32x16 v0, v1;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          v0[i] = mask_bit(acc0[i], w0, (t & 1) * 16 + i);
          v1[i] = mask_bit(acc1[i], w1, (t & 1) * 16 + i);
        }
        o0[2 * t] = acc_to_frag(v0, 0); o0[2 * t + 1] = acc_to_frag(v0, 1);
        o1[2 * t] = acc_to_frag(v1, 0); o1[2 * t + 1] = acc_to_frag(v1, 1);
        stage2(sg, lds, o0, o1, t, a.dzT + ((size_t)(hd * 4 + layer) * 256 + 32 * t) * S + col0, lane);
      };
    };
    auto e3 = mask_epi(A0, A1, 3, 0);
    auto e2 = mask_epi(B0, B1, 2, 1);
    auto e1 = mask_epi(A0, A1, 1, 2);
    auto e0 = mask_epi(B0, B1, 0, 3);
    auto fin = [&](auto& e) MLI_LAMBDA_FI { return [&](f32x16& q0, f32x16& q1) MLI_LAMBDA_FI { e(7, q0, q1); }; };
    if (DEFER) {
      // (the previous head's last tile is finished before this head's first chain)
      run_layer64<1, 8, true, 0, 0, true>(rg, lds, sg, S, &z40, &z41, lane, bytes, none, e3, p0, p1, pre(0));
      run_layer64<16, 8, true, 0, 0, true>(rg, lds, sg, S, A0, A1, lane, bytes, fin(e3), e2, p0, p1, pre(1));
      run_layer64<16, 8, true, 0, 0, true>(rg, lds, sg, S, B0, B1, lane, bytes, fin(e2), e1, p0, p1, pre(2));
      run_layer64<16, 8, true, 0, 0, true>(rg, lds, sg, S, A0, A1, lane, bytes, fin(e1), e0, p0, p1, pre(3));
      // the head's last tile: tile 6 (staged by the last phase) leaves first, then tile 7 is staged
      // and made visible for the next phase's flush
      if (sg.pend) flush64(sg, lds, S);
      e0(7, p0, p1);
      block_sync();
    } else {
      run_layer64<1, 8, true, 0, 0, false>(rg, lds, sg, S, &z40, &z41, lane, bytes, none, e3, p0, p1, pre(0));
      run_layer64<16, 8, true, 0, 0, false>(rg, lds, sg, S, A0, A1, lane, bytes, none, e2, p0, p1, pre(1));
      run_layer64<16, 8, true, 0, 0, false>(rg, lds, sg, S, B0, B1, lane, bytes, none, e1, p0, p1, pre(2));
      run_layer64<16, 8, true, 0, 0, false>(rg, lds, sg, S, A0, A1, lane, bytes, none, e0, p0, p1, pre(3));
    }
  }
  // the last staged tile, visible after the last barrier
  if (sg.pend) flush64(sg, lds, opaque_s(a.R * a.N));
  vm_wait(0);
}
static_assert(LDS_BWD64 <= 163840, "LDS");
}  // namespace

int mli_launch_rgb_bwd_w64(const mli_rgb_bwd_args* a, hipStream_t s, int variant) {
  const dim3 grid(a->R * a->N / 256), block(256);
  if (variant & 2) hipLaunchKernelGGL(rgb_bwd64_kernel<true>, grid, block, LDS_BWD64, s, *a);
  else hipLaunchKernelGGL(rgb_bwd64_kernel<false>, grid, block, LDS_BWD64, s, *a);
  MLI_LAUNCH_CHECK();
}

int mli_launch_rgb_fwd_w64(const mli_rgb_fwd_args* a, hipStream_t s, int variant) {
  const bool train = a->xT != nullptr, pq = a->weights != nullptr, defer = (variant & 2) != 0;
  const dim3 grid(a->R * a->N / 256), block(256);
  const int L = train ? G64::LDS_TRAIN : G64::LDS_EVAL;
#define MLI_W64_LAUNCH(T, P, D) hipLaunchKernelGGL((rgb_fwd64_kernel<T, P, D>), grid, block, L, s, *a)
  if (!train) { if (defer) MLI_W64_LAUNCH(false, false, true); else MLI_W64_LAUNCH(false, false, false); }
  else if (pq) { if (defer) MLI_W64_LAUNCH(true, true, true); else MLI_W64_LAUNCH(true, true, false); }
  else return (int)hipErrorInvalidValue;  // (training without PQ: not in this experiment)
#undef MLI_W64_LAUNCH
  MLI_LAUNCH_CHECK();
}
#endif
