// EXPERIMENT (round 4): eval heads forward with 64 samples per wave, one wave per SIMD.
// Each weight fragment read from the LDS ring feeds two MFMAs (two 32-sample column tiles), so
// the ring's LDS reads per MFMA halve and the two accumulation chains are independent.
#include "mlp_core.h"

#ifdef MLI_EXP_W64
namespace {

struct GW64 {
  static constexpr int NW = 4, ND = 4, THREADS = 256, SAMPLES = 256, PF = 4;
  static constexpr int RND = 5;                       // 20 pieces of 1 KiB per chunk / 4 waves
  static constexpr int SLOT = RND * ND * 1024;        // 20 KiB
  static constexpr int FKS = 12;                      // feat k-steps of each column kept in LDS
  static constexpr int FEAT_OFF = NSLOT * SLOT;
  static constexpr int FEAT_WAVE = 2 * FKS * 1024;
  static constexpr int LDS = FEAT_OFF + NW * FEAT_WAVE;  // 156 KiB
  template <int ROLE> static constexpr int ring_ops() { return RND; }
};
static_assert(GW64::LDS <= 163840, "LDS");

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

// one layer of NT n-tiles, both columns; EPI: global stores per epilogue (static, may undercount)
template <int KS, int NT, int EPI, class Bytes, class Epi>
MLI_FI void run_layer2(Ring& rg, uint8_t* lds, const half8* X0, const half8* X1, int lane, Bytes&& bytes, Epi&& epi) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    ring_issue<GW64, ALL>(rg, lds, bytes);
    f32x16 acc0, acc1;
    chunk_mma2<KS, GW64::PF>(lds + (rg.cur % NSLOT) * GW64::SLOT, X0, X1, lane, acc0, acc1);
    epi(t, acc0, acc1);
    vm_wait((DIST - 1) * GW64::RND + EPI * (t > 0 ? 2 : 1));
    block_sync();
    rg.cur++;
  }
}

// DEFER: the epilogue of tile t runs after the MFMA chain of tile t+1 has been issued (its
// accumulators carried across the barrier), so a wave's VALU epilogue can fill its own MFMA gaps;
// the layer's last tile is finished by the next layer (`prev`, before that layer's chain in program
// order: it produces the chain's last k-steps).  p0 / p1 carry the pending accumulators.
template <int KS, int NT, int EPI, class Bytes, class Prev, class Epi>
MLI_FI void run_layer2d(Ring& rg, uint8_t* lds, const half8* X0, const half8* X1, int lane, Bytes&& bytes,
                        Prev&& prev, Epi&& epi, f32x16& p0, f32x16& p1) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    ring_issue<GW64, ALL>(rg, lds, bytes);
    if (t == 0) prev(p0, p1);
    f32x16 acc0, acc1;
    chunk_mma2<KS, GW64::PF>(lds + (rg.cur % NSLOT) * GW64::SLOT, X0, X1, lane, acc0, acc1);
    if (t > 0) epi(t - 1, p0, p1);
    p0 = acc0;
    p1 = acc1;
    vm_wait((DIST - 1) * GW64::RND + EPI * (t > 0 ? 2 : 1));
    block_sync();
    rg.cur++;
  }
}

MLI_FI void extras2(const mli_rgb_fwd_args& a, int r, size_t slot, int h, half8 (&B)[19]) {
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
    B[16][j] = (f16)sel_mask(hm, 0.f, e16[j]);
    B[17][j] = (f16)sel_mask(hm, shl[8 + j], shl[j]);
    B[18][j] = (f16)sel_mask(hm, shv[8 + j], shv[j]);
  }
}

template <bool DEFER>
__global__ __launch_bounds__(256, 1) void rgb_fwd_w64_kernel(mli_rgb_fwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int tile0 = blockIdx.x * 8 + 2 * wave;
  int rc[2];
  size_t sc[2];
#pragma unroll
  for (int col = 0; col < 2; ++col) {
    const int m = (tile0 + col) * 32 + c;
    const int r = m / a.N, k = m - r * a.N;
    rc[col] = r;
    sc[col] = (size_t)k * a.R + r;
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
  extras2(a, rc[0], sc[0], h, B0);
  extras2(a, rc[1], sc[1], h, B1);
#pragma unroll
  for (int d = 0; d < DIST; ++d) ring_issue<GW64, ALL>(rg, lds, bytes);
  vm_wait((DIST - 1) * GW64::RND);
  block_sync();

  uint8_t* fl = lds + GW64::FEAT_OFF + wave * GW64::FEAT_WAVE;
  uint16_t* ft0 = a.feat_frag + (size_t)tile0 * FRAG_TILE;
  uint16_t* ft1 = a.feat_frag + (size_t)(tile0 + 1) * FRAG_TILE;
  run_layer2<16, 8, 0>(rg, lds, B0, B1, lane, bytes, [&](int t, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
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
      if (q < GW64::FKS) {
        *reinterpret_cast<half8*>(fl + q * 1024 + lane * 16) = A0[q];
        *reinterpret_cast<half8*>(fl + (GW64::FKS + q) * 1024 + lane * 16) = A1[q];
      } else {
        reinterpret_cast<half8*>(ft0)[q * 64 + lane] = A0[q];
        reinterpret_cast<half8*>(ft1)[q * 64 + lane] = A1[q];
      }
    }
  });
  for (int hd = 0; hd < a.n_heads; ++hd) {
    {
      const half8* i0 = reinterpret_cast<const half8*>(ft0) + opaque_v(lane);
      const half8* i1 = reinterpret_cast<const half8*>(ft1) + opaque_v(lane);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q < GW64::FKS) {
          B0[q] = *reinterpret_cast<const half8*>(fl + q * 1024 + lane * 16);
          B1[q] = *reinterpret_cast<const half8*>(fl + (GW64::FKS + q) * 1024 + lane * 16);
        } else {
          B0[q] = i0[q * 64];
          B1[q] = i1[q * 64];
        }
      }
    }
    auto relu_epi = [&](half8* o0, half8* o1) MLI_LAMBDA_FI {
      return [&, o0, o1](int t, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
        f32x16 v0, v1;
#pragma unroll
        for (int i = 0; i < 16; ++i) { v0[i] = relu1(acc0[i]); v1[i] = relu1(acc1[i]); }
        o0[2 * t] = acc_to_frag(v0, 0); o0[2 * t + 1] = acc_to_frag(v0, 1);
        o1[2 * t] = acc_to_frag(v1, 0); o1[2 * t + 1] = acc_to_frag(v1, 1);
      };
    };
    if constexpr (DEFER) {
      f32x16 p0, p1;
      auto none = [](f32x16&, f32x16&) MLI_LAMBDA_FI {};
      auto e0 = relu_epi(A0, A1), e1 = relu_epi(B0, B1);
      auto fin = [&](auto& e) MLI_LAMBDA_FI { return [&](f32x16& q0, f32x16& q1) MLI_LAMBDA_FI { e(7, q0, q1); }; };
      run_layer2d<19, 8, 0>(rg, lds, B0, B1, lane, bytes, none, e0, p0, p1);
      run_layer2d<16, 8, 0>(rg, lds, A0, A1, lane, bytes, fin(e0), e1, p0, p1);
      run_layer2d<16, 8, 0>(rg, lds, B0, B1, lane, bytes, fin(e1), e0, p0, p1);
      run_layer2d<16, 8, 0>(rg, lds, A0, A1, lane, bytes, fin(e0), e1, p0, p1);
      e1(7, p0, p1);
    } else {
      run_layer2<19, 8, 0>(rg, lds, B0, B1, lane, bytes, relu_epi(A0, A1));
      run_layer2<16, 8, 0>(rg, lds, A0, A1, lane, bytes, relu_epi(B0, B1));
      run_layer2<16, 8, 0>(rg, lds, B0, B1, lane, bytes, relu_epi(A0, A1));
      run_layer2<16, 8, 0>(rg, lds, A0, A1, lane, bytes, relu_epi(B0, B1));
    }
    const int no = hd == 2 ? 1 : 3;
    const int off = hd * 3;
    run_layer2<16, 1, 0>(rg, lds, B0, B1, lane, bytes, [&](int, const f32x16& acc0, const f32x16& acc1) MLI_LAMBDA_FI {
      if (h == 0) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (i < no) {
            a.y[8 * sc[0] + off + i] = sigmoidf_acc(acc0[i]);
            a.y[8 * sc[1] + off + i] = sigmoidf_acc(acc1[i]);
          }
      }
    });
  }
  vm_wait(0);
}

}  // namespace

int mli_launch_rgb_fwd_w64(const mli_rgb_fwd_args* a, hipStream_t s, int variant) {
  if (variant == 2)
    hipLaunchKernelGGL(rgb_fwd_w64_kernel<true>, dim3(a->R * a->N / 256), dim3(256), GW64::LDS, s, *a);
  else
    hipLaunchKernelGGL(rgb_fwd_w64_kernel<false>, dim3(a->R * a->N / 256), dim3(256), GW64::LDS, s, *a);
  MLI_LAUNCH_CHECK();
}
#endif
