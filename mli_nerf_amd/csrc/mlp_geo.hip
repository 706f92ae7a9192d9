// Stage-a geometry dX chain (the shared heads machinery: mlp_core.h).
#include "mlp_core.h"

namespace {

// ---------------------------------------------------------------------- stage a: geometry dX chain
// The single 'rgb' head (NeuralLumen/utils/modules.py:164-174) backward down to its inputs,
// then SDF layer 1.  Chunks: W4^T (8 x KS 1), W3^T, W2^T, W1^T (24 x KS 16), W0^T (9 n-tiles
// over packed input rows 0..287: feat (ACC order) + the p/normal k-step), W1sdf^T (8 x KS 16).
MLI_FI int geo_bytes(int c) { return c < 8 ? CH(1) : CH(16); }
constexpr int GEO_CHUNKS = 8 + 24 + 9 + 8;

typedef Geo<8, 17, false, 4> GGeo;

__global__ __launch_bounds__(GGeo::THREADS) void geo_bwd_kernel(mli_geo_bwd_args a) {
  typedef GGeo G;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tiles = S / 32;
  const int tile = blockIdx.x * G::NW + wave;
  const int m = tile * 32 + c;
  const int r = m / a.N, k = m - r * a.N;
  const size_t slot = (size_t)k * a.R + r;
  auto bytes = [](int cc) MLI_LAMBDA_FI { return geo_bytes(cc); };
  // ReLU-mask block of head layer 3 - L (L = 0..3), one 16 B DMA per thread into slot L & 1
  auto mask_dma = [&](int L) MLI_LAMBDA_FI {
    const int ml = 3 - min(L, 3);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.masks) +
                         (((size_t)ml * tiles + (size_t)blockIdx.x * G::NW) * 64) * 16;
    glds16(src + threadIdx.x * 16, lds + G::MASK_OFF + (L & 1) * G::MASKB + wave * 1024);
  };

  Ring rg;
  ring_start(rg, a.wgeo, GEO_CHUNKS, bytes);
  mask_dma(0);
#pragma unroll
  for (int d = 0; d < DIST; ++d) ring_issue<G, ALL>(rg, lds, bytes);
  vm_wait((DIST - 1) * G::template ring_ops<ALL>());
  block_sync();

  half8 A[16], B[16];
  half8 z4;
  {
    const float* dz = a.dz4 + 8 * slot;
#pragma unroll
    for (int j = 0; j < 8; ++j) z4[j] = (f16)0.f;
    if (h == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) z4[j] = (f16)dz[j];
    }
    // the output layer's dW operand: a one-k-step fragment image (rows 0..2)
    gstore_nt(reinterpret_cast<half8*>(a.dz4T + (size_t)tile * FRAG_KS) + lane, z4);
  }
  struct MaskPre {
    decltype(mask_dma)& dma;
    int next_layer;
    MLI_FI int count(int t) const { return t == 8 - DIST ? 1 : 0; }
    MLI_FI void issue(int t) const {
      if (t == 8 - DIST) dma(next_layer);
    }
  };
  auto pre = [&](int li) MLI_LAMBDA_FI { return MaskPre{mask_dma, li + 1}; };
  auto mask_epi = [&](half8* out, int layer, int li) MLI_LAMBDA_FI {
    return [&, out, layer, li](int t, const f32x16& acc) MLI_LAMBDA_FI {
      const u32x4 mv =
          *reinterpret_cast<const u32x4*>(lds + G::MASK_OFF + (li & 1) * G::MASKB + wave * 1024 + lane * 16);
      const int wi = t >> 1;
      const uint32_t word = wi == 0 ? mv[0] : wi == 1 ? mv[1] : wi == 2 ? mv[2] : mv[3];
      f32x16 v;
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = mask_bit(acc[i], word, (t & 1) * 16 + i);
      out[2 * t] = acc_to_frag(v, 0);
      out[2 * t + 1] = acc_to_frag(v, 1);
      frag_store2(a.dzT + ((size_t)layer * tiles + tile) * FRAG_TILE, t, out[2 * t], out[2 * t + 1], lane);
    };
  };
  run_layer<G, ALL, 1, 8, 2, false>(rg, lds, &z4, lane, bytes, pre(0), mask_epi(A, 3, 0));
  run_layer<G, ALL, 16, 8, 2, false>(rg, lds, A, lane, bytes, pre(1), mask_epi(B, 2, 1));
  run_layer<G, ALL, 16, 8, 2, false>(rg, lds, B, lane, bytes, pre(2), mask_epi(A, 1, 2));
  run_layer<G, ALL, 16, 8, 2, false>(rg, lds, A, lane, bytes, NoPre{}, mask_epi(B, 0, 3));
  // feat frags (softplus output of SDF layer 1, forward scratch), one tile ahead of its use:
  // tile 0 now, tile t+1 ahead of phase t's weight DMAs (counted as pre-issued VMEM ops).  Asm
  // loads (gload16) waited with counted vmcnts in the epilogue: compiler-visible loads among the
  // epilogue stores made it wait vmcnt(0) -- for the phase's weight DMAs too -- every phase.
  const half8* fsrc = reinterpret_cast<const half8*>(a.feat_frag + (size_t)tile * X0_TILE) + lane;
  half8 F[2][2];
  F[0][0] = gload16(fsrc);
  F[0][1] = gload16(fsrc + 64);
  struct FeatPre {
    const half8* src;
    half8 (&F)[2][2];
    MLI_FI int count(int t) const { return t < 7 ? 2 : 0; }
    MLI_FI void issue(int t) const {
      if (t < 7) {
        F[(t + 1) & 1][0] = gload16(src + (2 * t + 2) * 64);
        F[(t + 1) & 1][1] = gload16(src + (2 * t + 3) * 64);
      }
    }
  };
  constexpr int RO = G::template ring_ops<ALL>();
  // dX0 = W0^T dZ0: tiles 0..7 = d feat -> dZ1sdf = d feat * softplus'(z1), with
  // softplus'(z1) = 1 - exp(-100 feat) (torch: z/(z+1), z = e^{100 z1}; 1 past the threshold);
  // tile 8 = rows 256..287 (p 256..258, normal 259..261: (i=3,h=0), (i=0,h=1), (i=1,h=1))
  run_layer<G, ALL, 16, 9, 2, false>(rg, lds, B, lane, bytes, FeatPre{fsrc, F},
                                   [&](int t, const f32x16& acc) MLI_LAMBDA_FI {
    if (t < 8) {
      // tile t's feat loads: issued before the layer (t = 0) or at phase t - 1; after them went
      // phase t-1's DMAs and 2 epilogue stores (t >= 1), phase t's 2 loads of tile t+1 (t < 7)
      // and its DMAs
      vm_wait(t == 0 ? 2 + RO : RO + 2 + (t < 7 ? 2 : 0) + RO);
      tie(F[t & 1][0]);
      tie(F[t & 1][1]);
      f32x16 v;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)F[t & 1][s2][j];
          v[8 * s2 + j] = acc[8 * s2 + j] * (1.0f - __expf(-100.0f * f));
        }
      A[2 * t] = acc_to_frag(v, 0);
      A[2 * t + 1] = acc_to_frag(v, 1);
      frag_store2(a.dz1T + (size_t)tile * FRAG_TILE, t, A[2 * t], A[2 * t + 1], lane);
    } else {
      // (three store instructions, the lane halves diverging; counted as the EPI 2 of tiles 0..7:
      // undercounting only waits longer)
      float* dn = a.d_nrm + 4 * slot;
      if (h == 0) {
        gstore_f32(dn, acc[3]);
      } else {
        gstore_f32(dn + 1, acc[0]);
        gstore_f32(dn + 2, acc[1]);
      }
    }
  });
  // d h0 (layer-1 path) = W1sdf^T dZ1sdf -> frag image (ACC order, as the h0 image)
  uint16_t* dtile = a.dh0_frag + (size_t)tile * FRAG_TILE;
  run_layer<G, ALL, 16, 8, 2, false>(rg, lds, A, lane, bytes, NoPre{},
                                    [&](int t, const f32x16& acc) MLI_LAMBDA_FI {
    half8* dst = reinterpret_cast<half8*>(dtile) + (2 * t) * 64 + lane;
    gstore_nt(dst, acc_to_frag(acc, 0));
    gstore_nt(dst + 64, acc_to_frag(acc, 1));
  });
  vm_wait(0);
}

}  // namespace

extern "C" int mli_geo_bwd_workspace(const mli_geo_bwd_args* a, int64_t* bytes) {
  const int64_t S = (int64_t)a->R * a->N;
  if (S <= 0 || S % 256 != 0) return (int)hipErrorInvalidValue;
  bytes[0] = 4 * 256 * S * 2;  // dzT
  bytes[1] = S * 16 * 2;       // dz4T (one-k-step fragment image)
  bytes[2] = S * 4 * 4;        // d_nrm
  bytes[3] = 256 * S * 2;      // dz1T
  bytes[4] = S * 256 * 2;      // dh0_frag
  bytes[5] = 0;
  return 0;
}

extern "C" int mli_geo_bwd(const mli_geo_bwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S % 256 != 0) return (int)hipErrorInvalidValue;
  if (!a->dz4 || !a->wgeo || !a->masks || !a->feat_frag || !a->dzT || !a->dz4T || !a->d_nrm || !a->dz1T ||
      !a->dh0_frag)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(geo_bwd_kernel, dim3(S / GGeo::SAMPLES), dim3(GGeo::THREADS), GGeo::LDS_BWD, (hipStream_t)s,
                     *a);
  MLI_LAUNCH_CHECK();
}

