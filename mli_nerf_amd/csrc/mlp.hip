// Fused light-conditioned colour heads on gfx950 MFMA (forward + backward dX chain).
//
// Replaces MLPforNeuralSDF layer 1 (neuralangelo/utils/mlp.py:61-64) and
// LumenRGB.forward 'rgb_r_s' (NeuralLumen/utils/modules.py:148-163) with its three
// MLPwithSkipConnection heads (nerf_util.py:158-196), and their autograd backward.
//
// Structure (one workgroup = 8 waves = 256 samples, one wave = 32 samples):
//  * activations live in registers as MFMA B fragments of the transposed layer
//    Y^T = W X^T (rows = features in the accumulator registers, samples on lanes), so the
//    accumulator of layer l is the B operand of layer l+1 with no lane movement
//    (ACC k-order, guide §3 "accumulator tile as the next MFMA's operand");
//  * weights are pre-packed (mli_pack) into per-n-tile chunks of fp16 A fragments
//    (1 KiB per k-step, one ds_read_b128 per MFMA) + 32 fp32 biases, laid out in exactly
//    the order the kernel consumes them; all 8 waves share each chunk through a
//    register-staged double-buffered LDS pipeline (global loads of chunk c+1 in flight
//    while chunk c feeds the MFMAs).
//  * epilogues are fused: softplus(beta=100) for the SDF feature layer, ReLU (+ bit masks
//    + feature-major activation stores for the weight gradients in training), sigmoid
//    for the outputs.
#include "common.h"

namespace {

constexpr int THREADS = 512;
constexpr int WAVES = 8;
constexpr int BUF = 20480;  // >= 19 KiB + 128 B (largest chunk), multiple of 256
constexpr int CH(int ks) { return ks * 1024 + 128; }
constexpr int FRAG_TILE = 16 * 64 * 8;  // halves per 32-sample tile of a 256-wide frag image
// Feature-major activation tiles ([32 features][256 samples] fp16 per n-tile per workgroup)
// are transposed through LDS so each row leaves as 512 contiguous bytes in 16 B stores.
constexpr int SROW = 256 * 2 + 16;       // staged row stride (16 B pad)
constexpr int STAGE = 32 * SROW;
constexpr int LDS_BYTES = 2 * BUF + 2 * STAGE;

struct Pipe {
  const uint8_t* next;
  u32x4 st[3];
  int bytes;
  int buf;
};

MLI_FI void pipe_issue(Pipe& p, int bytes) {
  p.bytes = bytes;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int o = min((u * THREADS + (int)threadIdx.x) * 16, bytes - 16);
    p.st[u] = *reinterpret_cast<const u32x4*>(p.next + o);
  }
}

MLI_FI void pipe_commit(Pipe& p, uint8_t* lds) {
  uint8_t* dst = lds + (p.buf ^ 1) * BUF;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int o = (u * THREADS + (int)threadIdx.x) * 16;
    if (o < p.bytes) *reinterpret_cast<u32x4*>(dst + o) = p.st[u];
  }
  p.next += p.bytes;
  p.bytes = 0;
}

MLI_FI void pipe_start(Pipe& p, uint8_t* lds, int bytes) {
  p.buf = 1;  // commit writes buffer 0
  pipe_issue(p, bytes);
  pipe_commit(p, lds);
  p.buf = 0;
  __syncthreads();
}

// Double-buffered LDS staging of feature-major tiles: stage_tile() writes a tile (the
// accumulator layout: rows acc_row(i, h), sample column wave*32 + c) into one buffer; the
// next workgroup barrier (inside run_layer) makes it visible and stage_flush() writes it
// out while the other buffer takes the next tile.
struct Stager {
  uint16_t* pend;  // global address of (row 0, first sample of the block) of the staged tile
  int buf, pbuf;
};

MLI_FI void stage_tile(Stager& sg, uint8_t* lds, const f32x16& v, uint16_t* dst, int lane) {
  const int wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  uint8_t* sb = lds + 2 * BUF + sg.buf * STAGE + (4 * h) * SROW + (wave * 32 + c) * 2;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const f16 x = (f16)v[i];
    *reinterpret_cast<uint16_t*>(sb + ((i & 3) + 8 * (i >> 2)) * SROW) = __builtin_bit_cast(uint16_t, x);
  }
  sg.pend = dst;
  sg.pbuf = sg.buf;
  sg.buf ^= 1;
}

MLI_FI void stage_flush(Stager& sg, const uint8_t* lds, int S) {
  if (sg.pend == nullptr) return;
  const int row = threadIdx.x >> 5, col = threadIdx.x & 31;
  const uint8_t* sb = lds + 2 * BUF + sg.pbuf * STAGE;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = row + 16 * u;
    const u32x4 x = *reinterpret_cast<const u32x4*>(sb + r * SROW + col * 16);
    *reinterpret_cast<u32x4*>(sg.pend + (size_t)r * S + col * 8) = x;
  }
  sg.pend = nullptr;
}

// acc = W_chunk (32 x 16*KS) * X (16*KS x 32) + bias
template <int KS>
MLI_FI f32x16 chunk_mma(const uint8_t* chunk, const half8* X, int lane) {
  const int h = lane >> 5;
  f32x16 acc;
  const f32x4* bias = reinterpret_cast<const f32x4*>(chunk + KS * 1024 + h * 64);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 b = bias[u];
    acc[4 * u] = b[0]; acc[4 * u + 1] = b[1]; acc[4 * u + 2] = b[2]; acc[4 * u + 3] = b[3];
  }
  const half8* w = reinterpret_cast<const half8*>(chunk) + lane;
#pragma unroll
  for (int q = 0; q < KS; ++q) acc = mfma32(w[q * 64], X[q], acc);
  // keep at most RA weight fragments in flight (register pressure): RA reads, then one
  // read per MFMA
  constexpr int RA = KS < 4 ? KS : 4;
  __builtin_amdgcn_sched_group_barrier(0x100, RA, 0);
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (q + RA < KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
  return acc;
}

// One layer of NT n-tiles over KS k-steps; `next_bytes` = size of the chunk after this layer.
// epi(t, acc) consumes each finished tile.
template <int KS, int NT, class Epi>
MLI_FI void run_layer(Pipe& p, uint8_t* lds, Stager& sg, int S, const half8* X, int lane, int next_bytes,
                      Epi&& epi) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nb = (t + 1 < NT) ? CH(KS) : next_bytes;
    if (nb) pipe_issue(p, nb);
    const f32x16 acc = chunk_mma<KS>(lds + p.buf * BUF, X, lane);
    if (nb) pipe_commit(p, lds);
    __syncthreads();
    p.buf ^= 1;
    stage_flush(sg, lds, S);
    epi(t, acc);
  }
}

// ---------------------------------------------------------------------- forward
__global__ __launch_bounds__(THREADS) void rgb_fwd_kernel(mli_rgb_fwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tile = blockIdx.x * WAVES + wave;
  const int m = tile * 32 + c;
  const int r = m / a.N, k = m - r * a.N;
  const size_t slot = (size_t)k * a.R + r;
  const bool train = a.xT != nullptr;

  half8 A[16], B[19];
  // h0 frags (SDF layer-0 activations) -> B[0..15]
  {
    const half8* src = reinterpret_cast<const half8*>(a.h0 + (size_t)tile * FRAG_TILE) + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) B[q] = src[q * 64];
  }
  // extras (NAT order): k-step 16 = [p, n, 0...], 17 = SH(light), 18 = SH(view)
  {
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
        // feature-major rows 256..303 (k_nat order) from the fp32 sources
        a.x0T[(size_t)k_nat(16, h, j) * S + m] = __builtin_bit_cast(uint16_t, (f16)v16);
        a.x0T[(size_t)k_nat(17, h, j) * S + m] = __builtin_bit_cast(uint16_t, (f16)v17);
        a.x0T[(size_t)k_nat(18, h, j) * S + m] = __builtin_bit_cast(uint16_t, (f16)v18);
      }
    }
  }

  Pipe pipe;
  pipe.next = reinterpret_cast<const uint8_t*>(a.wfwd);
  pipe_start(pipe, lds, CH(16));
  Stager sg{nullptr, 0, 0};
  const size_t col0 = (size_t)blockIdx.x * 256;

  // SDF layer 1: feat = softplus(W1 h0 + b1) -> A; frag image scratch (+ x0T rows 0..255)
  uint16_t* ftile = a.feat_frag + (size_t)tile * FRAG_TILE;
  run_layer<16, 8>(pipe, lds, sg, S, B, lane, CH(19), [&](int t, const f32x16& acc) MLI_LAMBDA_FI {
    f32x16 v;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = softplus100(acc[i]);
    A[2 * t] = acc_to_frag(v, 0);
    A[2 * t + 1] = acc_to_frag(v, 1);
    half8* dst = reinterpret_cast<half8*>(ftile) + (2 * t) * 64 + lane;
    dst[0] = A[2 * t];
    dst[64] = A[2 * t + 1];
    if (train) stage_tile(sg, lds, v, a.x0T + (size_t)(32 * t) * S + col0, lane);
  });

  for (int hd = 0; hd < 3; ++hd) {
    const int S = opaque_s(a.R * a.N);
    // reload feat frags into B[0..15] (B[16..18] keep the extras); the lane offset is made
    // opaque per head so the 16 addresses are not hoisted out of the head loop (spills)
    {
      const half8* src = reinterpret_cast<const half8*>(ftile) + opaque_v(lane);
#pragma unroll
      for (int q = 0; q < 16; ++q) B[q] = src[q * 64];
    }
    uint32_t mbits[4];
    auto relu_epi = [&](half8* out, int layer) MLI_LAMBDA_FI {
      return [&, out, layer](int t, const f32x16& acc) MLI_LAMBDA_FI {
        f32x16 v;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = fmaxf(acc[i], 0.0f);
        out[2 * t] = acc_to_frag(v, 0);
        out[2 * t + 1] = acc_to_frag(v, 1);
        if (train) {
          uint32_t bits = 0;
#pragma unroll
          for (int i = 0; i < 16; ++i) bits |= (acc[i] > 0.0f ? 1u : 0u) << i;
          if (t & 1) mbits[t >> 1] |= bits << 16; else mbits[t >> 1] = bits;
          stage_tile(sg, lds, v, a.xT + ((size_t)(hd * 4 + layer) * 256 + 32 * t) * S + col0, lane);
          if (t == 7) {
            u32x4* mp = reinterpret_cast<u32x4*>(a.masks) +
                        ((size_t)(hd * 4 + layer) * (S / 32) + tile) * 64 + lane;
            *mp = u32x4{mbits[0], mbits[1], mbits[2], mbits[3]};
          }
        }
      };
    };
    run_layer<19, 8>(pipe, lds, sg, S, B, lane, CH(16), relu_epi(A, 0));
    run_layer<16, 8>(pipe, lds, sg, S, A, lane, CH(16), relu_epi(B, 1));
    run_layer<16, 8>(pipe, lds, sg, S, B, lane, CH(16), relu_epi(A, 2));
    run_layer<16, 8>(pipe, lds, sg, S, A, lane, CH(16), relu_epi(B, 3));
    const int after = (hd < 2) ? CH(19) : 0;
    const int no = hd == 2 ? 1 : 3;
    const int off = hd * 3;
    run_layer<16, 1>(pipe, lds, sg, S, B, lane, after, [&](int, const f32x16& acc) MLI_LAMBDA_FI {
      if (h == 0) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (i < no) a.y[8 * slot + off + i] = sigmoidf_acc(acc[i]);
      }
    });
  }
}

// ---------------------------------------------------------------------- backward dX chain
__global__ __launch_bounds__(THREADS) void rgb_bwd_kernel(mli_rgb_bwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tiles = S / 32;
  const int tile = blockIdx.x * WAVES + wave;
  const int m = tile * 32 + c;
  const int r = m / a.N, k = m - r * a.N;
  const size_t slot = (size_t)k * a.R + r;

  half8 A[16], B[16];
  Pipe pipe;
  pipe.next = reinterpret_cast<const uint8_t*>(a.wbwd);
  pipe_start(pipe, lds, CH(1));
  Stager sg{nullptr, 0, 0};
  const size_t col0 = (size_t)blockIdx.x * 256;
  for (int hd = 0; hd < 3; ++hd) {
    const int S = opaque_s(a.R * a.N);
    const int no = hd == 2 ? 1 : 3;
    half8 z4;
    {
      const float* dz = a.dz4 + 8 * slot + 3 * hd;
#pragma unroll
      for (int j = 0; j < 8; ++j) z4[j] = (f16)0.f;
      if (h == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (j < no) {
            const f16 zj = (f16)dz[j];  // never bit_cast a vector element (yields element 0)
            z4[j] = zj;
            a.dz4T[((size_t)hd * 4 + j) * S + m] = __builtin_bit_cast(uint16_t, zj);
          }
      }
    }
    auto mask_epi = [&](half8* out, int layer /* dZ index */, int mask_layer) MLI_LAMBDA_FI {
      return [&, out, layer, mask_layer](int t, const f32x16& acc) MLI_LAMBDA_FI {
        const u32x4 mv = *(reinterpret_cast<const u32x4*>(a.masks) +
                           ((size_t)(hd * 4 + mask_layer) * tiles + tile) * 64 + lane);
        const uint32_t words[4] = {mv[0], mv[1], mv[2], mv[3]};
        const uint32_t bits = words[t >> 1] >> ((t & 1) * 16);
        f32x16 v;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ((bits >> i) & 1u) ? acc[i] : 0.0f;
        out[2 * t] = acc_to_frag(v, 0);
        out[2 * t + 1] = acc_to_frag(v, 1);
        stage_tile(sg, lds, v, a.dzT + ((size_t)(hd * 4 + layer) * 256 + 32 * t) * S + col0, lane);
      };
    };
    run_layer<1, 8>(pipe, lds, sg, S, &z4, lane, CH(16), mask_epi(A, 3, 3));
    run_layer<16, 8>(pipe, lds, sg, S, A, lane, CH(16), mask_epi(B, 2, 2));
    run_layer<16, 8>(pipe, lds, sg, S, B, lane, CH(16), mask_epi(A, 1, 1));
    run_layer<16, 8>(pipe, lds, sg, S, A, lane, hd < 2 ? CH(1) : 0, mask_epi(B, 0, 0));
  }
  __syncthreads();
  stage_flush(sg, lds, opaque_s(a.R * a.N));
}

}  // namespace

extern "C" int mli_rgb_fwd(const mli_rgb_fwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S % 256 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rgb_fwd_kernel, dim3(S / 256), dim3(THREADS), LDS_BYTES, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_rgb_bwd(const mli_rgb_bwd_args* a, mli_stream_t s) {
  const int S = a->R * a->N;
  if (S % 256 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rgb_bwd_kernel, dim3(S / 256), dim3(THREADS), LDS_BYTES, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}
