// Micro-benchmark: the heads' layer chain with the weights stationary.
//
//   chain  -- the product pattern (tools/r5/heads_proto.hip, T = 1): each of the 8 waves of a
//             256-sample workgroup owns one 32-sample tile; its activations stay in registers and
//             every n-tile's weight chunk (16 k-steps x 1 KiB of A fragments) is read from LDS by
//             every wave: 8 waves x 8 n-tiles x 16 KiB = 1 MiB of LDS reads per layer and CU.
//   ws     -- weights stationary: each wave owns one n-tile of the layer for all 8 sample tiles;
//             its 16 A fragments are loaded once per layer into VGPRs (from L2), the activations
//             (the B operand, 8 tiles x 16 k-steps x 1 KiB = 128 KiB) are streamed from LDS:
//             8 waves x 8 tiles x 16 KiB = the same 1 MiB of LDS reads, plus 16 KiB of LDS writes
//             per wave for the layer output and the barriers that fence it (all waves must have
//             read a tile before it is overwritten).  ws2 computes the layer in two halves of 4
//             tiles (64 accumulator registers instead of 128; 3 barriers per layer).
//
// No weight DMA and no HBM stores in any arm: the chain pattern alone.  Random fp16 data.
// Build / run (GPU box): see tools/r6/heads_ws.sh.
#include "mlp_core.h"

#include <cstdio>
#include <hip/hip_runtime.h>

namespace {

template <int KS>
__device__ __forceinline__ void chunk_chain(const uint8_t* chunk, const half8 (&X)[19], f32x16& acc, int lane) {
  const half8* w = reinterpret_cast<const half8*>(chunk) + lane;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  half8 wr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) wr[q] = w[q * 64];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    acc = mfma32(wr[q % 4], X[q], acc);
    if (q + 4 < KS) wr[q % 4] = w[(q + 4) * 64];
  }
}

__device__ __forceinline__ half8 scale_relu(const f32x16& acc, int half) {
  f32x16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = relu1(acc[i]) * 0.001f;
  return acc_to_frag(v, half);
}

// chain: 1 tile per wave, weights from an LDS ring (the product's phase pattern, 2 n-tiles per barrier)
__global__ __launch_bounds__(512) void chain_kernel(const half8* in, half8* out, int n) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * 16384 / 16; i += 512)
    reinterpret_cast<half8*>(lds)[i] = in[i % 4096];
  __syncthreads();
  half8 A[19], B[19];
  const size_t tile = (size_t)blockIdx.x * 8 + wave;
#pragma unroll
  for (int q = 0; q < 19; ++q) B[q] = A[q] = in[(tile * 19 + q) * 64 + lane];
  auto layer = [&](auto& X, auto& Y, int b0) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      f32x16 acc;
      chunk_chain<16>(lds + ((b0 + t) & 3) * 16384, X, acc, lane);
      if (t & 1) __builtin_amdgcn_s_barrier();
      Y[2 * t] = scale_relu(acc, 0);
      Y[2 * t + 1] = scale_relu(acc, 1);
    }
  };
  for (int hd = 0; hd < n; ++hd) {
    layer(B, A, 0);
    layer(A, B, 1);
    layer(B, A, 2);
    layer(A, B, 3);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) out[(tile * 16 + q) * 64 + lane] = A[q] + B[q];
}

// ws: weights stationary in VGPRs, activations in LDS [tile][k-step][lane] (1 KiB per fragment)
template <int HALVES>
__global__ __launch_bounds__(512) void ws_kernel(const half8* in, const half8* wts, half8* out, int n) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  half8* X = reinterpret_cast<half8*>(lds);  // [8 tiles][16 k-steps][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t t0 = (size_t)blockIdx.x * 8;
  for (int i = threadIdx.x; i < 8 * 16 * 64; i += 512) {
    const int t = i / 1024, q = (i / 64) & 15, l = i & 63;
    X[i] = in[((t0 + t) * 19 + q) * 64 + l];
  }
  __syncthreads();
  constexpr int TPH = 8 / HALVES;  // tiles per half
  for (int li = 0; li < 4 * n; ++li) {
    // this wave's n-tile of layer li: 16 A fragments (L2-resident weights, [layer][n-tile][q][lane])
    half8 W[16];
    const half8* wl = wts + ((size_t)(li & 3) * 8 + wave) * 16 * 64 + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) W[q] = wl[q * 64];
#pragma unroll
    for (int hf = 0; hf < HALVES; ++hf) {
      f32x16 acc[TPH];
#pragma unroll
      for (int u = 0; u < TPH; ++u) {
        const half8* xb = X + (size_t)((hf * TPH + u) * 16) * 64 + lane;
        half8 br[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) br[q] = xb[q * 64];
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[u][e] = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          acc[u] = mfma32(W[q], br[q % 4], acc[u]);
          if (q + 4 < 16) br[q % 4] = xb[(q + 4) * 64];
        }
      }
      __syncthreads();  // every wave has read these tiles: their slots take the layer output
#pragma unroll
      for (int u = 0; u < TPH; ++u) {
        half8* yb = X + (size_t)((hf * TPH + u) * 16 + 2 * wave) * 64 + lane;
        yb[0] = scale_relu(acc[u], 0);
        yb[64] = scale_relu(acc[u], 1);
      }
    }
    __syncthreads();  // the layer output is complete before the next layer reads it
  }
  for (int i = threadIdx.x; i < 8 * 16 * 64; i += 512) {
    const int t = i / 1024, q = (i / 64) & 15, l = i & 63;
    out[((t0 + t) * 16 + q) * 64 + l] = X[i];
  }
}

__global__ void init_kernel(half8* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    half8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t x = (uint32_t)(i * 8 + j) * 2654435761u ^ seed;
      x ^= x >> 15;
      x *= 2246822519u;
      x ^= x >> 13;
      v[j] = (f16)(((float)(x & 0xFFFF) / 65535.0f - 0.5f) * 0.125f);
    }
    p[i] = v;
  }
}

template <class F>
float time_it(F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) launch();
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

}  // namespace

int main() {
  const int wgs = 2048, n = 3;  // 524288 samples; 3 heads x 4 layers of 256 x 256
  const size_t n_in = (size_t)wgs * 8 * 19 * 64, n_out = (size_t)wgs * 8 * 16 * 64, n_w = 4 * 8 * 16 * 64;
  half8 *in, *out, *wts;
  hipMalloc(&in, n_in * 16);
  hipMalloc(&out, n_out * 16);
  hipMalloc(&wts, n_w * 16);
  hipLaunchKernelGGL(init_kernel, dim3(1024), dim3(256), 0, 0, in, n_in, 1u);
  hipLaunchKernelGGL(init_kernel, dim3(64), dim3(256), 0, 0, wts, n_w, 7u);
  hipDeviceSynchronize();
  const double flops = 2.0 * 256 * 256 * 256.0 * wgs * n * 4;
  for (int rep = 0; rep < 2; ++rep) {
    const float tc = time_it([&] {
      hipLaunchKernelGGL(chain_kernel, dim3(wgs), dim3(512), 4 * 16384, 0, in, out, n);
    });
    const float tw = time_it([&] {
      hipLaunchKernelGGL((ws_kernel<1>), dim3(wgs), dim3(512), 8 * 16 * 1024, 0, in, wts, out, n);
    });
    const float tw2 = time_it([&] {
      hipLaunchKernelGGL((ws_kernel<2>), dim3(wgs), dim3(512), 8 * 16 * 1024, 0, in, wts, out, n);
    });
    printf("chain (1 tile / wave, weights from LDS)   %.3f ms  %.0f TF/s\n", tc, flops / tc / 1e9);
    printf("ws    (weights in VGPRs, X in LDS, 8 tiles) %.3f ms  %.0f TF/s\n", tw, flops / tw / 1e9);
    printf("ws2   (weights in VGPRs, 2 x 4 tiles)       %.3f ms  %.0f TF/s\n", tw2, flops / tw2 / 1e9);
  }
  hipError_t e = hipGetLastError();
  printf("status %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
