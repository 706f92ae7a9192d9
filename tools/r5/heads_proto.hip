// Micro-benchmark: the heads' per-phase pattern (a 32-output x KS chunk read from LDS by every
// wave, 16 dependent MFMAs per tile, ReLU epilogue into the next layer's operand), with one
// 32-sample tile per wave (8 waves) against two tiles per wave (4 waves), 256 samples per WG.
#include "mlp_core.h"
#include <cstdio>
#include <hip/hip_runtime.h>
namespace {
template <int KS, int T>
__device__ __forceinline__ void chunk2(const uint8_t* chunk, half8 (&X)[T][19], f32x16 (&acc)[T], int lane) {
  const half8* w = reinterpret_cast<const half8*>(chunk) + lane;
#pragma unroll
  for (int u = 0; u < T; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[u][e] = 0.f;
  half8 wr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) wr[q] = w[q * 64];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
#pragma unroll
    for (int u = 0; u < T; ++u) acc[u] = mfma32(wr[q % 4], X[u][q], acc[u]);
    if (q + 4 < KS) wr[q % 4] = w[(q + 4) * 64];
  }
}
}
template <int T, int NW>
__global__ __launch_bounds__(NW * 64) void heads_proto(const half8* in, half8* out, int n) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * 20480 / 16; i += NW * 64) reinterpret_cast<u32x4*>(lds)[i] = u32x4{0x3c003c00u, 0x3c003c00u, 0, 0};
  __syncthreads();
  half8 A[T][19], B[T][19];
  const size_t base = ((size_t)blockIdx.x * NW + wave) * T;
#pragma unroll
  for (int u = 0; u < T; ++u)
#pragma unroll
    for (int q = 0; q < 19; ++q) { B[u][q] = in[((base + u) * 19 + q) * 64 + lane]; A[u][q] = B[u][q]; }
  auto layer = [&](auto& X, auto& Y, int b0) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      f32x16 acc[T];
      chunk2<16, T>(lds + ((b0 + t) & 3) * 20480, X, acc, lane);
      if (t & 1) __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int u = 0; u < T; ++u) {
        f32x16 v;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = relu1(acc[u][i]) * 0.001f;
        Y[u][2 * t] = acc_to_frag(v, 0);
        Y[u][2 * t + 1] = acc_to_frag(v, 1);
      }
    }
  };
  for (int hd = 0; hd < n; ++hd) {
    layer(B, A, 0);
    layer(A, B, 1);
    layer(B, A, 2);
    layer(A, B, 3);
  }
#pragma unroll
  for (int u = 0; u < T; ++u)
#pragma unroll
    for (int q = 0; q < 16; ++q) out[((base + u) * 16 + q) * 64 + lane] = A[u][q] + B[u][q];
}
template <int T, int NW>
float run(const half8* in, half8* out, int wgs, int n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((heads_proto<T, NW>), dim3(wgs), dim3(NW * 64), 4 * 20480, 0, in, out, n);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((heads_proto<T, NW>), dim3(wgs), dim3(NW * 64), 4 * 20480, 0, in, out, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}
int main() {
  const int wgs = 2048, n = 3;  // 524288 samples, 3 heads x 4 layers x 8 tiles
  half8 *in, *out;
  hipMalloc(&in, (size_t)wgs * 256 / 32 * 19 * 64 * 16);
  hipMalloc(&out, (size_t)wgs * 256 / 32 * 16 * 64 * 16);
  hipMemset(in, 0, (size_t)wgs * 256 / 32 * 19 * 64 * 16);
  const double flops = 2.0 * 256 * 256 * 256.0 * wgs * n * 4;
  float t1 = run<1, 8>(in, out, wgs, n), t2 = run<2, 4>(in, out, wgs, n);
  printf("1 tile x 8 waves: %.3f ms (%.0f TF/s)\n2 tiles x 4 waves: %.3f ms (%.0f TF/s)\n", t1, flops / t1 / 1e9, t2,
         flops / t2 / 1e9);
  return 0;
}
