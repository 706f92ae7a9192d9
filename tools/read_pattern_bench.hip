// HBM read-pattern micro-benchmark for the weight-gradient operand streams (mli_wgrad BIG).
//
// Each workgroup reads its k-slice of `rows` operand rows in stages of 64 samples (128 B per
// row per stage), as the LDS-DMA ring does, either from the feature-major image [rows][S]
// (row segments 2 S bytes apart) or from a tile-blocked image [S/256][rows][256] (a stage is 4
// segments of one contiguous rows x 512 B block).  Mode `dma` lands the pieces in LDS with
// global_load_lds_dwordx4 through a 2-stage ring (vmcnt + barrier per stage, as the kernel);
// mode `reg` loads them into registers.
//   hipcc -O3 --offload-arch=gfx950 tools/read_pattern_bench.hip -o tools/read_pattern_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_cvoid_t;

// ILV: the workgroups' stages interleaved over k (stage st of workgroup w at k = (st * wgs + w) * 64)
// instead of contiguous k-slices: concurrent workgroups read neighbouring 128 B segments of a row
// JOBS > 1: the grid is JOBS jobs x (grid / JOBS) k-splits, job j reading its own ROWS-row region
// (mli_wgrad BIG: 9 jobs x 28 splits)
template <bool BLOCKED, bool DMA, int ROWS, bool ILV = false, int JOBS = 1>
__global__ __launch_bounds__(512) void read_kernel(const uint16_t* src0, size_t S, size_t k_split, u32x4* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int PIECES = ROWS * 8;  // 16 B pieces per stage
  constexpr int PPT = PIECES / 512;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nsp = gridDim.x / JOBS, job = blockIdx.x / nsp, sp = blockIdx.x - job * nsp;
  const uint16_t* src = src0 + (size_t)job * ROWS * S;
  const size_t T = S / 64;  // 64-sample stages of the whole k range
  const size_t per = k_split / 64;
  // this workgroup's stage i (i < n_st) is global stage gs(i), always < T
  const int n_st = ILV ? (int)((T - sp + nsp - 1) / nsp) : (int)(sp * per >= T ? 0 : (T - sp * per < per ? T - sp * per : per));
  auto gs = [&](int i) -> size_t { return ILV ? (size_t)i * nsp + sp : sp * per + i; };
  auto addr = [&](int p, size_t k) {
    const int row = p >> 3, ch = p & 7;
    return BLOCKED ? src + (k >> 8) * ((size_t)ROWS * 256) + (size_t)row * 256 + (k & 255) + ch * 8
                   : src + (size_t)row * S + k + ch * 8;
  };
  u32x4 acc = {0, 0, 0, 0};
  if (DMA) {
    // piece p = u * 512 + tid -> wave-instruction (u, wave) fills LDS [stage][u * 512 + wave * 64 .. ] x 16 B
    auto issue = [&](int st) {
      const size_t k = gs(max(0, min(st, n_st - 1))) * 64;
      uint8_t* base = lds + (st & 1) * PIECES * 16;
#pragma unroll
      for (int u = 0; u < PPT; ++u)
        __builtin_amdgcn_global_load_lds((gbl_cvoid_t*)addr(u * 512 + tid, k), (lds_void_t*)(base + (u * 512 + wave * 64) * 16), 16, 0, 0);
    };
    if (n_st == 0) return;
    issue(0);
    for (int st = 0; st < n_st; ++st) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      issue(st + 1);
      const uint8_t* base = lds + (st & 1) * PIECES * 16;
      acc ^= *reinterpret_cast<const u32x4*>(base + tid * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int st = 0; st < n_st; ++st) {
      const size_t k = gs(st) * 64;
#pragma unroll
      for (int u = 0; u < PPT; ++u) acc ^= *reinterpret_cast<const u32x4*>(addr(u * 512 + tid, k));
    }
  }
  if (acc[0] == 0x12345678u) out[blockIdx.x * 512 + tid] = acc;
}

template <bool BLOCKED, bool DMA, int ROWS, bool ILV = false, int JOBS = 1>
float run(const uint16_t* src, size_t S, int wgs, u32x4* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9f;
  const size_t k_split = (S / 64 + wgs / JOBS - 1) / (wgs / JOBS) * 64;
  const int lds = DMA ? 2 * ROWS * 8 * 16 : 0;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((read_kernel<BLOCKED, DMA, ROWS, ILV, JOBS>), dim3(wgs), dim3(512), lds, 0, src, S, k_split, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const size_t S = 524288;
  constexpr int ROWS = 512;  // BIG: dZ_l (256 rows) + X_l (256 rows)
  uint16_t* src;
  u32x4* out;
  const size_t bytes = (size_t)ROWS * S * 2 * 9;  // 9 jobs' worth, each launch reads one job region
  hipMalloc(&src, bytes);
  hipMalloc(&out, 4096 * 512 * 16);
  hipMemset(src, 1, bytes);
  for (int wgs : {256, 512}) {
    const double gb = (double)ROWS * S * 2 / 1e9;
    float t;
    t = run<false, true, ROWS>(src, S, wgs, out);
    printf("wgs %d  rows    dma : %.3f ms  %.2f TB/s\n", wgs, t, gb / t);
    t = run<true, true, ROWS>(src, S, wgs, out);
    printf("wgs %d  blocked dma : %.3f ms  %.2f TB/s\n", wgs, t, gb / t);
    t = run<false, false, ROWS>(src, S, wgs, out);
    printf("wgs %d  rows    reg : %.3f ms  %.2f TB/s\n", wgs, t, gb / t);
    t = run<true, false, ROWS>(src, S, wgs, out);
    printf("wgs %d  blocked reg : %.3f ms  %.2f TB/s\n", wgs, t, gb / t);
    t = run<false, true, ROWS, true>(src, S, wgs, out);
    printf("wgs %d  rows interleaved dma : %.3f ms  %.2f TB/s\n", wgs, t, gb / t);
  }
  {  // BIG's shape: 9 jobs x 28 splits, each job its own 512 rows
    const double gb = 9.0 * ROWS * S * 2 / 1e9;
    float t;
    t = run<false, true, ROWS, false, 9>(src, S, 252, out);
    printf("9 jobs x 28  rows    dma : %.3f ms  %.2f TB/s\n", t, gb / t);
    t = run<false, true, ROWS, true, 9>(src, S, 252, out);
    printf("9 jobs x 28  rows interleaved dma : %.3f ms  %.2f TB/s\n", t, gb / t);
    t = run<true, true, ROWS, false, 9>(src, S, 252, out);
    printf("9 jobs x 28  blocked dma : %.3f ms  %.2f TB/s\n", t, gb / t);
  }
  return 0;
}
