// HBM write-pattern micro-benchmark for the training activation images.
//
// The heads forward / backward write feature-major rows [rows][S] fp16: every 256-sample
// workgroup leaves one 512 B segment per row, rows S*2 bytes apart ("rows").  The
// alternative is a tile-blocked image [S/256][rows][256]: the same workgroup's segments are
// contiguous ("blocked").  Both write the same bytes with 16 B non-temporal stores, 512
// threads per workgroup, one workgroup per 256 samples.
//   hipcc -O3 --offload-arch=gfx950 tools/write_pattern_bench.hip -o /tmp/wpb && /tmp/wpb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool BLOCKED>
__global__ __launch_bounds__(512) void write_kernel(uint16_t* dst, size_t S, int rows) {
  const int tid = threadIdx.x;
  const size_t col0 = (size_t)blockIdx.x * 256;
  // 32 threads per 512 B row segment, 16 rows per pass
  for (int r0 = 0; r0 < rows; r0 += 16) {
    const int row = r0 + (tid >> 5), c = (tid & 31) * 8;
    if (row >= rows) break;
    uint16_t* p = BLOCKED ? dst + ((size_t)blockIdx.x * rows + row) * 256 + c : dst + (size_t)row * S + col0 + c;
    __builtin_nontemporal_store(u32x4{(uint32_t)row, (uint32_t)c, 1u, 2u}, reinterpret_cast<u32x4*>(p));
  }
}

int main() {
  const size_t S = 524288 * 2;
  const int rows = 1536;  // 3 heads x 2 layers x 256 rows: 3.2 GB per launch
  uint16_t* d;
  const size_t bytes = S * rows * 2;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode) {
    for (int it = 0; it < 3; ++it) {
      if (mode) write_kernel<true><<<S / 256, 512>>>(d, S, rows);
      else write_kernel<false><<<S / 256, 512>>>(d, S, rows);
    }
    hipEventRecord(e0);
    const int reps = 10;
    for (int it = 0; it < reps; ++it) {
      if (mode) write_kernel<true><<<S / 256, 512>>>(d, S, rows);
      else write_kernel<false><<<S / 256, 512>>>(d, S, rows);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-8s %.3f ms per launch  %.2f TB/s  (%.2f GB)\n", mode ? "blocked" : "rows", ms, bytes / (ms * 1e-3) / 1e12,
           bytes / 1e9);
  }
  hipFree(d);
  return 0;
}
