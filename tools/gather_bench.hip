// Micro-benchmark: the rate of random 16 B gathers (the hash-grid corner loads) by how many
// distinct 128 B lines one wave-instruction touches.  Mode 0: every lane a random line (64
// lines per instruction); mode 1: lane pairs read the two halves of one 32 B block (32 lines);
// mode 2: lane quads in one 64 B block (16 lines).  Same number of lanes and bytes loaded.
// Build: hipcc -O3 --offload-arch=gfx950 tools/gather_bench.hip -o tools/gather_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gather_kernel(const u32x4* __restrict__ table, uint32_t mask, int iters,
                                                     int mode, u32x4* out) {
  const int lane = threadIdx.x & 63;
  uint32_t s = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + 12345u;
  u32x4 acc = {0, 0, 0, 0};
  const int grp = mode == 0 ? 1 : (mode == 1 ? 2 : 4);
  for (int it = 0; it < iters; ++it) {
    uint32_t idx[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      // the group's leader draws the block; members take consecutive 16 B entries of it
      uint32_t r = (s ^ (c * 0x9E3779B9u)) * 747796405u + 2891336453u;
      r = (r >> 7) ^ r;
      const int lead = lane & ~(grp - 1);
      const uint32_t rl = __shfl(r, lead);
      idx[c] = ((rl & mask) & ~(uint32_t)(grp - 1)) + (lane & (grp - 1));
    }
    u32x4 v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = table[idx[c]];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc += v[c];
    s = s * 1664525u + 1013904223u + acc[0];
  }
  if (acc[0] == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const uint32_t entries = 1u << 22;  // 64 MiB of 16 B entries (one hashed level)
  u32x4* table;
  u32x4* out;
  hipMalloc(&table, (size_t)entries * 16);
  hipMalloc(&out, 256 * 1024 * 16);
  hipMemset(table, 1, (size_t)entries * 16);
  const int blocks = 256 * 12, iters = 64;  // 12 waves x 4 per CU: the encode5 occupancy
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (uint32_t ent : {entries, entries >> 4, entries >> 6})
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, 0, table, ent - 1, iters, mode, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double instr = (double)blocks * 4 * iters * 8;  // wave-instructions
    const double lanes = instr * 64;
    printf("table %5.1f MiB  mode %d (%2d lines/instr): %.3f ms  %.1f G lane-gathers/s  %.1f cycles/instr/CU at 2.4 GHz\n", ent * 16.0 / 1048576, mode,
           mode == 0 ? 64 : (mode == 1 ? 32 : 16), best, lanes / best / 1e6, best * 1e-3 * 2.4e9 * 256 / instr);
  }
  return 0;
}
