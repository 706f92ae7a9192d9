// Micro-benchmark of scattered fp32 / packed-16-bit atomics on gfx950 (design input for
// mli_hash_bwd): 8-feature slots of 32 B at random slot indices in a table of T slots.
//   lane8:  each lane adds its 8 features with 8 global_atomic_add_f32 (lane-private slot)
//   coal8:  8 lanes share a slot, one feature each (one instruction covers 8 slots)
//   pk16:   each lane adds 8 halves with 4 global_atomic_pk_add_f16 (fp16 table)
//   store8: plain 32 B store per lane (no atomic) for reference
// hipcc --offload-arch=gfx950 -O3 tools/atomic_bench.hip -o exp/atomic_bench
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void scatter(float* t, uint32_t slots, uint32_t per_thread, uint32_t seed) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = 0; i < per_thread; ++i) {
    if (MODE == 0) {  // lane8
      const uint32_t s = hash32(gid * per_thread + i + seed) % slots;
      float* p = t + (size_t)s * 8;
#pragma unroll
      for (int f = 0; f < 8; ++f) unsafeAtomicAdd(p + f, 1.0f);
    } else if (MODE == 1) {  // coal8: lane group of 8 -> one slot; 8 iterations = 8 slots / lane-group
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t s = hash32(((gid >> 3) * per_thread + i) * 8 + k + seed) % slots;
        unsafeAtomicAdd(t + (size_t)s * 8 + (gid & 7), 1.0f);
      }
    } else if (MODE == 2) {  // pk16
      const uint32_t s = hash32(gid * per_thread + i + seed) % slots;
      __half2* p = reinterpret_cast<__half2*>(reinterpret_cast<__half*>(t) + (size_t)s * 8);
#pragma unroll
      for (int f = 0; f < 4; ++f) unsafeAtomicAdd(p + f, __half2{(__half)1.0f, (__half)1.0f});
    } else {  // store8
      const uint32_t s = hash32(gid * per_thread + i + seed) % slots;
      float4* p = reinterpret_cast<float4*>(t + (size_t)s * 8);
      p[0] = float4{1.f, 1.f, 1.f, 1.f};
      p[1] = float4{1.f, 1.f, 1.f, 1.f};
    }
  }
}

int main() {
  const size_t max_slots = 45724048;  // the stage-a table: 45.7 M entries x 8 features
  float* t;
  hipMalloc(&t, max_slots * 32);
  hipMemset(t, 0, max_slots * 32);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint32_t threads = 256 * 4096, per = 8;  // 8.4 M slot updates = 67 M fp32 adds per launch
  const char* names[4] = {"lane8", "coal8", "pk16", "store8"};
  const size_t sizes[5] = {1u << 12, 1u << 16, 1u << 19, 1u << 22, max_slots};
  for (int mode = 0; mode < 4; ++mode)
    for (size_t si = 0; si < 5; ++si) {
      const uint32_t slots = (uint32_t)sizes[si];
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        if (mode == 0) scatter<0><<<threads / 256, 256>>>(t, slots, per, rep);
        if (mode == 1) scatter<1><<<threads / 256, 256>>>(t, slots, per, rep);
        if (mode == 2) scatter<2><<<threads / 256, 256>>>(t, slots, per, rep);
        if (mode == 3) scatter<3><<<threads / 256, 256>>>(t, slots, per, rep);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 2)
          printf("%-6s slots %9u (%8.1f MiB): %7.3f ms  %6.2f G slot-updates/s\n", names[mode], slots,
                 slots * 32.0 / 1048576.0, ms, threads * (double)per / ms / 1e6);
      }
    }
  hipFree(t);
  return 0;
}
