// Shared device helpers for the gfx950 kernels of libmli_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "mli_hip.h"

typedef _Float16 f16;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));
typedef __attribute__((address_space(3))) fp16x4_t lds_fp16x4_t;

#define MLI_FI __device__ __forceinline__

// ds_read_b64_tr_b16 (gfx950): a 16-lane group reads a 4-row x 16-column block of 16-bit
// elements; lane 4q+p of the group supplies the address of row q, columns 4p..4p+3 (8 B),
// lane i receives column i of the 4 rows (row q in element q).  EXEC must be all ones.
// (the builtin makes the compiler wait vmcnt(0) before it whenever an LDS-DMA is in flight: it
// cannot tell the read from the DMA's destination -- fine outside DMA loops; inside them use
// ds_tr16_at below)
MLI_FI half4 ds_read_tr16(const void* lds_addr) {
  return __builtin_bit_cast(half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_fp16x4_t*)lds_addr));
}
#define MLI_LAMBDA_FI __attribute__((always_inline))

// 32-bit LDS address of a pointer into the workgroup's LDS
MLI_FI uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)p);
}
// The same transposed read as inline asm, at byte offset OFF from a 32-bit LDS address: the
// compiler sees no LDS access, so it adds neither the vmcnt(0) wait behind in-flight LDS-DMAs
// (measured: with the builtin every k-slice stage of mli_wgrad waited for the NEXT stage's
// DMAs before its first read, so DMA and MFMA never overlapped) nor any lgkmcnt wait for the
// result: the caller waits with lgkm_wait() and ties the results with tie() before use.
template <int OFF>
MLI_FI half4 ds_tr16_at(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  half4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
// A 16 B global load as inline asm.  Loads, stores and LDS-DMAs of a wave retire in issue order
// (MI355X_MICROARCH.md, vmcnt), but the compiler treats a counter with loads AND stores pending
// as out of order and waits vmcnt(0) for any load result -- draining the weight DMAs and the
// activation stores in flight.  The caller waits with a counted vm_wait() (common.h) and tie()s
// the result; the memory clobber keeps the compiler's own VMEM ops on their side of it, so the
// counts stay exact.
MLI_FI half8 gload16(const void* p) {
  half8 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

// Global stores as inline asm (the heads / geometry kernels): with no store visible to it, the
// compiler counts the loads and LDS-DMAs it waits for as in order and waits exactly, instead of
// vmcnt(0) (see gload16).  No memory clobber: they may move among the compiler's own memory ops
// inside a phase, never across the volatile vm_wait / block_sync asm -- all the counted waits
// need.  (A later load of the same address by the same wave is ordered by the hardware.)
// (the s_nop 1: a VALU write of the data registers right after a dwordx4 store would change what
// it stores; hipcc pads its own stores, not asm ones -- the first build without it stored
// address bits into the x0 image)
MLI_FI void gstore_nt(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v));
}
MLI_FI void gstore_nt(void* p, half8 v) { gstore_nt(p, __builtin_bit_cast(u32x4, v)); }
MLI_FI void gstore_nt(void* p, f32x4 v) { gstore_nt(p, __builtin_bit_cast(u32x4, v)); }
MLI_FI void gstore(void* p, half8 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(__builtin_bit_cast(u32x4, v)));
}
MLI_FI void gstore_f32(void* p, float v) { asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v)); }

// LDS writes as inline asm: a compiler-visible LDS write while an LDS-DMA may be in flight is
// preceded by vmcnt(0) (the compiler cannot tell it from the DMA's destination).  The caller
// orders them against plain LDS accesses with asm("" ::: "memory") fences (LDS operations of a
// wave execute in order, so no wait is needed between a write and a later read of it).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
MLI_FI void ds_write_u16(uint32_t addr, uint32_t v) { asm volatile("ds_write_b16 %0, %1" ::"v"(addr), "v"(v)); }
MLI_FI void ds_write_u64(uint32_t addr, u32x2 v) { asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v)); }
MLI_FI void ds_write_f128(uint32_t addr, f32x4 v) {
  asm volatile("ds_write_b128 %0, %1\n\ts_nop 1" ::"v"(addr), "v"(v));
}

template <int N>
MLI_FI void lgkm_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt field");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}
// orders every later use of x behind the asm statements before it (an lgkm_wait)
template <class T>
MLI_FI void tie(T& x) {
  asm volatile("" : "+v"(x));
}
// f(std::integral_constant<int, I>) for I = 0 .. N-1, each I a constant expression
template <class F, int... I>
MLI_FI void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
MLI_FI void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// D = A(32x16) * B(16x32) + C on one wave (gfx950 v_mfma_f32_32x32x16_f16).
// Lane l (r = l & 31, h = l >> 5) holds A[r][k(h,j)] and B[k(h,j)][r] in element j;
// D register i of lane l is element (row = acc_row(i, h), col = r).
MLI_FI f32x16 mfma32(half8 a, half8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// Row of the 32x32 D tile held by accumulator register i in lane half h.
MLI_FI int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Packed-k index of element j, lane half h, k-step q:
//   NAT: the natural B-operand order; ACC: the order an accumulator tile has when its
//   registers 8s..8s+7 are reused as the B fragment of k-step 2t+s (guide §3).
MLI_FI int k_nat(int q, int h, int j) { return 16 * q + 8 * h + j; }
MLI_FI int k_acc(int q, int h, int j) { return 16 * q + 8 * (j >> 2) + 4 * h + (j & 3); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 half2 __attribute__((ext_vector_type(2)));

// Convert accumulator registers [8s, 8s+8) to the fp16 B fragment of k-step 2t+s: four
// v_cvt_pk_f16_f32 (round to nearest even, as the element-wise cast).  Written pairwise so the
// fragment is built from packed words; element-wise casts whose halves are also needed one by
// one (LDS staging) were assembled from 16 v_cvt_f16_f32 + 64 v_perm_b32 per 32 x 32 tile.
MLI_FI half8 acc_to_frag(const f32x16& v, int s) {
  u32x4 w;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    f32x2 f;
    f.x = v[8 * s + 2 * p];
    f.y = v[8 * s + 2 * p + 1];
    w[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, half2));
  }
  return __builtin_bit_cast(half8, w);
}

// torch.nn.functional.softplus(x, beta=100, threshold=20) as max(x, 0) + log(1 + e^{-|t|}) / 100,
// t = 100 x, on the raw v_exp_f32 / v_log_f32 (base 2: log2(1 + 2^{-|t| log2 e}) ln2 / 100; the
// log argument is in [1, 2], never denormal).  The same function as the threshold form: where
// the reference returns x (t > 20) this adds <= 2e-9 x 0.0069 (below an ulp of x), and the
// -|t| of the exp is a free source modifier, so no compare / select and no overflow guard.
// The pair form issues the multiplies / adds as packed fp32 (v_pk_mul_f32 / v_pk_add_f32 /
// v_pk_fma_f32, two elements per lane per issue) and computes bit-identical values; the
// layer-0 / layer-1 epilogues are VALU bound on this function.
// max(x, 0) as one v_max_i32 on the bit pattern (every negative float, -0 included, is a
// negative int32): fmaxf / fmed3 are lowered with a canonicalising v_max_f32 x, x first, a
// second instruction per element on the softplus epilogues.  (Not inline asm: the hazard
// recognizer does not see an asm operand read right after the MFMA that wrote it.)
MLI_FI float relu_f(float x) {
  const int b = __builtin_bit_cast(int, x);
  return __builtin_bit_cast(float, b > 0 ? b : 0);
}

MLI_FI float softplus100(float x) {
  const float u = x * 144.26950408889634f;  // 100 log2 e
  const float l = __builtin_amdgcn_logf(__builtin_amdgcn_exp2f(-fabsf(u)) + 1.0f);
  return fmaf(l, 0.0069314718055994531f, relu_f(x));
}

// MLI_PK_F32=1: the element-pair helpers below as v_pk_*_f32.  Default 0 (two scalar ops each):
// bit-identical, and measured faster -- FIELD 0.81 -> 0.77 ms, field_mlp 167 -> 118 VGPRs (four
// waves per SIMD), sdf_kernel 268 -> 200 registers, sdf_bwd 256 -> 207.
#ifndef MLI_PK_F32
#define MLI_PK_F32 0
#endif
MLI_FI f32x2 softplus100x2(f32x2 x) {
  if (!MLI_PK_F32) return (f32x2){softplus100(x.x), softplus100(x.y)};
  const f32x2 u = x * (f32x2){144.26950408889634f, 144.26950408889634f};
  f32x2 e;
  e.x = __builtin_amdgcn_exp2f(-fabsf(u.x));
  e.y = __builtin_amdgcn_exp2f(-fabsf(u.y));
  const f32x2 a = e + (f32x2){1.0f, 1.0f};
  f32x2 l;
  l.x = __builtin_amdgcn_logf(a.x);
  l.y = __builtin_amdgcn_logf(a.y);
  return __builtin_elementwise_fma(l, (f32x2){0.0069314718055994531f, 0.0069314718055994531f},
                                   (f32x2){relu_f(x.x), relu_f(x.y)});
}

// a + b * c on an element pair (v_pk_fma_f32, or two v_fma_f32 with MLI_PK_F32=0)
MLI_FI f32x2 fma_x2(f32x2 b, f32x2 c, f32x2 a) {
  if (!MLI_PK_F32) return (f32x2){fmaf(b.x, c.x, a.x), fmaf(b.y, c.y, a.y)};
  return __builtin_elementwise_fma(b, c, a);
}

// b0 + W[:, 0:3] . p on an element pair: three fmas per element, in this order.
MLI_FI f32x2 pterm_x2(f32x2 b0, f32x2 wx, f32x2 wy, f32x2 wz, float px, float py, float pz) {
  if (!MLI_PK_F32)
    return (f32x2){fmaf(wz.x, pz, fmaf(wy.x, py, fmaf(wx.x, px, b0.x))),
                   fmaf(wz.y, pz, fmaf(wy.y, py, fmaf(wx.y, px, b0.y)))};
  f32x2 v = __builtin_elementwise_fma(wx, (f32x2){px, px}, b0);
  v = __builtin_elementwise_fma(wy, (f32x2){py, py}, v);
  return __builtin_elementwise_fma(wz, (f32x2){pz, pz}, v);
}

MLI_FI float sigmoidf_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

// Real spherical harmonics, levels = 3 (projects/neuralangelo/utils/spherical_harmonics.py:47-84).
MLI_FI void sh16(float x, float y, float z, float* o) {
  const float C0 = 0.28209479177387814f, C1 = 0.4886025119029199f;
  const float C20 = 1.0925484305920792f, C21 = -1.0925484305920792f, C22 = 0.31539156525252005f,
              C23 = -1.0925484305920792f, C24 = 0.5462742152960396f;
  const float C30 = -0.5900435899266435f, C31 = 2.890611442640554f, C32 = -0.4570457994644658f,
              C33 = 0.3731763325901154f, C34 = -0.4570457994644658f, C35 = 1.445305721320277f,
              C36 = -0.5900435899266435f;
  const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
  o[0] = C0;
  o[1] = -C1 * y;
  o[2] = C1 * z;
  o[3] = -C1 * x;
  o[4] = C20 * xy;
  o[5] = C21 * yz;
  o[6] = C22 * (2.0f * zz - xx - yy);
  o[7] = C23 * xz;
  o[8] = C24 * (xx - yy);
  o[9] = C30 * y * (3.0f * xx - yy);
  o[10] = C31 * xy * z;
  o[11] = C32 * y * (4.0f * zz - xx - yy);
  o[12] = C33 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
  o[13] = C34 * x * (4.0f * zz - xx - yy);
  o[14] = C35 * z * (xx - yy);
  o[15] = C36 * x * (xx - 3.0f * yy);
}

// Opaque copy: defeats loop-invariant hoisting of address arithmetic built from x (the
// hoisted values otherwise stay live across the whole loop and spill).
MLI_FI int opaque_s(int x) {
  asm volatile("" : "+s"(x));
  return x;
}
MLI_FI int opaque_v(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
// Per-lane select hi/lo by a 0/~0 mask with integer ops: LLVM folds `c ? a[8+j] : a[j]` into a
// dynamically indexed load of a private array (scratch); the bitwise form stays in registers.
MLI_FI float sel_mask(uint32_t mask, float hi, float lo) {
  const uint32_t r = (__builtin_bit_cast(uint32_t, hi) & mask) | (__builtin_bit_cast(uint32_t, lo) & ~mask);
  return __builtin_bit_cast(float, r);
}

// ---------------------------------------------------------------- LDS-DMA pipelines
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_cvoid_t;

// 16 B per lane global -> LDS (global_load_lds_dwordx4): lane l lands at lds_wave_base + 16 l
MLI_FI void glds16(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_cvoid_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// s_waitcnt vmcnt(n) for a count known after unrolling (the switch folds; up to the 6-bit
// field's 63, larger counts wait for everything)
MLI_FI void vm_wait(int n) {
  switch (n) {
#define MLI_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MLI_VMW(1) MLI_VMW(2) MLI_VMW(3) MLI_VMW(4) MLI_VMW(5) MLI_VMW(6) MLI_VMW(7) MLI_VMW(8)
    MLI_VMW(9) MLI_VMW(10) MLI_VMW(11) MLI_VMW(12) MLI_VMW(13) MLI_VMW(14) MLI_VMW(15) MLI_VMW(16)
    MLI_VMW(17) MLI_VMW(18) MLI_VMW(19) MLI_VMW(20) MLI_VMW(21) MLI_VMW(22) MLI_VMW(23) MLI_VMW(24)
    MLI_VMW(25) MLI_VMW(26) MLI_VMW(27) MLI_VMW(28) MLI_VMW(29) MLI_VMW(30) MLI_VMW(31) MLI_VMW(32)
    MLI_VMW(33) MLI_VMW(34) MLI_VMW(35) MLI_VMW(36) MLI_VMW(37) MLI_VMW(38) MLI_VMW(39) MLI_VMW(40)
    MLI_VMW(41) MLI_VMW(42) MLI_VMW(43) MLI_VMW(44) MLI_VMW(45) MLI_VMW(46) MLI_VMW(47) MLI_VMW(48)
    MLI_VMW(49) MLI_VMW(50) MLI_VMW(51) MLI_VMW(52) MLI_VMW(53) MLI_VMW(54) MLI_VMW(55) MLI_VMW(56)
    MLI_VMW(57) MLI_VMW(58) MLI_VMW(59) MLI_VMW(60) MLI_VMW(61) MLI_VMW(62) MLI_VMW(63)
#undef MLI_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
// vm_wait for a wave-uniform count known only at run time (a scalar branch tree)
MLI_FI void vm_wait_rt(int n) { vm_wait(__builtin_amdgcn_readfirstlane(n)); }

// LDS writes visible to the workgroup; no vector-memory drain (raw barrier: __syncthreads'
// fence would wait for every outstanding DMA and store)
MLI_FI void block_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Ray bounds: intersect_with_sphere (nerf_util.py:199-205; r2 = fp32(radius**2)) with the
// NaN-miss dummy (neuralangelo/model.py:426-429), or the AABB slab test
// (NeuralLumen/utils/utils.py:86-123, neuralangelo/model.py:422-424).
MLI_FI void ray_bounds(const float (&c)[3], const float (&v)[3], int box, float r2, const float* aabb, float& nr,
                       float& fr, bool& out) {
  if (!box) {
    const float ctc = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
    const float ctv = (c[0] * v[0] + c[1] * v[1]) + c[2] * v[2];
    const float disc = ctv * ctv - (ctc - r2);
    const float sq = sqrtf(disc);
    const float n0 = -ctv - sq;
    out = isnan(n0);
    nr = out ? 1.0f : fmaxf(n0, 0.0f);
    fr = out ? 1.2f : -ctv + sq;
  } else {
    float tmin = -INFINITY, tmax = INFINITY;
    for (int i = 0; i < 3; ++i) {
      const float t0 = (aabb[i] - c[i]) / v[i];
      const float t1 = (aabb[3 + i] - c[i]) / v[i];
      tmin = fmaxf(tmin, fminf(t0, t1));
      tmax = fminf(tmax, fmaxf(t0, t1));
    }
    tmin = fminf(fmaxf(tmin, 0.0f), 1e10f);
    tmax = fminf(fmaxf(tmax, 0.0f), 1e10f);
    out = tmax <= tmin;
    nr = out ? 1.0f : tmin;
    fr = out ? 1.2f : tmax;
  }
}

#define MLI_LAUNCH_CHECK() return (int)hipGetLastError()
