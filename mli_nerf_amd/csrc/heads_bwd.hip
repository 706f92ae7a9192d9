// Fused backward of the three colour heads: dX chain + the 256 x 256 weight gradients.
//
// Replaces autograd through MLPwithSkipConnection (projects/nerf/utils/nerf_util.py:158-196)
// for the head layers 1..3: dZ_l = (W_{l+1}^T dZ_{l+1}) * relu'(Z_l) and dW_l = dZ_l^T X_l,
// db_l = sum_s dZ_l.  mli_rgb_bwd + the BIG class of mli_wgrad compute the same, with every
// dZ_l written to HBM by the first and read back by the second (2 x 2.4 GB per step at
// 4096 x 128); here dZ_l never leaves the CU.
//
// One workgroup = 4 waves (one per SIMD, up to 512 registers each) owns ONE dW_l of one head
// -- 256 x 256 fp32, 256 accumulator registers per lane: wave w holds columns 64w..64w+63 --
// over a contiguous range of 128-sample tiles (its k-slice).  Per tile it recomputes the dX
// chain from dz4 down to dZ_l for its 128 samples (wave w: samples 32w..32w+31, the
// activations in registers as MFMA B fragments exactly as mli_rgb_bwd), stages each 32-row
// n-tile of dZ_l^T in LDS and multiplies it into the accumulators against X_l^T, which the
// workgroup brings from HBM by LDS-DMA.  The l = 1 workgroups also write dZ_1 as an MFMA
// B-fragment image; a second launch (mlp.hip, dz0_kernel) takes the chain one layer further to
// dZ_0 rows, the operand of the layer-0 dW (mli_wgrad WIDE class).
//
// Work per tile: l = 3: 8 + 128 MFMAs per wave; l = 2: + the W3^T layer (128); l = 1: + W2^T:
// 392.  The k-slices per l are sized in that proportion (split[]).
//
// Queues: vmcnt retires in issue order, so a wave that waits for the next weight chunk every
// phase cannot also have a long-latency HBM load in flight.  Waves 0-1 (RING) issue the weight
// chunk DMAs and wait for them every phase (counted: their own stores after a chunk may stay
// in flight); waves 2-3 (LOAD) bring X_l, the ReLU masks and dz4 from HBM well ahead and wait
// for them only where the data is next needed.
#include "common.h"

#include <algorithm>

namespace {

constexpr int THREADS = 256;
constexpr int TILE = 128;                    // samples per tile: 4 waves x 32
constexpr int CH1 = 1024 + 128;              // mli_pack bwd image: W4^T chunk stride
constexpr int CH16 = 16 * 1024 + 128;        //   W3^T, W2^T, W1^T chunk stride
constexpr int HEAD_BYTES = 8 * CH1 + 24 * CH16;
constexpr int WCH = 16 * 1024;               // ring chunk: 16 A fragments (the zero bias is not loaded)
constexpr int NSLOT = 3, DIST = 2;
constexpr int RING_OPS = WCH / 1024 / 2;     // 1 KiB per LDS-DMA op, 2 RING waves: 8 ops each
constexpr int ZTB = TILE * 64;               // one staged dZ_l^T n-tile for the dW [128 samples][32 features]
constexpr int XW = 64 * 256;                 // one wave's X slice [64 rows][128 samples], swizzled
constexpr int MASKB = 4096;                  // one layer's ReLU masks for a tile [4 waves][64][16 B]
constexpr int Z4B = 4 * 3 * 256;             // dz4 of a tile [4 waves][3][64 lanes] fp32
constexpr int JOB_F = 256 * 256 + 256;       // floats of one dW + db

// LDS map.  l = 1, 2: W4^T | ring | X | 2 staged n-tiles | 4 mask slots | dz4.
// l = 3 (no ring): W4^T | 8 staged n-tiles (the whole dZ_3^T tile) | X | mask slot | dz4.
struct Map {
  int w4, ring, x, zt, mask, z4, end;
};
constexpr Map map_of(int L) {
  return L == 3 ? Map{0, 0, 8192 + 8 * ZTB, 8192, 8192 + 8 * ZTB + 4 * XW, 8192 + 8 * ZTB + 4 * XW + MASKB,
                      8192 + 8 * ZTB + 4 * XW + MASKB + Z4B}
                : Map{0, 8192, 8192 + NSLOT * WCH, 8192 + NSLOT * WCH + 4 * XW,
                      8192 + NSLOT * WCH + 4 * XW + 2 * ZTB, 8192 + NSLOT * WCH + 4 * XW + 2 * ZTB + 4 * MASKB,
                      8192 + NSLOT * WCH + 4 * XW + 2 * ZTB + 4 * MASKB + Z4B};
}
constexpr int LDS_BYTES = std::max(map_of(1).end, map_of(3).end);
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

enum Role { RING = 0, LOAD = 1 };

struct KArgs {
  mli_heads_bwd_args a;
  int S, tiles;
  int split[3];       // workgroups per (head, l) for l = 1, 2, 3
  int first[4];       // first block of each l group (first[3] = grid)
  int64_t part_base[9];
};

MLI_FI void glds4(const void* g, uint8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_cvoid_t*)g, (lds_void_t*)lds_wave_base, 4, 0, 0);
}

// s_waitcnt vmcnt(n), n known after unrolling (up to the 6-bit field's 63)
MLI_FI void vm_wait63(int n) {
  switch (n) {
#define V(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    V(1) V(2) V(3) V(4) V(5) V(6) V(7) V(8) V(9) V(10) V(11) V(12) V(13) V(14) V(15) V(16)
    V(17) V(18) V(19) V(20) V(21) V(22) V(23) V(24) V(25) V(26) V(27) V(28) V(29) V(30) V(31) V(32)
    V(33) V(34) V(35) V(36) V(37) V(38) V(39) V(40) V(41) V(42) V(43) V(44) V(45) V(46) V(47) V(48)
    V(49) V(50) V(51) V(52) V(53) V(54) V(55) V(56) V(57) V(58) V(59) V(60) V(61) V(62) V(63)
#undef V
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// X slice rows are stored with their 16 B chunks permuted per row (source-side swizzle of the
// LDS-DMA): the B-fragment reads of 32 rows at one chunk column are conflict-free.
MLI_FI int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// Sample order inside a tile for the dW contraction: k-step q, lane half h, element j <->
// sample 64h + 8q + j.  Both operands (dZ^T from the staged n-tile, X^T from the slice) are
// read in that order, so each lane's 8 samples are 16 contiguous bytes of a row.

struct Ctx {
  const mli_heads_bwd_args* a;
  int S, R, N, hd, L;
  uint8_t* lds;
  int lane, wave, c, h;
};

// ----------------------------------------------------------------------- LOAD-wave DMAs
// X_l^T of tile T: 4 slices x 16 ops of 4 rows x 256 B; LOAD wave lw issues 32.
template <int L, int COUNT>
MLI_FI void x_dma(const Ctx& k, const uint16_t* xrows, int T, int first) {
  constexpr Map M = map_of(L);
  // piece i (0..63): slice i >> 4, rows 4u .. 4u+3 (u = i & 15).  Row rho = 4u + (lane >> 4),
  // LDS chunk lane & 15 <- global chunk (lane & 15) ^ swz(rho) = c2 ^ (u & 3), c2 = (lane & 15)
  // ^ ((lane >> 4) << 2): four per-lane element offsets, everything else uniform
  const int rho_lo = k.lane >> 4, c2 = (k.lane & 15) ^ (rho_lo << 2);
  int lo[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) lo[v] = rho_lo * k.S + 8 * (c2 ^ v);
  const uint16_t* base = xrows + (size_t)T * TILE;
#pragma unroll
  for (int ii = 0; ii < COUNT; ++ii) {
    const int i = __builtin_amdgcn_readfirstlane(first + ii), ws = i >> 4, u = i & 15;
    const int v = u & 3;
    const int l = v == 0 ? lo[0] : v == 1 ? lo[1] : v == 2 ? lo[2] : lo[3];
    glds16(base + (size_t)(64 * ws + 4 * u) * k.S + l, k.lds + M.x + ws * XW + u * 1024);
  }
}

// ReLU masks of head layer ml for tile T into mask slot `slot`: 4 KiB, 2 ops per LOAD wave.
template <int L>
MLI_FI void mask_dma(const Ctx& k, const uint32_t* masks, int ml, int T, int slot, int lw) {
  constexpr Map M = map_of(L);
  const uint8_t* src = reinterpret_cast<const uint8_t*>(masks) +
                       (((size_t)(k.hd * 4 + ml) * (k.S / 32) + (size_t)4 * T) * 64) * 16;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int piece = 2 * lw + u;
    glds16(src + piece * 1024 + k.lane * 16, k.lds + M.mask + slot * MASKB + piece * 1024);
  }
}

// dz4 of tile T (fp32, slot-major [N][R][8]) into [wave][j][lane]: 6 ops per LOAD wave.
template <int L>
MLI_FI void z4_dma(const Ctx& k, int T, int lw) {
  constexpr Map M = map_of(L);
  const int no = k.hd == 2 ? 1 : 3;
#pragma unroll
  for (int ii = 0; ii < 6; ++ii) {
    const int wv = 2 * lw + ii / 3, j = ii % 3;
    const int m = T * TILE + wv * 32 + (k.lane & 31);
    const int r = m / k.N, kk = m - r * k.N;
    const size_t slot = (size_t)kk * k.R + r;
    glds4(k.a->dz4 + 8 * slot + 3 * k.hd + min(j, no - 1), k.lds + M.z4 + (wv * 3 + j) * 256);
  }
}

// W4^T (8 n-tiles x 1 KiB, KS 1), resident for the whole kernel: 2 ops per wave.
template <int L>
MLI_FI void w4_load(const Ctx& k) {
  constexpr Map M = map_of(L);
  const uint8_t* src = reinterpret_cast<const uint8_t*>(k.a->wbwd) + (size_t)k.hd * HEAD_BYTES;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int piece = 2 * k.wave + u;
    glds16(src + piece * CH1 + k.lane * 16, k.lds + M.w4 + piece * 1024);
  }
}

// ----------------------------------------------------------------------- weight ring
struct HRing {
  const uint8_t* base;  // chunk 0 of this (head, l): W3^T n-tile 0
  int next, total;
};

template <int L, int NPT>
MLI_FI void ring_issue(HRing& rg, const Ctx& k) {
  constexpr Map M = map_of(L);
  const int cidx = min(rg.next, rg.total - 1);  // past the end: a dummy re-load into a free slot
  const uint8_t* src = rg.base + (size_t)(cidx % NPT) * CH16;
  uint8_t* dst = k.lds + M.ring + (rg.next % NSLOT) * WCH;
#pragma unroll
  for (int u = 0; u < RING_OPS; ++u) {
    const int piece = 2 * u + k.wave;  // RING waves 0, 1
    glds16(src + piece * 1024 + k.lane * 16, dst + piece * 1024);
  }
  rg.next++;
}

// ----------------------------------------------------------------------- compute pieces
MLI_FI f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

MLI_FI f32x16 masked(const f32x16& acc, const u32x4& mv, int t) {
  const int wi = t >> 1;
  const uint32_t word = wi == 0 ? mv[0] : wi == 1 ? mv[1] : wi == 2 ? mv[2] : mv[3];
  const uint32_t bits = word >> ((t & 1) * 16);
  f32x16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = ((bits >> i) & 1u) ? acc[i] : 0.0f;
  return v;
}

// acc = W^T chunk (32 x 256) x IN (256 x 32 samples).  At one wave per SIMD nothing hides an
// LDS read's latency but the wave's own MFMAs: the 16 A fragments are read in groups of PF,
// group g+1 issued before the MFMAs of group g (the fence keeps the compiler from hoisting all
// 16 reads to the top, which costs 64 registers the dW tile needs).
constexpr int PF = 4;
MLI_FI void ld_fence() { asm volatile("" ::: "memory"); }
// x redefined here (after the stores before it): what consumes x is not hoisted above
MLI_FI void opaque_h8(half8& x) { asm volatile("" : "+v"(x)::"memory"); }

MLI_FI f32x16 chunk16(const uint8_t* chunk, const half8* in, int lane) {
  f32x16 acc = zero16();
  const half8* w = reinterpret_cast<const half8*>(chunk) + lane;
  half8 buf[2][PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) buf[0][i] = w[i * 64];
#pragma unroll
  for (int g = 0; g < 16 / PF; ++g) {
    if (g + 1 < 16 / PF) {
#pragma unroll
      for (int i = 0; i < PF; ++i) buf[(g + 1) & 1][i] = w[((g + 1) * PF + i) * 64];
    }
    ld_fence();
#pragma unroll
    for (int i = 0; i < PF; ++i) acc = mfma32(buf[g & 1][i], in[g * PF + i], acc);
  }
  return acc;
}

// dW staging: the n-tile as [128 samples][32 features] fp16, 64 B rows, 8-byte units XOR-swizzled
// by (sample >> 1) & 7.  A lane writes its 16 accumulator values (features 8g + 4h + 0..3 of
// its sample, g = 0..3) as 4 x 8 bytes; the A fragment of a dW k-step is read back transposed
// (ds_read_b64_tr_b16).  Both conflict-free.

MLI_FI int zswz(int s) { return (s >> 1) & 7; }

MLI_FI void stage_t(uint8_t* zb, const f32x16& v, const Ctx& k) {
  const int s = k.wave * 32 + k.c;
  uint8_t* row = zb + s * 64;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const half4 x = {(f16)v[4 * g], (f16)v[4 * g + 1], (f16)v[4 * g + 2], (f16)v[4 * g + 3]};
    *reinterpret_cast<half4*>(row + (((2 * g + k.h) ^ zswz(s)) << 3)) = x;
  }
}

// A fragment of dW k-step q: feature lane & 31, samples 64h + 8q + 0..7 (two 4-sample reads;
// the 16-lane group g of the read takes h = g >> 1 and features 16 (g & 1) + 0..15).  Row s =
// 64h + 8q + (i >> 2) (+4): the swizzle ((s >> 1) & 7) depends on q only through q & 1, so four
// per-lane offsets (Offs::z) serve every k-step (+ 512 q as an immediate).
struct Offs {
  int z[2][2];  // [q & 1][read]
  int x[8];     // X slice B fragment (cb 0) of k-step q: row r, chunk (8h + q) ^ swz(r)
};

MLI_FI Offs make_offs(const Ctx& k) {
  Offs o;
  const int i = k.lane & 15, grp = k.lane >> 4, u = 4 * (grp & 1) + (i & 3);
  const int s0 = 64 * (grp >> 1) + (i >> 2);
#pragma unroll
  for (int qp = 0; qp < 2; ++qp)
#pragma unroll
    for (int rd = 0; rd < 2; ++rd) {
      const int s = s0 + 8 * qp + 4 * rd;
      o.z[qp][rd] = (s - 8 * qp) * 64 + ((u ^ zswz(s)) << 3);
    }
  const int sw = swz(k.c);
#pragma unroll
  for (int q = 0; q < 8; ++q) o.x[q] = k.c * 256 + (((8 * k.h + q) ^ sw) << 4);
  return o;
}

MLI_FI half8 zt_frag(const uint8_t* zb, int q, const Offs& o) {
  const uint8_t* b = zb + 512 * q;
  const fp16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_fp16x4_t*)(b + o.z[q & 1][0]));
  const fp16x4_t c = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_fp16x4_t*)(b + o.z[q & 1][1]));
  const half4 ha = __builtin_bit_cast(half4, a), hc = __builtin_bit_cast(half4, c);
  return half8{ha[0], ha[1], ha[2], ha[3], hc[0], hc[1], hc[2], hc[3]};
}

MLI_FI float hsum8(const half8& v) {
  typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
  const half2_t one = {(f16)1.0f, (f16)1.0f};
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const half2_t x = {v[2 * p], v[2 * p + 1]};
    s = __builtin_amdgcn_fdot2(x, one, s, false);
  }
  return s;
}

// dW accumulators: 8 n-tiles x 2 column blocks x 16 fp32 = all 256 AGPRs of the lane, held
// in AGPRs by the constraints of the asm MFMAs below for the whole kernel (the chain MFMAs are
// compiled in VGPR form: -mllvm -amdgpu-mfma-vgpr-form, build.py).  hipcc pads no hazard
// inside or around an asm statement (guide 5.7): every statement opens with s_nop 1 (a VALU
// write of an A/B operand just before it), an accumulate chain needs no pad, and dw_release()
// pads the MFMA -> read of the accumulators before the epilogue reads them.
MLI_FI void dw_zero(f32x16& c) {
  const half8 z = {};
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %1, 0" : "=a"(c) : "v"(z));
}

// 2 k-steps x 2 column blocks: c0 += a0 x b00 + a1 x b01, c1 += a0 x b10 + a1 x b11
MLI_FI void dw_mma4(f32x16& c0, f32x16& c1, const half8& a0, const half8& a1, const half8& b00, const half8& b01,
                    const half8& b10, const half8& b11) {
  asm("s_nop 1\n\t"
      "v_mfma_f32_32x32x16_f16 %0, %2, %4, %0\n\t"
      "v_mfma_f32_32x32x16_f16 %1, %2, %6, %1\n\t"
      "v_mfma_f32_32x32x16_f16 %0, %3, %5, %0\n\t"
      "v_mfma_f32_32x32x16_f16 %1, %3, %7, %1"
      : "+a"(c0), "+a"(c1)
      : "v"(a0), "v"(a1), "v"(b00), "v"(b01), "v"(b10), "v"(b11));
}

MLI_FI void dw_release(f32x16 (&dw)[8][2]) {
  asm volatile("s_nop 15\n\ts_nop 15"
               : "+a"(dw[0][0]), "+a"(dw[0][1]), "+a"(dw[1][0]), "+a"(dw[1][1]), "+a"(dw[2][0]), "+a"(dw[2][1]),
                 "+a"(dw[3][0]), "+a"(dw[3][1]), "+a"(dw[4][0]), "+a"(dw[4][1]), "+a"(dw[5][0]), "+a"(dw[5][1]),
                 "+a"(dw[6][0]), "+a"(dw[6][1]), "+a"(dw[7][0]), "+a"(dw[7][1]));
}

// dW rows of n-tile nt (32) x this wave's 64 columns += staged dZ^T (zb) x X slice, over the
// tile's 128 samples (8 k-steps); the bias partial of the n-tile on wave nt & 3.
template <bool XREG>
MLI_FI void dw_tile(f32x16 (&acc)[2], const uint8_t* zb, const uint8_t* xs, const half8 (&xr)[2][8], const Offs& of,
                    bool do_bias, float& bp) {
  // operands of k-steps q, q+1: 2 dZ^T fragments + 4 X fragments (X: registers or the slice)
  struct Ops { half8 a[2], x[4]; };
  auto load = [&](Ops& o, int q) MLI_LAMBDA_FI {
#pragma unroll
    for (int u = 0; u < 2; ++u) o.a[u] = zt_frag(zb, q + u, of);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        o.x[2 * cb + u] = XREG ? xr[cb][q + u] : *reinterpret_cast<const half8*>(xs + 32 * 256 * cb + of.x[q + u]);
  };
  Ops ops[2];
  load(ops[0], 0);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    if (g + 1 < 4) load(ops[(g + 1) & 1], 2 * g + 2);
    ld_fence();
    const Ops& o = ops[g & 1];
    if (do_bias) bp += hsum8(o.a[0]) + hsum8(o.a[1]);
    dw_mma4(acc[0], acc[1], o.a[0], o.a[1], o.x[0], o.x[1], o.x[2], o.x[3]);
  }
}

template <int L>
MLI_FI void x_to_regs(half8 (&xr)[2][8], const Ctx& k, const Offs& of) {
  constexpr Map M = map_of(L);
  const uint8_t* xs = k.lds + M.x + k.wave * XW;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int q = 0; q < 8; ++q) xr[cb][q] = *reinterpret_cast<const half8*>(xs + 32 * 256 * cb + of.x[q]);
}

// dz4 B fragment (k-step of 16: rows 0..2 = the head's outputs, on lane half 0)
template <int L>
MLI_FI half8 z4_frag(const Ctx& k) {
  constexpr Map M = map_of(L);
  const int no = k.hd == 2 ? 1 : 3;
  half8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (f16)0.f;
  const float* zs = reinterpret_cast<const float*>(k.lds + M.z4 + k.wave * 3 * 256) + k.lane;
  if (k.h == 0) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < no) z[j] = (f16)zs[j * 64];
  }
  return z;
}

MLI_FI u32x4 mask_read(const uint8_t* slot, const Ctx& k) {
  return *reinterpret_cast<const u32x4*>(slot + k.wave * 1024 + k.lane * 16);
}

// W4^T (resident) x dz4 -> dZ_3 n-tile t, masked; the 8 fragments read up front
template <int L>
MLI_FI void w4_frags(half8 (&w)[8], const Ctx& k) {
  constexpr Map M = map_of(L);
#pragma unroll
  for (int t = 0; t < 8; ++t) w[t] = reinterpret_cast<const half8*>(k.lds + M.w4 + t * 1024)[k.lane];
}

MLI_FI f32x16 w4_tile(const half8& w, const half8& z, const u32x4& mv, int t) {
  return masked(mfma32(w, z, zero16()), mv, t);
}

// ----------------------------------------------------------------------- epilogue
// This workgroup's dW partial (+ db): fp32 atomics, or its slab in the deterministic workspace.
MLI_FI void write_out(const KArgs& ka, const Ctx& k, int split, f32x16 (&dw)[8][2], float (&bp)[2]) {
  const int job = k.hd * 3 + (k.L - 1);
  float tot[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) tot[u] = bp[u] + __shfl_xor(bp[u], 32);
  const int col0 = 64 * k.wave + k.c;
  if (ka.a.deterministic) {
    float* slab = ka.a.workspace + ka.part_base[job] + (int64_t)split * JOB_F;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) slab[(32 * t + acc_row(i, k.h)) * 256 + col0 + 32 * cb] = dw[t][cb][i];
    if (k.h == 0) {
      slab[65536 + 32 * k.wave + k.c] = tot[0];
      slab[65536 + 32 * (k.wave + 4) + k.c] = tot[1];
    }
  } else {
    float* dwp = ka.a.dw[job];
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < 16; ++i) atomicAdd(dwp + (32 * t + acc_row(i, k.h)) * 256 + col0 + 32 * cb, dw[t][cb][i]);
    if (k.h == 0) {
      atomicAdd(ka.a.db[job] + 32 * k.wave + k.c, tot[0]);
      atomicAdd(ka.a.db[job] + 32 * (k.wave + 4) + k.c, tot[1]);
    }
  }
}

// ----------------------------------------------------------------------- l = 1
// Tile phases: 0 (dW1 of n-tile 7 of tile T-1; W4^T -> dZ3), 1-8 (W3^T -> dZ2), 9-16 (W2^T ->
// dZ1: its B-fragment image out to HBM for the dZ_0 launch, the n-tile staged for dW1, dW1 of
// n-tile t-1).  LOAD waves: dz4 + masks 3 of T+1 in phase 1, masks 2 of T+1 in 2, X(T) over 1-6
// (X(T-1) is read until phase 0), masks 1 of T+1 in 10; wait(0) at the end of 8 and 16.  Every
// wave stores its dZ1 fragments (2 per phase) in 9-16: the RING waves' wait at the end of a
// phase allows the ops issued after the previous chunk: 8 (W3^T), 10 (first W2^T), 12 (W2^T).
constexpr int X_OFF[6] = {0, 6, 12, 17, 22, 27};  // X pieces per phase: 6, 6, 5, 5, 5, 5

template <int ROLE>
MLI_FI void body1(const KArgs& ka, const Ctx& k, int t0, int t1, int split) {
  constexpr int L = 1;
  constexpr Map M = map_of(L);
  const uint16_t* xrows = k.a->xT + (size_t)(k.hd * 4 + 0) * 256 * k.S;
  const int lw = k.wave - 2;
  const Offs of = make_offs(k);
  const bool bias_w[8] = {k.wave == 0, k.wave == 1, k.wave == 2, k.wave == 3,
                          k.wave == 0, k.wave == 1, k.wave == 2, k.wave == 3};
  HRing rg{reinterpret_cast<const uint8_t*>(k.a->wbwd) + (size_t)k.hd * HEAD_BYTES + 8 * CH1, 0, (t1 - t0) * 16};
  w4_load<L>(k);
  if (ROLE == LOAD) {
    z4_dma<L>(k, t0, lw);
    mask_dma<L>(k, k.a->masks, 3, t0, 3, lw);
    mask_dma<L>(k, k.a->masks, 2, t0, 2, lw);
    mask_dma<L>(k, k.a->masks, 1, t0, 1, lw);
  } else {
    ring_issue<L, 16>(rg, k);
    ring_issue<L, 16>(rg, k);
  }
  vm_wait63(0);
  block_sync();

  f32x16 dw[8][2];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    dw_zero(dw[t][0]);
    dw_zero(dw[t][1]);
  }
  float bp[2] = {0.f, 0.f};
  const half8 xr_unused[2][8] = {};
  const uint8_t* xs = k.lds + M.x + k.wave * XW;
  uint8_t* zt0 = k.lds + M.zt;
  half8* f1 = reinterpret_cast<half8*>(k.a->dz1f + (size_t)k.hd * 256 * k.S) + k.lane;
  int cur = 0;
  half8 A[16], B[16];
  for (int T = t0; T < t1; ++T) {
    const int Tn = min(T + 1, t1 - 1);
    // phase 0
    if (T != t0) dw_tile<false>(dw[7], zt0 + ZTB, xs, xr_unused, of, bias_w[7], bp[1]);
    __builtin_amdgcn_sched_barrier(0);
    {
      const half8 z = z4_frag<L>(k);
      const u32x4 mv = mask_read(k.lds + M.mask + 3 * MASKB, k);
      half8 zz = z, w4[8];
      w4_frags<L>(w4, k);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const f32x16 v = w4_tile(w4[t], zz, mv, t);
        A[2 * t] = acc_to_frag(v, 0);
        A[2 * t + 1] = acc_to_frag(v, 1);
        opaque_h8(zz);
      }
    }
    block_sync();
    // phases 1-8: W3^T -> dZ2 (B)
    {
      const u32x4 mv = mask_read(k.lds + M.mask + 2 * MASKB, k);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (ROLE == RING) ring_issue<L, 16>(rg, k);
        if (ROLE == LOAD) {
          if (t == 0) {
            z4_dma<L>(k, Tn, lw);
            mask_dma<L>(k, k.a->masks, 3, Tn, 3, lw);
          }
          if (t == 1) mask_dma<L>(k, k.a->masks, 2, Tn, 2, lw);
          if (t < 2) x_dma<L, 6>(k, xrows, T, 32 * lw + X_OFF[t]);
          else if (t < 6) x_dma<L, 5>(k, xrows, T, 32 * lw + X_OFF[t]);
        }
        const f32x16 v = masked(chunk16(k.lds + M.ring + (cur % NSLOT) * WCH, A, k.lane), mv, t);
        B[2 * t] = acc_to_frag(v, 0);
        B[2 * t + 1] = acc_to_frag(v, 1);
        if (ROLE == RING) vm_wait63(RING_OPS);
        if (ROLE == LOAD && t == 7) vm_wait63(0);
        block_sync();
        cur++;
      }
    }
    // phases 9-16: W2^T -> dZ1: B-fragment image out, staged for dW1; dW1 of n-tile t-1
    {
      const u32x4 mv = mask_read(k.lds + M.mask + 1 * MASKB, k);
      half8* ft = f1 + (size_t)(4 * T + k.wave) * 16 * 64;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (ROLE == RING) ring_issue<L, 16>(rg, k);
        if (ROLE == LOAD && t == 1) mask_dma<L>(k, k.a->masks, 1, Tn, 1, lw);
        // dW of the previous n-tile, then this n-tile's chain step: kept apart (sched_barrier)
        // so their operand registers are not live together
        if (t > 0) dw_tile<false>(dw[t - 1], zt0 + ((t - 1) & 1) * ZTB, xs, xr_unused, of, bias_w[t - 1], bp[(t - 1) >> 2]);
        __builtin_amdgcn_sched_barrier(0);
        const f32x16 v = masked(chunk16(k.lds + M.ring + (cur % NSLOT) * WCH, B, k.lane), mv, t);
        ft[(2 * t) * 64] = acc_to_frag(v, 0);
        ft[(2 * t + 1) * 64] = acc_to_frag(v, 1);
        stage_t(zt0 + (t & 1) * ZTB, v, k);
        if (ROLE == RING) vm_wait63(RING_OPS + (t == 0 ? 2 : 4));
        if (ROLE == LOAD && t == 7) vm_wait63(0);
        block_sync();
        cur++;
      }
    }
  }
  dw_tile<false>(dw[7], zt0 + ZTB, xs, xr_unused, of, bias_w[7], bp[1]);
  vm_wait63(0);
  dw_release(dw);
  write_out(ka, k, split, dw, bp);
}

// ----------------------------------------------------------------------- l = 2
// Tile phases: 0 (dW2 of n-tile 7 of T-1; X(T) to registers; W4^T -> dZ3), 1-8 (W3^T -> dZ2,
// staged; dW2 of n-tile t-1).  LOAD waves: X(T+1) over phases 1-6, dz4 + masks 3 and 2 of T+1
// in phase 1 (the mask-2 slot alternates by tile parity); wait(0) at the end of phase 8.

template <int ROLE>
MLI_FI void body2(const KArgs& ka, const Ctx& k, int t0, int t1, int split) {
  constexpr int L = 2;
  constexpr Map M = map_of(L);
  const uint16_t* xrows = k.a->xT + (size_t)(k.hd * 4 + 1) * 256 * k.S;
  const int lw = k.wave - 2;
  const Offs of = make_offs(k);
  const bool bias_w[8] = {k.wave == 0, k.wave == 1, k.wave == 2, k.wave == 3,
                          k.wave == 0, k.wave == 1, k.wave == 2, k.wave == 3};
  HRing rg{reinterpret_cast<const uint8_t*>(k.a->wbwd) + (size_t)k.hd * HEAD_BYTES + 8 * CH1, 0, (t1 - t0) * 8};
  w4_load<L>(k);
  if (ROLE == LOAD) {
    z4_dma<L>(k, t0, lw);
    mask_dma<L>(k, k.a->masks, 3, t0, 3, lw);
    mask_dma<L>(k, k.a->masks, 2, t0, 0, lw);
    x_dma<L, 32>(k, xrows, t0, 32 * lw);
  } else {
    ring_issue<L, 8>(rg, k);
    ring_issue<L, 8>(rg, k);
  }
  vm_wait63(0);
  block_sync();

  f32x16 dw[8][2];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    dw_zero(dw[t][0]);
    dw_zero(dw[t][1]);
  }
  float bp[2] = {0.f, 0.f};
  half8 xr[2][8];
  uint8_t* zt0 = k.lds + M.zt;
  int cur = 0;
  half8 A[16];
  for (int T = t0; T < t1; ++T) {
    const int Tn = min(T + 1, t1 - 1);
    const int par = (T - t0) & 1;
    // phase 0
    if (T != t0) dw_tile<true>(dw[7], zt0 + ZTB, nullptr, xr, of, bias_w[7], bp[1]);
    x_to_regs<L>(xr, k, of);
    {
      const half8 z = z4_frag<L>(k);
      const u32x4 mv = mask_read(k.lds + M.mask + 3 * MASKB, k);
      half8 zz = z, w4[8];
      w4_frags<L>(w4, k);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const f32x16 v = w4_tile(w4[t], zz, mv, t);
        A[2 * t] = acc_to_frag(v, 0);
        A[2 * t + 1] = acc_to_frag(v, 1);
        opaque_h8(zz);
      }
    }
    block_sync();
    // phases 1-8
    const u32x4 mv = mask_read(k.lds + M.mask + par * MASKB, k);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (ROLE == RING) ring_issue<L, 8>(rg, k);
      if (ROLE == LOAD) {
        if (t == 0) {
          z4_dma<L>(k, Tn, lw);
          mask_dma<L>(k, k.a->masks, 3, Tn, 3, lw);
          mask_dma<L>(k, k.a->masks, 2, Tn, par ^ 1, lw);
        }
        if (t < 2) x_dma<L, 6>(k, xrows, Tn, 32 * lw + X_OFF[t]);
        else if (t < 6) x_dma<L, 5>(k, xrows, Tn, 32 * lw + X_OFF[t]);
      }
      if (t > 0) dw_tile<true>(dw[t - 1], zt0 + ((t - 1) & 1) * ZTB, nullptr, xr, of, bias_w[t - 1], bp[(t - 1) >> 2]);
      __builtin_amdgcn_sched_barrier(0);
      const f32x16 v = masked(chunk16(k.lds + M.ring + (cur % NSLOT) * WCH, A, k.lane), mv, t);
      stage_t(zt0 + (t & 1) * ZTB, v, k);
      if (ROLE == RING) vm_wait63(RING_OPS);
      if (ROLE == LOAD && t == 7) vm_wait63(0);
      block_sync();
      cur++;
    }
  }
  dw_tile<true>(dw[7], zt0 + ZTB, nullptr, xr, of, bias_w[7], bp[1]);
  vm_wait63(0);
  dw_release(dw);
  write_out(ka, k, split, dw, bp);
}

// ----------------------------------------------------------------------- l = 3
// Tile phases: 0 (X(T) to registers; W4^T -> dZ3, all 8 n-tiles staged; dz4 rows written for
// the layer-4 dW), 1 (dW3 of the 8 n-tiles; every wave DMAs its own X slice of T+1, the LOAD
// waves dz4 and masks 3 of T+1; wait(0)).  (X_3 loaded straight into registers instead, double
// buffered, measured slower: 64 rows per load instruction.)
template <int ROLE>
MLI_FI void body3(const KArgs& ka, const Ctx& k, int t0, int t1, int split) {
  constexpr int L = 3;
  constexpr Map M = map_of(L);
  const uint16_t* xrows = k.a->xT + (size_t)(k.hd * 4 + 2) * 256 * k.S;
  const int lw = k.wave - 2;
  const Offs of = make_offs(k);
  const bool bias_w[8] = {k.wave == 0, k.wave == 1, k.wave == 2, k.wave == 3,
                          k.wave == 0, k.wave == 1, k.wave == 2, k.wave == 3};
  const int no = k.hd == 2 ? 1 : 3;
  w4_load<L>(k);
  if (ROLE == LOAD) {
    z4_dma<L>(k, t0, lw);
    mask_dma<L>(k, k.a->masks, 3, t0, 0, lw);
  }
  x_dma<L, 16>(k, xrows, t0, 16 * k.wave);
  vm_wait63(0);
  block_sync();

  f32x16 dw[8][2];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    dw_zero(dw[t][0]);
    dw_zero(dw[t][1]);
  }
  float bp[2] = {0.f, 0.f};
  half8 xr[2][8];
  uint8_t* img = k.lds + M.zt;
  for (int T = t0; T < t1; ++T) {
    const int Tn = min(T + 1, t1 - 1);
    x_to_regs<L>(xr, k, of);
    {
      const half8 z = z4_frag<L>(k);
      if (k.h == 0) {
        // the rows from the fp32 values (a bit_cast of a vector element can yield element 0)
        const float* zs = reinterpret_cast<const float*>(k.lds + M.z4 + k.wave * 3 * 256) + k.lane;
        const int m = T * TILE + k.wave * 32 + k.c;
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (j < no) {
            const f16 zj = (f16)zs[j * 64];
            k.a->dz4T[((size_t)k.hd * 4 + j) * k.S + m] = __builtin_bit_cast(uint16_t, zj);
          }
      }
      const u32x4 mv = mask_read(k.lds + M.mask, k);
      half8 zz = z, w4[8];
      w4_frags<L>(w4, k);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        stage_t(img + t * ZTB, w4_tile(w4[t], zz, mv, t), k);
        opaque_h8(zz);
      }
    }
    block_sync();
    // every wave brings its own X slice of tile T+1 (16 pieces); the LOAD waves dz4 and masks
    x_dma<L, 16>(k, xrows, Tn, 16 * k.wave);
    if (ROLE == LOAD) {
      z4_dma<L>(k, Tn, lw);
      mask_dma<L>(k, k.a->masks, 3, Tn, 0, lw);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) dw_tile<true>(dw[t], img + t * ZTB, nullptr, xr, of, bias_w[t], bp[t >> 2]);
    vm_wait63(0);
    block_sync();
  }
  vm_wait63(0);
  dw_release(dw);
  write_out(ka, k, split, dw, bp);
}

// ----------------------------------------------------------------------- kernel
__global__ __launch_bounds__(THREADS, 1) void heads_bwd_kernel(KArgs ka) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int b = blockIdx.x;
  const int L = b < ka.first[1] ? 1 : b < ka.first[2] ? 2 : 3;
  const int local = b - ka.first[L - 1];
  const int ns = ka.split[L - 1];
  const int hd = local / ns, split = local - hd * ns;
  const int t0 = (int)((int64_t)split * ka.tiles / ns), t1 = (int)((int64_t)(split + 1) * ka.tiles / ns);
  Ctx k;
  k.a = &ka.a;
  k.S = ka.S;
  k.R = ka.a.R;
  k.N = ka.a.N;
  k.hd = hd;
  k.L = L;
  k.lds = lds;
  k.lane = threadIdx.x & 63;
  k.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  k.c = k.lane & 31;
  k.h = k.lane >> 5;
  if (t0 >= t1) {
    // an empty k-slice still owns a slab in deterministic mode: zeros
    if (ka.a.deterministic) {
      float* slab = ka.a.workspace + ka.part_base[hd * 3 + L - 1] + (int64_t)split * JOB_F;
      for (int e = threadIdx.x; e < JOB_F; e += THREADS) slab[e] = 0.f;
    }
    return;
  }
  const bool load = k.wave >= 2;
#ifdef HB_ONLY
  if (L != HB_ONLY) return;
#endif
  if (L == 1) {
    if (load) body1<LOAD>(ka, k, t0, t1, split); else body1<RING>(ka, k, t0, t1, split);
  } else if (L == 2) {
    if (load) body2<LOAD>(ka, k, t0, t1, split); else body2<RING>(ka, k, t0, t1, split);
  } else {
    if (load) body3<LOAD>(ka, k, t0, t1, split); else body3<RING>(ka, k, t0, t1, split);
  }
}

// Deterministic mode: dw/db of the 9 jobs = the sum of their slabs in split order.
struct RArgs {
  const float* part;
  int64_t base[9];
  int n_split[9];
  float* dw[9];
  float* db[9];
};

__global__ __launch_bounds__(256) void heads_reduce_kernel(RArgs r) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= 9 * (int64_t)JOB_F) return;
  const int j = (int)(e / JOB_F), loc = (int)(e - (int64_t)j * JOB_F);
  const float* p = r.part + r.base[j] + loc;
  float acc = 0.f;
  for (int s = 0; s < r.n_split[j]; ++s) acc += p[(int64_t)s * JOB_F];
  if (loc < 65536) r.dw[j][loc] = acc;
  else r.db[j][loc - 65536] = acc;
}

// host: splits and slab layout
bool plan(const mli_heads_bwd_args* a, KArgs& ka) {
  const int64_t S = (int64_t)a->R * a->N;
  if (a->R <= 0 || a->N <= 0 || S % TILE != 0 || S > INT32_MAX) return false;
  ka.a = *a;
  ka.S = (int)S;
  ka.tiles = (int)(S / TILE);
  // default: ~one workgroup per CU (256), l = 1 : 2 : 3 work per tile 520 : 264 : 136 MFMAs
  const int def[3] = {48, 24, 12};
  for (int i = 0; i < 3; ++i) {
    ka.split[i] = a->split[i] > 0 ? a->split[i] : def[i];
    if (ka.split[i] > 4096) return false;
  }
  ka.first[0] = 0;
  for (int i = 0; i < 3; ++i) ka.first[i + 1] = ka.first[i] + 3 * ka.split[i];
  int64_t base = 0;
  for (int hd = 0; hd < 3; ++hd)
    for (int L = 1; L <= 3; ++L) {
      ka.part_base[hd * 3 + L - 1] = base;
      base += (int64_t)ka.split[L - 1] * JOB_F;
    }
  return true;
}

}  // namespace

namespace mli_detail {
int heads_dz0_launch(const mli_heads_bwd_args* a, hipStream_t s);  // mlp.hip
}

extern "C" int mli_heads_bwd(const mli_heads_bwd_args* a, mli_stream_t s) {
  KArgs ka;
  if (!plan(a, ka) || ka.S % 256 != 0) return (int)hipErrorInvalidValue;
  if (!a->dz4 || !a->wbwd || !a->masks || !a->xT || !a->dz0T || !a->dz4T || !a->dz1f) return (int)hipErrorInvalidValue;
  for (int j = 0; j < 9; ++j)
    if (!a->dw[j] || !a->db[j]) return (int)hipErrorInvalidValue;
  if (a->deterministic && !a->workspace) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(heads_bwd_kernel, dim3(ka.first[3]), dim3(THREADS), LDS_BYTES, (hipStream_t)s, ka);
  const int e = mli_detail::heads_dz0_launch(a, (hipStream_t)s);
  if (e || !a->deterministic) return e ? e : (int)hipGetLastError();
  RArgs r;
  r.part = a->workspace;
  for (int j = 0; j < 9; ++j) {
    r.base[j] = ka.part_base[j];
    r.n_split[j] = ka.split[j % 3];
    r.dw[j] = a->dw[j];
    r.db[j] = a->db[j];
  }
  hipLaunchKernelGGL(heads_reduce_kernel, dim3((9 * JOB_F + 255) / 256), dim3(256), 0, (hipStream_t)s, r);
  return (int)hipGetLastError();
}

extern "C" int mli_heads_bwd_workspace(const mli_heads_bwd_args* a, int64_t* bytes) {
  KArgs ka;
  const int64_t S = (int64_t)a->R * a->N;
  if (!plan(a, ka) || S % 256 != 0) return (int)hipErrorInvalidValue;
  bytes[0] = (int64_t)3 * 256 * S * 2;  // dz0T
  bytes[1] = (int64_t)3 * 4 * S * 2;    // dz4T
  bytes[2] = a->deterministic ? (int64_t)3 * (ka.split[0] + ka.split[1] + ka.split[2]) * JOB_F * 4 : 0;
  bytes[3] = (int64_t)3 * 256 * S * 2;  // dz1f
  return 0;
}
