// Weight / bias gradients of the colour heads: dW = dZ^T X, db = sum_s dZ (split-K MFMA).
//
// Replaces the autograd dW/db GEMMs of nn.Linear inside MLPwithSkipConnection
// (projects/nerf/utils/nerf_util.py:186-196).  The operands are fp16 images of [rows][S]
// matrices in one of three layouts (mli_wgrad_job): feature-major rows (samples contiguous, a
// plain NT GEMM), tile-blocked rows ([S/256][rows][256]), or -- what the heads kernels write
// since ABI 15 -- fragment images ([S/32][k-steps][64 lanes][8 halves], the accumulator
// registers of the producing kernel), whose MFMA operands are read back through LDS with the
// transposing ds_read_b64_tr_b16 (wgrad_frag_kernel).  Each workgroup owns a BM x BN output
// tile and a k_split-sample slice; partial sums land in the fp32 outputs by atomics (few: one
// per output element per slice), or -- deterministic mode -- go to a per-slice partial slab that
// wgrad_reduce_kernel sums in slice order.
#include "common.h"

#include <algorithm>

namespace {

constexpr int MAXJOBS = 16;
constexpr int BK = 64;                 // samples per k-step (4 MFMA k-steps)
constexpr int ROWB = BK * 2 + 16;      // LDS row stride in bytes (16 B pad: conflict-free b128)

struct Job {
  const uint16_t* a; const uint16_t* b;
  int M, K, ldw;
  float* dw; float* db;
  int tiles_n, tile_base;
  int a_tiled, b_tiled;  // operand layout (MLI_WGRAD_LAYOUT_*): 0 rows [n][S], 1 tile-blocked
                         // [S/256][n][256], 2 / 3 frag image ACC / NAT order
  int a_kst, b_kst;      // frag images: k-steps per 32-sample tile
  const uint16_t* b2;    // frag images: B's k-steps b2_q .. from this image (b2_kst per tile), or NULL
  int b2_q, b2_kst;
};

// Address of (row, sample k .. k + 63) of an operand with n_rows rows: feature-major rows or the
// tile-blocked image (a 64-sample stage never crosses a 256-sample block: k is a multiple of 64).
MLI_FI const uint16_t* operand_at(const uint16_t* base, bool tiled, int n_rows, int row, size_t S, int k) {
  return tiled ? base + (size_t)(k >> 8) * n_rows * 256 + (size_t)row * 256 + (k & 255) : base + (size_t)row * S + k;
}

struct KArgs {
  Job jobs[MAXJOBS];
  int n_jobs, S, k_split, n_split;
  int share;                 // SHARE_B layout (see wgrad_kernel): the launch picks that kernel
  float* part;               // deterministic: per-job slabs [n_split][M*K + M], else NULL
  int64_t part_base[MAXJOBS];
};

// Rows [t*ROWS, t*ROWS + ROWS) x BK samples from k, 8 x 16 B per row, rows clamped to n_rows.
template <int ROWS, int LOADS, bool KEEP = false>
MLI_FI void stage_load(u32x4 (&st)[LOADS], const uint16_t* __restrict__ base, bool tiled, int n_rows, int t,
                       size_t S, int k, int tid) {
#pragma unroll
  for (int u = 0; u < LOADS; ++u) {
    const int id = u * 512 + tid, row = min(id >> 3, ROWS - 1), col = id & 7;
    const int gr = min(t * ROWS + row, n_rows - 1);
    const u32x4* src = reinterpret_cast<const u32x4*>(operand_at(base, tiled, n_rows, gr, S, k) + col * 8);
    // streamed once: non-temporal (leave L2 to the dW atomics); KEEP: rows other workgroups of
    // this XCD read next (a shared B operand), through L2
    st[u] = KEEP ? *src : __builtin_nontemporal_load(src);
  }
}

template <int ROWS, int LOADS>
MLI_FI void stage_store(const u32x4 (&st)[LOADS], uint8_t* lds, int tid) {
#pragma unroll
  for (int u = 0; u < LOADS; ++u) {
    const int id = u * 512 + tid, row = id >> 3, col = id & 7;
    if (ROWS * 8 >= (u + 1) * 512 || row < ROWS) *reinterpret_cast<u32x4*>(lds + row * ROWB + col * 16) = st[u];
  }
}

template <int BM, int BN, int WM, int WN, int DEPTH, bool SHARE_B = false>
__global__ __launch_bounds__(512) void wgrad_kernel(KArgs ka) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* la = lds;
  uint8_t* lb = lds + BM * ROWB;
  // locate job / tile / split
  int bid = blockIdx.x;
  if (SHARE_B) {
    // jobs with one tile each and the same B rows: workgroup b runs on XCD b % 8 (round-robin
    // dispatch), so the n_jobs jobs of one k-slice take consecutive slots of one XCD and the
    // slice's B rows come from HBM once, then from that XCD's L2
    const int xcd = bid & 7, slot = bid >> 3;
    const int sp = (slot / ka.n_jobs) * 8 + xcd;
    if (sp >= ka.n_split) return;
    bid = (slot % ka.n_jobs) * ka.n_split + sp;
  }
  Job J = ka.jobs[0];
#pragma unroll
  for (int j = 1; j < MAXJOBS; ++j)
    if (j < ka.n_jobs && bid >= ka.jobs[j].tile_base) J = ka.jobs[j];
  const int local = bid - J.tile_base;
  const int split = local % ka.n_split;
  const int tt = local / ka.n_split;
  const int tm = tt / J.tiles_n, tn = tt - tm * J.tiles_n;
  const int k0 = split * ka.k_split;
  const int k1 = min(ka.S, k0 + ka.k_split);
  if (k0 >= k1) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const int h = lane >> 5, rl = lane & 31;
  const size_t S = ka.S;

  // staging map: 8 x 16 B per row of BK samples; DEPTH register sets in flight
  constexpr int A_LOADS = (BM * 8 + 511) / 512, B_LOADS = (BN * 8 + 511) / 512;
  u32x4 sa[DEPTH][A_LOADS], sb[DEPTH][B_LOADS];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const bool do_bias = (J.db != nullptr) && tn == 0;
  float bsum = 0.f;  // row (tid >> 1) of the A tile, half (tid & 1)

  // clamped prefetch: past the slice end it reloads the last valid k-step (never consumed)
  auto load = [&](int d, int kk) MLI_LAMBDA_FI {
    const int kc = min(kk, k1 - BK);
    stage_load<BM, A_LOADS>(sa[d], J.a, J.a_tiled, J.M, tm, S, kc, tid);
    stage_load<BN, B_LOADS, SHARE_B>(sb[d], J.b, J.b_tiled, J.K, tn, S, kc, tid);
  };
  auto step = [&](int d, int kk) MLI_LAMBDA_FI {
    __syncthreads();
    stage_store<BM, A_LOADS>(sa[d], la, tid);
    stage_store<BN, B_LOADS>(sb[d], lb, tid);
    __syncthreads();
    load(d, kk + DEPTH * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      half8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const half8*>(la + (wm * TM * 32 + i * 32 + rl) * ROWB + ks * 32 + h * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const half8*>(lb + (wn * TN * 32 + j * 32 + rl) * ROWB + ks * 32 + h * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
    if (do_bias && (tid >> 1) < BM) {
      const half8* rowp = reinterpret_cast<const half8*>(la + (tid >> 1) * ROWB + (tid & 1) * 64);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const half8 v = rowp[u];
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += (float)v[e];
      }
    }
  };

#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, k0 + d * BK);
  for (int kk = k0; kk < k1; kk += DEPTH * BK) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
      if (kk + d * BK < k1) step(d, kk + d * BK);
  }
  // deterministic: this slice's partial tile into its slab (the reduce launch sums slices in
  // order); else fp32 atomics into the caller-zeroed dw / db
  float* slab = nullptr;
  if (ka.part != nullptr) {
    int jx = 0;
#pragma unroll
    for (int j = 1; j < MAXJOBS; ++j)
      if (j < ka.n_jobs && bid >= ka.jobs[j].tile_base) jx = j;
    slab = ka.part + ka.part_base[jx] + (int64_t)split * ((int64_t)J.M * J.K + J.M);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = tm * BM + wm * TM * 32 + i * 32 + acc_row(e, h);
        const int col = tn * BN + wn * TN * 32 + j * 32 + rl;
        if (row < J.M && col < J.K) {
          if (slab) slab[(size_t)row * J.K + col] = acc[i][j][e];
          else atomicAdd(J.dw + (size_t)row * J.ldw + col, acc[i][j][e]);
        }
      }
  if (do_bias) {
    bsum += __shfl_xor(bsum, 1);
    const int row = tm * BM + (tid >> 1);
    if ((tid & 1) == 0 && (tid >> 1) < BM && row < J.M) {
      if (slab) slab[(size_t)J.M * J.K + row] = bsum;
      else atomicAdd(J.db + row, bsum);
    }
  }
}

// LDS-DMA variant: the operand rows go global -> LDS directly (global_load_lds_dwordx4), NBUF
// stages of BKD samples in a ring, NBUF - 1 of them in flight while one is consumed -- no
// register staging, so more bytes in flight per CU than the register-staged kernel can hold
// (its second stage spills).  A stage is [BM + BN rows][BKD * 2 bytes], unpadded; 16 B chunk c
// of row r sits at position c ^ ((r >> 2) & 3), so the 16 rows a ds_read_b128 lane group reads
// cover all 64 banks.  One DMA wave-instruction fills 16 rows (lane l: row l / 4, position l % 4).
// BKD samples per stage: CPR = BKD / 8 chunks of 16 B per row, 64 / CPR rows per DMA
// wave-instruction; chunk c of row r sits at c ^ ((r / (16 / CPR)) & (CPR - 1)) (32 samples:
// c ^ ((r >> 2) & 3); 64: c ^ ((r >> 1) & 7)), so each 16-lane group of a ds_read_b128 covers
// all 64 banks.
template <int BKD>
MLI_FI int swz(int r, int c) {
  constexpr int CPR = BKD / 8;
  return c ^ ((r / (16 / CPR)) & (CPR - 1));
}

template <int BM, int BN, int WM, int WN, int NBUF, bool SHARE_B, int BKD = 32>
__global__ __launch_bounds__(512) void wgrad_dma_kernel(KArgs ka) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int RBD = BKD * 2;  // bytes per row of a stage
  constexpr int CPR = BKD / 8, RPI = 64 / CPR;  // 16 B chunks per row, rows per DMA instruction
  constexpr int ROWS = BM + BN, STAGE = ROWS * RBD;
  constexpr int PIECES = ROWS / RPI, PPW = (PIECES + 7) / 8;  // DMA wave-instructions per stage / wave
  static_assert(ROWS % RPI == 0, "stage rows");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int bid = blockIdx.x;
  if (SHARE_B) {  // as wgrad_kernel
    const int xcd = bid & 7, slot = bid >> 3;
    const int sp = (slot / ka.n_jobs) * 8 + xcd;
    if (sp >= ka.n_split) return;
    bid = (slot % ka.n_jobs) * ka.n_split + sp;
  }
  Job J = ka.jobs[0];
#pragma unroll
  for (int j = 1; j < MAXJOBS; ++j)
    if (j < ka.n_jobs && bid >= ka.jobs[j].tile_base) J = ka.jobs[j];
  const int local = bid - J.tile_base;
  const int split = local % ka.n_split;
  const int tt = local / ka.n_split;
  const int tm = tt / J.tiles_n, tn = tt - tm * J.tiles_n;
  const int k0 = split * ka.k_split;
  const int k1 = min(ka.S, k0 + ka.k_split);
  if (k0 >= k1) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const int h = lane >> 5, rl = lane & 31;
  const size_t S = ka.S;

  // this lane's DMA source rows (piece u * 8 + wave, clamped: a duplicate of the last piece
  // rewrites the same bytes, so every wave issues PPW per stage and the vmcnt counts are uniform)
  const uint16_t* src[PPW];
  int dst[PPW], bst[PPW];  // bst: the tile-blocked operand's block stride (halves), 0: rows layout
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const int piece = min(u * 8 + wave, PIECES - 1);
    const int row = piece * RPI + lane / CPR, pos = lane % CPR;
    const int c = swz<BKD>(row, pos);  // the chunk that belongs at this position
    const bool in_a = row < BM;
    const bool tiled = in_a ? J.a_tiled : J.b_tiled;
    const int n_rows = in_a ? J.M : J.K;
    const int gr = in_a ? min(tm * BM + row, J.M - 1) : min(tn * BN + row - BM, J.K - 1);
    src[u] = operand_at(in_a ? J.a : J.b, tiled, n_rows, gr, S, 0) + c * 8;
    bst[u] = tiled ? n_rows * 256 : 0;
    dst[u] = piece * 1024;
  }
  auto issue = [&](int s, int buf) MLI_LAMBDA_FI {
    const int kk = min(k0 + s * BKD, k1 - BKD);  // past the end: a dummy refetch, never consumed
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const size_t off = bst[u] ? (size_t)(kk >> 8) * bst[u] + (kk & 255) : (size_t)kk;
      glds16(src[u] + off, lds + buf * STAGE + dst[u]);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const bool do_bias = (J.db != nullptr) && tn == 0;
  float bsum = 0.f;  // row (tid >> 1) of the A tile, chunks (CPR / 2) (tid & 1) ..

  const int n_st = (k1 - k0) / BKD;
#pragma unroll
  for (int d = 0; d < NBUF - 1; ++d) issue(d, d);
  for (int st = 0; st < n_st; ++st) {
    vm_wait((NBUF - 2) * PPW);  // this wave's DMAs of stage st have landed
    block_sync();               // ... every wave's; and everyone is done with stage st - 1
    issue(st + NBUF - 1, (st + NBUF - 1) % NBUF);
    const uint8_t* sb = lds + (st % NBUF) * STAGE;
#pragma unroll
    for (int ks = 0; ks < BKD / 16; ++ks) {
      half8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * TM * 32 + i * 32 + rl;
        fa[i] = *reinterpret_cast<const half8*>(sb + r * RBD + swz<BKD>(r, 2 * ks + h) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = BM + wn * TN * 32 + j * 32 + rl;
        fb[j] = *reinterpret_cast<const half8*>(sb + r * RBD + swz<BKD>(r, 2 * ks + h) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
    if (do_bias && (tid >> 1) < BM) {
      const int r = tid >> 1;
#pragma unroll
      for (int u = 0; u < CPR / 2; ++u) {
        const half8 v = *reinterpret_cast<const half8*>(sb + r * RBD + swz<BKD>(r, (CPR / 2) * (tid & 1) + u) * 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += (float)v[e];
      }
    }
  }
  vm_wait(0);  // the dummy refetches land before the workgroup's LDS is released
  float* slab = nullptr;
  if (ka.part != nullptr) {
    int jx = 0;
#pragma unroll
    for (int j = 1; j < MAXJOBS; ++j)
      if (j < ka.n_jobs && bid >= ka.jobs[j].tile_base) jx = j;
    slab = ka.part + ka.part_base[jx] + (int64_t)split * ((int64_t)J.M * J.K + J.M);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = tm * BM + wm * TM * 32 + i * 32 + acc_row(e, h);
        const int col = tn * BN + wn * TN * 32 + j * 32 + rl;
        if (row < J.M && col < J.K) {
          if (slab) slab[(size_t)row * J.K + col] = acc[i][j][e];
          else atomicAdd(J.dw + (size_t)row * J.ldw + col, acc[i][j][e]);
        }
      }
  if (do_bias) {
    bsum += __shfl_xor(bsum, 1);
    const int row = tm * BM + (tid >> 1);
    if ((tid & 1) == 0 && (tid >> 1) < BM && row < J.M) {
      if (slab) slab[(size_t)J.M * J.K + row] = bsum;
      else atomicAdd(J.db + row, bsum);
    }
  }
}

// Fragment-image operands (ABI 15; wgrad_frag_kernel).  A 64-sample stage of an operand is its
// two 32-sample tiles' k-steps, 1 KiB each and contiguous in HBM, copied by LDS-DMA one k-step per
// wave-instruction: stage = [A: 2 tiles x KA k-steps][B: 2 tiles x KB k-steps], KA = BM / 16.
// Within a k-step the 16 B chunk of (sample c, lane half hh) -- frag lane c + 32 hh -- lands at
// chunk 32 hh + (c ^ (hh << 2 | (q & 1) << 3)), q the LDS k-step index: the DMA picks each lane's
// source so.  An MFMA operand fragment (32 features x 8 samples per lane half) is two
// ds_read_b64_tr_b16: 16-lane group g reads features 16 (g & 1) .. + 15 (k-step 2 blk + (g & 1)) of
// 4 samples, lane 4 q' + p of the group addressing sample q' and features 4 p .. 4 p + 3, which
// sit in frag lane half hh at byte b8 of the sample's chunk:
//   ACC order: hh = p & 1, b8 = 8 (p >> 1);   NAT order: hh = p >> 1, b8 = 8 (p & 1).
// A 32-lane half then reads 4 samples x 2 lane halves x 2 k-steps = 16 distinct chunk positions
// mod 16: all 64 banks once (guide T10), conflict-free.
MLI_FI int frag_chunk(int c, int hh, int qpar) { return 32 * hh + (c ^ ((hh << 2) | (qpar << 3))); }

// byte offset inside a k-step block of lane `lane`'s transposed read r (0, 1: samples 4 r .. 4 r + 3
// of its 8) of MFMA k-step half `half` (samples 16 half .. + 15 of the tile)
MLI_FI int frag_read_off(int lane, int half, int r, bool nat) {
  const int g = lane >> 4, h = lane >> 5, qq = (lane & 15) >> 2, p = lane & 3;
  const int hh = nat ? (p >> 1) : (p & 1), b8 = nat ? 8 * (p & 1) : 8 * (p >> 1);
  const int c = 16 * half + 8 * h + 4 * r + qq;
  return (g & 1) * 1024 + frag_chunk(c, hh, g & 1) * 16 + b8;
}

template <int BM, int BN, int WM, int WN, int NBUF, bool SHARE_B, int TPS>
__global__ __launch_bounds__(512) void wgrad_frag_kernel(KArgs ka) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int KA = BM / 16, KB = BN / 16;           // k-steps per tile of each operand's block
  // a stage: TPS 32-sample tiles of both operand blocks
  constexpr int PIECES = TPS * (KA + KB), PPW = (PIECES + 7) / 8;
  constexpr int STAGE = PIECES * 1024, B_OFF = TPS * KA * 1024, STG = 32 * TPS;
  static_assert(64 % STG == 0, "the k-slices are whole stages");
  static_assert(KA % 2 == 0 && KB % 2 == 0, "operand blocks of whole 32-feature tiles");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int bid = blockIdx.x;
  if (SHARE_B) {  // as wgrad_kernel
    const int xcd = bid & 7, slot = bid >> 3;
    const int sp = (slot / ka.n_jobs) * 8 + xcd;
    if (sp >= ka.n_split) return;
    bid = (slot % ka.n_jobs) * ka.n_split + sp;
  }
  Job J = ka.jobs[0];
#pragma unroll
  for (int j = 1; j < MAXJOBS; ++j)
    if (j < ka.n_jobs && bid >= ka.jobs[j].tile_base) J = ka.jobs[j];
  const int local = bid - J.tile_base;
  const int split = local % ka.n_split;
  const int tt = local / ka.n_split;
  const int tm = tt / J.tiles_n, tn = tt - tm * J.tiles_n;
  const int k0 = split * ka.k_split;
  const int k1 = min(ka.S, k0 + ka.k_split);
  if (k0 >= k1) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const int h = lane >> 5, rl = lane & 31;

  // the DMA sources: piece u * 8 + wave (clamped: a duplicate of the last piece rewrites the
  // same bytes, so every wave issues PPW per stage and the vmcnt counts are uniform); k-steps
  // past the operand's last one (rows >= M or K) re-read that k-step, whose rows are discarded.
  // Per piece a wave-uniform base (SGPRs, the wave index made scalar) plus one of two per-lane
  // offsets (the chunk swizzle of even / odd k-steps): the DMAs take the saddr form and no
  // 64-bit address lives in VGPRs (VGPR-held sources spilled once the reads became asm, and the
  // spill reloads wait vmcnt(0) -- for the DMAs too)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const uint8_t* sbase[PPW];
  int tstride[PPW];  // bytes per 32-sample tile of the piece's image
  int odd[PPW];  // the piece's k-step parity, as the lane offset's swizzle bit (1 << 7)
  auto piece_of = [&](int u) MLI_LAMBDA_FI { return min(u * 8 + wv, PIECES - 1); };
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const int piece = piece_of(u);
    const bool in_a = piece < TPS * KA;
    const int pl = in_a ? piece : piece - TPS * KA, kq = in_a ? KA : KB;
    const int tl = pl / kq, q = pl - tl * kq;
    const int rows = in_a ? J.M : J.K, first = (in_a ? tm * BM : tn * BN) / 16;
    const int qg = min(first + q, (rows + 15) / 16 - 1);
    // (B's k-steps from b2_q on: the second image)
    const bool sec = !in_a && J.b2 != nullptr && qg >= J.b2_q;
    const int kst = in_a ? J.a_kst : sec ? J.b2_kst : J.b_kst;
    tstride[u] = kst * 1024;
    sbase[u] = reinterpret_cast<const uint8_t*>(in_a ? J.a : sec ? J.b2 : J.b) + (size_t)tl * tstride[u] +
               (sec ? qg - J.b2_q : qg) * 1024;
    odd[u] = (q & 1) << 7;
  }
  // lane (c, hh) of an even k-step's piece: 16 B at (32 hh + (c ^ 4 hh)) * 16; odd: c ^ 8 as well
  const uint32_t voff = (32 * (lane >> 5) + ((lane & 31) ^ ((lane >> 5) << 2))) * 16;
  auto issue = [&](int s, int buf) MLI_LAMBDA_FI {
    const int kk = min(k0 + s * STG, k1 - STG);  // past the end: a dummy refetch, never consumed
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const uint8_t* sp = sbase[u] + (size_t)(kk >> 5) * tstride[u];
      glds16(sp + (voff ^ (uint32_t)odd[u]), lds + buf * STAGE + piece_of(u) * 1024);
    }
  };
  // 32-bit LDS addresses (stage buffer 0) of this lane's transposed reads of its wave's operand
  // blocks, per (MFMA k-step half, read) combination; the block and tile offsets inside a stage
  // are the reads' immediate offsets
  const bool a_nat = J.a_tiled == 3, b_nat = J.b_tiled == 3;
  uint32_t ba[2][2], bb[2][2];
  {
    const uint32_t l0 = lds_addr(lds);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        ba[hf][r] = l0 + 2 * wm * TM * 1024 + frag_read_off(lane, hf, r, a_nat);
        bb[hf][r] = l0 + B_OFF + 2 * wn * TN * 1024 + frag_read_off(lane, hf, r, b_nat);
      }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // db: the waves of output column block 0 sum their A fragments (row rl of each of their TM
  // blocks, samples 8 h .. 8 h + 7 of every MFMA k-step), lane halves combined at the end
  const bool do_bias = (J.db != nullptr) && tn == 0 && wn == 0;
  float bsum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) bsum[i] = 0.f;
  const half2 ones = {(f16)1.f, (f16)1.f};

  const int n_st = (k1 - k0) / STG;
#pragma unroll
  for (int d = 0; d < NBUF - 1; ++d) issue(d, d);
  for (int st = 0; st < n_st; ++st) {
    vm_wait((NBUF - 2) * PPW);  // this wave's DMAs of stage st have landed
    block_sync();               // ... every wave's; and everyone is done with stage st - 1
    issue(st + NBUF - 1, (st + NBUF - 1) % NBUF);
    const uint32_t so = (st % NBUF) * STAGE;
    // The 2 TPS MFMA k-steps of the stage.  A fragments double-buffered: k-step ks + 1's go out
    // at the start of k-step ks.  B fragments single-buffered, refilled progressively: the MFMAs
    // run column block by column block (j), and B fragment j of k-step ks + 1 is read into the
    // registers of k-step ks's the moment its last MFMA has issued -- about TN MFMA pairs of
    // cover, 20 VGPRs fewer than double-buffering B (WIDE sits at the 256-register limit of two
    // waves per SIMD).  The reads are asm (ds_tr16_at): the counted waits below are exact.
    auto read_a = [&](auto KSc, half8 (&ra)[TM]) MLI_LAMBDA_FI {
      constexpr int ks = decltype(KSc)::value, tl = ks >> 1, hf = ks & 1;
      static_for<TM>([&](auto Ic) MLI_LAMBDA_FI {
        constexpr int o = (tl * KA + 2 * decltype(Ic)::value) * 1024;
        const half4 lo = ds_tr16_at<o>(ba[hf][0] + so), hi = ds_tr16_at<o>(ba[hf][1] + so);
        ra[decltype(Ic)::value] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      });
    };
    auto read_b = [&](auto KSc, auto Jc, half8& rb) MLI_LAMBDA_FI {
      constexpr int ks = decltype(KSc)::value, tl = ks >> 1, hf = ks & 1;
      constexpr int o = (tl * KB + 2 * decltype(Jc)::value) * 1024;
      const half4 lo = ds_tr16_at<o>(bb[hf][0] + so), hi = ds_tr16_at<o>(bb[hf][1] + so);
      rb = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    half8 fa[2][TM], fb[TN];
    read_a(std::integral_constant<int, 0>{}, fa[0]);
    static_for<TN>([&](auto Jc) MLI_LAMBDA_FI { read_b(std::integral_constant<int, 0>{}, Jc, fb[decltype(Jc)::value]); });
    static_for<2 * TPS>([&](auto KSc) MLI_LAMBDA_FI {
      constexpr int ks = decltype(KSc)::value, cb = ks & 1;
      constexpr bool next = ks + 1 < 2 * TPS;
      if constexpr (next) read_a(std::integral_constant<int, ks + 1>{}, fa[cb ^ 1]);
      static_for<TN>([&](auto Jc) MLI_LAMBDA_FI {
        constexpr int j = decltype(Jc)::value;
        // issued after B(ks)[j]: B(ks)[j+1 ..], A(ks+1), B(ks+1)[0 .. j-1] -- 2 reads each
        lgkm_wait<next ? 2 * (TN - 1 + TM) : 2 * (TN - 1 - j)>();
        if constexpr (j == 0) {
#pragma unroll
          for (int i = 0; i < TM; ++i) tie(fa[cb][i]);
        }
        tie(fb[j]);
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma32(fa[cb][i], fb[j], acc[i][j]);
        if constexpr (next) read_b(std::integral_constant<int, ks + 1>{}, Jc, fb[j]);
      });
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 8; e += 2)
            bsum[i] = __builtin_amdgcn_fdot2(half2{fa[cb][i][e], fa[cb][i][e + 1]}, ones, bsum[i], false);
      }
    });
  }
  vm_wait(0);  // the dummy refetches land before the workgroup's LDS is released
  float* slab = nullptr;
  if (ka.part != nullptr) {
    int jx = 0;
#pragma unroll
    for (int j = 1; j < MAXJOBS; ++j)
      if (j < ka.n_jobs && bid >= ka.jobs[j].tile_base) jx = j;
    slab = ka.part + ka.part_base[jx] + (int64_t)split * ((int64_t)J.M * J.K + J.M);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = tm * BM + wm * TM * 32 + i * 32 + acc_row(e, h);
        const int col = tn * BN + wn * TN * 32 + j * 32 + rl;
        if (row < J.M && col < J.K) {
          if (slab) slab[(size_t)row * J.K + col] = acc[i][j][e];
          else atomicAdd(J.dw + (size_t)row * J.ldw + col, acc[i][j][e]);
        }
      }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float v = bsum[i] + __shfl_xor(bsum[i], 32);
      const int row = tm * BM + wm * TM * 32 + i * 32 + rl;
      if (h == 0 && row < J.M) {
        if (slab) slab[(size_t)J.M * J.K + row] = v;
        else atomicAdd(J.db + row, v);
      }
    }
  }
}

// Deterministic mode: out = sum over slices 0..n_split-1 (in that order) of the partial slabs.
// One thread per output element of every job (dW [M][K] then db [M]).
struct RArgs {
  const float* part;
  int64_t base[MAXJOBS], first[MAXJOBS + 1];  // slab base / first global element of job j
  float* dw[MAXJOBS];
  float* db[MAXJOBS];
  int M[MAXJOBS], K[MAXJOBS], ldw[MAXJOBS];
  int n_jobs, n_split;
};

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(RArgs r) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= r.first[r.n_jobs]) return;
  int j = 0;
#pragma unroll
  for (int q = 1; q < MAXJOBS; ++q)
    if (q < r.n_jobs && e >= r.first[q]) j = q;
  const int64_t loc = e - r.first[j];
  const int64_t MK = (int64_t)r.M[j] * r.K[j], stride = MK + r.M[j];
  if (loc >= MK && r.db[j] == nullptr) return;
  const float* p = r.part + r.base[j] + loc;
  // 16 slices' loads in flight, summed in slice order (the same fixed order: bit-identical).
  // The plain loop was one load -> vmcnt(0) -> add per slice: 80 round trips, 150 us for the
  // WIDE slabs beside the prefetched geometry (profiles/r5/final2 trace).
  float acc = 0.f;
  int sp = 0;
  for (; sp + 16 <= r.n_split; sp += 16) {
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = p[(int64_t)(sp + q) * stride];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += v[q];
  }
  for (; sp < r.n_split; ++sp) acc += p[(int64_t)sp * stride];
  if (loc < MK) {
    const int row = (int)(loc / r.K[j]), col = (int)(loc - (int64_t)row * r.K[j]);
    r.dw[j][(size_t)row * r.ldw[j] + col] = acc;
  } else {
    r.db[j][loc - MK] = acc;
  }
}


// Frag image -> feature-major rows (the wgrad operand layout), 8 tiles = 256 samples per
// workgroup, one k-step at a time through an LDS transpose so every row leaves as 512 B.
constexpr int FR_ROW = 256 * 2 + 16;
__global__ __launch_bounds__(512) void frag_rows_kernel(mli_frag_rows_args a) {
  __shared__ __attribute__((aligned(16))) uint8_t st[16 * FR_ROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int c = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x * 8 + wave;
  const bool have = tile < a.tiles;
  const half8* src = reinterpret_cast<const half8*>(a.src + (size_t)(have ? tile : 0) * a.tile_stride) + lane;
  for (int q = 0; q < a.k_steps; ++q) {
    half8 v = src[q * 64];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = a.order ? (8 * (j >> 2) + 4 * h + (j & 3)) : (8 * h + j);
      *reinterpret_cast<f16*>(st + kk * FR_ROW + (wave * 32 + c) * 2) = v[j];
    }
    __syncthreads();
    const int row = tid >> 5, col = (tid & 31) * 8;
    const int64_t s0 = (int64_t)blockIdx.x * 256 + col;
    if (s0 < (int64_t)a.tiles * 32) {
      const u32x4 x = *reinterpret_cast<const u32x4*>(st + row * FR_ROW + col * 2);
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(a.dst + (a.row0 + 16 * q + row) * a.ld + a.col0 + s0));
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------- output layer from Q
// mli_dw4: dW4[c][f] = scale * sum_(wg,seg) dray[ray][3h + c] * q4[wg][seg][h][f][c] (rows f < 256)
// and db4 from row 256.  Pass 1: workgroup b sums the (wg, seg) items of workgroups
// [wg0(b), wg0(b+1)) -- one thread per row f (257 rows: thread 0 also takes row 256) -- into
// ws[b][h][257][4]; pass 2: one workgroup per (h, row) sums the slices in a fixed order.
constexpr int DW4_SLICES = 256;

__global__ __launch_bounds__(256) void dw4_partial_kernel(mli_dw4_args a) {
  const int N = a.N, nh = a.n_heads, segs = MLI_Q4_SEGS(N);
  const int wgs = a.R * N / 256;
  const int g0 = (int)((int64_t)wgs * blockIdx.x / gridDim.x);
  const int g1 = (int)((int64_t)wgs * (blockIdx.x + 1) / gridDim.x);
  const int f = threadIdx.x;
  f32x4 acc[3], accb[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) acc[h] = accb[h] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int g = g0; g < g1; ++g) {
    const int r0 = g * 256 / N, nseg = (g * 256 + 255) / N - r0 + 1;
    for (int sg = 0; sg < nseg; ++sg) {
      const float* d = a.dray + 8 * (r0 + sg);
      const f32x4* q = reinterpret_cast<const f32x4*>(a.q4) + ((size_t)g * segs + sg) * nh * 257;
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        if (h >= nh) break;
        f32x4 dv;
#pragma unroll
        for (int c = 0; c < 4; ++c) dv[c] = c < a.k_out[h] ? d[3 * h + c] : 0.f;
        acc[h] += dv * __builtin_nontemporal_load(q + h * 257 + f);
        if (f == 0) accb[h] += dv * __builtin_nontemporal_load(q + h * 257 + 256);
      }
    }
  }
  f32x4* ws = reinterpret_cast<f32x4*>(a.workspace) + (size_t)blockIdx.x * nh * 257;
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    if (h >= nh) break;
    ws[h * 257 + f] = acc[h];
    if (f == 0) ws[h * 257 + 256] = accb[h];
  }
}

// one workgroup per (h, row): thread j holds slice j (slices <= 256), then a fixed LDS tree
__global__ __launch_bounds__(256) void dw4_reduce_kernel(mli_dw4_args a, int slices) {
  __shared__ f32x4 red[256];
  const int nh = a.n_heads, e = blockIdx.x;  // (h, row)
  const int h = e / 257, row = e - h * 257, j = threadIdx.x;
  const f32x4* ws = reinterpret_cast<const f32x4*>(a.workspace);
  red[j] = j < slices ? ws[(size_t)j * nh * 257 + e] : f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (j < o) red[j] += red[j + o];
    __syncthreads();
  }
  if (j < a.k_out[h]) {
    const float s = red[0][j] * a.scale;
    if (row < 256) a.dw[h][j * 256 + row] = s;
    else a.db[h][j] = s;
  }
}

enum { CLS_BIG = 1, CLS_WIDE = 2, CLS_THIN = 4 };

// WIDE: the three heads' layer-0 jobs share their B rows (x0T) side by side on one XCD
// (SHARE_B) and stream through the LDS-DMA ring (wgrad_dma_kernel) with this many stages
// (register staging 0.425 ms, the ring 0.415 ms)
constexpr bool WIDE_SHARE = true;
// (4 stages of 32 samples 0.413 ms, 2 stages of 64 samples -- 128 B row segments
// -- 0.353 ms)
constexpr int WIDE_DMA = 2, WIDE_BKD = 64;
// BIG through the same ring, 2 stages of 64 samples: 0.898 -> 0.847 ms (register staging of 64
// samples before; the ring at 32-sample stages -- 64 B row segments -- measured 0.998 ms)
constexpr int BIG_DMA = 2;
// the fragment-image kernel (every class): FRAG_NBUF stages of FRAG_TPS 32-sample tiles.
// 4 stages of one tile (three in flight): measured slower than 2 x 2 tiles while every stage
// waited for the next one's DMAs (BIG 0.86 -> 0.99 ms, profiles/r5/tps); with the waits counted,
// a little faster (BIG 0.823 -> 0.814-0.817, WIDE 0.249-0.261 -> 0.245-0.247 ms,
// profiles/r5/tps2)
#ifndef MLI_FRAG_TPS
#define MLI_FRAG_TPS 1
#endif
#ifndef MLI_FRAG_NBUF
#define MLI_FRAG_NBUF 4
#endif
constexpr int FRAG_TPS = MLI_FRAG_TPS, FRAG_NBUF = MLI_FRAG_NBUF;

inline int job_class(const mli_wgrad_job& j) {
  return j.M <= 32 ? CLS_THIN : (j.K <= 256 ? CLS_BIG : CLS_WIDE);
}

inline bool is_frag(int layout) { return layout == MLI_WGRAD_LAYOUT_FRAG_ACC || layout == MLI_WGRAD_LAYOUT_FRAG_NAT; }

// a job's operands: both fragment images (with enough k-steps per tile) or neither
inline bool job_valid(const mli_wgrad_job& j, int S) {
  if (j.a_tiled < 0 || j.a_tiled > 3 || j.b_tiled < 0 || j.b_tiled > 3) return false;
  const bool fa = is_frag(j.a_tiled), fb = is_frag(j.b_tiled);
  if (fa != fb) return false;
  if (j.b2_rows && (!fb || j.b2_q <= 0 || j.b2_q > j.b_kst || j.b2_kst <= 0 ||
                    j.b2_q + j.b2_kst < (j.K + 15) / 16))
    return false;
  if (fa && (j.a_kst < (j.M + 15) / 16 || (!j.b2_rows && j.b_kst < (j.K + 15) / 16))) return false;
  if ((j.a_tiled == MLI_WGRAD_LAYOUT_TILED || j.b_tiled == MLI_WGRAD_LAYOUT_TILED) && S % 256 != 0) return false;
  return true;
}

// One launch per class and operand kind (fragment images or rows): tiles of all its jobs x
// n_split k-slices, n_split sized so the grid holds about OCC workgroups per CU (OCC = resident
// 512-thread workgroups per CU).  plan(): the jobs of (cls, frag) and the split (host only; also
// the workspace query); returns the floats of partial slabs the deterministic mode needs, -1 on
// invalid jobs.
template <int BM, int BN, int OCC, bool SHARE = false>
int64_t plan(const mli_wgrad_args* a, int cls, bool frag, KArgs& ka) {
  ka.S = a->S;
  int n = 0, tiles = 0;
  for (int i = 0; i < a->n_jobs; ++i) {
    const mli_wgrad_job& j = a->jobs[i];
    if (!job_valid(j, a->S)) return -1;
    if (job_class(j) != cls || is_frag(j.a_tiled) != frag) continue;
    if (n == MAXJOBS || j.ldw < j.K || j.M <= 0 || j.K <= 0) return -1;
    Job& J = ka.jobs[n++];
    J.a = j.a_rows; J.b = j.b_rows; J.M = j.M; J.K = j.K; J.ldw = j.ldw; J.dw = j.dw; J.db = j.db;
    J.a_tiled = j.a_tiled; J.b_tiled = j.b_tiled;
    J.a_kst = j.a_kst; J.b_kst = j.b_kst;
    J.b2 = j.b2_rows; J.b2_q = j.b2_q; J.b2_kst = j.b2_kst;
    J.tiles_n = (j.K + BN - 1) / BN;
    tiles += ((j.M + BM - 1) / BM) * J.tiles_n;
  }
  ka.n_jobs = n;
  ka.part = nullptr;
  if (n == 0) return 0;
  // SHARE: every job is one tile over the same B rows -> the jobs of a k-slice run side by side
  // on one XCD (wgrad_kernel).  Its 32 CUs must hold them all in one round: a 33rd workgroup on
  // an XCD doubles the launch (measured 0.44 -> 0.71 ms), so the split is 8 x (32 / jobs).
  ka.share = 0;
  if (SHARE) {
    bool ok = n > 1;
    for (int i = 0; ok && i < n; ++i) ok = ka.jobs[i].b == ka.jobs[0].b && ka.jobs[i].M <= BM && ka.jobs[i].tiles_n == 1;
    ka.share = ok ? 1 : 0;
  }
  const int want = ka.share ? 8 * std::max(1, 32 * OCC / n) : std::max(1, 256 * OCC / tiles);
  const int steps = a->S / BK;
  ka.k_split = ((steps + want - 1) / want) * BK;
  ka.n_split = (a->S + ka.k_split - 1) / ka.k_split;
  int base = 0;
  int64_t floats = 0;
  for (int i = 0; i < n; ++i) {
    ka.jobs[i].tile_base = base;
    base += ((ka.jobs[i].M + BM - 1) / BM) * ka.jobs[i].tiles_n * ka.n_split;
    ka.part_base[i] = floats;
    floats += (int64_t)ka.n_split * ((int64_t)ka.jobs[i].M * ka.jobs[i].K + ka.jobs[i].M);
  }
  return floats;
}

template <int BM, int BN, int WM, int WN, int OCC, int DEPTH, bool SHARE_B = false, int DMA_NBUF = 0, int DMA_BKD = 32>
int launch(const mli_wgrad_args* a, int cls, bool frag, hipStream_t s) {
  KArgs ka;
  const int64_t floats = plan<BM, BN, OCC, SHARE_B>(a, cls, frag, ka);
  if (floats < 0) return (int)hipErrorInvalidValue;
  if (ka.n_jobs == 0) return 0;
  if (a->deterministic) {
    if (a->workspace == nullptr) return (int)hipErrorInvalidValue;
    ka.part = a->workspace;
  }
  int grid = 0;
  for (int i = 0; i < ka.n_jobs; ++i) grid += ((ka.jobs[i].M + BM - 1) / BM) * ka.jobs[i].tiles_n * ka.n_split;
  if (frag) {
    // fragment images: the LDS-DMA ring, FRAG_NBUF stages of FRAG_TPS tiles
    constexpr int LDS = FRAG_NBUF * FRAG_TPS * (BM / 16 + BN / 16) * 1024;
    static_assert(LDS <= 160 * 1024, "LDS");
    if (SHARE_B && ka.share)
      hipLaunchKernelGGL((wgrad_frag_kernel<BM, BN, WM, WN, FRAG_NBUF, SHARE_B, FRAG_TPS>),
                         dim3(8 * ka.n_jobs * ((ka.n_split + 7) / 8)), dim3(512), LDS, s, ka);
    else
      hipLaunchKernelGGL((wgrad_frag_kernel<BM, BN, WM, WN, FRAG_NBUF, false, FRAG_TPS>), dim3(grid), dim3(512), LDS,
                         s, ka);
  } else if (SHARE_B && ka.share) {
    grid = 8 * ka.n_jobs * ((ka.n_split + 7) / 8);
    if constexpr (SHARE_B && DMA_NBUF > 0)
      hipLaunchKernelGGL((wgrad_dma_kernel<BM, BN, WM, WN, DMA_NBUF, true, DMA_BKD>), dim3(grid), dim3(512),
                         DMA_NBUF * (BM + BN) * DMA_BKD * 2, s, ka);
    else if constexpr (SHARE_B)
      hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, DEPTH, true>), dim3(grid), dim3(512), (BM + BN) * ROWB, s, ka);
  } else if constexpr (DMA_NBUF > 0) {  // (a WIDE class of one job -- stage a -- shares nothing)
    hipLaunchKernelGGL((wgrad_dma_kernel<BM, BN, WM, WN, DMA_NBUF, false, DMA_BKD>), dim3(grid), dim3(512),
                       DMA_NBUF * (BM + BN) * DMA_BKD * 2, s, ka);
  } else {
    hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, DEPTH>), dim3(grid), dim3(512), (BM + BN) * ROWB, s, ka);
  }
  if (!a->deterministic) return (int)hipGetLastError();
  RArgs r;
  r.part = a->workspace;
  r.n_jobs = ka.n_jobs;
  r.n_split = ka.n_split;
  int64_t first = 0;
  for (int i = 0; i < ka.n_jobs; ++i) {
    const Job& J = ka.jobs[i];
    r.base[i] = ka.part_base[i];
    r.first[i] = first;
    r.dw[i] = J.dw; r.db[i] = J.db; r.M[i] = J.M; r.K[i] = J.K; r.ldw[i] = J.ldw;
    first += (int64_t)J.M * J.K + J.M;
  }
  r.first[ka.n_jobs] = first;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((first + 255) / 256)), dim3(256), 0, s, r);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int mli_wgrad(const mli_wgrad_args* a, mli_stream_t s) {
  if (a->S <= 0 || a->S % BK != 0) return (int)hipErrorInvalidValue;
  int e = 0;
  for (int frag = 0; frag < 2 && !e; ++frag) {
    if (a->classes & CLS_BIG) e = launch<256, 256, 4, 2, 1, 2, false, BIG_DMA, 64>(a, CLS_BIG, frag, (hipStream_t)s);
    if (!e && (a->classes & CLS_WIDE))
      e = launch<256, 320, 4, 2, 1, 1, WIDE_SHARE, WIDE_DMA, WIDE_BKD>(a, CLS_WIDE, frag, (hipStream_t)s);
    if (!e && (a->classes & CLS_THIN)) e = launch<32, 256, 1, 8, 2, 2>(a, CLS_THIN, frag, (hipStream_t)s);
  }
  return e;
}

extern "C" int mli_wgrad_workspace(const mli_wgrad_args* a, int64_t* bytes) {
  bytes[0] = 0;
  if (a->S <= 0 || a->S % BK != 0) return (int)hipErrorInvalidValue;
  if (!a->deterministic) return 0;
  KArgs ka;
  int64_t mx = 0, f;
  for (int frag = 0; frag < 2; ++frag) {
    if (a->classes & CLS_BIG) { if ((f = plan<256, 256, 1>(a, CLS_BIG, frag, ka)) < 0) return (int)hipErrorInvalidValue; mx = std::max(mx, f); }
    if (a->classes & CLS_WIDE) { if ((f = plan<256, 320, 1, WIDE_SHARE>(a, CLS_WIDE, frag, ka)) < 0) return (int)hipErrorInvalidValue; mx = std::max(mx, f); }
    if (a->classes & CLS_THIN) { if ((f = plan<32, 256, 2>(a, CLS_THIN, frag, ka)) < 0) return (int)hipErrorInvalidValue; mx = std::max(mx, f); }
  }
  bytes[0] = mx * 4;
  return 0;
}

extern "C" int mli_frag_rows(const mli_frag_rows_args* a, mli_stream_t s) {
  if (a->tiles <= 0 || a->k_steps <= 0) return 0;
  if (a->tiles % 8 != 0 || (a->ld % 8) != 0 || (a->col0 % 8) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(frag_rows_kernel, dim3(a->tiles / 8), dim3(512), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

static bool dw4_valid(const mli_dw4_args* a) {
  if (a->R <= 0 || a->N <= 0 || a->N % 32 != 0 || (int64_t)a->R * a->N % 256 != 0 || a->n_heads < 1 ||
      a->n_heads > 3)
    return false;
  for (int h = 0; h < a->n_heads; ++h)
    if (a->k_out[h] < 1 || a->k_out[h] > 3 || 3 * h + a->k_out[h] > 8) return false;
  return true;
}

static int dw4_slices(const mli_dw4_args* a) { return std::min(DW4_SLICES, a->R * a->N / 256); }

extern "C" int mli_dw4(const mli_dw4_args* a, mli_stream_t s) {
  if (!dw4_valid(a) || !a->q4 || !a->dray || !a->workspace) return (int)hipErrorInvalidValue;
  for (int h = 0; h < a->n_heads; ++h)
    if (!a->dw[h] || !a->db[h]) return (int)hipErrorInvalidValue;
  const int slices = dw4_slices(a);
  hipLaunchKernelGGL(dw4_partial_kernel, dim3(slices), dim3(256), 0, (hipStream_t)s, *a);
  hipLaunchKernelGGL(dw4_reduce_kernel, dim3(a->n_heads * 257), dim3(256), 0, (hipStream_t)s, *a, slices);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_dw4_workspace(const mli_dw4_args* a, int64_t* bytes) {
  if (!dw4_valid(a)) return (int)hipErrorInvalidValue;
  bytes[0] = (int64_t)dw4_slices(a) * a->n_heads * 257 * 4 * 4;
  return 0;
}
