// Fused light-conditioned colour heads on gfx950 MFMA (forward + backward dX chain).
//
// Replaces MLPforNeuralSDF layer 1 (neuralangelo/utils/mlp.py:61-64) and
// LumenRGB.forward 'rgb_r_s' (NeuralLumen/utils/modules.py:148-163) with its three
// MLPwithSkipConnection heads (nerf_util.py:158-196), and their autograd backward.
//
// Structure (one workgroup = 8 waves = 256 samples, one wave = 32 samples; Geo below):
//  * activations live in registers as MFMA B fragments of the transposed layer
//    Y^T = W X^T (rows = features in the accumulator registers, samples on lanes), so the
//    accumulator of layer l is the B operand of layer l+1 with no lane movement
//    (ACC k-order, guide §3 "accumulator tile as the next MFMA's operand");
//  * weights are pre-packed (mli_pack) into per-n-tile chunks of fp16 A fragments
//    (1 KiB per k-step, one ds_read_b128 per MFMA) + 32 fp32 biases, laid out in exactly
//    the order the kernel consumes them.  All 8 waves share each chunk through a 3-slot
//    LDS ring filled by LDS-DMA (global_load_lds_dwordx4) two chunks ahead; each phase
//    ends with a COUNTED vmcnt that retires only the next chunk's DMA (the activation
//    stores issued since stay in flight: vmcnt counts loads and stores in issue order)
//    and a raw s_barrier (no __syncthreads fence, which would drain the stores);
//  * epilogues are fused: softplus(beta=100) for the SDF feature layer, ReLU (+ bit masks
//    + the activation stores for the weight gradients in training), sigmoid for the outputs.
//    The training activation / gradient images are fragment images (ABI 15, below): every wave
//    stores its own registers, 1 KiB contiguous per k-step, no LDS transpose.
#pragma once
#include "common.h"

#include <type_traits>

namespace {

constexpr int CH(int ks) { return ks * 1024 + 128; }
constexpr int FRAG_KS = 512;            // halves per k-step of a 32-sample tile's frag image (1 KiB)
constexpr int FRAG_TILE = 16 * FRAG_KS;  // halves per 32-sample tile of a 256-wide frag image
// the head layer-0 input image x0 (feat k-steps 0..15 + the extras 16..18) per 32-sample tile
constexpr int X0_KS = MLI_HEAD_K0 / 16;
constexpr int X0_TILE = X0_KS * FRAG_KS;
constexpr int Q4_SLOT = 257 * 16;  // one wave's output-layer partials Q in LDS (PQ mode, q4_tile)
constexpr int DIST = 2;                 // chunks in flight ahead of the one being read (3: no gain)
// Paired phases (run_layer_p): a barrier every second n-tile, the weight ring 4 slots deep.
// Measured (profiles/r5/pairq, alternating on one box, against a barrier per n-tile --
// MLI_HEADS_PAIR=0): rgb_fwd (train) 1.005-1.009 vs 1.030-1.042 ms, rgb_bwd 0.677-0.710 vs
// 0.716-0.745 ms, the step within noise.
#ifndef MLI_HEADS_PAIR
#define MLI_HEADS_PAIR 1
#endif
constexpr bool HEADS_PAIR = MLI_HEADS_PAIR;
constexpr int NSLOT = HEADS_PAIR ? 4 : DIST + 1;

// Wave roles.  ALL: every wave issues its share of the weight DMAs and waits.  Split (DMA +
// STORE): the first half of the waves (DMA) issue all the LDS-DMA (weights, ReLU masks) and are
// the only waves that wait on vmcnt in the phase loop; the second half (STORE) never wait there.
// Every wave stores its own activation fragments; vmcnt retires vector-memory ops in issue
// order, so the DMA waves' counted waits include the stores they issued after the chunk waited
// for (static counts per phase).
enum Role { ALL = 0, DMA = 1, STORE = 2 };

// Workgroup geometry: NW waves of 32 samples (NW * 32 samples per workgroup), a weight ring of
// NSLOT slots for chunks of up to MAXP 1 KiB pieces, split (DMA + STORE) or ALL wave roles.
// The ring DMA of one chunk is ND waves x RND pieces of 1 KiB (16 B per lane); the backward's
// ReLU-mask blocks are NW tiles x 1 KiB, double buffered.
template <int NW_, int MAXP, bool SPLIT_, int PF_ = 0>
struct Geo {
  static constexpr int NW = NW_;
  static constexpr int PF = PF_;  // weight-fragment read depth of chunk_mma
  static constexpr bool SPLIT = SPLIT_;
  static constexpr int THREADS = NW * 64;
  static constexpr int SAMPLES = NW * 32;
  static constexpr int ND = SPLIT ? NW / 2 : NW;
  static constexpr int RND = (MAXP + ND - 1) / ND;
  static constexpr int SLOT = RND * ND * 1024;
  static constexpr int RING = NSLOT * SLOT;
  static constexpr int MASKB = NW * 1024;
  static constexpr int MASK_OFF = RING;
  static constexpr int LDS_FWD = RING;
  static constexpr int LDS_BWD = MASK_OFF + 2 * MASKB;
  // PQ mode (rgb_fwd, q4_tile): the waves' Q partials parked for the cross-wave sum, then the
  // per-wave transpose scratch
  // (HEADS_PAIR: the park is two weight-ring slots free while q4_tile runs, q4_park below)
  static constexpr int QP_OFF = RING;
  static constexpr int PQ_WAVE = 2048 + 256;
  static constexpr int PQW_OFF = QP_OFF + (HEADS_PAIR ? 0 : NW * Q4_SLOT);
  static constexpr int LDS_FWD_PQ = PQW_OFF + NW * PQ_WAVE;
  // PQ mode: the first FEAT_KS k-steps of each wave's feat fragments also stay in a wave-private
  // LDS block, so the three heads re-read only the rest from the frag image
  // (even: the feat epilogue writes the two k-steps of a 32-feature tile together)
  static constexpr int FEAT_KS = 6;
  static_assert(FEAT_KS % 2 == 0, "whole 32-feature tiles of feat in LDS");
  static constexpr int LDS_FWD_PQF = LDS_FWD_PQ + NW * FEAT_KS * 1024;
  // the eval forward (no PQ blocks): 8 k-steps fit
  static constexpr int FEAT_KS_EVAL = 8;
  static_assert(FEAT_KS_EVAL % 2 == 0, "whole 32-feature tiles of feat in LDS");
  static constexpr int LDS_FWD_F = LDS_FWD + NW * FEAT_KS_EVAL * 1024;
  // ring DMAs per wave and chunk
  template <int ROLE> static constexpr int ring_ops() { return ROLE == STORE ? 0 : RND; }
};

// ---------------------------------------------------------------------- weight ring
struct Ring {
  const uint8_t* src;   // source of chunk `next`
  const uint8_t* last;  // source of the final chunk (dummy DMA past the end)
  int next, n, cur;     // next chunk to issue, total chunks, chunk being consumed
};

// The DMAs for chunk r.next into its slot (past the end: a dummy copy of the last chunk into a
// free slot, so every phase issues the same count).  bytes(c) = size of chunk c.  Piece
// u * ND + wave of the chunk (1 KiB, lanes clamped to the chunk's last 16 B) goes to the same
// offset of the slot.
template <class G, int ROLE>
MLI_FI void ring_pieces(const uint8_t* s, int nb, uint8_t* slot) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (ROLE != STORE) {
#pragma unroll
    for (int u = 0; u < G::RND; ++u)
      glds16(s + min((u * G::ND + wave) * 1024 + lane * 16, nb - 16), slot + (u * G::ND + wave) * 1024);
  }
}

template <class G, int ROLE, class Bytes>
MLI_FI void ring_issue(Ring& r, uint8_t* lds, Bytes&& bytes) {
  const bool real = r.next < r.n;
  const int nb = bytes(real ? r.next : r.n - 1);
  ring_pieces<G, ROLE>(real ? r.src : r.last, nb, lds + (r.next % NSLOT) * G::SLOT);
  if (real) r.src += nb;
  r.next++;
}

// Chunks at arbitrary places of a packed image: src(c) gives chunk c's address (its size CH(16))
struct ChunkAt {
  const uint8_t* image;
  int head_bytes;  // chunk c = (head c >> 3, n-tile c & 7) of the W1^T block of each head
  int first;       // byte offset of the W1^T block inside a head
  MLI_FI const uint8_t* src(int c) const { return image + (size_t)(c >> 3) * head_bytes + first + (c & 7) * CH(16); }
  MLI_FI int operator()(int) const { return CH(16); }
};

template <class G, int ROLE>
MLI_FI void ring_issue(Ring& r, uint8_t* lds, ChunkAt& at) {
  ring_pieces<G, ROLE>(at.src(min(r.next, r.n - 1)), CH(16), lds + (r.next % NSLOT) * G::SLOT);
  r.next++;
}

template <class Bytes>
MLI_FI void ring_start(Ring& r, const void* base, int n, Bytes&& bytes) {
  r.src = reinterpret_cast<const uint8_t*>(base);
  size_t total = 0;
  for (int c = 0; c + 1 < n; ++c) total += bytes(c);
  r.last = r.src + total;
  r.next = 0;
  r.n = n;
  r.cur = 0;
}

// ---------------------------------------------------------------------- activation images
// The training activation / gradient images the weight gradients read (the head input x0, X1..X3,
// dZ0..dZ3; stage a: dZ0..dZ4, dZ1sdf) are fragment images (ABI 15): [S/32][k-steps][64 lanes]
// [8 halves] fp16 in ACC order -- element j of lane (c, h) of k-step q is feature
// 16 q + 8 (j >> 2) + 4 h + (j & 3) of sample c of the 32-sample tile, exactly the registers
// acc_to_frag() produces.  Each wave stores its own fragments, 16 B per lane, 1 KiB contiguous
// per k-step (a tile's k-steps contiguous); mli_wgrad reads them back through LDS with
// transposing reads (ds_read_b64_tr_b16).  Measured against the tile-blocked rows of ABI 14
// (16 ds_write_b16 per lane into an LDS transpose tile, then 16 B flushes by the STORE waves):
// rgb_bwd 0.86 -> 0.74 ms, rgb_fwd 1.09 -> 1.05 ms, step 4.07 -> 3.85 ms (profiles/r5/direct).
MLI_FI void frag_store2(uint16_t* tile_img, int t, half8 f0, half8 f1, int lane) {
  // k-steps 2t and 2t+1 of the tile (a 32-feature accumulator tile t)
  half8* d = reinterpret_cast<half8*>(tile_img) + (2 * t) * 64 + lane;
  // streaming (non-temporal) stores: the activations are re-read only by a later kernel, so
  // they should not evict the weight chunks every phase re-reads from L2
  gstore_nt(d, f0);
  gstore_nt(d + 64, f1);
}

// ReLU as one v_max_i32 on the bit pattern: fmaxf on an MFMA result adds a canonicalising
// v_max first (measured 4 % of the heads forward). Every negative float (and -0) has the sign
// bit set, so max(bits, 0) is ReLU. Plain C++, not inline asm: the compiler must see the read
// of the MFMA result to insert the MFMA -> VALU wait states (an asm v_max_f32 read the
// accumulator before the MFMA had written it back).
MLI_FI float relu1(float x) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}
// The ReLU mask of an accumulator tile from its ReLU outputs r = relu1(acc): bit i = (r[i] > 0)
// = (acc[i] > 0) for every non-NaN acc.  Two VALU per element: a compare into VCC and
// b = b + b + VCC (v_addc), elements 15 .. 0 so that element i lands in bit i; the compiler's
// form (compare, select of 1 << i, or3) took 2.5.  The inputs are VALU results (relu1), not
// MFMA results, so the asm needs no MFMA -> VALU wait states.
// (the element goes through a float parameter: __builtin_bit_cast of a vector element expression
// reads element 0 -- every compare then saw the same value)
MLI_FI int f32_bits(float x) { return __builtin_bit_cast(int, x); }
MLI_FI uint32_t relu_bits16(const f32x16& r) {
  uint32_t b = 0;
#pragma unroll
  for (int i = 15; i >= 0; --i)
    asm("v_cmp_lt_i32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(b) : "v"(f32_bits(r[i])) : "vcc");
  return b;
}
// acc where bit `bit0 + i` of `bits` is set, else +0 (the backward's ReLU derivative): a signed
// one-bit field extract (0 / -1) and an and, two VALU per element (the compiler's form -- and,
// compare, select -- took three).
MLI_FI float mask_bit(float x, uint32_t bits, int bit) {
  return __builtin_bit_cast(float, __builtin_bit_cast(int, x) & __builtin_amdgcn_sbfe((int)bits, bit, 1));
}
// acc = W_chunk (32 x 16*KS) * X (16*KS x 32) + bias.  PF = 0: the compiler's schedule (it reads
// two weight fragments ahead and waits lgkmcnt(0) before every MFMA pair, so each pair pays the
// LDS latency); PF > 0: the fragments are read PF ahead, one read issued after each MFMA (the
// order pinned by sched_group_barrier).  Measured (profiles/r3/pf): PF = 4 takes the training
// heads forward 1.19 -> 1.15 ms and rgb_bwd 0.885 -> 0.86 ms; the eval forward was slower with
// it then (3.85 -> 3.95 ms per 20000-ray chunk) and took PF = 4 in round 5 (GFwd below).
template <int KS, int PF = 0>
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
  if constexpr (PF == 0) {
#pragma unroll
    for (int q = 0; q < KS; ++q) acc = mfma32(w[q * 64], X[q], acc);
  } else {
    constexpr int D = PF < KS ? PF : KS;
    half8 wr[D];
#pragma unroll
    for (int q = 0; q < D; ++q) wr[q] = w[q * 64];
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      acc = mfma32(wr[q % D], X[q], acc);
      if (q + D < KS) wr[q % D] = w[(q + D) * 64];
    }
    // the pipeline: D reads, then (MFMA, read) pairs, then the last D MFMAs
#pragma unroll
    for (int q = 0; q < D; ++q) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      if (q + D < KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  }
  return acc;
}

// One layer of NT n-tiles over KS k-steps; epi(t, acc) consumes each finished tile.
// Static store counts (for the counted vmcnt): EPI = unconditional global stores per epilogue,
// MASKED = one mask store at t == NT-1; pre.issue(t) issues pre.count(t) VMEM ops ahead of the
// weight DMAs.  STORE waves never wait in the loop: nothing they issue lands in LDS.
template <class G, int ROLE, int KS, int NT, int EPI, bool MASKED, class Bytes, class Pre, class Epi>
MLI_FI void run_layer(Ring& rg, uint8_t* lds, const half8* X, int lane, Bytes&& bytes, Pre&& pre, Epi&& epi) {
  // VMEM ops a phase issues after its weight DMAs (epilogue stores), per t in the layer
  auto stores = [](int t) MLI_LAMBDA_FI { return EPI + ((MASKED && t == NT - 1) ? 1 : 0); };
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    pre.issue(t);
    ring_issue<G, ROLE>(rg, lds, bytes);
    const f32x16 acc = chunk_mma<KS, G::PF>(lds + (rg.cur % NSLOT) * G::SLOT, X, lane);
    epi(t, acc);
    // retire chunk cur+1 (its DMAs went out DIST-1 phases ago): every VMEM op issued after
    // them may stay in flight -- the weight DMAs of the DIST-1 later phases, the mask DMAs
    // and stores of this and the previous phases (counted inside this layer, lower bound 0
    // across the layer boundary)
    if (ROLE != STORE) {
      int n = (DIST - 1) * G::template ring_ops<ROLE>() + pre.count(t) + stores(t);
#pragma unroll
      for (int b = 1; b < DIST; ++b) {
        if (t - b < 0) break;
        n += stores(t - b) + (b < DIST - 1 ? pre.count(t - b) : 0);
      }
      vm_wait(n);
    }
    block_sync();
    rg.cur++;
  }
}

struct NoPre {
  MLI_FI int count(int) const { return 0; }
  MLI_FI void issue(int) const {}
};

// run_layer with the epilogue deferred by one tile (DEFER): phase t issues the MFMA chain of tile
// t, then epi(t - 1) on the accumulators carried across the barrier (pacc), so the wave's own
// epilogue VALU work has the chain's MFMAs to hide behind instead of following them.  The last
// tile's epilogue is the caller's: the next layer runs it as `prev` at its first phase, before
// its chain in program order (it produces that chain's last k-steps).  The static store counts
// of the vmcnt waits count what is known to be issued after the chunk being retired (EPI stores
// of epi(t - 1)); undercounting only waits longer.
// MASKN: stores of the last tile's epilogue beyond EPI (the ReLU mask image); PREVN: stores that
// prev issues (the previous layer's deferred last tile); LASTN: stores the previous layer's last
// phase issued after its weight DMAs (retired at t = 0 with the chunk they follow).
template <class G, int ROLE, int KS, int NT, int EPI, int MASKN, int PREVN, bool DEFER, int LASTN = 0, class Bytes,
          class Pre, class Prev, class Epi>
MLI_FI void run_layer_d(Ring& rg, uint8_t* lds, const half8* X, int lane, Bytes&& bytes, Pre&& pre, Prev&& prev,
                        Epi&& epi, f32x16& pacc) {
  static_assert(ROLE != ALL, "split wave roles only");
  auto stores = [](int t) MLI_LAMBDA_FI {
    if (t < 0) return LASTN;
    const int pv = t == 0 ? PREVN : 0;
    if (DEFER) return pv + (t >= 1 ? EPI : 0);
    return pv + EPI + (t == NT - 1 ? MASKN : 0);
  };
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    pre.issue(t);
    ring_issue<G, ROLE>(rg, lds, bytes);
    if (t == 0) prev(pacc);
    const f32x16 acc = chunk_mma<KS, G::PF>(lds + (rg.cur % NSLOT) * G::SLOT, X, lane);
    if (DEFER) {
      if (t > 0) epi(t - 1, pacc);
      pacc = acc;
    } else {
      epi(t, acc);
    }
    if (ROLE != STORE) vm_wait((DIST - 1) * G::template ring_ops<ROLE>() + pre.count(t) + stores(t) + stores(t - 1));
    block_sync();
    rg.cur++;
  }
}

// run_layer_d in segments of two phases (HEADS_PAIR): the n-tiles of a layer are consumed two per
// barrier (a layer of one tile is a segment of its own), through a 4-slot ring.  At a segment's
// start its DMA waves issue the chunks of the NEXT segment (NEXTN of them after the layer's last
// segment) into the slots the previous segment read; at its end they wait for them -- every VMEM op
// issued after them is this segment's stores, counted statically -- and the barrier publishes them.
// A DMA has the same two phases to land as with DIST = 2, while the barriers per layer halve.
// pre.issue(t) runs at the start of the segment holding phase t, before its chunk DMAs.
template <class G, int ROLE, int KS, int NT, int EPI, int MASKN, int PREVN, bool DEFER, int NEXTN, class Bytes,
          class Pre, class Prev, class Epi>
MLI_FI void run_layer_p(Ring& rg, uint8_t* lds, const half8* X, int lane, Bytes&& bytes, Pre&& pre, Prev&& prev,
                        Epi&& epi, f32x16& pacc) {
  static_assert(ROLE != ALL, "split wave roles only");
  static_assert(NSLOT == 4, "two segments of two chunks in the ring");
  auto stores = [](int t) MLI_LAMBDA_FI {
    const int pv = t == 0 ? PREVN : 0;
    if (DEFER) return pv + (t >= 1 ? EPI : 0);
    return pv + EPI + (t == NT - 1 ? MASKN : 0);
  };
#pragma unroll
  for (int s = 0; s < NT; s += 2) {
    const int n_this = NT - s < 2 ? NT - s : 2;
    const int n_next = s + 2 < NT ? (NT - s - 2 < 2 ? NT - s - 2 : 2) : NEXTN;
#pragma unroll
    for (int t = s; t < s + n_this; ++t) pre.issue(t);
#pragma unroll
    for (int k = 0; k < n_next; ++k) ring_issue<G, ROLE>(rg, lds, bytes);
    int n = 0;
#pragma unroll
    for (int t = s; t < s + n_this; ++t) {
      if (t == 0) prev(pacc);
      const f32x16 acc = chunk_mma<KS, G::PF>(lds + (rg.cur % NSLOT) * G::SLOT, X, lane);
      if (DEFER) {
        if (t > 0) epi(t - 1, pacc);
        pacc = acc;
      } else {
        epi(t, acc);
      }
      n += stores(t);
      rg.cur++;
    }
    if (ROLE != STORE) vm_wait(n);
    block_sync();
  }
}

// One layer of the heads kernels: run_layer_d (a barrier per n-tile, LASTN) or, with HEADS_PAIR,
// run_layer_p (NEXTN: the chunks of the segment after this layer).
template <class G, int ROLE, int KS, int NT, int EPI, int MASKN, int PREVN, bool DEFER, int LASTN, int NEXTN,
          class Bytes, class Pre, class Prev, class Epi>
MLI_FI void heads_layer(Ring& rg, uint8_t* lds, const half8* X, int lane, Bytes&& bytes, Pre&& pre, Prev&& prev,
                        Epi&& epi, f32x16& pacc) {
  if constexpr (HEADS_PAIR)
    run_layer_p<G, ROLE, KS, NT, EPI, MASKN, PREVN, DEFER, NEXTN>(rg, lds, X, lane, bytes, pre, prev, epi, pacc);
  else
    run_layer_d<G, ROLE, KS, NT, EPI, MASKN, PREVN, DEFER, LASTN>(rg, lds, X, lane, bytes, pre, prev, epi, pacc);
}

// chunks the heads kernels' prologue issues and waits for before the first barrier
constexpr int PROLOGUE_CHUNKS = HEADS_PAIR ? 2 : DIST;

// The heads kernels defer every layer's epilogue by one tile.  Measured (profiles/r4/defer2,
// alternating on one box): step 4.29 / 4.30 -> 4.25 / 4.24 ms, rgb_fwd 1.150 -> 1.108-1.128 ms,
// rgb_bwd 0.926 -> 0.914-0.920 ms against the same kernels with the epilogue in place; bit-identical.
constexpr bool HEADS_DEFER = true;

// ---------------------------------------------------------------------- output-layer partials
// PQ mode (stage b): the output layer's weight gradient factors through the per-ray loss
// gradient.  The composited outputs are sums over a ray's samples, out_rc = sum_s w_s y_sc (+ bg),
// with weights w_s that do not depend on the heads, so d loss / d z4_sc = D_rc w_s y_sc (1 - y_sc)
// with D_rc = d loss / d out_rc (after the o_re chain).  Hence
//   dW4[c, :] = sum_s dz4_cs X3[:, s] = sum_tiles D[r(tile), c] Q[tile, c, :],
//   Q[tile, c, f] = sum_{s in tile} g_sc X3[f, s],   g_sc = w_s y_sc (1 - y_sc),
// and Q is formed here while X3 (the output layer's input) is still in registers: X3 never
// goes to HBM and the THIN dW GEMM that read it back is gone (mli_dw4 contracts Q with D).
// The tile's 32 samples belong to one ray (N % 32 == 0).
//
// Per 32-feature block: the wave's X3 fragments go to a wave-private LDS block as
// [32 samples][32 features] (8 B chunks XOR-swizzled by row: conflict-free b64 writes and
// transposed reads), ds_read_b64_tr_b16 returns them as B fragments with samples along k, and
// two MFMAs contract them with G^T [c][samples] (rows 0..2 = g of the head's outputs, scaled by
// MLI_Q4_SCALE into fp16 range; rows >= 3 zero).  Lane (f, h = 0) then holds Q[c = 0..3][f].
// Each wave parks its Q (257 rows of f32x4, the last one sum_s g_sc) in the Q park (QP_OFF);
// after a barrier the STORE waves sum the waves of each ray segment of the workgroup in wave
// order (fixed order: bit-reproducible) and write q4[wg][seg] -- N = 128: two rays per workgroup,
// a quarter of the per-tile partials -- and a second barrier frees the park again.
constexpr float Q4_SCALE = MLI_Q4_SCALE;  // g <= 1/4 -> fp16 <= 16384 (undone through mli_dw4 scale)

template <class G, int ROLE>
MLI_FI void q4_tile(const mli_rgb_fwd_args& a, uint8_t* lds, const half8 (&X)[19], const float (&gq)[3], int hd,
                   int lane, const Ring& rg) {
  const int wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  uint8_t* xr = lds + G::PQW_OFF + wave * G::PQ_WAVE;
  uint8_t* gr = xr + 2048;
  // the Q park of wave w.  HEADS_PAIR: after the output layer's segment the ring slots of its
  // chunk (rg.cur - 1) and of the chunk before (rg.cur - 2) are consumed, and the next DMAs into
  // them go out at the next head's first segment, after q4_tile's last barrier: waves 0..3 park in
  // the first, 4..7 in the second (4 x 4112 B <= SLOT each)
  auto q4_park = [&](int w) MLI_LAMBDA_FI {
    if constexpr (HEADS_PAIR) {
      static_assert(4 * Q4_SLOT <= G::SLOT && G::NW == 8, "Q park in two ring slots");
      const int slot = (rg.cur - (w < 4 ? 2 : 1)) % NSLOT;
      return lds + slot * G::SLOT + (w & 3) * Q4_SLOT;
    } else {
      return lds + G::QP_OFF + w * Q4_SLOT;
    }
  };
  uint8_t* qs = q4_park(wave);
  // (every LDS write and transposed read of q4_tile is asm: compiler-visible ones were preceded by
  // vmcnt(0) -- the next head's first weight DMAs are in flight -- draining the wave's stores)
  // G^T rows 0..3 (row 3 zero) from the lanes that hold the outputs
  if (h == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      ds_write_u16(lds_addr(gr + i * 64 + c * 2), __builtin_bit_cast(uint16_t, (f16)(i < 3 ? gq[i] : 0.f)));
  }
  asm volatile("" ::: "memory");
  half8 gf[2];
  {
    const int gi = min(c, 3);  // rows >= 3 read the zero row
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) gf[ks] = *reinterpret_cast<const half8*>(gr + gi * 64 + (16 * ks + 8 * h) * 2);
  }
  // transposed-read addressing: 16-lane group g16 covers features 16 (g16 & 1) .. + 15 of lane
  // half g16 >> 1; lane 4q + p of a group reads row (sample) q of the 4, chunk p of its 16 features
  const int g16 = (lane >> 4) & 3, q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = 4 * (g16 & 1) + p;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    // X3 features 32b .. 32b+31 of sample c: fragment element j of k-step 2b + u is feature
    // 16u + 8(j >> 2) + 4h + (j & 3) of the block -> 8 B chunk 4u + 2(j >> 2) + h
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const u32x4 w = __builtin_bit_cast(u32x4, X[2 * b + u]);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ch = (4 * u + 2 * jj + h) ^ ((c >> 1) & 7);
        ds_write_u64(lds_addr(xr + c * 64 + ch * 8), u32x2{w[2 * jj], w[2 * jj + 1]});
      }
    }
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    half8 xf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int s0 = 16 * ks + 8 * h + q, s1 = s0 + 4;
      const half4 lo = ds_tr16_at<0>(lds_addr(xr + s0 * 64 + (chunk ^ ((s0 >> 1) & 7)) * 8));
      const half4 hi = ds_tr16_at<0>(lds_addr(xr + s1 * 64 + (chunk ^ ((s1 >> 1) & 7)) * 8));
      xf[ks] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
    lgkm_wait<0>();
    tie(xf[0]);
    tie(xf[1]);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) acc = mfma32(gf[ks], xf[ks], acc);
    if (h == 0) ds_write_f128(lds_addr(qs + (32 * b + c) * 16), f32x4{acc[0], acc[1], acc[2], acc[3]});
  }
  // bias row 256: sum_s g_sc (fp32)
  float sb[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float v = gq[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    sb[i] = v;
  }
  if (lane == 0) ds_write_f128(lds_addr(qs + 256 * 16), f32x4{sb[0], sb[1], sb[2], 0.f});
  block_sync();
  if (ROLE != DMA) {
    // ray segments of the workgroup: tile t holds ray 32 t / N
    const int N = a.N, t0 = blockIdx.x * G::NW;
    const int r_first = t0 * 32 / N;
    const int nseg = ((t0 + G::NW) * 32 - 1) / N - r_first + 1;
    const int segs = MLI_Q4_SEGS(N);
    const int nthr = ROLE == STORE ? G::THREADS / 2 : G::THREADS;
    const int tid = ROLE == STORE ? threadIdx.x - G::THREADS / 2 : threadIdx.x;
    f32x4* qo = reinterpret_cast<f32x4*>(a.q4) + (size_t)blockIdx.x * segs * a.n_heads * 257;
    for (int it = tid; it < nseg * 257; it += nthr) {
      const int seg = it / 257, row = it - seg * 257;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < G::NW; ++w)
        if ((t0 + w) * 32 / N - r_first == seg) v += *reinterpret_cast<const f32x4*>(q4_park(w) + row * 16);
      gstore_nt(qo + ((size_t)seg * a.n_heads + hd) * 257 + row, v);
    }
  }
  block_sync();  // the Q park is free again
}

// ---------------------------------------------------------------------- forward
// chunk sizes in consumption order: SDF layer 1 (8 x KS 16), then per head L0 (8 x KS 19),
// L1..L3 (24 x KS 16), L4 (1 x KS 16)
MLI_FI int fwd_bytes(int c) { return (c >= 8 && (c - 8) % 33 < 8) ? CH(19) : CH(16); }

template <class G, bool TRAIN, bool PQ, int ROLE>
MLI_FI void rgb_fwd_body(const mli_rgb_fwd_args& a, uint8_t* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tile = blockIdx.x * G::NW + wave;
  const int m = tile * 32 + c;
  const int r = m / a.N, k = m - r * a.N;
  const size_t slot = (size_t)k * a.R + r;
  auto bytes = [](int cc) MLI_LAMBDA_FI { return fwd_bytes(cc); };
  constexpr int XL = PQ ? 3 : 4;  // activation layers stored per head (PQ: X3 is not)
  // feat k-steps the heads re-read from a wave-private LDS block (the rest: the frag image)
  constexpr int FKS = PQ ? G::FEAT_KS : (!TRAIN ? G::FEAT_KS_EVAL : 0);
  constexpr int FOFF = PQ ? G::LDS_FWD_PQ : G::LDS_FWD;
  const float wgt = PQ ? a.weights[slot] : 0.f;  // composite weight of the sample (PQ)

  Ring rg;
  ring_start(rg, a.wfwd, 8 + a.n_heads * 33, bytes);

  half8 A[16], B[19];
  // h0 frags (SDF layer-0 activations) -> B[0..15] (asm loads, waited after the prologue: see
  // gload16 -- with the extras stores pending the compiler waited vmcnt(0) for them inside the
  // feat layer, draining its first weight DMAs)
  {
    const half8* src = reinterpret_cast<const half8*>(a.h0 + (size_t)tile * FRAG_TILE) + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) B[q] = gload16(src + q * 64);
  }
  // extras (NAT order): k-step 16 = [p, n, 0...], 17 = SH(light), 18 = SH(view); in training
  // also as k-steps 16..18 of the x0 image, in ACC order (xe, stored after the prologue DMAs)
  half8 xe[3];
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
      if (TRAIN) {
        // ACC element j of lane half h is row 8 (j >> 2) + 4 h + (j & 3) of the k-step:
        // rows j / 4 + j (j < 4) and 4 + j / 8 + j (j >= 4) for h = 0 / 1
        const int lo = j < 4 ? j : 4 + j, hi = j < 4 ? 4 + j : 8 + j;
        xe[0][j] = (f16)sel_mask(hm, hi < 8 ? e16[hi & 7] : 0.f, lo < 8 ? e16[lo & 7] : 0.f);
        xe[1][j] = (f16)sel_mask(hm, shl[hi], shl[lo]);
        xe[2][j] = (f16)sel_mask(hm, shv[hi], shv[lo]);
      }
    }
  }
  // SDF layer 1's output feat (k-steps 0..15 of the tile's x0 image; in training the image is
  // also the WIDE dW operand, with the extras as k-steps 16..18)
  uint16_t* ftile = a.feat_frag + (size_t)tile * X0_TILE;
  // prologue: chunks 0 .. DIST-1 in flight, wait for chunk 0 (paired: both first chunks)
#pragma unroll
  for (int d = 0; d < PROLOGUE_CHUNKS; ++d) ring_issue<G, ROLE>(rg, lds, bytes);
  if (TRAIN) {
    half8* xd = reinterpret_cast<half8*>(ftile + 16 * FRAG_KS) + lane;
#pragma unroll
    for (int i = 0; i < 3; ++i) gstore_nt(xd + i * 64, xe[i]);
  }
  // (the h0 loads are older than the prologue DMAs and the extras stores: STORE waves, which
  // issue no DMAs, wait for them here too)
  vm_wait((HEADS_PAIR || ROLE == STORE ? 0 : (DIST - 1) * G::template ring_ops<ROLE>()) + (TRAIN ? 3 : 0));
#pragma unroll
  for (int q = 0; q < 16; ++q) tie(B[q]);
  block_sync();

  // SDF layer 1: feat = softplus(W1 h0 + b1) -> A and the x0 image
  f32x16 pacc;  // (HEADS_DEFER: the accumulators of the tile whose epilogue is pending)
  auto none = [](f32x16&) MLI_LAMBDA_FI {};
  auto feat_epi = [&](int t, const f32x16& acc) MLI_LAMBDA_FI {
    f32x16 v;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const f32x2 sp = softplus100x2((f32x2){acc[i], acc[i + 1]});
      v[i] = sp.x;
      v[i + 1] = sp.y;
    }
    A[2 * t] = acc_to_frag(v, 0);
    A[2 * t + 1] = acc_to_frag(v, 1);
    half8* dst = reinterpret_cast<half8*>(ftile) + (2 * t) * 64 + lane;
    gstore(dst, A[2 * t]);
    gstore(dst + 64, A[2 * t + 1]);
    if (2 * t + 1 < FKS) {  // (the image keeps every k-step: the vmcnt counts are static)
      half8* fl = reinterpret_cast<half8*>(lds + FOFF + wave * FKS * 1024) + (2 * t) * 64 + lane;
      fl[0] = A[2 * t];
      fl[64] = A[2 * t + 1];
    }
  };
  // (LASTN: the extras stores follow chunk 1's DMAs)
  heads_layer<G, ROLE, 16, 8, 2, 0, 0, HEADS_DEFER, TRAIN ? 3 : 0, 2>(rg, lds, B, lane, bytes, NoPre{}, none, feat_epi,
                                                                      pacc);
  if (HEADS_DEFER) feat_epi(7, pacc);  // the last feat tile, before the heads reload feat

  // feat into B[0..15] for each head (B[16..18] keep the extras).  Head 0: the feat layer's
  // output, still in A.  Heads 1, 2: k-steps < FKS from the wave's LDS block, the rest reloaded
  // from the frag image by asm loads (gload16), waited for by layer 0 after its first weight DMAs
  // went out (l0_wait): compiler-visible loads were waited with vmcnt(0), draining those DMAs.
  // The lane offset is made opaque per head so the addresses are not hoisted out of the head
  // loop (spills).
  for (int hd = 0; hd < a.n_heads; ++hd) {
    const int S = opaque_s(a.R * a.N);
    if (hd == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) B[q] = A[q];
    } else {
      const half8* src = reinterpret_cast<const half8*>(ftile) + opaque_v(lane);
      const half8* fl = reinterpret_cast<const half8*>(lds + FOFF + wave * (FKS > 0 ? FKS : 1) * 1024) + lane;
#pragma unroll
      for (int q = 0; q < 16; ++q) B[q] = q < FKS ? fl[q * 64] : gload16(src + q * 64);
    }
    // layer 0's prev hook (after its first segment's weight DMAs, before its first chain): the
    // reloads are older than those DMAs (the only VMEM ops issued since)
    auto l0_wait = [&](f32x16&) MLI_LAMBDA_FI {
      if (hd > 0) {
        vm_wait((HEADS_PAIR ? 2 : 1) * G::template ring_ops<ROLE>());
#pragma unroll
        for (int q = FKS; q < 16; ++q) tie(B[q]);
      }
    };
    uint32_t mbits[4];
    // stg: the layer's activations go to xT (PQ: not X3, the output layer's input)
    auto relu_epi = [&](half8* out, int layer, bool stg) MLI_LAMBDA_FI {
      return [&, out, layer, stg](int t, const f32x16& acc) MLI_LAMBDA_FI {
        f32x16 v;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = relu1(acc[i]);
        out[2 * t] = acc_to_frag(v, 0);
        out[2 * t + 1] = acc_to_frag(v, 1);
        if (TRAIN) {
          const uint32_t bits = relu_bits16(v);
          if (t & 1) mbits[t >> 1] |= bits << 16; else mbits[t >> 1] = bits;
          if (stg) frag_store2(a.xT + ((size_t)(hd * XL + layer) * (S / 32) + tile) * FRAG_TILE, t, out[2 * t],
                               out[2 * t + 1], lane);
          if (t == 7) {
            u32x4* mp = reinterpret_cast<u32x4*>(a.masks) +
                        ((size_t)(hd * 4 + layer) * (S / 32) + tile) * 64 + lane;
            gstore_nt(mp, u32x4{mbits[0], mbits[1], mbits[2], mbits[3]});
          }
        }
      };
    };
    auto e0 = relu_epi(A, 0, true);
    auto e1 = relu_epi(B, 1, true);
    auto e2 = relu_epi(A, 2, true);
    auto e3 = relu_epi(B, 3, !PQ);
    // (deferred: layer l's last tile is finished by layer l + 1's first phase)
    auto fin = [&](auto& e) MLI_LAMBDA_FI {
      return [&](f32x16& p) MLI_LAMBDA_FI {
        if (HEADS_DEFER) e(7, p);
      };
    };
    // static store counts of the counted waits: X = the activation fragments of an epilogue (2),
    // MN / PN = the mask store of a layer's last tile, in place / deferred to the next layer
    constexpr int MN = TRAIN ? 1 : 0, PN = TRAIN && HEADS_DEFER ? 1 : 0;
    constexpr int X = TRAIN ? 2 : 0, X3 = PQ ? 0 : X;
    constexpr int LN = HEADS_DEFER ? X : X + MN;  // stores of a layer's last phase (epi(6) when deferred)
    heads_layer<G, ROLE, 19, 8, X, MN, 0, HEADS_DEFER, 0, 2>(rg, lds, B, lane, bytes, NoPre{}, l0_wait, e0, pacc);
    heads_layer<G, ROLE, 16, 8, X, MN, PN + X, HEADS_DEFER, LN, 2>(rg, lds, A, lane, bytes, NoPre{}, fin(e0), e1, pacc);
    heads_layer<G, ROLE, 16, 8, X, MN, PN + X, HEADS_DEFER, LN, 2>(rg, lds, B, lane, bytes, NoPre{}, fin(e1), e2, pacc);
    heads_layer<G, ROLE, 16, 8, X3, MN, PN + X, HEADS_DEFER, LN, 1>(rg, lds, A, lane, bytes, NoPre{}, fin(e2), e3,
                                                                    pacc);
    const int no = hd == 2 ? 1 : 3;
    const int off = hd * 3;
    float gq[3] = {0.f, 0.f, 0.f};
    heads_layer<G, ROLE, 16, 1, 0, 0, PN + X3, false, HEADS_DEFER ? X3 : X3 + MN, 2>(rg, lds, B, lane, bytes, NoPre{},
                                                                                fin(e3),
                                          [&](int, const f32x16& acc) MLI_LAMBDA_FI {
      if (h == 0) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (i < no) {
            const float y = sigmoidf_acc(acc[i]);
            gstore_f32(a.y + 8 * slot + off + i, y);
            if (PQ) gq[i] = Q4_SCALE * wgt * (y * (1.0f - y));
          }
      }
    }, pacc);
    // (the q4 stores come from the STORE waves only: the DMA waves' counted waits are unchanged)
    if (PQ) q4_tile<G, ROLE>(a, lds, B, gq, hd, lane, rg);
  }
  vm_wait(0);  // no LDS-DMA may land after the workgroup's LDS is released
}

// Heads kernels: 8 waves (256 samples) per workgroup, one workgroup per CU.  Measured against
// 4 waves (128 samples, two independent workgroups per CU, so one workgroup's MFMAs could run
// beside the other's epilogue): training forward 1.37 vs 1.29 ms, eval 0.88 vs 0.80 ms, rgb_bwd
// 0.86 vs 0.81 ms -- the weight chunks stream through LDS once per workgroup, so halving the
// workgroup doubles the ring DMA and LDS-write work per sample.
// weight-fragment read depth of the training kernels (PF 3 / 4 / 6 measured: profiles/r3/heads_pf)
#ifndef MLI_HEADS_PF
#define MLI_HEADS_PF 4
#endif
constexpr int HEADS_PF = MLI_HEADS_PF;
// (the eval forward took PF = 0 until round 5: with the paired phases PF = 4 is faster there too,
// 800 x 800 inference 2.540-2.548 -> 2.572-2.575 M rays/s, profiles/r5/evalpf)
typedef Geo<8, 20, true, HEADS_PF> GFwd;   // eval forward
typedef Geo<8, 20, true, HEADS_PF> GFwdT;  // training forward (same layout)
typedef Geo<8, 17, true, HEADS_PF> GBwd;

// the first / second half of the waves take the DMA / STORE roles (see Role), compiled as two
// programs
template <bool TRAIN, bool PQ>
__global__ __launch_bounds__(GFwd::THREADS) void rgb_fwd_kernel(mli_rgb_fwd_args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  typedef typename std::conditional<TRAIN, GFwdT, GFwd>::type G;
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= G::NW / 2) rgb_fwd_body<G, TRAIN, PQ, STORE>(a, lds);
  else rgb_fwd_body<G, TRAIN, PQ, DMA>(a, lds);
}

// ---------------------------------------------------------------------- backward dX chain
// chunk sizes: per head W4^T (8 x KS 1), W3^T, W2^T, W1^T (24 x KS 16)
MLI_FI int bwd_bytes(int c) { return (c % 32) < 8 ? CH(1) : CH(16); }
constexpr int BWD_CHUNKS = 3 * 32;

template <class G, int ROLE>
MLI_FI void rgb_bwd_body(const mli_rgb_bwd_args& a, uint8_t* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int S = a.R * a.N;
  const int tiles = S / 32;
  const int tile = blockIdx.x * G::NW + wave;
  const int m = tile * 32 + c;
  const int r = m / a.N, k = m - r * a.N;
  const size_t slot = (size_t)k * a.R + r;
  auto bytes = [](int cc) MLI_LAMBDA_FI { return bwd_bytes(cc); };
  // ReLU-mask block of global layer L (= head*4 + li, li = 0..3 runs masks 3, 2, 1, 0): the
  // workgroup's NW tiles are contiguous (NW KiB), DMA'd by the DMA waves (two 16 B per thread)
  // into mask slot L&1
  constexpr int MASK_OPS = ROLE == DMA ? 2 : ROLE == ALL ? 1 : 0;
  auto mask_dma = [&](int L) MLI_LAMBDA_FI {
    const int Lc = min(L, 11);
    const int hd = Lc >> 2, ml = 3 - (Lc & 3);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.masks) +
                         (((size_t)(hd * 4 + ml) * tiles + (size_t)blockIdx.x * G::NW) * 64) * 16;
#pragma unroll
    for (int u = 0; u < MASK_OPS; ++u)
      glds16(src + u * (G::MASKB / 2) + threadIdx.x * 16,
             lds + G::MASK_OFF + (L & 1) * G::MASKB + u * (G::MASKB / 2) + wave * 1024);
  };

  // the sample's dz4 row (8 floats), loaded once before the ring starts: loaded per head, each
  // conditional load waited with vmcnt(0) -- for the weight DMAs in flight as well
  f32x4 dzv0, dzv1;
  {
    const f32x4* p = reinterpret_cast<const f32x4*>(a.dz4 + 8 * slot);
    dzv0 = p[0];
    dzv1 = p[1];
  }
  Ring rg;
  ring_start(rg, a.wbwd, BWD_CHUNKS, bytes);
  mask_dma(0);
#pragma unroll
  for (int d = 0; d < PROLOGUE_CHUNKS; ++d) ring_issue<G, ROLE>(rg, lds, bytes);
  if (ROLE != STORE) vm_wait(HEADS_PAIR ? 0 : (DIST - 1) * G::template ring_ops<ROLE>());
  block_sync();

  half8 A[16], B[16];
  for (int hd = 0; hd < 3; ++hd) {
    const int S = opaque_s(a.R * a.N);
    const int no = hd == 2 ? 1 : 3;
    half8 z4;
    {
      // dz4 columns 3 hd .. 3 hd + no - 1
      const float d0 = hd == 0 ? dzv0[0] : hd == 1 ? dzv0[3] : dzv1[2];
      const float d1 = hd == 0 ? dzv0[1] : dzv1[0];
      const float d2 = hd == 0 ? dzv0[2] : dzv1[1];
#pragma unroll
      for (int j = 0; j < 8; ++j) z4[j] = (f16)0.f;
      if (h == 0) {
        z4[0] = (f16)d0;
        if (no > 1) {
          z4[1] = (f16)d1;
          z4[2] = (f16)d2;
        }
      }
      // the THIN dW operand, a one-k-step fragment image (rows 0..2; NULL: the output-layer dW
      // comes from the forward's partials).  Rows j < 4 of lane half 0 are element j in both the
      // NAT and the ACC order.
      if (a.dz4T)
        gstore_nt(reinterpret_cast<half8*>(a.dz4T + ((size_t)hd * (S / 32) + tile) * FRAG_KS) + lane, z4);
    }
    // the phase whose weight DMAs fetch the next layer's first chunk (t == 8 - DIST) issues
    // that layer's mask DMA just before them
    struct MaskPre {
      decltype(mask_dma)& dma;
      int next_layer;
      MLI_FI int count(int t) const { return t == 8 - DIST ? MASK_OPS : 0; }
      MLI_FI void issue(int t) const {
        if (t == 8 - DIST) dma(next_layer);
      }
    };
    auto pre = [&](int li) MLI_LAMBDA_FI { return MaskPre{mask_dma, hd * 4 + li + 1}; };
    auto mask_epi = [&](half8* out, int layer /* dZ index */, int li) MLI_LAMBDA_FI {
      return [&, out, layer, li](int t, const f32x16& acc) MLI_LAMBDA_FI {
        const u32x4 mv =
            *reinterpret_cast<const u32x4*>(lds + G::MASK_OFF + (li & 1) * G::MASKB + wave * 1024 + lane * 16);
        const int wi = t >> 1;
        const uint32_t word = wi == 0 ? mv[0] : wi == 1 ? mv[1] : wi == 2 ? mv[2] : mv[3];
        f32x16 v;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = mask_bit(acc[i], word, (t & 1) * 16 + i);
        out[2 * t] = acc_to_frag(v, 0);
        out[2 * t + 1] = acc_to_frag(v, 1);
        frag_store2(a.dzT + ((size_t)(hd * 4 + layer) * (S / 32) + tile) * FRAG_TILE, t, out[2 * t], out[2 * t + 1],
                    lane);
      };
    };
    auto e3 = mask_epi(A, 3, 0);
    auto e2 = mask_epi(B, 2, 1);
    auto e1 = mask_epi(A, 1, 2);
    auto e0 = mask_epi(B, 0, 3);
    auto none = [](f32x16&) MLI_LAMBDA_FI {};
    auto fin = [&](auto& e) MLI_LAMBDA_FI {
      return [&](f32x16& p) MLI_LAMBDA_FI {
        if (HEADS_DEFER) e(7, p);
      };
    };
    f32x16 pacc;
    // static store counts: 2 dZ fragments per epilogue (EPI, PREVN and the previous layer's last
    // phase, LASTN)
    constexpr int X = 2, LN = X;
    heads_layer<G, ROLE, 1, 8, X, 0, 0, HEADS_DEFER, 0, 2>(rg, lds, &z4, lane, bytes, pre(0), none, e3, pacc);
    heads_layer<G, ROLE, 16, 8, X, 0, X, HEADS_DEFER, LN, 2>(rg, lds, A, lane, bytes, pre(1), fin(e3), e2, pacc);
    heads_layer<G, ROLE, 16, 8, X, 0, X, HEADS_DEFER, LN, 2>(rg, lds, B, lane, bytes, pre(2), fin(e2), e1, pacc);
    heads_layer<G, ROLE, 16, 8, X, 0, X, HEADS_DEFER, LN, 2>(rg, lds, A, lane, bytes, pre(3), fin(e1), e0, pacc);
    if (HEADS_DEFER) e0(7, pacc);  // the head's last tile (its mask slot is not refilled before the
                                   // next head's layer 0 has passed two barriers)
  }
  vm_wait(0);
}

}  // namespace

// launchers of the training forward (their kernels compile in their own translation units:
// mlp_fwd_pq.hip, mlp_fwd_train.hip)
__attribute__((visibility("hidden"))) int mli_launch_rgb_fwd_pq(const mli_rgb_fwd_args* a, hipStream_t s);
__attribute__((visibility("hidden"))) int mli_launch_rgb_fwd_train(const mli_rgb_fwd_args* a, hipStream_t s);
