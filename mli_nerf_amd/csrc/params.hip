// Parameter-side kernels: weight-norm fold + fp16 MFMA chunk packing, the weight-norm
// backward / grad assembly into the flat grad buffer, AdamW, fp16 shadow cast.
#include "common.h"

namespace {

// ---------------------------------------------------------------- pack
// Row scales g[row] / ||v[row, :]|| of every layer (torch weight_norm dim=0), one wave per
// row: blockIdx.y = layer, 4 rows per block.
__global__ __launch_bounds__(256) void row_scale_kernel(const mli_pack_layer* layers, float* row_scale) {
  const mli_pack_layer& L = layers[blockIdx.y];
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= L.n_out) return;
  const float* vr = L.v + (size_t)row * L.k_ref;
  float ss = 0.f;
  for (int k = lane; k < L.k_ref; k += 64) ss += vr[k] * vr[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if (lane == 0) row_scale[blockIdx.y * 256 + row] = L.g[row] / sqrtf(ss);
}

// One thread per 16-byte fragment block (t, q, lane) of one layer (blockIdx.y), plus
// 32 bias writers per n-tile (q == k_steps).  W = v * row_scale.
__global__ __launch_bounds__(256) void pack_kernel(const mli_pack_layer* layers, uint8_t* dst,
                                                   const float* row_scale) {
  const mli_pack_layer& L = layers[blockIdx.y];
  const float* rs = row_scale + blockIdx.y * 256;
  const int per_tile = (L.k_steps + 1) * 64;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= L.n_tiles * per_tile) return;
  const int t = gid / per_tile, rem = gid - t * per_tile;
  const int q = rem >> 6, lane = rem & 63;
  uint8_t* chunk = dst + L.dst_offset + (size_t)t * L.chunk_stride;
  const int rows_src = L.n_out, cols_src = L.k_ref;
  if (q == L.k_steps) {  // bias block: [h][i] in accumulator order
    if (lane >= 32) return;
    const int hh = lane >> 4, i = lane & 15;
    const int n = 32 * t + acc_row(i, hh);
    float b = 0.f;
    if (!L.transpose && L.bias && n < rows_src) b = L.bias[n];
    reinterpret_cast<float*>(chunk + L.k_steps * 1024)[hh * 16 + i] = b;
    return;
  }
  const int rl = lane & 31, hh = lane >> 5;
  const int n = 32 * t + rl;
  half8 out;
  const float sc_row = (!L.transpose && n < rows_src) ? rs[n] : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kk = L.kmode[q] ? k_acc(q, hh, j) : k_nat(q, hh, j);
    const int src = L.kmap[kk];
    float w = 0.f;
    if (src >= 0) {
      if (!L.transpose) {
        if (n < rows_src) w = L.v[(size_t)n * cols_src + src] * sc_row;
      } else {
        // A = W^T: row n indexes W's columns (through nmap), packed k indexes W's rows (src)
        const int col = L.nmap ? L.nmap[n] : (n < cols_src ? n : -1);
        if (col >= 0) w = L.v[(size_t)src * cols_src + col] * rs[src];
      }
    }
    out[j] = (f16)w;
  }
  *reinterpret_cast<half8*>(chunk + q * 1024 + lane * 16) = out;
}

// ---------------------------------------------------------------- grad assembly
// dW_ref[n][c] = dW_pack[n][kinv[c]] * inv_scale; weight-norm backward:
//   dg[n] = sum_c dW_ref[n][c] * v[n][c] / ||v_n||
//   dv[n][c] = g[n] / ||v_n|| * (dW_ref[n][c] - dg[n] * v[n][c] / ||v_n||)
// zero_dw (ABI 17): each dW / db element is set to 0 right after its last read, so the next
// split-K accumulation finds the buffer zeroed (no fill launch; the packed padding columns are
// never read and stay 0: their operand rows are exact zeros).
__global__ __launch_bounds__(256) void assemble_kernel(const mli_assemble_layer* layers, float inv_scale,
                                                       int zero_dw) {
  const mli_assemble_layer& L = layers[blockIdx.y];
  const int n = blockIdx.x;
  if (n >= L.n_out) return;
  __shared__ float red[2][256];
  const int tid = threadIdx.x;
  float* dwz = const_cast<float*>(L.dw);
  if (L.plain) {  // plain nn.Linear (linear_sdf, mlp.py:50): no weight-norm backward
    for (int c = tid; c < L.k_ref; c += 256) {
      const size_t i = (size_t)n * L.k_pack + L.kinv[c];
      L.grad_v[(size_t)n * L.k_ref + c] = L.dw[i] * inv_scale;
      if (zero_dw) dwz[i] = 0.f;
    }
    if (tid == 0) {
      L.grad_b[n] = L.db[n] * inv_scale;
      if (zero_dw) const_cast<float*>(L.db)[n] = 0.f;
    }
    return;
  }
  const float* vr = L.v + (size_t)n * L.k_ref;
  float ss = 0.f, dot = 0.f;
  for (int c = tid; c < L.k_ref; c += 256) {
    const float d = L.dw[(size_t)n * L.k_pack + L.kinv[c]] * inv_scale;
    ss += vr[c] * vr[c];
    dot += d * vr[c];
  }
  red[0][tid] = ss;
  red[1][tid] = dot;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      red[0][tid] += red[0][tid + s];
      red[1][tid] += red[1][tid + s];
    }
    __syncthreads();
  }
  const float nrm = sqrtf(red[0][0]);
  const float dg = red[1][0] / nrm;
  const float gs = L.g[n] / nrm;
  for (int c = tid; c < L.k_ref; c += 256) {
    const size_t i = (size_t)n * L.k_pack + L.kinv[c];
    const float d = L.dw[i] * inv_scale;
    L.grad_v[(size_t)n * L.k_ref + c] = gs * (d - dg * vr[c] / nrm);
    if (zero_dw) dwz[i] = 0.f;   // (this thread's last read of element i)
  }
  if (tid == 0) {
    L.grad_g[n] = dg;
    L.grad_b[n] = L.db[n] * inv_scale;
    if (zero_dw) const_cast<float*>(L.db)[n] = 0.f;
  }
}

// ---------------------------------------------------------------- AdamW (torch semantics)
// HBM-bound: 30 B per parameter (p, g, m, v read; p, m, v, fp16 shadow written).
// Coefficients formed in double on the host and rounded once, as torch.optim.AdamW's
// single-tensor path does with its Python scalars (torch/optim/adamw.py: lerp_(g, 1 - beta1),
// mul_(beta2).addcmul_(g, g, 1 - beta2), sqrt / bias_correction2_sqrt + eps, addcdiv_).
struct AdamwCoef {
  float decay, omb1, beta2, omb2, step_size, bc2_sqrt, eps;
};

__device__ __forceinline__ void adamw_one(const AdamwCoef& c, float& p, float g, float& m, float& v) {
  p = p * c.decay;
  m = m + (g - m) * c.omb1;
  v = v * c.beta2 + (g * g) * c.omb2;
  const float denom = sqrtf(v) / c.bc2_sqrt + c.eps;
  p = p - c.step_size * (m / denom);
}

// One parameter per lane: 6.0 TB/s on the 366 M-parameter stage-a table (11 GB per launch);
// a 4-per-lane 16 B vector variant measured 5.1 TB/s, so it is not used.
__global__ __launch_bounds__(256) void adamw_kernel(mli_adamw_args a, AdamwCoef c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  float p = a.p[i], m = a.m[i], v = a.v[i];
  const float g = a.g[i];
  adamw_one(c, p, g, m, v);
  a.p[i] = p;
  a.m[i] = m;
  a.v[i] = v;
  if (a.p16) a.p16[i] = __builtin_bit_cast(uint16_t, (f16)p);  // fp16 gather shadow (hash table)
  // the consumed gradient left zero for the next accumulation: only the entries the sparse
  // scatter touched are written (a masked store), not the whole buffer
  if (a.zero_grad && g != 0.0f) a.g[i] = 0.0f;
}

__global__ __launch_bounds__(256) void cast_kernel(mli_cast_args a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  a.dst[i] = __builtin_bit_cast(uint16_t, (f16)a.src[i]);
}

}  // namespace

extern "C" int mli_pack(const mli_pack_args* a, mli_stream_t s) {
  // the host passes max threads over layers through n_layers' descriptors; size generously
  const int max_threads = 8 * (19 + 1) * 64;
  if (a->n_layers <= 0) return 0;
  if (a->row_scale == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(row_scale_kernel, dim3(64, a->n_layers), dim3(256), 0, (hipStream_t)s, a->layers,
                     a->row_scale);
  hipLaunchKernelGGL(pack_kernel, dim3((max_threads + 255) / 256, a->n_layers), dim3(256), 0,
                     (hipStream_t)s, a->layers, a->dst, (const float*)a->row_scale);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_pack_workspace(const mli_pack_args* a, int64_t* bytes) {
  bytes[0] = (int64_t)(a->n_layers > 0 ? a->n_layers : 0) * 256 * 4;  // row_scale
  return 0;
}

extern "C" int mli_grad_assemble(const mli_assemble_args* a, mli_stream_t s) {
  hipLaunchKernelGGL(assemble_kernel, dim3(256, a->n_layers), dim3(256), 0, (hipStream_t)s,
                     a->layers, a->inv_scale, a->zero_dw);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_adamw(const mli_adamw_args* a, mli_stream_t s) {
  if (a->n <= 0) return 0;
  const double bc1 = 1.0 - pow(a->beta1, (double)a->step);
  const double bc2 = 1.0 - pow(a->beta2, (double)a->step);
  const AdamwCoef c = {(float)(1.0 - a->lr * a->weight_decay), (float)(1.0 - a->beta1), (float)a->beta2,
                       (float)(1.0 - a->beta2), (float)(a->lr / bc1), (float)sqrt(bc2), (float)a->eps};
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)((a->n + 255) / 256)), dim3(256), 0, (hipStream_t)s, *a, c);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_cast_f16(const mli_cast_args* a, mli_stream_t s) {
  if (a->n <= 0) return 0;
  hipLaunchKernelGGL(cast_kernel, dim3((unsigned)((a->n + 255) / 256)), dim3(256), 0, (hipStream_t)s, *a);
  MLI_LAUNCH_CHECK();
}

extern "C" int mli_abi_version(void) { return MLI_ABI_VERSION; }

#ifndef MLI_SOURCE_HASH
#define MLI_SOURCE_HASH "unknown"
#endif
// build.py's sha256 of the sources + flags, behind a marker it finds in the file without loading it
static const char mli_source_hash_tag[] __attribute__((used)) = "MLI_SOURCE_HASH=" MLI_SOURCE_HASH;
extern "C" const char* mli_source_hash(void) { return mli_source_hash_tag + 16; }

extern "C" const char* mli_error_string(int code) { return hipGetErrorString((hipError_t)code); }
