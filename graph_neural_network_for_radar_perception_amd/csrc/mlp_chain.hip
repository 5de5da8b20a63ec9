// Fused row-MLP chains on MFMA (gfx950): ffn_block sequences with bias, per-row
// channel_normalization and activation fused into the GEMM epilogue.
//
// Replaces, for every row-wise MLP of the reference forward:
//   ffn_block              modules/neural_net/common.py:185-205 (nn.Linear -> norm -> act)
//   channel_normalization  common.py:208-220  y = s*(x-mean)/(std_unbiased+1e-5) + m
//   Activation             common.py:256-267
//   graph_feature_encoding gnn_blocks.py:19-42, message / update MLPs gnn_blocks.py:104-113,
//   task-head stems + FFN_TaskSpecificHead gnn_blocks.py:167-389.
//
// Structure.  A wave owns a tile of 16 rows.  The tile's activations live in a
// wave-private LDS slab [16 rows][<=256 features]; every layer computes
// Y^T = W . X^T with 16x16 MFMAs (A = packed weight fragments, B = the slab),
// so lane (r = lane&15, g = lane>>4) ends up holding row r's output features
// {16m + 4g + 0..3} in its accumulators.  channel_normalization's row
// statistics are an in-lane sum plus two xor-shuffles (lanes r, r+16, r+32,
// r+48 share a row): no reduction tree, no extra LDS pass.  The normalised,
// activated row goes back to the slab as the next layer's input; only the last
// layer writes HBM.  When the chain's packed weights fit, they are staged in
// LDS once per workgroup (persistent grid), so L2 sees each weight once per
// CU instead of once per tile.
//
// dtype RG_F32 : v_mfma_f32_16x16x4_f32  (exact f32 products, k-ordered fma chain)
// dtype RG_BF16: v_mfma_f32_16x16x32_bf16 (bf16 operands, f32 accumulate and epilogue)
#include "rg_common.h"
#include "x3_common.h"

namespace rg {

static constexpr int CH_WAVES = 4;
static constexpr int CH_THREADS = CH_WAVES * 64;
static constexpr int MAXW = 256;
static constexpr int TR = 16;  // rows per wave tile
static constexpr float NORM_EPS = 1e-5f;  // constants.py:9
static constexpr size_t LDS_LIMIT = 160 * 1024 - 2048;

template <typename T> struct Cfg;
template <> struct Cfg<float> {
  static constexpr int KPAD = 16;           // 4 k-steps of 4 per float4 B read
  static constexpr int STRIDE = MAXW + 8;   // 1056 B rows: conflict-free ds_read_b128
};
template <> struct Cfg<uint16_t> {
  static constexpr int KPAD = 32;
  static constexpr int STRIDE = MAXW + 16;  // 544 B rows
};
template <> struct Cfg<_Float16> : Cfg<uint16_t> {};  // IEEE fp16 slab (RG_F16), bf16's layout

__host__ __device__ inline int kpad(int k, int p) { return (k + p - 1) / p * p; }

__host__ __device__ inline size_t frag_bytes(int in_dim, int out_dim, int dtype) {
  if (dtype == RG_PACK_F32_FAST)
    return (size_t)((out_dim + 31) / 32) * ((in_dim + 7) / 8) * 1024;
  if (dtype == RG_PACK_FAST_IN || dtype == RG_PACK_FAST_CHAIN || dtype == RG_PACK_FAST_UPD)
    return (size_t)((out_dim + 31) / 32) * ((in_dim + 15) / 16) * 64 * 8 * sizeof(uint16_t);
  const size_t mt = (size_t)(out_dim + 15) / 16;
  if (dtype == RG_F32) return mt * (kpad(in_dim, 16) / 16) * 64 * 4 * sizeof(float);
  return mt * (kpad(in_dim, 32) / 32) * 64 * 8 * sizeof(uint16_t);
}
static size_t packed_bytes(int in_dim, int out_dim, int dtype) {
  if (dtype & RG_PACK_X3)  // three bf16 planes, then the bias (accumulator order)
    return 3 * frag_bytes(in_dim, out_dim, dtype & ~RG_PACK_X3) + (size_t)kpad(out_dim, 32) * sizeof(float);
  const int bpad = (dtype == RG_PACK_FAST_IN || dtype == RG_PACK_FAST_CHAIN ||
                    dtype == RG_PACK_FAST_UPD || dtype == RG_PACK_F32_FAST) ? 32 : 16;
  return frag_bytes(in_dim, out_dim, dtype) + (size_t)kpad(out_dim, bpad) * sizeof(float);
}

struct ChainLayer {
  const void* w;  // packed fragments, followed by the f32 bias padded to 16*mt
  const float* mu;
  const float* sd;
  float* save_pre;  // training tape (f32 chains): z = x W^T + b, [rows][out]
  float* save_out;  // and the activation output, [rows][out]
  int in, out, act, woff;  // woff: byte offset of this layer in the LDS weight image
};

struct ChainArgs {
  ChainLayer L[RG_MAX_LAYERS];
  int nl;
  int in_mode, in_dtype;
  int w0, w1, w2;
  int ld0, ld1, ld2;
  int ld_res, res_dtype, ld_out, out_dtype;
  int wbytes;  // total packed bytes (LDS image size when staged)
  int sstride; // slab row stride (elements): f32 kpad(widest input, 64) + 8, bf16 MAXW + 16
  long rows;
  const int* rows_dev;
  const void* in0;
  const void* in1;
  const void* in2;
  const int* idx0;
  const int* idx1;
  const void* res;
  void* out;
};

// ------------------------------------------------------------------ packing
// f32 : [m][s4][lane][4] = W[16m + (lane&15)][16*s4 + 4*(lane>>4) + t]
// bf16: [m][s ][lane][8] = W[16m + (lane&15)][32*s  + 8*(lane>>4) + j]
// weights, then the nb bias entries that follow them in the image (zeros without a bias):
// one launch per packed f32 layer (the training step repacks every layer after each SGD step)
__global__ void pack_f32_kernel(const float* __restrict__ W, int in, int out, int transpose,
                                float* __restrict__ P, long total,
                                const float* __restrict__ bias = nullptr, int nb = 0, int ld = 0) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) {
    const long i = t - total;
    if (i < nb) P[t] = (bias && i < out) ? bias[i] : 0.f;
    return;
  }
  const int S4 = kpad(in, 16) / 16;
  const int e = (int)(t & 3);
  const int lane = (int)((t >> 2) & 63);
  const long ms = t >> 8;
  const int s4 = (int)(ms % S4);
  const int m = (int)(ms / S4);
  const int o = 16 * m + (lane & 15);
  const int k = 16 * s4 + 4 * (lane >> 4) + e;
  // transpose: W holds the [in][out] matrix whose transpose is the layer; ld: W's row stride
  // (0: dense) -- a column block of a wider matrix
  const int ldw = ld ? ld : (transpose ? out : in);
  P[t] = (o < out && k < in) ? (transpose ? W[(size_t)k * ldw + o] : W[(size_t)o * ldw + k]) : 0.f;
}

// plane p > 0: the p-th term of the exact three-term bf16 split (RG_PACK_X3 | RG_BF16, the
// generic chain's f32 arithmetic on bf16 products); transpose: W holds the [in][out] matrix
// f16: IEEE fp16 fragments (RG_BF16 | RG_PACK_F16, the generic chain's fp16 operands)
__global__ void pack_bf16_kernel(const float* __restrict__ W, int in, int out, int plane,
                                 int transpose, uint16_t* __restrict__ P, long total, int f16 = 0) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int S = kpad(in, 32) / 32;
  const int j = (int)(t & 7);
  const int lane = (int)((t >> 3) & 63);
  const long ms = t >> 9;
  const int s = (int)(ms % S);
  const int m = (int)(ms / S);
  const int o = 16 * m + (lane & 15);
  const int k = 32 * s + 8 * (lane >> 4) + j;
  float v = 0.f;
  if (o < out && k < in) v = transpose ? W[(size_t)k * out + o] : W[(size_t)o * in + k];
  for (int q = 0; q < plane; ++q) v -= bf16_to_f32(f32_to_bf16(v));  // exact residues
  P[t] = f16 ? f32_to_f16(v) : f32_to_bf16(v);
}

// 32x32x16 fragments: [m][s][lane][8] = W[32m + (lane&31)][k(s, lane>>5, j)] with
// FAST_IN   k = 16s + 8h + j                                  (operand loaded from memory)
// FAST_CHAIN k = 32(s>>1) + 16(s&1) + 8(j>>2) + 4h + (j&3)    (operand = previous layer's
//            accumulator registers 8(s&1)..8(s&1)+7 of M-tile s>>1, no lane movement)
// FAST_UPD  k-steps s < in/32 as FAST_IN (x[node] from memory), the rest as FAST_CHAIN
//           offset by in/2 (aggregate from accumulators): the fused conv layer's update
// plane p > 0 (RG_PACK_X3): the p-th bf16 term of the exact three-term split of each
// weight, w = bf16(w) + bf16(w - w0) + bf16(w - w0 - w1) (conv_x3.hip)
// f16 (RG_PACK_F16): IEEE fp16 fragments instead of bf16
__global__ void pack_fast_kernel(const float* __restrict__ W, int in, int out, int mem_steps,
                                 int center, int plane, int f16, uint16_t* __restrict__ P,
                                 long total) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int S = (in + 15) / 16;
  const int j = (int)(t & 7);
  const int lane = (int)((t >> 3) & 63);
  const long ms = t >> 9;
  const int s = (int)(ms % S);
  const int m = (int)(ms / S);
  const int h = lane >> 5;
  const int o = 32 * m + (lane & 31);
  const int sc = s - mem_steps;
  const int k = s < mem_steps
                    ? 16 * s + 8 * h + j
                    : 16 * mem_steps + 32 * (sc >> 1) + 16 * (sc & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
  float v = 0.f;
  if (o < out && k < in) {
    v = W[(size_t)o * in + k];
    if (center) {  // RG_PACK_CENTERED: subtract the mean over the outputs of column k
      float cs = 0.f;
      for (int oo = 0; oo < out; ++oo) cs += W[(size_t)oo * in + k];
      v -= cs / (float)out;
    }
  }
  for (int q = 0; q < plane; ++q) v -= bf16_to_f32(f32_to_bf16(v));  // exact residues
  P[t] = f16 ? f32_to_f16(v) : f32_to_bf16(v);
}

// RG_PACK_F32_FAST: [m][s4][lane][4] = W[32m + (lane&31)][8 s4 + 4 (lane>>5) + u]; the k
// order is what both a row loaded from memory (one float4 per lane half and s4) and the
// previous layer's 32x32 accumulators (register 4g + t of M-tile m' = k-step
// 16 m' + 4g + t) supply, so one format serves every layer of an f32 chain
__global__ void pack_f32_fast_kernel(const float* __restrict__ W, int in, int out, int transpose,
                                     float* __restrict__ P, long total, int ld = 0) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int S4 = (in + 7) / 8;
  const int u = (int)(t & 3);
  const int lane = (int)((t >> 2) & 63);
  const long ms = t >> 8;
  const int s4 = (int)(ms % S4);
  const int m = (int)(ms / S4);
  const int o = 32 * m + (lane & 31);
  const int k = 8 * s4 + 4 * (lane >> 5) + u;
  // transpose: W is the [in][out] weight of the forward layer, packed as its transpose;
  // ld: W's row stride (0: dense)
  const int ldw = ld ? ld : (transpose ? out : in);
  P[t] = (o < out && k < in) ? (transpose ? W[(size_t)k * ldw + o] : W[(size_t)o * ldw + k]) : 0.f;
}

__global__ void pack_bias_kernel(const float* __restrict__ b, int out, int n, float* __restrict__ P) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) P[t] = (b && t < out) ? b[t] : 0.f;
}

// fast formats: the bias in 32x32 accumulator order, [m][h][16] with entry
// 4g + j = bias[32m + 8g + 4h + j], so lane half h of M-tile m initialises its 16
// accumulators with four contiguous 16-B LDS reads (no register moves)
__global__ void pack_bias_frag_kernel(const float* __restrict__ b, int out, int n, int center,
                                      float* __restrict__ P) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int m = t >> 5, h = (t >> 4) & 1, g = (t >> 2) & 3, j = t & 3;
  const int f = 32 * m + 8 * g + 4 * h + j;
  float v = (b && f < out) ? b[f] : 0.f;
  if (center && b && f < out) {
    float cs = 0.f;
    for (int o = 0; o < out; ++o) cs += b[o];
    v -= cs / (float)out;
  }
  P[t] = v;
}

// ------------------------------------------------------------------ element access
__device__ __forceinline__ float ld_elem(const void* p, int dt, size_t i) {
  if (dt == RG_F32) return ((const float*)p)[i];
  const uint16_t h = ((const uint16_t*)p)[i];
  return dt == RG_F16 ? f16_to_f32(h) : bf16_to_f32(h);
}
__device__ __forceinline__ void st_elem(void* p, int dt, size_t i, float v) {
  if (dt == RG_F32) ((float*)p)[i] = v;
  else ((uint16_t*)p)[i] = dt == RG_F16 ? f32_to_f16(v) : f32_to_bf16(v);
}

// 4 consecutive elements of a row, as floats (vector load when aligned and complete)
__device__ __forceinline__ f32x4 ld4(const void* p, int dt, size_t i, int valid, bool vec) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (vec && valid >= 4) {
    if (dt == RG_F32) {
      v = *(const f32x4*)((const float*)p + i);
    } else if (dt == RG_F16) {
      const uint2 u = *(const uint2*)((const uint16_t*)p + i);
      v.x = f16_to_f32((uint16_t)(u.x & 0xffffu));
      v.y = f16_to_f32((uint16_t)(u.x >> 16));
      v.z = f16_to_f32((uint16_t)(u.y & 0xffffu));
      v.w = f16_to_f32((uint16_t)(u.y >> 16));
    } else {
      const uint2 u = *(const uint2*)((const uint16_t*)p + i);
      v.x = __uint_as_float(u.x << 16);
      v.y = __uint_as_float(u.x & 0xffff0000u);
      v.z = __uint_as_float(u.y << 16);
      v.w = __uint_as_float(u.y & 0xffff0000u);
    }
  } else {
    if (valid > 0) v.x = ld_elem(p, dt, i);
    if (valid > 1) v.y = ld_elem(p, dt, i + 1);
    if (valid > 2) v.z = ld_elem(p, dt, i + 2);
    if (valid > 3) v.w = ld_elem(p, dt, i + 3);
  }
  return v;
}

template <typename T> __device__ __forceinline__ void st4_slab(T* p, f32x4 v);
template <> __device__ __forceinline__ void st4_slab<float>(float* p, f32x4 v) { *(f32x4*)p = v; }
template <> __device__ __forceinline__ void st4_slab<uint16_t>(uint16_t* p, f32x4 v) {
  uint2 w;
  w.x = pack_bf16x2(v.x, v.y);
  w.y = pack_bf16x2(v.z, v.w);
  *(uint2*)p = w;
}
template <> __device__ __forceinline__ void st4_slab<_Float16>(_Float16* p, f32x4 v) {
  uint2 w;
  w.x = pack_f16x2(v.x, v.y);
  w.y = pack_f16x2(v.z, v.w);
  *(uint2*)p = w;
}

// element f of row `row` of the (concatenated / gathered) chain input
__device__ __forceinline__ float input_elem(const ChainArgs& a, long row, int f) {
  switch (a.in_mode) {
    case RG_IN_DENSE:
      return f < a.w0 ? ld_elem(a.in0, a.in_dtype, (size_t)row * a.ld0 + f) : 0.f;
    case RG_IN_CONCAT2:
      if (f < a.w0) return ld_elem(a.in0, a.in_dtype, (size_t)row * a.ld0 + f);
      if (f < a.w0 + a.w1) return ld_elem(a.in1, a.in_dtype, (size_t)row * a.ld1 + (f - a.w0));
      return 0.f;
    case RG_IN_GATHER3:
      if (f < a.w0) return ld_elem(a.in0, a.in_dtype, (size_t)a.idx0[row] * a.ld0 + f);
      if (f < 2 * a.w0) return ld_elem(a.in0, a.in_dtype, (size_t)a.idx1[row] * a.ld0 + (f - a.w0));
      if (f < 2 * a.w0 + a.w2)
        return ld_elem(a.in2, a.in_dtype, (size_t)row * a.ld2 + (f - 2 * a.w0));
      return 0.f;
    default:  // RG_IN_PAIRADD
      if (f < a.w0)
        return __fadd_rn(ld_elem(a.in0, a.in_dtype, (size_t)a.idx0[row] * a.ld0 + f),
                         ld_elem(a.in0, a.in_dtype, (size_t)a.idx1[row] * a.ld0 + f));
      return 0.f;
  }
}

// 4-feature chunk [f, f+4) of the chain input of row `row`; vector loads when the
// chunk lies inside one aligned segment, element loads otherwise
__device__ __forceinline__ f32x4 input_chunk(const ChainArgs& a, long row, int f, bool al0,
                                             bool al1, bool al2) {
  switch (a.in_mode) {
    case RG_IN_DENSE:
      if (al0 && f + 4 <= a.w0) return ld4(a.in0, a.in_dtype, (size_t)row * a.ld0 + f, 4, true);
      break;
    case RG_IN_CONCAT2:
      if (al0 && f + 4 <= a.w0) return ld4(a.in0, a.in_dtype, (size_t)row * a.ld0 + f, 4, true);
      if (al0 && al1 && f >= a.w0 && f + 4 <= a.w0 + a.w1)
        return ld4(a.in1, a.in_dtype, (size_t)row * a.ld1 + (f - a.w0), 4, true);
      break;
    case RG_IN_GATHER3:
      if (al0 && f + 4 <= a.w0)
        return ld4(a.in0, a.in_dtype, (size_t)a.idx0[row] * a.ld0 + f, 4, true);
      if (al0 && f >= a.w0 && f + 4 <= 2 * a.w0)
        return ld4(a.in0, a.in_dtype, (size_t)a.idx1[row] * a.ld0 + (f - a.w0), 4, true);
      if (al0 && al2 && f >= 2 * a.w0 && f + 4 <= 2 * a.w0 + a.w2)
        return ld4(a.in2, a.in_dtype, (size_t)row * a.ld2 + (f - 2 * a.w0), 4, true);
      break;
    default:
      if (al0 && f + 4 <= a.w0) {
        const f32x4 x0 = ld4(a.in0, a.in_dtype, (size_t)a.idx0[row] * a.ld0 + f, 4, true);
        const f32x4 x1 = ld4(a.in0, a.in_dtype, (size_t)a.idx1[row] * a.ld0 + f, 4, true);
        return (f32x4){__fadd_rn(x0.x, x1.x), __fadd_rn(x0.y, x1.y), __fadd_rn(x0.z, x1.z),
                       __fadd_rn(x0.w, x1.w)};
      }
      break;
  }
  f32x4 v;
  v.x = input_elem(a, row, f);
  v.y = input_elem(a, row, f + 1);
  v.z = input_elem(a, row, f + 2);
  v.w = input_elem(a, row, f + 3);
  return v;
}

// fill the wave slab with the chain input of rows [r0, r0+16), zero padded to K0p
template <typename T>
__device__ __forceinline__ void load_input(const ChainArgs& a, T* slab, long r0, long rows, int lane, int K0p) {
  const int SS = a.sstride;
  const int nch = K0p / 4;
  const int total = TR * nch;
  const bool al0 = (a.ld0 % 4 == 0) && (a.w0 % 4 == 0);
  const bool al1 = (a.ld1 % 4 == 0) && (a.w1 % 4 == 0);
  const bool al2 = (a.ld2 % 4 == 0) && (a.w2 % 4 == 0);
  for (int t = lane; t < total; t += 64) {
    const int r = t / nch;
    const int f = (t - r * nch) * 4;
    const long row = r0 + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < rows) v = input_chunk(a, row, f, al0, al1, al2);
    st4_slab<T>(slab + r * SS + f, v);
  }
}

// ------------------------------------------------------------------ MFMA layer body
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma;
template <> struct Mfma<float> {
  static __device__ __forceinline__ void run(f32x4 (&acc)[16], const float* slab, const float* P,
                                             int mt, int K, int lane, int SS) {
    const int S4 = kpad(K, 16) / 16;
    const float* brow = slab + (lane & 15) * SS + 4 * (lane >> 4);
    for (int s4 = 0; s4 < S4; ++s4) {
      const f32x4 b = *(const f32x4*)(brow + 16 * s4);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (m < mt) {
          const f32x4 av = *(const f32x4*)(P + (((size_t)m * S4 + s4) * 64 + lane) * 4);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b.x, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b.y, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, b.z, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, b.w, acc[m], 0, 0, 0);
        }
      }
    }
  }
};
template <> struct Mfma<uint16_t> {
  static __device__ __forceinline__ void run(f32x4 (&acc)[16], const uint16_t* slab,
                                             const uint16_t* P, int mt, int K, int lane, int SS) {
    const int S = kpad(K, 32) / 32;
    const uint16_t* brow = slab + (lane & 15) * SS + 8 * (lane >> 4);
    for (int s = 0; s < S; ++s) {
      const bf16x8_t b = __builtin_bit_cast(bf16x8_t, *(const u32x4*)(brow + 32 * s));
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (m < mt) {
          const u32x4 av = *(const u32x4*)(P + (((size_t)m * S + s) * 64 + lane) * 8);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av), b,
                                                            acc[m], 0, 0, 0);
        }
      }
    }
  }
};

template <> struct Mfma<_Float16> {  // RG_F16: v_mfma_f32_16x16x32_f16, bf16's fragment layout
  typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ void run(f32x4 (&acc)[16], const _Float16* slab,
                                             const _Float16* P, int mt, int K, int lane, int SS) {
    const int S = kpad(K, 32) / 32;
    const _Float16* brow = slab + (lane & 15) * SS + 8 * (lane >> 4);
    for (int s = 0; s < S; ++s) {
      const f16x8_t b = __builtin_bit_cast(f16x8_t, *(const u32x4*)(brow + 32 * s));
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (m < mt) {
          const u32x4 av = *(const u32x4*)(P + (((size_t)m * S + s) * 64 + lane) * 8);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, av), b,
                                                           acc[m], 0, 0, 0);
        }
      }
    }
  }
};

// float32 arithmetic on the bf16 matrix cores (RG_F32X3): the f32 slab's 8 k values per
// lane split exactly into three bf16 terms (x3_common.h), weights pre-split into three
// planes of the 16x16x32 fragment format; six products of weight <= 2 per k-step
struct MfmaX3 {
  static __device__ __forceinline__ void run(f32x4 (&acc)[16], const float* slab,
                                             const uint16_t* P, int mt, int K, int lane, int SS,
                                             size_t pl) {
    const int S = kpad(K, 32) / 32;
    const float* brow = slab + (lane & 15) * SS + 8 * (lane >> 4);
    for (int s = 0; s < S; ++s) {
      const x3::X3 b = x3::split8(*(const f32x4*)(brow + 32 * s), *(const f32x4*)(brow + 32 * s + 4));
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (m < mt) {
          const uint16_t* pa = P + (((size_t)m * S + s) * 64 + lane) * 8;
          const bf16x8_t a0 = __builtin_bit_cast(bf16x8_t, *(const u32x4*)pa);
          const bf16x8_t a1 = __builtin_bit_cast(bf16x8_t, *(const u32x4*)(pa + pl));
          const bf16x8_t a2 = __builtin_bit_cast(bf16x8_t, *(const u32x4*)(pa + 2 * pl));
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b.p0, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b.p1, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b.p2, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b.p0, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b.p1, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b.p0, acc[m], 0, 0, 0);
        }
      }
    }
  }
};

// bias (already in acc) -> channel_normalization -> activation; features >= out -> 0.
// Lane (r, g) holds features 16m + 4g + e of row r; the row's other features
// sit in lanes r^16, r^32, r^48.
__device__ __forceinline__ void epilogue(f32x4 (&acc)[16], const ChainLayer& L, int mt, int g) {
  const int out = L.out;
  if (L.mu) {
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (m < mt) s += (acc[m].x + acc[m].y) + (acc[m].z + acc[m].w);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mean = s / (float)out;
    float ss = 0.f;
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (m < mt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[m][e] - mean;
          ss += (16 * m + 4 * g + e) < out ? d * d : 0.f;
        }
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    const float stdv = __fsqrt_rn(ss / (float)(out - 1));
    const float inv = 1.f / (stdv + NORM_EPS);
    const float gs = *L.sd, gb = *L.mu;
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (m < mt)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[m][e] = __fadd_rn(__fmul_rn(gs, __fmul_rn(acc[m][e] - mean, inv)), gb);
  }
  act_dispatch(L.act, [&](auto A) {
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (m < mt)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[m][e] = (16 * m + 4 * g + e) < out ? act_t<decltype(A)::value>(acc[m][e]) : 0.f;
  });
}

// final layer -> HBM (optional residual add, gnn_blocks.py:109)
__device__ __forceinline__ void store_rows(const f32x4 (&acc)[16], const ChainArgs& a, long row,
                                           int mt, int out, int g) {
  const bool vec = (out % 4 == 0) && (a.ld_out % 4 == 0) && (!a.res || a.ld_res % 4 == 0);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    if (m < mt) {
      const int f0 = 16 * m + 4 * g;
      if (f0 >= out) continue;
      f32x4 v = acc[m];
      if (a.res) {
        const f32x4 rv = ld4(a.res, a.res_dtype, (size_t)row * a.ld_res + f0, out - f0, vec);
        v.x = __fadd_rn(rv.x, v.x);
        v.y = __fadd_rn(rv.y, v.y);
        v.z = __fadd_rn(rv.z, v.z);
        v.w = __fadd_rn(rv.w, v.w);
      }
      if (vec) {
        if (a.out_dtype == RG_F32) {
          *(f32x4*)((float*)a.out + (size_t)row * a.ld_out + f0) = v;
        } else if (a.out_dtype == RG_F16) {
          uint2 w;
          w.x = pack_f16x2(v.x, v.y);
          w.y = pack_f16x2(v.z, v.w);
          *(uint2*)((uint16_t*)a.out + (size_t)row * a.ld_out + f0) = w;
        } else {
          uint2 w;
          w.x = pack_bf16x2(v.x, v.y);
          w.y = pack_bf16x2(v.z, v.w);
          *(uint2*)((uint16_t*)a.out + (size_t)row * a.ld_out + f0) = w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (f0 + e < out) st_elem(a.out, a.out_dtype, (size_t)row * a.ld_out + f0 + e, v[e]);
      }
    }
  }
}

// training tape: row `row`'s features 16m + 4g + e (< out) -> dst[row][out]
__device__ __forceinline__ void save_rows(const f32x4 (&acc)[16], float* dst, long row, int mt,
                                          int out, int g) {
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    if (m < mt) {
      const int f0 = 16 * m + 4 * g;
      float* p = dst + (size_t)row * out + f0;
      if ((out & 3) == 0 && f0 < out) {
        *(f32x4*)p = acc[m];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (f0 + e < out) p[e] = acc[m][e];
      }
    }
  }
}

template <typename T, bool WLDS, bool X3 = false>
__global__ __launch_bounds__(CH_THREADS) void chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // layer descriptors: copied with static indices (a dynamically indexed kernel
  // argument would be spilled to scratch), then read with the runtime layer index
  ChainLayer* sL = (ChainLayer*)smem;
#pragma unroll
  for (int i = 0; i < RG_MAX_LAYERS; ++i)
    if (threadIdx.x == i) sL[i] = a.L[i];
  const int dbytes = (int)((sizeof(ChainLayer) * RG_MAX_LAYERS + 15) & ~(size_t)15);
  char* wimg = smem + dbytes;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, r = lane & 15;
  T* slab = (T*)(wimg + (WLDS ? ((a.wbytes + 15) & ~15) : 0) +
                 (size_t)wave * TR * a.sstride * sizeof(T));
  __syncthreads();
  if (WLDS) {
    // stage every layer's packed weights (+bias) into LDS once per workgroup
    for (int l = 0; l < a.nl; ++l) {
      const int nb = (l + 1 < a.nl ? sL[l + 1].woff : a.wbytes) - sL[l].woff;
      stage_lds<CH_THREADS>(wimg + sL[l].woff, sL[l].w, nb);
    }
    __syncthreads();
  }
  const long rows = a.rows_dev ? min((long)*a.rows_dev, a.rows) : a.rows;
  const long ntiles = (rows + TR - 1) / TR;
  const int dt = sizeof(T) == 4 ? RG_F32 : RG_BF16;
  constexpr int KP = X3 ? 32 : Cfg<T>::KPAD;  // k-step depth of the slab's zero padding
  const int K0p = kpad(sL[0].in, KP);
  for (long tile = (long)blockIdx.x * CH_WAVES + wave; tile < ntiles;
       tile += (long)gridDim.x * CH_WAVES) {
    const long r0 = tile * TR;
    load_input<T>(a, slab, r0, rows, lane, K0p);
    f32x4 acc[16];
    for (int l = 0; l < a.nl; ++l) {
      const ChainLayer L = sL[l];
      const int mt = (L.out + 15) / 16;
      const T* P = WLDS ? (const T*)(wimg + L.woff) : (const T*)L.w;
      const size_t fb = frag_bytes(L.in, L.out, X3 ? RG_BF16 : dt);
      const float* bias = (const float*)((const char*)P + (X3 ? 3 * fb : fb));
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (m < mt) acc[m] = *(const f32x4*)(bias + 16 * m + 4 * g);
      if constexpr (X3)
        MfmaX3::run(acc, slab, (const uint16_t*)P, mt, L.in, lane, a.sstride, fb / sizeof(uint16_t));
      else
        Mfma<T>::run(acc, slab, P, mt, L.in, lane, a.sstride);
      if (L.save_pre && r0 + r < rows) save_rows(acc, L.save_pre, r0 + r, mt, L.out, g);
      epilogue(acc, L, mt, g);
      if (L.save_out && r0 + r < rows) save_rows(acc, L.save_out, r0 + r, mt, L.out, g);
      if (l + 1 < a.nl) {
        T* row = slab + r * a.sstride;
#pragma unroll
        for (int m = 0; m < 16; ++m)
          if (m < mt) st4_slab<T>(row + 16 * m + 4 * g, acc[m]);
        // zero the next layer's K padding beyond the 16*mt features written above
        // (bf16 k-steps are 32 deep: an odd tile count leaves 16 stale columns)
        if (kpad(L.out, KP) > 16 * mt)
          st4_slab<T>(row + 16 * mt + 4 * g, (f32x4){0.f, 0.f, 0.f, 0.f});
      } else {
        const long row = r0 + r;
        if (row < rows) store_rows(acc, a, row, mt, L.out, g);
      }
    }
  }
}

template <typename T, bool WLDS, bool X3 = false>
static int launch_chain(const ChainArgs& a, long rows, hipStream_t st) {
  const size_t dbytes = (sizeof(ChainLayer) * RG_MAX_LAYERS + 15) & ~(size_t)15;
  const size_t lds = dbytes + (WLDS ? ((size_t)(a.wbytes + 15) & ~(size_t)15) : 0) +
                     (size_t)CH_WAVES * TR * a.sstride * sizeof(T);
  RG_ENSURE_LDS((chain_kernel<T, WLDS, X3>), (int)LDS_LIMIT);
  const long tiles = (rows + TR - 1) / TR;
  long blocks = (tiles + CH_WAVES - 1) / CH_WAVES;
  // persistent grid: enough resident workgroups to fill 256 CUs
  const int per_cu = lds <= 40 * 1024 ? 4 : (lds <= 78 * 1024 ? 2 : 1);
  const long cap = 256L * per_cu * (WLDS ? 1 : 4);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  chain_kernel<T, WLDS, X3><<<blocks, CH_THREADS, lds, st>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

}  // namespace rg

using namespace rg;

extern "C" size_t rg_packed_linear_bytes(int in_dim, int out_dim, int dtype) {
  return packed_bytes(in_dim, out_dim, dtype & ~(RG_PACK_CENTERED | RG_PACK_TRANSPOSE | RG_PACK_F16));
}

// RG_PACK_X3: three planes of one RG_PACK_FAST_* format, or of RG_BF16 (the generic chain's
// 16x16x32 fragments; transpose allowed), then the f32 bias
static int pack_x3(const float* weight, const float* bias, int in_dim, int out_dim, int fmt,
                   int center, int transpose, void* packed, hipStream_t st) {
  if (fmt == RG_BF16) {
    RG_REQUIRE(!center, RG_ERR_ARG, "rg_pack_linear: RG_PACK_CENTERED applies to the fast formats");
    const size_t fb = frag_bytes(in_dim, out_dim, RG_BF16);
    const long total = (long)fb / sizeof(uint16_t);
    for (int p = 0; p < 3; ++p)
      pack_bf16_kernel<<<ceil_div(total, 256), 256, 0, st>>>(
          weight, in_dim, out_dim, p, transpose, (uint16_t*)((char*)packed + p * fb), total);
    const int nb = kpad(out_dim, 32);
    pack_bias_kernel<<<ceil_div(nb, 256), 256, 0, st>>>(bias, out_dim, nb,
                                                        (float*)((char*)packed + 3 * fb));
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  RG_REQUIRE(!transpose, RG_ERR_ARG,
             "rg_pack_linear: RG_PACK_X3 with RG_PACK_TRANSPOSE applies to RG_BF16");
  RG_REQUIRE(fmt == RG_PACK_FAST_IN || fmt == RG_PACK_FAST_CHAIN || fmt == RG_PACK_FAST_UPD,
             RG_ERR_ARG, "rg_pack_linear: RG_PACK_X3 applies to RG_BF16 and the RG_PACK_FAST_* formats");
  const int ks = (in_dim + 15) / 16;
  RG_REQUIRE(fmt != RG_PACK_FAST_UPD || in_dim % 64 == 0, RG_ERR_ARG,
             "RG_PACK_FAST_UPD needs in_dim = 2*C with C a multiple of 32");
  const int mem_steps = fmt == RG_PACK_FAST_IN ? ks : (fmt == RG_PACK_FAST_CHAIN ? 0 : ks / 2);
  const size_t fb = frag_bytes(in_dim, out_dim, fmt);
  const long total = (long)fb / sizeof(uint16_t);
  for (int p = 0; p < 3; ++p)
    pack_fast_kernel<<<ceil_div(total, 256), 256, 0, st>>>(weight, in_dim, out_dim, mem_steps,
                                                           center, p, 0,
                                                           (uint16_t*)((char*)packed + p * fb), total);
  const int nb = kpad(out_dim, 32);
  pack_bias_frag_kernel<<<ceil_div(nb, 256), 256, 0, st>>>(bias, out_dim, nb, center,
                                                           (float*)((char*)packed + 3 * fb));
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_pack_linear(const float* weight, const float* bias, int in_dim, int out_dim,
                              int dtype, void* packed, void* stream) {
  RG_REQUIRE(in_dim > 0 && out_dim > 0 && in_dim <= MAXW && out_dim <= MAXW, RG_ERR_UNSUPPORTED,
             "rg_pack_linear: dims %dx%d outside 1..%d", out_dim, in_dim, MAXW);
  hipStream_t st = (hipStream_t)stream;
  const int f16 = (dtype & RG_PACK_F16) ? 1 : 0;
  dtype &= ~RG_PACK_F16;
  RG_REQUIRE(!f16 || dtype == RG_BF16 || ((dtype & ~RG_PACK_CENTERED) >= RG_PACK_FAST_IN &&
                                          (dtype & ~RG_PACK_CENTERED) <= RG_PACK_FAST_UPD),
             RG_ERR_ARG, "rg_pack_linear: RG_PACK_F16 applies to RG_BF16 and the RG_PACK_FAST_* formats");
  if (dtype & RG_PACK_X3) {
    return pack_x3(weight, bias, in_dim, out_dim,
                   dtype & ~(RG_PACK_X3 | RG_PACK_CENTERED | RG_PACK_TRANSPOSE),
                   (dtype & RG_PACK_CENTERED) ? 1 : 0, (dtype & RG_PACK_TRANSPOSE) ? 1 : 0, packed,
                   st);
  }
  const int center = (dtype & RG_PACK_CENTERED) ? 1 : 0;
  const int transpose = (dtype & RG_PACK_TRANSPOSE) ? 1 : 0;
  dtype &= ~(RG_PACK_CENTERED | RG_PACK_TRANSPOSE);
  RG_REQUIRE(!transpose || dtype == RG_F32 || dtype == RG_PACK_F32_FAST, RG_ERR_ARG,
             "rg_pack_linear: RG_PACK_TRANSPOSE applies to RG_F32 and RG_PACK_F32_FAST");
  RG_REQUIRE(!center || (dtype >= RG_PACK_FAST_IN && dtype <= RG_PACK_FAST_UPD), RG_ERR_ARG,
             "rg_pack_linear: RG_PACK_CENTERED applies to the bf16 RG_PACK_FAST_* formats");
  if (dtype == RG_F32) {
    // weights and bias in one launch (the bias follows the weights: pb below)
    const long total = (long)frag_bytes(in_dim, out_dim, dtype) / sizeof(float);
    const int nb = kpad(out_dim, 16);
    pack_f32_kernel<<<ceil_div(total + nb, 256), 256, 0, st>>>(weight, in_dim, out_dim, transpose,
                                                               (float*)packed, total, bias, nb);
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  if (dtype == RG_BF16) {
    long total = (long)frag_bytes(in_dim, out_dim, dtype) / sizeof(uint16_t);
    pack_bf16_kernel<<<ceil_div(total, 256), 256, 0, st>>>(weight, in_dim, out_dim, 0, 0,
                                                           (uint16_t*)packed, total, f16);
  } else if (dtype == RG_PACK_FAST_IN || dtype == RG_PACK_FAST_CHAIN || dtype == RG_PACK_FAST_UPD) {
    long total = (long)frag_bytes(in_dim, out_dim, dtype) / sizeof(uint16_t);
    const int ks = (in_dim + 15) / 16;
    RG_REQUIRE(dtype != RG_PACK_FAST_UPD || in_dim % 64 == 0, RG_ERR_ARG,
               "RG_PACK_FAST_UPD needs in_dim = 2*C with C a multiple of 32");
    const int mem_steps = dtype == RG_PACK_FAST_IN ? ks : (dtype == RG_PACK_FAST_CHAIN ? 0 : ks / 2);
    pack_fast_kernel<<<ceil_div(total, 256), 256, 0, st>>>(weight, in_dim, out_dim, mem_steps,
                                                           center, 0, f16, (uint16_t*)packed,
                                                           total);
  } else if (dtype == RG_PACK_F32_FAST) {
    long total = (long)frag_bytes(in_dim, out_dim, dtype) / sizeof(float);
    pack_f32_fast_kernel<<<ceil_div(total, 256), 256, 0, st>>>(weight, in_dim, out_dim, transpose,
                                                               (float*)packed, total);
  } else {
    RG_REQUIRE(false, RG_ERR_ARG, "rg_pack_linear: bad dtype %d", dtype);
  }
  const int nb = kpad(out_dim, (dtype >= RG_PACK_FAST_IN) ? 32 : 16);
  float* pb = (float*)((char*)packed + frag_bytes(in_dim, out_dim, dtype));
  if (dtype >= RG_PACK_FAST_IN)
    pack_bias_frag_kernel<<<ceil_div(nb, 256), 256, 0, st>>>(bias, out_dim, nb, center, pb);
  else
    pack_bias_kernel<<<ceil_div(nb, 256), 256, 0, st>>>(bias, out_dim, nb, pb);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_pack_linear_ld(const float* weight, const float* bias, int in_dim, int out_dim,
                                 int dtype, int ld, void* packed, void* stream) {
  const int transpose = (dtype & RG_PACK_TRANSPOSE) ? 1 : 0;
  const int fmt = dtype & ~RG_PACK_TRANSPOSE;
  RG_REQUIRE(fmt == RG_F32 || fmt == RG_PACK_F32_FAST, RG_ERR_ARG,
             "rg_pack_linear_ld: RG_F32 or RG_PACK_F32_FAST (| RG_PACK_TRANSPOSE)");
  RG_REQUIRE(in_dim > 0 && out_dim > 0 && in_dim <= MAXW && out_dim <= MAXW, RG_ERR_UNSUPPORTED,
             "rg_pack_linear_ld: dims %dx%d outside 1..%d", out_dim, in_dim, MAXW);
  RG_REQUIRE(ld == 0 || ld >= (transpose ? out_dim : in_dim), RG_ERR_ARG,
             "rg_pack_linear_ld: ld %d shorter than a row", ld);
  hipStream_t st = (hipStream_t)stream;
  const long total = (long)frag_bytes(in_dim, out_dim, fmt) / sizeof(float);
  if (fmt == RG_F32) {
    const int nb = kpad(out_dim, 16);
    pack_f32_kernel<<<ceil_div(total + nb, 256), 256, 0, st>>>(weight, in_dim, out_dim, transpose,
                                                               (float*)packed, total, bias, nb, ld);
  } else {
    pack_f32_fast_kernel<<<ceil_div(total, 256), 256, 0, st>>>(weight, in_dim, out_dim, transpose,
                                                               (float*)packed, total, ld);
    const int nb = kpad(out_dim, 32);
    pack_bias_frag_kernel<<<ceil_div(nb, 256), 256, 0, st>>>(
        bias, out_dim, nb, 0, (float*)((char*)packed + frag_bytes(in_dim, out_dim, fmt)));
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// rg_pack_linear_jobs: blockIdx.y = job, a grid-stride loop over its weights then its bias
// (RG_F32: plain, padded to 16; RG_PACK_F32_FAST: accumulator order, padded to 32) -- the same
// element formulas as pack_f32_kernel / pack_f32_fast_kernel / pack_bias_frag_kernel
__global__ void pack_jobs_kernel(const rg_pack_job* __restrict__ jobs) {
  const rg_pack_job j = jobs[blockIdx.y];
  const bool fast = j.fmt == RG_PACK_F32_FAST;
  const long total = (long)frag_bytes(j.in_dim, j.out_dim, j.fmt) / sizeof(float);
  const int nb = kpad(j.out_dim, fast ? 32 : 16);
  float* P = (float*)j.packed;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total + nb;
       t += (long)gridDim.x * blockDim.x) {
    if (t >= total) {
      const int i = (int)(t - total);
      int f = i;
      if (fast) {
        const int m = i >> 5, h = (i >> 4) & 1, g = (i >> 2) & 3, q = i & 3;
        f = 32 * m + 8 * g + 4 * h + q;
      }
      P[t] = (j.bias && f < j.out_dim) ? j.bias[f] : 0.f;
      continue;
    }
    const int e = (int)(t & 3);
    const int lane = (int)((t >> 2) & 63);
    const long ms = t >> 8;
    int o, k;
    if (fast) {
      const int S4 = (j.in_dim + 7) / 8;
      o = 32 * (int)(ms / S4) + (lane & 31);
      k = 8 * (int)(ms % S4) + 4 * (lane >> 5) + e;
    } else {
      const int S4 = kpad(j.in_dim, 16) / 16;
      o = 16 * (int)(ms / S4) + (lane & 15);
      k = 16 * (int)(ms % S4) + 4 * (lane >> 4) + e;
    }
    const int ldw = j.ld ? j.ld : (j.transpose ? j.out_dim : j.in_dim);
    P[t] = (o < j.out_dim && k < j.in_dim)
               ? (j.transpose ? j.weight[(size_t)k * ldw + o] : j.weight[(size_t)o * ldw + k])
               : 0.f;
  }
}

extern "C" int rg_pack_linear_jobs(const rg_pack_job* jobs, int n_jobs, void* stream) {
  RG_REQUIRE(n_jobs >= 0 && n_jobs <= 65535 && (jobs || n_jobs == 0), RG_ERR_ARG,
             "rg_pack_linear_jobs: %d jobs", n_jobs);
  if (n_jobs == 0) return RG_OK;
  // 64 blocks of 256 per job: the largest f32 image (256 x 256 + bias) in four passes
  pack_jobs_kernel<<<dim3(64, n_jobs), 256, 0, (hipStream_t)stream>>>(jobs);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_mlp_chain(int dtype, const rg_layer* layers, int n_layers, long rows,
                            const int* rows_dev, int in_mode, int in_dtype, const void* in0,
                            int ld0, int w0, const void* in1, int ld1, int w1, const void* in2,
                            int ld2, int w2, const int* idx0, const int* idx1,
                            const void* residual, int ld_res, int res_dtype, void* out,
                            int ld_out, int out_dtype, void* stream) {
  RG_REQUIRE(n_layers >= 1 && n_layers <= RG_MAX_LAYERS, RG_ERR_ARG,
             "rg_mlp_chain: n_layers=%d outside 1..%d", n_layers, RG_MAX_LAYERS);
  RG_REQUIRE(dtype == RG_F32 || dtype == RG_BF16 || dtype == RG_F16 || dtype == RG_F32X3, RG_ERR_ARG,
             "rg_mlp_chain: bad dtype");
  const bool x3 = dtype == RG_F32X3;
  // the layers' packed format (RG_F16: RG_BF16's fragments holding fp16, RG_PACK_F16)
  const int wfmt = x3 ? (RG_BF16 | RG_PACK_X3) : dtype == RG_F16 ? RG_BF16 : dtype;
  auto dt_ok = [&](int d) { return d == RG_F32 || d == RG_BF16 || d == RG_F16; };
  RG_REQUIRE(dt_ok(in_dtype), RG_ERR_ARG, "rg_mlp_chain: bad in_dtype");
  RG_REQUIRE(dt_ok(out_dtype), RG_ERR_ARG, "rg_mlp_chain: bad out_dtype");
  RG_REQUIRE(!residual || dt_ok(res_dtype), RG_ERR_ARG, "rg_mlp_chain: bad res_dtype");
  RG_REQUIRE(in_mode >= RG_IN_DENSE && in_mode <= RG_IN_PAIRADD, RG_ERR_ARG, "bad in_mode");
  RG_REQUIRE((in_mode != RG_IN_GATHER3 && in_mode != RG_IN_PAIRADD) || (idx0 && idx1), RG_ERR_ARG,
             "rg_mlp_chain: gather modes need idx0 and idx1");
  int expect_in = 0;
  switch (in_mode) {
    case RG_IN_DENSE: expect_in = w0; break;
    case RG_IN_CONCAT2: expect_in = w0 + w1; break;
    case RG_IN_GATHER3: expect_in = 2 * w0 + w2; break;
    default: expect_in = w0; break;
  }
  ChainArgs a;
  memset(&a, 0, sizeof(a));
  size_t woff = 0;
  for (int l = 0; l < n_layers; ++l) {
    const rg_layer& s = layers[l];
    RG_REQUIRE(s.w_packed != nullptr, RG_ERR_ARG, "rg_mlp_chain: layer %d missing weights", l);
    RG_REQUIRE(s.in_dim >= 1 && s.in_dim <= MAXW && s.out_dim >= 1 && s.out_dim <= MAXW,
               RG_ERR_UNSUPPORTED, "rg_mlp_chain: layer %d dims %d->%d outside 1..%d", l,
               s.in_dim, s.out_dim, MAXW);
    RG_REQUIRE(l == 0 ? s.in_dim == expect_in : s.in_dim == layers[l - 1].out_dim, RG_ERR_ARG,
               "rg_mlp_chain: layer %d in_dim %d does not match its input", l, s.in_dim);
    RG_REQUIRE(!s.norm_mu || (s.norm_std && s.out_dim >= 2), RG_ERR_ARG,
               "rg_mlp_chain: layer %d norm needs mu, std and out_dim >= 2", l);
    RG_REQUIRE((!s.save_pre && !s.save_out) || dtype == RG_F32 || x3, RG_ERR_ARG,
               "rg_mlp_chain: training tapes (save_pre / save_out) need dtype RG_F32 / RG_F32X3");
    a.L[l].w = s.w_packed;
    a.L[l].save_pre = s.save_pre;
    a.L[l].save_out = s.save_out;
    a.L[l].mu = s.norm_mu;
    a.L[l].sd = s.norm_std;
    a.L[l].in = s.in_dim;
    a.L[l].out = s.out_dim;
    a.L[l].act = s.act;
    a.L[l].woff = (int)woff;
    woff += packed_bytes(s.in_dim, s.out_dim, wfmt);
  }
  a.wbytes = (int)woff;
  a.nl = n_layers;
  a.in_mode = in_mode;
  a.in_dtype = in_dtype;
  a.w0 = w0; a.w1 = w1; a.w2 = w2;
  a.ld0 = ld0; a.ld1 = ld1; a.ld2 = ld2;
  a.ld_res = ld_res; a.res_dtype = res_dtype; a.ld_out = ld_out; a.out_dtype = out_dtype;
  a.rows = rows; a.rows_dev = rows_dev;
  a.in0 = in0; a.in1 = in1; a.in2 = in2; a.idx0 = idx0; a.idx1 = idx1;
  a.res = residual; a.out = out;
  if (rows <= 0) return RG_OK;
  hipStream_t st = (hipStream_t)stream;
  const size_t dbytes = (sizeof(ChainLayer) * RG_MAX_LAYERS + 15) & ~(size_t)15;
  if (dtype == RG_F32 || x3) {
    // f32 slab rows sized to the chain's widest input (kpad 64 + 8 keeps the B reads
    // conflict-free): single large layers (the training backward's W^T) then fit in LDS
    int kmax = layers[0].in_dim;
    for (int l = 0; l + 1 < n_layers; ++l) kmax = layers[l].out_dim > kmax ? layers[l].out_dim : kmax;
    a.sstride = kpad(kmax, 64) + 8;
    const size_t slabs = (size_t)CH_WAVES * TR * a.sstride * sizeof(float);
    // (reading the weights from L2 instead of staging them, for more resident workgroups per
    // CU, measured slower on the training tape: 9.8 -> 11.1-12.0 ms)
    const bool fits = dbytes + woff + slabs <= LDS_LIMIT;
    if (x3) return fits ? launch_chain<float, true, true>(a, rows, st)
                        : launch_chain<float, false, true>(a, rows, st);
    if (fits) return launch_chain<float, true>(a, rows, st);
    return launch_chain<float, false>(a, rows, st);
  }
  a.sstride = Cfg<uint16_t>::STRIDE;
  const size_t slabs = (size_t)CH_WAVES * TR * Cfg<uint16_t>::STRIDE * sizeof(uint16_t);
  const bool fits = dbytes + woff + slabs <= LDS_LIMIT;
  if (dtype == RG_F16)
    return fits ? launch_chain<_Float16, true>(a, rows, st) : launch_chain<_Float16, false>(a, rows, st);
  if (fits) return launch_chain<uint16_t, true>(a, rows, st);
  return launch_chain<uint16_t, false>(a, rows, st);
}
