// Training backward of the radar-GNN hot path, float32 (the reference trains in f32):
// Model_Training.forward + Loss_Graph + loss.backward() + torch.optim.SGD
// (gnn_detector.py:428-478, loss.py:37-76, lossfunc.py:20-55, training.py:66-85,
// set_param_for_training_gnn.py:44-46).
//
//   rg_ffn_backward         channel_normalization + activation backward, row per wave,
//                           statistics recomputed from the saved pre-norm rows
//   rg_linear_grad          dW += dZ^T X, db += sum dZ with X formed on the fly from the
//                           chain input modes (gathered / concatenated / pair-added rows):
//                           v_mfma_f32_16x16x4_f32 over 64-row LDS tiles, fixed row
//                           chunks, chunk partials reduced in a fixed order
//   rg_incidence            node -> items lists (transpose of an index_select)
//   rg_gather_segment_sum   per-node ordered sums of gradient rows
//   rg_segment_max_backward per-cluster channel max backward (first maximum)
//   rg_loss_graph(+_backward) the four losses, accuracies and logit gradients
//   rg_sgd_step             the SGD update on flat arrays
// The data GEMM of the backward (dX = dZ W) is rg_mlp_chain on W packed transposed
// (RG_PACK_TRANSPOSE).  Every reduction runs in a fixed order (no float atomics except
// rg_segment_max_backward, where clusters may share a node), so a step is
// bit-reproducible.
#include "rg_common.h"
#include "scan.h"

namespace rg {
namespace train {

static constexpr int PARTS = 512;          // fixed grid of the partial-sum kernels
static constexpr int FFN_PARTS_MAX = 4096;  // ffn_backward grid bound (workspace size)
static constexpr float NORM_EPS = 1e-5f;   // constants.py:9

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// d act(y) / d y as torch's backward kernels: leaky_relu (self > 0 ? 1 : slope),
// relu (result > 0), silu (s (1 + y (1 - s)))
__device__ __forceinline__ float act_grad(float y, int act) {
  if (act == ACT_LEAKY) return y > 0.f ? 1.f : 0.01f;
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == ACT_SWISH) {
    const float s = 1.f / (1.f + expf(-y));
    return s * (1.f + y * (1.f - s));
  }
  return 1.f;
}

// ------------------------------------------------------------------ ffn backward
// 16 lanes per row (4 rows per wave), feature f = q + 16 j (q = lane & 15): row sums are
// 4 xor-shuffles inside the 16-lane group.  Forward (common.py:215-220, as the chain
// kernel evaluates it): mean = sum z / C, d = z - mean, std = sqrt(sum d^2 / (C-1)),
// r = 1 / (std + eps), n = d r, y = s n + m, a = act(y).  Backward:
//   gy = da act'(y);  ds += sum gy n;  dm += sum gy;  gn = s gy;
//   gd = r gn - r^2 (sum gn d) d / ((C-1) std);  dz = gd - mean(gd).
__device__ __forceinline__ float group16_sum(float v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

template <int J>  // features per lane = J (C <= 16 J)
__global__ __launch_bounds__(256) void ffn_backward_kernel(
    const float* __restrict__ z, int ldz, const float* __restrict__ da, int ldda, long rows,
    int C, int has_norm, const float* __restrict__ mu, const float* __restrict__ sd, int act,
    float* __restrict__ dz, int lddz, double* __restrict__ part, const int* __restrict__ gidx,
    const float* __restrict__ gscale) {
  __shared__ double red[16][2];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, q = lane & 15;
  const float s = has_norm ? *sd : 1.f;
  const float m = has_norm ? *mu : 0.f;
  // per 16-lane group, rows in fixed order; in float64: d_mu / d_std are sums over every
  // element of the layer with heavy cancellation (each row's 16-lane sum stays float32)
  double acc_s = 0.0, acc_m = 0.0;
  for (long row = ((long)blockIdx.x * 4 + wave) * 4 + grp; row < rows;
       row += (long)gridDim.x * 16) {
    float zv[J], gv[J];
    // gathered input (rg_ffn_backward_gather): da row gidx[row], times gscale[gidx[row]]
    // (the reference's mean aggregation), rounded as rg_gather_segment_sum forms it
    const long arow = gidx ? (long)gidx[row] : row;
    const float gsc = gscale ? gscale[arow] : 1.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int f = q + 16 * j;
      zv[j] = f < C ? z[(size_t)row * ldz + f] : 0.f;
      const float g = f < C ? da[(size_t)arow * ldda + f] : 0.f;
      gv[j] = gscale ? __fmaf_rn(g, gsc, 0.f) : g;
    }
    if (has_norm) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) t += zv[j];
      const float mean = group16_sum(t) / (float)C;
      float d[J], ss = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        d[j] = (q + 16 * j) < C ? zv[j] - mean : 0.f;
        ss += d[j] * d[j];
      }
      ss = group16_sum(ss);
      const float stdv = __fsqrt_rn(ss / (float)(C - 1));
      const float r = 1.f / (stdv + NORM_EPS);
      float gn[J], ps = 0.f, pm = 0.f, A = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const float n = d[j] * r;
        const float y = __fadd_rn(__fmul_rn(s, n), m);
        const float gy = (q + 16 * j) < C ? gv[j] * act_grad(y, act) : 0.f;
        ps += gy * n;
        pm += gy;
        gn[j] = s * gy;
        A += gn[j] * d[j];
      }
      ps = group16_sum(ps);
      pm = group16_sum(pm);
      A = group16_sum(A);
      acc_s += (double)ps;
      acc_m += (double)pm;
      const float coef = stdv > 0.f ? r * r * A / ((float)(C - 1) * stdv) : 0.f;
      float gd[J], sg = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        gd[j] = (q + 16 * j) < C ? r * gn[j] - coef * d[j] : 0.f;
        sg += gd[j];
      }
      const float mg = group16_sum(sg) / (float)C;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int f = q + 16 * j;
        if (f < C) dz[(size_t)row * lddz + f] = gd[j] - mg;
      }
    } else {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int f = q + 16 * j;
        if (f < C) dz[(size_t)row * lddz + f] = gv[j] * act_grad(zv[j], act);
      }
    }
  }
  if (q == 0) {
    red[wave * 4 + grp][0] = acc_s;
    red[wave * 4 + grp][1] = acc_m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tm = 0.0;
    for (int i = 0; i < 16; ++i) {
      ts += red[i][0];
      tm += red[i][1];
    }
    part[2 * blockIdx.x] = ts;
    part[2 * blockIdx.x + 1] = tm;
  }
}

// sum of PARTS (s, m) partials in a fixed order, added to the parameter gradients
__global__ __launch_bounds__(256) void ffn_param_reduce(const double* __restrict__ part, int parts,
                                                        float* __restrict__ d_mu,
                                                        float* __restrict__ d_sd) {
  __shared__ double red[256][2];
  const int t = threadIdx.x;
  double s = 0.0, m = 0.0;
  for (int i = t; i < parts; i += 256) {
    s += part[2 * i];
    m += part[2 * i + 1];
  }
  red[t][0] = s;
  red[t][1] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {  // fixed tree order
    if (t < w) {
      red[t][0] += red[t + w][0];
      red[t][1] += red[t + w][1];
    }
    __syncthreads();
  }
  if (t == 0) {
    *d_sd = (float)((double)*d_sd + red[0][0]);
    *d_mu = (float)((double)*d_mu + red[0][1]);
  }
}

// ------------------------------------------------------------------ linear weight grad
struct GradIn {
  int mode, in_dim;
  const float* in0;
  const float* in1;
  const float* in2;
  int ld0, ld1, ld2, w0, w1, w2;
  const int* idx0;
  const int* idx1;
};

// element f of row `row` of the layer input; f == in_dim is the bias column (1)
__device__ __forceinline__ float x_elem(const GradIn& a, long row, int f) {
  if (f >= a.in_dim) return f == a.in_dim ? 1.f : 0.f;
  switch (a.mode) {
    case RG_IN_DENSE:
      return a.in0[(size_t)row * a.ld0 + f];
    case RG_IN_CONCAT2:
      return f < a.w0 ? a.in0[(size_t)row * a.ld0 + f] : a.in1[(size_t)row * a.ld1 + (f - a.w0)];
    case RG_IN_GATHER3:
      if (f < a.w0) return a.in0[(size_t)a.idx0[row] * a.ld0 + f];
      if (f < 2 * a.w0) return a.in0[(size_t)a.idx1[row] * a.ld0 + (f - a.w0)];
      return a.in2[(size_t)row * a.ld2 + (f - 2 * a.w0)];
    default:  // RG_IN_PAIRADD
      return __fadd_rn(a.in0[(size_t)a.idx0[row] * a.ld0 + f], a.in0[(size_t)a.idx1[row] * a.ld0 + f]);
  }
}

// 4 consecutive input features [f, f+4) of row `row` (vec: every segment width and row
// stride is a multiple of 4, so the group never straddles two segments)
__device__ __forceinline__ f32x4 x_chunk(const GradIn& a, long row, int f, bool vec) {
  if (vec && f + 4 <= a.in_dim) {
    switch (a.mode) {
      case RG_IN_DENSE:
        return *(const f32x4*)(a.in0 + (size_t)row * a.ld0 + f);
      case RG_IN_CONCAT2:
        return f < a.w0 ? *(const f32x4*)(a.in0 + (size_t)row * a.ld0 + f)
                        : *(const f32x4*)(a.in1 + (size_t)row * a.ld1 + (f - a.w0));
      case RG_IN_GATHER3:
        if (f < a.w0) return *(const f32x4*)(a.in0 + (size_t)a.idx0[row] * a.ld0 + f);
        if (f < 2 * a.w0) return *(const f32x4*)(a.in0 + (size_t)a.idx1[row] * a.ld0 + (f - a.w0));
        return *(const f32x4*)(a.in2 + (size_t)row * a.ld2 + (f - 2 * a.w0));
      default: {
        const f32x4 u = *(const f32x4*)(a.in0 + (size_t)a.idx0[row] * a.ld0 + f);
        const f32x4 v = *(const f32x4*)(a.in0 + (size_t)a.idx1[row] * a.ld0 + f);
        return (f32x4){__fadd_rn(u.x, v.x), __fadd_rn(u.y, v.y), __fadd_rn(u.z, v.z),
                       __fadd_rn(u.w, v.w)};
      }
    }
  }
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = f + e < a.in_dim ? x_elem(a, row, f + e) : 0.f;
  return v;
}

// Weight gradient tile: out rows [o0, o0 + 64 OW) x in columns [i0, i0 + 16 NT) over one
// chunk of rows.  Wave w owns out rows 16 OW w .. +16 OW and every column, so the whole
// tile stays in registers (OW * NT f32x4 accumulators) and dz / x rows are read once
// per chunk.  Rows are staged 32 at a time in LDS; one k-step = 4 rows = OW * NT
// v_mfma_f32_16x16x4_f32 (A = dz^T: lane -> (out 16m + (lane&15), row lane>>4);
// B = x: lane -> (row lane>>4, in 16n + (lane&15))).  The bias column sum is a VALU
// side sum of the staged dz rows.
static constexpr int GR = 32;  // rows per staged block
__host__ __device__ constexpr int grad_stride(int cols) { return (cols + 63) / 64 * 64 + 16; }

template <int OW, int NT>
__global__ __launch_bounds__(256) void linear_grad_kernel(const float* __restrict__ dz, int lddz,
                                                          long rows, int out_dim, GradIn in,
                                                          long rpc, int vec_x, int vec_z,
                                                          float* __restrict__ part,
                                                          float* __restrict__ part_b) {
  constexpr int OC = 64 * OW, IC = 16 * NT;
  constexpr int SZ = grad_stride(OC), SX = grad_stride(IC);
  __shared__ __attribute__((aligned(16))) float sZ[GR * SZ];
  __shared__ __attribute__((aligned(16))) float sX[GR * SX];
  const int chunk = blockIdx.x, ot = blockIdx.y, it = blockIdx.z;
  const int o0 = ot * OC, i0 = it * IC;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r_begin = (long)chunk * rpc;
  const long r_end = min(rows, r_begin + rpc);
  f32x4 acc[OW][NT];
#pragma unroll
  for (int m = 0; m < OW; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  // staging: every dz / x load of a block (x gathered for the GATHER3 / PAIRADD modes) is
  // issued before the first LDS store, so a thread's ~10 row pieces are in flight together
  // (a store-per-load loop waited one gather round trip per piece).  Carrying the next
  // block's pieces through the MFMAs instead (a register double buffer) took the 192-wide
  // gathered tiles to 256 VGPRs + 192 AGPRs, one wave per SIMD: not kept
  // x pieces: a thread keeps ONE column group for every row it stages (xc fixed, rows xr0,
  // xr0 + XR, ...), so the segment test of the gathered input modes is decided once per
  // thread, not per piece (IC = 192: 48 groups, 5 rows per pass, 240 threads busy)
  constexpr int ZI = GR * (OC / 4);   // dz f32x4 items per staged block
  constexpr int ZT = (ZI + 255) / 256;
  constexpr int XG = IC / 4;                    // x column groups
  constexpr int XR = 256 / XG < GR ? 256 / XG : GR;  // rows per pass
  constexpr int XT = (GR + XR - 1) / XR;        // passes
  const bool xon = (int)threadIdx.x < XR * XG;
  const int xc = 4 * ((int)threadIdx.x % XG), xr0 = (int)threadIdx.x / XG;
  f32x4 zr[ZT], xr[XT];
  auto fetch = [&](long rb) {
#pragma unroll
    for (int j = 0; j < ZT; ++j) {
      const int t = threadIdx.x + 256 * j;
      const int rr = t / (OC / 4), c = 4 * (t % (OC / 4));
      const long row = rb + rr;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (t < ZI && row < r_end) {
        const float* pz = dz + (size_t)row * lddz + o0 + c;
        if (vec_z && o0 + c + 4 <= out_dim) {
          v = *(const f32x4*)pz;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = o0 + c + e < out_dim ? pz[e] : 0.f;
        }
      }
      zr[j] = v;
    }
#pragma unroll
    for (int j = 0; j < XT; ++j) {
      const int rr = xr0 + XR * j;
      const long row = rb + rr;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (xon && rr < GR && row < r_end && i0 + xc < in.in_dim) v = x_chunk(in, row, i0 + xc, vec_x);
      xr[j] = v;
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < ZT; ++j) {
      const int t = threadIdx.x + 256 * j;
      if (t < ZI) *(f32x4*)(sZ + (t / (OC / 4)) * SZ + 4 * (t % (OC / 4))) = zr[j];
    }
#pragma unroll
    for (int j = 0; j < XT; ++j) {
      const int rr = xr0 + XR * j;
      if (xon && rr < GR) *(f32x4*)(sX + rr * SX + xc) = xr[j];
    }
  };
  for (long rb = r_begin; rb < r_end; rb += GR) {
    fetch(rb);
    put();
    __syncthreads();
    // operands one k-step ahead, as linear_grad_dma_kernel's compute
    float av[2][OW], bv[2][NT];
    auto ld = [&](int ks, int u) {
      const int kr = 4 * ks + (lane >> 4);
#pragma unroll
      for (int m = 0; m < OW; ++m) av[u][m] = sZ[kr * SZ + 16 * (OW * wave + m) + (lane & 15)];
#pragma unroll
      for (int n = 0; n < NT; ++n) bv[u][n] = sX[kr * SX + 16 * n + (lane & 15)];
    };
    ld(0, 0);
#pragma unroll
    for (int ks = 0; ks < GR / 4; ++ks) {
      const int u = ks & 1;
      if (ks + 1 < GR / 4) ld(ks + 1, u ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < OW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][m], bv[u][n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (it == 0 && threadIdx.x < OC) {
#pragma unroll 8
      for (int rr = 0; rr < GR; ++rr) bsum += sZ[rr * SZ + threadIdx.x];
    }
    __syncthreads();
  }
  // lane holds D[o = 16(OW wave + m) + 4(lane>>4) + e][i = 16n + (lane&15)]
  float* P = part + ((size_t)(chunk * gridDim.y + ot) * gridDim.z + it) * OC * IC;
#pragma unroll
  for (int m = 0; m < OW; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        P[(16 * (OW * wave + m) + 4 * (lane >> 4) + e) * IC + 16 * n + (lane & 15)] = acc[m][n][e];
  if (it == 0 && threadIdx.x < OC) part_b[((size_t)chunk * gridDim.y + ot) * OC + threadIdx.x] = bsum;
}

#ifndef RG_GRAD_DMA
#define RG_GRAD_DMA 1  // full row blocks staged by LDS DMA, double-buffered (below); 0 = the register-staged kernel only
#endif
#if RG_GRAD_DMA
// the 16-B source of input features [f, f + 4) of row `row` (x_chunk's vector path); j0 / j1:
// the row's gathered node indices (RG_IN_GATHER3)
__device__ __forceinline__ const float* x_src(const GradIn& a, long row, int f, int j0, int j1) {
  if (a.mode == RG_IN_GATHER3)
    return f < a.w0 ? a.in0 + (size_t)j0 * a.ld0 + f
         : f < 2 * a.w0 ? a.in0 + (size_t)j1 * a.ld0 + (f - a.w0)
                        : a.in2 + (size_t)row * a.ld2 + (f - 2 * a.w0);
  if (a.mode == RG_IN_CONCAT2 && f >= a.w0) return a.in1 + (size_t)row * a.ld1 + (f - a.w0);
  return a.in0 + (size_t)row * a.ld0 + f;
}
typedef __attribute__((address_space(3))) void* lds_ptr_t;
// The same tile as linear_grad_kernel (same k-step order: bit-identical partials) for a tile
// whose columns are all real features (no bias / padding column), 16-B aligned rows and a
// non-PAIRADD input: the full 32-row blocks go through the LDS by DMA (global_load_lds, one
// instruction per row and operand, no register round trip) into two buffers -- block b + 1
// lands while block b's MFMAs run; the barrier closing block b waits for it.  A partial last
// block is staged as in linear_grad_kernel.  One workgroup per CU (two 53-KB buffers).
template <int OW, int NT, bool G3>
__global__ __launch_bounds__(256) void linear_grad_dma_kernel(const float* __restrict__ dz,
                                                              int lddz, long rows, GradIn in,
                                                              long rpc, float* __restrict__ part,
                                                              float* __restrict__ part_b) {
  constexpr int OC = 64 * OW, IC = 16 * NT;
  constexpr int SZ = grad_stride(OC), SX = grad_stride(IC);
  constexpr int BUF = GR * SZ + GR * SX;
  static_assert(OC / 4 <= 64 && IC / 4 <= 64, "one DMA instruction per row");
  extern __shared__ __attribute__((aligned(16))) float glds[];
  const int chunk = blockIdx.x, ot = blockIdx.y, it = blockIdx.z;
  const int o0 = ot * OC, i0 = it * IC;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r_begin = (long)chunk * rpc;
  const long r_end = min(rows, r_begin + rpc);
  f32x4 acc[OW][NT];
#pragma unroll
  for (int m = 0; m < OW; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  // rows wave, wave + 4, ... of the block: their dz and x rows by DMA into buffer b.  A
  // gathered input's row indices come first, in one load (lanes 0-15) and one wait, then
  // broadcast: a per-row index load would wait, in order, for every DMA issued before it
  // (G3 is a template flag, not the runtime mode: with the index load on any path, the
  // compiler waits for every load in flight -- this block's DMA included -- at its first
  // readlane, and each block's issue then cost a full memory round trip before the MFMAs of
  // the block before it)
  const int f = i0 + 4 * lane;
  auto issue = [&](long rb, int b) {
    float* sZ = glds + b * BUF;
    float* sX = sZ + GR * SZ;
    int iv = 0;
    if constexpr (G3) {
      if (lane < 2 * (GR / 4)) {
        const long row = rb + wave + 4 * (lane % (GR / 4));
        iv = lane < GR / 4 ? in.idx0[row] : in.idx1[row];
      }
    }
#pragma unroll
    for (int j = 0; j < GR / 4; ++j) {
      const int rr = wave + 4 * j;
      const long row = rb + rr;
      if (lane < OC / 4)
        __builtin_amdgcn_global_load_lds((const void*)(dz + (size_t)row * lddz + o0 + 4 * lane),
                                         (lds_ptr_t)(sZ + rr * SZ), 16, 0, 0);
      const float* src = G3 ? x_src(in, row, f, __builtin_amdgcn_readlane(iv, j),
                                    __builtin_amdgcn_readlane(iv, GR / 4 + j))
                            : x_src(in, row, f, 0, 0);
      if (lane < IC / 4)
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(sX + rr * SX), 16, 0, 0);
    }
  };
  auto compute = [&](int b) {
    const float* sZ = glds + b * BUF;
    const float* sX = sZ + GR * SZ;
    // operands read one k-step ahead (fenced): left to itself the compiler re-used two
    // registers for the B operands and waited for each LDS read before its two MFMAs
    float av[2][OW], bv[2][NT];
    auto ld = [&](int ks, int u) {
      const int kr = 4 * ks + (lane >> 4);
#pragma unroll
      for (int m = 0; m < OW; ++m) av[u][m] = sZ[kr * SZ + 16 * (OW * wave + m) + (lane & 15)];
#pragma unroll
      for (int n = 0; n < NT; ++n) bv[u][n] = sX[kr * SX + 16 * n + (lane & 15)];
    };
    ld(0, 0);
#pragma unroll
    for (int ks = 0; ks < GR / 4; ++ks) {
      const int u = ks & 1;
      if (ks + 1 < GR / 4) ld(ks + 1, u ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < OW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][m], bv[u][n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (it == 0 && threadIdx.x < OC) {
#pragma unroll 8
      for (int rr = 0; rr < GR; ++rr) bsum += sZ[rr * SZ + threadIdx.x];
    }
  };
  const long nfull = (r_end - r_begin) / GR;
  if (nfull > 0) issue(r_begin, 0);
  __syncthreads();
  for (long b = 0; b < nfull; ++b) {
    if (b + 1 < nfull) issue(r_begin + (b + 1) * GR, (int)((b + 1) & 1));
    compute((int)(b & 1));
    __syncthreads();  // (waits for every wave's DMA of block b + 1; buffer b free again)
  }
  const long rb = r_begin + nfull * GR;
  if (rb < r_end) {  // the partial last block, staged through registers with zero rows
    float* sZ = glds;
    float* sX = glds + GR * SZ;
    for (int t = threadIdx.x; t < GR * (OC / 4); t += 256) {
      const int rr = t / (OC / 4), c = 4 * (t % (OC / 4));
      const long row = rb + rr;
      *(f32x4*)(sZ + rr * SZ + c) = row < r_end ? *(const f32x4*)(dz + (size_t)row * lddz + o0 + c)
                                                : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    for (int t = threadIdx.x; t < GR * (IC / 4); t += 256) {
      const int rr = t / (IC / 4), c = 4 * (t % (IC / 4));
      const long row = rb + rr;
      *(f32x4*)(sX + rr * SX + c) = row < r_end ? x_chunk(in, row, i0 + c, true)
                                                : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    compute(0);
  }
  float* P = part + ((size_t)(chunk * gridDim.y + ot) * gridDim.z + it) * OC * IC;
#pragma unroll
  for (int m = 0; m < OW; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        P[(16 * (OW * wave + m) + 4 * (lane >> 4) + e) * IC + 16 * n + (lane & 15)] = acc[m][n][e];
  if (it == 0 && threadIdx.x < OC) part_b[((size_t)chunk * gridDim.y + ot) * OC + threadIdx.x] = bsum;
}
#endif

struct GradGeom {
  int ow, nt, ot, it, nchunk;
  long rpc;  // rows per chunk (multiple of GR)
};
static GradGeom grad_geom(long rows, int out_dim, int in_dim) {
  GradGeom g;
  g.ow = out_dim > 64 ? 2 : 1;
  const int nt_need = (in_dim + 15) / 16;
  g.nt = nt_need <= 1 ? 1 : nt_need <= 4 ? 4 : nt_need <= 8 ? 8 : nt_need <= 12 ? 12 : 16;
  g.ot = (out_dim + 64 * g.ow - 1) / (64 * g.ow);
  g.it = (in_dim + 16 * g.nt - 1) / (16 * g.nt);
  const long blocks = (rows + GR - 1) / GR;
  // two workgroups per CU (one's row staging overlaps another's MFMAs: the kernel stages
  // single-buffered) and chunks of >= 4 staged blocks of GR rows (the partials' reduction
  // keeps eight loads in flight) -- c4 backward 20.4 -> 15.5 ms against one workgroup per
  // CU and >= 32 blocks (scripts/experiments/gpu_c4_grad.sh: 3 per CU 293, 4 per CU 278
  // frames/s against 2 per CU 309)
#ifndef RG_GRAD_WG_CU
#define RG_GRAD_WG_CU 2
#endif
#ifndef RG_GRAD_MIN_BLK
#define RG_GRAD_MIN_BLK 4
#endif
  constexpr int wg_cu = RG_GRAD_WG_CU, min_blk = RG_GRAD_MIN_BLK;
  long want = 256L * (wg_cu > 0 ? wg_cu : 1) / (g.ot * g.it);
  if (want < 1) want = 1;
  const long mb = min_blk > 0 ? min_blk : 1;
  if (want > (blocks + mb - 1) / mb) want = (blocks + mb - 1) / mb;
  if (want < 1) want = 1;
  g.rpc = ((blocks + want - 1) / want) * GR;
  g.nchunk = (int)((rows + g.rpc - 1) / g.rpc);
  if (g.nchunk < 1) g.nchunk = 1;
  return g;
}
static size_t grad_part_floats(const GradGeom& g) {
  return (size_t)g.nchunk * g.ot * g.it * (64 * g.ow) * (16 * g.nt);
}
static size_t grad_ws_bytes(const GradGeom& g) {
  return (grad_part_floats(g) + (size_t)g.nchunk * g.ot * 64 * g.ow) * sizeof(float);
}

// dW / db += the chunk partials in a fixed order: 64 consecutive (o, i) entries per
// workgroup, wave w of RW sums chunks w, w + RW, ... (eight loads in flight) and the RW wave
// sums combine in a fixed pairwise tree.  (Four waves per workgroup left ~70 workgroups on
// the chip for a 64 x 64 layer's 512 chunks: 16 dependent rounds per thread, 15 us.)
static constexpr int RW = 16;
__global__ __launch_bounds__(64 * RW) void linear_grad_reduce(
    const float* __restrict__ part, const float* __restrict__ part_b, int nchunk, int ot_n,
    int it_n, int oc, int ic, int out_dim, int in_dim, float* __restrict__ dW,
    float* __restrict__ db, int ld_dw) {
  __shared__ float red[RW][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long t = (long)blockIdx.x * 64 + lane;
  const long total = (long)out_dim * (in_dim + 1);
  float s = 0.f;
  int o = 0, i = 0;
  if (t < total) {
    o = (int)(t / (in_dim + 1));
    i = (int)(t % (in_dim + 1));
    const int ot = o / oc, oo = o % oc;
    // U chunks' loads in flight per wave, then summed in chunk order (c = wave, wave + RW,
    // ...): a 512-chunk reduction is two load rounds per wave instead of four
    constexpr int U = 16;
    const bool w_ = i < in_dim;
    const int it = i / ic, ii = i % ic;
    const size_t base = w_ ? ((size_t)ot * it_n + it) * oc * ic + (size_t)oo * ic + ii
                           : (size_t)ot * oc + oo;
    const size_t cstride = w_ ? (size_t)ot_n * it_n * oc * ic : (size_t)ot_n * oc;
    const float* src = w_ ? part : part_b;
    for (int c0 = wave; c0 < nchunk; c0 += RW * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + RW * u;
        v[u] = c < nchunk ? src[base + (size_t)c * cstride] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (c0 + RW * u < nchunk) s += v[u];
    }
  }
  red[wave][lane] = s;
  __syncthreads();
#pragma unroll
  for (int h = RW / 2; h > 0; h >>= 1) {
    if (wave < h) red[wave][lane] += red[wave + h][lane];
    __syncthreads();
  }
  if (wave == 0 && t < total) {
    const float v = red[0][lane];
    if (i < in_dim) dW[(size_t)o * ld_dw + i] += v;
    else if (db) db[o] += v;
  }
}

template <int OW, int NT>
static int launch_grad(const GradGeom& g, const float* dz, int lddz, long rows, int out_dim,
                       const GradIn& in, int vec_x, int vec_z, float* part, float* part_b,
                       hipStream_t st) {
#if RG_GRAD_DMA
  if (vec_x && vec_z && in.mode != RG_IN_PAIRADD && out_dim % (64 * OW) == 0 &&
      in.in_dim % (16 * NT) == 0 && g.rpc % GR == 0) {
    constexpr int lds = 2 * (GR * grad_stride(64 * OW) + GR * grad_stride(16 * NT)) * 4;
    auto kern = in.mode == RG_IN_GATHER3 ? linear_grad_dma_kernel<OW, NT, true>
                                         : linear_grad_dma_kernel<OW, NT, false>;
    RG_ENSURE_LDS(kern, lds);
    kern<<<dim3(g.nchunk, g.ot, g.it), 256, lds, st>>>(dz, lddz, rows, in, g.rpc, part, part_b);
    return RG_OK;
  }
#endif
  // (a split-bf16 x3 variant of this kernel measured slower on c4, 614 -> 574 frames/s: its
  // staging -- a three-term split per 8 values, transposed LDS stores -- outweighed the 2.7x
  // matrix rate at 32-row blocks, and was removed; the exact f32 MFMA kernel is the one)
  linear_grad_kernel<OW, NT><<<dim3(g.nchunk, g.ot, g.it), 256, 0, st>>>(
      dz, lddz, rows, out_dim, in, g.rpc, vec_x, vec_z, part, part_b);
  return RG_OK;
}

// ------------------------------------------------------------------ incidence lists
__global__ void inc_count(const int* __restrict__ a, const int* __restrict__ b, long n,
                          int* __restrict__ cnt) {
  const long u = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  atomicAdd(cnt + a[u], 1);
  if (b) atomicAdd(cnt + b[u], 1);
}
__global__ void inc_fill(const int* __restrict__ a, const int* __restrict__ b, long n,
                         int* __restrict__ cursor, int* __restrict__ list) {
  const long u = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  list[atomicAdd(cursor + a[u], 1)] = (int)u;
  if (b) list[atomicAdd(cursor + b[u], 1)] = (int)u;
}
// each list ascending (fill order is arbitrary); lists are short (node degrees)
__global__ void inc_sort(const int* __restrict__ ptr, int n_nodes, int* __restrict__ list) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_nodes) return;
  const int b = ptr[v], e = ptr[v + 1];
  for (int i = b + 1; i < e; ++i) {
    const int key = list[i];
    int j = i - 1;
    while (j >= b && list[j] > key) {
      list[j + 1] = list[j];
      --j;
    }
    list[j + 1] = key;
  }
}

// ------------------------------------------------------------------ gather-segment sum
__global__ __launch_bounds__(256) void gather_segsum_kernel(
    const float* __restrict__ src, int ld_src, int col0, int width, const int* __restrict__ ptr,
    const int* __restrict__ list, const float* __restrict__ scale, int n_nodes,
    float* __restrict__ out, int ld_out, int accumulate) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int v = blockIdx.x * 4 + wave; v < n_nodes; v += gridDim.x * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int b = ptr[v], e = ptr[v + 1];
    for (int k = b; k < e; ++k) {
      const int row = list ? list[k] : k;
      const float sc = scale ? scale[row] : 1.f;
      const float* p = src + (size_t)row * ld_src + col0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int f = lane + 64 * j;
        if (f < width) acc[j] = scale ? __fmaf_rn(p[f], sc, acc[j]) : __fadd_rn(acc[j], p[f]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = lane + 64 * j;
      if (f < width) {
        float* o = out + (size_t)v * ld_out + f;
        *o = accumulate ? *o + acc[j] : acc[j];
      }
    }
  }
}

// The same sums as a row stream per lane group (the streaming scatter-aggregate of
// segment_reduce.hip): 16 lanes per node, one 16-B piece of 4 columns per lane and row, U
// rows in flight per lane (their list indices first, then the rows), each node's rows
// summed in list order -- the order of gather_segsum_kernel, whose wave per node walked its
// rows one dependent load at a time (44 us per call on c4's 300 k edges).  Columns in
// passes of 64; needs 16-B aligned rows (ld_src, col0, width, ld_out multiples of 4).
template <bool SCALED, int U = 8>
__global__ __launch_bounds__(256) void gather_segsum_stream(
    const float* __restrict__ src, int ld_src, int col0, int width, const int* __restrict__ ptr,
    const int* __restrict__ list, const float* __restrict__ scale, int n_nodes,
    float* __restrict__ out, int ld_out, int accumulate) {
  const int sl = threadIdx.x & 15;
  const int v = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (v >= n_nodes) return;  // group-uniform
  const int b = ptr[v], e = ptr[v + 1];
  for (int c0 = 0; c0 < width; c0 += 64) {
    const int c = c0 + 4 * sl;
    const bool on = c < width;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int p = b; p < e; p += U) {
      int row[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = p + u < e ? p + u : e - 1;
        row[u] = list ? list[q] : q;
      }
      f32x4 x[U];
      float sc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u] = on ? *(const f32x4*)(src + (size_t)row[u] * ld_src + col0 + c)
                  : (f32x4){0.f, 0.f, 0.f, 0.f};
        sc[u] = SCALED ? scale[row[u]] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p + u < e) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i] = SCALED ? __fmaf_rn(x[u][i], sc[u], acc[i]) : __fadd_rn(acc[i], x[u][i]);
        }
      }
    }
    if (on) {
      f32x4* o = (f32x4*)(out + (size_t)v * ld_out + c);
      if (accumulate) {
        const f32x4 old = *o;
        acc = (f32x4){__fadd_rn(old[0], acc[0]), __fadd_rn(old[1], acc[1]),
                      __fadd_rn(old[2], acc[2]), __fadd_rn(old[3], acc[3])};
      }
      *o = acc;
    }
  }
}

// ------------------------------------------------------------------ segment max backward
__global__ void segmax_backward_kernel(const float* __restrict__ h, int ld_h, int C,
                                       const int* __restrict__ cptr, const int* __restrict__ cidx,
                                       int n_clusters, const float* __restrict__ dp, int ld_p,
                                       float* __restrict__ dh, int ld_dh) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)n_clusters * C) return;
  const int c = (int)(t / C), f = (int)(t % C);
  const int b = cptr[c], e = cptr[c + 1];
  if (b >= e) return;
  int best = cidx[b];
  float bv = h[(size_t)best * ld_h + f];
  for (int k = b + 1; k < e; ++k) {
    const int n = cidx[k];
    const float v = h[(size_t)n * ld_h + f];
    if (v > bv || (v != v && bv == bv)) {  // NaN propagates as the maximum (torch.max)
      bv = v;
      best = n;
    }
  }
  atomicAdd(dh + (size_t)best * ld_dh + f, dp[(size_t)c * ld_p + f]);
}

// ------------------------------------------------------------------ losses
// log-sum-exp and argmax (first maximum) of a logit row
__device__ __forceinline__ void row_stats(const float* x, int nc, float& lse, int& amax) {
  float mx = x[0];
  amax = 0;
  for (int c = 1; c < nc; ++c)
    if (x[c] > mx) {
      mx = x[c];
      amax = c;
    }
  float s = 0.f;
  for (int c = 0; c < nc; ++c) s += expf(x[c] - mx);
  lse = mx + logf(s);
}

// sigmoid_focal_loss (torchvision; alpha 0.25, gamma 2) of one logit and its 0/1 target,
// and its derivative
__device__ __forceinline__ float focal(float x, float t) {
  const float p = 1.f / (1.f + expf(-x));
  const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float at = 0.25f * t + 0.75f * (1.f - t);
  return at * ce * (1.f - pt) * (1.f - pt);
}
__device__ __forceinline__ float focal_grad(float x, float t) {
  const float p = 1.f / (1.f + expf(-x));
  const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float at = 0.25f * t + 0.75f * (1.f - t);
  const float q = 1.f - pt;
  return at * ((p - t) * q * q - 2.f * ce * q * (2.f * t - 1.f) * p * (1.f - p));
}

__device__ __forceinline__ long term_rows(const rg_loss_args& a, int term) {
  return term == 0 || term == 1 ? a.n_nodes : (term == 2 ? a.n_pairs : a.n_clusters);
}

// per (term, block): sum of the row losses (f64) and of the correct argmaxes
__global__ __launch_bounds__(256) void loss_rows_kernel(rg_loss_args a, double* __restrict__ pl,
                                                        int* __restrict__ pc) {
  __shared__ double rl[4];
  __shared__ int rc[4];
  const int term = blockIdx.y;
  const long rows = term_rows(a, term);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double sl = 0.0;
  int sc = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < rows; i += (long)gridDim.x * 256) {
    if (term == 0 || term == 3) {
      const int nc = a.n_classes;
      const float* x = term == 0 ? a.node_cls + (size_t)i * nc : a.obj + (size_t)i * nc;
      const int k = (int)(term == 0 ? a.node_class[i] : a.obj_class[i]);
      float lse;
      int am;
      row_stats(x, nc, lse, am);
      const float w = term == 0 ? a.class_w[k] : 1.f;
      sl += (double)(-(w * (x[k] - lse)));
      sc += am == k;
    } else if (term == 1) {
      const float t0 = (a.node_offsets[2 * i] - a.mu_x) / a.sigma_x;
      const float t1 = (a.node_offsets[2 * i + 1] - a.mu_y) / a.sigma_y;
      const float d0 = a.node_reg[2 * i] - t0, d1 = a.node_reg[2 * i + 1] - t1;
      sl += (double)(0.5f * (d0 * d0)) + (double)(0.5f * (d1 * d1));
    } else {
      const float* x = a.link + 2 * i;
      const int k = (int)a.edge_class[i];
      sl += (double)focal(x[0], k == 0 ? 1.f : 0.f) + (double)focal(x[1], k == 1 ? 1.f : 0.f);
      sc += (x[1] > x[0] ? 1 : 0) == k;
    }
  }
  sl = wave_sum_d(sl);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sc += __shfl_xor(sc, o, 64);
  if (lane == 0) {
    rl[wave] = sl;
    rc[wave] = sc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    pl[term * PARTS + blockIdx.x] = (rl[0] + rl[1]) + (rl[2] + rl[3]);
    pc[term * PARTS + blockIdx.x] = rc[0] + rc[1] + rc[2] + rc[3];
  }
}

__global__ __launch_bounds__(256) void loss_final_kernel(rg_loss_args a, const double* __restrict__ pl,
                                                         const int* __restrict__ pc,
                                                         float* __restrict__ losses,
                                                         float* __restrict__ acc) {
  __shared__ double rl[4];
  __shared__ long long rc[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int term = 0; term < 4; ++term) {
    double s = 0.0;
    long long c = 0;
    for (int i = threadIdx.x; i < PARTS; i += 256) {
      s += pl[term * PARTS + i];
      c += pc[term * PARTS + i];
    }
    s = wave_sum_d(s);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) {
      rl[wave] = s;
      rc[wave] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const double tot = (rl[0] + rl[1]) + (rl[2] + rl[3]);
      const long long cnt = rc[0] + rc[1] + rc[2] + rc[3];
      const long rows = term_rows(a, term);
      const float w = term == 0 ? a.w_node_cls : term == 1 ? a.w_node_reg
                                               : term == 2 ? a.w_edge_cls : a.w_obj_cls;
      losses[term] = (float)(tot / (double)rows) * w;  // 0 rows: NaN, as torch's 0 / 0
      const int ai = term == 0 ? 0 : term == 2 ? 1 : term == 3 ? 2 : -1;
      if (ai >= 0) acc[ai] = (float)((double)cnt / (double)rows);
    }
    __syncthreads();
  }
}

__global__ void loss_backward_kernel(rg_loss_args a, const float* __restrict__ g,
                                     float* __restrict__ dnc, float* __restrict__ dnr,
                                     float* __restrict__ dl, float* __restrict__ dob) {
  const int term = blockIdx.y;
  const float g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3];
  const long rows = term_rows(a, term);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
       i += (long)gridDim.x * blockDim.x) {
    if (term == 0 || term == 3) {
      const int nc = a.n_classes;
      const float* x = term == 0 ? a.node_cls + (size_t)i * nc : a.obj + (size_t)i * nc;
      float* d = term == 0 ? dnc + (size_t)i * nc : dob + (size_t)i * nc;
      const int k = (int)(term == 0 ? a.node_class[i] : a.obj_class[i]);
      float lse;
      int am;
      row_stats(x, nc, lse, am);
      const float w = term == 0 ? a.class_w[k] : 1.f;
      const float sc = term == 0 ? g0 * a.w_node_cls / (float)rows : g3 * a.w_obj_cls / (float)rows;
      for (int c = 0; c < nc; ++c) d[c] = sc * w * (expf(x[c] - lse) - (c == k ? 1.f : 0.f));
    } else if (term == 1) {
      const float t0 = (a.node_offsets[2 * i] - a.mu_x) / a.sigma_x;
      const float t1 = (a.node_offsets[2 * i + 1] - a.mu_y) / a.sigma_y;
      const float sc = g1 * a.w_node_reg / (float)rows;
      dnr[2 * i] = sc * (a.node_reg[2 * i] - t0);
      dnr[2 * i + 1] = sc * (a.node_reg[2 * i + 1] - t1);
    } else {
      const float* x = a.link + 2 * i;
      const int k = (int)a.edge_class[i];
      const float sc = g2 * a.w_edge_cls / (float)rows;
      dl[2 * i] = sc * focal_grad(x[0], k == 0 ? 1.f : 0.f);
      dl[2 * i + 1] = sc * focal_grad(x[1], k == 1 ? 1.f : 0.f);
    }
  }
}

// ------------------------------------------------------------------ SGD
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                           float* __restrict__ buf, long n, float lr, float momentum, float wd,
                           int first, float gscale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float d = fmaf(wd, p[i], __fmul_rn(g[i], gscale));  // d_p.add(p, alpha=wd)
  const float b = first ? d : __fadd_rn(__fmul_rn(momentum, buf[i]), d);  // buf.mul_(m).add_(d)
  buf[i] = b;
  p[i] = fmaf(-lr, b, p[i]);                          // p.add_(buf, alpha=-lr)
}

// ------------------------------------------------------------------ scheduled steps
// train_model's skip_batch + MultiStepLR on the device (rg_sgd_step_sched).  Every thread
// reads the applied-step counter k = state[parity] and the (all-reduced) losses; thread 0
// of block 0 writes k or k + 1 to state[parity ^ 1], a slot no thread of this launch reads.
struct StepCtl {
  bool skip;
  int k;        // applied steps before this one
  double lr;
};

__device__ __forceinline__ StepCtl step_control(const rg_lr_schedule& s, const float* losses,
                                                int n_losses, int* state, int parity) {
  StepCtl c;
  c.k = state[parity];
  c.skip = false;
  if (losses) {
    float t = losses[0];                      // total_loss = l0 + l1 + l2 + l3 (training.py:75)
    for (int i = 1; i < n_losses; ++i) t = __fadd_rn(t, losses[i]);
    c.skip = isnan(t);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) state[parity ^ 1] = c.k + (c.skip ? 0 : 1);
  double lr = s.lr[0];
#pragma unroll
  for (int j = 0; j < RG_LR_MILESTONES_MAX; ++j)
    if (j < s.n_milestones && s.milestones[j] <= c.k) lr = s.lr[j + 1];
  c.lr = lr;
  return c;
}

__global__ void sgd_sched_kernel(float* __restrict__ p, const float* __restrict__ g,
                                 float* __restrict__ buf, long n, rg_lr_schedule s,
                                 float momentum, float wd, float gscale,
                                 const float* __restrict__ losses, int n_losses, int* state,
                                 int parity) {
  const StepCtl c = step_control(s, losses, n_losses, state, parity);
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c.skip || i >= n) return;
  const float lr = (float)c.lr;
  const float d = fmaf(wd, p[i], __fmul_rn(g[i], gscale));
  const float b = c.k == 0 ? d : __fadd_rn(__fmul_rn(momentum, buf[i]), d);
  buf[i] = b;
  p[i] = fmaf(-lr, b, p[i]);
}

// torch.optim.AdamW's foreach update (torch/optim/adam.py _multi_tensor_adam, decoupled
// weight decay): the scalars are formed in double as Python forms them, the tensor ops in
// float32 as the foreach kernels run them
__global__ void adamw_sched_kernel(float* __restrict__ p, const float* __restrict__ g,
                                   float* __restrict__ m, float* __restrict__ v, long n,
                                   rg_lr_schedule s, double beta1, double beta2, double eps,
                                   double wd, float gscale, const float* __restrict__ losses,
                                   int n_losses, int* state, int parity) {
  const StepCtl c = step_control(s, losses, n_losses, state, parity);
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c.skip || i >= n) return;
  const double t = (double)(c.k + 1);
  const double bc1 = 1.0 - pow(beta1, t);
  const double bc2 = 1.0 - pow(beta2, t);
  const float step_size = (float)(-(c.lr / bc1));
  const float bc2_sqrt = (float)sqrt(bc2);
  const float decay = (float)(1.0 - c.lr * wd);
  const float gi = __fmul_rn(g[i], gscale);
  const float pi = __fmul_rn(p[i], decay);                    // p.mul_(1 - lr wd)
  const float w1 = (float)(1.0 - beta1);
  const float mi = m[i];
  const float mn = fmaf(w1, __fsub_rn(gi, mi), mi);            // lerp_(g, 1 - beta1), w < 0.5
  const float vn = fmaf(__fmul_rn((float)(1.0 - beta2), gi), gi, __fmul_rn(v[i], (float)beta2));
  m[i] = mn;
  v[i] = vn;
  const float den = __fadd_rn(__fdiv_rn(__fsqrt_rn(vn), bc2_sqrt), (float)eps);
  p[i] = fmaf(step_size, __fdiv_rn(mn, den), pi);              // addcdiv_(m, den, -step)
}

}  // namespace train
}  // namespace rg

using namespace rg;
using namespace rg::train;

// ----------------------------------------------------------------------------- C ABI
extern "C" size_t rg_ffn_backward_workspace_size(void) {
  return (size_t)FFN_PARTS_MAX * 2 * sizeof(double);
}

extern "C" int rg_ffn_backward_gather(const float* z, int ldz, const float* da, int ldda,
                                      const int* gidx, const float* gscale, long rows, int C,
                                      int has_norm, const float* mu, const float* std_, int act,
                                      float* dz, int lddz, float* d_mu, float* d_std,
                                      void* workspace, void* stream) {
  RG_REQUIRE(C >= 1 && C <= 256, RG_ERR_UNSUPPORTED, "rg_ffn_backward: C=%d outside 1..256", C);
  RG_REQUIRE(!has_norm || (mu && std_ && d_mu && d_std && C >= 2 && workspace), RG_ERR_ARG,
             "rg_ffn_backward: norm needs mu, std, their gradients, C >= 2 and a workspace");
  RG_REQUIRE(act >= ACT_NONE && act <= ACT_SWISH, RG_ERR_ARG, "rg_ffn_backward: act %d", act);
  RG_REQUIRE(!gidx || (const float*)dz != da, RG_ERR_ARG,
             "rg_ffn_backward_gather: dz may not alias a gathered da");
  if (rows <= 0) return RG_OK;
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)workspace;
  // 2048 workgroups (8 waves per SIMD: each 16-lane group's row loop is one dependent
  // load -> compute -> store chain; 512 left it latency-bound, c4 backward -0.7 ms; 1 024
  // and 4 096 the same within noise)
  constexpr int parts = 2048;
  static_assert(parts <= FFN_PARTS_MAX, "ffn backward partials");
  if (C <= 16)
    ffn_backward_kernel<1><<<parts, 256, 0, st>>>(z, ldz, da, ldda, rows, C, has_norm, mu, std_,
                                                  act, dz, lddz, part, gidx, gscale);
  else if (C <= 64)
    ffn_backward_kernel<4><<<parts, 256, 0, st>>>(z, ldz, da, ldda, rows, C, has_norm, mu, std_,
                                                  act, dz, lddz, part, gidx, gscale);
  else if (C <= 128)
    ffn_backward_kernel<8><<<parts, 256, 0, st>>>(z, ldz, da, ldda, rows, C, has_norm, mu, std_,
                                                  act, dz, lddz, part, gidx, gscale);
  else
    ffn_backward_kernel<16><<<parts, 256, 0, st>>>(z, ldz, da, ldda, rows, C, has_norm, mu, std_,
                                                   act, dz, lddz, part, gidx, gscale);
  RG_LAUNCH_CHECK();
  if (has_norm) {
    ffn_param_reduce<<<1, 256, 0, st>>>(part, parts, d_mu, d_std);
    RG_LAUNCH_CHECK();
  }
  return RG_OK;
}

extern "C" int rg_ffn_backward(const float* z, int ldz, const float* da, int ldda, long rows, int C,
                               int has_norm, const float* mu, const float* std_, int act,
                               float* dz, int lddz, float* d_mu, float* d_std, void* workspace,
                               void* stream) {
  return rg_ffn_backward_gather(z, ldz, da, ldda, nullptr, nullptr, rows, C, has_norm, mu, std_,
                                act, dz, lddz, d_mu, d_std, workspace, stream);
}

int rg_train_param_reduce(const double* part, int parts, float* d_mu, float* d_std, void* stream) {
  ffn_param_reduce<<<1, 256, 0, (hipStream_t)stream>>>(part, parts, d_mu, d_std);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_linear_grad_workspace_size(long rows, int out_dim, int in_dim) {
  if (rows <= 0) return 256;
  return grad_ws_bytes(grad_geom(rows, out_dim, in_dim));
}

extern "C" int rg_linear_grad_ld(const float* dz, int lddz, long rows, int out_dim, int in_dim,
                                 int in_mode, const float* in0, int ld0, int w0, const float* in1,
                                 int ld1, int w1, const float* in2, int ld2, int w2,
                                 const int* idx0, const int* idx1, float* dW, int ld_dw, float* db,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  RG_REQUIRE(out_dim >= 1 && in_dim >= 1, RG_ERR_ARG, "rg_linear_grad: dims");
  RG_REQUIRE(ld_dw >= in_dim, RG_ERR_ARG, "rg_linear_grad: ld_dw %d < in_dim %d", ld_dw, in_dim);
  RG_REQUIRE(in_mode >= RG_IN_DENSE && in_mode <= RG_IN_PAIRADD, RG_ERR_ARG, "bad in_mode");
  RG_REQUIRE((in_mode != RG_IN_GATHER3 && in_mode != RG_IN_PAIRADD) || (idx0 && idx1), RG_ERR_ARG,
             "rg_linear_grad: gather modes need idx0 and idx1");
  int expect = in_mode == RG_IN_CONCAT2 ? w0 + w1 : in_mode == RG_IN_GATHER3 ? 2 * w0 + w2 : w0;
  RG_REQUIRE(expect == in_dim, RG_ERR_ARG, "rg_linear_grad: input width %d != in_dim %d", expect,
             in_dim);
  if (rows <= 0) return RG_OK;
  const GradGeom g = grad_geom(rows, out_dim, in_dim);
  const size_t need = grad_ws_bytes(g);
  RG_REQUIRE(workspace_bytes >= need, RG_ERR_ARG, "rg_linear_grad: workspace %zu < %zu",
             workspace_bytes, need);
  GradIn in;
  in.mode = in_mode; in.in_dim = in_dim;
  in.in0 = in0; in.in1 = in1; in.in2 = in2;
  in.ld0 = ld0; in.ld1 = ld1; in.ld2 = ld2; in.w0 = w0; in.w1 = w1; in.w2 = w2;
  in.idx0 = idx0; in.idx1 = idx1;
  // vector (16-B) staging when no 4-feature group straddles a segment or a row
  const bool a0 = ld0 % 4 == 0 && w0 % 4 == 0;
  const bool a1 = in_mode != RG_IN_CONCAT2 || (ld1 % 4 == 0 && w1 % 4 == 0);
  const bool a2 = in_mode != RG_IN_GATHER3 || (ld2 % 4 == 0 && w2 % 4 == 0);
  const int vec_x = a0 && a1 && a2 && in_dim % 4 == 0;
  const int vec_z = lddz % 4 == 0;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  float* part_b = part + grad_part_floats(g);
#define RG_GRAD_CASE(OW, NT)                                                                   \
  if (g.ow == OW && g.nt == NT) {                                                              \
    const int rc = launch_grad<OW, NT>(g, dz, lddz, rows, out_dim, in, vec_x, vec_z, part, part_b, st); \
    if (rc != RG_OK) return rc;                                                                \
  }
  RG_GRAD_CASE(1, 1) RG_GRAD_CASE(1, 4) RG_GRAD_CASE(1, 8) RG_GRAD_CASE(1, 12) RG_GRAD_CASE(1, 16)
  RG_GRAD_CASE(2, 1) RG_GRAD_CASE(2, 4) RG_GRAD_CASE(2, 8) RG_GRAD_CASE(2, 12) RG_GRAD_CASE(2, 16)
#undef RG_GRAD_CASE
  RG_LAUNCH_CHECK();
  const long total = (long)out_dim * (in_dim + 1);
  linear_grad_reduce<<<ceil_div(total, 64), 64 * RW, 0, st>>>(part, part_b, g.nchunk, g.ot, g.it,
                                                           64 * g.ow, 16 * g.nt, out_dim, in_dim,
                                                           dW, db, ld_dw);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_linear_grad(const float* dz, int lddz, long rows, int out_dim, int in_dim,
                              int in_mode, const float* in0, int ld0, int w0, const float* in1,
                              int ld1, int w1, const float* in2, int ld2, int w2, const int* idx0,
                              const int* idx1, float* dW, float* db, void* workspace,
                              size_t workspace_bytes, void* stream) {
  return rg_linear_grad_ld(dz, lddz, rows, out_dim, in_dim, in_mode, in0, ld0, w0, in1, ld1, w1,
                           in2, ld2, w2, idx0, idx1, dW, in_dim, db, workspace, workspace_bytes,
                           stream);
}

extern "C" size_t rg_incidence_workspace_size(int n_nodes, long n_items) {
  (void)n_items;
  return ((size_t)2 * (n_nodes + 1) * sizeof(int) + 255) / 256 * 256 + scan_workspace_bytes(n_nodes);
}

extern "C" int rg_incidence(const int* a, const int* b, long n_items, int n_nodes, int* ptr,
                            int* list, void* workspace, size_t workspace_bytes, void* stream) {
  RG_REQUIRE(n_nodes >= 0 && n_items >= 0 && a, RG_ERR_ARG, "rg_incidence: args");
  RG_REQUIRE(workspace_bytes >= rg_incidence_workspace_size(n_nodes, n_items), RG_ERR_ARG,
             "rg_incidence: workspace");
  hipStream_t st = (hipStream_t)stream;
  int* cnt = (int*)workspace;
  int* cursor = cnt + (n_nodes + 1);
  void* sws = (char*)workspace + ((size_t)2 * (n_nodes + 1) * sizeof(int) + 255) / 256 * 256;
  if (n_nodes == 0) return RG_OK;
  RG_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)n_nodes * sizeof(int), st));
  if (n_items > 0) {
    inc_count<<<ceil_div(n_items, 256), 256, 0, st>>>(a, b, n_items, cnt);
    RG_LAUNCH_CHECK();
  }
  int rc = exclusive_scan(cnt, n_nodes, ptr, nullptr, sws, st);
  if (rc) return rc;
  if (n_items == 0) return RG_OK;
  RG_CHECK_HIP(hipMemcpyAsync(cursor, ptr, (size_t)n_nodes * sizeof(int), hipMemcpyDeviceToDevice, st));
  inc_fill<<<ceil_div(n_items, 256), 256, 0, st>>>(a, b, n_items, cursor, list);
  RG_LAUNCH_CHECK();
  inc_sort<<<ceil_div(n_nodes, 256), 256, 0, st>>>(ptr, n_nodes, list);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gather_segment_sum(const float* src, int ld_src, int col0, int width,
                                     const int* ptr, const int* list, const float* scale,
                                     int n_nodes, float* out, int ld_out, int accumulate,
                                     void* stream) {
  RG_REQUIRE(width >= 1 && width <= 256, RG_ERR_UNSUPPORTED, "rg_gather_segment_sum: width %d",
             width);
  if (n_nodes <= 0) return RG_OK;
  // the streaming kernel for 16-B aligned rows, the one-wave-per-node kernel otherwise (both
  // sum in list order: the parity test checks each against the sequential float32 sum)
  const bool al = ld_src % 4 == 0 && col0 % 4 == 0 && width % 4 == 0 && ld_out % 4 == 0 &&
                  (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0;
  if (al) {
    if (scale)
      gather_segsum_stream<true><<<ceil_div(n_nodes, 16), 256, 0, (hipStream_t)stream>>>(
          src, ld_src, col0, width, ptr, list, scale, n_nodes, out, ld_out, accumulate);
    else
      gather_segsum_stream<false><<<ceil_div(n_nodes, 16), 256, 0, (hipStream_t)stream>>>(
          src, ld_src, col0, width, ptr, list, scale, n_nodes, out, ld_out, accumulate);
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  int blocks = ceil_div(n_nodes, 4);
  if (blocks > 4096) blocks = 4096;
  gather_segsum_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(
      src, ld_src, col0, width, ptr, list, scale, n_nodes, out, ld_out, accumulate);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_segment_max_backward(const float* h, int ld_h, int C, const int* cluster_ptr,
                                       const int* cluster_idx, int n_clusters,
                                       const float* dpooled, int ld_p, float* dh, int ld_dh,
                                       void* stream) {
  if (n_clusters <= 0 || C <= 0) return RG_OK;
  const long total = (long)n_clusters * C;
  segmax_backward_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
      h, ld_h, C, cluster_ptr, cluster_idx, n_clusters, dpooled, ld_p, dh, ld_dh);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_loss_workspace_size(long n_nodes, long n_pairs, long n_clusters) {
  (void)n_nodes; (void)n_pairs; (void)n_clusters;
  return (size_t)4 * PARTS * (sizeof(double) + sizeof(int));
}

extern "C" int rg_loss_graph(const rg_loss_args* args, float* losses, float* acc, void* workspace,
                             size_t workspace_bytes, void* stream) {
  RG_REQUIRE(args && losses && acc, RG_ERR_ARG, "rg_loss_graph: args");
  RG_REQUIRE(args->n_classes >= 1 && args->n_classes <= 64, RG_ERR_UNSUPPORTED,
             "rg_loss_graph: n_classes");
  RG_REQUIRE(workspace_bytes >= rg_loss_workspace_size(0, 0, 0), RG_ERR_ARG,
             "rg_loss_graph: workspace");
  hipStream_t st = (hipStream_t)stream;
  double* pl = (double*)workspace;
  int* pc = (int*)(pl + 4 * PARTS);
  loss_rows_kernel<<<dim3(PARTS, 4), 256, 0, st>>>(*args, pl, pc);
  RG_LAUNCH_CHECK();
  loss_final_kernel<<<1, 256, 0, st>>>(*args, pl, pc, losses, acc);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_loss_graph_backward(const rg_loss_args* args, const float* g, float* d_node_cls,
                                      float* d_node_reg, float* d_link, float* d_obj,
                                      void* stream) {
  RG_REQUIRE(args && g, RG_ERR_ARG, "rg_loss_graph_backward: args");
  RG_REQUIRE(args->n_classes >= 1 && args->n_classes <= 64, RG_ERR_UNSUPPORTED,
             "rg_loss_graph_backward: n_classes");
  loss_backward_kernel<<<dim3(256, 4), 256, 0, (hipStream_t)stream>>>(
      *args, g, d_node_cls, d_node_reg, d_link, d_obj);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_sgd_step(float* param, const float* grad, float* momentum_buf, long n, float lr,
                           float momentum, float weight_decay, int first_step, float grad_scale,
                           void* stream) {
  if (n <= 0) return RG_OK;
  sgd_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(
      param, grad, momentum_buf, n, lr, momentum, weight_decay, first_step, grad_scale);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

static int check_sched(const rg_lr_schedule* s, const float* losses, int n_losses,
                       const int* step_state, int parity) {
  RG_REQUIRE(s && step_state, RG_ERR_ARG, "optimizer step: schedule and step_state required");
  RG_REQUIRE(s->n_milestones >= 0 && s->n_milestones <= RG_LR_MILESTONES_MAX, RG_ERR_ARG,
             "optimizer step: %d milestones (max %d)", s->n_milestones, RG_LR_MILESTONES_MAX);
  for (int j = 0; j < s->n_milestones; ++j)
    RG_REQUIRE(s->milestones[j] >= 0 && (j == 0 || s->milestones[j] > s->milestones[j - 1]),
               RG_ERR_ARG, "optimizer step: milestones must be distinct, ascending, >= 0");
  RG_REQUIRE(!losses || (n_losses >= 1 && n_losses <= 16), RG_ERR_ARG,
             "optimizer step: n_losses %d", n_losses);
  RG_REQUIRE(parity == 0 || parity == 1, RG_ERR_ARG, "optimizer step: parity %d", parity);
  return RG_OK;
}

extern "C" int rg_sgd_step_sched(float* param, const float* grad, float* momentum_buf, long n,
                                 const rg_lr_schedule* sched, float momentum, float weight_decay,
                                 float grad_scale, const float* losses, int n_losses,
                                 int* step_state, int parity, void* stream) {
  const int rc = check_sched(sched, losses, n_losses, step_state, parity);
  if (rc != RG_OK) return rc;
  // one block even for n = 0: the counter still advances (an empty model's step counts)
  sgd_sched_kernel<<<n > 0 ? ceil_div(n, 256) : 1, 256, 0, (hipStream_t)stream>>>(
      param, grad, momentum_buf, n, *sched, momentum, weight_decay, grad_scale, losses,
      n_losses, step_state, parity);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_adamw_step_sched(float* param, const float* grad, float* exp_avg,
                                   float* exp_avg_sq, long n, const rg_lr_schedule* sched,
                                   double beta1, double beta2, double eps, double weight_decay,
                                   float grad_scale, const float* losses, int n_losses,
                                   int* step_state, int parity, void* stream) {
  const int rc = check_sched(sched, losses, n_losses, step_state, parity);
  if (rc != RG_OK) return rc;
  RG_REQUIRE(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0,
             RG_ERR_ARG, "rg_adamw_step_sched: betas / eps");
  adamw_sched_kernel<<<n > 0 ? ceil_div(n, 256) : 1, 256, 0, (hipStream_t)stream>>>(
      param, grad, exp_avg, exp_avg_sq, n, *sched, beta1, beta2, eps, weight_decay, grad_scale,
      losses, n_losses, step_state, parity);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
