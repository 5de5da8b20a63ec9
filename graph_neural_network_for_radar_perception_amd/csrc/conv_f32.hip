// Fused float32 residual_graph_conv_block (gnn_blocks.py:96-113) -- the reference
// precision -- for the shipped widths (C = 64 node / edge channels, message MLP
// 192 -> 128 -> 64, update 128 -> 64, channel_normalization + activation on every block,
// aggregation add or mean).  Exact f32 products on v_mfma_f32_32x32x2_f32.
//
// One C-ABI call = two launches:
//  1. projections (chain_f32.hip, 64 -> 256 per node): P[i] = W_xi x[i] + b1 and
//     Q[j] = W_xj x[j], the x_i and x_j thirds of the first message layer, computed once
//     per NODE instead of once per edge (msg0(cat(x_i, x_j, e)) = P[i] + Q[j] + W_e e);
//     this launch also zeroes the work counters of launch 2;
//  2. the fused layer: work block = 32 destination nodes and their incoming edges (one
//     contiguous range of the destination-major CSR).  Per 32-edge tile a wave computes
//        h = act(norm(P[dst] + Q[src] + W_e e))         128 MFMAs (K = 64, N = 128)
//        m = act(norm(W_2 h + b2))                       128 MFMAs (K = 128, N = 64)
//     (layer 2 takes layer 1's accumulators as its B operand in registers), then the
//     segmented sum: the message tile goes through a wave-private LDS tile so that lane
//     = feature, and every lane adds the tile's messages IN EDGE ORDER into a running
//     sum, starting a new sum at each change of destination (the destination of an
//     edge is wave-uniform: a scalar compare) -- the reference scatter_add_ order, no
//     MFMA spent on the reduction.  After the block's last tile the aggregates (LDS,
//     row = node) and x[node] are the update MLP's B operand; update + norm + act +
//     residual, store.  Messages and aggregates never touch HBM.
// Two waves per SIMD (conv_f32_kernel2 below).  Workgroups are persistent; block ids come from one atomic counter per XCD over that
// XCD's contiguous eighth of the nodes (workgroup w runs on XCD w % 8), so each frame's
// x, P and Q rows are gathered from one L2.
#include "rg_common.h"

#include <stdlib.h>

namespace rg {
namespace convf32 {

static constexpr int FT = 256;       // 4 waves, one per SIMD
static constexpr int NW = FT / 64;
static constexpr int C = 64;         // node / edge / message / output channels
static constexpr int HID = 128;      // msg_mlp_hidden_dim
static constexpr int NBLK = 32;      // destination nodes per work block
static constexpr int TS = 68;        // LDS row stride (floats) of the message half-tile
static constexpr int AS = 68;        // LDS row stride (floats) of the aggregate rows
static constexpr float NORM_EPS = 1e-5f;
static constexpr int NXCD = 8;

__host__ __device__ constexpr int fbytes(int K, int N) {
  return (N / 32) * ((K + 7) / 8) * 1024 + N * 4;
}
static constexpr int W_E_OFF = 0;                                       // W_e: 64 -> 128
static constexpr int W_2_OFF = (fbytes(C, HID) + 15) & ~15;             // W_2: 128 -> 64
static constexpr int W_U_OFF = W_2_OFF + ((fbytes(HID, C) + 15) & ~15);  // W_u: 128 -> 64
static constexpr int W_BYTES = W_U_OFF + ((fbytes(2 * C, C) + 15) & ~15);
static constexpr int WAVE_LDS = (16 * TS + NBLK * AS) * 4;
static constexpr int LDS_BYTES = W_BYTES + NW * WAVE_LDS;
static_assert(LDS_BYTES <= DYN_LDS_MAX, "conv_f32 LDS");

struct Args {
  const float* x;
  const float* e;
  const float* pq;  // [N][256]: P (0..127) | Q (128..255)
  const int* seg_ptr;
  const int* src;
  const int* dst;
  float* x_out;
  int* counters;  // [NXCD], zero at launch (zeroed by the projection launch)
  const void* w[3];  // W_e, W_2, W_u (RG_PACK_F32_FAST)
  const float* mu[3];
  const float* sd[3];
  int ldx, lde, ldpq, ldo;
  int n_nodes, n_blocks;
  int aggr_mean;
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int S4, int MT, typename BOp>
__device__ __forceinline__ void layer(f32x16 (&acc)[MT], const char* w, int lane, BOp&& bop) {
  const f32x4* wa = (const f32x4*)w + lane;
  f32x4 a[2][MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) a[0][m] = wa[(m * S4) * 64];
#pragma unroll
  for (int s4 = 0; s4 < S4; ++s4) {
    if (s4 + 1 < S4) {
#pragma unroll
      for (int m = 0; m < MT; ++m) a[(s4 + 1) & 1][m] = wa[(m * S4 + s4 + 1) * 64];
    }
    const f32x4 b = bop(s4);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = mfma(a[s4 & 1][m][u], b[u], acc[m]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// channel_normalization (common.py:208-220) + activation over a row's 32*MT features
template <int MT>
__device__ __forceinline__ void norm_act(f32x16 (&acc)[MT], float mu, float sd, int act) {
  constexpr int N = 32 * MT;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      s0 += acc[m][q];
      s1 += acc[m][q + 1];
    }
  const float mean = add_xor32(s0 + s1) * (1.f / N);
  float q0 = 0.f, q1 = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      const float d0 = acc[m][q] - mean, d1 = acc[m][q + 1] - mean;
      q0 = fmaf(d0, d0, q0);
      q1 = fmaf(d1, d1, q1);
    }
  const float ss = add_xor32(q0 + q1);
  const float inv = 1.f / (sqrtf(ss / (float)(N - 1)) + NORM_EPS);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q)
      acc[m][q] = __fadd_rn(__fmul_rn(sd, __fmul_rn(acc[m][q] - mean, inv)), mu);
  act_dispatch(act, [&](auto A) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] = act_t<decltype(A)::value>(acc[m][q]);
  });
}

struct Rows {
  f32x4 p[16];  // P[dst]: features 32m + 8g + 4h .. +3 at [4m + g]
  f32x4 q[16];  // Q[src]
  f32x4 e[8];   // e[edge]: features 8 s4 + 4h .. +3 at [s4]
};
struct Idx {
  int d, s;
};

// ---------------------------------------------------------------------------------------
// Two waves per SIMD (512-thread workgroups, <= 256 registers per wave): the second wave
// of a SIMD issues its MFMAs while the first runs its epilogues or waits for its rows, so
// the matrix pipe is fed without hand-interleaving.  LDS: W_e and W_2 (66 KiB) stay
// resident; W_u (once per block) is read from L2; per wave an 8-edge message tile and
// the block's 32 aggregate rows.  The channel_normalization + LeakyReLU epilogue is five
// VALU ops per feature: sum, x - mean, sum of squares, y' = x a + b with the 0.505 of
// leaky(y) = 0.505 y + 0.495 |y| folded into a and b, then |y'| C + y' (C = 0.495 / 0.505).
#ifndef RG_CF32_PQLATE
#define RG_CF32_PQLATE 0
#endif
#ifndef RG_CF32_PRIO
#define RG_CF32_PRIO 0
#endif
static constexpr int FT2 = 512;
static constexpr int NW2 = FT2 / 64;
static constexpr int TR2 = 8;   // message rows per LDS pass
static constexpr int W2_BYTES = W_U_OFF;  // W_e + W_2 staged; W_u streamed
static constexpr int WAVE_LDS2 = (TR2 * TS + NBLK * AS) * 4;
static constexpr int LDS_BYTES2 = W2_BYTES + NW2 * WAVE_LDS2;
static_assert(LDS_BYTES2 <= DYN_LDS_MAX, "conv_f32 (2 waves / SIMD) LDS");
static constexpr float LEAKY_PRE2 = 0.505f;
static constexpr float LEAKY_C2 = 0.495f / 0.505f;

// channel_normalization + LeakyReLU (common.py:208-220, 256-267), five ops per feature
template <int MT>
__device__ __forceinline__ void norm_leaky5(f32x16 (&acc)[MT], float mu, float sd) {
  constexpr int N = 32 * MT;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      s0 += acc[m][q];
      s1 += acc[m][q + 1];
    }
  const float mean = add_xor32(s0 + s1) * (1.f / N);
  float q0 = 0.f, q1 = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      acc[m][q] -= mean;
      acc[m][q + 1] -= mean;
      q0 = fmaf(acc[m][q], acc[m][q], q0);
      q1 = fmaf(acc[m][q + 1], acc[m][q + 1], q1);
    }
  const float ss = add_xor32(q0 + q1);
  const float inv = 1.f / (sqrtf(ss / (float)(N - 1)) + NORM_EPS);
  const float ga = LEAKY_PRE2 * (sd * inv), gb = LEAKY_PRE2 * mu;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float y = fmaf(acc[m][q], ga, gb);
      acc[m][q] = fmaf(fabsf(y), LEAKY_C2, y);
    }
}

// layer with A fragments from global memory (L2), prefetched two k-quads ahead
template <int S4, int MT, typename BOp>
__device__ __forceinline__ void layer_g(f32x16 (&acc)[MT], const char* w, int lane, BOp&& bop) {
  const f32x4* wa = (const f32x4*)w + lane;
  constexpr int PD = 2, NB = PD + 1;
  f32x4 a[NB][MT];
#pragma unroll
  for (int s = 0; s < PD; ++s)
#pragma unroll
    for (int m = 0; m < MT; ++m) a[s][m] = wa[(m * S4 + s) * 64];
#pragma unroll
  for (int s4 = 0; s4 < S4; ++s4) {
    if (s4 + PD < S4) {
#pragma unroll
      for (int m = 0; m < MT; ++m) a[(s4 + PD) % NB][m] = wa[(m * S4 + s4 + PD) * 64];
    }
    const f32x4 b = bop(s4);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = mfma(a[s4 % NB][m][u], b[u], acc[m]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

__global__ __launch_bounds__(FT2) void conv_f32_kernel2(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[6];
  if (threadIdx.x < 3) {
    nrm[2 * threadIdx.x] = *a.mu[threadIdx.x];
    nrm[2 * threadIdx.x + 1] = *a.sd[threadIdx.x];
  }
  {
    const int nb[2] = {fbytes(C, HID), fbytes(HID, C)};
    const int off[2] = {W_E_OFF, W_2_OFF};
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      stage_lds<FT2>(lds + off[l], a.w[l], nb[l]);
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
#if RG_CF32_PRIO
  // the second wave of each SIMD (waves 4-7) yields the issue port: the pair drifts out
  // of lock-step, so one wave's epilogue runs under the other's MFMAs
  if (wave >= NW2 / 2) __builtin_amdgcn_s_setprio(1);
#endif
  float* T = (float*)(lds + W2_BYTES + wave * WAVE_LDS2);  // [TR2][TS] message rows
  float* Agg = T + TR2 * TS;                              // [NBLK][AS] aggregates
  const char* wE = lds + W_E_OFF;
  const char* w2 = lds + W_2_OFF;
  const char* wU = (const char*)a.w[2];
  const float* bias2 = (const float*)(w2 + 2 * 16 * 1024);
  const float* biasU = (const float*)(wU + 2 * 16 * 1024);
  const float mu0 = nrm[0], sd0 = nrm[1], mu1 = nrm[2], sd1 = nrm[3], muU = nrm[4], sdU = nrm[5];

  const int xcd = blockIdx.x % NXCD;
  const int blo = (int)((long)a.n_blocks * xcd / NXCD);
  const int bhi = (int)((long)a.n_blocks * (xcd + 1) / NXCD);
  int* ctr = a.counters + xcd;

  for (;;) {
    int bi = 0;
    if (lane == 0) bi = atomicAdd(ctr, 1);
    const int blk = blo + __shfl(bi, 0, 64);
    if (blk >= bhi) break;
    const int n0 = blk * NBLK;
    const int n1 = min(n0 + NBLK, a.n_nodes);
    const int e0 = a.seg_ptr[n0], e1 = a.seg_ptr[n1];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = lane + 64 * i;
      *(f32x4*)(Agg + (idx >> 4) * AS + 4 * (idx & 15)) = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    float run = 0.f;
    int cur = -1;
    int pn = min(e0 + r, e1 - 1);
    int dn = e0 < e1 ? a.dst[pn] : 0, sn = e0 < e1 ? a.src[pn] : 0;
    for (int t0 = e0; t0 < e1; t0 += 32) {
      const int p = pn, d = dn, sj = sn;
      // the next tile's indices now (their latency hides behind this tile)
      pn = min(t0 + 32 + r, e1 - 1);
      dn = a.dst[pn];
      sn = a.src[pn];
      // ---- layer 1: h = P[dst] + Q[src] + W_e e
      f32x16 acc1[4];
#if RG_CF32_PQLATE
      // the MFMAs need only the e rows: P and Q arrive while they run and are added after
      {
        const float* pe = a.e + (size_t)p * a.lde + 4 * h;
        const float* pp = a.pq + (size_t)d * a.ldpq + 4 * h;
        const float* pq = a.pq + (size_t)sj * a.ldpq + HID + 4 * h;
        f32x4 eb[8], pv[16], qv[16];
#pragma unroll
        for (int s4 = 0; s4 < 8; ++s4) eb[s4] = *(const f32x4*)(pe + 8 * s4);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          pv[i] = *(const f32x4*)(pp + 8 * i);
          qv[i] = *(const f32x4*)(pq + 8 * i);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) acc1[m] = (f32x16){0.f};
        layer<8, 4>(acc1, wE, lane, [&](int s4) { return eb[s4]; });
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc1[m][4 * g + t] += pv[4 * m + g][t] + qv[4 * m + g][t];
      }
#else
      {
        const float* pp = a.pq + (size_t)d * a.ldpq + 4 * h;
        const float* pq = a.pq + (size_t)sj * a.ldpq + HID + 4 * h;
        f32x4 pv[16], qv[16];
        {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            pv[i] = *(const f32x4*)(pp + 8 * i);
            qv[i] = *(const f32x4*)(pq + 8 * i);
          }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc1[m][4 * g + t] = pv[4 * m + g][t] + qv[4 * m + g][t];
      }
      {
        const float* pe = a.e + (size_t)p * a.lde + 4 * h;
        f32x4 eb[8];
#pragma unroll
        for (int s4 = 0; s4 < 8; ++s4) eb[s4] = *(const f32x4*)(pe + 8 * s4);
        layer<8, 4>(acc1, wE, lane, [&](int s4) { return eb[s4]; });
      }
#endif
      norm_leaky5<4>(acc1, mu0, sd0);
      // ---- layer 2
      f32x16 acc2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) acc2[m] = ld_bias_frag(bias2, m, h);
      layer<16, 2>(acc2, w2, lane, [&](int s4) {
        const f32x16& q = acc1[s4 >> 2];
        const int o = 4 * (s4 & 3);
        return (f32x4){q[o], q[o + 1], q[o + 2], q[o + 3]};
      });
      norm_leaky5<2>(acc2, mu1, sd1);
      // ---- segmented sum in edge order, 8 edges per LDS pass
#pragma unroll
      for (int c = 0; c < 32 / TR2; ++c) {
        if (t0 + TR2 * c >= e1) break;  // wave-uniform
        if (r / TR2 == c) {
          float* row = T + (r % TR2) * TS + 4 * h;
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *(f32x4*)(row + 32 * m + 8 * g) = (f32x4){acc2[m][4 * g], acc2[m][4 * g + 1],
                                                        acc2[m][4 * g + 2], acc2[m][4 * g + 3]};
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < TR2; ++j) {
          const int eo = TR2 * c + j;
          if (t0 + eo < e1) {
            const float v = T[j * TS + lane];
            const int slot = __builtin_amdgcn_readlane(d, eo) - n0;
            run = slot == cur ? run + v : v;
            Agg[slot * AS + lane] = run;
            cur = slot;
          }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();

    // ---- update MLP on cat(x[node], agg[node]) + residual (gnn_blocks.py:103-109)
    const int node = n0 + r;
    const bool nvalid = node < n1;
    const float* px = a.x + (size_t)(nvalid ? node : n0) * a.ldx + 4 * h;
    f32x4 xb[8], ab[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) xb[s] = *(const f32x4*)(px + 8 * s);
    float cnt = 1.f;
    if (a.aggr_mean) {  // PyG mean: sum / max(count, 1)
      const int deg = nvalid ? a.seg_ptr[node + 1] - a.seg_ptr[node] : 1;
      cnt = (float)(deg > 0 ? deg : 1);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      f32x4 v = *(const f32x4*)(Agg + r * AS + 8 * s + 4 * h);
      if (a.aggr_mean) v = (f32x4){div_rn(v.x, cnt), div_rn(v.y, cnt), div_rn(v.z, cnt), div_rn(v.w, cnt)};
      ab[s] = v;
    }
    f32x16 accu[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) accu[m] = ld_bias_frag(biasU, m, h);
    layer_g<16, 2>(accu, wU, lane, [&](int s4) { return s4 < 8 ? xb[s4] : ab[s4 - 8]; });
    norm_leaky5<2>(accu, muU, sdU);
    if (nvalid) {
      float* po = a.x_out + (size_t)node * a.ldo + 4 * h;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 xr = xb[4 * m + g];
          *(f32x4*)(po + 32 * m + 8 * g) =
              (f32x4){__fadd_rn(xr.x, accu[m][4 * g]), __fadd_rn(xr.y, accu[m][4 * g + 1]),
                      __fadd_rn(xr.z, accu[m][4 * g + 2]), __fadd_rn(xr.w, accu[m][4 * g + 3])};
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace convf32
}  // namespace rg

using namespace rg;
using namespace rg::convf32;

int rg_f32_chain_launch(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                        int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                        const int* idx1, float* out, int ld_out, int* zero_ptr, int zero_n,
                        void* stream);

extern "C" size_t rg_conv_layer_f32_workspace_size(int n_nodes) {
  return 256 + (size_t)(n_nodes > 0 ? n_nodes : 1) * 2 * HID * sizeof(float);
}

extern "C" int rg_conv_layer_f32(const rg_layer* layers, int aggr, const float* x, int ldx,
                                 const float* e, int lde, const int* seg_ptr, const int* src,
                                 const int* dst, int n_nodes, float* x_out, int ld_out,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const rg_layer& pq = layers[0];
  const rg_layer& m0 = layers[1];
  const rg_layer& m1 = layers[2];
  const rg_layer& u = layers[3];
  if (!(pq.in_dim == C && pq.out_dim == 2 * HID && m0.in_dim == C && m0.out_dim == HID &&
        m1.in_dim == HID && m1.out_dim == C && u.in_dim == 2 * C && u.out_dim == C))
    return RG_ERR_UNSUPPORTED;
  if (aggr != RG_REDUCE_SUM && aggr != RG_REDUCE_MEAN) return RG_ERR_UNSUPPORTED;
  if (pq.norm_mu || pq.act != ACT_NONE) return RG_ERR_UNSUPPORTED;
  if (!m0.norm_mu || !m1.norm_mu || !u.norm_mu) return RG_ERR_UNSUPPORTED;
  if (m0.act != ACT_LEAKY || m1.act != ACT_LEAKY || u.act != ACT_LEAKY) return RG_ERR_UNSUPPORTED;
  RG_REQUIRE(ldx % 4 == 0 && lde % 4 == 0 && ld_out % 4 == 0, RG_ERR_UNSUPPORTED,
             "rg_conv_layer_f32: row strides must be multiples of 4");
  RG_REQUIRE(x != x_out, RG_ERR_ARG, "rg_conv_layer_f32: x_out must not alias x");
  RG_REQUIRE(workspace_bytes >= rg_conv_layer_f32_workspace_size(n_nodes), RG_ERR_ARG,
             "rg_conv_layer_f32: workspace too small");
  if (n_nodes <= 0) return RG_OK;
  Args a;
  memset(&a, 0, sizeof(a));
  a.counters = (int*)workspace;
  float* pqbuf = (float*)((char*)workspace + 256);
  // launch 1: P | Q for every node (+ zero the work counters)
  int rc = rg_f32_chain_launch(&pq, 1, n_nodes, nullptr, RG_IN_DENSE, x, ldx, C, nullptr, nullptr,
                               pqbuf, 2 * HID, a.counters, NXCD, stream);
  if (rc) return rc;
  a.x = x;
  a.e = e;
  a.pq = pqbuf;
  a.seg_ptr = seg_ptr;
  a.src = src;
  a.dst = dst;
  a.x_out = x_out;
  a.w[0] = m0.w_packed;
  a.w[1] = m1.w_packed;
  a.w[2] = u.w_packed;
  const rg_layer* ls[3] = {&m0, &m1, &u};
  for (int l = 0; l < 3; ++l) {
    a.mu[l] = ls[l]->norm_mu;
    a.sd[l] = ls[l]->norm_std;
  }
  a.ldx = ldx;
  a.lde = lde;
  a.ldpq = 2 * HID;
  a.ldo = ld_out;
  a.n_nodes = n_nodes;
  a.n_blocks = (n_nodes + NBLK - 1) / NBLK;
  a.aggr_mean = aggr == RG_REDUCE_MEAN;
  // one workgroup per CU (LDS); at least one per XCD counter.  (A one-wave-per-SIMD variant
  // with the next tile's rows prefetched measured slower and was removed.)
  int blocks = 256;
  const int need = (a.n_blocks + NW2 - 1) / NW2;
  if (blocks > need) blocks = need;
  if (blocks < NXCD) blocks = NXCD;
  RG_ENSURE_LDS(conv_f32_kernel2, DYN_LDS_MAX);
  conv_f32_kernel2<<<blocks, FT2, LDS_BYTES2, st>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
