// Float32 residual_graph_conv_block (gnn_blocks.py:96-113) on the bf16 matrix cores:
// every f32 operand is split EXACTLY into three bf16 terms, v = v0 + v1 + v2 (round to
// nearest even at each step: v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1); the
// residues are exact in f32 and the third term holds the last 8 significant bits), and a
// product a.b is formed from the six terms of weight <= 2,
//     a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0,
// on v_mfma_f32_32x32x16_bf16 with f32 accumulation.  The dropped terms a1 b2 + a2 b1 +
// a2 b2 are below 2^-23 |a b|: each product carries about the error of one f32 rounding,
// the accumulation is f32 -- the arithmetic of the reference's fp32 path, not of bf16.
// Six 32-cycle bf16 MFMAs replace eight 64-cycle f32 MFMAs per 16-deep k-step (2.7x the
// matrix rate of v_mfma_f32_32x32x2_f32, conv_f32.hip).
//
// One layer = an edge launch and a node launch (rg_conv_layer_x3):
//  * edge launch for centred layers (the shipped packing) below 4 Mi nodes: conv_x3_sp_kernel,
//    one wave per SIMD, each wave one contiguous range of whole destinations with an equal
//    share of the edges (the wave table, rg_conv_x3_blocks), walked in 32-edge tiles that may
//    span destinations and software-pipelined across tiles (its own comment below);
//    otherwise conv_x3_kernel, two waves per SIMD: work block = 32 destination nodes and their
//    incoming edges (destination-major CSR); workgroups are persistent and take blocks from
//    one counter per XCD over that XCD's share, stealing from the other XCDs' tails once
//    theirs is empty; the last workgroup out re-zeroes the counters;
//  * per 32-edge tile a wave computes
//        h = act(norm(P[dst] + Q[src] + W_e e))     P | Q = the per-node projections of
//                                                   msg0's x_i / x_j columns (+ b1)
//        m = act(norm(W_2 h + b2))                   (h stays in registers: layer 2's B)
//    then the segmented sum: the message tile is transposed through a wave-private LDS
//    tile (lane = feature) and summed IN EDGE ORDER into a running sum that starts anew
//    at each change of destination (wave-uniform), the reference scatter_add_ order --
//    branch-free, one add and one select per edge; a finished destination's sum is stored
//    as one 256-B row to the aggregate scratch;
//  * node launch (node_x3_kernel): update MLP on cat(x, agg) (agg read back from L2),
//    norm + act + residual -> x_out, and -- when the next layer is also this kernel --
//    the NEXT layer's projections P' | Q' = W'_pq x_out (+ [b1'; 0]) from the same
//    registers, so x_out is never re-read for them.
// The first layer's projections come from rg_conv_proj_x3.
#include <type_traits>

#ifndef RG_X3_SPLIT
#define RG_X3_SPLIT 4  // builtin conversions in the splits: no inline-asm s_nop pads (M: the
                       // one-wave edge launch 0.620 -> 0.606 ms per layer; the chains keep 0)
#endif
#include "x3_common.h"

namespace rg {
namespace convx3 {

using namespace ::rg::x3;

static constexpr int C = 64;      // node / edge / message / output channels
static constexpr int HID = 128;   // msg_mlp_hidden_dim
static constexpr int PQW = 2 * HID;
static constexpr int NBLK = 32;   // destination nodes per work block
static constexpr int NXCD = 8;
static constexpr int CTR_STRIDE = 32;  // block counters one 128-B line apart (per-line atomics)
static constexpr int CTR_BYTES = 2048; // counter area at the front of the workspace
static constexpr int FT = 512;         // edge launch: 8 waves, two per SIMD
static constexpr int NW = FT / 64;
// a wave whose XCD queue drained takes blocks from the others (M: conv -1.1 %; only with >= 2
// blocks per wave: on C5's small blocks the 16-bit conv lost 23 % to stealers saturating the
// other heads)
static constexpr bool STEAL = true;
static constexpr int TR = 16;     // message rows per LDS transposition pass
static constexpr int TS = 68;     // LDS row stride (floats) of the message tile

static constexpr int WE_OFF = 0;                                   // W_e 64 -> 128 (FAST_IN)
static constexpr int W2_OFF = al16(x3_bytes(C, HID));              // W_2 128 -> 64 (FAST_CHAIN)
static constexpr int W_LDS = W2_OFF + al16(x3_bytes(HID, C));
static constexpr int T_BYTES = TR * TS * 4;
static constexpr int LDS_BYTES = W_LDS + NW * T_BYTES;
static_assert(LDS_BYTES <= DYN_LDS_MAX, "conv_x3 LDS");

// P' | Q' of 32 rows held in accumulator layout (xo[2]: features 32m + 8g + 4h + t at
// register 4g + t of tile m) -> pq rows [256] f32; W'_pq packed FAST_CHAIN x3 (K = 64): the
// row's B operand is split once, then four passes of two M-tiles keep the live registers
// bounded
template <typename WSrc>
__device__ __forceinline__ void project_rows(const f32x16 (&xo)[2], const WSrc& W, const float* bias,
                                             float* pq_row, bool valid, int lane) {
  const int h = lane >> 5;
  X3 b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) b[s] = split_acc(xo[s >> 1], s & 1);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x16 acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m] = ld_bias_frag(bias, 2 * q + m, h);
    layer_x3<4, 2, 8, true>(acc, W, 2 * q, [&](int s) { return b[s]; });
    if (valid) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = {acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]};
          *(f32x4*)(pq_row + 64 * q + 32 * m + 8 * g + 4 * h) = v;
        }
    }
  }
}

struct Args {
  const float* x;
  const float* e;
  const float* pq;       // [N][256]: P | Q of this layer
  const int* seg_ptr;
  const int* src;
  const int* dst;
  float* x_out;
  float* pq_out;         // [N][256] the next layer's P | Q, or null
  float* agg;            // [N][64] aggregate scratch
  int* counters;         // NXCD block counters + done counter, CTR_STRIDE apart; zero at launch
  const char* w[3];      // W_e (FAST_IN), W_2 (FAST_CHAIN), W_u (FAST_IN over cat(x, agg)), x3
  const char* wpq;       // the next layer's projection (FAST_CHAIN x3) or null
  const float* mu[3];
  const float* sd[3];
  int ldx, lde, ldo;
  int n_nodes, n_blocks;
  int steal;  // STEAL and >= 2 blocks per wave (small graphs: the heads would saturate)
  int aggr_mean;
  int slabs;  // one-wave edge launch: pieces per wave (x3_slabs)
};

// the rows the node phase of nodes n0 .. n1 - 1 reads first (lane r = node): the segment
// bounds (degree), x[node] and agg[node] in k order (features 16 s + 8 h .. + 7)
struct NodeRows {
  int s0, s1;
  f32x4 xb[4][2], ab[4][2];
};
__device__ __forceinline__ void load_node_rows(const Args& a, int n0, int n1, int lane,
                                               NodeRows& w) {
  const int r = lane & 31, h = lane >> 5;
  const int node = n0 + r;
  const int nrow = node < n1 ? node : n0;
  w.s0 = a.seg_ptr[nrow];
  w.s1 = a.seg_ptr[nrow + 1];
  const float* px = a.x + (size_t)nrow * a.ldx;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    w.xb[s][0] = *(const f32x4*)(px + 16 * s + 8 * h);
    w.xb[s][1] = *(const f32x4*)(px + 16 * s + 8 * h + 4);
  }
  const f32x4* pa = (const f32x4*)(a.agg + (size_t)nrow * C + 8 * h);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    w.ab[s][0] = __builtin_nontemporal_load(pa + 4 * s);
    w.ab[s][1] = __builtin_nontemporal_load(pa + 4 * s + 1);
  }
}

// ---- update MLP on cat(x[node], agg[node]) + residual (gnn_blocks.py:103-109) for the 32
//      nodes n0 .. n1 - 1 (lane r = node) from their loaded rows, then -- when a.pq_out is
//      set -- the next layer's projections from the same registers
template <bool CENT, typename WU, typename WP>
__device__ __forceinline__ void node_compute(const Args& a, const NodeRows& w, int n0, int n1,
                                             const WU& wU, const float* biasU, const WP& wPQ,
                                             const float* biasPQ, float muU, float sdU, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int node = n0 + r;
  const bool nvalid = node < n1;
  const int nrow = nvalid ? node : n0;
  const int deg = nvalid ? w.s1 - w.s0 : 0;
  f32x4 ab[4][2];
  {
    // no incoming edges: PyG leaves the aggregate at zero; mean = sum / max(count, 1)
    const float sc = deg > 0 ? (float)deg : 1.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x4 v = deg > 0 ? w.ab[s][u] : (f32x4){0.f, 0.f, 0.f, 0.f};
        if (a.aggr_mean) v = (f32x4){div_rn(v.x, sc), div_rn(v.y, sc), div_rn(v.z, sc), div_rn(v.w, sc)};
        ab[s][u] = v;
      }
  }
  f32x16 accu[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) accu[m] = ld_bias_frag(biasU, m, h);
  layer_x3<8, 2, 2, true>(accu, wU, 0, [&](int s) {
    return s < 4 ? split8(w.xb[s][0], w.xb[s][1]) : split8(ab[s - 4][0], ab[s - 4][1]);
  });
  norm_leaky<2, CENT>(accu, muU, sdU);
  {
    // the residual x[node] in accumulator order (features 32 m + 8 g + 4 h + t) from the
    // k-order rows already in registers (features 16 s + 8 h + 4 u + t): the value lives in
    // lane half g & 1 at xb[2 m + (g >> 1)][h].  v_permlane32_swap(vdst = xb[s][0],
    // src = xb[s][1]) swaps vdst's lanes 32-63 with src's lanes 0-31, which leaves every
    // lane's even-g value in the new vdst and its odd-g value in the new src -- no reload
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(w.xb[s][0][t]),
                                                         __float_as_uint(w.xb[s][1][t]), false, false);
        const int m = s >> 1, g0 = 2 * (s & 1);
        accu[m][4 * g0 + t] = __fadd_rn(__uint_as_float(sw[0]), accu[m][4 * g0 + t]);
        accu[m][4 * (g0 + 1) + t] = __fadd_rn(__uint_as_float(sw[1]), accu[m][4 * (g0 + 1) + t]);
      }
  }
  if (nvalid) {
    float* po = a.x_out + (size_t)node * a.ldo + 4 * h;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(f32x4*)(po + 32 * m + 8 * g) = (f32x4){accu[m][4 * g], accu[m][4 * g + 1],
                                                 accu[m][4 * g + 2], accu[m][4 * g + 3]};
  }
  if (a.pq_out) project_rows(accu, wPQ, biasPQ, a.pq_out + (size_t)nrow * PQW, nvalid, lane);
}

template <bool CENT>
__global__ __launch_bounds__(FT) void conv_x3_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[4];
  if (threadIdx.x < 2) {
    nrm[2 * threadIdx.x] = *a.mu[threadIdx.x];
    nrm[2 * threadIdx.x + 1] = *a.sd[threadIdx.x];
  }
  stage_lds<FT>(lds + WE_OFF, a.w[0], x3_bytes(C, HID));
  stage_lds<FT>(lds + W2_OFF, a.w[1], x3_bytes(HID, C));
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  float* T = (float*)(lds + W_LDS + wave * T_BYTES);  // [TR][TS] message rows
  const WLds wE{lds + WE_OFF + lane * 16, plane_bytes(C, HID)};
  const WLds w2{lds + W2_OFF + lane * 16, plane_bytes(HID, C)};
  const float* bias2 = (const float*)(lds + W2_OFF + 3 * plane_bytes(HID, C));
  const float mu0 = nrm[0], sd0 = nrm[1], mu1 = nrm[2], sd1 = nrm[3];

  // this XCD's share of the NBLK-node blocks: [xlo(xcd), xlo(xcd + 1))
  const int xcd = blockIdx.x % NXCD;
  auto xlo = [&](int x) { return (int)((long)a.n_blocks * x / NXCD); };
  int blo = xlo(xcd), bhi = xlo(xcd + 1);
  int* ctr = a.counters + CTR_STRIDE * xcd;
  int steal = 0;  // other XCDs' queues visited after this one drained
  for (;;) {
    int bi = 0;
    if (lane == 0) bi = atomicAdd(ctr, 1);
    // readfirstlane, not a shuffle: the block id, its node / edge range and the segment
    // state below are then provably wave-uniform (scalar registers and scalar branches)
    const int blk = blo + __builtin_amdgcn_readfirstlane(bi);
    if (blk >= bhi) {
      if (!STEAL || !a.steal || ++steal >= NXCD) break;
      // this XCD's queue is empty: take the tail of the next one (cold rows, only at the end)
      const int x2 = (xcd + steal) % NXCD;
      blo = xlo(x2);
      bhi = xlo(x2 + 1);
      ctr = a.counters + CTR_STRIDE * x2;
      continue;
    }
    const int n0 = blk * NBLK;
    const int n1 = min(n0 + NBLK, a.n_nodes);
    const int e0 = a.seg_ptr[n0], e1 = a.seg_ptr[n1];
    float run = 0.f;  // lane = feature: running sum of the current destination
    // its aggregate row (wave-uniform); before the block's first destination a dummy row past
    // the last node, so a flush never tests for "no destination yet"
    int crow = a.n_nodes;
    // one tile's gathered rows: P[dst] and Q[src] in accumulator order (features
    // 32m + 8g + 4h .. +3 at [4m + g]), e[edge] in k order (16 s + 8 h .. +3, +4 .. +7 at
    // [2s], [2s + 1])
    struct Rows {
      f32x4 p[16], q[16], e[8];
    };
    auto load_e = [&](int q, Rows& w) {
      const float* pe = a.e + (size_t)q * a.lde + 8 * h;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w.e[2 * i] = *(const f32x4*)(pe + 16 * i);
        w.e[2 * i + 1] = *(const f32x4*)(pe + 16 * i + 4);
      }
    };
    auto load_pq = [&](int dq, int sq, Rows& w) {
      const float* pp = a.pq + (size_t)dq * PQW + 4 * h;
      const float* pqq = a.pq + (size_t)sq * PQW + HID + 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i) w.p[i] = *(const f32x4*)(pp + 8 * i);
#pragma unroll
      for (int i = 0; i < 16; ++i) w.q[i] = *(const f32x4*)(pqq + 8 * i);
    };
    // tile indices (past the block's last edge clamped: a re-read of a cached row)
    auto tile_idx = [&](int t, int& q, int& dq, int& sq) {
      q = min(t + r, e1 - 1);
      dq = a.dst[q];
      sq = a.src[q];
    };
    // the next tile's e rows (streamed from HBM) are loaded right after this tile's layer 2
    // and land behind norm 2 and the segmented sum; its P / Q rows (L2 / MALL) at its start
    // (M: -1.4 .. -2.2 % against all rows at the tile start)
    int p1 = 0, d1 = 0, s1 = 0;
    Rows rw;       // loop-carried: e loaded in the previous tile's second half
    int dcur = 0;  // the destinations of the rows in rw
    int scur = 0;  // their sources
    if (e0 < e1) {
      tile_idx(e0, p1, d1, s1);
      load_e(p1, rw);
      dcur = d1;
      scur = s1;
      tile_idx(e0 + 32, p1, d1, s1);
    }
    for (int t0 = e0; t0 < e1; t0 += 32) {
      const int d = dcur;
      load_pq(d, scur, rw);
      // destination-change mask of this tile's edges (bit j: edge t0 + j starts a segment)
      const int dprev = __shfl_up(d, 1, 64);
      const uint32_t smask =
          (uint32_t)__ballot(r == 0 ? d != crow : d != dprev) &
          (e1 - t0 >= 32 ? 0xffffffffu : ((1u << (e1 - t0)) - 1u));
      // ---- layer 1: h = P[dst] + Q[src] + W_e e
      f32x16 acc1[4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc1[m][4 * g + t] = rw.p[4 * m + g][t] + rw.q[4 * m + g][t];
      layer_x3<4, 4, 4>(acc1, wE, 0, [&](int s) { return split8(rw.e[2 * s], rw.e[2 * s + 1]); });
      // norm 1's statistics now; its scale + LeakyReLU inside layer 2's B operand
      const Pend pn1 = pend_norm_leaky<4, CENT>(acc1, mu0, sd0);
      // ---- layer 2 (B operand = layer 1's accumulators)
      f32x16 acc2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) acc2[m] = ld_bias_frag(bias2, m, h);
      layer_x3<8, 2, 2, 1>(acc2, w2, 0,
                           [&](int s) { return split_acc_pend<1>(acc1[s >> 1], s & 1, pn1); });
      // acc1 and this tile's rows are dead: the next tile's e rows go out now and arrive
      // behind norm 2 and the segmented sum (no registers beyond the rows' own)
      __builtin_amdgcn_sched_barrier(0);
      if (t0 + 32 < e1) {
        load_e(p1, rw);
        scur = s1;
        dcur = d1;
        tile_idx(t0 + 64, p1, d1, s1);
      }
      norm_leaky<2, CENT>(acc2, mu1, sd1);
      // ---- segmented sum in edge order, TR edges per LDS pass: a full pass runs without
      //      bounds checks, each edge one add and one select; a destination change (a set
      //      bit of smask, wave-uniform, ~2.5 per tile) flushes the finished sum to its row
      const int nv = min(32, e1 - t0);
#pragma unroll
      for (int c = 0; c < 32 / TR; ++c) {
        if (TR * c >= nv) break;  // wave-uniform
        if (r / TR == c) {
          float* row = T + (r % TR) * TS + 4 * h;
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *(f32x4*)(row + 32 * m + 8 * g) = (f32x4){acc2[m][4 * g], acc2[m][4 * g + 1],
                                                        acc2[m][4 * g + 2], acc2[m][4 * g + 3]};
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        float v[TR];  // all rows of the pass in flight at once
#pragma unroll
        for (int j = 0; j < TR; ++j) v[j] = T[j * TS + lane];
        // branch-free scan: rv[j] = the running sum after edge TR c + j (a set bit restarts
        // it: rv[j] = v[j]); edges past the block's end add nothing (v = 0, no bit)
        const uint32_t pm = (smask >> (TR * c)) & ((1u << TR) - 1u);
        if (TR * c + TR > nv) {
#pragma unroll
          for (int j = 0; j < TR; ++j) v[j] = TR * c + j < nv ? v[j] : 0.f;
        }
        float rv[TR];
#pragma unroll
        for (int j = 0; j < TR; ++j) {
          const float prev = j == 0 ? run : rv[j - 1];
          rv[j] = ((pm >> j) & 1u) ? v[j] : prev + v[j];
        }
        // the finished sums (~2.5 per tile): at a set bit j the sum before it belongs to the
        // destination that ended there (crow), then crow = the new edge's destination
        for (uint32_t m = pm; m; m &= m - 1) {
          const int j = __builtin_ctz(m);
          float fin = run;
#pragma unroll
          for (int k = 0; k + 1 < TR; ++k) fin = (j == k + 1) ? rv[k] : fin;
          a.agg[(size_t)crow * C + lane] = fin;
          crow = __builtin_amdgcn_readlane(d, TR * c + j);
        }
        run = rv[TR - 1];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    }
    a.agg[(size_t)crow * C + lane] = run;  // (a block without edges: 0 to the dummy row)
  }
  // the last workgroup out re-zeroes the counters for the next launch (stream order)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(a.counters + CTR_STRIDE * NXCD, 1) == (int)gridDim.x - 1) {
#pragma unroll
      for (int i = 0; i <= NXCD; ++i) a.counters[CTR_STRIDE * i] = 0;
    }
  }
}

// The node launch: W_u and W'_pq both staged in LDS (145 KB), one 32-node tile per wave and
// step; the aggregate rows come from the edge launch's scratch.  8 waves per workgroup, two
// per SIMD (M: 12 waves 0.603 vs 0.600-0.603 ms per layer -- its time is the P | Q write
// volume; 16 waves spill).
static constexpr int NU_OFF = 0;
static constexpr int NPQ_OFF = al16(x3_bytes(2 * C, C));
static constexpr int NODE_LDS = NPQ_OFF + al16(x3_bytes(C, PQW));
static constexpr int NFT = 512, NW_NODE = NFT / 64;
static_assert(NODE_LDS <= DYN_LDS_MAX, "node_x3 LDS");
template <bool CENT>
__global__ __launch_bounds__(NFT) void node_x3_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[2];
  if (threadIdx.x == 0) {
    nrm[0] = *a.mu[2];
    nrm[1] = *a.sd[2];
  }
  stage_lds<NFT>(lds + NU_OFF, a.w[2], x3_bytes(2 * C, C));
  stage_lds<NFT>(lds + NPQ_OFF, a.wpq, a.wpq ? x3_bytes(C, PQW) : 0);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const WLds wU{lds + NU_OFF + lane * 16, plane_bytes(2 * C, C)};
  const WLds wPQ{lds + NPQ_OFF + lane * 16, plane_bytes(C, PQW)};
  const float* biasU = (const float*)(lds + NU_OFF + 3 * plane_bytes(2 * C, C));
  const float* biasPQ = (const float*)(lds + NPQ_OFF + 3 * plane_bytes(C, PQW));
  const float muU = nrm[0], sdU = nrm[1];
  const int ntiles = (a.n_nodes + 31) / 32;
  const int stride = gridDim.x * NW_NODE;
  for (int t = blockIdx.x * NW_NODE + wave; t < ntiles; t += stride) {
    NodeRows w;
    const int n0 = 32 * t, n1 = min(32 * t + 32, a.n_nodes);
    load_node_rows(a, n0, n1, lane, w);
    node_compute<CENT>(a, w, n0, n1, wU, biasU, wPQ, biasPQ, muU, sdU, lane);
  }
}

// P | Q = W_pq x + [b1; 0] for dense float32 rows (the first layer's projections):
// W_pq packed FAST_IN x3 (K = 64, N = 256), staged in LDS; one 32-row tile per wave
static constexpr int PFT = 256;
__global__ __launch_bounds__(PFT) void proj_x3_kernel(const float* x, int ldx, int n_nodes,
                                                      const char* wpq, float* pq) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int NB = x3_bytes(C, PQW);
  stage_lds<PFT>(lds, wpq, NB);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const float* bias = (const float*)(lds + 3 * plane_bytes(C, PQW));
  const long ntiles = (n_nodes + 31) / 32;
  for (long t = (long)blockIdx.x * (PFT / 64) + wave; t < ntiles; t += (long)gridDim.x * (PFT / 64)) {
    const long row = t * 32 + r;
    const bool valid = row < n_nodes;
    const float* px = x + (size_t)(valid ? row : 0) * ldx + 8 * h;
    f32x4 xb[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      xb[s][0] = *(const f32x4*)(px + 16 * s);
      xb[s][1] = *(const f32x4*)(px + 16 * s + 4);
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x16 acc[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = ld_bias_frag(bias, 4 * half + m, h);
      layer_x3<4, 4, 8>(acc, WLds{lds + lane * 16, plane_bytes(C, PQW)}, 4 * half, [&](int s) { return split8(xb[s][0], xb[s][1]); });
      if (valid) {
        float* po = pq + (size_t)row * PQW + 128 * half + 4 * h;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *(f32x4*)(po + 32 * m + 8 * g) =
                (f32x4){acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]};
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// The edge launch with one wave per SIMD, software-pipelined (conv_x3_sp_kernel).
//
// conv_x3_kernel runs the whole tile program per wave, two waves per SIMD: its MFMA phases
// (layers 1 and 2) and its vector / memory phases (gathers, e split, norms, segmented sum)
// run back to back in each wave and overlap only as far as the SIMD's two waves happen to
// interleave.  Here each SIMD holds ONE wave that keeps the matrix pipe fed by itself: the
// 192 MFMAs of tile i are cut into sub-chunks of 4 - 12 (a sched_barrier each) and every
// piece of vector / memory work is placed in one of them:
//   * layer 1 of tile i (region A, 96 MFMAs): the split of tile i's e rows (its B operand),
//     the P + Q init of its accumulator tiles 1-3, norm 2 of tile i - 1 and its message
//     transposes, the in-order running sums (8 edges per sub-chunk) and the first four
//     finished destinations (one per sub-chunk), norm 1's partial sums, the loads of tile
//     i + 1 (e rows, Q rows, ring rows) and the indices of tile i + 2;
//   * between the layers (region B): norm 1's scale;
//   * layer 2 of tile i (96 MFMAs): its B operand one k-step ahead (norm 1 + LeakyReLU +
//     split), tile i + 1's ring rows and its first accumulator tile, its first B operand.
// Work: the destination-major CSR cut into one contiguous range of whole destinations per
// wave with equal edge counts (the wave table: rg_conv_x3_blocks, or built into the
// workspace; XCD-major ranks, so an XCD's waves hold one contiguous node range), walked in
// 32-edge tiles that may span destinations -- each destination's messages are still summed
// in CSR order by one wave, the running sum carried from tile to tile.
// Registers: the weight fragments are read from LDS into AGPRs (inline ds_read, the MFMA
// takes its A operand from AGPRs), the rest stays in VGPRs (256 + ~110 AGPRs, no scratch).
// LDS: the W_e and W_2 planes (96 KiB), layer 2's bias, and per wave the message transpose
// tile and a ring of the P rows of its last 8 destinations (a tile's P[dst] is one row per
// destination: 2 rows loaded per tile instead of one row per edge).
typedef float f32x32 __attribute__((ext_vector_type(32)));
namespace sp {
constexpr int FT = 256, NW = FT / 64;
constexpr int PLE = plane_bytes(C, HID), PL2 = plane_bytes(HID, C);  // 16 KiB each
constexpr int OFF_W2 = 3 * PLE;
constexpr int OFF_BUF = OFF_W2 + 3 * PL2;
constexpr int TS2 = 68;            // message transpose: row stride (floats)
constexpr int TBUF = 32 * TS2 * 4;  // per wave: one tile's messages while transposing
constexpr int RING = 8;             // per wave: P rows of the last RING destinations (slot = node & 7)
// ring row stride: a row plus 4 floats, so the rows of two destinations read by one lane group
// of a ds_read_b128 (bank = dword mod 64) start 4 banks apart instead of on the same banks
// (at 128 floats every edge group spanning two destinations was a 2-way conflict)
#ifndef RG_SP_RING_PAD
#define RG_SP_RING_PAD 4
#endif
constexpr int RS = HID + RG_SP_RING_PAD;
constexpr int BUF = TBUF + RING * RS * 4;
constexpr int OFF_BIAS = OFF_BUF + NW * BUF;  // layer 2's bias, accumulator order
constexpr int OFF_NZ = OFF_BIAS + C * 4;       // a row of -0.0: the "P" of a slow-path tile
constexpr int LDS = OFF_NZ + HID * 4;
static_assert(LDS <= 160 * 1024, "conv_x3_sp LDS");
constexpr int GMAX = 256;          // workgroups (one per CU)
constexpr int WMAX = GMAX * NW;    // waves
constexpr int SMAX = 8;            // slabs: the table holds WMAX * SMAX + 1 node boundaries
}  // namespace sp

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }
// one weight fragment LDS -> AGPRs (the MFMA reads its A operand from there); completion is
// not tracked by the compiler: wait_frags before use
template <int OFF>
__device__ __forceinline__ bf16x8_t dsa(uint32_t a) {
  bf16x8_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=a"(r) : "v"(a), "i"(OFF));
  return r;
}
// every LDS read issued so far has landed; the fragments are tied to the wait so no MFMA
// that reads them can be scheduled above it.  The wait itself is the s_waitcnt builtin, not
// inline asm: the compiler's own counter model then knows every older LDS read is done (its
// later waits for its own reads never stall on the untracked fragment reads issued after)
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)
template <int N>
__device__ __forceinline__ void wait_frags(bf16x8_t (&f)[N][3]);
template <>
__device__ __forceinline__ void wait_frags<4>(bf16x8_t (&f)[4][3]) {
  wait_lgkm0();
  asm volatile(""
               : "+a"(f[0][0]), "+a"(f[0][1]), "+a"(f[0][2]), "+a"(f[1][0]), "+a"(f[1][1]),
                 "+a"(f[1][2]), "+a"(f[2][0]), "+a"(f[2][1]), "+a"(f[2][2]), "+a"(f[3][0]),
                 "+a"(f[3][1]), "+a"(f[3][2]));
}
template <>
__device__ __forceinline__ void wait_frags<2>(bf16x8_t (&f)[2][3]) {
  wait_lgkm0();
  asm volatile("" : "+a"(f[0][0]), "+a"(f[0][1]), "+a"(f[0][2]), "+a"(f[1][0]), "+a"(f[1][1]),
                    "+a"(f[1][2]));
}
// layer 1's A fragments of k-step S (W_e FAST_IN x3: K = 64, four M-tiles)
template <int S>
__device__ __forceinline__ void lda1(uint32_t b, bf16x8_t (&f)[4][3]) {
#define RG_SP_L1(M, P) f[M][P] = dsa<P * sp::PLE + (M * 4 + S) * 1024>(b)
  RG_SP_L1(0, 0); RG_SP_L1(0, 1); RG_SP_L1(0, 2); RG_SP_L1(1, 0); RG_SP_L1(1, 1); RG_SP_L1(1, 2);
  RG_SP_L1(2, 0); RG_SP_L1(2, 1); RG_SP_L1(2, 2); RG_SP_L1(3, 0); RG_SP_L1(3, 1); RG_SP_L1(3, 2);
#undef RG_SP_L1
}
// layer 2's A fragments of k-step S (W_2 FAST_CHAIN x3: K = 128, two M-tiles); b = W_2's base
template <int S>
__device__ __forceinline__ void lda2(uint32_t b, bf16x8_t (&f)[2][3]) {
#define RG_SP_L2(M, P) f[M][P] = dsa<P * sp::PL2 + (M * 8 + S) * 1024>(b)
  RG_SP_L2(0, 0); RG_SP_L2(0, 1); RG_SP_L2(0, 2); RG_SP_L2(1, 0); RG_SP_L2(1, 1); RG_SP_L2(1, 2);
#undef RG_SP_L2
}
// the six products of one k-step (weights of term <= 2, small terms first: layer_x3's order)
// for M-tiles [0, MT); MMAJOR: tile by tile (its result complete early), else product-major
template <int MT, bool MMAJOR>
__device__ __forceinline__ void x3_step(f32x16 (&acc)[MT], const bf16x8_t (&A)[MT][3], const X3& b) {
  if constexpr (MMAJOR) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      acc[m] = mf(A[m][2], b.p0, acc[m]);
      acc[m] = mf(A[m][1], b.p1, acc[m]);
      acc[m] = mf(A[m][0], b.p2, acc[m]);
      acc[m] = mf(A[m][1], b.p0, acc[m]);
      acc[m] = mf(A[m][0], b.p1, acc[m]);
      acc[m] = mf(A[m][0], b.p0, acc[m]);
    }
  } else {
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][2], b.p0, acc[m]);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][1], b.p1, acc[m]);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][0], b.p2, acc[m]);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][1], b.p0, acc[m]);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][0], b.p1, acc[m]);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][0], b.p0, acc[m]);
  }
}
// one product of a k-step (x3_step's order: P = 0 .. 5) on every M-tile
template <int P, int MT>
__device__ __forceinline__ void x3_prod(f32x16 (&acc)[MT], const bf16x8_t (&A)[MT][3], const X3& b) {
  constexpr int ia = P == 0 ? 2 : (P == 1 || P == 3) ? 1 : 0;
  constexpr int ib = (P == 0 || P == 3 || P == 5) ? 0 : (P == 1 || P == 4) ? 1 : 2;
  const bf16x8_t bb = ib == 0 ? b.p0 : ib == 1 ? b.p1 : b.p2;
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mf(A[m][ia], bb, acc[m]);
}
// the six products of a k-step on M-tile M alone (the same order per accumulator)
template <int M, int MT>
__device__ __forceinline__ void x3_tile(f32x16 (&acc)[MT], const bf16x8_t (&A)[MT][3], const X3& b) {
  acc[M] = mf(A[M][2], b.p0, acc[M]);
  acc[M] = mf(A[M][1], b.p1, acc[M]);
  acc[M] = mf(A[M][0], b.p2, acc[M]);
  acc[M] = mf(A[M][1], b.p0, acc[M]);
  acc[M] = mf(A[M][0], b.p1, acc[M]);
  acc[M] = mf(A[M][0], b.p0, acc[M]);
}
// keeps a value computed where it stands (IR sinking would otherwise move work whose only
// use lies past a branch into the block after it, out of the sub-chunk it was placed in)
template <int N>
__device__ __forceinline__ void pin(float (&u)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(u[i]));
}
// `n` groups of (one MFMA, v VALU) in program order: the scheduler fills them from the
// region's MFMAs and independent vector work (the region's other instructions float)
template <int N, int V, int M = 0>
__device__ __forceinline__ void interleave() {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
    if (M > 0 && i % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x010, M, 0);  // VMEM
  }
}
__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// sum of squares of one 16-value accumulator tile into eight partial sums (row_inv_std's
// order: partial q & 7)
__device__ __forceinline__ void sq_partial(const f32x16& t, float (&u)[8], bool first) {
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = first ? t[i] * t[i] : fmaf(t[i], t[i], u[i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = fmaf(t[i + 8], t[i + 8], u[i]);
}
// channel_normalization's scale from the partial sums of a CENTRED layer of N features
// (row_inv_std<MT, true>): 0.505 sd / (std + eps), the LeakyReLU prescale folded in
template <int N>
__device__ __forceinline__ Pend finish_norm(const float (&u)[8], float mu, float sd) {
  const float ss = add_xor32(((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7])));
  const float inv =
      __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(ss * (1.f / (float)(N - 1))) + X3_NORM_EPS);
  return Pend{X3_LEAKY_PRE * (sd * inv), X3_LEAKY_PRE * mu};
}

#ifndef RG_CX3_SP_STAMP
#define RG_CX3_SP_STAMP 0  // diagnostic build: per-region s_memtime sums (rg_debug_sp_stamps)
#endif
#if RG_CX3_SP_STAMP
__device__ unsigned long long g_sp_stamp[16];
#define SP_STAMP(i)                                               \
  do {                                                            \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();   \
    st_acc[i] += _n - st_last;                                    \
    st_last = _n;                                                 \
  } while (0)
#else
#define SP_STAMP(i) do {} while (0)
#endif

template <bool CENT>
__global__ __launch_bounds__(sp::FT) __attribute__((amdgpu_waves_per_eu(1, 1)))
void conv_x3_sp_kernel(Args a, const int* __restrict__ wtab) {
  static_assert(CENT, "the one-wave edge launch takes centred layers");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  stage_lds<sp::FT>(lds, a.w[0], 3 * sp::PLE);
  stage_lds<sp::FT>(lds + sp::OFF_W2, a.w[1], 3 * sp::PL2);
  stage_lds<sp::FT>(lds + sp::OFF_BIAS, a.w[1] + 3 * sp::PL2, C * 4);
  if (threadIdx.x < HID) ((float*)(lds + sp::OFF_NZ))[threadIdx.x] = -0.f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int xcd = blockIdx.x % NXCD, slot = blockIdx.x / NXCD;
  const int WX = ((int)gridDim.x / NXCD) * sp::NW;  // waves per XCD
  const int j = slot * sp::NW + wave;
  const int rank = xcd * WX + j;
  // the wave's S pieces (one per slab of its XCD's node range, x3_slabs): piece k = table
  // entry (xcd S + k) WX + j, whole destinations, walked as ONE virtual edge sequence --
  // positions [vbase[k], vbase[k + 1]) are the real edges v + voff[k].  While the XCD's waves
  // work through slab k together, their Q[src] gathers stay inside 1 / S of its nodes (L2).
  const int S = a.slabs;
  typedef int i8v __attribute__((ext_vector_type(sp::SMAX)));
  i8v vbase, voff;  // (vectors, not arrays: the lambdas below capture them)
  int V = 0;
#pragma unroll
  for (int k = 0; k < sp::SMAX; ++k) {
    const int q = (xcd * S + min(k, S - 1)) * WX + j;
    const int e0 = __builtin_amdgcn_readfirstlane(a.seg_ptr[__builtin_amdgcn_readfirstlane(wtab[q])]);
    const int e1 = __builtin_amdgcn_readfirstlane(a.seg_ptr[__builtin_amdgcn_readfirstlane(wtab[q + 1])]);
    vbase[k] = k < S ? V : 0x7fffffff;
    voff[k] = e0 - V;
    V += k < S ? e1 - e0 : 0;
  }
  const int T = (V + 31) >> 5;
  if (T <= 0) return;
  const float mu0 = *a.mu[0], sd0 = *a.sd[0], mu1 = *a.mu[1], sd1 = *a.sd[1];
  const float* bias2 = (const float*)(lds + sp::OFF_BIAS);  // layer 2's bias
  const uint32_t lb = lds_addr(lds);
  const uint32_t aw = lb + lane * 16;  // + the fragment's immediate offset
  const uint32_t aw2 = aw + sp::OFF_W2;
  char* bufp = lds + sp::OFF_BUF + wave * sp::BUF;
  float* Tm = (float*)bufp;  // [32][TS2] message rows while transposing

  // ---- per-tile inputs
  auto edge_of = [&](int t) {  // the real edge of lane r in tile t (past the end: the last)
    const int v = min(32 * t + r, V - 1);
    int off = voff[0];
#pragma unroll
    for (int k = 1; k < sp::SMAX; ++k) off = v >= vbase[k] ? voff[k] : off;
    return v + off;
  };
  // Q[src] rows of a tile in accumulator order (features 32 m + 8 g + 4 h + t at [4 m + g])
  auto load_q_part = [&](int s, f32x4 (&q)[16], int i0, int i1) {
    const float* g = a.pq + (size_t)s * PQW + HID + 4 * h;
#pragma unroll
    for (int i = i0; i < i1; ++i) q[i] = *(const f32x4*)(g + 8 * i);
  };
  auto load_q = [&](int s, f32x4 (&q)[16]) { load_q_part(s, q, 0, 16); };
  auto load_p = [&](int d, f32x4 (&p)[16]) {  // P[dst] in accumulator order (slow path)
    const float* g = a.pq + (size_t)d * PQW + 4 * h;
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = *(const f32x4*)(g + 8 * i);
  };
  auto load_e = [&](int q, f32x4 (&ev)[8]) {  // e[edge] in k order
    const float* g = a.e + (size_t)q * a.lde + 8 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ev[2 * i] = *(const f32x4*)(g + 16 * i);
      ev[2 * i + 1] = *(const f32x4*)(g + 16 * i + 4);
    }
  };
  // P rows through a ring of the wave's last RING destinations in LDS (slot = node & 7): a
  // tile's P[dst] is one row per DESTINATION (~4 per kNN tile), gathered per edge it was 16
  // vector loads per tile.  Before tile t + 1 the rows dl - 3 .. dl of its last destination
  // dl are loaded (two 16-B pieces per lane, half a wave per row); with at most four new
  // destinations per tile the ring then holds every row the tile needs, and the rows it
  // overwrites (dl - 11 .. dl - 8) belong to no tile still to be initialised.  A tile with
  // more new destinations takes its P rows straight from memory (fast = false).
  float* ring = (float*)(bufp + sp::TBUF);
  auto ring_row = [&](int dl, int k) {  // the row loaded by piece k for a last destination dl
    return min(max(dl - 3 + 2 * k + h, 0), a.n_nodes - 1);
  };
  auto ring_load = [&](int dl, f32x4 (&rp)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) rp[k] = *(const f32x4*)(a.pq + (size_t)ring_row(dl, k) * PQW + 4 * r);
  };
  auto ring_store = [&](int dl, const f32x4 (&rp)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) *(f32x4*)(ring + (ring_row(dl, k) & (sp::RING - 1)) * sp::RS + 4 * r) = rp[k];
  };
  // tile accumulator init: Q + P with P from the ring -- or, when the slow path has already
  // added P into q (fast = false: the tile being initialised), from a row of -0.0, which
  // adds nothing (q + -0 = q, signed zeros included), so no ring row of another node
  // reaches the sum
  bool fast = false;  // tile 0's P is in qn
  const float* nzrow = (const float*)(lds + sp::OFF_NZ);
  auto ring_p = [&](int d, int m, f32x4 (&p)[4]) {  // M-tile m of P[d] from the ring
    const float* rp = (fast ? ring + (d & (sp::RING - 1)) * sp::RS : nzrow) + 4 * h + 32 * m;
#pragma unroll
    for (int g = 0; g < 4; ++g) p[g] = *(const f32x4*)(rp + 8 * g);
  };
  auto init_from = [&](const f32x4 (&p)[4], const f32x4 (&q)[16], f32x16& acc, int m) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[4 * g + t] = __fadd_rn(p[g][t], q[4 * m + g][t]);
  };
  auto init_tile = [&](int d, const f32x4 (&q)[16], f32x16& acc, int m) {
    f32x4 p[4];
    ring_p(d, m, p);
    init_from(p, q, acc, m);
  };
  // destination-change mask of a tile (bit j: edge j starts a new destination; edges past
  // the range's end carry no bit); dlast = the destination of the previous tile's last edge
  auto tile_mask = [&](int t, int d, int dlast) {
    const int dprev = __builtin_amdgcn_mov_dpp(d, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const int nv = min(32, V - 32 * t);  // (<= 0 past the range: no bits)
    const uint32_t live = nv >= 32 ? 0xffffffffu : nv <= 0 ? 0u : ((1u << nv) - 1u);
    return (uint32_t)__ballot(r == 0 ? d != dlast : d != dprev) & live;
  };
  // message rows of a tile (lane = edge) -> the buffer; its columns (lane = feature) back
  auto write_msg = [&](const f32x16& m2, int m) {
    float* row = Tm + r * sp::TS2 + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(f32x4*)(row + 32 * m + 8 * g) = (f32x4){m2[4 * g], m2[4 * g + 1], m2[4 * g + 2], m2[4 * g + 3]};
  };
  auto write_msgs = [&](const f32x16 (&m2)[2]) {
    write_msg(m2[0], 0);
    write_msg(m2[1], 1);
  };
  // in-order running sums (lane = feature): rv[j] = the sum after edge j, a set mask bit
  // restarting it (the reference scatter_add_ order of a destination-major CSR); edges
  // [j0, j1) continuing from prev
  // the scan's factor for edge j: keep = 0 at a set mask bit, else 1 -- formed in scalar
  // registers from the wave-uniform mask (bit j of ~mask times the bits of 1.0f), a scalar
  // operand of the scan's fma (compiled from C the select is materialised per lane: one more
  // VALU per edge), and a sub-chunk ahead of its use (a VALU read right behind an inline-asm
  // result costs an s_nop)
  auto keeps = [&](int j0, int j1, uint32_t mask, uint32_t (&kb)[32]) {
#pragma unroll
    for (int j = j0; j < j1; ++j)
      asm("s_bfe_u32 %0, %1, %2\n\ts_mul_i32 %0, %0, 0x3f800000"
          : "=s"(kb[j]) : "s"(~mask), "i"(j | (1 << 16)));
  };
  auto scan_part = [&](int j0, int j1, const float (&cv)[32], const uint32_t (&kb)[32],
                       float& prev, f32x32& rv) {
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      // prev * keep + v: exactly v at a set bit (keep = 0), prev + v otherwise (keep = 1)
      prev = fmaf(prev, __uint_as_float(kb[j]), cv[j]);
      rv[j] = prev;
    }
  };
  auto scan = [&](const float (&cv)[32], uint32_t mask, float run_in, f32x32& rv) {
    float prev = run_in;
    uint32_t kb[32];
    keeps(0, 32, mask, kb);
    scan_part(0, 32, cv, kb, prev, rv);
  };
  // the norm 2 scale + LeakyReLU of one message tile
  auto norm2_apply = [&](f32x16& m2, Pend pn, int i0, int i1) {
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const float y = fmaf(m2[i], pn.ga, pn.gb);
      m2[i] = fmaf(fabsf(y), X3_LEAKY_C, y);
    }
  };
  // the finished destinations of a tile: at a set bit j the sum before edge j belongs to the
  // destination that ended there (crow); then crow = edge j's destination
  auto flush = [&](uint32_t mask, const f32x32& rv, float run_in, int d, int& crow) {
    for (uint32_t m = mask; m; m &= m - 1) {
      const int j = __builtin_ctz(m);
      a.agg[(size_t)crow * C + lane] = j == 0 ? run_in : rv[j - 1];
      crow = __builtin_amdgcn_readlane(d, j);
    }
  };
  // one of them without branches (the first four go through slots, a kNN tile has ~2.5): an
  // unused slot stores to the wave's own dummy row; clears the bit it took from m
  const int dummy = a.n_nodes + 1 + rank;
  auto flush_slot = [&](uint32_t& m, const f32x32& rv, float run_in, int d, int& crow) {
    const bool any = m != 0;
    const int j = __builtin_amdgcn_readfirstlane(any ? __builtin_ctz(m) : 0);
    const int jm = __builtin_amdgcn_readfirstlane(j > 0 ? j - 1 : 0);
    const float v = rv[jm];
    const int row = __builtin_amdgcn_readfirstlane(any ? crow : dummy);
    a.agg[(size_t)row * C + lane] = j == 0 ? run_in : v;
    const int nc = __builtin_amdgcn_readlane(d, j);
    crow = any ? nc : crow;
    m &= m - 1;
  };

  // ---- prologue: the ring zeroed (its stale slots are only ever multiplied by 0), tile
  //      0's inputs (P straight from memory), tile 1's indices
#pragma unroll
  for (int k = 0; k < sp::RING * HID / 256; ++k) {
    const int i = 64 * k + lane;  // piece i % 32 of row i / 32
    *(f32x4*)(ring + (i >> 5) * sp::RS + 4 * (i & 31)) = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  int q_n = edge_of(0);
  const int d0 = a.dst[q_n], s0 = a.src[q_n];
  f32x4 qn[16], en[8], rp[2];
  load_q(s0, qn);
  load_e(q_n, en);
  const int dl0 = __builtin_amdgcn_readlane(d0, 31);
  ring_load(dl0, rp);
  {
    f32x4 pg[16];
    load_p(d0, pg);
#pragma unroll
    for (int i = 0; i < 16; ++i) qn[i] += pg[i];
  }
  ring_store(dl0, rp);
  int q_nn = edge_of(1);
  int d_nn = a.dst[q_nn], s_nn = a.src[q_nn];
  f32x16 acc1[4];
  init_tile(d0, qn, acc1[0], 0);
  f32x4 pr[4];  // the ring rows of the next M-tile to initialise, read one sub-chunk ahead
  ring_p(d0, 1, pr);
  X3 b1 = split8(en[0], en[1]);
  uint32_t mask_c = tile_mask(0, d0, a.n_nodes);
  int d_c = d0;
  // the previous tile's state (none yet: no mask bits, zero messages)
  f32x16 acc2p[2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc2p[m][i] = 0.f;
  uint32_t mask_p = 0;
  int d_p = 0;
  float run = 0.f;       // lane = feature: the running sum carried into the previous tile
  f32x32 rv;             // the previous tile's running sums
  int crow = a.n_nodes;  // the destination row of `run` (a dummy row before the first)
  bf16x8_t A1[2][4][3], A2[2][2][3];
  lda1<0>(aw, A1[0]);
#if RG_CX3_SP_STAMP
  unsigned long long st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

  for (int t = 0; t < T; ++t) {
    SP_STAMP(0);  // (loop back edge)
    f32x4 ev[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ev[i] = en[i];
    float cv[32];
    // Region A = layer 1 of tile t, cut into sub-chunks of 4 - 8 MFMAs with the vector work
    // each one carries placed beside it (a sched_barrier per sub-chunk: left to itself the
    // scheduler bunches the MFMAs of a 24-MFMA region and leaves dependent runs -- the scan,
    // the flushes, the transposes -- without any beside them)
    // ======== A0: k-step 0 tile by tile; beside M-tile m the P + Q init of M-tile m + 1;
    //          the split of k-step 1; norm 2's statistics of tile t - 1
    wait_frags<4>(A1[0]);
    lda1<1>(aw, A1[1]);
    X3 b1n = split8(ev[2], ev[3]);
    init_from(pr, qn, acc1[1], 1);
    ring_p(d_c, 2, pr);
    x3_tile<0>(acc1, A1[0], b1);
    interleave<6, 5>();
    fence();
    float u2[8];
    init_from(pr, qn, acc1[2], 2);
    ring_p(d_c, 3, pr);
    sq_partial(acc2p[0], u2, true);
    x3_tile<1>(acc1, A1[0], b1);
    interleave<6, 6>();
    fence();
    init_from(pr, qn, acc1[3], 3);
    sq_partial(acc2p[1], u2, false);
    x3_tile<2>(acc1, A1[0], b1);
    interleave<6, 6>();
    fence();
    const Pend pn2 = finish_norm<C>(u2, mu1, sd1);
    x3_tile<3>(acc1, A1[0], b1);
    interleave<6, 4>();
    fence();
    SP_STAMP(7);  // A0
    // ======== A1: k-step 1 product by product; the split of k-step 2; tile t - 1: norm 2's
    //          scale + LeakyReLU, its message rows to the buffer and its columns back (one
    //          wave's LDS operations complete in order: no wait between them)
    wait_frags<4>(A1[1]);
    lda1<2>(aw, A1[0]);
    b1 = split8(ev[4], ev[5]);
    norm2_apply(acc2p[0], pn2, 0, 4);
    x3_prod<0>(acc1, A1[1], b1n);
    interleave<4, 5>();
    fence();
    norm2_apply(acc2p[0], pn2, 4, 12);
    x3_prod<1>(acc1, A1[1], b1n);
    interleave<4, 4>();
    fence();
    norm2_apply(acc2p[0], pn2, 12, 16);
    write_msg(acc2p[0], 0);
    x3_prod<2>(acc1, A1[1], b1n);
    interleave<4, 4>();
    fence();
    norm2_apply(acc2p[1], pn2, 0, 8);
    x3_prod<3>(acc1, A1[1], b1n);
    interleave<4, 4>();
    fence();
    norm2_apply(acc2p[1], pn2, 8, 16);
    x3_prod<4>(acc1, A1[1], b1n);
    interleave<4, 4>();
    fence();
    write_msg(acc2p[1], 1);
#pragma unroll
    for (int j = 0; j < 32; ++j) cv[j] = Tm[j * sp::TS2 + lane];
    x3_prod<5>(acc1, A1[1], b1n);
    interleave<4, 2>();
    fence();
    SP_STAMP(8);  // A1
    // ======== A2: k-step 2 product by product; the split of k-step 3; tile t - 1's running
    //          sums; tile t + 1's e rows
    wait_frags<4>(A1[0]);
    lda1<3>(aw, A1[1]);
    b1n = split8(ev[6], ev[7]);
    uint32_t kb[32];
    keeps(0, 16, mask_p, kb);
    x3_prod<0>(acc1, A1[0], b1);
    interleave<4, 3>();
    fence();
    const float run_in = run;
    float prev = run_in;
    keeps(16, 32, mask_p, kb);
    scan_part(0, 8, cv, kb, prev, rv);
    x3_prod<1>(acc1, A1[0], b1);
    interleave<4, 2>();
    fence();
    scan_part(8, 16, cv, kb, prev, rv);
    x3_prod<2>(acc1, A1[0], b1);
    interleave<4, 2>();
    fence();
    scan_part(16, 24, cv, kb, prev, rv);
    x3_prod<3>(acc1, A1[0], b1);
    interleave<4, 2>();
    fence();
    scan_part(24, 32, cv, kb, prev, rv);
    x3_prod<4>(acc1, A1[0], b1);
    interleave<4, 2>();
    fence();
    load_e(q_nn, en);
    x3_prod<5>(acc1, A1[0], b1);
    interleave<4, 0, 2>();
    fence();
    SP_STAMP(9);  // A2
    // ======== A3: k-step 3 tile by tile (norm 1's partial sums follow one tile behind);
    //          tile t - 1's first four finished destinations, one per sub-chunk; tile t + 1's
    //          Q rows and ring rows, the indices of tile t + 2 (a one-wave SIMD pays each
    //          vector-memory instruction's issue in its own stream, so the loads are spread
    //          over the sub-chunks)
    wait_frags<4>(A1[1]);
    lda2<0>(aw2, A2[0]);
    uint32_t mask_rest = mask_p;
    const int dl_c = __builtin_amdgcn_readlane(d_c, 31);   // tile t's last destination
    const int dl_n = __builtin_amdgcn_readlane(d_nn, 31);  // tile t + 1's
    const int q_3 = edge_of(t + 2);
    const int d_3 = a.dst[q_3], s_3 = a.src[q_3];
    load_q_part(s_nn, qn, 0, 6);
    flush_slot(mask_rest, rv, run_in, d_p, crow);
    x3_tile<0>(acc1, A1[1], b1n);
    interleave<6, 4, 2>();
    fence();
    SP_STAMP(10);  // A3.0
    float u1[8];
    load_q_part(s_nn, qn, 6, 12);
    flush_slot(mask_rest, rv, run_in, d_p, crow);
    sq_partial(acc1[0], u1, true);
    x3_tile<1>(acc1, A1[1], b1n);
    interleave<6, 6, 2>();
    fence();
    SP_STAMP(11);  // A3.1
    load_q_part(s_nn, qn, 12, 16);
    ring_load(dl_n, rp);
    flush_slot(mask_rest, rv, run_in, d_p, crow);
    sq_partial(acc1[1], u1, false);
    x3_tile<2>(acc1, A1[1], b1n);
    interleave<6, 6, 2>();
    fence();
    SP_STAMP(14);  // A3.2
    flush_slot(mask_rest, rv, run_in, d_p, crow);
    sq_partial(acc1[2], u1, false);
    pin(u1);
    x3_tile<3>(acc1, A1[1], b1n);
    interleave<6, 6>();
    fence();
    SP_STAMP(1);  // region A
    // the slow path: more than four new destinations in tile t + 1 (never on a kNN graph of
    // degree >= 8): its P rows straight from memory, added into its Q rows
    fast = dl_n - dl_c <= 4;
    if (!fast) {
      asm volatile("");  // a real branch: the compiler would otherwise speculate the loads
      f32x4 pg[16];
      load_p(d_nn, pg);
#pragma unroll
      for (int i = 0; i < 16; ++i) qn[i] += pg[i];
    }
    SP_STAMP(4);  // the slow path
    // ======== B: tile t - 1's remaining finished destinations (a kNN tile has none); norm
    //          1's scale; layer 2's bias
    flush(mask_rest, rv, run_in, d_p, crow);
    run = rv[31];
    sq_partial(acc1[3], u1, false);
    const Pend pn1 = finish_norm<HID>(u1, mu0, sd0);
    f32x16 acc2[2] = {ld_bias_frag(bias2, 0, h), ld_bias_frag(bias2, 1, h)};
    fence();
    SP_STAMP(2);  // region B
    // ======== C: layer 2 of tile t, its B operand one k-step ahead; beside k-step 3 tile
    //          t + 1's ring rows go in (tile t's accumulators were all initialised in A0),
    //          beside k-step 6 its first accumulator tile (acc1[0] is dead after k-step 1's
    //          split; its ring rows read one k-step ahead), beside k-step 7 its first B
    //          operand
    X3 b2 = split_acc_pend<1>(acc1[0], 0, pn1);
    X3 b2n;
    // the next k-step's fragment reads right behind the chunk's first product (two MFMAs):
    // issued later in the chunk they are still in flight at the next chunk's wait
#define RG_SP_C(S, BUFI, NEXT, EXTRA)                                  \
    wait_frags<2>(A2[BUFI]);                                           \
    x3_prod<0>(acc2, A2[BUFI], S % 2 ? b2n : b2);                      \
    lda2<S + 1>(aw2, A2[BUFI ^ 1]);                                     \
    fence();                                                           \
    NEXT = split_acc_pend<1>(acc1[(S + 1) >> 1], (S + 1) & 1, pn1);    \
    EXTRA;                                                             \
    x3_prod<1>(acc2, A2[BUFI], S % 2 ? b2n : b2);                      \
    x3_prod<2>(acc2, A2[BUFI], S % 2 ? b2n : b2);                      \
    x3_prod<3>(acc2, A2[BUFI], S % 2 ? b2n : b2);                      \
    x3_prod<4>(acc2, A2[BUFI], S % 2 ? b2n : b2);                      \
    x3_prod<5>(acc2, A2[BUFI], S % 2 ? b2n : b2);                      \
    interleave<10, 6>();                                               \
    fence();
    RG_SP_C(0, 0, b2n, (void)0)
    RG_SP_C(1, 1, b2, (void)0)
    RG_SP_C(2, 0, b2n, (void)0)
    RG_SP_C(3, 1, b2, ring_store(dl_n, rp))
    RG_SP_C(4, 0, b2n, (void)0)
    RG_SP_C(5, 1, b2, ring_p(d_nn, 0, pr))
    RG_SP_C(6, 0, b2n, init_from(pr, qn, acc1[0], 0))
#undef RG_SP_C
    SP_STAMP(3);  // C0 - C6
    wait_frags<2>(A2[1]);
    x3_prod<0>(acc2, A2[1], b2n);
    lda1<0>(aw, A1[0]);  // the next tile's first layer-1 fragments
    fence();
    b1 = split8(en[0], en[1]);
    x3_prod<1>(acc2, A2[1], b2n);
    x3_prod<2>(acc2, A2[1], b2n);
    x3_prod<3>(acc2, A2[1], b2n);
    x3_prod<4>(acc2, A2[1], b2n);
    x3_prod<5>(acc2, A2[1], b2n);
    ring_p(d_nn, 1, pr);
    const uint32_t mask_n = tile_mask(t + 1, d_nn, dl_c);
    interleave<12, 2>();
    fence();
    SP_STAMP(5);  // C7
    // rotate the pipeline
#pragma unroll
    for (int m = 0; m < 2; ++m) acc2p[m] = acc2[m];
    mask_p = mask_c;
    d_p = d_c;
    mask_c = mask_n;
    d_c = d_nn;
    q_nn = q_3;
    d_nn = d_3;
    s_nn = s_3;
  }
  // ---- epilogue: the last tile's norm 2, running sums and flushes; the final sum goes to
  //      the destination of the range's last edge (edges past it carry no bit and are not
  //      counted: the sum after edge nv - 1)
  wait_lgkm0();
  norm_leaky<2, CENT>(acc2p, mu1, sd1);
  write_msgs(acc2p);
  wait_lgkm0();
  float cv[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) cv[j] = Tm[j * sp::TS2 + lane];
  const float run_in = run;
  scan(cv, mask_p, run_in, rv);
  flush(mask_p, rv, run_in, d_p, crow);
  const int nv = V - 32 * (T - 1);
  a.agg[(size_t)crow * C + lane] = rv[nv - 1];
#if RG_CX3_SP_STAMP
  SP_STAMP(6);  // epilogue
  if (lane == 0) {
    for (int i = 0; i < 16; ++i)
      if (i != 12 && i != 13) atomicAdd(&g_sp_stamp[i], st_acc[i]);
    atomicAdd(&g_sp_stamp[12], (unsigned long long)T);
    atomicAdd(&g_sp_stamp[13], 1ull);
  }
#endif
}

// Node boundaries of the edge launch's pieces: piece w = the destinations [wtab[w], wtab[w + 1]),
// wtab[w] the first node whose CSR start reaches E w / W (equal edge counts; every
// destination whole in one piece); W = waves x slabs
__global__ __launch_bounds__(256) void conv_x3_waves_kernel(const int* __restrict__ seg_ptr,
                                                            int n, int W, int* __restrict__ wtab) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w > W) return;
  const long E = seg_ptr[n];
  const long target = E * w / W;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (seg_ptr[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  wtab[w] = w == W ? n : lo;
}

}  // namespace convx3
}  // namespace rg

using namespace rg;
using namespace rg::convx3;

static size_t x3_agg_bytes(int n_nodes) {
  // the aggregate rows, one dummy row (the flush target before a block's / wave's first
  // destination) and one per wave of the one-wave launch (its unused branch-free flushes)
  return (size_t)((n_nodes > 0 ? n_nodes : 1) + 1 + sp::WMAX) * C * sizeof(float);
}
// workgroups of the one-wave-per-SIMD edge launch (a multiple of the 8 XCDs, one per CU at most)
static int x3_sp_groups(int n_nodes) {
  const int g = (n_nodes / 128 + NXCD - 1) / NXCD * NXCD;
  return g < NXCD ? NXCD : g > sp::GMAX ? sp::GMAX : g;
}
#if RG_CX3_SP_STAMP
// diagnostic builds only (not in radar_gnn.h): read and clear the region sums
extern "C" int rg_debug_sp_stamps(unsigned long long* out_host) {
  RG_CHECK_HIP(hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_sp_stamp), sizeof(g_sp_stamp)));
  static const unsigned long long z[16] = {0};
  RG_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sp_stamp), z, sizeof(z)));
  return RG_OK;
}
#endif
extern "C" size_t rg_conv_layer_x3_workspace_size(int n_nodes) {
  static_assert((CTR_STRIDE * NXCD + 1) * sizeof(int) <= CTR_BYTES, "counter area");
  // + the wave table when the layer has to build it (no rg_conv_x3_blocks table)
  return CTR_BYTES + x3_agg_bytes(n_nodes) + (size_t)(sp::WMAX * sp::SMAX + 1) * sizeof(int);
}

extern "C" int rg_conv_proj_x3(const rg_layer* pq, const float* x, int ldx, int n_nodes,
                               float* pq_out, void* stream) {
  RG_REQUIRE(pq && pq->in_dim == C && pq->out_dim == PQW && !pq->norm_mu && pq->act == RG_ACT_NONE,
             RG_ERR_UNSUPPORTED, "rg_conv_proj_x3: expects the 64 -> 256 projection");
  RG_REQUIRE(ldx % 4 == 0, RG_ERR_UNSUPPORTED, "rg_conv_proj_x3: row stride must be a multiple of 4");
  if (n_nodes <= 0) return RG_OK;
  constexpr int lds = x3_bytes(C, PQW);
  RG_ENSURE_LDS(proj_x3_kernel, lds);
  const long tiles = (n_nodes + 31) / 32;
  long blocks = (tiles + 3) / 4;
  if (blocks > 256) blocks = 256;
  proj_x3_kernel<<<blocks, PFT, lds, (hipStream_t)stream>>>(x, ldx, n_nodes,
                                                           (const char*)pq->w_packed, pq_out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_conv_x3_blocks_bytes(int n_nodes) {
  (void)n_nodes;
  return (size_t)(sp::WMAX * sp::SMAX + 1) * sizeof(int);
}

// slabs per XCD node range for the one-wave launch: ~RG_CX3_SLAB_NODES nodes each, at most
// sp::SMAX (M: 4 slabs of 6000 nodes, 3 MB of Q rows, against the XCD's 4 MB L2; the
// launch's fetched bytes 1.77 -> 0.96 GB at 8 slabs, its time unchanged,
// profiles/r06_slab_ab.log, r06_slab_fetch.json)
#ifndef RG_CX3_SLAB_NODES
#define RG_CX3_SLAB_NODES 6000
#endif
static int x3_slabs(int n_nodes) {
  const int s = (n_nodes / NXCD + RG_CX3_SLAB_NODES / 2) / RG_CX3_SLAB_NODES;
  return s < 1 ? 1 : s > sp::SMAX ? sp::SMAX : s;
}
static int x3_wave_table(const int* seg_ptr, int n_nodes, int* table, void* stream) {
  const int W = x3_sp_groups(n_nodes) * sp::NW * x3_slabs(n_nodes);
  conv_x3_waves_kernel<<<(W + 256) / 256, 256, 0, (hipStream_t)stream>>>(seg_ptr, n_nodes, W, table);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_conv_x3_blocks(const int* seg_ptr, int n_nodes, int* table, void* stream) {
  RG_REQUIRE(seg_ptr && table && n_nodes >= 1, RG_ERR_ARG, "rg_conv_x3_blocks: bad argument");
  return x3_wave_table(seg_ptr, n_nodes, table, stream);
}

static int conv_layer_x3(const rg_layer* layers, const rg_layer* next_pq, int aggr, const float* x,
                         int ldx, const float* e, int lde, const float* pq, const int* seg_ptr,
                         const int* src, const int* dst, int n_nodes, float* x_out, int ld_out,
                         float* pq_out, const int* table, void* workspace, size_t workspace_bytes,
                         void* stream);

extern "C" int rg_conv_layer_x3(const rg_layer* layers, const rg_layer* next_pq, int aggr,
                                const float* x, int ldx, const float* e, int lde, const float* pq,
                                const int* seg_ptr, const int* src, const int* dst, int n_nodes,
                                float* x_out, int ld_out, float* pq_out, void* workspace,
                                size_t workspace_bytes, void* stream) {
  return conv_layer_x3(layers, next_pq, aggr, x, ldx, e, lde, pq, seg_ptr, src, dst, n_nodes,
                       x_out, ld_out, pq_out, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int rg_conv_layer_x3_blocks(const rg_layer* layers, const rg_layer* next_pq, int aggr,
                                       const float* x, int ldx, const float* e, int lde,
                                       const float* pq, const int* seg_ptr, const int* src,
                                       const int* dst, int n_nodes, float* x_out, int ld_out,
                                       float* pq_out, const int* table, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  RG_REQUIRE(table, RG_ERR_ARG, "rg_conv_layer_x3_blocks: table from rg_conv_x3_blocks");
  return conv_layer_x3(layers, next_pq, aggr, x, ldx, e, lde, pq, seg_ptr, src, dst, n_nodes,
                       x_out, ld_out, pq_out, table, workspace, workspace_bytes, stream);
}

static int conv_layer_x3(const rg_layer* layers, const rg_layer* next_pq, int aggr,
                         const float* x, int ldx, const float* e, int lde, const float* pq,
                         const int* seg_ptr, const int* src, const int* dst, int n_nodes,
                         float* x_out, int ld_out, float* pq_out, const int* table,
                         void* workspace, size_t workspace_bytes, void* stream) {
  const rg_layer& m0 = layers[0];
  const rg_layer& m1 = layers[1];
  const rg_layer& u = layers[2];
  if (!(m0.in_dim == C && m0.out_dim == HID && m1.in_dim == HID && m1.out_dim == C &&
        u.in_dim == 2 * C && u.out_dim == C))
    return RG_ERR_UNSUPPORTED;
  if (aggr != RG_REDUCE_SUM && aggr != RG_REDUCE_MEAN) return RG_ERR_UNSUPPORTED;
  if (!m0.norm_mu || !m1.norm_mu || !u.norm_mu) return RG_ERR_UNSUPPORTED;
  if (m0.act != ACT_LEAKY || m1.act != ACT_LEAKY || u.act != ACT_LEAKY) return RG_ERR_UNSUPPORTED;
  // centred (RG_LAYER_CENTERED) on all three normalised layers -- and then on the
  // projections, which are msg0's other columns -- or on none
  const int cent = m0.flags & m1.flags & u.flags & RG_LAYER_CENTERED;
  if (!cent && ((m0.flags | m1.flags | u.flags) & RG_LAYER_CENTERED)) return RG_ERR_UNSUPPORTED;
  RG_REQUIRE(!next_pq == !pq_out, RG_ERR_ARG, "rg_conv_layer_x3: next_pq and pq_out go together");
  RG_REQUIRE(!next_pq || (next_pq->in_dim == C && next_pq->out_dim == PQW && !next_pq->norm_mu &&
                          next_pq->act == RG_ACT_NONE),
             RG_ERR_UNSUPPORTED, "rg_conv_layer_x3: next_pq must be the 64 -> 256 projection");
  RG_REQUIRE(ldx % 4 == 0 && ld_out % 4 == 0 && lde % 4 == 0, RG_ERR_UNSUPPORTED,
             "rg_conv_layer_x3: row strides must be multiples of 4");
  RG_REQUIRE(x != x_out, RG_ERR_ARG, "rg_conv_layer_x3: x_out must not alias x");
  RG_REQUIRE(!pq_out || pq_out != pq, RG_ERR_ARG, "rg_conv_layer_x3: pq_out must not alias pq");
  RG_REQUIRE(workspace_bytes >= rg_conv_layer_x3_workspace_size(n_nodes), RG_ERR_ARG,
             "rg_conv_layer_x3: workspace too small");
  if (n_nodes <= 0) return RG_OK;
  Args a;
  memset(&a, 0, sizeof(a));
  a.x = x;
  a.e = e;
  a.pq = pq;
  a.seg_ptr = seg_ptr;
  a.src = src;
  a.dst = dst;
  a.x_out = x_out;
  a.pq_out = pq_out;
  a.counters = (int*)workspace;
  a.agg = (float*)((char*)workspace + CTR_BYTES);
  a.w[0] = (const char*)m0.w_packed;
  a.w[1] = (const char*)m1.w_packed;
  a.w[2] = (const char*)u.w_packed;
  a.wpq = next_pq ? (const char*)next_pq->w_packed : nullptr;
  const rg_layer* ls[3] = {&m0, &m1, &u};
  for (int l = 0; l < 3; ++l) {
    a.mu[l] = ls[l]->norm_mu;
    a.sd[l] = ls[l]->norm_std;
  }
  a.ldx = ldx;
  a.lde = lde;
  a.ldo = ld_out;
  a.n_nodes = n_nodes;
  a.n_blocks = (n_nodes + NBLK - 1) / NBLK;
  a.aggr_mean = aggr == RG_REDUCE_MEAN;
  // (the one-wave launch addresses Q rows with 32-bit byte offsets: < 4 Mi nodes)
  if (cent && n_nodes < (1 << 22)) {
    const int* wtab = table;
    if (!wtab) {  // no per-graph table: build the wave ranges into the workspace
      int* ws_tab = (int*)((char*)workspace + CTR_BYTES + x3_agg_bytes(n_nodes));
      const int rc = x3_wave_table(seg_ptr, n_nodes, ws_tab, stream);
      if (rc != RG_OK) return rc;
      wtab = ws_tab;
    }
    a.slabs = x3_slabs(n_nodes);
    auto edge = conv_x3_sp_kernel<true>;
    RG_ENSURE_LDS(edge, sp::LDS);
    edge<<<x3_sp_groups(n_nodes), sp::FT, sp::LDS, (hipStream_t)stream>>>(a, wtab);
    RG_LAUNCH_CHECK();
  } else {  // (a wave table, if given, is not used: NBLK-node blocks)
  int blocks = 256;  // one workgroup per CU (LDS); a multiple of the 8 XCDs
  const int need = (a.n_blocks + NW - 1) / NW;
  if (blocks > need) blocks = (need + NXCD - 1) / NXCD * NXCD;
  if (blocks < NXCD) blocks = NXCD;
  a.steal = a.n_blocks >= 2 * blocks * NW;
  auto edge = cent ? conv_x3_kernel<true> : conv_x3_kernel<false>;
  RG_ENSURE_LDS(edge, LDS_BYTES);
  edge<<<blocks, FT, LDS_BYTES, (hipStream_t)stream>>>(a);
  RG_LAUNCH_CHECK_ZERO(a.counters, CTR_BYTES, stream);
  }
  auto node = cent ? node_x3_kernel<true> : node_x3_kernel<false>;
  RG_ENSURE_LDS(node, NODE_LDS);
  const int tiles = (n_nodes + 31) / 32;
  const int nblk = (tiles + NW_NODE - 1) / NW_NODE < 256 ? (tiles + NW_NODE - 1) / NW_NODE : 256;
  node<<<nblk, NFT, NODE_LDS, (hipStream_t)stream>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
