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
//  * work block = 32 destination nodes and their incoming edges (destination-major CSR; with
//    the block table, 8-node blocks for the launch tail); workgroups are persistent and take
//    blocks from one counter per XCD over that XCD's share, stealing from the other XCDs'
//    tails once theirs is empty; the last workgroup out re-zeroes the counters;
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

#include "x3_common.h"

namespace rg {
namespace convx3 {

using namespace ::rg::x3;

static constexpr int C = 64;      // node / edge / message / output channels
static constexpr int HID = 128;   // msg_mlp_hidden_dim
static constexpr int PQW = 2 * HID;
static constexpr int NBLK = 32;   // destination nodes per work block
static constexpr int NXCD = 8;
static constexpr int TBL_HDR = 16;  // block table: NXCD + 1 block offsets, padded, then pairs
static constexpr int TAIL_PCT = 15; // percent of each XCD's nodes cut into TAILN-node blocks (launch tail)
static constexpr int TAILN = 8;
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
  const int* table;      // optional work-block table (rg_conv_x3_blocks), else NBLK-node runs
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

  // with a block table: this XCD's blocks are table[xcd] .. table[xcd + 1] of the (first,
  // end) node pairs at table + TBL_HDR, largest first
  const int xcd = blockIdx.x % NXCD;
  auto xlo = [&](int x) { return a.table ? a.table[x] : (int)((long)a.n_blocks * x / NXCD); };
  int blo = xlo(xcd), bhi = xlo(xcd + 1);
  const int* pairs = a.table ? a.table + TBL_HDR : nullptr;
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
    const int n0 = pairs ? pairs[2 * blk] : blk * NBLK;
    const int n1 = pairs ? pairs[2 * blk + 1] : min(n0 + NBLK, a.n_nodes);
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

}  // namespace convx3
}  // namespace rg

using namespace rg;
using namespace rg::convx3;

extern "C" size_t rg_conv_layer_x3_workspace_size(int n_nodes) {
  static_assert((CTR_STRIDE * NXCD + 1) * sizeof(int) <= CTR_BYTES, "counter area");
  // the aggregate rows and one dummy row (the edge launch's flush target before a block's
  // first destination)
  return CTR_BYTES + (size_t)((n_nodes > 0 ? n_nodes : 1) + 1) * C * sizeof(float);
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

// Work blocks of the edge launch for one graph: XCD x's share of the nodes
// [N x / 8, N (x + 1) / 8) -- its frames' rows in one L2 -- as 32-node runs over the first
// (100 - TAIL_PCT) % and TAILN-node runs over the rest, all ordered by edge tiles, largest
// first: the waves take the big blocks first and end on the small ones, so the launch tail
// (waves idle until the last block of their workgroup ends: 14 % of the wave time with
// 32-node blocks only, M) shrinks to a few tiles.  Order and size change no result: each
// destination's messages are summed in CSR order within one block.
__host__ __device__ inline void x3_share(int n, int x, int& a0, int& sp, int& b0) {
  a0 = (int)((long)n * x / NXCD);
  b0 = (int)((long)n * (x + 1) / NXCD);
  sp = a0 + (int)((long)(b0 - a0) * (100 - TAIL_PCT) / 100 / NBLK) * NBLK;
}
__host__ __device__ inline int x3_share_blocks(int n, int x) {
  int a0, sp, b0;
  x3_share(n, x, a0, sp, b0);
  return (sp - a0 + NBLK - 1) / NBLK + (b0 - sp + TAILN - 1) / TAILN;
}
// order: 0 = every block by edge tiles, largest first;
// 1 = the 32-node blocks in node order (consecutive blocks share their frame's rows in
// L2), then the tail blocks largest first; 2 = every block in node order
__global__ __launch_bounds__(256) void conv_x3_blocks_kernel(const int* __restrict__ seg_ptr,
                                                             int n, int* __restrict__ table,
                                                             int order) {
  constexpr int NBIN = 64;
  __shared__ int hist[NBIN];
  const int x = blockIdx.x;
  int off = 0;
  for (int xx = 0; xx < x; ++xx) off += x3_share_blocks(n, xx);
  int a0, sp, b0;
  x3_share(n, x, a0, sp, b0);
  const int nmain = (sp - a0 + NBLK - 1) / NBLK;
  const int m = nmain + (b0 - sp + TAILN - 1) / TAILN;
  if (threadIdx.x == 0) {
    table[x] = off;
    if (x == NXCD - 1) table[NXCD] = off + m;
  }
  if (threadIdx.x < NBIN) hist[threadIdx.x] = 0;
  __syncthreads();
  auto block = [&](int i, int& n0, int& n1) {
    if (i < nmain) {
      n0 = a0 + NBLK * i;
      n1 = min(n0 + NBLK, sp);
    } else {
      n0 = sp + TAILN * (i - nmain);
      n1 = min(n0 + TAILN, b0);
    }
    const int t = (seg_ptr[n1] - seg_ptr[n0] + 31) / 32;
    return NBIN - 1 - min(t, NBIN - 1);  // bin 0 = the most tiles
  };
  const int sorted0 = order == 0 ? 0 : order == 1 ? nmain : m;  // blocks [sorted0, m) sorted
  for (int i = sorted0 + threadIdx.x; i < m; i += blockDim.x) {
    int n0, n1;
    atomicAdd(&hist[block(i, n0, n1)], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NBIN; ++i) {
      const int c = hist[i];
      hist[i] = acc;
      acc += c;
    }
  }
  __syncthreads();
  int* pairs = table + TBL_HDR;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    int n0, n1;
    const int bin = block(i, n0, n1);
    const int pos = off + (i < sorted0 ? i : sorted0 + atomicAdd(&hist[bin], 1));
    pairs[2 * pos] = n0;
    pairs[2 * pos + 1] = n1;
  }
}

static int x3_total_blocks(int n) {
  int t = 0;
  for (int x = 0; x < NXCD; ++x) t += x3_share_blocks(n, x);
  return t;
}

extern "C" size_t rg_conv_x3_blocks_bytes(int n_nodes) {
  return (size_t)(TBL_HDR + 2 * x3_total_blocks(n_nodes > 0 ? n_nodes : 1)) * sizeof(int);
}

extern "C" int rg_conv_x3_blocks(const int* seg_ptr, int n_nodes, int* table, void* stream) {
  RG_REQUIRE(seg_ptr && table && n_nodes >= 1, RG_ERR_ARG, "rg_conv_x3_blocks: bad argument");
  conv_x3_blocks_kernel<<<NXCD, 256, 0, (hipStream_t)stream>>>(seg_ptr, n_nodes, table, 0);
  RG_LAUNCH_CHECK();
  return RG_OK;
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
  a.n_blocks = table ? x3_total_blocks(n_nodes) : (n_nodes + NBLK - 1) / NBLK;
  a.table = table;
  a.aggr_mean = aggr == RG_REDUCE_MEAN;
  int blocks = 256;  // one workgroup per CU (LDS); a multiple of the 8 XCDs
  const int need = (a.n_blocks + NW - 1) / NW;
  if (blocks > need) blocks = (need + NXCD - 1) / NXCD * NXCD;
  if (blocks < NXCD) blocks = NXCD;
  a.steal = a.n_blocks >= 2 * blocks * NW;
  auto edge = cent ? conv_x3_kernel<true> : conv_x3_kernel<false>;
  RG_ENSURE_LDS(edge, LDS_BYTES);
  edge<<<blocks, FT, LDS_BYTES, (hipStream_t)stream>>>(a);
  RG_LAUNCH_CHECK_ZERO(a.counters, CTR_BYTES, stream);
  auto node = cent ? node_x3_kernel<true> : node_x3_kernel<false>;
  RG_ENSURE_LDS(node, NODE_LDS);
  const int tiles = (n_nodes + 31) / 32;
  const int nblk = (tiles + NW_NODE - 1) / NW_NODE < 256 ? (tiles + NW_NODE - 1) / NW_NODE : 256;
  node<<<nblk, NFT, NODE_LDS, (hipStream_t)stream>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
