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
// One layer = an edge launch and a node launch (rg_conv_layer_x3; RG_CX3_NODE_KERNEL = 0 runs
// the node phase at each block's end inside the edge launch instead):
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
#ifndef RG_CX3_PQNT
#define RG_CX3_PQNT 0  // non-temporal P | Q stores (M: +3 %, rejected)
#endif
#ifndef RG_CX3_NBLK
#define RG_CX3_NBLK 32
#endif
#ifndef RG_CX3_DB1
#define RG_CX3_DB1 0  // double-buffered A fragments in message layer 1 / layer 2
#endif
#ifndef RG_CX3_DB2
#define RG_CX3_DB2 1
#endif
#ifndef RG_CX3_STATIC
#define RG_CX3_STATIC 0  // static edge-balanced wave ranges instead of per-XCD block counters
                         // (measured: no gain, 0.642 vs 0.637 ms per M layer)
#endif
#ifndef RG_CX3_PRIO
#define RG_CX3_PRIO 0
#endif
#ifndef RG_CX3_STAGGER
#define RG_CX3_STAGGER 0  // waves 4-7 (each SIMD's second wave) start after N x s_sleep(127)
                          // (~8k cycles each): the two waves of a SIMD run the same tile
                          // program, and in lockstep their MFMA phases collide while their
                          // gather / norm phases leave the matrix pipe idle
#endif
static constexpr int NBLK = RG_CX3_NBLK;   // destination nodes per work block
#ifndef RG_CX3_PP
#define RG_CX3_PP 0  // 1 / 2: the edge launch as a two-group ping-pong (conv_x3_pp_kernel, barrier / token; measured slower)
#endif
#ifndef RG_CX3_PP_PQ
#define RG_CX3_PP_PQ 2
#endif
#ifndef RG_CX3_PP_PRIO
#define RG_CX3_PP_PRIO 0
#endif
#ifndef RG_CX3_PP_PF
#define RG_CX3_PP_PF 1  // dequeue the next block ahead (conv_x3_pp_kernel prefetch)
#endif
#ifndef RG_CX3_PP_N2M
#define RG_CX3_PP_N2M 0  // 1: norm 2 at the end of the M phase instead of the start of V
#endif
#ifndef RG_CX3_STAMP
#define RG_CX3_STAMP 0  // diagnostic build: per-phase s_memtime sums in g_cx3_stamp
#endif
#if RG_CX3_STAMP
__device__ unsigned long long g_cx3_stamp[16];
#define STAMP(i)                                            \
  do {                                                      \
    const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += _n - st_last;                              \
    st_last = _n;                                           \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#endif
static constexpr int NXCD = 8;
static constexpr int TBL_HDR = 16;  // block table: NXCD + 1 block offsets, padded, then pairs
#ifndef RG_CX3_TAIL
#define RG_CX3_TAIL 15  // percent of each XCD's nodes cut into TAILN-node blocks (launch tail)
#endif
#ifndef RG_CX3_TAILN
#define RG_CX3_TAILN 8
#endif
static constexpr int TAILN = RG_CX3_TAILN;
static constexpr int CTR_STRIDE = 32;  // block counters one 128-B line apart (per-line atomics)
static constexpr int CTR_BYTES = 2048; // counter area at the front of the workspace
#ifndef RG_CX3_FT
#define RG_CX3_FT 512
#endif
#ifndef RG_CX3_RPF
#define RG_CX3_RPF 0  // the next tile's P / Q / e rows prefetched (160 registers: one wave
                      // per SIMD, RG_CX3_FT = 256)
#endif
static constexpr int FT = RG_CX3_FT;  // 512: two waves per SIMD
static constexpr int NW = FT / 64;
#ifndef RG_CX3_JIT
#define RG_CX3_JIT 1  // message layer 1's norm scale + act applied in layer 2's B operand
#endif
#ifndef RG_CX3_NODE_PF
#define RG_CX3_NODE_PF 0  // 1: node launch loads the next tile's rows while a tile computes (M: slower, 256 VGPRs)
#endif
#ifndef RG_CX3_NODE_KERNEL
#define RG_CX3_NODE_KERNEL 1  // the update / projection phase as a second launch (LDS weights)
#endif
#ifndef RG_CX3_LATE
#define RG_CX3_LATE 4  // 4: the next tile's e rows (streamed from HBM, 32 registers) loaded right after this
                      // tile's layer 2, P / Q rows (L2 / MALL) at the tile start (M: -1.4..-2.2 %);
                      // 1: all its rows there (M: 0.62 -> 0.84 ms, spills); 0: all at the tile start
#endif
#ifndef RG_CX3_STEAL
#define RG_CX3_STEAL 1  // a wave whose XCD queue drained takes blocks from the others (M: conv
                       // -1.1 %; only with >= 2 blocks per wave: on C5's small blocks the
                       // 16-bit conv lost 23 % to stealers saturating the other heads)
#endif
#ifndef RG_CX3_ENT
#define RG_CX3_ENT 0  // 1: non-temporal e loads (M: +2.7 %, rejected)
#endif
#ifndef RG_CX3_MO
#define RG_CX3_MO 0  // bit 0: message layer 1, bit 1: layer 2 issued M-tile by M-tile (layer_x3_mo:
                     // 24 registers of A fragments instead of 48; bit-identical)
#endif
#ifndef RG_CX3_RESREG
#define RG_CX3_RESREG 1  // the update's residual x[node] from the rows in registers
                         // (v_permlane32_swap) instead of a second load of x (M: flat, -0.3 %)
#endif
#ifndef RG_CX3_QLATE
#define RG_CX3_QLATE 0  // 1: layer 1 accumulates onto P[dst] only and Q[src] (the random gather
                        // from L2 / MALL) is added after its MFMAs, so the gather's latency
                        // sits behind the 96 layer-1 MFMAs instead of in front of them
#endif
#ifndef RG_CX3_WU_LDS
#define RG_CX3_WU_LDS 0  // W_u staged in LDS too, 4-row passes (M: 0.650 vs 0.638 ms/layer, slower)
#endif
static constexpr int TR = RG_CX3_WU_LDS ? 4 : 16;  // message rows per LDS transposition pass
static constexpr int TS = 68;     // LDS row stride (floats) of the message tile
#ifndef RG_CX3_EXP
#define RG_CX3_EXP 0  // timing experiments only (wrong results): 1 no tile norm epilogues,
                      // 2 no segmented sum, 3 no P / Q gathers, 4 no B splits (one plane
                      // copied), 5 no tile MFMAs, 6 no update / projection phase,
                      // 7 no P | Q stores, 8 no P gathers (Q[src] only), 9 no P gathers and
                      // no P half of the node launch's projection (the bound of computing P
                      // per block inside the edge launch)
#endif

static constexpr int WE_OFF = 0;                                   // W_e 64 -> 128 (FAST_IN)
static constexpr int W2_OFF = al16(x3_bytes(C, HID));              // W_2 128 -> 64 (FAST_CHAIN)
static constexpr int WU_OFF = W2_OFF + al16(x3_bytes(HID, C));   // W_u (FAST_IN), optional
static constexpr int W_LDS = WU_OFF + (RG_CX3_WU_LDS ? al16(x3_bytes(2 * C, C)) : 0);
static constexpr int T_BYTES = TR * TS * 4;
static constexpr int LDS_BYTES = W_LDS + NW * T_BYTES;
static_assert(LDS_BYTES <= DYN_LDS_MAX, "conv_x3 LDS");

// timing experiments: keep a split alive without its MFMAs
__device__ __forceinline__ float xor_first(const X3& b) {
  return __uint_as_float(__builtin_bit_cast(u32x4, b.p0)[0] ^ __builtin_bit_cast(u32x4, b.p1)[0] ^
                         __builtin_bit_cast(u32x4, b.p2)[0]);
}
// P' | Q' of 32 rows held in accumulator layout (xo[2]: features 32m + 8g + 4h + t at
// register 4g + t of tile m) -> pq rows [256] f32; W'_pq packed FAST_CHAIN x3 (K = 64), read
// from global memory (L2): the row's B operand is split once, then four passes of two
// M-tiles keep the live registers bounded
template <typename WSrc>
__device__ __forceinline__ void project_rows(const f32x16 (&xo)[2], const WSrc& W, const float* bias,
                                             float* pq_row, bool valid, int lane) {
  const int h = lane >> 5;
  X3 b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) b[s] = split_acc(xo[s >> 1], s & 1);
#pragma unroll
  for (int q = RG_CX3_EXP == 9 ? 2 : 0; q < 4; ++q) {
    f32x16 acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m] = ld_bias_frag(bias, 2 * q + m, h);
    layer_x3<4, 2, 8, true>(acc, W, 2 * q, [&](int s) { return b[s]; });
    if (valid && RG_CX3_EXP != 7) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = {acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]};
#if RG_CX3_PQNT
          __builtin_nontemporal_store(v, (f32x4*)(pq_row + 64 * q + 32 * m + 8 * g + 4 * h));
#else
          *(f32x4*)(pq_row + 64 * q + 32 * m + 8 * g + 4 * h) = v;
#endif
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
  int steal;  // RG_CX3_STEAL and >= 2 blocks per wave (small graphs: the heads would saturate)
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
#if RG_CX3_RESREG
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
#else
  {
    const float* pxr = a.x + (size_t)nrow * a.ldx + 4 * h;  // x[node] in accumulator order
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 xr = *(const f32x4*)(pxr + 32 * m + 8 * g);
        accu[m][4 * g + 0] = __fadd_rn(xr.x, accu[m][4 * g + 0]);
        accu[m][4 * g + 1] = __fadd_rn(xr.y, accu[m][4 * g + 1]);
        accu[m][4 * g + 2] = __fadd_rn(xr.z, accu[m][4 * g + 2]);
        accu[m][4 * g + 3] = __fadd_rn(xr.w, accu[m][4 * g + 3]);
      }
  }
#endif
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

template <bool CENT, typename WU, typename WP>
__device__ __forceinline__ void node_update(const Args& a, int n0, int n1, const WU& wU,
                                            const float* biasU, const WP& wPQ,
                                            const float* biasPQ, float muU, float sdU, int lane) {
  NodeRows w;
  load_node_rows(a, n0, n1, lane, w);
  node_compute<CENT>(a, w, n0, n1, wU, biasU, wPQ, biasPQ, muU, sdU, lane);
}

template <bool CENT, bool NODE>
__global__ __launch_bounds__(FT) void conv_x3_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[6];
  if (threadIdx.x < 3) {
    nrm[2 * threadIdx.x] = *a.mu[threadIdx.x];
    nrm[2 * threadIdx.x + 1] = *a.sd[threadIdx.x];
  }
  {
    const int nb[3] = {x3_bytes(C, HID), x3_bytes(HID, C), x3_bytes(2 * C, C)};
    const int off[3] = {WE_OFF, W2_OFF, WU_OFF};
#pragma unroll
    for (int l = 0; l < (RG_CX3_WU_LDS ? 3 : 2); ++l) {
      stage_lds<FT>(lds + off[l], a.w[l], nb[l]);
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  if (RG_CX3_PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if (RG_CX3_STAGGER && wave >= NW / 2) {
    for (int i = 0; i < RG_CX3_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
  }
  float* T = (float*)(lds + W_LDS + wave * T_BYTES);  // [TR][TS] message rows
  const WLds wE{lds + WE_OFF + lane * 16, plane_bytes(C, HID)};
  const WLds w2{lds + W2_OFF + lane * 16, plane_bytes(HID, C)};
#if RG_CX3_WU_LDS
  const WLds wU{lds + WU_OFF + lane * 16, plane_bytes(2 * C, C)};
#else
  const WBuf wU = wbuf(a.w[2], x3_bytes(2 * C, C), plane_bytes(2 * C, C), lane);
#endif
  const WBuf wPQ = wbuf(a.wpq, a.wpq ? x3_bytes(C, PQW) : 0, plane_bytes(C, PQW), lane);
  const float* bias2 = (const float*)(lds + W2_OFF + 3 * plane_bytes(HID, C));
  const float* biasU = (const float*)(a.w[2] + 3 * plane_bytes(2 * C, C));
  const float* biasPQ = a.wpq ? (const float*)(a.wpq + 3 * plane_bytes(C, PQW)) : nullptr;
  const float mu0 = nrm[0], sd0 = nrm[1], mu1 = nrm[2], sd1 = nrm[3], muU = nrm[4], sdU = nrm[5];

  const int xcd = blockIdx.x % NXCD;
#if RG_CX3_STATIC
  // static, edge-balanced work: the XCD's contiguous eighth of the nodes (its frames' rows
  // stay in one L2) is cut into one range per wave of that XCD with equal edge counts
  // (binary search over seg_ptr); the wave walks its range in blocks of up to NBLK nodes.
  // Dynamic block counters left up to one ~12-tile block of tail imbalance per wave.
  const int xlo = (int)((long)a.n_nodes * xcd / NXCD);
  const int xhi = (int)((long)a.n_nodes * (xcd + 1) / NXCD);
  const int nwx = (int)(gridDim.x / NXCD) * NW;               // waves on this XCD
  const int gw = (int)(blockIdx.x / NXCD) * NW + wave;        // this wave among them
  auto node_at_edge = [&](long target) {  // first node n in [xlo, xhi] with seg_ptr[n] >= target
    int lo = xlo, hi = xhi;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (a.seg_ptr[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const long ex0 = a.seg_ptr[xlo], ex1 = a.seg_ptr[xhi];
  const int wlo = gw == 0 ? xlo : node_at_edge(ex0 + (ex1 - ex0) * gw / nwx);
  const int whi = gw + 1 == nwx ? xhi : node_at_edge(ex0 + (ex1 - ex0) * (gw + 1) / nwx);
  int nb0 = __builtin_amdgcn_readfirstlane(wlo);
  const int nend = __builtin_amdgcn_readfirstlane(whi);
#else
  // with a block table: this XCD's blocks are table[xcd] .. table[xcd + 1] of the (first,
  // end) node pairs at table + TBL_HDR, largest first
  auto xlo = [&](int x) { return a.table ? a.table[x] : (int)((long)a.n_blocks * x / NXCD); };
  int blo = xlo(xcd), bhi = xlo(xcd + 1);
  const int* pairs = a.table ? a.table + TBL_HDR : nullptr;
  int* ctr = a.counters + CTR_STRIDE * xcd;
  int steal = 0;  // RG_CX3_STEAL: other XCDs' queues visited after this one drained
#endif

#if RG_CX3_STAMP
  unsigned long long st_acc[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
  for (;;) {
#if RG_CX3_STATIC
    if (nb0 >= nend) break;
    const int n0 = nb0;
    const int n1 = min(n0 + NBLK, nend);
    nb0 = n1;
#else
    int bi = 0;
    if (lane == 0) bi = atomicAdd(ctr, 1);
    // readfirstlane, not a shuffle: the block id, its node / edge range and the segment
    // state below are then provably wave-uniform (scalar registers and scalar branches)
    const int blk = blo + __builtin_amdgcn_readfirstlane(bi);
    if (blk >= bhi) {
      if (!RG_CX3_STEAL || !a.steal || ++steal >= NXCD) break;
      // this XCD's queue is empty: take the tail of the next one (cold rows, only at the end)
      const int x2 = (xcd + steal) % NXCD;
      blo = xlo(x2);
      bhi = xlo(x2 + 1);
      ctr = a.counters + CTR_STRIDE * x2;
      continue;
    }
    const int n0 = pairs ? pairs[2 * blk] : blk * NBLK;
    const int n1 = pairs ? pairs[2 * blk + 1] : min(n0 + NBLK, a.n_nodes);
#endif
    const int e0 = a.seg_ptr[n0], e1 = a.seg_ptr[n1];
    STAMP(0);  // block fetch
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
    // layer 1's B operand of k-step s
    auto eop = [&](const Rows& w, int s, int) { return split8(w.e[2 * s], w.e[2 * s + 1]); };
    auto load_e = [&](int q, Rows& w) {
      const float* pe = a.e + (size_t)q * a.lde + 8 * h;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#if RG_CX3_ENT  // streamed once per layer: non-temporal (keeps the reused P | Q rows in L2)
        w.e[2 * i] = __builtin_nontemporal_load((const f32x4*)(pe + 16 * i));
        w.e[2 * i + 1] = __builtin_nontemporal_load((const f32x4*)(pe + 16 * i + 4));
#else
        w.e[2 * i] = *(const f32x4*)(pe + 16 * i);
        w.e[2 * i + 1] = *(const f32x4*)(pe + 16 * i + 4);
#endif
      }
    };
    auto load_rows = [&](int q, int dq, int sq, Rows& w) {
      const float* pp = a.pq + (size_t)(RG_CX3_EXP == 3 ? n0 : dq) * PQW + 4 * h;
      const float* pqq = a.pq + (size_t)(RG_CX3_EXP == 3 ? n0 : sq) * PQW + HID + 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i) w.p[i] = *(const f32x4*)(pp + 8 * i);
#pragma unroll
      for (int i = 0; i < 16; ++i) w.q[i] = *(const f32x4*)(pqq + 8 * i);
      load_e(q, w);
    };
    auto load_pq = [&](int dq, int sq, Rows& w) {
      const float* pp = a.pq + (size_t)dq * PQW + 4 * h;
      const float* pqq = a.pq + (size_t)sq * PQW + HID + 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        w.p[i] = (RG_CX3_EXP == 8 || RG_CX3_EXP == 9) ? (f32x4){0.f, 0.f, 0.f, 0.f}
                                                       : *(const f32x4*)(pp + 8 * i);
#pragma unroll
      for (int i = 0; i < 16; ++i) w.q[i] = *(const f32x4*)(pqq + 8 * i);
    };
    // tile indices (past the block's last edge clamped: a re-read of a cached row)
    auto tile_idx = [&](int t, int& q, int& dq, int& sq) {
      q = min(t + r, e1 - 1);
      dq = a.dst[q];
      sq = a.src[q];
    };
    int p1 = 0, d1 = 0, s1 = 0, p2 = 0, d2 = 0, s2 = 0;
    Rows nrows;
    Rows rw;       // RG_CX3_LATE: loop-carried, loaded in the previous tile's second half
    int dcur = 0;  // RG_CX3_LATE: the destinations of the rows in rw
    int scur = 0;  // RG_CX3_LATE 4: their sources
    if (e0 < e1) {
      tile_idx(e0, p1, d1, s1);
      if constexpr (RG_CX3_RPF) {  // rows of tile 0 now, indices of tile 1
        load_rows(p1, d1, s1, nrows);
        tile_idx(e0 + 32, p2, d2, s2);
      } else if constexpr (RG_CX3_LATE == 4) {
        load_e(p1, rw);
        dcur = d1;
        scur = s1;
        tile_idx(e0 + 32, p1, d1, s1);
      } else if constexpr (RG_CX3_LATE) {
        load_rows(p1, d1, s1, rw);
        dcur = d1;
        tile_idx(e0 + 32, p1, d1, s1);
      }
    }
    for (int t0 = e0; t0 < e1; t0 += 32) {
      const int d = RG_CX3_LATE ? dcur : d1;
      if constexpr (RG_CX3_LATE == 4) {
        load_pq(d, scur, rw);  // e already in flight since the previous tile's second half
      } else if constexpr (RG_CX3_LATE) {
        // rows already in flight since the previous tile's second half
      } else if constexpr (RG_CX3_RPF) {
        // rows of the next tile now (indices loaded one tile earlier), indices of the tile
        // after: the whole gather latency hides behind this tile
        rw = nrows;
        load_rows(p2, d2, s2, nrows);
        p1 = p2; d1 = d2; s1 = s2;
        tile_idx(t0 + 64, p2, d2, s2);
      } else {
        load_rows(p1, d1, s1, rw);
        tile_idx(t0 + 32, p1, d1, s1);  // the next tile's indices (latency behind this tile)
      }
      // destination-change mask of this tile's edges (bit j: edge t0 + j starts a segment)
      const int dprev = __shfl_up(d, 1, 64);
      const uint32_t smask =
          (uint32_t)__ballot(r == 0 ? d != crow : d != dprev) &
          (e1 - t0 >= 32 ? 0xffffffffu : ((1u << (e1 - t0)) - 1u));
      // ---- layer 1: h = P[dst] + Q[src] + W_e e
      const int qt = min(t0 + r, e1 - 1);  // this lane's edge (tile_idx)
      f32x16 acc1[4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc1[m][4 * g + t] = RG_CX3_QLATE ? rw.p[4 * m + g][t] : rw.p[4 * m + g][t] + rw.q[4 * m + g][t];
      {
        if constexpr (RG_CX3_EXP != 5) {
          if constexpr (RG_CX3_MO & 1)
            layer_x3_mo<4, 4>(acc1, wE, 0, [&](int s) { return eop(rw, s, qt); });
          else
            layer_x3<4, 4, 4, RG_CX3_DB1>(acc1, wE, 0, [&](int s) { return eop(rw, s, qt); });
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc1[s][0] += xor_first(eop(rw, s, qt));
        }
      }
      if constexpr (RG_CX3_QLATE) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc1[m][4 * g + t] += rw.q[4 * m + g][t];
      }
      STAMP(1);  // gathers + layer 1 issue
#if RG_CX3_JIT
      // norm 1's statistics now; its scale + LeakyReLU inside layer 2's B operand
      const Pend pn1 = pend_norm_leaky<4, CENT>(acc1, mu0, sd0);
#else
      if constexpr (RG_CX3_EXP != 1) norm_leaky<4, CENT>(acc1, mu0, sd0);
#endif
      STAMP(2);  // norm 1 (waits for layer 1)
      // ---- layer 2 (B operand = layer 1's accumulators)
      f32x16 acc2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) acc2[m] = ld_bias_frag(bias2, m, h);
      if constexpr (RG_CX3_EXP != 5) {
#if RG_CX3_JIT
        if constexpr ((RG_CX3_MO & 2) != 0)
          layer_x3_mo<8, 2>(acc2, w2, 0, [&](int s) { return split_acc_pend<1>(acc1[s >> 1], s & 1, pn1); });
        else
          layer_x3<8, 2, 2, RG_CX3_DB2>(acc2, w2, 0,
                                        [&](int s) { return split_acc_pend<1>(acc1[s >> 1], s & 1, pn1); });
#else
        layer_x3<8, 2, 2, RG_CX3_DB2>(acc2, w2, 0, [&](int s) { return split_acc(acc1[s >> 1], s & 1); });
#endif
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const X3 b = split_acc(acc1[s >> 1], s & 1);
          acc2[s & 1][s] += xor_first(b);
        }
      }
      if constexpr (RG_CX3_LATE) {
        // acc1 and this tile's rows are dead: the next tile's rows go out now and arrive
        // behind norm 2 and the segmented sum (no registers beyond the rows' own)
        if constexpr (RG_CX3_LATE == 4) __builtin_amdgcn_sched_barrier(0);
        if (t0 + 32 < e1) {
          if constexpr (RG_CX3_LATE == 4) {
            load_e(p1, rw);
            scur = s1;
          } else {
            load_rows(p1, d1, s1, rw);
          }
          dcur = d1;
          tile_idx(t0 + 64, p1, d1, s1);
        }
      }
      STAMP(3);  // layer 2 issue
      if constexpr (RG_CX3_EXP != 1) norm_leaky<2, CENT>(acc2, mu1, sd1);
      STAMP(4);  // norm 2
      if constexpr (RG_CX3_EXP == 2) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int q = 0; q < 16; ++q) run += acc2[m][q];
        crow = n0;
        continue;
      }
      // ---- segmented sum in edge order, TR edges per LDS pass: a full pass runs without
      //      bounds checks, each edge one add; a destination change (a set bit of smask,
      //      wave-uniform, ~2.5 per tile) flushes the finished sum to its row out of line
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
      STAMP(5);  // segmented sum
    }
    STAMP(9);  // tile loop exit
    a.agg[(size_t)crow * C + lane] = run;  // (a block without edges: 0 to the dummy row)
    // the aggregate rows were written by this wave's lanes = features; read them back as
    // rows (lane = node) from L2: stores complete (vmcnt 0), loads bypass L1 (nt)
    if constexpr (NODE) __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)

    if constexpr (RG_CX3_EXP == 6) {
      if (n0 + r < n1) a.x_out[(size_t)(n0 + r) * a.ldo + h] = run;
      continue;
    }
    if constexpr (NODE) {
      node_update<CENT>(a, n0, n1, wU, biasU, wPQ, biasPQ, muU, sdU, lane);
    }
    STAMP(8);  // next layer's projections
  }
  // the last workgroup out re-zeroes the counters for the next launch (stream order)
  __syncthreads();
#if RG_CX3_STAMP
  STAMP(10);  // end-of-launch wait (this wave idle until its workgroup's last wave is done)
  if (lane == 0)
    for (int i = 0; i < 11; ++i) atomicAdd(&g_cx3_stamp[i], st_acc[i]);
#endif
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(a.counters + CTR_STRIDE * NXCD, 1) == (int)gridDim.x - 1) {
#pragma unroll
      for (int i = 0; i <= NXCD; ++i) a.counters[CTR_STRIDE * i] = 0;
    }
  }
}

// ---------------------------------------------------------------------------------------
// The edge launch as a two-group ping-pong (RG_CX3_PP, the default).
//
// conv_x3_kernel's waves each run the whole tile program -- gathers, layer 1, norm 1,
// layer 2, norm 2, segmented sum -- and the two waves of a SIMD drift freely, so their
// matrix phases collide as often as they interleave: the tile MFMAs (0.22 ms of the M
// layer) and everything else (0.36 ms) measured serial.  Here a tile is cut into
//   M: h = P[dst] + Q[src] + W_e e (acc1 from V), norm 1's statistics, layer 2   (192 MFMAs)
//   V: norm 2 + the segmented sum of the tile M just finished, then the NEXT tile's set-up:
//      block fetch when the block is exhausted, P | Q gathers, destination mask, acc1 = P + Q
// and the workgroup alternates them in lock-step slots separated by s_barrier: waves 0-3
// (one per SIMD) run M while waves 4-7 (the other wave of each SIMD) run V, then the roles
// swap.  The matrix pipe of every SIMD then always has one wave feeding it, and the other
// wave's gathers, norms and LDS work issue in the MFMA shadow.  A slot lasts as long as
// its longest M phase (one tile each, equal work); a V phase is a fraction of that.
// Each destination still sums its edges in CSR order inside one block: bit-identical to
// conv_x3_kernel.  The two groups run separate loops (V, M / M, V) so that every register
// array has one producer phase and one consumer phase and is dead in between.
// Termination: a wave with no work left sets its bit in a per-slot-parity LDS word; every
// wave reads the word of the slot it just closed after the barrier, so all waves leave
// after the same slot (the word of slot s is next written in slot s + 2, after the barrier
// every reader of slot s must reach first).
template <bool CENT, int MODE>
__global__ __launch_bounds__(FT) void conv_x3_pp_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[4];
  __shared__ uint32_t done_w[2];
  __shared__ int tok[NW / 2];  // MODE 2: per SIMD pair, the group whose M phase is next (2: free)
  if (threadIdx.x < 2) {
    nrm[2 * threadIdx.x] = *a.mu[threadIdx.x];
    nrm[2 * threadIdx.x + 1] = *a.sd[threadIdx.x];
    done_w[threadIdx.x] = 0;
  }
  if (threadIdx.x < NW / 2) tok[threadIdx.x] = 0;
  stage_lds<FT>(lds + WE_OFF, a.w[0], x3_bytes(C, HID));
  stage_lds<FT>(lds + W2_OFF, a.w[1], x3_bytes(HID, C));
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  float* T = (float*)(lds + W_LDS + wave * T_BYTES);  // [TR][TS] message rows
  const WLds wE{lds + WE_OFF + lane * 16, plane_bytes(C, HID)};
  const WLds w2{lds + W2_OFF + lane * 16, plane_bytes(HID, C)};
  const float* bias2 = (const float*)(lds + W2_OFF + 3 * plane_bytes(HID, C));
  const float mu0 = nrm[0], sd0 = nrm[1], mu1 = nrm[2], sd1 = nrm[3];

  const int xcd = blockIdx.x % NXCD;
  auto xlo = [&](int x) { return a.table ? a.table[x] : (int)((long)a.n_blocks * x / NXCD); };
  int blo = xlo(xcd), bhi = xlo(xcd + 1);
  const int* pairs = a.table ? a.table + TBL_HDR : nullptr;
  int* ctr = a.counters + CTR_STRIDE * xcd;
  int steal = 0;

  int n0 = 0, e1 = 0;  // current block: first node, edge end
  int tn = 0;          // first edge of the next tile to set up (tn >= e1: block exhausted)
  bool alive = true;   // blocks may remain
  bool have = false;   // acc1 holds a set-up tile for the M phase
  bool pend = false;   // acc2 holds a tile's layer-2 output for the V phase
  int tc = 0;          // first edge of the tile in acc1 / acc2
  uint32_t smask = 0;  // its destination-change mask
  int d = 0;           // this lane's destination in it
  float run = 0.f;     // lane = feature: running sum of the current destination
  int cur = -1;        // its slot in the block (wave-uniform)
  int p1 = 0, d1 = 0, s1 = 0;  // edge / destination / source of this lane in tile tn
  f32x4 ev[8];         // e rows of tile tn (k order), in flight from the previous M phase
  f32x16 acc1[4], acc2[2];
  int slot = 0;
#if RG_CX3_STAMP
  // diagnostic build: [0] V work, [1] of it in block-fetch slots, [2] M work, [3] barrier
  // wait after V, [4] after M, [5] V slots, [6] fetch slots, [7] M slots with a tile,
  // [8] norm 2 + segmented sum, [9] the rest of V after it (gathers' waits, adds)
  // [10] norm 2 alone, [11] layer 1 (M), [12] norm 1's statistics (M), [13] M slots' stamps
  unsigned long long st[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
  auto tick = [&]() {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    const unsigned long long dlt = n - t_last;
    t_last = n;
    return dlt;
  };
  bool vlast = false;
#endif

  auto tile_idx = [&](int t) {
    p1 = min(t + r, e1 - 1);  // past the block's last edge clamped: a re-read of a cached row
    d1 = a.dst[p1];
    s1 = a.src[p1];
  };
  auto load_e = [&]() {
    const float* pe = a.e + (size_t)p1 * a.lde + 8 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ev[2 * i] = *(const f32x4*)(pe + 16 * i);
      ev[2 * i + 1] = *(const f32x4*)(pe + 16 * i + 4);
    }
  };
  // the next block with edges: its bounds, first tile indices and e rows
  // the next block with edges from the queues (stealing from the other XCDs' tails once
  // this one drained): its first node and edge range; false when every queue is empty
  bool dry = false;
  auto dequeue = [&](int& b0, int& be0, int& be1) {
    while (!dry) {
      int bi = 0;
      if (lane == 0) bi = atomicAdd(ctr, 1);
      const int blk = blo + __builtin_amdgcn_readfirstlane(bi);
      if (blk >= bhi) {
        if (!RG_CX3_STEAL || !a.steal || ++steal >= NXCD) {
          dry = true;
          break;
        }
        const int x2 = (xcd + steal) % NXCD;  // this XCD's queue is empty: the next one's tail
        blo = xlo(x2);
        bhi = xlo(x2 + 1);
        ctr = a.counters + CTR_STRIDE * x2;
        continue;
      }
      b0 = pairs ? pairs[2 * blk] : blk * NBLK;
      const int nb1 = pairs ? pairs[2 * blk + 1] : min(b0 + NBLK, a.n_nodes);
      be0 = a.seg_ptr[b0];
      be1 = a.seg_ptr[nb1];
      if (be0 < be1) return true;  // (a block without edges leaves its aggregate rows unwritten: degree 0)
    }
    return false;
  };
  // RG_CX3_PP_PF: the next block is dequeued while the current one runs -- its bounds in the
  // V phase of the current block's second tile, its first tile's indices in the third's --
  // so a block switch costs one gather round trip like any other tile, not the dequeue ->
  // bounds -> indices -> rows chain (pf: 0 nothing prefetched, 1 bounds, 2 and indices)
  int pf = 0, pn0 = 0, pe0 = 0, pe1 = 0;
  int pp1 = 0, pd1 = 0, ps1 = 0;
  auto fetch = [&]() {
    int e0 = 0;
    if (pf > 0) {
      n0 = pn0;
      e0 = pe0;
      e1 = pe1;
    } else if (!dequeue(n0, e0, e1)) {
      alive = false;
      return;
    }
    tn = e0;
    if (pf == 2) {
      p1 = pp1;
      d1 = pd1;
      s1 = ps1;
    } else {
      tile_idx(tn);
    }
    pf = 0;
    load_e();
  };
  auto prefetch = [&]() {
    if (pf == 0 && !dry) {
      if (dequeue(pn0, pe0, pe1)) pf = 1;
    } else if (pf == 1) {
      pp1 = min(pe0 + r, pe1 - 1);
      pd1 = a.dst[pp1];
      ps1 = a.src[pp1];
      pf = 2;
    }
  };
  // P[dst] | Q[src] rows of M-tile m (accumulator order) of this lane's edge in tile tn
  auto ld_pq = [&](int m, f32x4 (&pr)[4], f32x4 (&qr)[4]) {
    const float* pp = a.pq + (size_t)d1 * PQW + 4 * h + 32 * m;
    const float* pq = a.pq + (size_t)s1 * PQW + HID + 4 * h + 32 * m;
#pragma unroll
    for (int g = 0; g < 4; ++g) pr[g] = *(const f32x4*)(pp + 8 * g);
#pragma unroll
    for (int g = 0; g < 4; ++g) qr[g] = *(const f32x4*)(pq + 8 * g);
  };
  auto add_pq = [&](int m, const f32x4 (&pr)[4], const f32x4 (&qr)[4]) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc1[m][4 * g + t] = pr[g][t] + qr[g][t];
  };

  // ================= V phase: norm 2 + segmented sum of acc2, then the next tile into acc1
  auto vphase = [&]() {
    const int bn0 = n0, be1 = e1;  // the pending tile's block
    const bool fresh = alive && tn >= e1;
#if RG_CX3_STAMP
    vlast = true;
    tick();
    st[5] += 1;
    st[6] += fresh;
#endif
    if (fresh) fetch();
    // the first two M-tiles' P | Q rows (RG_CX3_PP_PQ 4: all four) fly behind norm 2 and
    // the segmented sum
    f32x4 pr0[4], qr0[4], pr1[4], qr1[4];
#if RG_CX3_PP_PQ == 4
    f32x4 pr2[4], qr2[4], pr3[4], qr3[4];
#endif
    if (alive) {
      ld_pq(0, pr0, qr0);
      ld_pq(1, pr1, qr1);
#if RG_CX3_PP_PQ == 4
      ld_pq(2, pr2, qr2);
      ld_pq(3, pr3, qr3);
#endif
    }
    if (pend) {
      if (!RG_CX3_PP_N2M) norm_leaky<2, CENT>(acc2, mu1, sd1);
#if RG_CX3_STAMP
      {
        const unsigned long long d2 = tick();
        st[10] += d2;
        st[8] += d2;
      }
#endif
#pragma unroll
      for (int c = 0; c < 32 / TR; ++c) {
        if (tc + TR * c >= be1) break;  // wave-uniform
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
        float v[TR];
#pragma unroll
        for (int j = 0; j < TR; ++j) v[j] = T[j * TS + lane];
        // branch-free scan as in conv_x3_kernel, the finished sums out of line
        const int nv = be1 - tc;
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
        for (uint32_t m = pm; m; m &= m - 1) {
          const int j = __builtin_ctz(m);
          float fin = run;
#pragma unroll
          for (int k = 0; k + 1 < TR; ++k) fin = (j == k + 1) ? rv[k] : fin;
          if (cur >= 0) a.agg[(size_t)(bn0 + cur) * C + lane] = fin;
          cur = __builtin_amdgcn_readlane(d, TR * c + j) - bn0;
        }
        run = rv[TR - 1];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
      pend = false;
    }
#if RG_CX3_STAMP
    const unsigned long long dseg = tick();  // (+ the block fetch in fresh slots)
    st[8] += dseg;
#endif
    if (fresh) {  // the previous block is done: its last destination's sum
      if (cur >= 0) a.agg[(size_t)(bn0 + cur) * C + lane] = run;
      cur = -1;
      run = 0.f;
    }
    if (alive) {
      d = d1;
      tc = tn;
      const int dprev = __shfl_up(d, 1, 64);
      smask = (uint32_t)__ballot(r == 0 ? d - n0 != cur : d != dprev) &
              (e1 - tc >= 32 ? 0xffffffffu : ((1u << (e1 - tc)) - 1u));
#if RG_CX3_PP_PQ == 4
      add_pq(0, pr0, qr0);
      add_pq(1, pr1, qr1);
      add_pq(2, pr2, qr2);
      add_pq(3, pr3, qr3);
      tn += 32;
      if (tn < e1) tile_idx(tn);
#else
      f32x4 pr2[4], qr2[4];
      add_pq(0, pr0, qr0);
      ld_pq(2, pr2, qr2);
      add_pq(1, pr1, qr1);
      ld_pq(3, pr0, qr0);
      tn += 32;
      if (tn < e1) tile_idx(tn);
      add_pq(2, pr2, qr2);
      add_pq(3, pr0, qr0);
#endif
      if (RG_CX3_PP_PF && !fresh) prefetch();
      have = true;
    } else {
      // nothing set up: acc1 defined on every path (else its old value counts as live here)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc1[m] = (f32x16){};
    }
#if RG_CX3_STAMP
    const unsigned long long dv = tick();
    st[9] += dv;
    st[0] += dseg + dv;
    if (fresh) st[1] += dseg + dv;
#endif
  };
  // ================= M phase: layer 1, norm 1's statistics, layer 2 (acc1 -> acc2)
  auto mphase = [&]() {
#if RG_CX3_STAMP
    vlast = false;
    tick();
    st[7] += have;
#endif
    if (have) {
      if (RG_CX3_PP_PRIO) __builtin_amdgcn_s_setprio(1);
      layer_x3<4, 4, 4, RG_CX3_DB1>(acc1, wE, 0, [&](int s) { return split8(ev[2 * s], ev[2 * s + 1]); });
#if RG_CX3_STAMP
      {
        const unsigned long long d1 = tick();
        st[11] += d1;
        st[2] += d1;
      }
#endif
      const Pend pn1 = pend_norm_leaky<4, CENT>(acc1, mu0, sd0);
#if RG_CX3_STAMP
      {
        const unsigned long long d1 = tick();
        st[12] += d1;
        st[2] += d1;
      }
#endif
#pragma unroll
      for (int m = 0; m < 2; ++m) acc2[m] = ld_bias_frag(bias2, m, h);
      layer_x3<8, 2, 2, RG_CX3_DB2>(acc2, w2, 0,
                                    [&](int s) { return split_acc_pend<1>(acc1[s >> 1], s & 1, pn1); });
      // the next tile's e rows (the only rows streamed from HBM) arrive behind the slot
      if (tn < e1) load_e();
      if (RG_CX3_PP_N2M) norm_leaky<2, CENT>(acc2, mu1, sd1);  // norm 2 here, not in V
      if (RG_CX3_PP_PRIO) __builtin_amdgcn_s_setprio(0);
      have = false;
      pend = true;
    } else {
#pragma unroll
      for (int m = 0; m < 2; ++m) acc2[m] = (f32x16){};
    }
#if RG_CX3_STAMP
    st[2] += tick();
#endif
  };
  // close the slot: true when every wave of the workgroup is out of work
  auto sync = [&]() {
    if (!alive && !pend && !have) atomicOr(&done_w[slot & 1], 1u << wave);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the done word is visible past the barrier
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#if RG_CX3_STAMP
    st[vlast ? 3 : 4] += tick();
#endif
    const bool all = done_w[slot & 1] == (1u << NW) - 1u;
    ++slot;
    return all;
  };
  if constexpr (MODE == 2) {
    // RG_CX3_PP 2: no workgroup lock-step -- each wave loops V, M on its own, and the two
    // waves of a SIMD (w, w + 4) pass a matrix-pipe token: a wave starts its M phase only
    // when the token is its group's (or free), and hands it over at the M phase's end.  The
    // token orders nothing the results depend on (every wave computes its own tiles), so the
    // wait is bounded and a wave leaving sets it free for good.
    const int pair = wave & (NW / 2 - 1), g = wave >= NW / 2;
    for (;;) {
      vphase();
      if (!have) break;  // no block left (the last V phase flushed the last sum)
#if RG_CX3_STAMP
      tick();
#endif
      for (int spin = 0; spin < (1 << 16); ++spin) {
        const int t = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&tok[pair], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (t == g || t == 2) break;
        __builtin_amdgcn_s_sleep(1);
      }
#if RG_CX3_STAMP
      st[4] += tick();
#endif
      mphase();
      if (lane == 0) atomicCAS(&tok[pair], g, 1 - g);
    }
    if (lane == 0) atomicExch(&tok[pair], 2);
  } else if (wave < NW / 2) {  // waves 0-3: V first
    for (;;) {
      vphase();
      if (sync()) break;
      mphase();
      if (sync()) break;
    }
  } else {              // waves 4-7: M first (the first one idle)
    for (;;) {
      mphase();
      if (sync()) break;
      vphase();
      if (sync()) break;
    }
  }
#if RG_CX3_STAMP
  if (lane == 0)
    for (int i = 0; i < 14; ++i) atomicAdd(&g_cx3_stamp[i], st[i]);
#endif
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(a.counters + CTR_STRIDE * NXCD, 1) == (int)gridDim.x - 1) {
#pragma unroll
      for (int i = 0; i <= NXCD; ++i) a.counters[CTR_STRIDE * i] = 0;
    }
  }
}

// The node phase as a launch of its own (RG_CX3_NODE_KERNEL): W_u and W'_pq both staged in
// LDS (145 KB), one 32-node tile per wave and step; the aggregate rows come from the
// edge launch's scratch.  In the single-launch layer the same phase runs at each block's
// end with both weight images read from L2 (the edge weights fill the LDS).
static constexpr int NU_OFF = 0;
static constexpr int NPQ_OFF = al16(x3_bytes(2 * C, C));
static constexpr int NODE_LDS = NPQ_OFF + al16(x3_bytes(C, PQW));
#ifndef RG_CX3_NODE_FT
#define RG_CX3_NODE_FT 512  // node launch workgroup: 8 waves = two per SIMD (170 VGPRs)
#endif
static constexpr int NFT = RG_CX3_NODE_FT, NW_NODE = NFT / 64;
static_assert(NODE_LDS <= DYN_LDS_MAX, "node_x3 LDS");
template <bool CENT>
__global__ __launch_bounds__(NFT) void node_x3_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[2];
  if (threadIdx.x == 0) {
    nrm[0] = *a.mu[2];
    nrm[1] = *a.sd[2];
  }
  {
    const int nb[2] = {x3_bytes(2 * C, C), a.wpq ? x3_bytes(C, PQW) : 0};
    const char* src[2] = {a.w[2], a.wpq};
    const int off[2] = {NU_OFF, NPQ_OFF};
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      stage_lds<NFT>(lds + off[l], src[l], nb[l]);
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const WLds wU{lds + NU_OFF + lane * 16, plane_bytes(2 * C, C)};
  const WLds wPQ{lds + NPQ_OFF + lane * 16, plane_bytes(C, PQW)};
  const float* biasU = (const float*)(lds + NU_OFF + 3 * plane_bytes(2 * C, C));
  const float* biasPQ = (const float*)(lds + NPQ_OFF + 3 * plane_bytes(C, PQW));
  const float muU = nrm[0], sdU = nrm[1];
  const int ntiles = (a.n_nodes + 31) / 32;
  const int stride = gridDim.x * NW_NODE;
  // the next tile's rows are loaded while this one computes; unrolled by two with separate
  // row buffers (a register copy of a loaded value would wait for the load)
#if !RG_CX3_NODE_PF
  for (int t = blockIdx.x * NW_NODE + wave; t < ntiles; t += stride)
    node_update<CENT>(a, 32 * t, min(32 * t + 32, a.n_nodes), wU, biasU, wPQ, biasPQ, muU, sdU,
                      lane);
  return;
#endif
  NodeRows rA, rB;
  int t = blockIdx.x * NW_NODE + wave;
  auto tile_end = [&](int tt) { return min(32 * tt + 32, a.n_nodes); };
  if (t < ntiles) load_node_rows(a, 32 * t, tile_end(t), lane, rA);
  while (t < ntiles) {
    int tn = t + stride;
    if (tn < ntiles) load_node_rows(a, 32 * tn, tile_end(tn), lane, rB);
    node_compute<CENT>(a, rA, 32 * t, tile_end(t), wU, biasU, wPQ, biasPQ, muU, sdU, lane);
    t = tn;
    if (t >= ntiles) break;
    tn = t + stride;
    if (tn < ntiles) load_node_rows(a, 32 * tn, tile_end(tn), lane, rA);
    node_compute<CENT>(a, rB, 32 * t, tile_end(t), wU, biasU, wPQ, biasPQ, muU, sdU, lane);
    t = tn;
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

#if RG_CX3_STAMP
// diagnostic builds only (not in radar_gnn.h): read and clear the phase sums
extern "C" int rg_debug_cx3_stamps(unsigned long long* out_host) {
  RG_CHECK_HIP(hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_cx3_stamp), sizeof(g_cx3_stamp)));
  static const unsigned long long z[16] = {0};
  RG_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_cx3_stamp), z, sizeof(z)));
  return RG_OK;
}
#endif

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
// (100 - RG_CX3_TAIL) % and TAILN-node runs over the rest, all ordered by edge tiles, largest
// first: the waves take the big blocks first and end on the small ones, so the launch tail
// (waves idle until the last block of their workgroup ends: 14 % of the wave time with
// 32-node blocks only, M) shrinks to a few tiles.  Order and size change no result: each
// destination's messages are summed in CSR order within one block.
__host__ __device__ inline void x3_share(int n, int x, int& a0, int& sp, int& b0) {
  a0 = (int)((long)n * x / NXCD);
  b0 = (int)((long)n * (x + 1) / NXCD);
  sp = a0 + (int)((long)(b0 - a0) * (100 - RG_CX3_TAIL) / 100 / NBLK) * NBLK;
}
__host__ __device__ inline int x3_share_blocks(int n, int x) {
  int a0, sp, b0;
  x3_share(n, x, a0, sp, b0);
  return (sp - a0 + NBLK - 1) / NBLK + (b0 - sp + TAILN - 1) / TAILN;
}
// order (RG_CX3_ORDER, measurement knob): 0 = every block by edge tiles, largest first;
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
  // RG_LAYER_E_SPLIT: e = the pre-split planes (rg_mlp_chain_x3_split), lde in BYTES
  RG_REQUIRE(ldx % 4 == 0 && ld_out % 4 == 0 && lde % 4 == 0,
             RG_ERR_UNSUPPORTED,
             "rg_conv_layer_x3: row strides must be multiples of 4 (pre-split e: 16 bytes, >= 384)");
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
  constexpr bool NODE = !RG_CX3_NODE_KERNEL;  // node phase inside the edge launch
  auto edge = cent ? conv_x3_kernel<true, NODE> : conv_x3_kernel<false, NODE>;
  if constexpr (RG_CX3_PP != 0 && !NODE)  // (variant builds only)
    edge = cent ? conv_x3_pp_kernel<true, RG_CX3_PP> : conv_x3_pp_kernel<false, RG_CX3_PP>;
  RG_ENSURE_LDS(edge, LDS_BYTES);
  edge<<<blocks, FT, LDS_BYTES, (hipStream_t)stream>>>(a);
  RG_LAUNCH_CHECK_ZERO(a.counters, CTR_BYTES, stream);
  if constexpr (!NODE) {
    auto node = cent ? node_x3_kernel<true> : node_x3_kernel<false>;
    RG_ENSURE_LDS(node, NODE_LDS);
    const int tiles = (n_nodes + 31) / 32;
    const int nblk = (tiles + NW_NODE - 1) / NW_NODE < 256 ? (tiles + NW_NODE - 1) / NW_NODE : 256;
    node<<<nblk, NFT, NODE_LDS, (hipStream_t)stream>>>(a);
    RG_LAUNCH_CHECK();
  }
  return RG_OK;
}
