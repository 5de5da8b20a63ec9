// Fused residual_graph_conv_block on 16-bit operands: the kernel of conv_fused.hip, compiled
// once per operand type (RG_HALF_F16 = 0: bf16 in namespace rg::conv; 1: IEEE fp16 in
// rg::conv_f16).  No include guard: conv_fused.hip includes it twice.
namespace rg {
namespace RG_CONV_NS {

using HT = ::rg::H16<RG_HALF_F16 != 0>;  // the 16-bit operand type (bf16 / fp16)

typedef HT::v8 bf16x8_t;  // (named for the bf16 build; fp16 lanes in the fp16 build)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static constexpr int CT = 512;  // threads per workgroup (8 waves, 2 per SIMD)
static constexpr int CW = CT / 64;
static constexpr int NB = 8;         // destination nodes per work block
static constexpr int C = 64;         // node / edge / message / output channels
static constexpr int HID = 128;      // msg_mlp_hidden_dim
// wave-private LDS: P (NB rows of HID f32, row stride PST: the 4-float pad puts the rows of
// different nodes on different banks -- at HID they all mapped to the same four), message
// tile (32 x C bf16)
static constexpr int PST = HID + 4;
static constexpr int WAVE_LDS = NB * PST * 4 + 32 * C * 2;
static constexpr float NORM_EPS = 1e-5f;
// Work-block heads: one per XCD (workgroup b runs on XCD b % 8), each on a 128-B line of
// its own.  One shared head saturates at ~88 dequeues/us (MI355X_MICROARCH.md, dequeue):
// measured here, both the C2 and C5 layers ran at exactly one block per ~22 ns with it.
static constexpr int NQ = 8;
static constexpr int CTR_STRIDE = 32;

// the one-hot segment matrix from a 256-entry LDS table: entry b = eight 16-bit ONEs / zeros
// for the bits of b (4 KiB of LDS)
static constexpr int LUT_BYTES = 256 * 16;

#ifndef RG_CONV_STAMP
#define RG_CONV_STAMP 0  // diagnostic build: per-phase s_memtime sums in g_conv_stamp
#endif
#if RG_CONV_STAMP
// [0] staging [1] block head + P [2] edge tiles [3] update + store [4] blocks [5] tiles
// [6] end-of-kernel wait [8] min start [9] max end (s_memrealtime, 100 MHz)
__device__ unsigned long long g_conv_stamp[16];
#define CSTAMP(i)                                              \
  do {                                                         \
    const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += _n - st_last;                                 \
    st_last = _n;                                              \
  } while (0)
#else
#define CSTAMP(i) do {} while (0)
#endif

struct CLayer {
  int woff, bytes, out, act, centered;
  const float* mu;
  const float* sd;
  const void* src;
};

struct CArgs {
  CLayer L[3];  // msg0 (192->128), msg1 (128->64), upd (128->64)
  int total_bytes;
  int aggr_mean;
  int n_nodes;
  int n_blocks;
  const uint16_t* x;
  const uint16_t* e;
  const int* seg_ptr;
  const int* src;
  const int* dst;
  uint16_t* x_out;
  int* counter;  // NQ block heads, one per XCD, CTR_STRIDE ints apart, then the done counter
  int ldx, lde, ldo;
  // optional edge-balanced work blocks (rg_conv_blocks): block b = nodes
  // [blk_nodes[2b], blk_nodes[2b + 1]), at most NB, *n_blk_dev blocks (each XCD's share
  // largest first, rg_conv_blocks); null: b = 8-node run
  const int* blk_nodes;
  const int* n_blk_dev;
  // optional static schedule (rg_conv_wave_nodes): wave rank w owns the nodes
  // [wave_nodes[w], wave_nodes[w + 1]) -- equal shares of degree + WAVE_NODE_COST -- and walks
  // them in NB-node blocks; no work counters.  Ranks are XCD-major (workgroup b is on XCD
  // b % NQ), so an XCD's waves hold one contiguous node range.
  const int* wave_nodes;
};

__device__ __forceinline__ uint32_t bf2(float a, float b) { return HT::pack2(a, b); }
__device__ __forceinline__ bf16x8_t ld_bf8(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *(const u32x4*)p);
}
__device__ __forceinline__ bf16x8_t zero_bf8() {
  return __builtin_bit_cast(bf16x8_t, (u32x4){0u, 0u, 0u, 0u});
}

// k-steps [S0, S0 + KS) of a packed 32x32x16 layer with KT k-steps in total
// (fragment (m, s) at byte (m * KT + s) * 1024); acc holds the initial values.
// Software pipelined: the A fragments of step s+1 are read from LDS while the MFMAs of
// step s issue, so an MFMA never waits for the LDS read that feeds it; one scheduling
// fence per step keeps the compiler from hoisting the whole layer's fragments.
static constexpr int PD = 1;  // A-fragment prefetch distance (k-steps)

template <int KS, int MT, int KT, int S0>
__device__ __forceinline__ void mfma_steps(const bf16x8_t* b, f32x16 (&acc)[MT], const char* w,
                                           int lane) {
  const char* wl = w + lane * 16;
  bf16x8_t f[KS][MT];
#pragma unroll
  for (int s = 0; s < PD && s < KS; ++s)
#pragma unroll
    for (int m = 0; m < MT; ++m) f[s][m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KT + S0 + s) * 1024));
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + PD < KS) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        f[s + PD][m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KT + S0 + s + PD) * 1024));
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
      acc[m] = HT::mfma(f[s][m], b[s], acc[m]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the same k-steps with the B operand of step s formed by bop(s) one step ahead, beside the
// MFMAs of step s - 1 (a normalised previous layer's scale + LeakyReLU + bf16 pack then issue
// in the matrix pipe's shadow instead of between the layers)
template <int KS, int MT, int KT, int S0, typename BOp>
__device__ __forceinline__ void mfma_steps_jit(BOp&& bop, f32x16 (&acc)[MT], const char* w,
                                               int lane) {
  const char* wl = w + lane * 16;
  bf16x8_t f[KS][MT];
#pragma unroll
  for (int s = 0; s < PD && s < KS; ++s)
#pragma unroll
    for (int m = 0; m < MT; ++m) f[s][m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KT + S0 + s) * 1024));
  bf16x8_t bq = bop(0);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + PD < KS) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        f[s + PD][m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KT + S0 + s + PD) * 1024));
    }
    bf16x8_t bn = bq;
    if (s + 1 < KS) bn = bop(s + 1);
#pragma unroll
    for (int m = 0; m < MT; ++m)
      acc[m] = HT::mfma(f[s][m], bq, acc[m]);
    bq = bn;
    __builtin_amdgcn_sched_barrier(0);
  }
}


// channel_normalization (common.py:208-220) + activation (rg_common.h)
// (every block is normalised; with ACT >= 0 every block uses ACT and was packed
// RG_PACK_CENTERED: host-checked)
// (mu, sd = the layer's channel_normalization scalars, staged in LDS once per kernel)
template <int ACT, int MT>
__device__ __forceinline__ void norm_act(f32x16 (&acc)[MT], const CLayer& L, float mu, float sd) {
#ifndef RG_NO_FUSED_LEAKY
  if constexpr (ACT == ACT_LEAKY) {  // centred (host-checked): norm + leaky in two fmas
    channel_norm_leaky_centered<MT>(acc, mu, sd, NORM_EPS);
    return;
  }
#endif
  if constexpr (ACT >= 0) channel_norm_pk_centered<MT>(acc, mu, sd, NORM_EPS);
  else if (L.centered) channel_norm_pk_centered<MT>(acc, mu, sd, NORM_EPS);
  else channel_norm_pk<MT>(acc, mu, sd, NORM_EPS);
  if constexpr (ACT >= 0) act_pk_all<ACT, MT>(acc);
  else act_dispatch(L.act, [&](auto A) { act_pk_all<decltype(A)::value, MT>(acc); });
}

template <int MT>
__device__ __forceinline__ void pack_acc(const f32x16 (&acc)[MT], bf16x8_t* nb) {
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int q = 8 * hf;
      nb[2 * m + hf] = __builtin_bit_cast(
          bf16x8_t, (u32x4){bf2(acc[m][q + 0], acc[m][q + 1]), bf2(acc[m][q + 2], acc[m][q + 3]),
                            bf2(acc[m][q + 4], acc[m][q + 5]), bf2(acc[m][q + 6], acc[m][q + 7])});
    }
}

// XOR swizzle of the 4-feature granules of message-tile row `row` (64 bf16 = 128 B per
// row).  Row stores (ds_write_b64, lane = row) and transposed reads (ds_read_b64_tr_b16,
// 4 rows x 8 granules per half-wave) are both bank-conflict free: granule g of row r
// lives at g ^ swz(r), swz a bijection on 0..15 whose bit 3 differs for rows r, r + 2.
__device__ __forceinline__ int swz(int row) {
  return (row & 7) | ((((row >> 1) ^ (row >> 3)) & 1) << 3);
}

template <int ACT>
__global__ __launch_bounds__(CT) void fused_conv_kernel(CArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
#if RG_CONV_STAMP
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
  const unsigned long long st_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  __shared__ float nrm[6];  // (mu, sd) of the three channel_normalizations
  if (threadIdx.x == 0) {  // static layer indices: a dynamic a.L[i] would copy a to scratch
#pragma unroll
    for (int l = 0; l < 3; ++l) {
      nrm[2 * l] = *a.L[l].mu;
      nrm[2 * l + 1] = *a.L[l].sd;
    }
  }
  // stage weights (static indices)
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    stage_lds<CT>(lds + a.L[l].woff, a.L[l].src, a.L[l].bytes);
  }
  for (int b = threadIdx.x; b < 256; b += CT) {
    u32x4 e;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      e[i] = (((b >> (2 * i)) & 1) ? HT::ONE : 0u) | ((((b >> (2 * i + 1)) & 1) ? HT::ONE : 0u) << 16);
    *(u32x4*)(lds + a.total_bytes + 16 * b) = e;
  }
  __syncthreads();
  CSTAMP(0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  // wave-private: P [NB][MT=4][h][16] f32, message tile [32][64] bf16
  const u32x4* lut = (const u32x4*)(lds + a.total_bytes);
  char* wbase = lds + a.total_bytes + LUT_BYTES + wave * WAVE_LDS;
  float* P = (float*)wbase;
  uint16_t* tile = (uint16_t*)(wbase + NB * PST * 4);
  const char* w0 = lds + a.L[0].woff;
  const char* w1 = lds + a.L[1].woff;
  const char* w2 = lds + a.L[2].woff;
  const float* bias0 = (const float*)(w0 + 4 * 12 * 1024);
  const float* bias1 = (const float*)(w1 + 2 * 8 * 1024);
  const float* bias2 = (const float*)(w2 + 2 * 8 * 1024);

  // block ids come from an atomic counter (dynamic balance); the NEXT block's id and
  // edge range are fetched at the start of the current block, so a block starts with
  // two dependent global round trips (indices -> rows) instead of four
  const int n_blocks = a.blk_nodes ? *a.n_blk_dev : a.n_blocks;
  // this XCD's share of the blocks: contiguous destination ranges (its L2 then holds the
  // neighbourhoods it gathers), dequeued from its own head
  const int xcd = blockIdx.x % NQ;
  const int blo = __builtin_amdgcn_readfirstlane((int)((long)n_blocks * xcd / NQ));
  const int bhi = __builtin_amdgcn_readfirstlane((int)((long)n_blocks * (xcd + 1) / NQ));
  int* head = a.counter + CTR_STRIDE * xcd;
  // node range of work block b (its edges are the CSR range seg_ptr[n0] .. seg_ptr[n1])
  auto block_nodes = [&](int b, int& n0, int& n1) {
    if (a.blk_nodes) {
      n0 = a.blk_nodes[2 * b];
      n1 = a.blk_nodes[2 * b + 1];
    } else {
      n0 = b * NB;
      n1 = min(n0 + NB, a.n_nodes);
    }
  };
  int blk = 0;
  int e0 = 0, e1 = 0, bn0 = 0, bn1 = 0;
  int s_hi = 0;  // static schedule: the end of this wave's node range
  if (a.wave_nodes) {
    const int rank = (blockIdx.x % NQ) * (int)(gridDim.x / NQ) * CW + (blockIdx.x / NQ) * CW + wave;
    bn0 = a.wave_nodes[rank];
    s_hi = a.wave_nodes[rank + 1];
    bn1 = min(bn0 + NB, s_hi);
    blk = bn0 < s_hi ? 0 : -1;
  } else {
    if (lane == 0) blk = atomicAdd(head, 1);
    blk = blo + __builtin_amdgcn_readfirstlane(blk);  // (lane 0's value: every lane is active)
    if (blk >= bhi) blk = -1;
    if (blk >= 0) block_nodes(blk, bn0, bn1);
  }
  if (blk >= 0) {
    e0 = a.seg_ptr[bn0];
    e1 = a.seg_ptr[bn1];
  }
  while (blk >= 0) {
    const int n0 = bn0;
    const int n1 = bn1;
    int nxt_raw = 0;
    if (!a.wave_nodes && lane == 0) nxt_raw = atomicAdd(head, 1);
    // the block's node r (= one-hot column / slot r) owns the CSR range [sst, sen); lanes
    // past the block's nodes get an empty range (clamped loads, no branch)
    const int sst = a.seg_ptr[min(n0 + r, n1)], sen = a.seg_ptr[min(n0 + r + 1, n1)];
    f32x16 agg[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) agg[m] = (f32x16){0.f};

    // ---- edge tiles, software pipelined: while tile t computes, the rows of tile t+1
    //      (x[src], e) and the indices of tile t+2 are in flight.  The loop is unrolled
    //      by two with separate A / B registers for rows AND indices, so no loaded value
    //      is ever copied (a copy would wait for the load and serialise the pipeline).
    //      Lanes past the end of the block's edges load the last edge (finite data) and
    //      aggregate into the unused slot 31.
    struct Idx { int di, sj; };
    auto load_idx = [&](int t0) {
      const int p = min(t0 + r, e1 - 1);
      return Idx{a.dst[p], a.src[p]};
    };
    auto load_rows = [&](int t0, const Idx& ix, bf16x8_t (&bb)[8]) {
      const int p = min(t0 + r, e1 - 1);
      const uint16_t* pj = a.x + (size_t)ix.sj * a.ldx + 8 * h;
      const uint16_t* pe = a.e + (size_t)p * a.lde + 8 * h;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bb[s] = ld_bf8(pj + 16 * s);
        bb[4 + s] = ld_bf8(pe + 16 * s);
      }
    };
    auto compute = [&](const bf16x8_t (&b)[8], int slot, int t0) {
      f32x16 acc1[4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
        acc1[m] = ld_bias_frag(P + slot * PST, m, h);
      mfma_steps<8, 4, 12, 4>(b, acc1, w0, lane);  // k-steps 4..11: x[src], e
      f32x16 acc2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) acc2[m] = ld_bias_frag(bias1, m, h);
#ifndef RG_NO_FUSED_LEAKY
      if constexpr (ACT == ACT_LEAKY) {
        // the same values as norm_act + pack_acc (same fmas, same order), formed per k-step
        const f32x2 sc = norm_leaky_scale<4>(acc1, nrm[0], nrm[1], NORM_EPS);
        mfma_steps_jit<8, 2, 8, 0>([&](int s) {
          const f32x16& t = acc1[s >> 1];
          const int q = 8 * (s & 1);
          float v[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float y = fmaf(t[q + i], sc.x, sc.y);
            v[i] = fmaf(fabsf(y), LEAKY_C, y);
          }
          return __builtin_bit_cast(bf16x8_t, (u32x4){bf2(v[0], v[1]), bf2(v[2], v[3]),
                                                      bf2(v[4], v[5]), bf2(v[6], v[7])});
        }, acc2, w1, lane);
      } else
#endif
      {
        norm_act<ACT, 4>(acc1, a.L[0], nrm[0], nrm[1]);
        bf16x8_t b2[8];
        pack_acc<4>(acc1, b2);
        mfma_steps<8, 2, 8, 0>(b2, acc2, w1, lane);
      }
      norm_act<ACT, 2>(acc2, a.L[1], nrm[2], nrm[3]);
      // ---- message tile M -> LDS rows [edge][feature] (8-B stores of 4 features)
      const int sr = swz(r);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint2 wv;
          wv.x = bf2(acc2[m][4 * g + 0], acc2[m][4 * g + 1]);
          wv.y = bf2(acc2[m][4 * g + 2], acc2[m][4 * g + 3]);
          const int gr = (8 * m + 2 * g + h) ^ sr;
          *(uint2*)(tile + r * C + 4 * gr) = wv;
        }
      // slot r's edges in this tile: bits [sst - t0, sen - t0) of a 32-bit mask (edges past
      // the block's end belong to no slot)
      const int lo_b = min(max(sst - t0, 0), 32), hi_b = min(max(sen - t0, 0), 32);
      const uint32_t mhi = hi_b >= 32 ? 0xffffffffu : ((1u << hi_b) - 1u);
      const uint32_t mlo = lo_b >= 32 ? 0xffffffffu : ((1u << lo_b) - 1u);
      const uint32_t smask = mhi & ~mlo;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      // ---- Agg[feature][slot] += sum_edges M[feature][edge] * S[edge][slot]
      // A = M (features x edges) via ds_read_b64_tr_b16: lane 4q+p of each 16-lane
      // group G addresses row (edge) row0+q, granule col0/4+p; lane i of the group
      // receives column (feature) col0+i of the 4 rows.
      const int G = (lane >> 4) & 3, q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // B = S (k = edge 16s + 8h + j, col = slot r): one-hot bf16
        const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, lut[(smask >> (16 * s + 8 * h)) & 0xffu]);
        const int row_lo = 16 * s + 8 * (G >> 1) + q4, row_hi = row_lo + 4;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int gcol = 8 * m + 4 * (G & 1) + p4;
          typedef short v4s __attribute__((ext_vector_type(4)));
          typedef __attribute__((address_space(3))) v4s lds_v4s;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4s*)(tile + row_lo * C + 4 * (gcol ^ swz(row_lo))));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4s*)(tile + row_hi * C + 4 * (gcol ^ swz(row_hi))));
          const bf16x8_t mf = __builtin_bit_cast(
              bf16x8_t, (short __attribute__((ext_vector_type(8)))){lo[0], lo[1], lo[2], lo[3],
                                                                  hi[0], hi[1], hi[2], hi[3]});
          agg[m] = HT::mfma(mf, sf, agg[m]);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    };

    bf16x8_t bA[8], bB[8];
    Idx iA{0, 0}, iB{0, 0};
    if (e0 < e1) {
      iA = load_idx(e0);
      iB = load_idx(e0 + 32);  // clamped: harmless when the block has one tile
    }
    // ---- P[node] = W1[:, x_i part] x[node] + b1 for the block's nodes: the x_i = x[dst]
    //      third of the message MLP's first layer is the same for every edge into a node,
    //      so it is computed once per node here instead of once per edge
    {
      const int node = min(n0 + r, n1 - 1);
      const uint16_t* px = a.x + (size_t)node * a.ldx + 8 * h;
      bf16x8_t bx[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) bx[s] = ld_bf8(px + 16 * s);
      f32x16 accp[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) accp[m] = ld_bias_frag(bias0, m, h);
      // tile 0's rows go out while P is computed (their indices were issued above)
      if (e0 < e1) load_rows(e0, iA, bA);
      mfma_steps<4, 4, 12, 0>(bx, accp, w0, lane);
      if (r < NB) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          f32x4* pw = (f32x4*)(P + r * PST + (2 * m + h) * 16);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            pw[q] = (f32x4){accp[m][4 * q], accp[m][4 * q + 1], accp[m][4 * q + 2], accp[m][4 * q + 3]};
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): P visible to the whole wave
      __builtin_amdgcn_wave_barrier();
    }
    CSTAMP(1);

    int nxt = 0;
    int ne0 = 0, ne1 = 0, nn0 = 0, nn1 = 0;
    if (a.wave_nodes) {
      nn0 = n1;
      nn1 = min(n1 + NB, s_hi);
      nxt = nn0 < s_hi ? 0 : -1;
    } else {
      nxt = blo + __builtin_amdgcn_readfirstlane(nxt_raw);
      if (nxt >= bhi) nxt = -1;
      if (nxt >= 0) block_nodes(nxt, nn0, nn1);
    }
    if (nxt >= 0) {
      ne0 = a.seg_ptr[nn0];
      ne1 = a.seg_ptr[nn1];
    }

    // The next tile's rows and the tile after's indices are loaded UNCONDITIONALLY
    // (clamped to the block's last edge: past the end every lane reads one row): a load
    // under a branch leaves the compiler unsure how many loads are in flight at the
    // join, and it then waits for the freshly issued prefetch before this tile's MFMAs.
    if (e0 < e1) {
      for (int t0 = e0;;) {
        const int slotA = iA.di - n0;
        load_rows(t0 + 32, iB, bB);
        iA = load_idx(t0 + 64);
        compute(bA, slotA, t0);
        t0 += 32;
        if (t0 >= e1) break;
        const int slotB = iB.di - n0;
        load_rows(t0 + 32, iA, bA);
        iB = load_idx(t0 + 64);
        compute(bB, slotB, t0);
        t0 += 32;
        if (t0 >= e1) break;
      }
    }
#if RG_CONV_STAMP
    CSTAMP(2);
    st_acc[4] += 1;
    st_acc[5] += (e1 - e0 + 31) / 32;
#endif
    // ---- update MLP on cat(x[node], agg[node]) + residual (gnn_blocks.py:103-109)
    const int node = n0 + r;
    const bool nvalid = r < NB && node < n1;
    if (a.aggr_mean) {
      // PyG mean: sum / max(count, 1)
      const int deg = nvalid ? a.seg_ptr[node + 1] - a.seg_ptr[node] : 1;
      const float cnt = (float)(deg > 0 ? deg : 1);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 16; ++q) agg[m][q] = div_rn(agg[m][q], cnt);
    }
    bf16x8_t bu[8];
    const uint16_t* px = a.x + (size_t)(nvalid ? node : n0) * a.ldx + 8 * h;
#pragma unroll
    for (int s = 0; s < 4; ++s) bu[s] = ld_bf8(px + 16 * s);
    pack_acc<2>(agg, bu + 4);
    f32x16 accu[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) accu[m] = ld_bias_frag(bias2, m, h);
    mfma_steps<8, 2, 8, 0>(bu, accu, w2, lane);
    norm_act<ACT, 2>(accu, a.L[2], nrm[4], nrm[5]);
    if (nvalid) {
      // (row offsets with the lane's 4 h folded in: pointer + lane-offset pairs hoisted out of
      //  the block loop were the kernel's spilled 64-bit values)
      uint16_t* po = a.x_out + ((size_t)node * a.ldo + 4 * h);
      const uint16_t* pr = a.x + ((size_t)node * a.ldx + 4 * h);
      // all residual loads first: interleaved with the stores, each load would wait
      // for the previous store (possible aliasing) -- eight serial round trips
      uint2 rv[2][4];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) rv[m][g] = *(const uint2*)(pr + 32 * m + 8 * g);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int f0 = 32 * m + 8 * g + 4 * h;
          const uint2 r2 = rv[m][g];
          const float v0 = __fadd_rn(HT::lo(r2.x), accu[m][4 * g + 0]);
          const float v1 = __fadd_rn(HT::hi(r2.x), accu[m][4 * g + 1]);
          const float v2 = __fadd_rn(HT::lo(r2.y), accu[m][4 * g + 2]);
          const float v3 = __fadd_rn(HT::hi(r2.y), accu[m][4 * g + 3]);
          uint2 o;
          o.x = bf2(v0, v1);
          o.y = bf2(v2, v3);
          *(uint2*)(po + (f0 - 4 * h)) = o;
        }
    }
#if RG_CONV_STAMP
    __builtin_amdgcn_s_waitcnt(0);
#endif
    CSTAMP(3);
    blk = nxt;
    e0 = ne0;
    e1 = ne1;
    bn0 = nn0;
    bn1 = nn1;
  }
  // the last workgroup out re-zeroes the block counter for the next launch (no memset
  // per layer: each cost a ~10 us stream gap).  Every wave's final counter atomic has
  // returned before its workgroup reaches the barrier, so when `done` reaches the grid
  // size no workgroup can touch the counter again.
  __syncthreads();
#if RG_CONV_STAMP
  CSTAMP(6);
  if (lane == 0) {
    for (int i = 0; i < 8; ++i) atomicAdd(&g_conv_stamp[i], st_acc[i]);
    atomicMin(&g_conv_stamp[8], st_rt0);
    atomicMax(&g_conv_stamp[9], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
#endif
  if (threadIdx.x == 0) {
    if (atomicAdd(a.counter + CTR_STRIDE * NQ, 1) == (int)gridDim.x - 1) {
#pragma unroll
      for (int q = 0; q <= NQ; ++q) atomicExch(a.counter + CTR_STRIDE * q, 0);
    }
  }
}

// Edge-balanced work blocks: each run of NB nodes is split at node boundaries wherever
// its running edge count would pass `cap` (a single node is never split), so no work
// block holds many more edges than the mean share of a wave.  cap = max(CAP_MIN, E / 4096)
// (4096 = two blocks per wave of the 256 x 8-wave grid): a 20 000-node radius frame
// (~160 edges per 8 nodes, hubs of ~100) is cut to ~4-tile blocks, while a C2 batch
// (~300 edges per 8 nodes, cap 1 778) keeps its 8-node runs.
static constexpr int CAP_MIN = 128;

__device__ __forceinline__ int block_cap(const int* seg_ptr, int n_nodes, int cap_min,
                                         int cap_div) {
  return max(cap_min, seg_ptr[n_nodes] / cap_div);
}

// the static schedule's per-node cost in edge units (the block head (P) and update of an
// NB-node block, per node)
static constexpr int WAVE_NODE_COST = 4;
__global__ void conv_wave_nodes_kernel(const int* __restrict__ seg_ptr, int n_nodes, int n_waves,
                                       int node_cost, int* __restrict__ wave_nodes) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_waves) return;
  // first node n with cost(n) = seg_ptr[n] + node_cost n >= total i / n_waves
  const long total = (long)seg_ptr[n_nodes] + (long)node_cost * n_nodes;
  const long target = total * i / n_waves;
  int lo = 0, hi = n_nodes;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((long)seg_ptr[mid] + (long)node_cost * mid < target) lo = mid + 1;
    else hi = mid;
  }
  wave_nodes[i] = i == n_waves ? n_nodes : lo;
}

template <bool EMIT>
__global__ void conv_blocks_kernel(const int* __restrict__ seg_ptr, int n_nodes,
                                   int* __restrict__ cnt, const int* __restrict__ off,
                                   int* __restrict__ blk_nodes, int cap_min, int cap_div) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int nb8 = (n_nodes + NB - 1) / NB;
  if (b >= nb8) return;
  const int cap = block_cap(seg_ptr, n_nodes, cap_min, cap_div);
  const int n0 = b * NB, n1 = min(n0 + NB, n_nodes);
  int c = 0, acc = 0, o = EMIT ? off[b] : 0;
  for (int n = n0; n < n1; ++n) {
    const int d = seg_ptr[n + 1] - seg_ptr[n];
    if (n == n0 || (acc > 0 && acc + d > cap)) {
      if (EMIT) blk_nodes[o + c] = n;
      ++c;
      acc = 0;
    }
    acc += d;
  }
  if (!EMIT) cnt[b] = c;
  if (EMIT && b == nb8 - 1) blk_nodes[o + c] = n_nodes;  // sentinel
}

#if RG_CONV_STAMP
static int conv_stamps(unsigned long long* out_host) {
  RG_CHECK_HIP(hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_conv_stamp), sizeof(g_conv_stamp)));
  unsigned long long z[16] = {0};
  z[8] = ~0ull;
  RG_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_conv_stamp), z, sizeof(z)));
  return RG_OK;
}
#endif

// the C-ABI entry of this operand type (rg_conv_layer_fused_blocks dispatches on RG_LAYER_F16)
static int conv_fused_entry(const rg_layer* msg_layers, const rg_layer* upd_layer,
                                          int aggr, const void* x, int ldx, const void* e,
                                          int lde, const int* seg_ptr, const int* src,
                                          const int* dst, int n_nodes, void* x_out, int ld_out,
                                          const int* blk_nodes, const int* n_blocks_dev,
                                          const int* wave_nodes, int n_waves,
                                          void* workspace, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const rg_layer& m0 = msg_layers[0];
  const rg_layer& m1 = msg_layers[1];
  const rg_layer& u = *upd_layer;
  if (!(m0.in_dim == 3 * C && m0.out_dim == HID && m1.in_dim == HID && m1.out_dim == C &&
        u.in_dim == 2 * C && u.out_dim == C))
    return RG_ERR_UNSUPPORTED;
  if (aggr != RG_REDUCE_SUM && aggr != RG_REDUCE_MEAN) return RG_ERR_UNSUPPORTED;
  if (!m0.norm_mu || !m1.norm_mu || !u.norm_mu) return RG_ERR_UNSUPPORTED;  // norm assumed
  RG_REQUIRE(ldx % 8 == 0 && lde % 8 == 0 && ld_out % 8 == 0, RG_ERR_UNSUPPORTED,
             "rg_conv_layer_fused: strides must be multiples of 8");
  RG_REQUIRE(x != x_out, RG_ERR_ARG, "rg_conv_layer_fused: x_out must not alias x");
  CArgs a;
  memset(&a, 0, sizeof(a));
  const rg_layer* ls[3] = {&m0, &m1, &u};
  const int fmts[3] = {RG_PACK_FAST_IN, RG_PACK_FAST_CHAIN, RG_PACK_FAST_UPD};
  int off = 0;
  for (int l = 0; l < 3; ++l) {
    a.L[l].src = ls[l]->w_packed;
    a.L[l].mu = ls[l]->norm_mu;
    a.L[l].sd = ls[l]->norm_std;
    a.L[l].woff = off;
    a.L[l].bytes = (int)rg_packed_linear_bytes(ls[l]->in_dim, ls[l]->out_dim, fmts[l]);
    a.L[l].out = ls[l]->out_dim;
    a.L[l].act = ls[l]->act;
    a.L[l].centered = (ls[l]->flags & RG_LAYER_CENTERED) ? 1 : 0;
    off += (a.L[l].bytes + 15) & ~15;
  }
  a.total_bytes = off;
  a.aggr_mean = aggr == RG_REDUCE_MEAN;
  a.n_nodes = n_nodes;
  a.n_blocks = (n_nodes + NB - 1) / NB;
  a.x = (const uint16_t*)x;
  a.e = (const uint16_t*)e;
  a.seg_ptr = seg_ptr;
  a.src = src;
  a.dst = dst;
  a.x_out = (uint16_t*)x_out;
  a.counter = (int*)workspace;  // NQ heads + workgroups done: zero between launches
  a.ldx = ldx; a.lde = lde; a.ldo = ld_out;
  RG_REQUIRE((blk_nodes == nullptr) == (n_blocks_dev == nullptr), RG_ERR_ARG,
             "rg_conv_layer_fused_blocks: block table and count go together");
  a.blk_nodes = blk_nodes;
  a.n_blk_dev = n_blocks_dev;
  RG_REQUIRE(!wave_nodes || (!blk_nodes && n_waves >= CW * NQ && n_waves % (CW * NQ) == 0),
             RG_ERR_ARG, "rg_conv_layer_fused_waves: n_waves %d must be a multiple of %d", n_waves,
             CW * NQ);
  a.wave_nodes = wave_nodes;
  if (n_nodes <= 0) return RG_OK;
  const size_t lds = (size_t)off + LUT_BYTES + (size_t)CW * WAVE_LDS;
  RG_REQUIRE(lds <= DYN_LDS_MAX, RG_ERR_UNSUPPORTED, "rg_conv_layer_fused: LDS %zu", lds);
  // the yml activation (LeakyReLU, configuration_radarscenes_gnn.yml:50) on all three
  // blocks selects the compile-time variant; anything else dispatches per layer
  const bool leaky = m0.act == ACT_LEAKY && m1.act == ACT_LEAKY && u.act == ACT_LEAKY &&
                     (m0.flags & m1.flags & u.flags & RG_LAYER_CENTERED);
  auto kern = leaky ? fused_conv_kernel<ACT_LEAKY> : fused_conv_kernel<-1>;
  RG_ENSURE_LDS(kern, DYN_LDS_MAX);
  int blocks = 256;  // a block table has at least ceil(N / NB) entries
  if (blocks * CW > a.n_blocks) blocks = (a.n_blocks + CW - 1) / CW;
  blocks = (blocks + NQ - 1) / NQ * NQ;  // every head has workgroups of its own
  if (wave_nodes) blocks = n_waves / CW;  // one workgroup per CW ranks of the schedule
  kern<<<blocks, CT, lds, st>>>(a);
  const hipError_t le = hipGetLastError();
  if (le != hipSuccess) {
    // a launch that did not run leaves the counters as they were; one that failed part
    // way could leave them nonzero: re-zero so the next launch does not skip blocks
    (void)hipMemsetAsync(workspace, 0, (CTR_STRIDE * NQ + 1) * sizeof(int), st);
    set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__, hipGetErrorString(le));
    return RG_ERR_HIP;
  }
  return RG_OK;
}

}  // namespace RG_CONV_NS
}  // namespace rg
