// Register-resident FLOAT32 MLP chains on the bf16 matrix cores (x3_common.h: every
// product from the exact three-term bf16 splits of both operands, f32 accumulation) for
// the widths of the shipped architecture: the fp32 path's node / edge encoders
// (graph_feature_encoding, gnn_blocks.py:19-42) and the task-head chains
// (gnn_blocks.py:167-389).  Same semantics as rg_mlp_chain_f32 (ffn_block chains: Linear
// -> channel_normalization -> activation, common.py:185-220).
//
//  * a wave owns RT tiles of 32 rows; a layer's accumulators, split into their bf16 terms,
//    are the next layer's B operand in registers (RG_PACK_FAST_CHAIN k order), so
//    activations never leave registers between layers;
//  * the encoders' un-normalised first layer (<= 8 inputs) is fused tile by tile into the
//    second: each 32-feature output tile of layer 0 is activated, split and consumed at
//    once as two k-steps of layer 1 (the 256-wide activation never exists in full);
//  * packed weights (RG_PACK_X3) are staged in LDS per layer and plane where they fit
//    (LMASK, 3 bits per layer); the rest is read from L2 through a buffer resource.  The
//    7 -> 256 -> 128 -> 128 -> 64 edge encoder is 361 KiB of split weights: layer 0 and
//    planes 0 / 1 of layer 1 (153 KiB) live in LDS, the others stream from L2, and two
//    row tiles per wave halve that stream per flop.
#include "x3_common.h"

namespace rg {
namespace cx3 {

using namespace ::rg::x3;

#ifndef RG_X3_DB
#define RG_X3_DB 1  // weight fragments read this many k-steps ahead in the chained layers
                    // (1 vs 0, M: edge encoder 1.52 -> 1.45 ms)
#endif
#ifndef RG_X3_DB_MT2
#define RG_X3_DB_MT2 RG_X3_DB  // the same for layers of <= 2 M-tiles (a k-step of 6 MT RT MFMAs
                               // is then shorter than an L2 round trip)
#endif
template <int MT>
constexpr int x3_db() {
  return MT <= 2 ? RG_X3_DB_MT2 : RG_X3_DB;
}

enum { IN_SMALL = 0,   // float32 rows of <= 8 features; layer 0 (no norm) fused into layer 1
       IN_DENSE = 1,   // float32 rows, K0 % 16 == 0
       IN_PAIR = 2,    // float32 x[idx0[r]] + x[idx1[r]] (edge_formation, gnn_blocks.py:297)
       IN_PAIRPRE = 3 };  // layer 0's pre-activation t[idx0[r]] + t[idx1[r]] + b0 from per-node
                          // rows t = W0 x (RG_IN_PAIRPRE: layer 0's weights are not read)

// SPEC: bit l = layer l normalised, bit 8 + l = activated (LeakyReLU), bit 16 = every
// normalised layer packed centred (RG_LAYER_CENTERED)
constexpr int spec(int norm_mask, int act_mask, bool centred = false) {
  return norm_mask | (act_mask << 8) | (centred ? 1 << 16 : 0);
}
constexpr bool sp_norm(int sp, int l) { return ((sp >> l) & 1) != 0; }
constexpr bool sp_act(int sp, int l) { return ((sp >> (8 + l)) & 1) != 0; }
constexpr bool sp_cent(int sp) { return ((sp >> 16) & 1) != 0; }
constexpr int lmask(int m, int l) { return (m >> (3 * l)) & 7; }

template <int K0, int... Ns>
struct Shape {
  static constexpr int NL = sizeof...(Ns);
  static constexpr int N[NL] = {Ns...};
  static constexpr int K(int l) { return l == 0 ? K0 : N[l - 1]; }
  static constexpr int pl(int l) { return plane_bytes(K(l), N[l]); }
  static constexpr int bytes(int l) { return x3_bytes(K(l), N[l]); }
  // LDS image: every layer's staged planes, then every layer's bias
  static constexpr int planes_lds(int LM, int l) {
    return (lmask(LM, l) & 1) + ((lmask(LM, l) >> 1) & 1) + ((lmask(LM, l) >> 2) & 1);
  }
  static constexpr int woff(int LM, int l) {
    int o = 0;
    for (int i = 0; i < l; ++i) o += planes_lds(LM, i) * pl(i);
    return o;
  }
  static constexpr int boff(int LM, int l) {
    int o = woff(LM, NL);
    for (int i = 0; i < l; ++i) o += N[i] * 4;
    return o;
  }
  static constexpr int lds_bytes(int LM) { return boff(LM, NL); }
};

struct Layer {
  const char* src;  // x3 image (global)
  const float* mu;
  const float* sd;
};

struct Args {
  Layer L[RG_MAX_LAYERS];
  long rows;
  const int* rows_dev;
  const float* in0;
  int ld0, w0real;
  const int* idx0;
  const int* idx1;
  float* out;
  int ld_out, out_real;
};

// the weight source of layer l: LDS planes where staged (in plane order), else L2
template <int LM, int l>
struct Src {
  const char* lds;  // LDS base + lane * 16 of the layer's first staged plane
  int pl;
  WBuf g;
  __device__ __forceinline__ bf16x8_t operator()(int plane, int off) const {
    constexpr int m = lmask(LM, l);
    if ((m >> plane) & 1) {
      const int slot = plane == 0 ? 0 : (plane == 1 ? (m & 1) : (m & 1) + ((m >> 1) & 1));
      return ld_bf8(lds + slot * pl + off);
    }
    return g(plane, off);
  }
};

template <typename S, int LM, int l>
__device__ __forceinline__ Src<LM, l> src_of(const Args& a, const char* lds, int lane) {
  return Src<LM, l>{lds + S::woff(LM, l) + lane * 16, S::pl(l),
                    wbuf(a.L[l].src, S::bytes(l), S::pl(l), lane)};
}

template <int SPEC, int l, int MT>
__device__ __forceinline__ void epilogue(f32x16 (&acc)[MT], const float* nrm) {
  if constexpr (sp_norm(SPEC, l) && sp_act(SPEC, l)) {
    norm_leaky<MT, sp_cent(SPEC)>(acc, nrm[2 * l], nrm[2 * l + 1]);
  } else if constexpr (sp_norm(SPEC, l)) {
    norm_only<MT, sp_cent(SPEC)>(acc, nrm[2 * l], nrm[2 * l + 1]);
  } else if constexpr (sp_act(SPEC, l)) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] = act_t<ACT_LEAKY>(acc[m][q]);
  }
}

template <int RT, int MT, bool FULL = false>
__device__ __forceinline__ void store_rows(const f32x16 (&acc)[RT][MT], const Args& a, long row0,
                                           long rows, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int out = a.out_real;
  if constexpr (FULL) {
    // full-width, 16-B aligned rows (host-checked): branch-free buffer stores, a row past the
    // end dropped by the hardware (offset past the buffer) -- the compiler then counts these
    // stores, and the next tile's wait for its prefetched inputs does not wait for them too
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        a.out, 0, (int)(((rows - 1) * a.ld_out + 32 * MT) * 4), 0x00020000);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const long row = row0 + 32 * t + r;
      const int off = row < rows ? (int)((row * a.ld_out + 4 * h) * 4) : 0x7ffff000;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          const u32x4_t v = {__float_as_uint(acc[t][m][4 * g]), __float_as_uint(acc[t][m][4 * g + 1]),
                             __float_as_uint(acc[t][m][4 * g + 2]), __float_as_uint(acc[t][m][4 * g + 3])};
          __builtin_amdgcn_raw_buffer_store_b128(v, rs, off + (32 * m + 8 * g) * 4, 0, 0);
        }
    }
    return;
  }
  // every feature of the tile stored whole in 16-B pieces (wave-uniform: the encoders' rows),
  // else piece by piece below (padded head outputs; the per-lane test there costs a divergent
  // branch and a saved mask per piece)
  if (out >= 32 * MT && (a.ld_out & 3) == 0) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const long row = row0 + 32 * t + r;
      if (row >= rows) continue;
      float* o = a.out + (size_t)row * a.ld_out + 4 * h;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *(f32x4*)(o + 32 * m + 8 * g) = (f32x4){acc[t][m][4 * g], acc[t][m][4 * g + 1],
                                                  acc[t][m][4 * g + 2], acc[t][m][4 * g + 3]};
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const long row = row0 + 32 * t + r;
    if (row >= rows) continue;
    float* o = a.out + (size_t)row * a.ld_out;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int f0 = 32 * m + 8 * g + 4 * h;
        if (f0 + 4 <= out && (a.ld_out & 3) == 0) {
          *(f32x4*)(o + f0) = (f32x4){acc[t][m][4 * g], acc[t][m][4 * g + 1], acc[t][m][4 * g + 2],
                                      acc[t][m][4 * g + 3]};
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (f0 + u < out) o[f0 + u] = acc[t][m][4 * g + u];
        }
      }
  }
}

#ifndef RG_X3_INPF
#define RG_X3_INPF 1  // encoders: the next tile's input rows loaded during this tile's last layer
#endif
#ifndef RG_X3_ENC_BUF
#define RG_X3_ENC_BUF 1  // encoders: output rows by branch-free buffer stores, next-tile inputs loaded
                         // unconditionally and masked at use (counted waits; host-checked sizes)
#endif
#ifndef RG_X3_SKEW
#define RG_X3_SKEW 1  // row tile 1's epilogue issued under row tile 0's first k-step of the next
                      // layer (layer_x3's pre1) when a wave holds two row tiles (M edge encoder
                      // 1.362 -> 1.347 ms, three interleaved rounds, profiles/r05_enc_skew_ab.log)
#endif

#ifndef RG_X3_JIT
#define RG_X3_JIT 1  // a normalised layer's scale + act applied in the next layer's B operand
#endif
// what layer l leaves pending for the next one (split_acc_pend): 1 norm + LeakyReLU,
// 2 norm only, 0 nothing (its epilogue, if any, runs in full)
template <int SPEC, int l>
constexpr int pend_kind() {
  return !RG_X3_JIT ? 0 : (sp_norm(SPEC, l) && sp_act(SPEC, l)) ? 1 : sp_norm(SPEC, l) ? 2 : 0;
}
// layer l's epilogue when a next layer follows: statistics only for a pending kind
template <int SPEC, int l, int MT, int RT>
__device__ __forceinline__ void epilogue_pend(f32x16 (&acc)[RT][MT], const float* nrm,
                                              Pend (&pn)[RT]) {
  constexpr int K = pend_kind<SPEC, l>();
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    if constexpr (K == 1) {
      pn[t] = pend_norm_leaky<MT, sp_cent(SPEC)>(acc[t], nrm[2 * l], nrm[2 * l + 1]);
    } else if constexpr (K == 2) {
      pn[t] = pend_norm_only<MT, sp_cent(SPEC)>(acc[t], nrm[2 * l], nrm[2 * l + 1]);
    } else {
      epilogue<SPEC, l, MT>(acc[t], nrm);
      pn[t] = Pend{0.f, 0.f};
    }
  }
}

// epilogue_pend of row tile t only
template <int SPEC, int l, int MT>
__device__ __forceinline__ void epilogue_pend_one(f32x16 (&acc)[MT], const float* nrm, Pend& pn) {
  constexpr int K = pend_kind<SPEC, l>();
  if constexpr (K == 1) {
    pn = pend_norm_leaky<MT, sp_cent(SPEC)>(acc, nrm[2 * l], nrm[2 * l + 1]);
  } else if constexpr (K == 2) {
    pn = pend_norm_only<MT, sp_cent(SPEC)>(acc, nrm[2 * l], nrm[2 * l + 1]);
  } else {
    epilogue<SPEC, l, MT>(acc, nrm);
    pn = Pend{0.f, 0.f};
  }
}
// a layer's epilogue before the next layer: every row tile, or with RG_X3_SKEW at two row
// tiles only tile 0 (tile 1's runs as the next layer_x3's pre1)
template <int SPEC, int l, int MT, int RT>
__device__ __forceinline__ void epilogue_next(f32x16 (&acc)[RT][MT], const float* nrm,
                                              Pend (&pn)[RT]) {
  if constexpr (RG_X3_SKEW && RT == 2) {
    epilogue_pend_one<SPEC, l, MT>(acc[0], nrm, pn[0]);
    pn[1] = Pend{0.f, 0.f};
  } else {
    epilogue_pend<SPEC, l, MT, RT>(acc, nrm, pn);
  }
}

// layers l.. of the chain; prev = the previous layer's activations (RT row tiles), with
// the previous layer's norm / act still pending (PEND) where pend_kind says so (with
// RG_X3_SKEW at RT = 2: row tile 1's epilogue of layer l - 1 not yet run at all)
// pre: run after the last layer's MFMAs are issued, before its epilogue (the encoders' next-tile
// input loads: the only loads then in flight, so no weight wait stalls behind them)
template <typename S, int SPEC, int LM, int l, int RT, int PMT, int PEND, bool FULL = false,
          typename Pre = NoHook>
__device__ __forceinline__ void run_rest(const Args& a, f32x16 (&prev)[RT][PMT], Pend (&pend)[RT],
                                         const char* lds, const float* nrm, long row0, long rows,
                                         int lane, Pre&& pre = Pre{}) {
  constexpr int N = S::N[l], MT = N / 32, KS = S::K(l) / 16;
  static_assert(S::K(l) == 32 * PMT, "chained width");
  const int h = lane >> 5;
  const float* bias = (const float*)(lds + S::boff(LM, l));
  f32x16 acc[RT][MT];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = ld_bias_frag(bias, m, h);
  auto bop = [&](int s, int t) { return split_acc_pend<PEND>(prev[t][s >> 1], s & 1, pend[t]); };
  if constexpr (RG_X3_SKEW && RT == 2) {
    layer_x3<KS, MT, MT, RT, x3_db<MT>()>(acc, src_of<S, LM, l>(a, lds, lane), 0, bop, [&]() {
      epilogue_pend_one<SPEC, l - 1, PMT>(prev[1], nrm, pend[1]);
    });
  } else {
    layer_x3<KS, MT, MT, RT, x3_db<MT>()>(acc, src_of<S, LM, l>(a, lds, lane), 0, bop);
  }
  if constexpr (l + 1 < S::NL) {
    Pend pn[RT];
    epilogue_next<SPEC, l, MT, RT>(acc, nrm, pn);
    run_rest<S, SPEC, LM, l + 1, RT, MT, pend_kind<SPEC, l>(), FULL>(a, acc, pn, lds, nrm, row0,
                                                                    rows, lane, pre);
  } else {
    pre();
#pragma unroll
    for (int t = 0; t < RT; ++t) epilogue<SPEC, l, MT>(acc[t], nrm);
    store_rows<RT, MT, FULL>(acc, a, row0, rows, lane);
  }
}

// layer 0 over split inputs b0[t][s] (KS0 k-steps)
template <typename S, int SPEC, int LM, int RT, int KS0>
__device__ __forceinline__ void run_first(const Args& a, const X3 (&b0)[RT][KS0], const char* lds,
                                          const float* nrm, long row0, long rows, int lane) {
  constexpr int N = S::N[0], MT = N / 32;
  const int h = lane >> 5;
  const float* bias = (const float*)(lds + S::boff(LM, 0));
  f32x16 acc[RT][MT];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = ld_bias_frag(bias, m, h);
  layer_x3<KS0, MT, MT, RT, x3_db<MT>()>(acc, src_of<S, LM, 0>(a, lds, lane), 0,
                                  [&](int s, int t) { return b0[t][s]; });
  if constexpr (S::NL > 1) {
    Pend pn[RT];
    epilogue_next<SPEC, 0, MT, RT>(acc, nrm, pn);
    run_rest<S, SPEC, LM, 1, RT, MT, pend_kind<SPEC, 0>()>(a, acc, pn, lds, nrm, row0, rows, lane);
  } else {
#pragma unroll
    for (int t = 0; t < RT; ++t) epilogue<SPEC, 0, MT>(acc[t], nrm);
    store_rows<RT, MT>(acc, a, row0, rows, lane);
  }
}

// RG_IN_PAIRPRE: layer 0 is linear before its norm, W0 (x_i + x_j) + b0 = t_i + t_j + b0 with
// t = W0 x per NODE (rg_mlp_chain_x3 over the nodes, a bare last layer): the pair chain starts
// from the gathered sum -- no layer-0 MFMAs and no split of the pair input (the link head's
// pairs outnumber the nodes ~6x)
template <typename S, int SPEC, int LM, int RT>
__device__ __forceinline__ void run_pre(const Args& a, const char* lds, const float* nrm, long row0,
                                        long rows, int lane) {
  constexpr int N = S::N[0], MT = N / 32;
  static_assert(S::K(0) == N, "per-node rows t have layer 0's output width");
  const int r = lane & 31, h = lane >> 5;
  const float* bias = (const float*)(lds + S::boff(LM, 0));
  f32x16 acc[RT][MT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const long row = row0 + 32 * t + r;
    const bool ok = row < rows;
    const int i = ok ? a.idx0[row] : 0, j = ok ? a.idx1[row] : 0;
    const float* pi = a.in0 + (size_t)i * a.ld0 + 4 * h;
    const float* pj = a.in0 + (size_t)j * a.ld0 + 4 * h;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const f32x16 b = ld_bias_frag(bias, m, h);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 ti = *(const f32x4*)(pi + 32 * m + 8 * g);
        const f32x4 tj = *(const f32x4*)(pj + 32 * m + 8 * g);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[t][m][4 * g + u] = __fadd_rn(__fadd_rn(ti[u], tj[u]), b[4 * g + u]);
      }
    }
  }
  static_assert(S::NL > 1, "a pair chain continues after layer 0");
  Pend pn[RT];
  epilogue_next<SPEC, 0, MT, RT>(acc, nrm, pn);
  run_rest<S, SPEC, LM, 1, RT, MT, pend_kind<SPEC, 0>()>(a, acc, pn, lds, nrm, row0, rows, lane);
}

// encoders: layer 0 (one k-step of <= 8 inputs, no normalisation) fused tile by tile into
// layer 1: tile m0 of layer 0 is layer 1's k-steps 2 m0 and 2 m0 + 1
template <typename S, int SPEC, int LM, int RT, typename Pre = NoHook>
__device__ __forceinline__ void run_fused01(const Args& a, const X3 (&b0)[RT][1], const char* lds,
                                            const float* nrm, long row0, long rows, int lane,
                                            Pre&& pre = Pre{}) {
  constexpr int MT0 = S::N[0] / 32, MT1 = S::N[1] / 32, KS1 = S::N[0] / 16;
  static_assert(S::K(0) <= 16, "fused first layer takes one k-step");
  static_assert(!sp_norm(SPEC, 0), "fused first layer is not normalised");
  const int h = lane >> 5;
  const float* bias0 = (const float*)(lds + S::boff(LM, 0));
  const float* bias1 = (const float*)(lds + S::boff(LM, 1));
  const auto W0 = src_of<S, LM, 0>(a, lds, lane);
  const auto W1 = src_of<S, LM, 1>(a, lds, lane);
  f32x16 acc[RT][MT1];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int m = 0; m < MT1; ++m) acc[t][m] = ld_bias_frag(bias1, m, h);
  // layer-1 A fragments of layer-0 tile m0 (k-steps 2 m0, 2 m0 + 1), read one tile ahead
  auto lda1 = [&](int m0, bf16x8_t (&d)[2][MT1][3]) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int m = 0; m < MT1; ++m)
#pragma unroll
        for (int p = 0; p < 3; ++p) d[hf][m][p] = W1(p, (m * KS1 + 2 * m0 + hf) * 1024);
  };
  // (measured: rolling this loop two tiles per iteration, 67 -> 47 KB of code, made the
  // edge encoder 12 % slower)
  bf16x8_t A1[2][2][MT1][3];
  lda1(0, A1[0]);
#pragma unroll
  for (int m0 = 0; m0 < MT0; ++m0) {
    const int u = m0 & 1;
    if (m0 + 1 < MT0) lda1(m0 + 1, A1[(u + 1) & 1]);
    f32x16 y[RT][1];
#pragma unroll
    for (int t = 0; t < RT; ++t) y[t][0] = ld_bias_frag(bias0, m0, h);
    layer_x3<1, 1, MT0, RT>(y, W0, m0, [&](int, int t) { return b0[t][0]; });
    if constexpr (sp_act(SPEC, 0)) {
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) y[t][0][q] = act_t<ACT_LEAKY>(y[t][0][q]);
    }
    // layer-1 k-steps 2 m0, 2 m0 + 1 from this tile
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bf16x8_t(&A)[MT1][3] = A1[u][hf];
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const X3 b = split_acc(y[t][0], hf);
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[t][m] = mf(A[m][2], b.p0, acc[t][m]);
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[t][m] = mf(A[m][1], b.p1, acc[t][m]);
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[t][m] = mf(A[m][0], b.p2, acc[t][m]);
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[t][m] = mf(A[m][1], b.p0, acc[t][m]);
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[t][m] = mf(A[m][0], b.p1, acc[t][m]);
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[t][m] = mf(A[m][0], b.p0, acc[t][m]);
      }
    }
    // (the last tile unfenced, as layer_x3: layer 1's epilogue of row tile 0 may interleave
    // with tile 1's last MFMAs)
    if (m0 + 1 < MT0) __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (S::NL > 2) {
    Pend pn[RT];
    epilogue_next<SPEC, 1, MT1, RT>(acc, nrm, pn);
    run_rest<S, SPEC, LM, 2, RT, MT1, pend_kind<SPEC, 1>(), RG_X3_ENC_BUF>(a, acc, pn, lds, nrm, row0,
                                                                         rows, lane, pre);
  } else {
    pre();
#pragma unroll
    for (int t = 0; t < RT; ++t) epilogue<SPEC, 1, MT1>(acc[t], nrm);
    store_rows<RT, MT1, RG_X3_ENC_BUF>(acc, a, row0, rows, lane);
  }
}

template <int MODE, int SPEC, int LM, int RT, int FT, int K0, int... Ns>
__global__ __launch_bounds__(FT) void chain_x3_kernel(Args a) {
  using S = Shape<K0, Ns...>;
  constexpr int NL = S::NL;
  constexpr int KS0 = (MODE == IN_SMALL || MODE == IN_PAIRPRE) ? 1 : K0 / 16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[2 * RG_MAX_LAYERS];
  if (threadIdx.x == 0) {
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      nrm[2 * l] = a.L[l].mu ? *a.L[l].mu : 0.f;
      nrm[2 * l + 1] = a.L[l].sd ? *a.L[l].sd : 0.f;
    }
  }
  // stage the LDS planes and every bias (static layer indices: no scratch copy of a.L)
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int m = lmask(LM, l);
    int slot = 0;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if ((m >> p) & 1) {
        stage_lds<FT>(lds + S::woff(LM, l) + slot * S::pl(l), a.L[l].src + p * S::pl(l), S::pl(l));
        ++slot;
      }
    }
    const u32x4* bsrc = (const u32x4*)(a.L[l].src + 3 * S::pl(l));
    u32x4* bdst = (u32x4*)(lds + S::boff(LM, l));
    for (int i = threadIdx.x; i < S::N[l] / 4; i += FT) bdst[i] = bsrc[i];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const long rows = a.rows_dev ? min((long)*a.rows_dev, a.rows) : a.rows;
  constexpr int TROWS = 32 * RT;
  const long ntiles = (rows + TROWS - 1) / TROWS;
  const long tstride = (long)gridDim.x * (FT / 64);
  // IN_SMALL (the encoders, <= 8 inputs per row): this tile's raw rows, loaded during the
  // previous tile's last layer (RG_X3_INPF) instead of at the tile's start, where the HBM
  // round trip stood in front of the first MFMA with nothing else to issue
  float vin[RT][8];
  auto load_in = [&](long tl) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const long row = tl * TROWS + 32 * t + r;
      const bool ok = row < rows;
      const float* p = a.in0 + (size_t)(ok ? row : 0) * a.ld0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (RG_X3_ENC_BUF)
          vin[t][j] = p[min(j, a.w0real - 1)];  // unconditional (masked at use)
        else
          vin[t][j] = (ok && h == 0 && j < a.w0real) ? p[j] : 0.f;
      }
    }
  };
  if constexpr (MODE == IN_SMALL && RG_X3_INPF) {
    const long t0 = (long)blockIdx.x * (FT / 64) + wave;
    if (t0 < ntiles) load_in(t0);
    // nothing in flight at the loop entry: the loop-top wait for the prefetched rows is counted
    if constexpr (RG_X3_ENC_BUF) __builtin_amdgcn_s_waitcnt(0x0f70);
  }
  for (long tile = (long)blockIdx.x * (FT / 64) + wave; tile < ntiles; tile += tstride) {
    const long row0 = tile * TROWS;
    if constexpr (MODE == IN_PAIRPRE) {
      run_pre<S, SPEC, LM, RT>(a, lds, nrm, row0, rows, lane);
    } else {
    X3 b0[RT][KS0];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const long row = row0 + 32 * t + r;
      const bool ok = row < rows;
      if constexpr (MODE == IN_SMALL) {
        float v[8];
        if constexpr (RG_X3_INPF) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = (!RG_X3_ENC_BUF || (ok && h == 0 && j < a.w0real)) ? vin[t][j] : 0.f;
        } else {
          const float* p = a.in0 + (size_t)(ok ? row : 0) * a.ld0;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (ok && h == 0 && j < a.w0real) ? p[j] : 0.f;
        }
        b0[t][0] = split8((f32x4){v[0], v[1], v[2], v[3]}, (f32x4){v[4], v[5], v[6], v[7]});
      } else if constexpr (MODE == IN_DENSE) {
        const float* p = a.in0 + (size_t)(ok ? row : 0) * a.ld0 + 8 * h;
#pragma unroll
        for (int s = 0; s < KS0; ++s)
          b0[t][s] = split8(*(const f32x4*)(p + 16 * s), *(const f32x4*)(p + 16 * s + 4));
      } else {
        const int i = ok ? a.idx0[row] : 0, j = ok ? a.idx1[row] : 0;
        const float* pi = a.in0 + (size_t)i * a.ld0 + 8 * h;
        const float* pj = a.in0 + (size_t)j * a.ld0 + 8 * h;
#pragma unroll
        for (int s = 0; s < KS0; ++s) {
          f32x4 u[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const f32x4 xi = *(const f32x4*)(pi + 16 * s + 4 * k);
            const f32x4 xj = *(const f32x4*)(pj + 16 * s + 4 * k);
            u[k] = (f32x4){__fadd_rn(xi.x, xj.x), __fadd_rn(xi.y, xj.y), __fadd_rn(xi.z, xj.z),
                           __fadd_rn(xi.w, xj.w)};
          }
          b0[t][s] = split8(u[0], u[1]);
        }
      }
    }
    if constexpr (MODE == IN_SMALL && RG_X3_INPF)
      run_fused01<S, SPEC, LM, RT>(a, b0, lds, nrm, row0, rows, lane, [&]() {
        if (tile + tstride < ntiles) load_in(tile + tstride);
      });
    else if constexpr (MODE == IN_SMALL)
      run_fused01<S, SPEC, LM, RT>(a, b0, lds, nrm, row0, rows, lane);
    else
      run_first<S, SPEC, LM, RT, KS0>(a, b0, lds, nrm, row0, rows, lane);
    }
  }
}

template <int MODE, int SPEC, int LM, int RT, int FT, int K0, int... Ns>
static int launch(const Args& a, hipStream_t st) {
  using S = Shape<K0, Ns...>;
  constexpr int lds = S::lds_bytes(LM);
  static_assert(lds <= DYN_LDS_MAX, "chain_x3: LDS image too large");
  auto kern = chain_x3_kernel<MODE, SPEC, LM, RT, FT, K0, Ns...>;
  RG_ENSURE_LDS(kern, lds);
  const long tiles = (a.rows + 32 * RT - 1) / (32 * RT);
  long blocks = (tiles + FT / 64 - 1) / (FT / 64);
  const int per_cu = (FT <= 256 && lds <= 76 * 1024) ? 2 : 1;  // persistent
  if (blocks > 256L * per_cu) blocks = 256L * per_cu;
  if (blocks < 1) blocks = 1;
  kern<<<blocks, FT, lds, st>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

struct Key {
  int mode, k0, sp, nl;
  int n[RG_MAX_LAYERS];
};

static bool match(const Key& k, int mode, int k0, int sp, std::initializer_list<int> ns) {
  if (k.mode != mode || k.k0 != k0 || k.sp != sp || k.nl != (int)ns.size()) return false;
  int i = 0;
  for (int v : ns)
    if (k.n[i++] != v) return false;
  return true;
}

#ifndef RG_X3_ENC_RT
#define RG_X3_ENC_RT 2  // row tiles per wave of the encoders (1 wave / SIMD at 2)
#endif
#ifndef RG_X3_ENC_FT
#define RG_X3_ENC_FT 0  // encoder threads per workgroup (0: 256 at RT >= 2, else 512; RT 2 at 512,
                        // two waves per SIMD: 1.2 KB of spills per lane, not run)
#endif

#ifndef RG_X3_HEAD_FT
#define RG_X3_HEAD_FT 512  // the task-head chains (768 = 3 waves per SIMD: node heads -4 %, the
                           // small chains slower, the step flat -- kept at 2)
#endif
#ifndef RG_X3_PAIR_FT
#define RG_X3_PAIR_FT 768  // link pair chain: 12 waves, 3 per SIMD (133 VGPRs; 238.7 -> 233.2 us, M)
#endif
#ifndef RG_X3_HEAD_RT
#define RG_X3_HEAD_RT 1  // row tiles per wave of the 5-layer task-head chains (two waves / SIMD at 1)
#endif

static int dispatch(const Key& k, const Args& a, hipStream_t st) {
#define RG_X3C(MODE, K0, SP, LM, RT, FT, ...) \
  if (match(k, MODE, K0, SP, {__VA_ARGS__})) return launch<MODE, SP, LM, RT, FT, K0, __VA_ARGS__>(a, st);
  constexpr int ALL = 07777777;  // every plane of every layer in LDS
  constexpr int EFT = RG_X3_ENC_FT ? RG_X3_ENC_FT : (RG_X3_ENC_RT >= 2 ? 256 : 512);
  // edge encoder 7 -> 256 -> 128 -> 128 -> 64 (gnn_blocks.py:19-42, block 0 without norm):
  // LDS = layer 0 + planes 0, 1 of layer 1
  // (each shape twice: normalised layers packed centred -- the engine's choice -- or not)
#define RG_X3C2(MODE, K0, NM, AM, LM, RT, FT, ...)                      \
  RG_X3C(MODE, K0, spec(NM, AM, true), LM, RT, FT, __VA_ARGS__)         \
  RG_X3C(MODE, K0, spec(NM, AM, false), LM, RT, FT, __VA_ARGS__)
  RG_X3C2(IN_SMALL, 7, 0b1110, 0b1111, 07 | (03 << 3), RG_X3_ENC_RT, EFT, 256, 128, 128, 64)
  // node encoder 6 -> 256 -> 128 -> 64
  RG_X3C2(IN_SMALL, 6, 0b110, 0b111, 07 | (03 << 3), RG_X3_ENC_RT, EFT, 256, 128, 64)
  // task heads: 3-block stem + FFN_TaskSpecificHead (ffn + bare Linear -> 7 / 2, padded)
  constexpr int HFT = RG_X3_HEAD_RT == 1 ? RG_X3_HEAD_FT : 256;
  RG_X3C2(IN_DENSE, 64, 0b1111, 0b1111, ALL, RG_X3_HEAD_RT, HFT, 64, 64, 64, 64, 32)
  RG_X3C2(IN_PAIR, 64, 0b1111, 0b1111, ALL, RG_X3_HEAD_RT, HFT, 64, 64, 64, 64, 32)
  // the same link chain from per-node pre-projections (layer 0's planes are not staged), and
  // the per-node rows t: the compute_edge stem block + the bare layer 0 of the pair chain, or
  // the bare layer alone (no stem)
  RG_X3C2(IN_PAIRPRE, 64, 0b1111, 0b1111, ALL & ~07, RG_X3_HEAD_RT, RG_X3_PAIR_FT ? RG_X3_PAIR_FT : HFT,
          64, 64, 64, 64, 32)
  RG_X3C2(IN_DENSE, 64, 0b01, 0b01, ALL, 1, RG_X3_HEAD_FT, 64, 64)
  RG_X3C2(IN_DENSE, 64, 0, 0, ALL, 1, RG_X3_HEAD_FT, 64)
  // link edge_formation stem (1 block), object-class stem (3 blocks), object head
  RG_X3C2(IN_DENSE, 64, 0b1, 0b1, ALL, 1, RG_X3_HEAD_FT, 64)
  RG_X3C2(IN_DENSE, 64, 0b111, 0b111, ALL, 1, 512, 64, 64, 64)  // (176 B of spills at 768)
  RG_X3C2(IN_DENSE, 64, 0b01, 0b01, ALL, 1, RG_X3_HEAD_FT, 64, 32)
#undef RG_X3C2
#undef RG_X3C
  return RG_ERR_UNSUPPORTED;
}

}  // namespace cx3
}  // namespace rg

using namespace rg;
using namespace rg::cx3;

static int chain_x3(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                    int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                    const int* idx1, float* out, int ld_out, void* stream);

extern "C" int rg_mlp_chain_x3(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                               int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                               const int* idx1, float* out, int ld_out, void* stream) {
  return chain_x3(layers, n_layers, rows, rows_dev, in_mode, in0, ld0, w0, idx0, idx1, out,
                  ld_out, stream);
}

static int chain_x3(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                    int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                    const int* idx1, float* out, int ld_out, void* stream) {
  RG_REQUIRE(n_layers >= 1 && n_layers <= RG_MAX_LAYERS, RG_ERR_ARG, "rg_mlp_chain_x3: n_layers");
  RG_REQUIRE((in_mode != RG_IN_PAIRADD && in_mode != RG_IN_PAIRPRE) || (idx0 && idx1), RG_ERR_ARG,
             "rg_mlp_chain_x3: RG_IN_PAIRADD / RG_IN_PAIRPRE need idx0 and idx1");
  RG_REQUIRE(in_mode != RG_IN_PAIRPRE || (w0 == layers[0].out_dim && ld0 % 4 == 0), RG_ERR_ARG,
             "rg_mlp_chain_x3: RG_IN_PAIRPRE rows have layer 0's output width (stride % 4)");
  Key k;
  memset(&k, 0, sizeof(k));
  Args a;
  memset(&a, 0, sizeof(a));
  if (in_mode == RG_IN_DENSE && w0 <= 8 && n_layers >= 2 && !layers[0].norm_mu)
    k.mode = IN_SMALL;
  else if (in_mode == RG_IN_DENSE)
    k.mode = IN_DENSE;
  else if (in_mode == RG_IN_PAIRADD)
    k.mode = IN_PAIR;
  else if (in_mode == RG_IN_PAIRPRE)
    k.mode = IN_PAIRPRE;
  else
    return RG_ERR_UNSUPPORTED;
  RG_REQUIRE(k.mode == IN_SMALL || (w0 % 16 == 0 && ld0 % 4 == 0), RG_ERR_UNSUPPORTED,
             "rg_mlp_chain_x3: dense input width / stride must be multiples of 16 / 4");
  k.k0 = w0;
  k.nl = n_layers;
  int nm = 0, am = 0;
  for (int l = 0; l < n_layers; ++l) {
    const rg_layer& s = layers[l];
    RG_REQUIRE(s.w_packed, RG_ERR_ARG, "rg_mlp_chain_x3: layer %d weights", l);
    if (s.save_pre || s.save_out) return RG_ERR_UNSUPPORTED;
    RG_REQUIRE(!s.norm_mu || (s.norm_std && s.out_dim >= 2), RG_ERR_ARG, "norm params");
    RG_REQUIRE(l == 0 ? s.in_dim == w0 : s.in_dim == layers[l - 1].out_dim, RG_ERR_ARG,
               "rg_mlp_chain_x3: layer %d width", l);
    if (l + 1 < n_layers && s.out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
    if (s.norm_mu && s.out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
    if (s.norm_mu) nm |= 1 << l;
    if (s.act == ACT_LEAKY) am |= 1 << l;
    else if (s.act != ACT_NONE) return RG_ERR_UNSUPPORTED;
    k.n[l] = (s.out_dim + 31) / 32 * 32;
    a.L[l].src = (const char*)s.w_packed;
    a.L[l].mu = s.norm_mu;
    a.L[l].sd = s.norm_std;
  }
  // every normalised layer centred, or none (an un-normalised layer's flag is irrelevant)
  int cm = 0;
  for (int l = 0; l < n_layers; ++l)
    if (layers[l].norm_mu && (layers[l].flags & RG_LAYER_CENTERED)) cm |= 1 << l;
  if (cm != 0 && cm != nm) return RG_ERR_UNSUPPORTED;
  k.sp = spec(nm, am, cm != 0);
  a.rows = rows;
  a.rows_dev = rows_dev;
  a.in0 = in0;
  a.ld0 = ld0;
  a.w0real = w0;
  a.idx0 = idx0;
  a.idx1 = idx1;
  a.out = out;
  a.ld_out = ld_out;
  a.out_real = layers[n_layers - 1].out_dim;
  if (rows <= 0) return RG_OK;
  // encoders' buffer stores (RG_X3_ENC_BUF): full-width 16-B aligned rows, 32-bit byte offsets
  if (RG_X3_ENC_BUF && k.mode == IN_SMALL &&
      (a.out_real != k.n[n_layers - 1] || ld_out % 4 != 0 || (double)rows * ld_out * 4 > 0x7ff00000))
    return RG_ERR_UNSUPPORTED;
  return dispatch(k, a, (hipStream_t)stream);
}
