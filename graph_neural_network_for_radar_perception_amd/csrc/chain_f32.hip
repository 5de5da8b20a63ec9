// Register-resident float32 MLP chains on v_mfma_f32_32x32x2_f32 (exact f32 products,
// the reference precision): the fp32 path's encoders, task heads and the per-node
// projections of the fused f32 conv layer (conv_f32.hip).
//
// Same semantics as rg_mlp_chain with dtype RG_F32 (ffn_block chains: Linear ->
// channel_normalization -> activation, common.py:185-220, gnn_blocks.py:19-389), for the
// widths of the shipped architecture, every width a compile-time constant:
//
//  * one wave = 32 rows; Y^T = W . X^T, so lane (r = lane&31, h = lane>>5) holds row r's
//    features {32m + 8g + 4h + t} in accumulator register 4g + t of M-tile m;
//  * the k order of every packed layer (RG_PACK_F32_FAST) is k(s4, u, h) = 8 s4 + 4h + u,
//    which is BOTH a float4 of a row loaded from memory and registers 4g..4g+3 of the
//    previous layer's M-tile s4/4 (g = s4%4): layers chain in registers with no data
//    movement at all;
//  * channel_normalization (mean, unbiased std, correctly rounded sqrt / divide) is an
//    in-lane sum plus one v_permlane32_swap per statistic;
//  * one wave per SIMD (256-thread workgroups, up to 512 registers per lane): an f32 MFMA
//    keeps the matrix pipe busy for 64 cycles, room for ~14 independent instructions of
//    the same wave, so the epilogues and the next rows' loads hide behind the MFMAs;
//  * layers whose packed weights fit (<= ~155 KiB in total) are staged in LDS once per
//    persistent workgroup; larger chains (the 7 -> 256 -> 128 -> 128 -> 64 edge encoder is
//    232 KiB of f32 weights) read the remaining layers' fragments from global memory
//    (L2-resident, prefetched several k-steps ahead).
#include "rg_common.h"

namespace rg {
namespace f32c {

static constexpr float NORM_EPS = 1e-5f;  // constants.py:9
static constexpr int FT = 256;            // 4 waves, one per SIMD
#ifndef RG_CF32_DIVR
#define RG_CF32_DIVR 1  // the tape's channel-norm divides as reciprocal + one correction (0: __fdiv_rn)
#endif

// bytes of one RG_PACK_F32_FAST layer (fragments + accumulator-order bias)
__host__ __device__ constexpr int fbytes(int K, int N) {
  return (N / 32) * ((K + 7) / 8) * 1024 + N * 4;
}
__host__ __device__ constexpr int falign(int b) { return (b + 15) & ~15; }

struct Layer {
  const void* src;  // packed weights + bias (global)
  const float* mu;
  const float* sd;
  int out;
  int act;
  float* zs;        // training tape (TAPE kernels): z = x W^T + b, float32 [rows][out]
  float* as;        // and the activation output a, float32 [rows][out]
};

struct Args {
  Layer L[RG_MAX_LAYERS];
  int nl;
  long rows;
  const int* rows_dev;
  const float* in0;
  int ld0, w0real;
  const float* in1;  // IN_CONCAT2: second part of the row (the aggregate)
  int ld1;
  const float* in2;  // IN_GATHER3: third part (the encoded edge rows)
  int ld2;
  const int* idx0;
  const int* idx1;
  const float* res;  // optional residual added to the chain output (identity, gnn_blocks.py:109)
  int ld_res;
  float* out;
  int ld_out, out_real;
  int* zero_ptr;  // optional: zeroed by workgroup 0 (the next kernel's work counters)
  int zero_n;
};

// input modes of layer 0 (k-step order 8 s4 + 4h + u)
enum { IN_SMALL = 0,    // float32 rows of <= 8 features (encoders), one k-quad per lane half
       IN_DENSE = 1,    // float32 rows, K0 % 8 == 0
       IN_PAIR = 2,     // float32 x[idx0[r]] + x[idx1[r]] (edge_formation, gnn_blocks.py:297)
       IN_GATHER3 = 3,  // cat(x[idx0[r]], x[idx1[r]], e[r]): the message MLP input
                        // (x_i, x_j, edge; gnn_blocks.py:112-113), 64 + 64 + 64 features
       IN_CONCAT2 = 4 };  // cat(x[r], agg[r]): the update MLP input (gnn_blocks.py:108), 64 + 64
static constexpr int GW = 64;  // part width of the gather / concat modes (the yml widths)

// training tape: the 32 rows' features of accumulator tiles -> [rows][out] float32 (only the
// `out` real columns of a padded last layer)
template <int MT>
__device__ __forceinline__ void tape_rows(const f32x16 (&acc)[MT], float* base, int out, long row,
                                          int h) {
  float* o = base + (size_t)row * out;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * m + 8 * g + 4 * h;
      if (f0 + 4 <= out && (out & 3) == 0) {
        *(f32x4*)(o + f0) = (f32x4){acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2],
                                    acc[m][4 * g + 3]};
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (f0 + t < out) o[f0 + t] = acc[m][4 * g + t];
      }
    }
}

#ifndef RG_CF32_TAPE_BUF
#define RG_CF32_TAPE_BUF 1
#endif
// the same rows through a buffer resource for a full-width layer (out = 32 MT): one store per
// 16 B, issued for every row -- a row past the end gets an offset past the buffer's size and
// the hardware drops it.  With no branch around them the compiler counts these stores exactly,
// so the next tile's wait for its prefetched rows does not wait for them as well.
template <int MT>
__device__ __forceinline__ void tape_rows_buf(const f32x16 (&acc)[MT], float* base, long rows,
                                              long row, bool valid, int h) {
  constexpr int OUT = 32 * MT;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(rows * OUT * 4), 0x00020000);
  const int off = valid ? (int)(row * OUT * 4) : 0x7ffff000;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
      const u32x4_t v = {__float_as_uint(acc[m][4 * g]), __float_as_uint(acc[m][4 * g + 1]),
                         __float_as_uint(acc[m][4 * g + 2]), __float_as_uint(acc[m][4 * g + 3])};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, off + (32 * m + 8 * g + 4 * h) * 4, 0, 0);
    }
}

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// the 16 bias values of M-tile m, lane half h (accumulator order, 4 x 16-B reads)
__device__ __forceinline__ f32x16 bias_frag(const float* bias, int m, int h) {
  return ld_bias_frag(bias, m, h);
}

// One layer: acc (holding the bias) += W . X^T over S4 k-quads.  bop(s4) returns the
// f32x4 B operand of k-steps 4 s4 .. 4 s4 + 3.  A fragments (one f32x4 = 4 k-steps per
// M-tile) are read PD quads ahead: from LDS one quad ahead, from global memory (L2)
// four quads ahead.
template <int S4, int MT, bool G, typename BOp>
__device__ __forceinline__ void layer(f32x16 (&acc)[MT], const char* w, int lane, BOp&& bop) {
  const f32x4* wa = (const f32x4*)w + lane;
  constexpr int PD = G ? 4 : 1;
  constexpr int NB = PD + 1;
  f32x4 a[NB][MT];
#pragma unroll
  for (int s = 0; s < PD && s < S4; ++s)
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
    // one fence per k-quad: the compiler would otherwise hoist every fragment load of
    // the fully unrolled layer (hundreds of registers, then scratch)
    __builtin_amdgcn_sched_barrier(0);
  }
}

// channel_normalization (common.py:208-220): y = s (x - mean) / (std_unbiased + eps) + m
// over the row's 32*MT features (lane pair (lane, lane^32) holds one row)
template <int MT>
__device__ __forceinline__ void channel_norm(f32x16 (&acc)[MT], float mu, float sd) {
  constexpr int N = 32 * MT;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      s0 += acc[m][q];
      s1 += acc[m][q + 1];
    }
  const float mean = add_xor32(s0 + s1) * (1.f / N);  // N is a power of two: exact
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
}

template <int ACT, int MT>
__device__ __forceinline__ void act_all(f32x16 (&acc)[MT]) {
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[m][q] = act_t<ACT>(acc[m][q]);
}

// SPEC: bits 0-7 the activation, bit 8 + l layer l normalised, bit 16 + l layer l
// activated (else identity), bit 24 + l layer l's weights read from global memory
// (else staged in LDS) -- all host-checked against the layer descriptors
constexpr int spec(int act, int norm_mask, int act_mask, int gmask) {
  return act | (norm_mask << 8) | (act_mask << 16) | (gmask << 24);
}
constexpr bool spec_norm(int sp, int l) { return ((sp >> (8 + l)) & 1) != 0; }
constexpr bool spec_act(int sp, int l) { return ((sp >> (16 + l)) & 1) != 0; }
constexpr bool spec_glob(int sp, int l) { return ((sp >> (24 + l)) & 1) != 0; }

// channel_normalization + LeakyReLU in five ops per feature: sum, x - mean, sum of
// squares, y' = x a + b with the 0.505 of leaky(y) = 0.505 y + 0.495 |y| folded into a and
// b, then |y'| C + y' (C = 0.495 / 0.505; a free |.| source modifier)
template <int MT>
__device__ __forceinline__ void channel_norm_leaky(f32x16 (&acc)[MT], float mu, float sd) {
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
  const float ga = LEAKY_PRE * (sd * inv), gb = LEAKY_PRE * mu;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float y = fmaf(acc[m][q], ga, gb);
      acc[m][q] = fmaf(fabsf(y), LEAKY_C, y);
    }
}

// channel_normalization in the reference's operation order (common.py:215-220:
// (x - mean) / (std + eps), then std_param * . + mu_param, correctly rounded sqrt and
// divide) -- the training tape's epilogue, so the saved activations are the values the
// backward's recomputation (rg_ffn_backward) assumes
template <int MT>
__device__ __forceinline__ void channel_norm_ref(f32x16 (&acc)[MT], float mu, float sd) {
  constexpr int N = 32 * MT;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      s0 += acc[m][q];
      s1 += acc[m][q + 1];
    }
  const float mean = add_xor32(s0 + s1) * (1.f / N);  // N is a power of two: exact
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
  const float den = __fadd_rn(__fsqrt_rn(__fdiv_rn(add_xor32(q0 + q1), (float)(N - 1))), NORM_EPS);
#if RG_CF32_DIVR
  // x / den as RN(x * r) plus one fma residual correction with r = RN(1 / den): the
  // correctly rounded quotient while the quotient is a normal number (Markstein's result;
  // scripts/experiments/div_check.hip checks it for 64 chosen divisors over x in
  // [2^-100, 2^100), not exhaustively); e == 0 keeps q itself (a signed zero stays signed).
  // A nonzero |x| < 2 FLT_MIN den can give a subnormal quotient, outside that result: a wave
  // holding one divides with __fdiv_rn instead (wave-uniform branch, practically never taken)
  bool tiny = false;
  const float lim = __fmul_rn(2.f * 1.17549435e-38f, den);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) tiny |= acc[m][q] != 0.f && fabsf(acc[m][q]) < lim;
  if (__builtin_amdgcn_ballot_w64(tiny)) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] = __fadd_rn(__fmul_rn(sd, __fdiv_rn(acc[m][q], den)), mu);
    return;
  }
  const float rd = __fdiv_rn(1.f, den);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float x = acc[m][q];
      const float y = __fmul_rn(x, rd);
      const float e = fmaf(-y, den, x);
      acc[m][q] = __fadd_rn(__fmul_rn(sd, e == 0.f ? y : fmaf(e, rd, y)), mu);
    }
#else
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[m][q] = __fadd_rn(__fmul_rn(sd, __fdiv_rn(acc[m][q], den)), mu);
#endif
}

template <int SPEC, int LI, int MT, bool TAPE = false>
__device__ __forceinline__ void epilogue(f32x16 (&acc)[MT], const float* nrm) {
  if constexpr (TAPE) {
    if constexpr (spec_norm(SPEC, LI)) channel_norm_ref<MT>(acc, nrm[2 * LI], nrm[2 * LI + 1]);
    if constexpr (spec_act(SPEC, LI)) act_all<(SPEC & 0xff), MT>(acc);
    return;
  }
  if constexpr (spec_norm(SPEC, LI) && spec_act(SPEC, LI) && (SPEC & 0xff) == ACT_LEAKY) {
    channel_norm_leaky<MT>(acc, nrm[2 * LI], nrm[2 * LI + 1]);
    return;
  }
  if constexpr (spec_norm(SPEC, LI)) channel_norm<MT>(acc, nrm[2 * LI], nrm[2 * LI + 1]);
  if constexpr (spec_act(SPEC, LI)) act_all<(SPEC & 0xff), MT>(acc);
}

// LDS offsets: layers staged in LDS are packed back to back in layer order
template <int SPEC, int LI, int K, int... Ns> struct LdsOff;
template <int SPEC, int LI, int K> struct LdsOff<SPEC, LI, K> {
  static constexpr int get(int) { return 0; }
  static constexpr int total() { return 0; }
};
template <int SPEC, int LI, int K, int N, int... Rest> struct LdsOff<SPEC, LI, K, N, Rest...> {
  static constexpr int mine() { return spec_glob(SPEC, LI) ? 0 : falign(fbytes(K, N)); }
  static constexpr int get(int l) { return l == LI ? 0 : mine() + LdsOff<SPEC, LI + 1, N, Rest...>::get(l); }
  static constexpr int total() { return mine() + LdsOff<SPEC, LI + 1, N, Rest...>::total(); }
};

template <int MT>
__device__ __forceinline__ void store_out(const f32x16 (&acc)[MT], const Args& a, long row, int h) {
  float* o = a.out + (size_t)row * a.ld_out;
  const float* rs = a.res ? a.res + (size_t)row * a.ld_res : nullptr;
  const int out = a.out_real;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * m + 8 * g + 4 * h;
      if (f0 + 4 <= out && (a.ld_out & 3) == 0 && (!rs || (a.ld_res & 3) == 0)) {
        f32x4 v = {acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]};
        if (rs) {  // identity + upd(...) (gnn_blocks.py:109), one rounding per element
          const f32x4 x = *(const f32x4*)(rs + f0);
          v = (f32x4){__fadd_rn(x.x, v.x), __fadd_rn(x.y, v.y), __fadd_rn(x.z, v.z),
                      __fadd_rn(x.w, v.w)};
        }
        *(f32x4*)(o + f0) = v;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (f0 + t < out) o[f0 + t] = rs ? __fadd_rn(rs[f0 + t], acc[m][4 * g + t]) : acc[m][4 * g + t];
      }
    }
}

// the weight image of layer LI: LDS (staged) or global
template <int SPEC, int LI, int OFF>
__device__ __forceinline__ const char* wbase(const Args& a, const char* lds) {
  if constexpr (spec_glob(SPEC, LI)) return (const char*)a.L[LI].src;
  else return lds + OFF;
}

// layers LI.. of the chain; `prev` holds the previous layer's activations (B operands).
// TAPE: every layer's z (before its epilogue) and a (after it) also go to the tape.
template <int SPEC, bool TAPE, int LI, int K, int N, int... Rest, int PMT, typename Off>
__device__ __forceinline__ void run_rest(const Args& a, const f32x16 (&prev)[PMT], const char* lds,
                                         const float* nrm, long row, bool valid, int lane, Off) {
  constexpr int S4 = K / 8, MT = N / 32;
  static_assert(K == 32 * PMT, "chained width");
  const int h = lane >> 5;
  const char* w = wbase<SPEC, LI, Off::get(LI)>(a, lds);
  const float* bias = (const float*)(w + MT * S4 * 1024);
  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = bias_frag(bias, m, h);
  layer<S4, MT, spec_glob(SPEC, LI)>(acc, w, lane, [&](int s4) {
    const f32x16& p = prev[s4 >> 2];
    const int q = 4 * (s4 & 3);
    return (f32x4){p[q], p[q + 1], p[q + 2], p[q + 3]};
  });
  if constexpr (TAPE) {
    if constexpr (RG_CF32_TAPE_BUF && sizeof...(Rest) > 0) tape_rows_buf<MT>(acc, a.L[LI].zs, a.rows, row, valid, h);
    else if (valid) tape_rows<MT>(acc, a.L[LI].zs, a.L[LI].out, row, h);
  }
  epilogue<SPEC, LI, MT, TAPE>(acc, nrm);
  if constexpr (TAPE) {
    if constexpr (RG_CF32_TAPE_BUF && sizeof...(Rest) > 0) tape_rows_buf<MT>(acc, a.L[LI].as, a.rows, row, valid, h);
    else if (valid && a.L[LI].as) tape_rows<MT>(acc, a.L[LI].as, a.L[LI].out, row, h);
  }
  if constexpr (sizeof...(Rest) > 0) {
    run_rest<SPEC, TAPE, LI + 1, N, Rest...>(a, acc, lds, nrm, row, valid, lane, Off{});
  } else {
    if (valid) store_out<MT>(acc, a, row, h);
  }
}

template <int SPEC, bool TAPE, int K0, int N0, int... Rest, typename Off>
__device__ __forceinline__ void run_chain(const Args& a, const f32x4 (&bin)[(K0 + 7) / 8], const char* lds,
                                          const float* nrm, long row, bool valid, int lane, Off) {
  constexpr int S4 = (K0 + 7) / 8, MT = N0 / 32;
  const int h = lane >> 5;
  const char* w = wbase<SPEC, 0, Off::get(0)>(a, lds);
  const float* bias = (const float*)(w + MT * S4 * 1024);
  f32x16 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = bias_frag(bias, m, h);
  layer<S4, MT, spec_glob(SPEC, 0)>(acc, w, lane, [&](int s4) { return bin[s4]; });
  if constexpr (TAPE) {
    if constexpr (RG_CF32_TAPE_BUF && sizeof...(Rest) > 0) tape_rows_buf<MT>(acc, a.L[0].zs, a.rows, row, valid, h);
    else if (valid) tape_rows<MT>(acc, a.L[0].zs, a.L[0].out, row, h);
  }
  epilogue<SPEC, 0, MT, TAPE>(acc, nrm);
  if constexpr (TAPE) {
    if constexpr (RG_CF32_TAPE_BUF && sizeof...(Rest) > 0) tape_rows_buf<MT>(acc, a.L[0].as, a.rows, row, valid, h);
    else if (valid && a.L[0].as) tape_rows<MT>(acc, a.L[0].as, a.L[0].out, row, h);
  }
  if constexpr (sizeof...(Rest) > 0) {
    run_rest<SPEC, TAPE, 1, N0, Rest...>(a, acc, lds, nrm, row, valid, lane, Off{});
  } else {
    if (valid) store_out<MT>(acc, a, row, h);
  }
}

// Encoders (graph_feature_encoding, gnn_blocks.py:19-42): layer 0 (<= 8 inputs, no
// normalisation) fused tile by tile into layer 1 -- each 32-feature output tile of layer
// 0 (4 MFMAs) is activated and consumed at once as 16 k-steps of layer 1, so layer 0's
// 256-wide activation never exists in full.
template <int SPEC, bool TAPE, int K0, int N0, int N1, int... Rest, typename Off>
__device__ __forceinline__ void run_chain01(const Args& a, const f32x4 (&bin)[1], const char* lds,
                                            const float* nrm, long row, bool valid, int lane, Off) {
  static_assert(K0 <= 8, "fused first layer takes <= 8 inputs");
  constexpr int MT0 = N0 / 32, S41 = N0 / 8, MT1 = N1 / 32;
  const int h = lane >> 5;
  const char* w0 = wbase<SPEC, 0, Off::get(0)>(a, lds);
  const char* w1 = wbase<SPEC, 1, Off::get(1)>(a, lds);
  const float* bias0 = (const float*)(w0 + MT0 * 1024);
  const float* bias1 = (const float*)(w1 + MT1 * S41 * 1024);
  const f32x4* wa0 = (const f32x4*)w0 + lane;
  const f32x4* wa1 = (const f32x4*)w1 + lane;
  constexpr bool G1 = spec_glob(SPEC, 1);
  f32x16 acc[MT1];
#pragma unroll
  for (int m = 0; m < MT1; ++m) acc[m] = bias_frag(bias1, m, h);
  const f32x4 b0 = bin[0];
#pragma unroll
  for (int m0 = 0; m0 < MT0; ++m0) {
    // layer-1 A fragments of this layer-0 tile (k-quads 4 m0 .. 4 m0 + 3), issued first
    f32x4 f[4][MT1];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int m = 0; m < MT1; ++m) f[g][m] = wa1[(m * S41 + 4 * m0 + g) * 64];
    f32x16 t = bias_frag(bias0, m0, h);
    const f32x4 a0 = wa0[m0 * 64];
#pragma unroll
    for (int u = 0; u < 4; ++u) t = mfma(a0[u], b0[u], t);
    if constexpr (TAPE) {  // layer 0's z / a one 32-feature tile at a time
      if (valid) {
        f32x16 one[1] = {t};
        tape_rows<1>(one, a.L[0].zs + 32 * m0, a.L[0].out, row, h);
      }
    }
    if constexpr (spec_act(SPEC, 0)) {
#pragma unroll
      for (int q = 0; q < 16; ++q) t[q] = act_t<(SPEC & 0xff)>(t[q]);
    }
    if constexpr (TAPE) {
      if (valid) {
        f32x16 one[1] = {t};
        tape_rows<1>(one, a.L[0].as + 32 * m0, a.L[0].out, row, h);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int m = 0; m < MT1; ++m) acc[m] = mfma(f[g][m][u], t[4 * g + u], acc[m]);
    (void)G1;
    __builtin_amdgcn_sched_barrier(0);  // bound the live fragments to one layer-0 tile
  }
  if constexpr (TAPE) {
    if (valid) tape_rows<MT1>(acc, a.L[1].zs, a.L[1].out, row, h);
  }
  epilogue<SPEC, 1, MT1, TAPE>(acc, nrm);
  if constexpr (TAPE) {
    if (valid && a.L[1].as) tape_rows<MT1>(acc, a.L[1].as, a.L[1].out, row, h);
  }
  if constexpr (sizeof...(Rest) > 0) {
    run_rest<SPEC, TAPE, 2, N1, Rest...>(a, acc, lds, nrm, row, valid, lane, Off{});
  } else {
    if (valid) store_out<MT1>(acc, a, row, h);
  }
}

// NT threads per workgroup: 256 = one wave per SIMD, the next tile's input rows prefetched
// into registers; 512 = two waves per SIMD within 256 registers, no register prefetch (the
// other wave's work covers the row loads)
template <int MODE, int K0, int SPEC, bool FUSE01, bool TAPE, int NT, int... Ns>
__global__ __launch_bounds__(NT) void chain_f32_kernel(Args a) {
  static_assert(NT == FT || NT == 2 * FT, "chain_f32: 256 or 512 threads");
  constexpr bool PF = NT == FT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[2 * RG_MAX_LAYERS];
  using Off = LdsOff<SPEC, 0, K0, Ns...>;
  constexpr int NL = sizeof...(Ns);
  constexpr int S40 = (K0 + 7) / 8;
  if (blockIdx.x == 0 && a.zero_ptr && (int)threadIdx.x < a.zero_n) a.zero_ptr[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int l = 0; l < RG_MAX_LAYERS; ++l) {
      const bool n = l < NL && a.L[l].mu;
      nrm[2 * l] = n ? *a.L[l].mu : 0.f;
      nrm[2 * l + 1] = n ? *a.L[l].sd : 0.f;
    }
  }
  // stage the LDS layers (static indices: a dynamically indexed a.L would go to scratch)
  {
    constexpr int Ks[NL] = {Ns...};
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      if (!spec_glob(SPEC, l)) {
        const int K = l == 0 ? K0 : Ks[l - 1];
        stage_lds<NT>(lds + Off::get(l), a.L[l].src, fbytes(K, Ks[l]));
      }
    }
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const long rows = a.rows_dev ? min((long)*a.rows_dev, a.rows) : a.rows;
  const long ntiles = (rows + 31) / 32;
  const long tstride = (long)gridDim.x * (NT / 64);
  // layer-0 operands of tile t (prefetched one tile ahead at NT = 256)
  // IN_GATHER3: the two row indices of the tile fetch() is called for next
  int2 gi = {0, 0};
  auto fetch_idx = [&](long t) {
    const long row = t * 32 + r;
    const long rr = (t < ntiles && row < rows) ? row : 0;
    return int2{a.idx0[rr], a.idx1[rr]};
  };
  // layer-0 operands of tile t (prefetched one tile ahead at NT = 256).  Every load is
  // unconditional -- rows past the end read row 0, whose results are never stored -- so the
  // compiler counts the loads in flight: a load under a branch (or a select of its result)
  // made it wait for the prefetch it had just issued, every tile.  IN_SMALL's padding
  // columns are zeroed when the tile is taken (take), not when its loads are issued.
  auto fetch = [&](long t, f32x4 (&b)[S40]) {
    const long row = t * 32 + r;
    const long rr = (t < ntiles && row < rows) ? row : 0;
    if constexpr (MODE == IN_SMALL) {
      const float* p = a.in0 + (size_t)rr * a.ld0;
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = p[min(4 * h + u, a.w0real - 1)];
      b[0] = (f32x4){v[0], v[1], v[2], v[3]};
    } else if constexpr (MODE == IN_DENSE) {
      const float* p = a.in0 + (size_t)rr * a.ld0 + 4 * h;
#pragma unroll
      for (int s = 0; s < S40; ++s) b[s] = *(const f32x4*)(p + 8 * s);
    } else if constexpr (MODE == IN_GATHER3) {
      // k-quad s: x[idx0] features 8 s + 4 h (s < 8), x[idx1] (8 <= s < 16), e (s >= 16);
      // the indices come from gi, loaded one tile earlier (a load used right after its
      // issue waits for every older memory operation: the previous tile's tape stores)
      static_assert(K0 == 3 * GW, "gather3 width");
      const float* pi = a.in0 + (size_t)gi.x * a.ld0 + 4 * h;
      const float* pj = a.in0 + (size_t)gi.y * a.ld0 + 4 * h;
      const float* pe = a.in2 + (size_t)rr * a.ld2 + 4 * h;
#pragma unroll
      for (int s = 0; s < S40; ++s) {
        const float* p = s < GW / 8 ? pi + 8 * s : s < GW / 4 ? pj + 8 * (s - GW / 8) : pe + 8 * (s - GW / 4);
        b[s] = *(const f32x4*)p;
      }
    } else if constexpr (MODE == IN_CONCAT2) {
      static_assert(K0 == 2 * GW, "concat2 width");
      const float* p0 = a.in0 + (size_t)rr * a.ld0 + 4 * h;
      const float* p1 = a.in1 + (size_t)rr * a.ld1 + 4 * h;
#pragma unroll
      for (int s = 0; s < S40; ++s)
        b[s] = *(const f32x4*)(s < GW / 8 ? p0 + 8 * s : p1 + 8 * (s - GW / 8));
    } else {
      const float* pi = a.in0 + (size_t)a.idx0[rr] * a.ld0 + 4 * h;
      const float* pj = a.in0 + (size_t)a.idx1[rr] * a.ld0 + 4 * h;
#pragma unroll
      for (int s = 0; s < S40; ++s) {
        const f32x4 xi = *(const f32x4*)(pi + 8 * s), xj = *(const f32x4*)(pj + 8 * s);
        b[s] = (f32x4){__fadd_rn(xi.x, xj.x), __fadd_rn(xi.y, xj.y), __fadd_rn(xi.z, xj.z),
                       __fadd_rn(xi.w, xj.w)};
      }
    }
  };
  // the operands of a fetched tile as layer 0 takes them (IN_SMALL: padding columns zero)
  auto take = [&](f32x4 (&b)[S40]) {
    if constexpr (MODE == IN_SMALL) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (4 * h + u >= a.w0real) b[0][u] = 0.f;
    }
  };
  long tile = (long)blockIdx.x * (NT / 64) + wave;
  f32x4 nb[S40];
  if constexpr (PF) {
    if constexpr (MODE == IN_GATHER3) gi = fetch_idx(tile);
    fetch(tile, nb);
    if constexpr (MODE == IN_GATHER3) gi = fetch_idx(tile + tstride);
    // the first tile's loads complete before the loop: with them still pending on the way
    // in, the compiler's wait at the loop top (for the tile fetched one iteration earlier)
    // could not count past the previous tile's stores and waited for them all (vmcnt(0))
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  }
  for (; tile < ntiles; tile += tstride) {
    f32x4 b[S40];
    if constexpr (PF) {
#pragma unroll
      for (int s = 0; s < S40; ++s) b[s] = nb[s];
      fetch(tile + tstride, nb);
      if constexpr (MODE == IN_GATHER3) gi = fetch_idx(tile + 2 * tstride);
    } else {
      if constexpr (MODE == IN_GATHER3) gi = fetch_idx(tile);
      fetch(tile, b);
    }
    take(b);
    const long row = tile * 32 + r;
    const bool valid = row < rows;
    if constexpr (FUSE01) run_chain01<SPEC, TAPE, K0, Ns...>(a, b, lds, nrm, row, valid, lane, Off{});
    else run_chain<SPEC, TAPE, K0, Ns...>(a, b, lds, nrm, row, valid, lane, Off{});
  }
}

template <int MODE, int K0, int SPEC, bool FUSE01, bool TAPE, int NT, int... Ns>
static int launch(const Args& a, hipStream_t st) {
  using Off = LdsOff<SPEC, 0, K0, Ns...>;
  constexpr int lds = Off::total();
  static_assert(lds <= DYN_LDS_MAX, "LDS image too large: read more layers from global memory");
  auto kern = chain_f32_kernel<MODE, K0, SPEC, FUSE01, TAPE, NT, Ns...>;
  RG_ENSURE_LDS(kern, DYN_LDS_MAX);
  const long tiles = (a.rows + 31) / 32;
  constexpr int WPG = NT / 64;
  long blocks = (tiles + WPG - 1) / WPG;
  const long cap = lds <= 76 * 1024 ? 512 : 256;  // persistent: workgroups that fit at once
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  kern<<<blocks, NT, lds, st>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

struct Key {
  int mode, k0, spec_lo, nl;  // spec_lo: act | norm | act masks (bits 0..23)
  int tape;                   // training tape (every layer's save_pre / save_out)
  int n[RG_MAX_LAYERS];
};

static bool match(const Key& k, int mode, int k0, int sp, bool tape, std::initializer_list<int> ns) {
  if (k.mode != mode || k.k0 != k0 || k.spec_lo != (sp & 0xffffff) || k.nl != (int)ns.size() ||
      k.tape != (int)tape)
    return false;
  int i = 0;
  for (int v : ns)
    if (k.n[i++] != v) return false;
  return true;
}

static int dispatch(const Key& k, const Args& a, hipStream_t st) {
  constexpr int L = ACT_LEAKY;
#define RG_F32C(MODE, K0, SP, F01, ...) \
  if (match(k, MODE, K0, SP, false, {__VA_ARGS__})) return launch<MODE, K0, (SP), F01, false, FT, __VA_ARGS__>(a, st);
  // training forward (rg_mlp_chain_f32_ex with every layer's save_pre / save_out set)
#define RG_F32T(MODE, K0, SP, F01, ...) \
  if (match(k, MODE, K0, SP, true, {__VA_ARGS__})) return launch<MODE, K0, (SP), F01, true, FT, __VA_ARGS__>(a, st);
  // the same at two waves per SIMD (512 threads, no register prefetch)
#define RG_F32T2(MODE, K0, SP, F01, ...) \
  if (match(k, MODE, K0, SP, true, {__VA_ARGS__})) return launch<MODE, K0, (SP), F01, true, 2 * FT, __VA_ARGS__>(a, st);
  // edge encoder 7 -> 256 -> 128 -> 128 -> 64 (gnn_blocks.py:19-42, block 0 without norm):
  // layers 0 + 1 (136 KiB) in LDS, layers 2 + 3 (96 KiB) from L2
  RG_F32C(IN_SMALL, 7, spec(L, 0b1110, 0b1111, 0b1100), true, 256, 128, 128, 64)
  // node encoder 6 -> 256 -> 128 -> 64
  RG_F32C(IN_SMALL, 6, spec(L, 0b110, 0b111, 0b100), true, 256, 128, 64)
  // per-node projections of the fused f32 conv layer: [W_xi; W_xj] x + [b; 0], 64 -> 256
  RG_F32C(IN_DENSE, 64, spec(L, 0, 0, 0), false, 256)
  // task heads: 3-block stem + FFN_TaskSpecificHead (ffn + bare Linear -> 7 / 2, padded)
  RG_F32C(IN_DENSE, 64, spec(L, 0b1111, 0b1111, 0), false, 64, 64, 64, 64, 32)
  RG_F32C(IN_PAIR, 64, spec(L, 0b1111, 0b1111, 0), false, 64, 64, 64, 64, 32)
  // link edge_formation stem (1 block), object-class stem (3 blocks), object head
  RG_F32C(IN_DENSE, 64, spec(L, 0b1, 0b1, 0), false, 64)
  RG_F32C(IN_DENSE, 64, spec(L, 0b111, 0b111, 0), false, 64, 64, 64)
  RG_F32C(IN_DENSE, 64, spec(L, 0b01, 0b01, 0), false, 64, 32)
  // ---- training tapes of the yml architecture (Model_Training.forward, training.py)
  // message MLP 192 -> 128 -> 64 on cat(x_i, x_j, e) (gnn_blocks.py:104-113), 131 KiB in LDS
#ifndef RG_CF32_MSG_WPS
#define RG_CF32_MSG_WPS 1  // 2: the 512-thread form (232 VGPRs, no register prefetch): c4 800.8 vs 800.4 frames/s, flat (profiles/r06_c4_msg_wps_ab.log)
#endif
#if RG_CF32_MSG_WPS == 2
  RG_F32T2(IN_GATHER3, 192, spec(L, 0b11, 0b11, 0), false, 128, 64)
#else
  RG_F32T(IN_GATHER3, 192, spec(L, 0b11, 0b11, 0), false, 128, 64)
#endif
  // update MLP 128 -> 64 on cat(x, agg), + identity
  RG_F32T(IN_CONCAT2, 128, spec(L, 0b1, 0b1, 0), false, 64)
  // encoders (layer 0's tape written one 32-feature tile at a time)
  RG_F32T(IN_SMALL, 7, spec(L, 0b1110, 0b1111, 0b1100), true, 256, 128, 128, 64)
  RG_F32T(IN_SMALL, 6, spec(L, 0b110, 0b111, 0b100), true, 256, 128, 64)
  // task heads, link pairs, link / object stems, object head
  RG_F32T(IN_DENSE, 64, spec(L, 0b1111, 0b1111, 0), false, 64, 64, 64, 64, 32)
  RG_F32T(IN_PAIR, 64, spec(L, 0b1111, 0b1111, 0), false, 64, 64, 64, 64, 32)
  RG_F32T(IN_DENSE, 64, spec(L, 0b1, 0b1, 0), false, 64)
  RG_F32T(IN_DENSE, 64, spec(L, 0b111, 0b111, 0), false, 64, 64, 64)
  RG_F32T(IN_DENSE, 64, spec(L, 0b01, 0b01, 0), false, 64, 32)
  // the backward's data GEMMs dX = dZ W (weights packed RG_PACK_F32_FAST | RG_PACK_TRANSPOSE,
  // one bare layer, optionally accumulating through the residual input): message layers
  // 64 -> 128 and 128 -> 192, update 64 -> 128, stems 64 -> 64, encoder layers
  RG_F32C(IN_DENSE, 64, spec(L, 0, 0, 0), false, 64)
  RG_F32C(IN_DENSE, 64, spec(L, 0, 0, 0), false, 128)
  RG_F32C(IN_DENSE, 128, spec(L, 0, 0, 0), false, 128)
  RG_F32C(IN_DENSE, 128, spec(L, 0, 0, 0), false, 64)   // column blocks of msg0 (training.py)
  RG_F32C(IN_DENSE, 128, spec(L, 0, 0, 0), false, 192)
  RG_F32C(IN_DENSE, 128, spec(L, 0, 0, 0), false, 256)
#undef RG_F32C
#undef RG_F32T
#undef RG_F32T2
  return RG_ERR_UNSUPPORTED;
}

// ---------------------------------------------------------------- dX + norm backward
// The training backward's dA = dZ W (one transposed layer, as the dX chains above) with
// the previous ffn_block's channel_normalization + activation backward applied in the same
// registers (rg_dx_norm_backward): dz = ffn_backward(z, dA) without dA ever reaching
// memory.  The arithmetic is rg_ffn_backward's (train.hip) with the row sums taken over
// this layout (in-lane, then the lane pair):
//   gy = dA act'(y);  ds += sum gy n;  dm += sum gy;  gn = s gy;
//   gd = r gn - r^2 (sum gn d) d / ((C-1) std);  dz = gd - mean(gd)
// with the d mu / d std sums of each row in float32 and over rows in float64, one partial
// per workgroup (fixed order), reduced by the caller.
struct NormBwd {
  const float* z;  // the norm's input (pre-norm tape), [rows][C]
  int ldz;
  const float* mu;
  const float* sd;
  int act;
  double* part;    // [gridDim.x][2]: (sum gy n, sum gy)
};

__device__ __forceinline__ float nb_act_grad(float y, int act) {
  if (act == ACT_LEAKY) return y > 0.f ? 1.f : 0.01f;  // torch's leaky_relu backward
  return 1.f;
}

#ifndef RG_DXNB_WPS
#define RG_DXNB_WPS 2  // waves per SIMD (<= 256 registers per lane): one wave's z / dZ loads
                       // behind the other's MFMAs and epilogue (K0 = 128: one, 99 spills at two)
#endif
template <int K0>
constexpr int dxnb_wps() { return K0 >= 128 ? 1 : RG_DXNB_WPS; }
template <int K0, int N>
__global__ __launch_bounds__(FT, dxnb_wps<K0>()) void dx_norm_bwd_kernel(Args a, NormBwd nb) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ double red[FT / 64][2];
  constexpr int S40 = K0 / 8, MT = N / 32, C = N;
  static_assert(K0 % 8 == 0 && N % 32 == 0, "dx_norm_bwd widths");
  stage_lds<FT>(lds, a.L[0].src, fbytes(K0, N));
  const float sp = *nb.sd, mp = *nb.mu;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const long rows = a.rows;
  const long ntiles = (rows + 31) / 32;
  const long tstride = (long)gridDim.x * (FT / 64);
  const float* bias = (const float*)(lds + MT * S40 * 1024);
  auto fetch = [&](long t, f32x4 (&b)[S40]) {  // unconditional loads (chain_f32_kernel's fetch)
    const long row = t * 32 + r;
    const float* p = a.in0 + (size_t)((t < ntiles && row < rows) ? row : 0) * a.ld0 + 4 * h;
#pragma unroll
    for (int s = 0; s < S40; ++s) b[s] = *(const f32x4*)(p + 8 * s);
  };
  double acc_s = 0.0, acc_m = 0.0;
  long tile = (long)blockIdx.x * (FT / 64) + wave;
  f32x4 nbuf[S40];
  fetch(tile, nbuf);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): see chain_f32_kernel
  for (; tile < ntiles; tile += tstride) {
    f32x4 b[S40];
#pragma unroll
    for (int s = 0; s < S40; ++s) b[s] = nbuf[s];
    fetch(tile + tstride, nbuf);
    const long row = tile * 32 + r;
    const bool valid = row < rows;
    // the row's z (issued before the MFMAs)
    f32x4 zq[MT][4];
    const float* zr = nb.z + (size_t)(valid ? row : 0) * nb.ldz + 4 * h;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        zq[m][g] = valid ? *(const f32x4*)(zr + 32 * m + 8 * g) : (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x16 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = bias_frag(bias, m, h);
    layer<S40, MT, false>(acc, lds, lane, [&](int s4) { return b[s4]; });
    // acc[m][4g + t] = dA of feature 32 m + 8 g + 4 h + t; zq the same features
    float t0 = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 4; ++t) t0 += zq[m][g][t];
    const float mean = add_xor32(t0) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          zq[m][g][t] = zq[m][g][t] - mean;  // d
          ss += zq[m][g][t] * zq[m][g][t];
        }
    ss = add_xor32(ss);
    const float stdv = __fsqrt_rn(ss / (float)(C - 1));
    const float rr = 1.f / (stdv + NORM_EPS);
    float ps = 0.f, pm = 0.f, A = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float d = zq[m][g][t];
          const float n = d * rr;
          const float y = __fadd_rn(__fmul_rn(sp, n), mp);
          const float gy = acc[m][4 * g + t] * nb_act_grad(y, nb.act);
          ps += gy * n;
          pm += gy;
          const float gn = sp * gy;
          acc[m][4 * g + t] = gn;
          A += gn * d;
        }
    ps = add_xor32(ps);
    pm = add_xor32(pm);
    A = add_xor32(A);
    if (valid && h == 0) {
      acc_s += (double)ps;
      acc_m += (double)pm;
    }
    const float coef = stdv > 0.f ? rr * rr * A / ((float)(C - 1) * stdv) : 0.f;
    float sg = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        acc[m][q] = rr * acc[m][q] - coef * zq[m][q >> 2][q & 3];
        sg += acc[m][q];
      }
    const float mg = add_xor32(sg) / (float)C;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] = acc[m][q] - mg;
    if (valid) store_out<MT>(acc, a, row, h);
  }
  // per-workgroup partials: a fixed butterfly over the wave, the waves in order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    acc_s += __shfl_xor(acc_s, o, 64);
    acc_m += __shfl_xor(acc_m, o, 64);
  }
  if (lane == 0) {
    red[wave][0] = acc_s;
    red[wave][1] = acc_m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tm = 0.0;
#pragma unroll
    for (int w = 0; w < FT / 64; ++w) {
      ts += red[w][0];
      tm += red[w][1];
    }
    nb.part[2 * blockIdx.x] = ts;
    nb.part[2 * blockIdx.x + 1] = tm;
  }
}

template <int K0, int N>
static int launch_dxnb(const Args& a, const NormBwd& nb, long blocks, hipStream_t st) {
  auto kern = dx_norm_bwd_kernel<K0, N>;
  RG_ENSURE_LDS(kern, DYN_LDS_MAX);
  kern<<<blocks, FT, fbytes(K0, N), st>>>(a, nb);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

}  // namespace f32c
}  // namespace rg

using namespace rg;
using namespace rg::f32c;

// internal entry (conv_f32.hip): the per-node projection chain, also zeroing the conv's
// work counters (zero_ptr) in the same launch
int rg_f32_chain_launch(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                        int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                        const int* idx1, float* out, int ld_out, int* zero_ptr, int zero_n,
                        void* stream);

static int f32_chain_launch(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                            int in_mode, const float* in0, int ld0, int w0, const float* in1,
                            int ld1, int w1, const float* in2, int ld2, int w2, const int* idx0,
                            const int* idx1, const float* res, int ld_res, float* out, int ld_out,
                            int* zero_ptr, int zero_n, void* stream) {
  RG_REQUIRE(n_layers >= 1 && n_layers <= RG_MAX_LAYERS, RG_ERR_ARG, "rg_mlp_chain_f32: n_layers");
  RG_REQUIRE(zero_n <= FT, RG_ERR_ARG, "rg_mlp_chain_f32: zero_n");
  Key k;
  memset(&k, 0, sizeof(k));
  Args a;
  memset(&a, 0, sizeof(a));
  int k0 = w0;
  if (in_mode == RG_IN_DENSE && w0 <= 8 && n_layers >= 2 && !layers[0].norm_mu) {
    k.mode = IN_SMALL;
  } else if (in_mode == RG_IN_DENSE) {
    k.mode = IN_DENSE;
  } else if (in_mode == RG_IN_PAIRADD) {
    k.mode = IN_PAIR;
  } else if (in_mode == RG_IN_GATHER3) {
    if (w0 != GW || w2 != GW || !in2 || !idx0 || !idx1 || ld2 % 4) return RG_ERR_UNSUPPORTED;
    k.mode = IN_GATHER3;
    k0 = 2 * w0 + w2;
  } else if (in_mode == RG_IN_CONCAT2) {
    if (w0 != GW || w1 != GW || !in1 || ld1 % 4) return RG_ERR_UNSUPPORTED;
    k.mode = IN_CONCAT2;
    k0 = w0 + w1;
  } else {
    return RG_ERR_UNSUPPORTED;
  }
  RG_REQUIRE(k.mode == IN_SMALL || (w0 % 8 == 0 && ld0 % 4 == 0), RG_ERR_UNSUPPORTED,
             "rg_mlp_chain_f32: dense input width / stride must be multiples of 8 / 4");
  k.k0 = k0;
  k.nl = n_layers;
  // training tape: every layer saves (z, a) or none does
  k.tape = layers[0].save_pre != nullptr;
  int nm = 0, am = 0;
  for (int l = 0; l < n_layers; ++l) {
    const rg_layer& s = layers[l];
    RG_REQUIRE(s.w_packed, RG_ERR_ARG, "rg_mlp_chain_f32: layer %d weights", l);
    if (s.flags & RG_LAYER_CENTERED) return RG_ERR_UNSUPPORTED;
    // (the last layer's save_out may be NULL: its activation is the chain output, which the
    // backward never reads back -- one [rows][out] write less)
    if ((s.save_pre != nullptr) != (bool)k.tape ||
        ((s.save_out != nullptr) != (bool)k.tape && !(k.tape && l == n_layers - 1)))
      return RG_ERR_UNSUPPORTED;
    RG_REQUIRE(!s.norm_mu || (s.norm_std && s.out_dim >= 2), RG_ERR_ARG, "norm params");
    RG_REQUIRE(l == 0 ? s.in_dim == k0 : s.in_dim == layers[l - 1].out_dim, RG_ERR_ARG,
               "rg_mlp_chain_f32: layer %d width", l);
    if (l + 1 < n_layers && s.out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
    if (s.norm_mu && s.out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
    if (s.norm_mu) nm |= 1 << l;
    if (s.act == ACT_LEAKY) am |= 1 << l;
    else if (s.act != ACT_NONE) return RG_ERR_UNSUPPORTED;
    k.n[l] = (s.out_dim + 31) / 32 * 32;
    a.L[l].src = s.w_packed;
    a.L[l].mu = s.norm_mu;
    a.L[l].sd = s.norm_std;
    a.L[l].out = s.out_dim;
    a.L[l].act = s.act;
    a.L[l].zs = s.save_pre;
    a.L[l].as = s.save_out;
  }
  // (tape_rows_buf: a non-last layer's tape is a 32-bit-addressed buffer resource)
  if (k.tape)
    for (int l = 0; l + 1 < n_layers; ++l)
      if ((double)rows * k.n[l] * 4 >= 2147483648.0 || layers[l].out_dim != k.n[l]) return RG_ERR_UNSUPPORTED;
  k.spec_lo = spec(ACT_LEAKY, nm, am, 0);
  a.nl = n_layers;
  a.rows = rows;
  a.rows_dev = rows_dev;
  a.in0 = in0;
  a.ld0 = ld0;
  a.w0real = w0;
  a.in1 = in1;
  a.ld1 = ld1;
  a.in2 = in2;
  a.ld2 = ld2;
  a.idx0 = idx0;
  a.idx1 = idx1;
  a.res = res;
  a.ld_res = ld_res;
  a.out = out;
  a.ld_out = ld_out;
  a.out_real = layers[n_layers - 1].out_dim;
  a.zero_ptr = zero_ptr;
  a.zero_n = zero_n;
  if (rows <= 0 && !zero_ptr) return RG_OK;
  return dispatch(k, a, (hipStream_t)stream);
}

int rg_f32_chain_launch(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                        int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                        const int* idx1, float* out, int ld_out, int* zero_ptr, int zero_n,
                        void* stream) {
  return f32_chain_launch(layers, n_layers, rows, rows_dev, in_mode, in0, ld0, w0, nullptr, 0, 0,
                          nullptr, 0, 0, idx0, idx1, nullptr, 0, out, ld_out, zero_ptr, zero_n,
                          stream);
}

extern "C" int rg_mlp_chain_f32(const rg_layer* layers, int n_layers, long rows,
                                const int* rows_dev, int in_mode, const float* in0, int ld0,
                                int w0, const int* idx0, const int* idx1, float* out, int ld_out,
                                void* stream) {
  RG_REQUIRE(in_mode != RG_IN_PAIRADD || (idx0 && idx1), RG_ERR_ARG,
             "rg_mlp_chain_f32: RG_IN_PAIRADD needs idx0 and idx1");
  if (in_mode != RG_IN_DENSE && in_mode != RG_IN_PAIRADD) return RG_ERR_UNSUPPORTED;
  return rg_f32_chain_launch(layers, n_layers, rows, rows_dev, in_mode, in0, ld0, w0, idx0, idx1,
                             out, ld_out, nullptr, 0, stream);
}

extern "C" int rg_mlp_chain_f32_ex(const rg_layer* layers, int n_layers, long rows,
                                   const int* rows_dev, int in_mode, const float* in0, int ld0,
                                   int w0, const float* in1, int ld1, int w1, const float* in2,
                                   int ld2, int w2, const int* idx0, const int* idx1,
                                   const float* residual, int ld_res, float* out, int ld_out,
                                   void* stream) {
  RG_REQUIRE((in_mode != RG_IN_PAIRADD && in_mode != RG_IN_GATHER3) || (idx0 && idx1), RG_ERR_ARG,
             "rg_mlp_chain_f32_ex: gathered input modes need idx0 and idx1");
  return f32_chain_launch(layers, n_layers, rows, rows_dev, in_mode, in0, ld0, w0, in1, ld1, w1, in2,
                          ld2, w2, idx0, idx1, residual, ld_res, out, ld_out, nullptr, 0, stream);
}

// train.hip: sum of `parts` (s, m) float64 partials in a fixed order into *d_mu / *d_std
int rg_train_param_reduce(const double* part, int parts, float* d_mu, float* d_std, void* stream);

extern "C" size_t rg_dx_norm_backward_workspace_size(long rows) {
  const long tiles = (rows + 31) / 32;
  long blocks = (tiles + 3) / 4;
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  return (size_t)blocks * 2 * sizeof(double);
}

extern "C" int rg_dx_norm_backward(const rg_layer* layer, long rows, const float* dz_next,
                                   int ld_dzn, const float* z, int ldz, const float* mu,
                                   const float* std_, int act, float* dz, int lddz, float* d_mu,
                                   float* d_std, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  RG_REQUIRE(layer && layer->w_packed, RG_ERR_ARG, "rg_dx_norm_backward: layer");
  RG_REQUIRE(mu && std_ && d_mu && d_std && z && dz_next && dz, RG_ERR_ARG,
             "rg_dx_norm_backward: pointers");
  RG_REQUIRE(act == ACT_NONE || act == ACT_LEAKY, RG_ERR_UNSUPPORTED, "rg_dx_norm_backward: act");
  RG_REQUIRE(ld_dzn % 4 == 0 && ldz % 4 == 0 && lddz % 4 == 0, RG_ERR_UNSUPPORTED,
             "rg_dx_norm_backward: strides must be multiples of 4");
  RG_REQUIRE((const float*)dz != dz_next && (const float*)dz != z, RG_ERR_ARG,
             "rg_dx_norm_backward: dz may not alias its inputs");
  if (rows <= 0) return RG_OK;
  const size_t need = rg_dx_norm_backward_workspace_size(rows);
  RG_REQUIRE(workspace && workspace_bytes >= need, RG_ERR_ARG,
             "rg_dx_norm_backward: workspace %zu < %zu", workspace_bytes, need);
  const long blocks = (long)(need / (2 * sizeof(double)));
  Args a;
  memset(&a, 0, sizeof(a));
  a.L[0].src = layer->w_packed;
  a.nl = 1;
  a.rows = rows;
  a.in0 = dz_next;
  a.ld0 = ld_dzn;
  a.w0real = layer->in_dim;
  a.out = dz;
  a.ld_out = lddz;
  a.out_real = layer->out_dim;
  NormBwd nb;
  nb.z = z;
  nb.ldz = ldz;
  nb.mu = mu;
  nb.sd = std_;
  nb.act = act;
  nb.part = (double*)workspace;
  hipStream_t st = (hipStream_t)stream;
  int rc = RG_ERR_UNSUPPORTED;
  const int K = layer->in_dim, N = layer->out_dim;
  if (K == 64 && N == 128) rc = launch_dxnb<64, 128>(a, nb, blocks, st);
  else if (K == 128 && N == 128) rc = launch_dxnb<128, 128>(a, nb, blocks, st);
  else if (K == 64 && N == 64) rc = launch_dxnb<64, 64>(a, nb, blocks, st);
  if (rc != RG_OK) return rc;
  return rg_train_param_reduce((const double*)workspace, (int)blocks, d_mu, d_std, stream);
}
