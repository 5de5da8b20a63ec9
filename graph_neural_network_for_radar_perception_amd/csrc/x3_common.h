// Float32 arithmetic on the bf16 matrix cores (conv_x3.hip, chain_x3.hip).
//
// Every f32 operand is split EXACTLY into three bf16 terms, v = v0 + v1 + v2 (round to
// nearest even at each step: v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1); the
// residues are exact in f32, and the third term holds the last 8 significant bits), and a
// product a.b is formed from the six terms of weight <= 2,
//     a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0,
// on v_mfma_f32_32x32x16_bf16 with f32 accumulation.  The dropped terms a1 b2 + a2 b1 +
// a2 b2 are below 2^-23 |a b|: each product carries about the error of one f32 rounding and
// the accumulation is f32 -- the arithmetic of the reference's fp32 path, not of bf16.
// Six 32-cycle bf16 MFMAs replace eight 64-cycle f32 MFMAs per 16-deep k-step: 2.7x the
// matrix rate of v_mfma_f32_32x32x2_f32.
//
// Packed weights (rg_pack_linear with RG_PACK_X3): three planes of a 32x32x16 fragment
// format (RG_PACK_FAST_IN / _CHAIN), back to back, then the f32 bias in accumulator order.
// Lane (r = lane & 31, h = lane >> 5) of an accumulator tile m holds row r's features
// {32m + 8(q >> 2) + 4h + (q & 3)} in register q.
#pragma once

#include "rg_common.h"

namespace rg {
namespace x3 {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int plane_bytes(int K, int N) { return (N / 32) * ((K + 15) / 16) * 1024; }
__host__ __device__ constexpr int x3_bytes(int K, int N) { return 3 * plane_bytes(K, N) + N * 4; }
__host__ __device__ constexpr int al16(int b) { return (b + 15) & ~15; }

__device__ __forceinline__ bf16x8_t ld_bf8(const char* p) {
  return __builtin_bit_cast(bf16x8_t, *(const u32x4*)p);
}
__device__ __forceinline__ f32x16 mf(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

struct X3 {
  bf16x8_t p0, p1, p2;
};

// v_cvt_pk_bf16_f32 (round to nearest even) as an opaque instruction: through the builtin
// the compiler re-derives each element's bf16 with a second conversion instead of taking
// it from the packed word (two extra instructions per pair)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

#ifndef RG_X3_PIPE
#define RG_X3_PIPE 1  // layer_x3 computes the B operand of k-step s + 1 beside step s's MFMAs
#endif
#ifndef RG_X3_LASTSB
#define RG_X3_LASTSB 0  // 0: no fence after the last k-step (M edge encoder 1.41 -> 1.38 ms, conv flat)
#endif
#ifndef RG_X3_SPLIT
#define RG_X3_SPLIT 0  // split8: 0 pair by pair through the inline-asm conversion (the chains),
                       // 4 builtin conversions (no asm: no s_nop pads; conv_x3.hip)
#endif

// the two f32 values of a packed bf16 pair
__device__ __forceinline__ f32x2 unpk(uint32_t u) {
  return (f32x2){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// v_cvt_pk_bf16_f32 through the generic conversion: the compiler takes each element's value
// from the packed word (no inline asm: an asm result costs an s_nop before its first reader,
// the hazard recognizer having to assume a transcendental)
__device__ __forceinline__ uint32_t cvt_pk_bf16_c(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2_t));
}
__device__ __forceinline__ f32x2 unpk_c(uint32_t u) {
  return __builtin_convertvector(__builtin_bit_cast(bf16x2_t, u), f32x2);
}

// 8 consecutive k values of one row -> the three exact bf16 terms (the residues of a
// pair in one v_pk_add_f32)
__device__ __forceinline__ X3 split8(const f32x4 lo, const f32x4 hi) {
  const f32x2 v[4] = {{lo.x, lo.y}, {lo.z, lo.w}, {hi.x, hi.y}, {hi.z, hi.w}};
  u32x4 w0, w1, w2;
#if RG_X3_SPLIT == 4
  // builtin conversions, scalar residues: 3 conversions + 4 unpacks + 4 subtractions per pair
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t u0 = cvt_pk_bf16_c(v[i].x, v[i].y);
    const f32x2 u0f = unpk_c(u0);
    const float rx = v[i].x - u0f.x, ry = v[i].y - u0f.y;
    const uint32_t u1 = cvt_pk_bf16_c(rx, ry);
    const f32x2 u1f = unpk_c(u1);
    w0[i] = u0;
    w1[i] = u1;
    w2[i] = cvt_pk_bf16_c(rx - u1f.x, ry - u1f.y);
  }
#else
  // the inline-asm conversion, scalar residues
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t u0 = cvt_pk_bf16(v[i].x, v[i].y);
    const f32x2 u0f = unpk(u0);
    const f32x2 r = {v[i].x - u0f.x, v[i].y - u0f.y};
    const uint32_t u1 = cvt_pk_bf16(r.x, r.y);
    const f32x2 u1f = unpk(u1);
    const f32x2 t = {r.x - u1f.x, r.y - u1f.y};
    w0[i] = u0;
    w1[i] = u1;
    w2[i] = cvt_pk_bf16(t.x, t.y);
  }
#endif
  return X3{__builtin_bit_cast(bf16x8_t, w0), __builtin_bit_cast(bf16x8_t, w1),
            __builtin_bit_cast(bf16x8_t, w2)};
}
// registers 8 hf .. 8 hf + 7 of an accumulator tile (one RG_PACK_FAST_CHAIN k-step)
__device__ __forceinline__ X3 split_acc(const f32x16& t, int hf) {
  const int q = 8 * hf;
  return split8((f32x4){t[q], t[q + 1], t[q + 2], t[q + 3]},
                (f32x4){t[q + 4], t[q + 5], t[q + 6], t[q + 7]});
}

// ---------------------------------------------------------------- weight sources
// W(p, off): the 16 bytes of this lane in plane p at byte offset off of the plane.
// LDS-staged images, or global memory / L2 through a buffer resource (one lane-offset
// register, the fragment offset as a scalar: plain global pointers make the compiler hoist
// one 64-bit address per fragment out of a persistent loop and spill them).
struct WLds {
  const char* p;  // image base + lane * 16
  int pl;         // plane stride
  __device__ __forceinline__ bf16x8_t operator()(int plane, int off) const {
    return ld_bf8(p + plane * pl + off);
  }
};
struct WBuf {
  __amdgpu_buffer_rsrc_t rs;
  int voff;  // lane * 16
  int pl;
  __device__ __forceinline__ bf16x8_t operator()(int plane, int off) const {
    return __builtin_bit_cast(bf16x8_t,
                              __builtin_amdgcn_raw_buffer_load_b128(rs, voff, plane * pl + off, 0));
  }
};
__device__ __forceinline__ WBuf wbuf(const void* img, int bytes, int pl, int lane) {
  return WBuf{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(img), 0, bytes, 0x00020000),
              lane * 16, pl};
}
// planes in LDS for bit p of MASK, else global
template <int MASK>
struct WMix {
  WLds l;
  WBuf g;
  __device__ __forceinline__ bf16x8_t operator()(int plane, int off) const {
    return ((MASK >> plane) & 1) ? l(plane, off) : g(plane, off);
  }
};

struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// acc[t][m] += W[m-tile m0 + m] . B_t over KS k-steps for RT row tiles t; W an x3 image of
// MTW M-tiles; bop(s, t) returns the split B operand of k-step s, row tile t.  Per k-step
// the A fragments are issued first and the B operands are split while they arrive; the
// small terms go first.
// DB: the A fragments of k-step s + 1 are issued before the MFMAs of step s (double
// buffer: MT * 12 more registers, no wait on the fragment loads between k-steps).
// pre1 (RT = 2): the previous layer's epilogue of row tile 1, run after row tile 0's first
// MFMAs are issued instead of before the layer -- a one-k-step skew of the two row tiles at
// the layer boundary, so that epilogue (row statistics, a dependent reduction) issues while
// the matrix pipe works on tile 0 rather than in front of an idle pipe.
template <int KS, int MT, int MTW, int RT, int DB = 0, typename WSrc, typename BOp,
          typename Hook = NoHook>
__device__ __forceinline__ void layer_x3(f32x16 (&acc)[RT][MT], const WSrc& W, int m0, BOp&& bop,
                                         Hook&& pre1 = Hook{}) {
  constexpr bool LAZY = RT == 2 && !std::is_same<std::decay_t<Hook>, NoHook>::value;
  // DB: A fragments read DB k-steps ahead (a ring of DB + 1 buffers); 0: at their step
  constexpr int NBUF = DB + 1;
  bf16x8_t Ab[NBUF][MT][3];
  auto lda = [&](int s, bf16x8_t (&d)[MT][3]) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int p = 0; p < 3; ++p) d[m][p] = W(p, ((m0 + m) * KS + s) * 1024);
  };
  if constexpr (DB > 0) {
#pragma unroll
    for (int q = 0; q < DB && q < KS; ++q) lda(q, Ab[q % NBUF]);
  }
  // B operands one k-step ahead (RG_X3_PIPE): the split of step s + 1 is independent of
  // step s's MFMAs, so its VALU work can issue in their shadow instead of between them
  X3 bq[RG_X3_PIPE ? RT : 1];
  if constexpr (RG_X3_PIPE) {
#pragma unroll
    for (int t = 0; t < (LAZY ? 1 : RT); ++t) bq[t] = bop(0, t);
  } else if constexpr (LAZY) {
    static_assert(!LAZY, "pre1 needs the B-operand pipeline");
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if constexpr (DB > 0) {
      if (s + DB < KS) lda(s + DB, Ab[(s + DB) % NBUF]);
    } else {
      lda(s, Ab[0]);
    }
    const bf16x8_t(&A)[MT][3] = Ab[DB > 0 ? s % NBUF : 0];
    X3 bn[RG_X3_PIPE ? RT : 1];
    if constexpr (RG_X3_PIPE) {
      if (s + 1 < KS) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
          if (!(LAZY && s == 0 && t == 1)) bn[t] = bop(s + 1, t);
      }
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      if constexpr (LAZY) {
        if (s == 0 && t == 1) {  // tile 0's first MFMAs are issued: tile 1's epilogue now
          pre1();
          bq[1] = bop(0, 1);
          if (s + 1 < KS) bn[1] = bop(1, 1);
        }
      }
      const X3 b = RG_X3_PIPE ? bq[t] : bop(s, t);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][2], b.p0, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][1], b.p1, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][0], b.p2, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][1], b.p0, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][0], b.p1, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][0], b.p0, acc[t][m]);
    }
    if constexpr (RG_X3_PIPE) {
      if (s + 1 < KS) {
#pragma unroll
        for (int t = 0; t < RT; ++t) bq[t] = bn[t];
      }
    }
    // RG_X3_LASTSB 0: no fence after the last k-step, so the caller's epilogue of row tile 0
    // may interleave with the last MFMAs of the other row tiles
    if (RG_X3_LASTSB || s + 1 < KS) __builtin_amdgcn_sched_barrier(0);
  }
}
// The same products in the same order per accumulator as layer_x3 (one row tile), issued
// M-tile by M-tile: the six MFMAs of tile m chain on acc[m] back to back, and only two
// M-tiles' A fragments are live (the next tile's three are read while the current tile's
// MFMAs run: 24 registers instead of MT * 12).  Bit-identical to layer_x3.
template <int KS, int MT, typename WSrc, typename BOp>
__device__ __forceinline__ void layer_x3_mo(f32x16 (&acc)[MT], const WSrc& W, int m0, BOp&& bop) {
  auto lda = [&](int s, int m, bf16x8_t (&d)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) d[p] = W(p, ((m0 + m) * KS + s) * 1024);
  };
  X3 bq = bop(0);
  bf16x8_t A[2][3];
  lda(0, 0, A[0]);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    X3 bn;
    if (s + 1 < KS) bn = bop(s + 1);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int u = (s * MT + m) & 1;
      if (m + 1 < MT) lda(s, m + 1, A[u ^ 1]);
      else if (s + 1 < KS) lda(s + 1, 0, A[u ^ 1]);
      acc[m] = mf(A[u][2], bq.p0, acc[m]);
      acc[m] = mf(A[u][1], bq.p1, acc[m]);
      acc[m] = mf(A[u][0], bq.p2, acc[m]);
      acc[m] = mf(A[u][1], bq.p0, acc[m]);
      acc[m] = mf(A[u][0], bq.p1, acc[m]);
      acc[m] = mf(A[u][0], bq.p0, acc[m]);
    }
    if (s + 1 < KS) bq = bn;
    __builtin_amdgcn_sched_barrier(0);
  }
}

// one row tile
template <int KS, int MT, int MTW, int DB = 0, typename WSrc, typename BOp>
__device__ __forceinline__ void layer_x3(f32x16 (&acc)[MT], const WSrc& W, int m0, BOp&& bop) {
  layer_x3<KS, MT, MTW, 1, DB>(*reinterpret_cast<f32x16(*)[1][MT]>(&acc), W, m0,
                               [&](int s, int) { return bop(s); });
}

static constexpr float X3_NORM_EPS = 1e-5f;  // constants.py:9
static constexpr float X3_LEAKY_PRE = 0.505f;
static constexpr float X3_LEAKY_C = 0.495f / 0.505f;

// row statistics of channel_normalization over the 32 MT features of a lane pair: eight
// independent partial sums per statistic (short dependent chains: the epilogue sits on the
// critical path between two layers), then one v_permlane32_swap each.  1 / (std + eps)
// from the hardware sqrt and reciprocal (~1 ulp each, 2e-7 relative on the scale; the
// float32 MFMA path keeps the correctly rounded sequences).  CENT: the layer's weights and
// bias were packed zero-mean over the outputs (RG_LAYER_CENTERED), so the row mean of the
// pre-activations is zero up to f32 rounding and its pass is skipped -- the normalisation
// is invariant to the shift, and the centred form avoids the cancellation of x - mean.
template <int MT, bool CENT>
__device__ __forceinline__ float row_inv_std(f32x16 (&acc)[MT]) {
  constexpr int N = 32 * MT;
  if constexpr (!CENT) {
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = acc[0][i] + acc[0][i + 8];
#pragma unroll
    for (int m = 1; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) s[q & 7] += acc[m][q];
    const float mean =
        add_xor32(((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]))) * (1.f / N);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] -= mean;
  }
  float u[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = acc[0][i] * acc[0][i];
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = fmaf(acc[0][i + 8], acc[0][i + 8], u[i]);
#pragma unroll
  for (int m = 1; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) u[q & 7] = fmaf(acc[m][q], acc[m][q], u[q & 7]);
  const float ss = add_xor32(((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7])));
  return __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(ss * (1.f / (float)(N - 1))) + X3_NORM_EPS);
}

// channel_normalization (common.py:208-220) + LeakyReLU (common.py:256-267, constants.py:10):
// after the statistics, two fmas per feature -- y' = x a + b with the 0.505 of
// leaky(y) = 0.505 y + 0.495 |y| folded into a and b, then |y'| C + y'
template <int MT, bool CENT = false>
__device__ __forceinline__ void norm_leaky(f32x16 (&acc)[MT], float mu, float sd) {
  const float inv = row_inv_std<MT, CENT>(acc);  // acc now centred
  const float ga = X3_LEAKY_PRE * (sd * inv), gb = X3_LEAKY_PRE * mu;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x2 y = {fmaf(acc[m][2 * i], ga, gb), fmaf(acc[m][2 * i + 1], ga, gb)};
      set_pair(acc[m], i, (f32x2){fmaf(fabsf(y.x), X3_LEAKY_C, y.x), fmaf(fabsf(y.y), X3_LEAKY_C, y.y)});
    }
}

// channel_normalization without activation
template <int MT, bool CENT = false>
__device__ __forceinline__ void norm_only(f32x16 (&acc)[MT], float mu, float sd) {
  const float ga = sd * row_inv_std<MT, CENT>(acc);
  const f32x2 ga2 = {ga, ga}, mu2 = {mu, mu};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; ++i) set_pair(acc[m], i, fma2(pair(acc[m], i), ga2, mu2));
}

// A normalised layer's scale and activation applied when the NEXT layer reads it, eight
// values per k-step (its B operand), instead of over the whole tile between the layers:
// that VALU work then issues beside the next layer's MFMAs (layer_x3's one-step-ahead B).
// PEND 1: norm + LeakyReLU (ga, gb as in norm_leaky), 2: norm only, 0: nothing pending.
struct Pend {
  float ga, gb;
};
template <int MT, bool CENT>
__device__ __forceinline__ Pend pend_norm_leaky(f32x16 (&acc)[MT], float mu, float sd) {
  const float inv = row_inv_std<MT, CENT>(acc);
  return Pend{X3_LEAKY_PRE * (sd * inv), X3_LEAKY_PRE * mu};
}
template <int MT, bool CENT>
__device__ __forceinline__ Pend pend_norm_only(f32x16 (&acc)[MT], float mu, float sd) {
  return Pend{sd * row_inv_std<MT, CENT>(acc), mu};
}
template <int PEND>
__device__ __forceinline__ X3 split_acc_pend(const f32x16& t, int hf, Pend p) {
  if constexpr (PEND == 0) {
    return split_acc(t, hf);
  } else {
    const int q = 8 * hf;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float y = fmaf(t[q + i], p.ga, p.gb);
      if constexpr (PEND == 1) y = fmaf(fabsf(y), X3_LEAKY_C, y);
      v[i] = y;
    }
    return split8((f32x4){v[0], v[1], v[2], v[3]}, (f32x4){v[4], v[5], v[6], v[7]});
  }
}

}  // namespace x3
}  // namespace rg
