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

// 8 consecutive k values of one row -> the three exact bf16 terms
__device__ __forceinline__ X3 split8(const f32x4 lo, const f32x4 hi) {
  const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4 w0, w1, w2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = v[2 * i], b = v[2 * i + 1];
    const uint32_t u0 = cvt_pk_bf16(a, b);
    const float ra = a - __uint_as_float(u0 << 16), rb = b - __uint_as_float(u0 & 0xffff0000u);
    const uint32_t u1 = cvt_pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(u1 << 16), sb = rb - __uint_as_float(u1 & 0xffff0000u);
    w0[i] = u0;
    w1[i] = u1;
    w2[i] = cvt_pk_bf16(sa, sb);
  }
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

// acc[t][m] += W[m-tile m0 + m] . B_t over KS k-steps for RT row tiles t; W an x3 image of
// MTW M-tiles; bop(s, t) returns the split B operand of k-step s, row tile t.  Per k-step
// the A fragments are issued first and the B operands are split while they arrive; the
// small terms go first.
// DB: the A fragments of k-step s + 1 are issued before the MFMAs of step s (double
// buffer: MT * 12 more registers, no wait on the fragment loads between k-steps).
template <int KS, int MT, int MTW, int RT, bool DB = false, typename WSrc, typename BOp>
__device__ __forceinline__ void layer_x3(f32x16 (&acc)[RT][MT], const WSrc& W, int m0, BOp&& bop) {
  bf16x8_t Ab[DB ? 2 : 1][MT][3];
  auto lda = [&](int s, bf16x8_t (&d)[MT][3]) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int p = 0; p < 3; ++p) d[m][p] = W(p, ((m0 + m) * KS + s) * 1024);
  };
  if constexpr (DB) lda(0, Ab[0]);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if constexpr (DB) {
      if (s + 1 < KS) lda(s + 1, Ab[(s + 1) & 1]);
    } else {
      lda(s, Ab[0]);
    }
    const bf16x8_t(&A)[MT][3] = Ab[DB ? (s & 1) : 0];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const X3 b = bop(s, t);
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
    __builtin_amdgcn_sched_barrier(0);
  }
}
// one row tile
template <int KS, int MT, int MTW, bool DB = false, typename WSrc, typename BOp>
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
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = acc[0][i] * acc[0][i];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = fmaf(acc[0][i + 8], acc[0][i + 8], v[i]);
#pragma unroll
  for (int m = 1; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q & 7] = fmaf(acc[m][q], acc[m][q], v[q & 7]);
  const float ss = add_xor32(((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7])));
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
    for (int q = 0; q < 16; ++q) {
      const float y = fmaf(acc[m][q], ga, gb);
      acc[m][q] = fmaf(fabsf(y), X3_LEAKY_C, y);
    }
}

// channel_normalization without activation
template <int MT, bool CENT = false>
__device__ __forceinline__ void norm_only(f32x16 (&acc)[MT], float mu, float sd) {
  const float ga = sd * row_inv_std<MT, CENT>(acc);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[m][q] = fmaf(acc[m][q], ga, mu);
}

}  // namespace x3
}  // namespace rg
