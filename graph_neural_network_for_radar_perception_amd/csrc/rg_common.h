// Shared helpers for the radar-GNN HIP library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "../../include/radar_gnn.h"

namespace rg {

// ---------------------------------------------------------------------------
// error reporting: every C-ABI entry point returns 0 or a nonzero code and
// leaves a message retrievable with rg_last_error().
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize, bytes) once per (kernel, device): the
// attribute is per device, and a process may drive several GPUs (thread-safe)
hipError_t ensure_max_lds(const void* kernel, int bytes);

#define RG_ENSURE_LDS(kern, bytes) RG_CHECK_HIP(::rg::ensure_max_lds((const void*)(kern), (bytes)))

#define RG_CHECK_HIP(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      ::rg::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,                \
                      hipGetErrorString(_e));                                     \
      return RG_ERR_HIP;                                                          \
    }                                                                             \
  } while (0)

#define RG_REQUIRE(cond, code, ...)                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      ::rg::set_error(__VA_ARGS__);                                               \
      return (code);                                                              \
    }                                                                             \
  } while (0)

#define RG_LAUNCH_CHECK()                                                         \
  do {                                                                            \
    hipError_t _e = hipGetLastError();                                            \
    if (_e != hipSuccess) {                                                       \
      ::rg::set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__,            \
                      hipGetErrorString(_e));                                     \
      return RG_ERR_HIP;                                                          \
    }                                                                             \
  } while (0)

// a launch whose work counters are re-zeroed by its own last workgroup: when the launch
// fails, re-zero them on the stream so the next launch on this workspace starts from zero
#define RG_LAUNCH_CHECK_ZERO(ctr, bytes, stream)                                  \
  do {                                                                            \
    hipError_t _e = hipGetLastError();                                            \
    if (_e != hipSuccess) {                                                       \
      ::rg::set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__,            \
                      hipGetErrorString(_e));                                     \
      (void)hipMemsetAsync((ctr), 0, (bytes), (hipStream_t)(stream));             \
      return RG_ERR_HIP;                                                          \
    }                                                                             \
  } while (0)

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------
// bf16 <-> f32 (round to nearest even; NaN stays NaN via the hardware cvt)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// round-to-nearest-even through the hardware converter (v_cvt_pk_bf16_f32 on
// gfx950; NaN stays NaN)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16x2_hw v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// Correctly rounded f32 sqrt / division (numpy semantics).  The bare v_sqrt_f32 /
// v_rcp_f32 (and __fsqrt_rn, which is v_sqrt_f32 with denormal scaling) are not
// correctly rounded.  sqrtf compiles (HIP's default correctly rounded f32 sqrt) to
// v_sqrt_f32 plus the exact two-neighbour fma residual fix-up, ~14 f32 instructions;
// the division goes through f64: the f64 quotient rounded once to f32 is exact (53 >=
// 2*24 + 2 bits, so the double rounding cannot differ).
__device__ __forceinline__ float sqrt_rn(float x) { return sqrtf(x); }
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }

// dynamic LDS a kernel may request: 160 KiB per CU minus room for the few static
// __shared__ scalars the fused kernels keep (norm parameters)
static constexpr int DYN_LDS_MAX = 160 * 1024 - 1024;

// MFMA operand / accumulator vector types
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// ---------------------------------------------------------------------------
// The two 16-bit operand types of the half-precision kernels (chain_fast.hip,
// conv_fused.hip, segment_reduce.hip): bf16 (8-bit exponent) and IEEE fp16 (5-bit
// exponent, 3 more mantissa bits; BASELINE config 5).  Same 32x32x16 MFMA shape and rate.
// Conversions from f32 round to nearest even (v_cvt_pk_bf16_f32 / v_cvt_f16_f32).
// ---------------------------------------------------------------------------
typedef _Float16 f16x2_hw __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_f16x2(float lo, float hi) {
  const f16x2_hw v = {(_Float16)lo, (_Float16)hi};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  return (float)__builtin_bit_cast(_Float16, h);
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}

template <bool F16>
struct H16;
template <>
struct H16<false> {  // bf16
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ uint32_t pack2(float a, float b) { return pack_bf16x2(a, b); }
  // the low / high element of a packed pair as f32
  static __device__ __forceinline__ float lo(uint32_t u) { return __uint_as_float(u << 16); }
  static __device__ __forceinline__ float hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
  template <int D>
  static __device__ __forceinline__ float half(uint32_t u, int which) { return which ? hi(u) : lo(u); }
  static __device__ __forceinline__ float to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
  static __device__ __forceinline__ uint16_t from_f32(float f) { return f32_to_bf16(f); }
  static __device__ __forceinline__ f32x16 mfma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static constexpr uint16_t ONE = 0x3f80;
};
template <>
struct H16<true> {  // IEEE fp16
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ uint32_t pack2(float a, float b) { return pack_f16x2(a, b); }
  static __device__ __forceinline__ float lo(uint32_t u) { return f16_to_f32((uint16_t)(u & 0xffffu)); }
  static __device__ __forceinline__ float hi(uint32_t u) { return f16_to_f32((uint16_t)(u >> 16)); }
  template <int D>
  static __device__ __forceinline__ float half(uint32_t u, int which) { return which ? hi(u) : lo(u); }
  static __device__ __forceinline__ float to_f32(uint16_t h) { return f16_to_f32(h); }
  static __device__ __forceinline__ uint16_t from_f32(float f) { return f32_to_f16(f); }
  static __device__ __forceinline__ f32x16 mfma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static constexpr uint16_t ONE = 0x3c00;
};


// activation codes (Activation, common.py:256-267)
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY = 2, ACT_SWISH = 3 };

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == ACT_LEAKY) return v > 0.f ? v : v * 0.01f;   // constants.py:10
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_SWISH) return v / (1.f + expf(-v));
  return v;
}

template <int ACT>
__device__ __forceinline__ float act_t(float v) {
  // leaky: max(v, 0.01 v) == (v > 0 ? v : 0.01 v) for every finite v (slope < 1)
  if constexpr (ACT == ACT_LEAKY) return fmaxf(v, v * 0.01f);
  else if constexpr (ACT == ACT_RELU) return v > 0.f ? v : 0.f;
  else if constexpr (ACT == ACT_SWISH) return v / (1.f + expf(-v));
  else return v;
}

// activation over a whole register array with ONE wave-uniform branch (a
// per-element switch inside unrolled loops explodes into thousands of blocks)
template <typename F>
__device__ __forceinline__ void act_dispatch(int act, F&& f) {
  if (act == ACT_LEAKY) f(std::integral_constant<int, ACT_LEAKY>{});
  else if (act == ACT_RELU) f(std::integral_constant<int, ACT_RELU>{});
  else if (act == ACT_SWISH) f(std::integral_constant<int, ACT_SWISH>{});
  else f(std::integral_constant<int, ACT_NONE>{});
}

// ---------------------------------------------------------------------------
// Row epilogue of the register-resident bf16 kernels (chain_fast.hip, conv_fused.hip):
// a row's MT*32 features live in MT f32x16 MFMA accumulators of one lane pair
// (lane, lane ^ 32).  channel_normalization (common.py:208-220,
// y = s (x - mean) / (std_unbiased + eps) + m) and the activation run in packed f32
// math (v_pk_add_f32 / v_pk_fma_f32 / v_pk_mul_f32: two features per instruction).
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Global -> LDS copy of a weight image by a whole workgroup of NT threads, UNR 16-B loads
// in flight per thread.  (A plain load-store loop waits one full memory round trip per
// 16 B per thread: 145 KB staged by 512 threads was 18 serial round trips.)
template <int NT, int UNR = 8>
__device__ __forceinline__ void stage_lds(void* lds_dst, const void* gsrc, int bytes) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u* s = (const v4u*)gsrc;
  v4u* d = (v4u*)lds_dst;
  const int n = bytes / 16;
  int i = threadIdx.x;
  for (; i + (UNR - 1) * NT < n; i += UNR * NT) {
    v4u v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) v[k] = s[i + k * NT];
#pragma unroll
    for (int k = 0; k < UNR; ++k) d[i + k * NT] = v[k];
  }
  for (; i < n; i += NT) d[i] = s[i];
}

// x[lane] + x[lane ^ 32] with v_permlane32_swap (a VALU lane exchange on gfx950; the
// generic __shfl_xor goes through ds_bpermute and an LDS round trip on the critical path)
__device__ __forceinline__ float add_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// the 16 bias values of M-tile m, lane half h, from a fast-format bias stored in
// accumulator order (rg_pack_linear, pack_bias_frag_kernel): four 16-B reads
__device__ __forceinline__ f32x16 ld_bias_frag(const float* bias, int m, int h) {
  const f32x4* p = (const f32x4*)(bias + (2 * m + h) * 16);
  const f32x4 a = p[0], b = p[1], c = p[2], d = p[3];
  return (f32x16){a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
}

__device__ __forceinline__ f32x2 pair(const f32x16& v, int i) { return (f32x2){v[2 * i], v[2 * i + 1]}; }

// two-feature math: v_pk_*_f32 by default; RG_NO_PK (timing experiments) keeps it scalar
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) {
#ifdef RG_NO_PK
  return (f32x2){fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)};
#else
  return __builtin_elementwise_fma(a, b, c);
#endif
}
__device__ __forceinline__ f32x2 mul2(f32x2 a, f32x2 b) {
#ifdef RG_NO_PK
  return (f32x2){a.x * b.x, a.y * b.y};
#else
  return a * b;
#endif
}
__device__ __forceinline__ f32x2 add2(f32x2 a, f32x2 b) {
#ifdef RG_NO_PK
  return (f32x2){a.x + b.x, a.y + b.y};
#else
  return a + b;
#endif
}
__device__ __forceinline__ void set_pair(f32x16& v, int i, f32x2 p) {
  v[2 * i] = p.x;
  v[2 * i + 1] = p.y;
}

template <int ACT>
__device__ __forceinline__ f32x2 act_pk(f32x2 y) {
  if constexpr (ACT == ACT_LEAKY) {
    // max(y, 0.01 y) (constants.py:10): one v_pk_mul_f32 + two v_max_f32
    const f32x2 z = mul2(y, (f32x2){0.01f, 0.01f});
    float a, b;  // plain v_max_f32: no operand canonicalisation (the compiler would add a
                 // v_max x, x per MFMA-produced operand in IEEE mode)
    asm("v_max_f32 %0, %1, %2" : "=v"(a) : "v"(y.x), "v"(z.x));
    asm("v_max_f32 %0, %1, %2" : "=v"(b) : "v"(y.y), "v"(z.y));
    return (f32x2){a, b};
  } else {
    return (f32x2){act_t<ACT>(y.x), act_t<ACT>(y.y)};
  }
}

// 1 / (sqrt(ss / (N - 1)) + eps) of the bf16 kernels' channel_normalization: the raw
// v_sqrt_f32 and v_rcp_f32 (~1 ulp each) instead of the correctly rounded sequences
// (~20 dependent instructions on the critical path of every epilogue).  The scale they
// feed multiplies values rounded to bf16 right after (2^-9 relative), so the <= 3-ulp
// (2e-7) difference is invisible; the f32 parity path (mlp_chain.hip) stays exact.
__device__ __forceinline__ float inv_std_bf16(float ss, int n, float eps) {
#ifdef RG_EXACT_NORM
  return 1.f / (__fsqrt_rn(ss * (1.f / (float)(n - 1))) + eps);
#else
  return __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(ss * (1.f / (float)(n - 1))) + eps);
#endif
}

template <int MT>
__device__ __forceinline__ void channel_norm_pk(f32x16 (&acc)[MT], float mu, float sd, float eps) {
  constexpr int N = 32 * MT;
  f32x2 s0 = {0.f, 0.f}, s1 = {0.f, 0.f};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      s0 = add2(s0, pair(acc[m], i));
      s1 = add2(s1, pair(acc[m], i + 1));
    }
  const f32x2 st = add2(s0, s1);
  float s = st.x + st.y;
  s = add_xor32(s);
  const float mean = s * (1.f / N);  // N is a power of two: exact
  const f32x2 nm = {-mean, -mean};
  f32x2 q0 = {0.f, 0.f}, q1 = {0.f, 0.f};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const f32x2 d0 = add2(pair(acc[m], i), nm), d1 = add2(pair(acc[m], i + 1), nm);
      q0 = fma2(d0, d0, q0);
      q1 = fma2(d1, d1, q1);
    }
  const f32x2 qt = add2(q0, q1);
  float ss = qt.x + qt.y;
  ss = add_xor32(ss);
  const float inv = inv_std_bf16(ss, N, eps);
  // s*(x-mean)/(std+eps) + m as ONE fma per feature: x*gs + (m - mean*gs)
  const float gs = sd * inv, gb = fmaf(-mean, gs, mu);
  const f32x2 gs2 = {gs, gs}, gb2 = {gb, gb};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; ++i) set_pair(acc[m], i, fma2(pair(acc[m], i), gs2, gb2));
}

// channel_normalization of a CENTRED layer (weights packed with RG_PACK_CENTERED): the
// pre-activations already have zero mean over the features, so only the sum of squares
// is needed (one v_pk_fma_f32 per two features) -- the mean pass disappears.
template <int MT>
__device__ __forceinline__ void channel_norm_pk_centered(f32x16 (&acc)[MT], float mu, float sd,
                                                         float eps) {
  constexpr int N = 32 * MT;
  f32x2 q0 = {0.f, 0.f}, q1 = {0.f, 0.f};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const f32x2 d0 = pair(acc[m], i), d1 = pair(acc[m], i + 1);
      q0 = fma2(d0, d0, q0);
      q1 = fma2(d1, d1, q1);
    }
  const f32x2 qt = add2(q0, q1);
  float ss = qt.x + qt.y;
  ss = add_xor32(ss);
  const float inv = inv_std_bf16(ss, N, eps);
  const float gs = sd * inv;
  const f32x2 gs2 = {gs, gs}, mu2 = {mu, mu};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; ++i) set_pair(acc[m], i, fma2(pair(acc[m], i), gs2, mu2));
}

// channel_normalization of a CENTRED layer fused with LeakyReLU(0.01) (constants.py:10):
// leaky(y) = 0.505 y + 0.495 |y|, and |.| is a free source modifier of v_fma_f32, so with
// y' = 0.505 y = x (0.505 gs) + 0.505 mu (one fma, the 0.505 folded into the row scale)
// the activation is ONE fma per feature, out = |y'| C + y', C = 0.495 / 0.505 -- instead
// of a multiply and a max.  Exact up to f32 rounding: y > 0 gives y' (1 + C) = y (1 +-
// a few ulp), y < 0 gives 0.01 y to ~3e-6 relative (the cancellation in 1 - C), far
// below the bf16 rounding the result goes through next.
static constexpr float LEAKY_PRE = 0.505f;
static constexpr float LEAKY_C = 0.495f / 0.505f;

// the row statistics of channel_norm_leaky_centered: y' = x gs + gb then |y'| C + y'
template <int MT>
__device__ __forceinline__ f32x2 norm_leaky_scale(const f32x16 (&acc)[MT], float mu, float sd,
                                                  float eps) {
  constexpr int N = 32 * MT;
  f32x2 q0 = {0.f, 0.f}, q1 = {0.f, 0.f};
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const f32x2 d0 = pair(acc[m], i), d1 = pair(acc[m], i + 1);
      q0 = fma2(d0, d0, q0);
      q1 = fma2(d1, d1, q1);
    }
  const f32x2 qt = add2(q0, q1);
  float ss = qt.x + qt.y;
  ss = add_xor32(ss);
  const float inv = inv_std_bf16(ss, N, eps);
  return (f32x2){LEAKY_PRE * (sd * inv), LEAKY_PRE * mu};
}

template <int MT>
__device__ __forceinline__ void channel_norm_leaky_centered(f32x16 (&acc)[MT], float mu, float sd,
                                                            float eps) {
  const f32x2 sc = norm_leaky_scale<MT>(acc, mu, sd, eps);
  const float gs = sc.x;
  const f32x2 gs2 = {gs, gs}, mu2 = {LEAKY_PRE * mu, LEAKY_PRE * mu};
  // all of a tile's packed fmas first, then the scalar ones: a v_fma_f32 reading a
  // v_pk_fma_f32 result right after it costs an s_nop (gfx950 hazard) -- one per pair
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    f32x2 y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = fma2(pair(acc[m], i), gs2, mu2);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      set_pair(acc[m], i, (f32x2){fmaf(fabsf(y[i].x), LEAKY_C, y[i].x),
                                  fmaf(fabsf(y[i].y), LEAKY_C, y[i].y)});
  }
}

template <int ACT, int MT>
__device__ __forceinline__ void act_pk_all(f32x16 (&acc)[MT]) {
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 8; ++i) set_pair(acc[m], i, act_pk<ACT>(pair(acc[m], i)));
}

// normalisation (if has_norm; mu / sd are the channel_normalization scalars, read once
// per kernel -- a per-tile load of them would be a vector-memory load whose wait also
// drains every prefetch in flight) + activation; ACT >= 0: compile-time activation applied when
// act == ACT (any other act is the identity, as checked by the launchers); ACT < 0:
// one run-time dispatch
template <int ACT, int MT>
__device__ __forceinline__ void norm_act_rows(f32x16 (&acc)[MT], bool has_norm, float mu, float sd,
                                              int act, float eps, bool centered) {
  if (has_norm) {
    if (centered) channel_norm_pk_centered<MT>(acc, mu, sd, eps);
    else channel_norm_pk<MT>(acc, mu, sd, eps);
  }
  if constexpr (ACT >= 0) {
    if (act == ACT) act_pk_all<ACT, MT>(acc);
  } else {
    act_dispatch(act, [&](auto A) { act_pk_all<decltype(A)::value, MT>(acc); });
  }
}

}  // namespace rg
