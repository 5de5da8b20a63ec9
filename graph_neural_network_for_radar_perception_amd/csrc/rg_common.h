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

// Correctly rounded f32 sqrt / division (numpy semantics).  The hardware f32
// v_sqrt / v_rcp paths are not correctly rounded; the f64 result rounded once
// to f32 is (53 >= 2*24 + 2 bits, so the double rounding is exact).
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }

// MFMA operand / accumulator vector types
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

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

}  // namespace rg
