// Clock calibration for bench.py (not on any product path): the shader clock the chip
// holds right before and right after a timed region, so a bench line can tell a slower
// box (DVFS, a lower-clocked device) from a slower kernel.
//
// Every wave runs one dependent chain of v_mfma_f32_32x32x16_bf16 on non-trivial register
// operands (zero operands raise the clock: MI355X_MICROARCH.md "DVFS give-back" (1), (7))
// and stamps s_memtime (shader cycles) and s_memrealtime (the constant wall clock) around
// the chain; clock = d(memtime) / d(realtime) x wall-clock rate, per workgroup, and the
// host takes the median.  The stamps go only to the probe's own buffer.
#include "rg_common.h"

namespace rg {
namespace {

__global__ __launch_bounds__(256) void clock_probe_kernel(int n_mfma,
                                                          unsigned long long* __restrict__ out,
                                                          float* __restrict__ sink) {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  const int lane = threadIdx.x & 63;
  v8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.25f + 0.001f * (float)((lane * 8 + i) % 97));
    b[i] = (__bf16)(-0.5f + 0.002f * (float)((lane * 5 + 3 * i + blockIdx.x) % 89));
  }
  f32x16 acc = {};
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  // (|a b| summed over 16 products per step stays ~2: 10^5 steps cannot overflow f32); 64
  // MFMAs per loop trip, so the loop's scalar compare and branch sit under the chain
  for (int i = 0; i < n_mfma; i += 64) {
#pragma unroll
    for (int j = 0; j < 64; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i];
  if (lane == 0) sink[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

}  // namespace
}  // namespace rg

extern "C" int rg_clock_probe(int n_blocks, int n_mfma, unsigned long long* out, float* sink,
                              int* wall_clock_khz_host, void* stream) {
  RG_REQUIRE(n_blocks >= 1 && n_blocks <= 65536 && n_mfma >= 64 && n_mfma % 64 == 0 && out && sink,
             RG_ERR_ARG,
             "rg_clock_probe: n_blocks %d n_mfma %d", n_blocks, n_mfma);
  if (wall_clock_khz_host) {
    int dev = 0;
    RG_CHECK_HIP(hipGetDevice(&dev));
    RG_CHECK_HIP(hipDeviceGetAttribute(wall_clock_khz_host, hipDeviceAttributeWallClockRate, dev));
  }
  rg::clock_probe_kernel<<<n_blocks, 256, 0, (hipStream_t)stream>>>(n_mfma, out, sink);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
