// Diagnostic (not product code): is the residual x - f32(bf16(x)) computed by
// v_dot2c_f32_bf16 (the rounded pair times (-1, 0) / (0, -1), accumulated onto x) bit-identical
// to the unpack + v_sub_f32 form the exact 3-term split uses, and what does each cost beside
// MFMAs?  Part 1 splits 64 Mi values (random bits over the whole finite range, plus signed
// zeros, denormals and the largest finite values) both ways and counts differing words.
// Part 2 times 12 MFMAs with five fillers per gap at one wave per SIMD: the fillers one pair
// split level in the sub form (2 unpacks + 2 subs + 1 conversion) vs the dot form (2 dots
// + 1 conversion, then two independent VALU to keep five).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/experiments/dot2_split_check.hip -o scripts/bin/dot2_split_check
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2_t));
}
__device__ __forceinline__ float rlo(uint32_t u, float x) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, u),
                                         __builtin_bit_cast(bf16x2_t, 0x0000bf80u), x, false);
}
__device__ __forceinline__ float rhi(uint32_t u, float y) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, u),
                                         __builtin_bit_cast(bf16x2_t, 0xbf800000u), y, false);
}

__device__ __forceinline__ uint32_t mix(uint32_t h) {
  h ^= h >> 16; h *= 0x7feb352dU; h ^= h >> 15; h *= 0x846ca68bU; h ^= h >> 16;
  return h;
}

__global__ void check(unsigned long long* bad, uint32_t* first) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t bx = mix(2 * i + 1), by = mix(2 * i + 2);
  // keep it finite: clear an all-ones exponent
  if (((bx >> 23) & 0xff) == 0xff) bx &= ~(1u << 30);
  if (((by >> 23) & 0xff) == 0xff) by &= ~(1u << 30);
  if (i < 64) {  // specials
    const uint32_t sp[8] = {0u, 0x80000000u, 1u, 0x807fffffu, 0x7f7fffffu, 0xff7fffffu,
                            0x00800000u, 0x3f808001u};
    bx = sp[i & 7]; by = sp[(i >> 3) & 7];
  }
  const float x = __uint_as_float(bx), y = __uint_as_float(by);
  // sub form
  const uint32_t u0 = cvt(x, y);
  const float sx = x - __uint_as_float(u0 << 16), sy = y - __uint_as_float(u0 & 0xffff0000u);
  const uint32_t s1 = cvt(sx, sy);
  const float tx = sx - __uint_as_float(s1 << 16), ty = sy - __uint_as_float(s1 & 0xffff0000u);
  const uint32_t s2 = cvt(tx, ty);
  // dot form
  const float dx = rlo(u0, x), dy = rhi(u0, y);
  const uint32_t d1 = cvt(dx, dy);
  const float ex = rlo(d1, dx), ey = rhi(d1, dy);
  const uint32_t d2 = cvt(ex, ey);
  const bool ok = s1 == d1 && s2 == d2 && __float_as_uint(sx) == __float_as_uint(dx) &&
                  __float_as_uint(sy) == __float_as_uint(dy);
  if (!ok) {
    if (atomicAdd(bad, 1ull) == 0) {
      first[0] = bx; first[1] = by; first[2] = __float_as_uint(sx); first[3] = __float_as_uint(dx);
      first[4] = __float_as_uint(sy); first[5] = __float_as_uint(dy);
    }
  }
}

#define ITERS 256
#define MF "v_mfma_f32_32x32x16_bf16 v[0:15], a[0:3], v[16:19], v[0:15]\n"
// one split level of a pair in the sub form: unpack x, unpack y, two subs, one conversion
#define SUB5 \
  "v_lshlrev_b32 v22, 16, v21\n v_and_b32 v23, 0xffff0000, v21\n v_sub_f32 v24, v30, v22\n" \
  " v_sub_f32 v25, v31, v23\n v_cvt_pk_bf16_f32 v21, v24, v25\n"
// the dot form: two dots, one conversion, two unrelated fillers
#define DOT5 \
  "v_dot2c_f32_bf16 v24, -1.0, v21\n v_dot2c_f32_bf16 v25, v26, v21\n v_cvt_pk_bf16_f32 v21, v24, v25\n" \
  " v_fma_f32 v32, v33, v34, v35\n v_fma_f32 v36, v33, v34, v35\n"
#define DOT3 \
  "v_dot2c_f32_bf16 v24, -1.0, v21\n v_dot2c_f32_bf16 v25, v26, v21\n v_cvt_pk_bf16_f32 v21, v24, v25\n"
#define CLOB                                                                                   \
  "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", \
      "v15", "v16", "v17", "v18", "v19", "v21", "v22", "v23", "v24", "v25", "v26", "v30", "v31", \
      "v32", "v33", "v34", "v35", "v36", "a0", "a1", "a2", "a3", "memory"

template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void bench(unsigned long long* out) {
  asm volatile("v_mov_b32 v26, 0xbf800000\n v_mov_b32 v21, 0\n v_mov_b32 v30, 0\n v_mov_b32 v31, 0" ::: CLOB);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (K == 0) {
      asm volatile(MF SUB5 MF SUB5 MF SUB5 MF SUB5 MF SUB5 MF SUB5 MF SUB5 MF SUB5 MF SUB5 MF SUB5
                       MF SUB5 MF SUB5 ::: CLOB);
    } else if constexpr (K == 1) {
      asm volatile(MF DOT5 MF DOT5 MF DOT5 MF DOT5 MF DOT5 MF DOT5 MF DOT5 MF DOT5 MF DOT5 MF DOT5
                       MF DOT5 MF DOT5 ::: CLOB);
    } else {
      asm volatile(MF DOT3 MF DOT3 MF DOT3 MF DOT3 MF DOT3 MF DOT3 MF DOT3 MF DOT3 MF DOT3 MF DOT3
                       MF DOT3 MF DOT3 ::: CLOB);
    }
  }
  asm volatile("s_nop 0" ::: CLOB);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 32);
  hipMemset(bad, 0, 8);
  hipMemset(first, 0, 32);
  const int n = 64 << 20;
  check<<<n / 256, 256>>>(bad, first);
  unsigned long long hb = 0;
  uint32_t hf[8];
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(hf, first, 32, hipMemcpyDeviceToHost);
  printf("split check: %d pairs, %llu differ", n, hb);
  if (hb) printf(" (first: x %08x y %08x  sub rx %08x dot rx %08x  sub ry %08x dot ry %08x)", hf[0], hf[1], hf[2], hf[3], hf[4], hf[5]);
  printf("\n");

  unsigned long long* d;
  const int G = 256;
  hipMalloc(&d, G * 4 * sizeof(unsigned long long));
  unsigned long long h[G * 4];
  const char* names[3] = {"sub form (5 per gap)", "dot form + 2 fillers", "dot form alone (3)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int k = 0; k < 3; ++k) {
      hipMemset(d, 0, sizeof(h));
      if (k == 0) bench<0><<<G, 256>>>(d);
      if (k == 1) bench<1><<<G, 256>>>(d);
      if (k == 2) bench<2><<<G, 256>>>(d);
      hipDeviceSynchronize();
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      double s = 0;
      int m = 0;
      for (int i = 0; i < G * 4; ++i)
        if (h[i]) { s += (double)h[i]; ++m; }
      if (rep == 1) printf("%-24s %.3f cycles per MFMA (%d waves)\n", names[k], s / m / (ITERS * 12.0), m);
    }
  hipFree(d);
  return hb ? 1 : 0;
}
