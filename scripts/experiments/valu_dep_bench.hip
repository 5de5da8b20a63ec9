// Microbenchmark (diagnostic, not product code): cycles per v_mfma_f32_32x32x16_bf16 at one
// wave per SIMD when each MFMA gap carries five VALU instructions that are
//   A: absent (MFMAs back to back: the floor),
//   B: independent of each other,
//   C: one dependent chain (each reads the previous one's result),
//   D: the exact-split pattern (fma, fma |x|, cvt_pk, and, lshl: each reads the previous).
// Inline asm keeps the stream in program order.  Build: hipcc -O3 --offload-arch=gfx950
// scripts/experiments/valu_dep_bench.hip -o valu_dep_bench; run on one GPU.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 256

#define MF "v_mfma_f32_32x32x16_bf16 v[0:15], a[0:3], v[16:19], v[0:15]\n"
#define B5 \
  "v_fma_f32 v20, v30, v31, v32\n v_fma_f32 v21, v30, v31, v33\n v_fma_f32 v22, v30, v31, v34\n" \
  " v_fma_f32 v23, v30, v31, v35\n v_fma_f32 v24, v30, v31, v36\n"
#define C5 \
  "v_fma_f32 v20, v20, v31, v32\n v_fma_f32 v20, v20, v31, v32\n v_fma_f32 v20, v20, v31, v32\n" \
  " v_fma_f32 v20, v20, v31, v32\n v_fma_f32 v20, v20, v31, v32\n"
#define D5 \
  "v_fma_f32 v20, v21, v31, v32\n v_fma_f32 v22, |v20|, s2, v20\n v_cvt_pk_bf16_f32 v23, v22, v20\n" \
  " v_and_b32 v24, 0xffff0000, v23\n v_lshlrev_b32 v21, 16, v24\n"

template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void bench(unsigned long long* out) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (K == 0) {
      asm volatile(MF MF MF MF MF MF MF MF MF MF MF MF ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6",
                   "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v16", "v17", "v18", "v19", "a0", "a1", "a2", "a3", "memory");
    } else if constexpr (K == 1) {
      asm volatile(MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 MF B5 ::: "v0",
                   "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",
                   "v14", "v15", "v20", "v21", "v22", "v23", "v24", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v16", "v17", "v18", "v19", "a0", "a1", "a2", "a3", "memory");
    } else if constexpr (K == 2) {
      asm volatile(MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 MF C5 ::: "v0",
                   "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",
                   "v14", "v15", "v20", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v16", "v17", "v18", "v19", "a0", "a1", "a2", "a3", "memory");
    } else {
      asm volatile(MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 MF D5 ::: "v0",
                   "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",
                   "v14", "v15", "v20", "v21", "v22", "v23", "v24", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v16", "v17", "v18", "v19", "a0", "a1", "a2", "a3", "memory");
    }
  }
  asm volatile("s_nop 0" ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v16", "v17", "v18", "v19", "a0", "a1", "a2", "a3", "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  unsigned long long* d;
  const int G = 256;
  hipMalloc(&d, G * 4 * sizeof(unsigned long long));
  unsigned long long h[G * 4];
  const char* names[4] = {"A back-to-back", "B 5 independent VALU", "C 5-deep chain", "D split chain"};
  for (int rep = 0; rep < 2; ++rep)
    for (int k = 0; k < 4; ++k) {
      hipMemset(d, 0, G * 4 * sizeof(unsigned long long));
      if (k == 0) bench<0><<<G, 256>>>(d);
      if (k == 1) bench<1><<<G, 256>>>(d);
      if (k == 2) bench<2><<<G, 256>>>(d);
      if (k == 3) bench<3><<<G, 256>>>(d);
      hipDeviceSynchronize();
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      double s = 0;
      int n = 0;
      for (int i = 0; i < G * 4; ++i)
        if (h[i]) { s += (double)h[i]; ++n; }
      if (rep == 1) printf("%-22s %.1f cycles per MFMA (%d waves)\n", names[k], s / n / (ITERS * 12.0), n);
    }
  hipFree(d);
  return 0;
}
