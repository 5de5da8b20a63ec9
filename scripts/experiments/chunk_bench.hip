// Microbenchmark (diagnostic, not product code): one layer-2 sub-chunk of conv_x3_sp_kernel
// exactly as the compiler emitted it (12 MFMAs, their vector fillers and the next k-step's
// fragment reads; the ring-row store at its end left out), looped at one wave per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/experiments/chunk_bench.hip -o scripts/bin/chunk_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 256
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void bench(unsigned long long* out) {
  extern __shared__ char lds[];
  asm volatile("v_mbcnt_lo_u32_b32 v241, -1, 0\n v_mbcnt_hi_u32_b32 v241, -1, v241\n v_lshlrev_b32 v241, 4, v241" ::: "v241");
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("s_waitcnt lgkmcnt(0)\ns_nop 0\nv_mfma_f32_32x32x16_bf16 v[96:111], a[16:19], v[20:23], v[96:111]\nv_fma_f32 v16, v128, v28, v249\nv_fma_f32 v17, |v16|, s5, v16\nv_fma_f32 v16, v129, v28, v249\nv_fma_f32 v18, |v16|, s5, v16\nv_fma_f32 v16, v130, v28, v249\nv_mfma_f32_32x32x16_bf16 v[0:15], a[24:27], v[20:23], v[0:15]\nv_fma_f32 v19, |v16|, s5, v16\nv_fma_f32 v16, v131, v28, v249\nv_fma_f32 v25, |v16|, s5, v16\nv_fma_f32 v16, v132, v28, v249\nv_fma_f32 v26, |v16|, s5, v16\nv_mfma_f32_32x32x16_bf16 v[96:111], a[8:11], v[148:151], v[96:111]\nv_fma_f32 v16, v133, v28, v249\nv_fma_f32 v27, |v16|, s5, v16\nv_fma_f32 v16, v134, v28, v249\nv_fma_f32 v29, |v16|, s5, v16\nv_fma_f32 v16, v135, v28, v249\nv_mfma_f32_32x32x16_bf16 v[0:15], a[0:3], v[148:151], v[0:15]\nv_fma_f32 v30, |v16|, s5, v16\nv_cvt_pk_bf16_f32 v16, v17, v18\nv_and_b32_e32 v24, 0xffff0000, v16\nv_lshlrev_b32_e32 v128, 16, v16\nv_sub_f32_e32 v17, v17, v128\nv_mfma_f32_32x32x16_bf16 v[96:111], a[4:7], v[144:147], v[96:111]\nv_sub_f32_e32 v18, v18, v24\nv_cvt_pk_bf16_f32 v24, v17, v18\nv_lshlrev_b32_e32 v129, 16, v24\nv_and_b32_e32 v128, 0xffff0000, v24\nv_sub_f32_e32 v17, v17, v129\nv_mfma_f32_32x32x16_bf16 v[0:15], a[20:23], v[144:147], v[0:15]\nv_sub_f32_e32 v18, v18, v128\nv_cvt_pk_bf16_f32 v128, v17, v18\nv_cvt_pk_bf16_f32 v17, v19, v25\nv_and_b32_e32 v18, 0xffff0000, v17\nv_lshlrev_b32_e32 v129, 16, v17\nv_mfma_f32_32x32x16_bf16 v[96:111], a[8:11], v[20:23], v[96:111]\nv_sub_f32_e32 v19, v19, v129\nv_sub_f32_e32 v18, v25, v18\nv_cvt_pk_bf16_f32 v25, v19, v18\nv_and_b32_e32 v129, 0xffff0000, v25\nv_lshlrev_b32_e32 v130, 16, v25\nv_mfma_f32_32x32x16_bf16 v[0:15], a[0:3], v[20:23], v[0:15]\nv_sub_f32_e32 v19, v19, v130\nv_sub_f32_e32 v18, v18, v129\nv_cvt_pk_bf16_f32 v129, v19, v18\nv_cvt_pk_bf16_f32 v18, v26, v27\nv_and_b32_e32 v19, 0xffff0000, v18\nds_read_b128 a[0:3], v241 offset:0x1000\nds_read_b128 a[8:11], v241 offset:0x5000\nv_mfma_f32_32x32x16_bf16 v[96:111], a[4:7], v[148:151], v[96:111]\nv_lshlrev_b32_e32 v130, 16, v18\nv_sub_f32_e32 v130, v26, v130\nv_sub_f32_e32 v19, v27, v19\nv_cvt_pk_bf16_f32 v26, v130, v19\nv_and_b32_e32 v27, 0xffff0000, v26\nds_read_b128 a[12:15], v241 offset:0x9000\nds_read_b128 a[16:19], v241 offset:0x3000\nv_mfma_f32_32x32x16_bf16 v[0:15], a[20:23], v[148:151], v[0:15]\nv_lshlrev_b32_e32 v131, 16, v26\nv_sub_f32_e32 v130, v130, v131\nv_sub_f32_e32 v19, v19, v27\nv_cvt_pk_bf16_f32 v130, v130, v19\nv_cvt_pk_bf16_f32 v19, v29, v30\nv_mfma_f32_32x32x16_bf16 v[96:111], a[4:7], v[20:23], v[96:111]\nv_and_b32_e32 v27, 0xffff0000, v19\nv_lshlrev_b32_e32 v131, 16, v19\nv_sub_f32_e32 v29, v29, v131\nv_sub_f32_e32 v30, v30, v27\nv_cvt_pk_bf16_f32 v27, v29, v30\nds_read_b128 a[4:7], v241 offset:0x7000\nds_read_b128 a[24:27], v241 offset:0xb000\nv_mfma_f32_32x32x16_bf16 v[0:15], a[20:23], v[20:23], v[0:15]\nv_and_b32_e32 v20, 0xffff0000, v27\nv_lshlrev_b32_e32 v21, 16, v27\nv_sub_f32_e32 v21, v29, v21\nv_sub_f32_e32 v20, v30, v20\nv_cvt_pk_bf16_f32 v131, v21, v20" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "s5", "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v241", "v249", "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  if (threadIdx.x == 1023) lds[0] = 0;
}
int main() {
  unsigned long long* d;
  const int G = 256;
  hipMalloc(&d, G * 4 * sizeof(unsigned long long));
  unsigned long long h[G * 4];
  hipFuncSetAttribute((const void*)bench, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(d, 0, sizeof(h));
    bench<<<G, 256, 65536>>>(d);
    hipDeviceSynchronize();
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0; int n = 0;
    for (int i = 0; i < G * 4; ++i) if (h[i]) { s += (double)h[i]; ++n; }
    printf("rep %d: %.1f cycles per MFMA of the chunk (%d waves)\n", rep, s / n / (ITERS * 12.0), n);
  }
  return 0;
}
