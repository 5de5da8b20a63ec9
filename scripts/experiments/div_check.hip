// Exhaustive check (per divisor) of the reciprocal-and-one-correction quotient against the
// correctly rounded division: q = x * r, e = fma(-q, d, x), q' = e == 0 ? q : fma(e, r, q)
// with r = RN(1 / d), for every positive float x in [2^-100, 2^100) and a set of divisors
// (the channel norm's per-row denominator std + eps, >= 1e-5).  Prints mismatches per divisor.
// Build: hipcc -O3 --offload-arch=gfx950 div_check.hip -o div_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

__global__ void check(const float* __restrict__ dens, int nd, uint32_t lo, uint32_t n,
                      unsigned long long* __restrict__ bad, uint32_t* __restrict__ first) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (int k = 0; k < nd; ++k) {
    const float d = dens[k];
    const float r = __fdiv_rn(1.0f, d);
    unsigned long long cnt = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const uint32_t bits = lo + i;
      float x;
      memcpy(&x, &bits, 4);
      const float want = __fdiv_rn(x, d);
      const float q = __fmul_rn(x, r);
      const float e = fmaf(-q, d, x);
      const float got = e == 0.f ? q : fmaf(e, r, q);
      if (__float_as_uint(got) != __float_as_uint(want)) {
        ++cnt;
        atomicMin(first + k, bits);
      }
    }
    if (cnt) atomicAdd(bad + k, cnt);
  }
}

int main() {
  std::vector<float> dens = {1.0f, 1e-5f, 1.00001f, 0.1f, 3.0f, 10.0f, 1.5f, 0.75f, 7.0f, 1e3f,
                             0.3333333f, 123.456f};
  uint32_t u;
  u = 0x3fffffffu; float f; memcpy(&f, &u, 4); dens.push_back(f);  // 2 - 2^-23
  u = 0x3f800001u; memcpy(&f, &u, 4); dens.push_back(f);           // 1 + 2^-23
  u = 0x3f7fffffu; memcpy(&f, &u, 4); dens.push_back(f);           // 1 - 2^-24
  u = 0x3fb504f3u; memcpy(&f, &u, 4); dens.push_back(f);           // ~sqrt 2
  std::mt19937 g(1234);
  std::uniform_real_distribution<float> ex(-16.f, 12.f);
  while (dens.size() < 48) dens.push_back(std::exp2(ex(g)) * (1.0f + 1e-5f));
  std::uniform_int_distribution<uint32_t> man(0, (1u << 23) - 1);
  for (int i = 0; i < 16; ++i) {  // random mantissas at exponent 0
    uint32_t b = 0x3f800000u | man(g);
    memcpy(&f, &b, 4);
    dens.push_back(f);
  }
  const int nd = (int)dens.size();
  const uint32_t lo = 0x0d800000u, hi = 0x71800000u;  // [2^-100, 2^100)
  float* dd; unsigned long long* bad; uint32_t* first;
  hipMalloc(&dd, nd * 4); hipMalloc(&bad, nd * 8); hipMalloc(&first, nd * 4);
  hipMemcpy(dd, dens.data(), nd * 4, hipMemcpyHostToDevice);
  hipMemset(bad, 0, nd * 8);
  hipMemset(first, 0xff, nd * 4);
  check<<<8192, 256>>>(dd, nd, lo, hi - lo, bad, first);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
  std::vector<unsigned long long> hb(nd); std::vector<uint32_t> hf(nd);
  hipMemcpy(hb.data(), bad, nd * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hf.data(), first, nd * 4, hipMemcpyDeviceToHost);
  unsigned long long tot = 0;
  for (int k = 0; k < nd; ++k) {
    tot += hb[k];
    if (hb[k]) printf("d=%.9g mismatches=%llu first x bits=%08x\n", dens[k], hb[k], hf[k]);
  }
  printf("divisors=%d x per divisor=%u total mismatches=%llu\n", nd, hi - lo, tot);
  return tot ? 1 : 0;
}
