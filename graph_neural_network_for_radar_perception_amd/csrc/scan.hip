// Exclusive prefix sums (int32) used by every CSR builder in the library.
// Small arrays: one launch (scan_small); larger: three launches, per-block sums -> scan of
// the block sums -> add offsets.
#include "rg_common.h"
#include "scan.h"

namespace rg {

static constexpr int SCAN_BLOCK = 256;
static constexpr int SCAN_ITEMS = 8;  // elements per thread
static constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// block-wide exclusive scan of one int per thread; returns the block total in *total
__device__ int block_excl_scan(int v, int* total) {
  __shared__ int wsum[SCAN_BLOCK / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = wave_incl_scan(v);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < SCAN_BLOCK / 64; ++w) {
    int s = wsum[w];
    if (w < wid) off += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

__global__ __launch_bounds__(SCAN_BLOCK) void scan_block_sums(const int* __restrict__ in, long n,
                                                              int* __restrict__ block_sums) {
  long base = (long)blockIdx.x * SCAN_TILE;
  int s = 0;
#pragma unroll
  for (int t = 0; t < SCAN_ITEMS; ++t) {
    long i = base + (long)t * SCAN_BLOCK + threadIdx.x;
    if (i < n) s += in[i];
  }
  int tot;
  block_excl_scan(s, &tot);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

// single block: exclusive scan of nb block sums in place, writes grand total
__global__ __launch_bounds__(SCAN_BLOCK) void scan_partials(int* __restrict__ sums, int nb,
                                                            int* __restrict__ total_out) {
  int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += SCAN_BLOCK) {
    int i = b0 + threadIdx.x;
    int v = i < nb ? sums[i] : 0;
    int tot;
    int ex = block_excl_scan(v, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void scan_apply(const int* __restrict__ in, long n,
                                                         const int* __restrict__ block_offs,
                                                         int* __restrict__ out) {
  // each thread owns SCAN_ITEMS consecutive elements (coalesced enough: tile is L1/L2 hot)
  long base = (long)blockIdx.x * SCAN_TILE + (long)threadIdx.x * SCAN_ITEMS;
  int v[SCAN_ITEMS];
  int s = 0;
#pragma unroll
  for (int t = 0; t < SCAN_ITEMS; ++t) {
    long i = base + t;
    v[t] = i < n ? in[i] : 0;
    s += v[t];
  }
  int tot;
  int ex = block_excl_scan(s, &tot) + block_offs[blockIdx.x];
#pragma unroll
  for (int t = 0; t < SCAN_ITEMS; ++t) {
    long i = base + t;
    if (i < n) out[i] = ex;
    ex += v[t];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_BLOCK - 1) out[n] = ex;
}

// n <= SMALL_N: ONE launch of one 1024-thread workgroup.  Wave w owns the contiguous chunk
// [2048 w, 2048 w + 2048): coalesced loads into LDS, then lane l scans the 32 consecutive
// elements 32 l .. 32 l + 31 of its chunk serially in registers (LDS rows padded by one
// word per 32: conflict-free), one wave scan of the lane sums, the 16 chunk totals through
// LDS, and coalesced stores.  The three-launch form costs ~15 us of launch floor for a few
// us of work on the graph builders' small arrays.
static constexpr int SMALL_T = 1024;
static constexpr int SMALL_I = 32;
static constexpr long SMALL_N = (long)SMALL_T * SMALL_I;
static constexpr int CHUNK = 64 * SMALL_I;           // elements per wave
static constexpr int CHUNK_P = CHUNK + CHUNK / 32;   // padded LDS words per wave

__device__ __forceinline__ int pad32(int j) { return j + (j >> 5); }

__global__ __launch_bounds__(SMALL_T) void scan_small(const int* __restrict__ in, long n,
                                                      int* __restrict__ out,
                                                      int* __restrict__ total_out) {
  extern __shared__ int sm[];  // SMALL_T / 64 chunk totals, then the padded chunks
  int* wsum = sm;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int* ch = sm + SMALL_T / 64 + wid * CHUNK_P;
  const long base = (long)wid * CHUNK;
  {
    int v[SMALL_I];
#pragma unroll
    for (int k = 0; k < SMALL_I; ++k) {
      const long i = base + 64 * k + lane;
      v[k] = i < n ? in[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < SMALL_I; ++k) ch[pad32(64 * k + lane)] = v[k];
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's chunk is in LDS
  __builtin_amdgcn_wave_barrier();
  int v[SMALL_I];
  int s = 0;
#pragma unroll
  for (int t = 0; t < SMALL_I; ++t) {
    v[t] = ch[pad32(SMALL_I * lane + t)];
  }
#pragma unroll
  for (int t = 0; t < SMALL_I; ++t) {
    const int x = v[t];
    v[t] = s;
    s += x;
  }
  const int inc = wave_incl_scan(s);
  const int lane_off = inc - s;
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < SMALL_T / 64; ++w) {
    const int x = wsum[w];
    if (w < wid) off += x;
    tot += x;
  }
#pragma unroll
  for (int t = 0; t < SMALL_I; ++t) ch[pad32(SMALL_I * lane + t)] = off + lane_off + v[t];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < SMALL_I; ++k) {
    const long i = base + 64 * k + lane;
    if (i < n) out[i] = ch[pad32(64 * k + lane)];
  }
  if (threadIdx.x == 0) {
    out[n] = tot;
    if (total_out) *total_out = tot;
  }
}
static constexpr int SMALL_LDS = (SMALL_T / 64 + (SMALL_T / 64) * CHUNK_P) * 4;

size_t scan_workspace_bytes(long n) {
  long nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  return (size_t)((nb + 1 + 63) / 64 * 64) * sizeof(int);
}

int exclusive_scan(const int* in, long n, int* out, int* total_out, void* ws, hipStream_t st) {
  if (n <= SMALL_N) {
    RG_ENSURE_LDS(scan_small, SMALL_LDS);
    scan_small<<<1, SMALL_T, SMALL_LDS, st>>>(in, n, out, total_out);
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  long nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) nb = 1;
  int* sums = (int*)ws;
  scan_block_sums<<<nb, SCAN_BLOCK, 0, st>>>(in, n, sums);
  scan_partials<<<1, SCAN_BLOCK, 0, st>>>(sums, (int)nb, total_out);
  scan_apply<<<nb, SCAN_BLOCK, 0, st>>>(in, n, sums, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

}  // namespace rg
