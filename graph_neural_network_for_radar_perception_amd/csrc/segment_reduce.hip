// CSR segmented reductions: the scatter-aggregate of message passing and the
// per-cluster max-pool of the object head.
//
//   PyG MessagePassing aggregation (gnn_blocks.py:57 aggr=cfg.aggregation, yml:55 'add'):
//     out[i] = sum / mean / max over messages whose target is i
//     (reference CPU: new_zeros(N,C).scatter_add_(0, ei[1], msg); PyG max/mean:
//      scatter_reduce include_self=False -> empty segments are 0)
//   object_classification cluster pooling (gnn_blocks.py:384-387):
//     out[c] = max over member rows of the stem output
//
// Layout: one segment per group of 64/VEC lanes, VEC consecutive channels per lane
// (one 16-B load per row and lane: 8 bf16 or 4 f32 channels; 8-B bf16 loads only when
// C or the row stride is not a multiple of 8), so a 64-channel row is one fully used
// 128-B (bf16) / 256-B (f32) line per lane group.  Rows of a segment are read in
// segment order and summed sequentially, so for a destination-major CSR whose sources
// ascend the f32 sum is bit-identical to the reference scatter_add_ order.  Each lane
// keeps U = 8 row loads in flight: the loop issues 8 loads (indices clamped to the
// segment's last row) before the first add, and a row past the end is masked out of
// the sum -- the tail never falls back to one dependent load at a time.
#include "rg_common.h"

namespace rg {

// a lane's VEC channels of one row as loaded (16 B, or 8 B for the bf16 VEC=4 fallback);
// rows in flight stay in this raw form (4 VGPRs per bf16 row instead of 8 unpacked
// floats: 8 waves per SIMD instead of 5) and are unpacked only when summed
template <typename TS, int VEC>
using raw_t = std::conditional_t<sizeof(TS) == 4 || VEC == 8, uint4, uint2>;

template <typename TS, int VEC>
__device__ __forceinline__ raw_t<TS, VEC> load_raw(const TS* __restrict__ p) {
  static_assert(sizeof(TS) == 2 || VEC == 4, "f32 rows: 4 channels per lane");
  return *(const raw_t<TS, VEC>*)p;
}

template <typename TS, int VEC>
__device__ __forceinline__ float chan(const raw_t<TS, VEC>& x, int i) {
  if constexpr (sizeof(TS) == 4) {
    return __uint_as_float(((const uint32_t*)&x)[i]);
  } else {
    const uint32_t w = ((const uint32_t*)&x)[i >> 1];
    return (i & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
  }
}

template <typename TO, int VEC>
__device__ __forceinline__ void store_vec(TO* __restrict__ o, const float (&a)[VEC]) {
  if constexpr (sizeof(TO) == 4) {
#pragma unroll
    for (int i = 0; i < VEC; i += 4) *(f32x4*)(o + i) = (f32x4){a[i], a[i + 1], a[i + 2], a[i + 3]};
  } else if constexpr (VEC == 8) {
    *(uint4*)o = (uint4){pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(a[4], a[5]),
                         pack_bf16x2(a[6], a[7])};
  } else {
    *(uint2*)o = (uint2){pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3])};
  }
}

template <typename TS, typename TO, int OP, int VEC>
__global__ __launch_bounds__(256) void segment_reduce_kernel(const TS* __restrict__ src, int ld_src,
                                                             const int* __restrict__ seg_ptr,
                                                             const int* __restrict__ seg_end,
                                                             const int* __restrict__ idx,
                                                             int n_seg, int C,
                                                             TO* __restrict__ out, int ld_out) {
  constexpr int LPS = 64 / VEC;          // lanes per segment: 64 channels per pass
  constexpr int SPB = 256 / LPS;         // segments per workgroup
  constexpr int U = 8;                   // row loads in flight per lane
  const int g = threadIdx.x % LPS;
  const int seg_in_block = threadIdx.x / LPS;
  const int stride = gridDim.x * SPB;
  for (int s = blockIdx.x * SPB + seg_in_block; s < n_seg; s += stride) {
    const int b = seg_ptr[s], e = seg_end ? seg_end[s] : seg_ptr[s + 1];
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + VEC * g;
      if (c >= C) continue;
      float a[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) a[i] = OP == RG_REDUCE_MAX ? -__int_as_float(0x7f800000) : 0.f;
      for (int p = b; p < e; p += U) {
        raw_t<TS, VEC> x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int q = p + u < e ? p + u : e - 1;
          const size_t row = idx ? (size_t)idx[q] : (size_t)q;
          x[u] = load_raw<TS, VEC>(src + row * ld_src + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (p + u < e) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
              const float v = chan<TS, VEC>(x[u], i);
              a[i] = OP == RG_REDUCE_MAX ? fmaxf(a[i], v) : __fadd_rn(a[i], v);
            }
          }
        }
      }
      if (OP == RG_REDUCE_MAX) {
        if (e == b)
#pragma unroll
          for (int i = 0; i < VEC; ++i) a[i] = 0.f;
      } else if (OP == RG_REDUCE_MEAN) {
        const float n = (float)(e - b > 0 ? e - b : 1);
#pragma unroll
        for (int i = 0; i < VEC; ++i) a[i] = __fdiv_rn(a[i], n);
      }
      store_vec<TO, VEC>(out + (size_t)s * ld_out + c, a);
    }
  }
}

template <typename TS, typename TO, int VEC>
static void launch_seg(int op, hipStream_t st, const void* src, int ld_src, const int* seg_ptr,
                       const int* seg_end, const int* idx, int n_seg, int C, void* out,
                       int ld_out) {
  constexpr int SPB = 256 / (64 / VEC);
  int grid = ceil_div(n_seg, SPB);
  if (grid > 16384) grid = 16384;
  if (op == RG_REDUCE_SUM)
    segment_reduce_kernel<TS, TO, RG_REDUCE_SUM, VEC><<<grid, 256, 0, st>>>(
        (const TS*)src, ld_src, seg_ptr, seg_end, idx, n_seg, C, (TO*)out, ld_out);
  else if (op == RG_REDUCE_MEAN)
    segment_reduce_kernel<TS, TO, RG_REDUCE_MEAN, VEC><<<grid, 256, 0, st>>>(
        (const TS*)src, ld_src, seg_ptr, seg_end, idx, n_seg, C, (TO*)out, ld_out);
  else
    segment_reduce_kernel<TS, TO, RG_REDUCE_MAX, VEC><<<grid, 256, 0, st>>>(
        (const TS*)src, ld_src, seg_ptr, seg_end, idx, n_seg, C, (TO*)out, ld_out);
}

}  // namespace rg

using namespace rg;

static int segment_reduce_impl(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                               const int* seg_end, const int* idx, int n_seg, int C, int op,
                               void* out, int out_dtype, int ld_out, void* stream) {
  RG_REQUIRE(op >= RG_REDUCE_SUM && op <= RG_REDUCE_MAX, RG_ERR_ARG, "bad reduce op %d", op);
  RG_REQUIRE(C > 0 && C <= 256 && C % 4 == 0 && ld_src % 4 == 0 && ld_out % 4 == 0,
             RG_ERR_UNSUPPORTED, "rg_segment_reduce: C=%d ld_src=%d ld_out=%d must be multiples of 4",
             C, ld_src, ld_out);
  if (n_seg <= 0) return RG_OK;
  hipStream_t st = (hipStream_t)stream;
  // bf16 rows: 16-B loads (8 channels per lane) when C and the row stride allow
  const bool v8 = C % 8 == 0 && ld_src % 8 == 0 && (out_dtype == RG_F32 || ld_out % 8 == 0) &&
                  (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0;
  if (src_dtype == RG_F32 && out_dtype == RG_F32)
    launch_seg<float, float, 4>(op, st, src, ld_src, seg_ptr, seg_end, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_BF16 && out_dtype == RG_F32 && v8)
    launch_seg<uint16_t, float, 8>(op, st, src, ld_src, seg_ptr, seg_end, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_BF16 && out_dtype == RG_F32)
    launch_seg<uint16_t, float, 4>(op, st, src, ld_src, seg_ptr, seg_end, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_BF16 && out_dtype == RG_BF16 && v8)
    launch_seg<uint16_t, uint16_t, 8>(op, st, src, ld_src, seg_ptr, seg_end, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_BF16 && out_dtype == RG_BF16)
    launch_seg<uint16_t, uint16_t, 4>(op, st, src, ld_src, seg_ptr, seg_end, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_F32 && out_dtype == RG_BF16)
    launch_seg<float, uint16_t, 4>(op, st, src, ld_src, seg_ptr, seg_end, idx, n_seg, C, out, ld_out);
  else
    RG_REQUIRE(false, RG_ERR_ARG, "rg_segment_reduce: bad dtypes");
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_segment_reduce(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                                 const int* idx, int n_seg, int C, int op, void* out,
                                 int out_dtype, int ld_out, void* stream) {
  return segment_reduce_impl(src, src_dtype, ld_src, seg_ptr, nullptr, idx, n_seg, C, op, out,
                             out_dtype, ld_out, stream);
}

extern "C" int rg_segment_reduce_ranges(const void* src, int src_dtype, int ld_src,
                                        const int* seg_begin, const int* seg_end, int n_seg, int C,
                                        int op, void* out, int out_dtype, int ld_out,
                                        void* stream) {
  RG_REQUIRE(seg_begin && seg_end, RG_ERR_ARG, "rg_segment_reduce_ranges: begin / end missing");
  return segment_reduce_impl(src, src_dtype, ld_src, seg_begin, seg_end, nullptr, n_seg, C, op,
                             out, out_dtype, ld_out, stream);
}
