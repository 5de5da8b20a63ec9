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
// Layout: 16 lanes per segment, 4 consecutive channels per lane (16-B f32 /
// 8-B bf16 loads), 4 segments per wave.  Rows of a segment are read in segment
// order and summed sequentially, so for a destination-major CSR whose sources
// ascend the f32 sum is bit-identical to the reference scatter_add_ order.
// Reads are unrolled 4 deep to keep several row loads in flight per lane.
#include "rg_common.h"

namespace rg {

template <typename TS, typename TO, int OP>
__global__ __launch_bounds__(256) void segment_reduce_kernel(const TS* __restrict__ src, int ld_src,
                                                             const int* __restrict__ seg_ptr,
                                                             const int* __restrict__ idx,
                                                             int n_seg, int C,
                                                             TO* __restrict__ out, int ld_out) {
  const int g = threadIdx.x & 15;
  const int seg_in_block = threadIdx.x >> 4;
  const int stride = gridDim.x * 16;
  for (int s = blockIdx.x * 16 + seg_in_block; s < n_seg; s += stride) {
    const int b = seg_ptr[s], e = seg_ptr[s + 1];
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + 4 * g;
      if (c >= C) continue;
      float a0, a1, a2, a3;
      if (OP == RG_REDUCE_MAX) {
        a0 = a1 = a2 = a3 = -__int_as_float(0x7f800000);
      } else {
        a0 = a1 = a2 = a3 = 0.f;
      }
      auto load4 = [&](int p, float& v0, float& v1, float& v2, float& v3) {
        const size_t row = idx ? (size_t)idx[p] : (size_t)p;
        if constexpr (sizeof(TS) == 4) {
          const f32x4 v = *(const f32x4*)((const float*)src + row * ld_src + c);
          v0 = v.x; v1 = v.y; v2 = v.z; v3 = v.w;
        } else {
          const uint2 v = *(const uint2*)((const uint16_t*)src + row * ld_src + c);
          v0 = __uint_as_float(v.x << 16);
          v1 = __uint_as_float(v.x & 0xffff0000u);
          v2 = __uint_as_float(v.y << 16);
          v3 = __uint_as_float(v.y & 0xffff0000u);
        }
      };
      auto acc = [&](float v0, float v1, float v2, float v3) {
        if (OP == RG_REDUCE_MAX) {
          a0 = fmaxf(a0, v0); a1 = fmaxf(a1, v1); a2 = fmaxf(a2, v2); a3 = fmaxf(a3, v3);
        } else {
          a0 = __fadd_rn(a0, v0); a1 = __fadd_rn(a1, v1);
          a2 = __fadd_rn(a2, v2); a3 = __fadd_rn(a3, v3);
        }
      };
      int p = b;
      for (; p + 4 <= e; p += 4) {
        float x[4][4];
        load4(p, x[0][0], x[0][1], x[0][2], x[0][3]);
        load4(p + 1, x[1][0], x[1][1], x[1][2], x[1][3]);
        load4(p + 2, x[2][0], x[2][1], x[2][2], x[2][3]);
        load4(p + 3, x[3][0], x[3][1], x[3][2], x[3][3]);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc(x[u][0], x[u][1], x[u][2], x[u][3]);
      }
      for (; p < e; ++p) {
        float v0, v1, v2, v3;
        load4(p, v0, v1, v2, v3);
        acc(v0, v1, v2, v3);
      }
      if (OP == RG_REDUCE_MAX) {
        if (e == b) a0 = a1 = a2 = a3 = 0.f;
      } else if (OP == RG_REDUCE_MEAN) {
        const float n = (float)(e - b > 0 ? e - b : 1);
        a0 = __fdiv_rn(a0, n); a1 = __fdiv_rn(a1, n); a2 = __fdiv_rn(a2, n); a3 = __fdiv_rn(a3, n);
      }
      TO* o = out + (size_t)s * ld_out + c;
      if constexpr (sizeof(TO) == 4) {
        *(f32x4*)o = (f32x4){a0, a1, a2, a3};
      } else {
        uint2 w;
        w.x = pack_bf16x2(a0, a1);
        w.y = pack_bf16x2(a2, a3);
        *(uint2*)o = w;
      }
    }
  }
}

template <typename TS, typename TO>
static void launch_seg(int op, int grid, hipStream_t st, const void* src, int ld_src,
                       const int* seg_ptr, const int* idx, int n_seg, int C, void* out,
                       int ld_out) {
  if (op == RG_REDUCE_SUM)
    segment_reduce_kernel<TS, TO, RG_REDUCE_SUM><<<grid, 256, 0, st>>>(
        (const TS*)src, ld_src, seg_ptr, idx, n_seg, C, (TO*)out, ld_out);
  else if (op == RG_REDUCE_MEAN)
    segment_reduce_kernel<TS, TO, RG_REDUCE_MEAN><<<grid, 256, 0, st>>>(
        (const TS*)src, ld_src, seg_ptr, idx, n_seg, C, (TO*)out, ld_out);
  else
    segment_reduce_kernel<TS, TO, RG_REDUCE_MAX><<<grid, 256, 0, st>>>(
        (const TS*)src, ld_src, seg_ptr, idx, n_seg, C, (TO*)out, ld_out);
}

}  // namespace rg

using namespace rg;

extern "C" int rg_segment_reduce(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                                 const int* idx, int n_seg, int C, int op, void* out,
                                 int out_dtype, int ld_out, void* stream) {
  RG_REQUIRE(op >= RG_REDUCE_SUM && op <= RG_REDUCE_MAX, RG_ERR_ARG, "bad reduce op %d", op);
  RG_REQUIRE(C > 0 && C <= 256 && C % 4 == 0 && ld_src % 4 == 0 && ld_out % 4 == 0,
             RG_ERR_UNSUPPORTED, "rg_segment_reduce: C=%d ld_src=%d ld_out=%d must be multiples of 4",
             C, ld_src, ld_out);
  if (n_seg <= 0) return RG_OK;
  int grid = ceil_div(n_seg, 16);
  if (grid > 16384) grid = 16384;
  hipStream_t st = (hipStream_t)stream;
  if (src_dtype == RG_F32 && out_dtype == RG_F32)
    launch_seg<float, float>(op, grid, st, src, ld_src, seg_ptr, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_BF16 && out_dtype == RG_F32)
    launch_seg<uint16_t, float>(op, grid, st, src, ld_src, seg_ptr, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_BF16 && out_dtype == RG_BF16)
    launch_seg<uint16_t, uint16_t>(op, grid, st, src, ld_src, seg_ptr, idx, n_seg, C, out, ld_out);
  else if (src_dtype == RG_F32 && out_dtype == RG_BF16)
    launch_seg<float, uint16_t>(op, grid, st, src, ld_src, seg_ptr, idx, n_seg, C, out, ld_out);
  else
    RG_REQUIRE(false, RG_ERR_ARG, "rg_segment_reduce: bad dtypes");
  RG_LAUNCH_CHECK();
  return RG_OK;
}
