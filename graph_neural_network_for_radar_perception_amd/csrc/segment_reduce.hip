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

static constexpr int RANGE_BLOCK = 32;   // rows per block maximum (range max-pool)

// a lane's VEC channels of one row as loaded (16 B, or 8 B for the bf16 VEC=4 fallback);
// rows in flight stay in this raw form (4 VGPRs per bf16 row instead of 8 unpacked
// floats: 8 waves per SIMD instead of 5) and are unpacked only when summed
template <typename TS, int VEC>
using raw_t = std::conditional_t<sizeof(TS) == 4 || VEC == 8, uint4, uint2>;

template <typename TS, int VEC, bool NT = false>
__device__ __forceinline__ raw_t<TS, VEC> load_raw(const TS* __restrict__ p) {
  static_assert(sizeof(TS) == 2 || VEC == 4, "f32 rows: 4 channels per lane");
  if constexpr (NT) {
    constexpr int W = sizeof(raw_t<TS, VEC>) / 4;
    typedef uint32_t vw __attribute__((ext_vector_type(W)));
    const vw v = __builtin_nontemporal_load((const vw*)p);
    raw_t<TS, VEC> r;
    __builtin_memcpy(&r, &v, sizeof(r));
    return r;
  } else
    return *(const raw_t<TS, VEC>*)p;
}

// element types: float, uint16_t = bf16 bits, _Float16 = IEEE fp16
template <typename TS, int VEC>
__device__ __forceinline__ float chan(const raw_t<TS, VEC>& x, int i) {
  if constexpr (sizeof(TS) == 4) {
    return __uint_as_float(((const uint32_t*)&x)[i]);
  } else {
    const uint32_t w = ((const uint32_t*)&x)[i >> 1];
    return H16<std::is_same_v<TS, _Float16>>::template half<0>(w, i & 1);
  }
}

template <typename TO, int VEC>
__device__ __forceinline__ void store_vec(TO* __restrict__ o, const float (&a)[VEC]) {
  if constexpr (sizeof(TO) == 4) {
#pragma unroll
    for (int i = 0; i < VEC; i += 4) *(f32x4*)(o + i) = (f32x4){a[i], a[i + 1], a[i + 2], a[i + 3]};
  } else if constexpr (VEC == 8) {
    using H = H16<std::is_same_v<TO, _Float16>>;
    *(uint4*)o = (uint4){H::pack2(a[0], a[1]), H::pack2(a[2], a[3]), H::pack2(a[4], a[5]),
                         H::pack2(a[6], a[7])};
  } else {
    using H = H16<std::is_same_v<TO, _Float16>>;
    *(uint2*)o = (uint2){H::pack2(a[0], a[1]), H::pack2(a[2], a[3])};
  }
}

// rows [b, e) of src (row(p) = idx ? idx[p] : p) folded into a[]: U = 8 row loads in
// flight, indices past e clamped to e - 1 (cache hits) and masked out of the fold
template <typename TS, int VEC, int OP, int U = 8, bool NT = false>
__device__ __forceinline__ void fold_rows(const TS* __restrict__ src, int ld, const int* __restrict__ idx,
                                          int c, int b, int e, float (&a)[VEC]) {
  for (int p = b; p < e; p += U) {
    raw_t<TS, VEC> x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = p + u < e ? p + u : e - 1;
      const size_t row = idx ? (size_t)idx[q] : (size_t)q;
      x[u] = load_raw<TS, VEC, NT>(src + row * ld + c);
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
}

// Segment s covers rows [b, e): b = seg_ptr[s], e = seg_end ? seg_end[s] : seg_ptr[s+1];
// uniform mode (uni > 0): b = s * uni, e = min(b + uni, n_uni) -- the 32-row block maxima
// of the range max-pool.  bm (max only): 32-row block maxima of src; a long range then
// reads its head rows, its whole blocks from bm and its tail rows (exact: max is
// order-free).
template <typename TS, typename TO, int OP, int VEC, int U = 8, bool NT = false>
__global__ __launch_bounds__(256) void segment_reduce_kernel(const TS* __restrict__ src, int ld_src,
                                                             const int* __restrict__ seg_ptr,
                                                             const int* __restrict__ seg_end,
                                                             const int* __restrict__ idx,
                                                             int uni, int n_uni,
                                                             const TS* __restrict__ bm, int ld_bm,
                                                             int n_seg, int C,
                                                             TO* __restrict__ out, int ld_out) {
  constexpr int LPS = 64 / VEC;          // lanes per segment: 64 channels per pass
  constexpr int SPB = 256 / LPS;         // segments per workgroup
  const int g = threadIdx.x % LPS;
  const int seg_in_block = threadIdx.x / LPS;
  const int stride = gridDim.x * SPB;
  for (int s = blockIdx.x * SPB + seg_in_block; s < n_seg; s += stride) {
    int b, e;
    if (uni > 0) {
      b = s * uni;
      e = min(b + uni, n_uni);
    } else {
      b = seg_ptr[s];
      e = seg_end ? seg_end[s] : seg_ptr[s + 1];
    }
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + VEC * g;
      if (c >= C) continue;
      float a[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) a[i] = OP == RG_REDUCE_MAX ? -__int_as_float(0x7f800000) : 0.f;
      if (OP == RG_REDUCE_MAX && bm && e - b >= 2 * RANGE_BLOCK) {
        const int hb = (b + RANGE_BLOCK - 1) / RANGE_BLOCK, te = e / RANGE_BLOCK;
        fold_rows<TS, VEC, OP>(src, ld_src, nullptr, c, b, hb * RANGE_BLOCK, a);
        fold_rows<TS, VEC, OP>(bm, ld_bm, nullptr, c, hb, te, a);
        fold_rows<TS, VEC, OP>(src, ld_src, nullptr, c, te * RANGE_BLOCK, e, a);
      } else {
        fold_rows<TS, VEC, OP, U, NT>(src, ld_src, idx, c, b, e, a);
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

// Short destination segments (kNN graphs: ~13 rows of 128 B per bf16 segment) leave the
// one-segment-per-group kernel a seg_ptr -> rows round trip per 1.6 KiB.  This variant
// gives each lane group G consecutive segments as ONE contiguous row stream
// [seg_ptr[s0], seg_ptr[s0 + G]) (destination-major messages are contiguous): 8 row loads
// in flight across segment boundaries, a finished segment stored and the sum restarted at
// each boundary (segment pointers held one per lane of the group, read by shuffle).  Each
// segment is still summed from its first row in order: bit-identical to the kernel above.
// Sum / mean / max, no row index, C a multiple of 64.
//
// order (G = 1 only, else null): group i reduces segment order[i] (rg_segment_order: longest
// first), so the segments a wave holds have similar lengths -- a wave waits for its longest.
template <typename TS, typename TO, int OP, int VEC, int G, bool NT, int U = 8>
__global__ __launch_bounds__(256) void segment_stream_kernel(const TS* __restrict__ src, int ld_src,
                                                             const int* __restrict__ seg_ptr,
                                                             const int* __restrict__ order,
                                                             int n_seg, int C, TO* __restrict__ out,
                                                             int ld_out) {
  constexpr int LPS = 64 / VEC;
  constexpr int GPB = 256 / LPS;
  static_assert(G <= LPS, "one segment pointer per lane of the group");
  const int g = threadIdx.x % LPS;
  const int lin = (blockIdx.x * GPB + threadIdx.x / LPS) * G;
  if (lin >= n_seg) return;
  const int s0 = (G == 1 && order) ? order[lin] : lin;
  const int ns = min(G, n_seg - lin);
  const int my_ptr = seg_ptr[s0 + min(g, ns)];
  const int p_end = seg_ptr[s0 + ns];
  // ptr_at(j) is called with j uniform over the lane group (all its lanes active)
  auto ptr_at = [&](int j) { return j >= ns ? p_end : __shfl(my_ptr, j, LPS); };
  const int p_beg = ptr_at(0);
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + VEC * g;
    constexpr float A0 = OP == RG_REDUCE_MAX ? -__builtin_inff() : 0.f;
    float a[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) a[i] = A0;
    int s = 0, b_cur = p_beg, e_cur = ptr_at(1);
    auto finish = [&]() {
      if (OP == RG_REDUCE_MEAN) {
        const float n = (float)(e_cur - b_cur > 0 ? e_cur - b_cur : 1);
#pragma unroll
        for (int i = 0; i < VEC; ++i) a[i] = __fdiv_rn(a[i], n);
      } else if (OP == RG_REDUCE_MAX && e_cur == b_cur) {  // empty segment -> 0
#pragma unroll
        for (int i = 0; i < VEC; ++i) a[i] = 0.f;
      }
      store_vec<TO, VEC>(out + (size_t)(s0 + s) * ld_out + c, a);
#pragma unroll
      for (int i = 0; i < VEC; ++i) a[i] = A0;
      ++s;
      b_cur = e_cur;
      e_cur = ptr_at(s + 1);
    };
    for (int p = p_beg; p < p_end; p += U) {
      raw_t<TS, VEC> x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = p + u < p_end ? p + u : p_end - 1;
        x[u] = load_raw<TS, VEC, NT>(src + (size_t)q * ld_src + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p + u < p_end) {
          while (p + u >= e_cur) finish();
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            const float v = chan<TS, VEC>(x[u], i);
            a[i] = OP == RG_REDUCE_MAX ? fmaxf(a[i], v) : __fadd_rn(a[i], v);
          }
        }
      }
    }
    while (s < ns) finish();
  }
}

struct SegArgs {
  const void* src;
  int ld_src;
  const int* seg_ptr;
  const int* order;  // rg_segment_order permutation (streaming kernel, G = 1), or null
  const int* seg_end;
  const int* idx;
  int uni, n_uni;
  const void* bm;
  int ld_bm;
  int n_seg, C;
  void* out;
  int ld_out;
};

// the streaming schedule of a plain CSR: G segments per lane group (0: the one-segment-per-
// group kernel), U rows in flight per lane
struct Sched {
  int G, U;
};
// the compiled (G, U) pairs of the streaming kernel
static bool sched_compiled(Sched s) {
  return s.G == 0 || (s.G == 1 && (s.U == 4 || s.U == 8 || s.U == 12 || s.U == 16)) ||
         (s.G == 2 && (s.U == 4 || s.U == 8)) || (s.G == 4 && s.U == 8);
}

template <typename TS, typename TO, int VEC>
static void launch_seg(int op, hipStream_t st, const SegArgs& g, Sched sc) {
  constexpr int SPB = 256 / (64 / VEC);
  int grid = ceil_div(g.n_seg, SPB);
  if (grid > 16384) grid = 16384;
#define RG_SEG_ARGS                                                                         \
  (const TS*)g.src, g.ld_src, g.seg_ptr, g.seg_end, g.idx, g.uni, g.n_uni, (const TS*)g.bm,   \
      g.ld_bm, g.n_seg, g.C, (TO*)g.out, g.ld_out
  // sum / mean / max over a plain CSR: the streaming kernel, non-temporal row loads (M's
  // CSR, bf16: 0.56 -> 0.70 of HBM with two segments per group; scripts/seg_variants.py).
  // The schedule comes from the caller (default_sched; rg_segment_reduce_sched for sweeps).
  constexpr int GPB = 256 / (64 / VEC);
  if (sc.G > 0 && !g.idx && !g.seg_end && !g.bm && g.uni == 0 && g.C % 64 == 0) {
    int G = g.order ? 1 : sc.G, U = sc.U;
#define RG_STREAM_ARGS \
  (const TS*)g.src, g.ld_src, g.seg_ptr, ord_, g.n_seg, g.C, (TO*)g.out, g.ld_out
#define RG_STREAM(G_, U_)                                                                        \
  {                                                                                              \
    const int grid_s = ceil_div(ceil_div(g.n_seg, G_), GPB);                                     \
    const int* ord_ = G_ == 1 ? g.order : nullptr;                                               \
    if (op == RG_REDUCE_SUM)                                                                     \
      segment_stream_kernel<TS, TO, RG_REDUCE_SUM, VEC, G_, true, U_><<<grid_s, 256, 0, st>>>(   \
          RG_STREAM_ARGS);                                                                       \
    else if (op == RG_REDUCE_MEAN)                                                               \
      segment_stream_kernel<TS, TO, RG_REDUCE_MEAN, VEC, G_, true, U_><<<grid_s, 256, 0, st>>>(  \
          RG_STREAM_ARGS);                                                                       \
    else                                                                                         \
      segment_stream_kernel<TS, TO, RG_REDUCE_MAX, VEC, G_, true, U_><<<grid_s, 256, 0, st>>>(   \
          RG_STREAM_ARGS);                                                                       \
  }
    if (G == 2 && U == 8)
      RG_STREAM(2, 8)
    else if (G == 1 && U == 4)
      RG_STREAM(1, 4)
    else if (G == 2 && U == 4)
      RG_STREAM(2, 4)
    else if (G == 4 && U == 8)
      RG_STREAM(4, 8)
    else if (G == 1 && U == 16)
      RG_STREAM(1, 16)
    else if (G == 1 && U == 12)
      RG_STREAM(1, 12)
    else
      RG_STREAM(1, 8)
#undef RG_STREAM
#undef RG_STREAM_ARGS
  } else if (op == RG_REDUCE_SUM)
    segment_reduce_kernel<TS, TO, RG_REDUCE_SUM, VEC><<<grid, 256, 0, st>>>(RG_SEG_ARGS);
  else if (op == RG_REDUCE_MEAN)
    segment_reduce_kernel<TS, TO, RG_REDUCE_MEAN, VEC><<<grid, 256, 0, st>>>(RG_SEG_ARGS);
  else
    segment_reduce_kernel<TS, TO, RG_REDUCE_MAX, VEC><<<grid, 256, 0, st>>>(RG_SEG_ARGS);
#undef RG_SEG_ARGS
}

// dispatch on (src dtype, out dtype, 16-B / 8-B lanes)
static int launch_any(int op, int src_dtype, int out_dtype, bool v8, hipStream_t st,
                      const SegArgs& g, Sched sc) {
  if (src_dtype == RG_F32 && out_dtype == RG_F32)
    launch_seg<float, float, 4>(op, st, g, sc);
  else if (src_dtype == RG_BF16 && out_dtype == RG_F32 && v8)
    launch_seg<uint16_t, float, 8>(op, st, g, sc);
  else if (src_dtype == RG_BF16 && out_dtype == RG_F32)
    launch_seg<uint16_t, float, 4>(op, st, g, sc);
  else if (src_dtype == RG_BF16 && out_dtype == RG_BF16 && v8)
    launch_seg<uint16_t, uint16_t, 8>(op, st, g, sc);
  else if (src_dtype == RG_BF16 && out_dtype == RG_BF16)
    launch_seg<uint16_t, uint16_t, 4>(op, st, g, sc);
  else if (src_dtype == RG_F32 && out_dtype == RG_BF16)
    launch_seg<float, uint16_t, 4>(op, st, g, sc);
  else if (src_dtype == RG_F16 && out_dtype == RG_F32 && v8)
    launch_seg<_Float16, float, 8>(op, st, g, sc);
  else if (src_dtype == RG_F16 && out_dtype == RG_F32)
    launch_seg<_Float16, float, 4>(op, st, g, sc);
  else if (src_dtype == RG_F16 && out_dtype == RG_F16 && v8)
    launch_seg<_Float16, _Float16, 8>(op, st, g, sc);
  else if (src_dtype == RG_F16 && out_dtype == RG_F16)
    launch_seg<_Float16, _Float16, 4>(op, st, g, sc);
  else if (src_dtype == RG_F32 && out_dtype == RG_F16)
    launch_seg<float, _Float16, 4>(op, st, g, sc);
  else
    RG_REQUIRE(false, RG_ERR_ARG, "rg_segment_reduce: bad dtypes");
  RG_LAUNCH_CHECK();
  return RG_OK;
}

}  // namespace rg

using namespace rg;

// (segments per lane group, rows in flight per lane) measured on C5's radius CSR (one 20 000-
// node frame, 20 rows per segment on average, 63 at most) and on M's kNN CSR (192 000
// segments of ~13 rows), scripts/seg_few.py: (1, 8) beat (2, 8) on both -- more waves, and a
// wave waits for its longest segment either way; with the longest-first order 12 rows in
// flight and 8-B lanes (C5 sorted: bf16 0.56 -> 0.67 of HBM)
static Sched default_sched(bool ordered) { return Sched{1, ordered ? 12 : 8}; }

static bool check_shape(int C, int ld_src, int ld_out) {
  return C > 0 && C <= 256 && C % 4 == 0 && ld_src % 4 == 0 && ld_out % 4 == 0;
}

// bf16 rows: 16-B loads (8 channels per lane) when C, the strides and the pointers allow
static bool vec8(int C, int ld_src, int out_dtype, int ld_out, const void* src, const void* out) {
  return C % 8 == 0 && ld_src % 8 == 0 && (out_dtype == RG_F32 || ld_out % 8 == 0) &&
         (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0;
}

extern "C" int rg_segment_reduce(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                                 const int* idx, int n_seg, int C, int op, void* out,
                                 int out_dtype, int ld_out, void* stream) {
  RG_REQUIRE(op >= RG_REDUCE_SUM && op <= RG_REDUCE_MAX, RG_ERR_ARG, "bad reduce op %d", op);
  RG_REQUIRE(check_shape(C, ld_src, ld_out), RG_ERR_UNSUPPORTED,
             "rg_segment_reduce: C=%d ld_src=%d ld_out=%d must be multiples of 4", C, ld_src,
             ld_out);
  if (n_seg <= 0) return RG_OK;
  const SegArgs g = {src, ld_src, seg_ptr, nullptr, nullptr, idx, 0, 0, nullptr, 0, n_seg, C, out, ld_out};
  return launch_any(op, src_dtype, out_dtype, vec8(C, ld_src, out_dtype, ld_out, src, out),
                    (hipStream_t)stream, g, default_sched(false));
}

extern "C" int rg_segment_reduce_sched(const void* src, int src_dtype, int ld_src,
                                       const int* seg_ptr, const int* order, int n_seg, int C,
                                       int op, void* out, int out_dtype, int ld_out, int groups,
                                       int rows_in_flight, int narrow_lanes, void* stream) {
  RG_REQUIRE(op >= RG_REDUCE_SUM && op <= RG_REDUCE_MAX, RG_ERR_ARG, "bad reduce op %d", op);
  RG_REQUIRE(check_shape(C, ld_src, ld_out), RG_ERR_UNSUPPORTED,
             "rg_segment_reduce_sched: C=%d ld_src=%d ld_out=%d must be multiples of 4", C, ld_src,
             ld_out);
  const Sched sc{groups, rows_in_flight};
  RG_REQUIRE(sched_compiled(sc) && (!order || groups == 1), RG_ERR_UNSUPPORTED,
             "rg_segment_reduce_sched: (groups %d, rows %d%s) is not a compiled schedule", groups,
             rows_in_flight, order ? ", ordered" : "");
  if (n_seg <= 0) return RG_OK;
  const SegArgs g = {src, ld_src, seg_ptr, order, nullptr, nullptr, 0, 0, nullptr, 0, n_seg, C,
                     out, ld_out};
  return launch_any(op, src_dtype, out_dtype,
                    !narrow_lanes && vec8(C, ld_src, out_dtype, ld_out, src, out),
                    (hipStream_t)stream, g, sc);
}

static int bm_ld(int C) { return (C + 7) / 8 * 8; }

extern "C" size_t rg_segment_reduce_ranges_workspace_size(long n_rows, int C, int src_dtype) {
  const size_t es = (src_dtype == RG_BF16 || src_dtype == RG_F16) ? 2 : 4;
  return ((size_t)(n_rows + RANGE_BLOCK - 1) / RANGE_BLOCK) * bm_ld(C) * es + 256;
}

extern "C" int rg_segment_reduce_ranges(const void* src, int src_dtype, int ld_src, long n_rows,
                                        const int* seg_begin, const int* seg_end, int n_seg, int C,
                                        int op, void* out, int out_dtype, int ld_out,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  RG_REQUIRE(seg_begin && seg_end, RG_ERR_ARG, "rg_segment_reduce_ranges: begin / end missing");
  RG_REQUIRE(op >= RG_REDUCE_SUM && op <= RG_REDUCE_MAX, RG_ERR_ARG, "bad reduce op %d", op);
  RG_REQUIRE(check_shape(C, ld_src, ld_out), RG_ERR_UNSUPPORTED,
             "rg_segment_reduce_ranges: C=%d ld_src=%d ld_out=%d must be multiples of 4", C,
             ld_src, ld_out);
  if (n_seg <= 0) return RG_OK;
  hipStream_t st = (hipStream_t)stream;
  const void* bm = nullptr;
  const int ldb = bm_ld(C);
  if (op == RG_REDUCE_MAX && workspace && n_rows >= 2 * RANGE_BLOCK &&
      workspace_bytes >= rg_segment_reduce_ranges_workspace_size(n_rows, C, src_dtype)) {
    // pass 1: 32-row block maxima of src, in src's dtype (exact)
    void* w = (void*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    const int nb = (int)((n_rows + RANGE_BLOCK - 1) / RANGE_BLOCK);
    const SegArgs g1 = {src, ld_src, nullptr, nullptr, nullptr, nullptr, RANGE_BLOCK, (int)n_rows,
                        nullptr, 0, nb, C, w, ldb};
    const int rc = launch_any(op, src_dtype, src_dtype,
                              vec8(C, ld_src, src_dtype, ldb, src, w), st, g1, default_sched(false));
    if (rc) return rc;
    bm = w;
  }
  const SegArgs g = {src, ld_src, seg_begin, nullptr, seg_end, nullptr, 0, 0, bm, ldb, n_seg, C,
                     out, ld_out};
  return launch_any(op, src_dtype, out_dtype, vec8(C, ld_src, out_dtype, ld_out, src, out) &&
                                                  (!bm || ldb % 8 == 0),
                    st, g, default_sched(false));
}

// ---- longest-first segment order (rg_segment_order): a counting sort of the segments by
//      length, descending, lengths capped at ORD_BINS - 1, in ONE workgroup (the order is
//      used for graphs of a few ten thousand segments, where one launch beats three plus a
//      memset): per-wave LDS histograms (contention only inside a wave), the cursors of bin b
//      = the segments in longer bins + those of bin b in lower waves, then each wave places
//      its segments at its cursors.  The order inside a bin depends on timing; no result
//      does (every segment's reduction is independent of the schedule).
namespace rg {
static constexpr int ORD_BINS = 256;
static constexpr int ORD_T = 1024;
static constexpr int ORD_W = ORD_T / 64;

__device__ __forceinline__ int ord_bin(const int* seg_ptr, int s) {
  return min(seg_ptr[s + 1] - seg_ptr[s], ORD_BINS - 1);
}

__global__ __launch_bounds__(ORD_T) void seg_order_kernel(const int* __restrict__ seg_ptr,
                                                          int n_seg, int* __restrict__ order) {
  __shared__ int cnt[ORD_W][ORD_BINS];  // per-wave counts, then per-wave cursors
  __shared__ int tot[ORD_BINS];
  const int t = threadIdx.x, w = t >> 6;
  for (int i = t; i < ORD_W * ORD_BINS; i += ORD_T) (&cnt[0][0])[i] = 0;
  __syncthreads();
  for (int s = t; s < n_seg; s += ORD_T) atomicAdd(&cnt[w][ord_bin(seg_ptr, s)], 1);
  __syncthreads();
  if (t < ORD_BINS) {  // thread t: bin ORD_BINS - 1 - t (longest first)
    const int bn = ORD_BINS - 1 - t;
    int run = 0;
    for (int v = 0; v < ORD_W; ++v) {
      const int c = cnt[v][bn];
      cnt[v][bn] = run;  // offset of wave v inside the bin
      run += c;
    }
    tot[t] = run;
  }
  __syncthreads();
  // inclusive scan of tot over the descending bins (Hillis-Steele, 8 steps)
  for (int o = 1; o < ORD_BINS; o <<= 1) {
    const int v = t < ORD_BINS && t >= o ? tot[t - o] : 0;
    __syncthreads();
    if (t < ORD_BINS) tot[t] += v;
    __syncthreads();
  }
  if (t < ORD_BINS) {
    const int bn = ORD_BINS - 1 - t;
    const int base = t > 0 ? tot[t - 1] : 0;
    for (int v = 0; v < ORD_W; ++v) cnt[v][bn] += base;
  }
  __syncthreads();
  for (int s = t; s < n_seg; s += ORD_T) order[atomicAdd(&cnt[w][ord_bin(seg_ptr, s)], 1)] = s;
}
}  // namespace rg

extern "C" size_t rg_segment_order_workspace_size(void) { return 0; }

extern "C" int rg_segment_order(const int* seg_ptr, int n_seg, int* order, void* workspace,
                                size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  if (n_seg <= 0) return RG_OK;
  seg_order_kernel<<<1, ORD_T, 0, (hipStream_t)stream>>>(seg_ptr, n_seg, order);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// graphs with more segments than this keep the plain order in rg_segment_reduce_ordered:
// M's 192 000 kNN segments (lengths 10..25, rows contiguous in node order) measured
// 0.73 -> 0.61-0.66 of HBM in bf16 with the longest-first order (the groups' rows then lie
// scattered), C5's 20 000 radius segments (20 rows on average, 63 at most) 0.55 -> 0.65
#ifndef RG_SEG_ORDER_MAX
#define RG_SEG_ORDER_MAX 65536
#endif

extern "C" int rg_segment_reduce_ordered(const void* src, int src_dtype, int ld_src,
                                         const int* seg_ptr, const int* order, int n_seg, int C,
                                         int op, void* out, int out_dtype, int ld_out,
                                         void* stream) {
  RG_REQUIRE(op >= RG_REDUCE_SUM && op <= RG_REDUCE_MAX, RG_ERR_ARG, "bad reduce op %d", op);
  RG_REQUIRE(check_shape(C, ld_src, ld_out) && C % 64 == 0, RG_ERR_UNSUPPORTED,
             "rg_segment_reduce_ordered: C=%d must be a multiple of 64, ld_src=%d ld_out=%d of 4",
             C, ld_src, ld_out);
  RG_REQUIRE(order, RG_ERR_ARG, "rg_segment_reduce_ordered: order missing");
  if (n_seg <= 0) return RG_OK;
  const bool use = n_seg <= RG_SEG_ORDER_MAX;
  const SegArgs g = {src, ld_src, seg_ptr, use ? order : nullptr, nullptr, nullptr, 0, 0, nullptr,
                     0, n_seg, C, out, ld_out};
  // with the order, 16-bit rows as 8-B lane loads (16 lanes per 64 channels: twice the lane
  // groups; C5 bf16 0.57 -> 0.65)
  const bool v8 = !use && vec8(C, ld_src, out_dtype, ld_out, src, out);
  return launch_any(op, src_dtype, out_dtype, v8, (hipStream_t)stream, g, default_sched(use));
}
