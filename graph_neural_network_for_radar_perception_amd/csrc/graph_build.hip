// Batched radar-frame graph build on gfx950.
//
// Replaces modules/compute_features/graph_features.py:11-164 (reference v2):
// the dense O(N^2) numpy distance matrix, np.argsort kNN, ball query and
// np.where edge list become
//   1. knn_scan   : one thread per node row, frame points streamed through LDS,
//                   exact fp32 distances (no FMA), top-(k+1) by (distance, index)
//                   kept sorted in registers, ball-query count, optional radius bits;
//   2. knn_mark   : kNN pairs set in a per-row bitset both ways (atomicOr);
//   3. row_count  : one wave per row, popcount of the bitset row;
//   4. exclusive scan -> CSR row_ptr;
//   5. row_emit   : one wave per row, ascending set bits -> CSR columns.
// The bitset IS the reference's N x N bool adjacency, at 1 bit per entry.
#include "rg_common.h"
#include "scan.h"

// exact numpy distances: no FMA contraction anywhere in this file
#pragma clang fp contract(off)

#include <stdarg.h>

namespace rg {

static char g_err[1024];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

static constexpr int KNN_BLOCK = 256;
static constexpr int KNN_CHUNK = 2048;  // points per LDS stage (16 KiB)

// fp32 squared distance exactly as numpy evaluates graph_features.py:72-73:
// two products and one sum, each rounded, no fused multiply-add.
__device__ __forceinline__ float sqdist(float xi, float yi, float xj, float yj) {
  float dx = (xi - xj);
  float dy = (yi - yj);
  return ((dx * dx) + (dy * dy));
}

// K = list length kept per row (>= k+1).  Ties: a later (larger) j never
// displaces an equal distance, i.e. "equal distance -> lower index first".
template <int K>
__global__ __launch_bounds__(KNN_BLOCK) void knn_scan(
    const float* __restrict__ px, const float* __restrict__ py, const int* __restrict__ frame_ptr,
    int kk, float eps2, int mode, int* __restrict__ knn_idx, int* __restrict__ knn_cnt,
    int* __restrict__ ball_deg, uint32_t* __restrict__ bits, int W) {
  __shared__ float2 pts[KNN_CHUNK];
  const int f = blockIdx.y;
  const int base = frame_ptr[f];
  const int nf = frame_ptr[f + 1] - base;
  if ((int)(blockIdx.x * KNN_BLOCK) >= nf) return;  // block-uniform exit
  const int il = blockIdx.x * KNN_BLOCK + threadIdx.x;
  const bool active = il < nf;
  const float xi = active ? px[base + il] : 0.f;
  const float yi = active ? py[base + il] : 0.f;
  const bool want_knn = mode != RG_GRAPH_RADIUS;
  const bool want_rad = mode != RG_GRAPH_KNN;

  float bd[K];
  int bi[K];
#pragma unroll
  for (int s = 0; s < K; ++s) {
    bd[s] = __int_as_float(0x7f800000);  // +inf
    bi[s] = -1;
  }
  int ball = 0;
  uint32_t* rowbits = bits + (size_t)(base + il) * W;

  for (int c0 = 0; c0 < nf; c0 += KNN_CHUNK) {
    const int cn = min(KNN_CHUNK, nf - c0);
    __syncthreads();
    for (int t = threadIdx.x; t < cn; t += KNN_BLOCK)
      pts[t] = make_float2(px[base + c0 + t], py[base + c0 + t]);
    __syncthreads();
    if (!active) continue;
    for (int t0 = 0; t0 < cn; t0 += 32) {
      uint32_t word = 0;
      const int tn = min(32, cn - t0);
      for (int u = 0; u < tn; ++u) {
        const float2 p = pts[t0 + u];
        const int j = c0 + t0 + u;
        const float d = sqdist(xi, yi, p.x, p.y);
        const bool inball = (d <= eps2) && (j != il);
        ball += inball ? 1 : 0;
        word |= (inball ? 1u : 0u) << u;
        if (want_knn && d < bd[K - 1]) {
          // sorted insert, stable w.r.t. j (strict compares)
#pragma unroll
          for (int s = K - 1; s > 0; --s) {
            const bool shift = d < bd[s - 1];
            const bool here = !shift && d < bd[s];
            bd[s] = shift ? bd[s - 1] : (here ? d : bd[s]);
            bi[s] = shift ? bi[s - 1] : (here ? j : bi[s]);
          }
          if (d < bd[0]) {
            bd[0] = d;
            bi[0] = j;
          }
        }
      }
      if (want_rad) rowbits[(c0 + t0) >> 5] = word;
    }
  }
  if (!active) return;
  ball_deg[base + il] = ball;
  if (want_knn) {
    const int cnt = min(kk, nf);
    knn_cnt[base + il] = cnt;
    int* out = knn_idx + (size_t)(base + il) * K;
#pragma unroll
    for (int s = 0; s < K; ++s)
      if (s < cnt) out[s] = bi[s];
  }
}

// frame base of each global row (needed to translate frame-local <-> global ids)
__global__ void row_frame_base(const int* __restrict__ frame_ptr, int n_frames,
                               int* __restrict__ row_base, int n_nodes) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  int lo = 0, hi = n_frames;  // frame_ptr[lo] <= i < frame_ptr[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (frame_ptr[mid] <= i) lo = mid; else hi = mid;
  }
  row_base[i] = frame_ptr[lo];
}

// set bits (i, j) and (j, i) for every kNN pair with j != i (graph_features.py:38-43)
__global__ void knn_mark(const int* __restrict__ row_base, const int* __restrict__ knn_idx,
                          const int* __restrict__ knn_cnt, int K, int n_nodes,
                          uint32_t* __restrict__ bits, int W) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(t / K);
  const int s = (int)(t % K);
  if (i >= n_nodes) return;
  if (s >= knn_cnt[i]) return;
  const int b = row_base[i];
  const int il = i - b;
  const int jl = knn_idx[(size_t)i * K + s];
  if (jl == il || jl < 0) return;
  atomicOr(bits + (size_t)i * W + (jl >> 5), 1u << (jl & 31));
  atomicOr(bits + (size_t)(b + jl) * W + (il >> 5), 1u << (il & 31));
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// one wave per row: number of set bits in the row's valid columns
__global__ __launch_bounds__(256) void row_count(const int* __restrict__ row_base,
                                                 const int* __restrict__ frame_ptr_unused,
                                                 const uint32_t* __restrict__ bits, int W,
                                                 int n_nodes, int* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_nodes) return;
  const uint32_t* rb = bits + (size_t)row * W;
  int c = 0;
  for (int w = lane; w < W; w += 64) c += __popc(rb[w]);
  c = wave_sum(c);
  if (lane == 0) cnt[row] = c;
}

// one wave per row: emit ascending set columns as global node ids
__global__ __launch_bounds__(256) void row_emit(const int* __restrict__ row_base,
                                                const uint32_t* __restrict__ bits, int W,
                                                int n_nodes, const int* __restrict__ row_ptr,
                                                int* __restrict__ col, long cap) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_nodes) return;
  const uint32_t* rb = bits + (size_t)row * W;
  const int b = row_base[row];
  long pos = row_ptr[row];
  if ((long)row_ptr[row + 1] > cap) return;  // overflow: caller sees n_edges > capacity
  for (int w0 = 0; w0 < W; w0 += 64) {
    const int w = w0 + lane;
    uint32_t word = w < W ? rb[w] : 0u;
    int c = __popc(word);
    int inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      int t = __shfl_up(inc, d, 64);
      if (lane >= d) inc += t;
    }
    long p = pos + inc - c;
    while (word) {
      int bit = __ffs(word) - 1;
      word &= word - 1;
      col[p++] = b + w * 32 + bit;
    }
    pos += __shfl(inc, 63, 64);
  }
}

}  // namespace rg

using namespace rg;

extern "C" const char* rg_last_error(void) { return g_err; }
extern "C" int rg_version(void) { return 1; }

static int knn_list_len(int kk) {
  static const int Ks[] = {2, 4, 8, 11, 16, 17, 24, 32, 33, 48, 64};
  for (int K : Ks)
    if (K >= kk) return K;
  return -1;
}

struct GraphWs {
  uint32_t* bits;
  int* knn_idx;
  int* knn_cnt;
  int* row_base;
  int* cnt;
  void* scan_ws;
};

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

static size_t graph_ws_layout(int n_nodes, int max_frame_nodes, int k, int mode, GraphWs* ws,
                              char* base) {
  const int W = (max_frame_nodes + 31) / 32;
  const int K = mode == RG_GRAPH_RADIUS ? 1 : knn_list_len(k + 1);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += align_up(bytes);
    return p;
  };
  char* p_bits = take((size_t)n_nodes * W * sizeof(uint32_t));
  char* p_idx = take((size_t)n_nodes * (K > 0 ? K : 1) * sizeof(int));
  char* p_cnt = take((size_t)n_nodes * sizeof(int));
  char* p_rb = take((size_t)n_nodes * sizeof(int));
  char* p_c2 = take((size_t)n_nodes * sizeof(int));
  char* p_sc = take(scan_workspace_bytes(n_nodes));
  if (ws) {
    ws->bits = (uint32_t*)p_bits;
    ws->knn_idx = (int*)p_idx;
    ws->knn_cnt = (int*)p_cnt;
    ws->row_base = (int*)p_rb;
    ws->cnt = (int*)p_c2;
    ws->scan_ws = p_sc;
  }
  return off;
}

extern "C" size_t rg_build_graph_workspace_size(int n_nodes, int n_frames, int max_frame_nodes,
                                                int k, int mode) {
  (void)n_frames;
  return graph_ws_layout(n_nodes, max_frame_nodes, k, mode, nullptr, nullptr);
}

template <int K>
static void launch_knn(dim3 grid, hipStream_t st, const float* px, const float* py,
                       const int* frame_ptr, int kk, float eps2, int mode, GraphWs& ws,
                       int* ball_degree, int W) {
  knn_scan<K><<<grid, KNN_BLOCK, 0, st>>>(px, py, frame_ptr, kk, eps2, mode, ws.knn_idx,
                                          ws.knn_cnt, ball_degree, ws.bits, W);
}

extern "C" int rg_build_graph(const float* px, const float* py, const int* frame_ptr, int n_nodes,
                              int n_frames, int max_frame_nodes, int k, float eps2, int mode,
                              int* row_ptr, int* col, long col_capacity, int* ball_degree,
                              int* n_edges_out, void* workspace, size_t workspace_bytes,
                              void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_nodes >= 0 && n_frames >= 1 && max_frame_nodes >= 0, RG_ERR_ARG,
             "rg_build_graph: bad sizes n_nodes=%d n_frames=%d", n_nodes, n_frames);
  RG_REQUIRE(mode >= 0 && mode <= 2, RG_ERR_ARG, "rg_build_graph: bad mode %d", mode);
  RG_REQUIRE(k >= 0, RG_ERR_ARG, "rg_build_graph: k must be >= 0");
  const int kk = k + 1;
  const int K = mode == RG_GRAPH_RADIUS ? 1 : knn_list_len(kk);
  RG_REQUIRE(K > 0, RG_ERR_UNSUPPORTED, "rg_build_graph: k=%d > 63 unsupported", k);
  GraphWs ws;
  size_t need = graph_ws_layout(n_nodes, max_frame_nodes, k, mode, &ws, (char*)workspace);
  RG_REQUIRE(workspace_bytes >= need, RG_ERR_ARG,
             "rg_build_graph: workspace %zu < required %zu", workspace_bytes, need);
  if (n_nodes == 0) {
    RG_CHECK_HIP(hipMemsetAsync(row_ptr, 0, sizeof(int), st));
    RG_CHECK_HIP(hipMemsetAsync(n_edges_out, 0, sizeof(int), st));
    return RG_OK;
  }
  const int W = (max_frame_nodes + 31) / 32;
  RG_CHECK_HIP(hipMemsetAsync(ws.bits, 0, (size_t)n_nodes * W * sizeof(uint32_t), st));
  row_frame_base<<<ceil_div(n_nodes, 256), 256, 0, st>>>(frame_ptr, n_frames, ws.row_base,
                                                         n_nodes);
  dim3 grid(ceil_div(max_frame_nodes, KNN_BLOCK), n_frames);
  switch (K) {
    case 1: launch_knn<1>(grid, st, px, py, frame_ptr, 1, eps2, mode, ws, ball_degree, W); break;
    case 2: launch_knn<2>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 4: launch_knn<4>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 8: launch_knn<8>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 11: launch_knn<11>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 16: launch_knn<16>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 17: launch_knn<17>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 24: launch_knn<24>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 32: launch_knn<32>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 33: launch_knn<33>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 48: launch_knn<48>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    case 64: launch_knn<64>(grid, st, px, py, frame_ptr, kk, eps2, mode, ws, ball_degree, W); break;
    default: RG_REQUIRE(false, RG_ERR_UNSUPPORTED, "knn list %d", K);
  }
  RG_LAUNCH_CHECK();
  if (mode != RG_GRAPH_RADIUS) {
    long tot = (long)n_nodes * K;
    knn_mark<<<ceil_div(tot, 256), 256, 0, st>>>(ws.row_base, ws.knn_idx, ws.knn_cnt, K, n_nodes,
                                                  ws.bits, W);
    RG_LAUNCH_CHECK();
  }
  row_count<<<ceil_div(n_nodes, 4), 256, 0, st>>>(ws.row_base, frame_ptr, ws.bits, W, n_nodes,
                                                  ws.cnt);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(ws.cnt, n_nodes, row_ptr, n_edges_out, ws.scan_ws, st);
  if (rc) return rc;
  row_emit<<<ceil_div(n_nodes, 4), 256, 0, st>>>(ws.row_base, ws.bits, W, n_nodes, row_ptr, col,
                                                 col_capacity);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
