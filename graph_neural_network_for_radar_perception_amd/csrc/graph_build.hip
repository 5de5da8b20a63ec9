// Batched radar-frame graph build on gfx950.
//
// Replaces modules/compute_features/graph_features.py:11-164 (reference v2):
// the dense O(N^2) numpy distance matrix, np.argsort kNN, ball query and
// np.where edge list become
//   0. grid_setup / grid_count / scan / grid_scatter: per frame, points bucketed
//                   into a uniform grid of ~3-point cells (cell-ordered copy);
//   1. knn_select : one thread per point, Chebyshev ring search over the cells,
//                   exact fp32 distances (no FMA), counting selection of the top-(k+1)
//                   (distance, index) keys through a per-row LDS histogram, ball-query
//                   count, optional radius bits, stopping once no unvisited cell can
//                   change the result (knn_grid: exact sorted-insert variant for rows
//                   with massive distance ties);
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

#include <mutex>
#include <set>
#include <tuple>

namespace rg {

// per host thread: two threads driving two GPUs never see each other's message
static thread_local char g_err[1024];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

hipError_t ensure_max_lds(const void* kernel, int bytes) {
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({kernel, dev, bytes})) return hipSuccess;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert({kernel, dev, bytes});
  return e;
}

static constexpr int KNN_BLOCK = 256;


// fp32 squared distance exactly as numpy evaluates graph_features.py:72-73:
// two products and one sum, each rounded, no fused multiply-add.
__device__ __forceinline__ float sqdist(float xi, float yi, float xj, float yj) {
  float dx = (xi - xj);
  float dy = (yi - yj);
  return ((dx * dx) + (dy * dy));
}

// ---------------------------------------------------------------------------------
// Uniform-grid neighbour search.  The reference ranks a row against the WHOLE frame
// (N x N distance matrix + argsort, graph_features.py:25-44); the result -- the k+1
// smallest (distance, index) keys, the ball-query count and the radius set -- only
// depends on points near the row, so each frame's points are bucketed into square
// cells of side s (~3 points per cell) and a row visits cells in Chebyshev rings
// r = 0, 1, 2, ... around its own cell.  Every point in a cell beyond ring r is at
// least (r - 0.01) s away (0.01 covers the f32 rounding of the cell coordinates), so
// once the current (k+1)-th key and eps2 are below that bound squared (minus a 1e-5
// relative margin for the f32 distance rounding) no unvisited point can enter the
// result: the selection equals the full scan's, ties included (keys compare as (d, j)).
// ---------------------------------------------------------------------------------
struct FrameGrid {
  float xmin, ymin, inv_s, s;
  int gw, gh, cell0, n;
};

// the build's first kernel: row frames (row_frame_base's work) and every zero the build
// needs -- redo flags, cell counts, both scatter cursors -- in one launch instead of a
// memset / copy each (each cost a ~10 us stream gap)
__global__ void build_init(const int* __restrict__ frame_ptr, int n_frames,
                           int* __restrict__ row_base, int* __restrict__ row_frame, int n_nodes,
                           int* __restrict__ redo, long n_cells, int* __restrict__ cell_cnt,
                           int* __restrict__ cursor, int* __restrict__ cursor_t) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_cells) {
    cell_cnt[i] = 0;
    cursor[i] = 0;
    cursor_t[i] = 0;
  }
  if (i >= n_nodes) return;
  int lo = 0, hi = n_frames;  // frame_ptr[lo] <= i < frame_ptr[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (frame_ptr[mid] <= i) lo = mid; else hi = mid;
  }
  row_base[i] = frame_ptr[lo];
  row_frame[i] = lo;
  redo[i] = 0;
}

// frame id and frame base of every global row (disjoint-union batch)
__global__ void row_frame_base(const int* __restrict__ frame_ptr, int n_frames,
                               int* __restrict__ row_base, int* __restrict__ row_frame,
                               int n_nodes) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  int lo = 0, hi = n_frames;  // frame_ptr[lo] <= i < frame_ptr[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (frame_ptr[mid] <= i) lo = mid; else hi = mid;
  }
  row_base[i] = frame_ptr[lo];
  row_frame[i] = lo;
}

// one block per frame: bounding box -> cell size and grid shape (<= cpf cells)
static constexpr int GS_T = 1024;  // a 20 000-point frame is 20 loads per thread
__global__ __launch_bounds__(GS_T) void grid_setup(const float* __restrict__ px,
                                                   const float* __restrict__ py,
                                                   const int* __restrict__ frame_ptr, int cpf,
                                                   FrameGrid* __restrict__ fg) {
  __shared__ float r[4][GS_T];
  const int f = blockIdx.x;
  const int b = frame_ptr[f], e = frame_ptr[f + 1];
  float x0 = __int_as_float(0x7f800000), y0 = x0, x1 = -x0, y1 = -x0;
  for (int i = b + threadIdx.x; i < e; i += GS_T) {
    const float x = px[i], y = py[i];
    x0 = fminf(x0, x); x1 = fmaxf(x1, x);
    y0 = fminf(y0, y); y1 = fmaxf(y1, y);
  }
  r[0][threadIdx.x] = x0; r[1][threadIdx.x] = x1;
  r[2][threadIdx.x] = y0; r[3][threadIdx.x] = y1;
  __syncthreads();
  for (int st = GS_T / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
      const int o = threadIdx.x + st;
      r[0][threadIdx.x] = fminf(r[0][threadIdx.x], r[0][o]);
      r[1][threadIdx.x] = fmaxf(r[1][threadIdx.x], r[1][o]);
      r[2][threadIdx.x] = fminf(r[2][threadIdx.x], r[2][o]);
      r[3][threadIdx.x] = fmaxf(r[3][threadIdx.x], r[3][o]);
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const int n = e - b;
  FrameGrid g;
  g.cell0 = f * cpf;
  g.n = n;
  g.xmin = n > 0 ? r[0][0] : 0.f;
  g.ymin = n > 0 ? r[2][0] : 0.f;
  const float w = n > 0 ? r[1][0] - r[0][0] : 0.f;
  const float h = n > 0 ? r[3][0] - r[2][0] : 0.f;
  const float ext = fmaxf(w, h);
  int gw = 1, gh = 1;
  float s = 1.f;
  if (ext > 0.f && ext < 1.0e30f && n > 3) {  // finite extent: ~3 points per cell
    const int target = min(max(n / 3, 1), cpf);
    const float wm = fmaxf(w, ext * 1e-3f), hm = fmaxf(h, ext * 1e-3f);
    s = sqrtf(wm * hm / (float)target);
    for (;;) {
      gw = (int)(w / s) + 1;
      gh = (int)(h / s) + 1;
      if ((long)gw * gh <= cpf) break;
      s *= 1.25f;
    }
  }
  g.s = s;
  g.inv_s = 1.f / s;
  g.gw = gw;
  g.gh = gh;
  fg[f] = g;
}

__device__ __forceinline__ int cell_coord(float v, float v0, float inv_s, int gdim) {
  const int c = (int)((v - v0) * inv_s);
  return c < 0 ? 0 : (c >= gdim ? gdim - 1 : c);
}

__global__ void grid_count(const float* __restrict__ px, const float* __restrict__ py,
                           const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
                           int n_nodes, int* __restrict__ cell_of, int* __restrict__ cell_cnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  const FrameGrid g = fg[row_frame[i]];
  const int cx = cell_coord(px[i], g.xmin, g.inv_s, g.gw);
  const int cy = cell_coord(py[i], g.ymin, g.inv_s, g.gh);
  const int c = g.cell0 + cy * g.gw + cx;
  cell_of[i] = c;
  atomicAdd(cell_cnt + c, 1);
}

// points regrouped by cell: {x, y, frame-local index, cell}.  The order inside a cell
// depends on atomic arrival and does not matter: every consumer compares full keys.
__global__ void grid_scatter(const float* __restrict__ px, const float* __restrict__ py,
                             const int* __restrict__ row_base, const int* __restrict__ cell_of,
                             int n_nodes, int* __restrict__ cursor, float4* __restrict__ pts,
                             const int* __restrict__ base = nullptr) {
  // position = base[c] + arrival (cursor zeroed), or cursor pre-set to the cell starts
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  const int c = cell_of[i];
  const int pos = (base ? base[c] : 0) + atomicAdd(cursor + c, 1);
  pts[pos] = make_float4(px[i], py[i], __int_as_float(i - row_base[i]), __int_as_float(c));
}

__device__ __forceinline__ bool key_less(float d, int j, float bd, int bj) {
  return d < bd || (d == bd && j < bj);
}

// Visit the points of the cells at Chebyshev distance exactly r from (cx, cy): grid
// rows cy-r and cy+r in full, then columns cx-r and cx+r strictly between them.
template <typename F>
__device__ __forceinline__ void for_ring(const FrameGrid& g, const int* __restrict__ cell_start,
                                         const float4* __restrict__ pts, int cx, int cy, int r,
                                         F&& body) {
  for (int side = 0; side < 4; ++side) {
    int ya, yb, xa, xb;
    if (side < 2) {
      const int yy = side == 0 ? cy - r : cy + r;
      if (yy < 0 || yy >= g.gh || (side == 1 && r == 0)) continue;
      ya = yb = yy;
      xa = max(cx - r, 0);
      xb = min(cx + r, g.gw - 1);
    } else {
      if (r == 0) continue;
      const int xx = side == 2 ? cx - r : cx + r;
      if (xx < 0 || xx >= g.gw) continue;
      xa = xb = xx;
      ya = max(cy - r + 1, 0);
      yb = min(cy + r - 1, g.gh - 1);
    }
    for (int yy = ya; yy <= yb; ++yy) {
      // cells xa..xb of one grid row are contiguous in the cell order
      const int c = g.cell0 + yy * g.gw;
      const int p0 = cell_start[c + xa], p1 = cell_start[c + xb + 1];
      // four candidate loads in flight per lane before any is consumed
      for (int p = p0; p < p1; p += 4) {
        float4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = pts[min(p + u, p1 - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (p + u < p1) body(q[u]);
      }
    }
  }
}

// lower bound (squared, f32-safe) on the distance of every point beyond ring r
__device__ __forceinline__ float ring_bound(const FrameGrid& g, int r) {
  const float lb = fmaxf((float)r - 0.01f, 0.f) * g.s;
  return lb * lb * (1.f - 1e-5f);
}

// Exact sorted-insert search: one thread per point in cell order (a wave = spatially
// adjacent rows, so the cells it visits are shared through L1), K = list length kept
// per row (>= kk = k + 1).  Used for the rows knn_select flags (massive exact ties).
template <int K>
__global__ __launch_bounds__(KNN_BLOCK) void knn_grid(
    const float4* __restrict__ pts, const int* __restrict__ cell_start,
    const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
    const int* __restrict__ frame_ptr, int n_nodes, int kk, float eps2, int mode,
    int* __restrict__ knn_idx, int* __restrict__ knn_cnt, int* __restrict__ ball_deg,
    uint32_t* __restrict__ bits, int W, const int* __restrict__ only, int2* __restrict__ kth) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_nodes) return;
  if (only && !only[t]) return;  // fallback pass: just the rows knn_select flagged
  const int f = row_frame[t];  // the cell-ordered points of frame f fill its row range
  const FrameGrid g = fg[f];
  const int base = frame_ptr[f];
  const float4 me = pts[t];
  const float xi = me.x, yi = me.y;
  const int il = __float_as_int(me.z);
  const int cme = __float_as_int(me.w) - g.cell0;
  const int cx = cme % g.gw, cy = cme / g.gw;
  const bool want_knn = mode != RG_GRAPH_RADIUS;
  const bool want_rad = mode != RG_GRAPH_KNN;
  uint32_t* rowbits = bits + (size_t)(base + il) * W;

  float bd[K];
  int bi[K];
#pragma unroll
  for (int q = 0; q < K; ++q) {
    bd[q] = __int_as_float(0x7f800000);  // +inf
    bi[q] = 0x7fffffff;
  }
  int ball = 0;
  const int rmax = max(max(cx, g.gw - 1 - cx), max(cy, g.gh - 1 - cy));
  bool knn_done = !want_knn, ball_done = false;
  for (int r = 0; r <= rmax && !(knn_done && ball_done); ++r) {
    for_ring(g, cell_start, pts, cx, cy, r, [&](const float4& q) {
      const int j = __float_as_int(q.z);
      const float d = sqdist(xi, yi, q.x, q.y);
      const bool inball = (d <= eps2) && (j != il);
      ball += inball ? 1 : 0;
      if (want_rad && inball) atomicOr(rowbits + (j >> 5), 1u << (j & 31));
      if (want_knn && key_less(d, j, bd[K - 1], bi[K - 1])) {
        // sorted insert by (d, j): branch-free pass from the tail
#pragma unroll
        for (int s2 = K - 1; s2 > 0; --s2) {
          const bool shift = key_less(d, j, bd[s2 - 1], bi[s2 - 1]);
          const bool here = !shift && key_less(d, j, bd[s2], bi[s2]);
          bd[s2] = shift ? bd[s2 - 1] : (here ? d : bd[s2]);
          bi[s2] = shift ? bi[s2 - 1] : (here ? j : bi[s2]);
        }
        if (key_less(d, j, bd[0], bi[0])) {
          bd[0] = d;
          bi[0] = j;
        }
      }
    });
    const float bound = ring_bound(g, r);
    if (eps2 < bound) ball_done = true;
    if (!knn_done) {
      float dk = bd[0];  // the kk-th key so far (+inf while fewer are held)
#pragma unroll
      for (int q = 1; q < K; ++q) dk = q == kk - 1 ? bd[q] : dk;
      if (dk < bound) knn_done = true;
    }
  }
  const int row = base + il;
  ball_deg[row] = ball;
  if (want_knn) {
    const int cnt = min(kk, g.n);
    knn_cnt[row] = cnt;
    float kd = bd[0];
    int kj = bi[0];
#pragma unroll
    for (int q = 1; q < K; ++q)
      if (q == cnt - 1) { kd = bd[q]; kj = bi[q]; }
    kth[row] = cnt < kk ? make_int2(0x7f800000, 0x7fffffff) : make_int2(__float_as_int(kd), kj);
    int* out = knn_idx + (size_t)row * K;
#pragma unroll
    for (int q = 0; q < K; ++q)
      if (q < cnt) {
        out[q] = bi[q];
        if (bi[q] != il) atomicOr(rowbits + (bi[q] >> 5), 1u << (bi[q] & 31));
      }
  }
}

static constexpr int HB = 64;     // distance histogram bins per row (4 per octave of d)
static constexpr int HSHIFT = 21; // d's bits >> 21 = exponent + 2 mantissa bits
static constexpr int HW = HB / 2; // LDS words per row: two 16-bit bin counters per word
static constexpr int BBUF = HW;   // boundary-bin candidates a row may buffer (indices)

// Counting selection of the k+1 nearest (distance, index) keys -- the same set the
// sorted-insert search (knn_grid) and the reference's argsort pick:
//   pass 1: rings are visited until the (k+1)-th key is provably inside; each candidate
//           only bumps a per-row LDS histogram of its squared distance (bins are the
//           exponent + 2 mantissa bits of d, monotone in d), so the bin b* holding the
//           (k+1)-th key and the count below it follow from a prefix over 64 counters;
//   pass 2: the same rings again: keys in bins < b* are selected outright, keys in b*
//           go to a per-row LDS buffer (indices) from which the missing few are picked
//           exactly, ordered by (d, j) with d recomputed bit-identically.
// Per candidate that is ~10 instructions instead of a k-long register insert, which
// under SIMT divergence ran for almost every candidate of the wave.  A row whose
// boundary bin holds more than BBUF keys (massive exact ties: duplicates, lattices)
// is flagged and redone by knn_grid.  Ball-query degree and radius bits are produced
// here for every row.
// Ring visit for the selection, over TWO cell-ordered copies of the frame: the grid
// rows cy - r and cy + r are contiguous position ranges of the row-major copy, the
// columns cx - r and cx + r (strictly between them) contiguous ranges of the
// column-major copy, so ring r is at most four ranges whose eight bounds are loaded
// together -- one dependent round trip per ring instead of one per cell of the two
// columns (a ring-r column side is 2r - 1 cells of ~3 points each).
template <typename F>
__device__ __forceinline__ void for_ring_rc(const FrameGrid& g, const int* __restrict__ cs_r,
                                            const float4* __restrict__ pts_r,
                                            const int* __restrict__ cs_c,
                                            const float4* __restrict__ pts_c, int cx, int cy,
                                            int r, F&& body) {
  const int xa = max(cx - r, 0), xb = min(cx + r, g.gw - 1);
  const int ya = max(cy - r + 1, 0), yb = min(cy + r - 1, g.gh - 1);
  const bool s0 = cy - r >= 0;
  const bool s1 = r > 0 && cy + r < g.gh;
  const bool s2 = r > 0 && cx - r >= 0 && ya <= yb;
  const bool s3 = r > 0 && cx + r < g.gw && ya <= yb;
  const int c0 = g.cell0 + (cy - r) * g.gw, c1 = g.cell0 + (cy + r) * g.gw;
  const int c2 = g.cell0 + (cx - r) * g.gh, c3 = g.cell0 + (cx + r) * g.gh;
  int b[4], e[4];
  b[0] = s0 ? cs_r[c0 + xa] : 0; e[0] = s0 ? cs_r[c0 + xb + 1] : 0;
  b[1] = s1 ? cs_r[c1 + xa] : 0; e[1] = s1 ? cs_r[c1 + xb + 1] : 0;
  b[2] = s2 ? cs_c[c2 + ya] : 0; e[2] = s2 ? cs_c[c2 + yb + 1] : 0;
  b[3] = s3 ? cs_c[c3 + ya] : 0; e[3] = s3 ? cs_c[c3 + yb + 1] : 0;
#pragma unroll
  for (int side = 0; side < 4; ++side) {
    const float4* __restrict__ pts = side < 2 ? pts_r : pts_c;
    const int p0 = b[side], p1 = e[side];
    for (int p = p0; p < p1; p += 4) {
      float4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = pts[min(p + u, p1 - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (p + u < p1) body(q[u]);
    }
  }
}

// One row of the counting selection (see below); H = the row's LDS histogram column
// (stride 64 words), redo_flag = where to flag the row for knn_grid.
template <typename RING>
__device__ __forceinline__ void knn_select_row(
    uint32_t* H, const FrameGrid& g, RING&& ring, const float* __restrict__ fx,
    const float* __restrict__ fy, float xi, float yi, int il, int cx, int cy, int row, int kk,
    int K, float eps2, int mode, int* __restrict__ knn_idx, int* __restrict__ knn_cnt,
    int* __restrict__ ball_deg, uint32_t* __restrict__ rowbits, int* redo_flag,
    int2* __restrict__ kth) {
  const bool want_knn = mode != RG_GRAPH_RADIUS;
  const bool want_rad = mode != RG_GRAPH_KNN;
  // bins: d's exponent + 2 mantissa bits, 16 octaves centred on the cell area s^2
  const int bin0 = (int)(__float_as_uint(g.s * g.s) >> HSHIFT) - HB / 2;
  auto bin_of = [&](float d) {
    const int b = (int)(__float_as_uint(d) >> HSHIFT) - bin0;
    return b < 0 ? 0 : (b >= HB ? HB - 1 : b);
  };
  if (want_knn) {
#pragma unroll
    for (int b = 0; b < HW; ++b) H[b * 64] = 0u;
  }
  const int rmax = max(max(cx, g.gw - 1 - cx), max(cy, g.gh - 1 - cy));
  int ball = 0, total = 0, r_knn = rmax;
  bool knn_done = !want_knn, ball_done = false;
  for (int r = 0; r <= rmax && !(knn_done && ball_done); ++r) {
    const bool count_knn = !knn_done;
    ring(r, [&](const float4& q) {
      const int j = __float_as_int(q.z);
      const float d = sqdist(xi, yi, q.x, q.y);
      if (!ball_done) {
        const bool inball = (d <= eps2) && (j != il);
        ball += inball ? 1 : 0;
        if (want_rad && inball) atomicOr(rowbits + (j >> 5), 1u << (j & 31));
      }
      if (count_knn) {
        const int bb = bin_of(d);
        atomicAdd(H + (bb >> 1) * 64, 1u << ((bb & 1) << 4));  // ds_add_u32: the row owns the column
        ++total;
      }
    });
    const float bound = ring_bound(g, r);
    if (eps2 < bound) ball_done = true;
    if (count_knn && total >= kk) {
      // upper edge of the bin holding the kk-th key bounds the kk-th distance
      int cum = 0, bs = HB - 1;
      for (int b = 0; b < HB; ++b) {
        cum += (int)((H[(b >> 1) * 64] >> ((b & 1) << 4)) & 0xffffu);
        if (cum >= kk) { bs = b; break; }
      }
      const int ub_bits = bin0 + bs + 1;
      const float ub = bs == HB - 1 ? __int_as_float(0x7f800000)
                                    : (ub_bits <= 0 ? 0.f : __uint_as_float((uint32_t)ub_bits << HSHIFT));
      if (ub <= bound) {
        knn_done = true;
        r_knn = r;
      }
    }
  }
  ball_deg[row] = ball;
  if (!want_knn) return;
  // ---- selection: bins below b* entirely, the rest of the kk from bin b* exactly
  int bs = HB, below = total, in_bs = 0;  // total <= kk: every visited key is selected
  if (total > kk) {
    int cum = 0;
    for (int b = 0; b < HB; ++b) {
      const int c = (int)((H[(b >> 1) * 64] >> ((b & 1) << 4)) & 0xffffu);
      if (cum + c >= kk) { bs = b; below = cum; in_bs = c; break; }
      cum += c;
    }
  }
  const int cnt = min(kk, total);
  // A boundary bin with more than BBUF keys is refined in place: the same rings again,
  // histogramming the next 6 bits of d's pattern among the keys of the boundary prefix
  // (d >= 0, so its bit pattern is monotone), until the boundary prefix holds <= BBUF
  // keys.  Only exact ties beyond BBUF (every bit equal: duplicates, lattices) or a
  // boundary in a clamped edge bin still go to the sorted-insert pass (knn_grid), which
  // runs one thread per row and would otherwise cost a whole wave per flagged row.
  int sh = -1;         // refined: the boundary keys are those with (bits >> sh) == pref
  uint32_t pref = 0;
  if (in_bs > BBUF && bs > 0 && bs < HB - 1) {
    sh = HSHIFT;
    pref = (uint32_t)(bin0 + bs);
    while (in_bs > BBUF && sh > 0) {
      const int nsh = sh > 6 ? sh - 6 : 0;
      const uint32_t msk = (1u << (sh - nsh)) - 1u;
#pragma unroll
      for (int b = 0; b < HW; ++b) H[b * 64] = 0u;
      for (int r = 0; r <= r_knn; ++r) {
        ring(r, [&](const float4& q) {
          const uint32_t bits = __float_as_uint(sqdist(xi, yi, q.x, q.y));
          if ((bits >> sh) == pref) {
            const uint32_t sub = (bits >> nsh) & msk;
            atomicAdd(H + (sub >> 1) * 64, 1u << ((sub & 1) << 4));
          }
        });
      }
      int cum = 0, sb = (int)msk;
      for (int b = 0; b <= (int)msk; ++b) {
        const int c = (int)((H[(b >> 1) * 64] >> ((b & 1) << 4)) & 0xffffu);
        if (below + cum + c >= kk) { sb = b; in_bs = c; break; }
        cum += c;
      }
      below += cum;
      pref = (pref << (sh - nsh)) | (uint32_t)sb;
      sh = nsh;
    }
  }
  const int need = cnt - below;
  if (in_bs > BBUF) {  // exact ties beyond the buffer: exact insert path
    *redo_flag = 1;
    return;
  }
  // key class: 0 selected outright, 1 boundary (buffered), 2 beyond
  auto key_class = [&](float d) {
    if (sh < 0) {
      const int b = bin_of(d);
      return b < bs ? 0 : (b == bs ? 1 : 2);
    }
    const uint32_t p = __float_as_uint(d) >> sh;
    return p < pref ? 0 : (p == pref ? 1 : 2);
  };
  uint32_t* Bj = H;  // boundary-key indices reuse the histogram column: [e][lane], e < BBUF
  int* out = knn_idx + (size_t)row * K;
  int n_out = 0, nb = 0;
  float md = -1.f;  // largest key selected outright (the kk-th key when need == 0)
  int mj = -1;
  for (int r = 0; r <= r_knn; ++r) {
    ring(r, [&](const float4& q) {
      const int j = __float_as_int(q.z);
      const float d = sqdist(xi, yi, q.x, q.y);
      const int kc = key_class(d);
      if (kc == 0) {
        if (key_less(md, mj, d, j)) { md = d; mj = j; }
        out[n_out++] = j;
        if (j != il) atomicOr(rowbits + (j >> 5), 1u << (j & 31));  // fire-and-forget
      } else if (kc == 1) {
        Bj[nb * 64] = (uint32_t)j;
        ++nb;
      }
    });
  }
  // the need smallest (d, j) of the boundary keys (d recomputed bit-identically)
  int last_j = -1;
  float last_d = -1.f;
  for (int q = 0; q < need; ++q) {
    float bd = __int_as_float(0x7f800000);
    int bj = 0x7fffffff;
    for (int e = 0; e < nb; ++e) {
      const int j = (int)Bj[e * 64];
      const float d = sqdist(xi, yi, fx[j], fy[j]);
      // next key strictly after the previous pick
      if (key_less(last_d, last_j, d, j) && key_less(d, j, bd, bj)) { bd = d; bj = j; }
    }
    out[n_out++] = bj;
    if (bj != il) atomicOr(rowbits + (bj >> 5), 1u << (bj & 31));
    last_d = bd;
    last_j = bj;
  }
  knn_cnt[row] = cnt;
  // the kk-th key (+inf when the frame has fewer than kk points: every point is in)
  if (cnt < kk) kth[row] = make_int2(0x7f800000, 0x7fffffff);
  else kth[row] = need > 0 ? make_int2(__float_as_int(last_d), last_j)
                           : make_int2(__float_as_int(md), mj);
}

// one thread per cell-ordered point (row-major copy: a wave is a patch of neighbours)
__global__ __launch_bounds__(KNN_BLOCK) void knn_select(
    const float4* __restrict__ pts, const int* __restrict__ cell_start,
    const float4* __restrict__ pts_t, const int* __restrict__ cell_start_t,
    const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
    const int* __restrict__ frame_ptr, const float* __restrict__ px,
    const float* __restrict__ py, int n_nodes, int kk, int K, float eps2, int mode,
    int* __restrict__ knn_idx, int* __restrict__ knn_cnt, int* __restrict__ ball_deg,
    uint32_t* __restrict__ bits, int W, int* __restrict__ redo, int2* __restrict__ kth) {
  // per wave: [bin pair][lane], 16-bit counters (a row has < 65536 candidates per bin:
  // frames are far smaller); 8 KiB per wave lets 4-5 blocks share a CU
  __shared__ uint32_t lds[KNN_BLOCK / 64][HW * 64];
  const int lane = threadIdx.x & 63;
  uint32_t* H = lds[threadIdx.x >> 6] + lane;  // this row's column (stride 64 words)
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_nodes) return;  // no block barriers below: rows own disjoint LDS columns
  const int f = row_frame[t];  // the cell-ordered points of frame f fill its row range
  const FrameGrid g = fg[f];
  const int base = frame_ptr[f];
  const float4 me = pts[t];
  const int il = __float_as_int(me.z);
  const int cme = __float_as_int(me.w) - g.cell0;
  const int cx = cme % g.gw, cy = cme / g.gw;
  const int row = base + il;
  knn_select_row(H, g,
                 [&](int r, auto&& body) {
                   for_ring_rc(g, cell_start, pts, cell_start_t, pts_t, cx, cy, r, body);
                 },
                 px + base, py + base, me.x, me.y, il, cx, cy, row, kk, K, eps2, mode, knn_idx,
                 knn_cnt, ball_deg, bits + (size_t)row * W, redo + t, kth);
}

// ---------------------------------------------------------------------------------
// Cooperative counting selection (pure kNN mode): a group of CL lanes per row instead
// of one thread per row.  The ring ranges of for_ring_rc are flattened into one index
// space and the group's lanes load CL consecutive candidates at a time (four loads in
// flight per lane), so a ring costs ceil(T / 4CL) dependent round trips instead of
// ~T/4 per thread, and a wave's lanes no longer idle on the longest row's ring walk.
// Same two passes and the same keys as knn_select_row: pass 1 histograms the candidate
// distances in the row's LDS counters (shared by the group, ds_add), pass 2 selects the
// keys below the boundary bin (ballot-compacted) and buffers the boundary keys
// (distance bits + index) in LDS, from which the missing `need` are taken by rank.
// The selected SET, the kk-th key, the ball count and the redo flag equal knn_select's;
// only the order inside a row's knn_idx list differs (no consumer depends on it).
// ---------------------------------------------------------------------------------
#ifndef RG_KNN_COOP
#define RG_KNN_COOP 1  // pure kNN mode: the cooperative selection (0: one thread per row)
#endif
#ifndef RG_KNN_CL
#define RG_KNN_CL 16
#endif
static constexpr int CL = RG_KNN_CL;             // lanes per row
static constexpr int CO_ROWS = KNN_BLOCK / CL;   // rows per workgroup
static constexpr int CO_BUF = 32;                // boundary keys a row may buffer
#ifndef RG_KNN_CAP
#define RG_KNN_CAP 128
#endif
static constexpr int CO_CAP = RG_KNN_CAP;        // pass-1 keys cached per row for pass 2

__device__ __forceinline__ void grp_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS traffic landed
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ int grp_sum(int v) {
#pragma unroll
  for (int d = 1; d < CL; d <<= 1) v += __shfl_xor(v, d, CL);
  return v;
}
__device__ __forceinline__ int grp_incl_scan(int v, int sl) {
#pragma unroll
  for (int d = 1; d < CL; d <<= 1) {
    const int t = __shfl_up(v, d, CL);
    if (sl >= d) v += t;
  }
  return v;
}

// first bin b (of 64 16-bit counters in 32 words H[0..31]) with cum(0..b) >= target;
// returns b (63 if never reached), the count below it and its own count
struct BinPick { int bs, below, in_bs; };
__device__ __forceinline__ BinPick grp_find_bin(const uint32_t* H, int sl, int target) {
  constexpr int WPL = HW / CL;  // words (two 16-bit bins each) per lane
  int c[2 * WPL];
  int cl = 0;
#pragma unroll
  for (int w = 0; w < WPL; ++w) {
    const uint32_t v = H[WPL * sl + w];
    c[2 * w] = (int)(v & 0xffffu);
    c[2 * w + 1] = (int)(v >> 16);
    cl += c[2 * w] + c[2 * w + 1];
  }
  const int excl = grp_incl_scan(cl, sl) - cl;
  const bool mine = excl < target && target <= excl + cl;
  int bl = 0, cb = 0, own = 0, pre = excl;
  bool found = false;
#pragma unroll
  for (int q = 0; q < 2 * WPL; ++q) {
    if (!found && pre + c[q] >= target) { found = true; bl = q; cb = pre; own = c[q]; }
    pre += c[q];
  }
  const uint64_t gm = ((1ull << CL) - 1ull) << (__lane_id() & ~(CL - 1));
  const uint64_t m = __ballot(mine) & gm;
  BinPick p{HB - 1, 0, 0};  // not reached (cannot happen for target <= the counted keys)
  if (m == 0ull) return p;
  const int src = (__ffsll((unsigned long long)m) - 1) & (CL - 1);
  p.bs = __shfl(2 * WPL * sl + bl, src, CL);
  p.below = __shfl(cb, src, CL);
  p.in_bs = __shfl(own, src, CL);
  return p;
}

// ring r of for_ring_rc, flattened: the group's lanes take candidates sl, sl + CL, ...
// body(q, ok, o) runs on every lane of the group (ok = the lane holds a real candidate,
// o = its index in the ring), so ballots inside it see the whole group; returns the
// ring's candidate count
template <typename F>
__device__ __forceinline__ int ring_coop(const FrameGrid& g, const int* __restrict__ cs_r,
                                         const float4* __restrict__ pts_r,
                                         const int* __restrict__ cs_c,
                                         const float4* __restrict__ pts_c, int cx, int cy, int r,
                                         int sl, F&& body) {
  const int xa = max(cx - r, 0), xb = min(cx + r, g.gw - 1);
  const int ya = max(cy - r + 1, 0), yb = min(cy + r - 1, g.gh - 1);
  const bool s0 = cy - r >= 0;
  const bool s1 = r > 0 && cy + r < g.gh;
  const bool s2 = r > 0 && cx - r >= 0 && ya <= yb;
  const bool s3 = r > 0 && cx + r < g.gw && ya <= yb;
  const int c0 = g.cell0 + (cy - r) * g.gw, c1 = g.cell0 + (cy + r) * g.gw;
  const int c2 = g.cell0 + (cx - r) * g.gh, c3 = g.cell0 + (cx + r) * g.gh;
  const int b0 = s0 ? cs_r[c0 + xa] : 0, e0 = s0 ? cs_r[c0 + xb + 1] : 0;
  const int b1 = s1 ? cs_r[c1 + xa] : 0, e1 = s1 ? cs_r[c1 + xb + 1] : 0;
  const int b2 = s2 ? cs_c[c2 + ya] : 0, e2 = s2 ? cs_c[c2 + yb + 1] : 0;
  const int b3 = s3 ? cs_c[c3 + ya] : 0, e3 = s3 ? cs_c[c3 + yb + 1] : 0;
  const int n0 = e0 - b0, n01 = n0 + (e1 - b1), n012 = n01 + (e2 - b2), T = n012 + (e3 - b3);
  for (int o0 = 0; o0 < T; o0 += 4 * CL) {
    float4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = min(o0 + sl + CL * u, T - 1);
      const bool rm = o < n01;  // row-major copy (sides 0, 1) or column-major (2, 3)
      const int p = o < n0 ? b0 + o : (o < n01 ? b1 + (o - n0) : (o < n012 ? b2 + (o - n01) : b3 + (o - n012)));
      q[u] = rm ? pts_r[p] : pts_c[p];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body(q[u], o0 + sl + CL * u < T, o0 + sl + CL * u);
  }
  return T;
}

__global__ __launch_bounds__(KNN_BLOCK) void knn_select_coop(
    const float4* __restrict__ pts, const int* __restrict__ cell_start,
    const float4* __restrict__ pts_t, const int* __restrict__ cell_start_t,
    const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
    const int* __restrict__ frame_ptr, int n_nodes, int kk, int K, float eps2,
    int* __restrict__ knn_idx, int* __restrict__ knn_cnt, int* __restrict__ ball_deg,
    uint32_t* __restrict__ bits, int W, int* __restrict__ redo, int2* __restrict__ kth) {
  __shared__ uint32_t hist_s[CO_ROWS][HW];
  __shared__ uint32_t bufd_s[CO_ROWS][CO_BUF];
  __shared__ int bufj_s[CO_ROWS][CO_BUF];
  __shared__ uint2 cache_s[CO_ROWS][CO_CAP];  // (distance bits, index) of the counted keys
  const int sl = threadIdx.x & (CL - 1), grp = threadIdx.x / CL;
  const int lane = __lane_id();
  const uint64_t gm = ((1ull << CL) - 1ull) << (lane & ~(CL - 1));
  const uint64_t lt = (1ull << lane) - 1ull;
  const int t = blockIdx.x * CO_ROWS + grp;  // cell-ordered point (neighbouring rows share a wave)
  if (t >= n_nodes) return;                  // group-uniform; no block barriers below
  uint32_t* H = hist_s[grp];
  uint32_t* Bd = bufd_s[grp];
  int* Bj = bufj_s[grp];
  uint2* Ck = cache_s[grp];
  const int f = row_frame[t];
  const FrameGrid g = fg[f];
  const int base = frame_ptr[f];
  const float4 me = pts[t];
  const float xi = me.x, yi = me.y;
  const int il = __float_as_int(me.z);
  const int cme = __float_as_int(me.w) - g.cell0;
  const int cx = cme % g.gw, cy = cme / g.gw;
  const int row = base + il;
  uint32_t* rowbits = bits + (size_t)row * W;
  // this row's bitset words are zeroed here (no memset of the whole N x W bitset): only
  // this row's selection writes the row before knn_mark; the release fence orders the
  // zeros before every later atomicOr of the group
  for (int w = sl; w < W; w += CL) rowbits[w] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  auto ring = [&](int r, auto&& body) {
    return ring_coop(g, cell_start, pts, cell_start_t, pts_t, cx, cy, r, sl, body);
  };
  const int bin0 = (int)(__float_as_uint(g.s * g.s) >> HSHIFT) - HB / 2;
  auto bin_of = [&](float d) {
    const int b = (int)(__float_as_uint(d) >> HSHIFT) - bin0;
    return b < 0 ? 0 : (b >= HB ? HB - 1 : b);
  };
  for (int w = sl; w < HW; w += CL) H[w] = 0u;
  grp_sync();
  // ---- pass 1: histogram until the kk-th key is provably inside; ball count
  const int rmax = max(max(cx, g.gw - 1 - cx), max(cy, g.gh - 1 - cy));
  int ball = 0, total = 0, r_knn = rmax;
  bool knn_done = false, ball_done = false;
  for (int r = 0; r <= rmax && !(knn_done && ball_done); ++r) {
    const bool count_knn = !knn_done, count_ball = !ball_done;
    const int T = ring(r, [&](const float4& q, bool ok, int o) {
      if (!ok) return;
      const int j = __float_as_int(q.z);
      const float d = sqdist(xi, yi, q.x, q.y);
      if (count_ball) ball += ((d <= eps2) && (j != il)) ? 1 : 0;
      if (count_knn) {
        const int bb = bin_of(d);
        atomicAdd(H + (bb >> 1), 1u << ((bb & 1) << 4));
        if (total + o < CO_CAP) Ck[total + o] = make_uint2(__float_as_uint(d), (uint32_t)j);
      }
    });
    const float bound = ring_bound(g, r);
    if (eps2 < bound) ball_done = true;
    if (count_knn) {
      total += T;
      if (total >= kk) {
        grp_sync();
        const BinPick bp = grp_find_bin(H, sl, kk);
        const int ub_bits = bin0 + bp.bs + 1;
        const float ub = bp.bs == HB - 1 ? __int_as_float(0x7f800000)
                                         : (ub_bits <= 0 ? 0.f : __uint_as_float((uint32_t)ub_bits << HSHIFT));
        if (ub <= bound) {
          knn_done = true;
          r_knn = r;
        }
      }
    }
  }
  ball = grp_sum(ball);
  if (sl == 0) ball_deg[row] = ball;
  grp_sync();
  // ---- boundary bin (and in-place refinement of an over-full one, as knn_select_row)
  int bs = HB, below = total, in_bs = 0;
  if (total > kk) {
    const BinPick bp = grp_find_bin(H, sl, kk);
    bs = bp.bs; below = bp.below; in_bs = bp.in_bs;
  }
  const int cnt = min(kk, total);
  // the counted keys again: from the LDS cache when they all fit, else the same rings
  const bool cached = total <= CO_CAP;
  auto visit = [&](auto&& body) {
    if (cached) {
      for (int e0 = 0; e0 < total; e0 += CL) {
        const int e = e0 + sl;
        const uint2 kv = Ck[min(e, total - 1)];
        body(__uint_as_float(kv.x), (int)kv.y, e < total);
      }
    } else {
      for (int r = 0; r <= r_knn; ++r)
        ring(r, [&](const float4& q, bool ok, int) {
          body(sqdist(xi, yi, q.x, q.y), __float_as_int(q.z), ok);
        });
    }
  };
  int sh = -1;
  uint32_t pref = 0;
  if (in_bs > CO_BUF && bs > 0 && bs < HB - 1) {
    sh = HSHIFT;
    pref = (uint32_t)(bin0 + bs);
    while (in_bs > CO_BUF && sh > 0) {
      const int nsh = sh > 6 ? sh - 6 : 0;
      const uint32_t msk = (1u << (sh - nsh)) - 1u;
      grp_sync();
      for (int w = sl; w < HW; w += CL) H[w] = 0u;
      grp_sync();
      visit([&](float d, int, bool ok) {
        const uint32_t bits = __float_as_uint(d);
        if (ok && (bits >> sh) == pref) {
          const uint32_t sub = (bits >> nsh) & msk;
          atomicAdd(H + (sub >> 1), 1u << ((sub & 1) << 4));
        }
      });
      grp_sync();
      const BinPick bp = grp_find_bin(H, sl, kk - below);
      below += bp.below;
      in_bs = bp.in_bs;
      pref = (pref << (sh - nsh)) | (uint32_t)bp.bs;
      sh = nsh;
    }
  }
  const int need = cnt - below;
  if (in_bs > CO_BUF) {  // exact ties beyond the buffer: the sorted-insert pass redoes the row
    if (sl == 0) redo[t] = 1;
    return;
  }
  auto key_class = [&](float d) {
    if (sh < 0) {
      const int b = bin_of(d);
      return b < bs ? 0 : (b == bs ? 1 : 2);
    }
    const uint32_t p = __float_as_uint(d) >> sh;
    return p < pref ? 0 : (p == pref ? 1 : 2);
  };
  // ---- pass 2: keys below the boundary selected outright, boundary keys buffered
  int* out = knn_idx + (size_t)row * K;
  int n_out = 0, nb = 0;
  float md = -1.f;  // largest key selected outright (this lane's share)
  int mj = -1;
  visit([&](float d, int j, bool ok) {
    const int kc = ok ? key_class(d) : 2;
    const uint64_t ms = __ballot(kc == 0) & gm;
    const uint64_t mb = __ballot(kc == 1) & gm;
    if (kc == 0) {
      if (key_less(md, mj, d, j)) { md = d; mj = j; }
      out[n_out + __popcll(ms & lt)] = j;
      if (j != il) atomicOr(rowbits + (j >> 5), 1u << (j & 31));
    } else if (kc == 1) {
      const int e = nb + __popcll(mb & lt);
      if (e < CO_BUF) { Bd[e] = __float_as_uint(d); Bj[e] = j; }
    }
    n_out += __popcll(ms);
    nb += __popcll(mb);
  });
  grp_sync();
  // ---- the need smallest (d, j) boundary keys, by rank (keys are distinct: j is)
  nb = min(nb, CO_BUF);
  for (int e = sl; e < nb; e += CL) {
    const float de = __uint_as_float(Bd[e]);
    const int je = Bj[e];
    int rank = 0;
    for (int e2 = 0; e2 < nb; ++e2) rank += key_less(__uint_as_float(Bd[e2]), Bj[e2], de, je) ? 1 : 0;
    if (rank < need) {
      out[n_out + rank] = je;
      if (je != il) atomicOr(rowbits + (je >> 5), 1u << (je & 31));
      if (rank == need - 1 && cnt >= kk) kth[row] = make_int2(__float_as_int(de), je);
    }
  }
  // the kk-th key when nothing came from the boundary: the largest key selected outright
#pragma unroll
  for (int dd = 1; dd < CL; dd <<= 1) {
    const float od = __shfl_xor(md, dd, CL);
    const int oj = __shfl_xor(mj, dd, CL);
    if (key_less(md, mj, od, oj)) { md = od; mj = oj; }
  }
  if (sl == 0) {
    knn_cnt[row] = cnt;
    if (cnt < kk) kth[row] = make_int2(0x7f800000, 0x7fffffff);
    else if (need <= 0) kth[row] = make_int2(__float_as_int(md), mj);
  }
}

// ---------------------------------------------------------------------------------
// Pure radius graph (compute_ball_query + np.where, graph_features.py:11-22, 79) without
// the N x N_f bitset: the ball relation is symmetric bit for bit (sqdist of (i, j) and
// (j, i) square the same magnitudes), so row i's columns are exactly the points j != i
// with d(i, j) <= eps^2, ascending.  A group of CL lanes per row walks the rings
// cooperatively (ring_coop) twice: radius_count_coop counts the row (= its ball degree),
// and after the scan radius_emit_coop gathers the row's columns in LDS (ballot-compacted)
// and writes each at its rank among them -- ascending, the np.where order.  A row with
// more than RAD_CAP columns instead sweeps the frame's index range in windows of
// 32 x RAD_CAP indices, each an LDS bitmask emitted in bit order.  (The bitset path wrote
// and scanned 4 x N x N_f / 32 bytes: 50 MB at C5's 20 000-point frame.)
// ---------------------------------------------------------------------------------
#ifndef RG_RADIUS_COOP
#define RG_RADIUS_COOP 1
#endif
static constexpr int RAD_CAP = 128;

template <typename F>
__device__ __forceinline__ void radius_walk(const FrameGrid& g, const int* __restrict__ cs_r,
                                            const float4* __restrict__ pts_r,
                                            const int* __restrict__ cs_c,
                                            const float4* __restrict__ pts_c, int cx, int cy,
                                            float xi, float yi, int il, float eps2, int sl,
                                            F&& in_ball) {
  const int rmax = max(max(cx, g.gw - 1 - cx), max(cy, g.gh - 1 - cy));
  for (int r = 0; r <= rmax; ++r) {
    ring_coop(g, cs_r, pts_r, cs_c, pts_c, cx, cy, r, sl, [&](const float4& q, bool ok, int) {
      const int j = __float_as_int(q.z);
      in_ball(j, ok && (sqdist(xi, yi, q.x, q.y) <= eps2) && (j != il));
    });
    if (eps2 < ring_bound(g, r)) break;
  }
}

__global__ __launch_bounds__(KNN_BLOCK) void radius_count_coop(
    const float4* __restrict__ pts, const int* __restrict__ cell_start,
    const float4* __restrict__ pts_t, const int* __restrict__ cell_start_t,
    const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
    const int* __restrict__ frame_ptr, int n_nodes, float eps2, int* __restrict__ ball_deg,
    int* __restrict__ cnt) {
  const int sl = threadIdx.x & (CL - 1), grp = threadIdx.x / CL;
  const int t = blockIdx.x * CO_ROWS + grp;
  if (t >= n_nodes) return;  // group-uniform
  const int f = row_frame[t];
  const FrameGrid g = fg[f];
  const float4 me = pts[t];
  const int il = __float_as_int(me.z);
  const int cme = __float_as_int(me.w) - g.cell0;
  int ball = 0;
  radius_walk(g, cell_start, pts, cell_start_t, pts_t, cme % g.gw, cme / g.gw, me.x, me.y, il,
              eps2, sl, [&](int, bool in) { ball += in ? 1 : 0; });
  ball = grp_sum(ball);
  if (sl == 0) {
    const int row = frame_ptr[f] + il;
    ball_deg[row] = ball;
    cnt[row] = ball;
  }
}

__global__ __launch_bounds__(KNN_BLOCK) void radius_emit_coop(
    const float4* __restrict__ pts, const int* __restrict__ cell_start,
    const float4* __restrict__ pts_t, const int* __restrict__ cell_start_t,
    const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
    const int* __restrict__ frame_ptr, int n_nodes, float eps2,
    const int* __restrict__ row_ptr, int* __restrict__ col, long cap) {
  __shared__ int buf_s[CO_ROWS][RAD_CAP];
  const int sl = threadIdx.x & (CL - 1), grp = threadIdx.x / CL;
  const int lane = __lane_id();
  const uint64_t gm = ((1ull << CL) - 1ull) << (lane & ~(CL - 1));
  const uint64_t lt = (1ull << lane) - 1ull;
  const int t = blockIdx.x * CO_ROWS + grp;
  if (t >= n_nodes) return;  // group-uniform
  const int f = row_frame[t];
  const FrameGrid g = fg[f];
  const int base = frame_ptr[f];
  const float4 me = pts[t];
  const int il = __float_as_int(me.z);
  const int cme = __float_as_int(me.w) - g.cell0;
  const int cx = cme % g.gw, cy = cme / g.gw;
  const int row = base + il;
  const long p0 = row_ptr[row], p1 = row_ptr[row + 1];
  if (p1 > cap) return;  // overflow: the caller sees n_edges > capacity (as row_emit)
  const int n = (int)(p1 - p0);
  int* B = buf_s[grp];
  if (n <= RAD_CAP) {
    int nb = 0;
    radius_walk(g, cell_start, pts, cell_start_t, pts_t, cx, cy, me.x, me.y, il, eps2, sl,
                [&](int j, bool in) {
                  const uint64_t m = __ballot(in) & gm;
                  if (in) B[nb + __popcll(m & lt)] = j;
                  nb += __popcll(m);
                });
    grp_sync();
    for (int e = sl; e < n; e += CL) {
      const int je = B[e];
      int rank = 0;
      for (int e2 = 0; e2 < n; ++e2) rank += B[e2] < je ? 1 : 0;
      col[p0 + rank] = base + je;
    }
    return;
  }
  // a long row: windows of 32 x RAD_CAP frame-local indices, one LDS bitmask each
  const int nf = frame_ptr[f + 1] - base;
  constexpr int WPL = RAD_CAP / CL;  // mask words per lane, contiguous
  uint32_t* M = (uint32_t*)B;
  long pos = p0;
  for (int w0 = 0; w0 < nf; w0 += 32 * RAD_CAP) {
    grp_sync();
    for (int w = sl; w < RAD_CAP; w += CL) M[w] = 0u;
    grp_sync();
    radius_walk(g, cell_start, pts, cell_start_t, pts_t, cx, cy, me.x, me.y, il, eps2, sl,
                [&](int j, bool in) {
                  const int o = j - w0;
                  if (in && o >= 0 && o < 32 * RAD_CAP) atomicOr(M + (o >> 5), 1u << (o & 31));
                });
    grp_sync();
    int c = 0;
#pragma unroll
    for (int w = 0; w < WPL; ++w) c += __popc(M[WPL * sl + w]);
    long p = pos + grp_incl_scan(c, sl) - c;
#pragma unroll
    for (int w = 0; w < WPL; ++w) {
      uint32_t word = M[WPL * sl + w];
      while (word) {
        const int bit = __ffs(word) - 1;
        word &= word - 1;
        col[p++] = base + w0 + 32 * (WPL * sl + w) + bit;
      }
    }
    pos += grp_sum(c);
  }
}

// column-major copy of the grid (for_ring_rc): transposed cell counts, then points
// scattered by transposed cell (cell index cell0 + cx * gh + cy)
__global__ void grid_transpose_counts(const FrameGrid* __restrict__ fg, int cpf, long n_cells,
                                      const int* __restrict__ cell_cnt,
                                      int* __restrict__ cell_cnt_t) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cells) return;
  const int f = (int)(c / cpf);
  const int cr = (int)(c - (long)f * cpf);
  const FrameGrid g = fg[f];
  if (cr < g.gw * g.gh) {
    const int cx = cr % g.gw, cy = cr / g.gw;
    cell_cnt_t[g.cell0 + cx * g.gh + cy] = cell_cnt[c];
  } else {
    cell_cnt_t[c] = 0;
  }
}

__global__ void grid_scatter_t(const float* __restrict__ px, const float* __restrict__ py,
                               const int* __restrict__ row_base, const int* __restrict__ row_frame,
                               const FrameGrid* __restrict__ fg, const int* __restrict__ cell_of,
                               int n_nodes, int* __restrict__ cursor,
                               float4* __restrict__ pts_t, const int* __restrict__ base) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  const FrameGrid g = fg[row_frame[i]];
  const int cr = cell_of[i] - g.cell0;
  const int ct = g.cell0 + (cr % g.gw) * g.gh + cr / g.gw;
  const int pos = base[ct] + atomicAdd(cursor + ct, 1);
  pts_t[pos] = make_float4(px[i], py[i], __int_as_float(i - row_base[i]), __int_as_float(ct));
}

// the transposed half of knn | knn^T (graph_features.py:38-43): bit (j, i) for every
// kNN pair (i, j); bit (i, j) was set by the row's own search.  Mutual neighbours are
// common and need no write: i is in row j's own kNN set iff key (d_ij, i) <= row j's
// kk-th key (the same (distance, index) order the selection used; d_ij recomputed
// bit-identically from the coordinates), so the test reads two small L2-resident
// arrays instead of a cache line of the bitset per pair, and only a missing bit costs
// an atomic.
// row j's position and kk-th key in one 16-B record, so knn_mark gathers one line per
// pair instead of three (px[j], py[j], kth[j])
__global__ void node_key_pack(const float* __restrict__ px, const float* __restrict__ py,
                              const int2* __restrict__ kth, int n, int4* __restrict__ nk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int2 k = kth[i];
    nk[i] = make_int4(__float_as_int(px[i]), __float_as_int(py[i]), k.x, k.y);
  }
}

__global__ void knn_mark(const int* __restrict__ row_base, const int* __restrict__ knn_idx,
                         const int* __restrict__ knn_cnt, const int4* __restrict__ nk, int K,
                         int n_nodes, uint32_t* __restrict__ bits, int W) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(t / K);
  const int s = (int)(t % K);
  if (i >= n_nodes) return;
  if (s >= knn_cnt[i]) return;
  const int b = row_base[i];
  const int il = i - b;
  const int jl = knn_idx[(size_t)i * K + s];
  if (jl == il || jl < 0) return;
  const int j = b + jl;
  const int4 rj = nk[j], ri = nk[i];
  const float d = sqdist(__int_as_float(rj.x), __int_as_float(rj.y), __int_as_float(ri.x),
                         __int_as_float(ri.y));
  if (!key_less(__int_as_float(rj.z), rj.w, d, il)) return;  // (d, il) <= row j's kk-th key
  atomicOr(bits + (size_t)j * W + (il >> 5), 1u << (il & 31));
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// 16 lanes per row (a row of a 3 000-point frame is 94 words: one wave per row left
// most lanes idle on the second pass): number of set bits in the row
__global__ __launch_bounds__(256) void row_count(const int* __restrict__ row_base,
                                                 const int* __restrict__ frame_ptr_unused,
                                                 const uint32_t* __restrict__ bits, int W,
                                                 int n_nodes, int* __restrict__ cnt) {
  const int sl = threadIdx.x & 15;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (row >= n_nodes) return;  // group-uniform
  const uint32_t* rb = bits + (size_t)row * W;
  int c = 0;
  for (int w = sl; w < W; w += 16) c += __popc(rb[w]);
#pragma unroll
  for (int d = 8; d > 0; d >>= 1) c += __shfl_xor(c, d, 16);
  if (sl == 0) cnt[row] = c;
}

// 16 lanes per row: emit ascending set columns as global node ids (each pass of 16
// words: popcounts, a 16-lane exclusive scan, every lane writes its word's columns)
__global__ __launch_bounds__(256) void row_emit(const int* __restrict__ row_base,
                                                const uint32_t* __restrict__ bits, int W,
                                                int n_nodes, const int* __restrict__ row_ptr,
                                                int* __restrict__ col, long cap) {
  const int sl = threadIdx.x & 15;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (row >= n_nodes) return;  // group-uniform
  const uint32_t* rb = bits + (size_t)row * W;
  const int b = row_base[row];
  long pos = row_ptr[row];
  if ((long)row_ptr[row + 1] > cap) return;  // overflow: caller sees n_edges > capacity
  for (int w0 = 0; w0 < W; w0 += 16) {
    const int w = w0 + sl;
    uint32_t word = w < W ? rb[w] : 0u;
    const int c = __popc(word);
    int inc = c;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const int t = __shfl_up(inc, d, 16);
      if (sl >= d) inc += t;
    }
    long p = pos + inc - c;
    while (word) {
      const int bit = __ffs(word) - 1;
      word &= word - 1;
      col[p++] = b + w * 32 + bit;
    }
    pos += __shfl(inc, 15, 16);
  }
}

// ---------------------------------------------------------------------------------
// Connected components for the proposal branch (Simple_DBSCAN, clustering.py:43-93:
// breadth-first components of the eps-graph on predicted centres, numbered by each
// component's lowest node index).  Lock-free union-find: a union hooks the LARGER root
// under the smaller one with atomicCAS, so a root only ever gains a smaller parent and
// every component's final root is its minimum node index -- the label is independent
// of thread timing.  parent[x] <= x holds throughout, so finds always terminate.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ int cc_find(volatile int* parent, int x) {
  for (;;) {
    const int p = parent[x];
    if (p == x) return x;
    const int gp = parent[p];
    if (gp == p) return p;
    parent[x] = gp;  // path halving: stores an ancestor, a benign race
    x = gp;
  }
}

__device__ __forceinline__ void cc_union(int* parent, int a, int b) {
  int ra = cc_find(parent, a), rb = cc_find(parent, b);
  while (ra != rb) {
    if (ra > rb) { const int t = ra; ra = rb; rb = t; }
    const int old = atomicCAS(parent + rb, rb, ra);
    if (old == rb) return;
    rb = cc_find(parent, old);
    ra = cc_find(parent, ra);
  }
}

__global__ void cc_init(int* __restrict__ parent, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) parent[i] = i;
}

// eps-graph edges (squared distance <= eps2, clustering.py:26-39) found by the same
// ring search as the ball query, one thread per point in cell order
__global__ __launch_bounds__(KNN_BLOCK) void cc_radius_hook(
    const float4* __restrict__ pts, const int* __restrict__ cell_start,
    const int* __restrict__ row_frame, const FrameGrid* __restrict__ fg,
    const int* __restrict__ frame_ptr, int n_nodes, float eps2, int* parent) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_nodes) return;
  const int f = row_frame[t];
  const FrameGrid g = fg[f];
  const int base = frame_ptr[f];
  const float4 me = pts[t];
  const int il = __float_as_int(me.z);
  const int cme = __float_as_int(me.w) - g.cell0;
  const int cx = cme % g.gw, cy = cme / g.gw;
  const int rmax = max(max(cx, g.gw - 1 - cx), max(cy, g.gh - 1 - cy));
  for (int r = 0; r <= rmax; ++r) {
    for_ring(g, cell_start, pts, cx, cy, r, [&](const float4& q) {
      const int j = __float_as_int(q.z);
      if (j > il && sqdist(me.x, me.y, q.x, q.y) <= eps2) cc_union(parent, base + il, base + j);
    });
    if (eps2 < ring_bound(g, r)) break;
  }
}

// predicted links (argmax of the 2-class logits == 1, gnn_detector.py:158-159) among the
// link pairs, dropped when sqrt(dx^2 + dy^2) >= eps (clustering.py:8-23)
__global__ void cc_pairs_hook(const float* __restrict__ px, const float* __restrict__ py,
                              const int* __restrict__ pair_src, const int* __restrict__ pair_dst,
                              const int* __restrict__ n_pairs_dev, long n_pairs,
                              const float* __restrict__ logits, int ld, float eps, int* parent) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long np_ = n_pairs_dev ? min((long)*n_pairs_dev, n_pairs) : n_pairs;
  if (p >= np_) return;
  if (!(logits[p * ld + 1] > logits[p * ld + 0])) return;
  const int a = pair_src[p], b = pair_dst[p];
  const float dx = px[a] - px[b], dy = py[a] - py[b];
  const float dist = sqrt_rn((dx * dx) + (dy * dy));
  if (dist >= eps) return;
  cc_union(parent, a, b);
}

__global__ void cc_compress(int* parent, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) parent[i] = cc_find(parent, i);
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
  int* row_frame;
  int* cnt;
  FrameGrid* fg;
  int* cell_cnt;
  int* cell_start;
  int* cursor;
  int* cell_of;
  float4* pts;
  int* redo;
  void* scan_ws;
  int2* kth;   // per row: the kk-th (distance bits, frame-local index) key of its kNN set
  int* cell_cnt_t;     // column-major copy of the grid (for_ring_rc)
  int* cell_start_t;
  float4* pts_t;
  int* cursor_t;       // arrival counters of the column-major scatter
  int4* nkey;          // per row: (x, y, kk-th key) for knn_mark
  int cpf;
  long n_cells;
};

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

// grid cells per frame: room for ~3 points per cell at the largest frame
static int cells_per_frame(int max_frame_nodes) { return max(16, max_frame_nodes / 2); }

static size_t graph_ws_layout(int n_nodes, int n_frames, int max_frame_nodes, int k, int mode,
                              GraphWs* ws, char* base) {
  const int W = (max_frame_nodes + 31) / 32;
  const int K = mode == RG_GRAPH_RADIUS ? 1 : knn_list_len(k + 1);
  const int cpf = cells_per_frame(max_frame_nodes);
  const long n_cells = (long)n_frames * cpf;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += align_up(bytes);
    return p;
  };
  // the pure radius graph builds its CSR without the bitset (radius_count / emit_coop)
  const bool no_bits = RG_RADIUS_COOP && mode == RG_GRAPH_RADIUS;
  char* p_bits = take(no_bits ? 0 : (size_t)n_nodes * W * sizeof(uint32_t));
  char* p_idx = take((size_t)n_nodes * (K > 0 ? K : 1) * sizeof(int));
  char* p_cnt = take((size_t)n_nodes * sizeof(int));
  char* p_rb = take((size_t)n_nodes * sizeof(int));
  char* p_rf = take((size_t)n_nodes * sizeof(int));
  char* p_c2 = take((size_t)n_nodes * sizeof(int));
  char* p_fg = take((size_t)n_frames * sizeof(FrameGrid));
  char* p_cc = take((size_t)n_cells * sizeof(int));
  char* p_cs = take((size_t)(n_cells + 1) * sizeof(int));
  char* p_cu = take((size_t)n_cells * sizeof(int));
  char* p_co = take((size_t)n_nodes * sizeof(int));
  char* p_pt = take((size_t)n_nodes * sizeof(float4));
  char* p_rd = take((size_t)n_nodes * sizeof(int));
  char* p_sc = take(scan_workspace_bytes(max((long)n_nodes, n_cells)));
  char* p_kt = take((size_t)n_nodes * sizeof(int2));
  char* p_ct = take((size_t)n_cells * sizeof(int));
  char* p_st = take((size_t)(n_cells + 1) * sizeof(int));
  char* p_pq = take((size_t)n_nodes * sizeof(float4));
  char* p_cv = take((size_t)n_cells * sizeof(int));
  char* p_nk = take((size_t)n_nodes * sizeof(int4));
  if (ws) {
    ws->nkey = (int4*)p_nk;
    ws->cursor_t = (int*)p_cv;
    ws->kth = (int2*)p_kt;
    ws->cell_cnt_t = (int*)p_ct;
    ws->cell_start_t = (int*)p_st;
    ws->pts_t = (float4*)p_pq;
    ws->bits = (uint32_t*)p_bits;
    ws->knn_idx = (int*)p_idx;
    ws->knn_cnt = (int*)p_cnt;
    ws->row_base = (int*)p_rb;
    ws->row_frame = (int*)p_rf;
    ws->cnt = (int*)p_c2;
    ws->fg = (FrameGrid*)p_fg;
    ws->cell_cnt = (int*)p_cc;
    ws->cell_start = (int*)p_cs;
    ws->cursor = (int*)p_cu;
    ws->cell_of = (int*)p_co;
    ws->pts = (float4*)p_pt;
    ws->redo = (int*)p_rd;
    ws->scan_ws = p_sc;
    ws->cpf = cpf;
    ws->n_cells = n_cells;
  }
  return off;
}

extern "C" size_t rg_build_graph_workspace_size(int n_nodes, int n_frames, int max_frame_nodes,
                                                int k, int mode) {
  return graph_ws_layout(n_nodes, n_frames, max_frame_nodes, k, mode, nullptr, nullptr);
}

// counting selection for every row, then the exact sorted-insert search for the rows
// it flagged (their outputs are rewritten identically)
template <int K>
static void launch_knn(hipStream_t st, const float* px, const float* py, const int* frame_ptr,
                       int n_nodes, int kk, float eps2, int mode, GraphWs& ws, int* ball_degree,
                       int W) {
  if (RG_KNN_COOP && mode == RG_GRAPH_KNN) {
    knn_select_coop<<<ceil_div(n_nodes, CO_ROWS), KNN_BLOCK, 0, st>>>(
        ws.pts, ws.cell_start, ws.pts_t, ws.cell_start_t, ws.row_frame, ws.fg, frame_ptr,
        n_nodes, kk, K, eps2, ws.knn_idx, ws.knn_cnt, ball_degree, ws.bits, W, ws.redo, ws.kth);
  } else {
    knn_select<<<ceil_div(n_nodes, KNN_BLOCK), KNN_BLOCK, 0, st>>>(
        ws.pts, ws.cell_start, ws.pts_t, ws.cell_start_t, ws.row_frame, ws.fg, frame_ptr, px, py,
        n_nodes, kk, K, eps2, mode, ws.knn_idx, ws.knn_cnt, ball_degree, ws.bits, W, ws.redo,
        ws.kth);
  }
  if (mode == RG_GRAPH_RADIUS) return;
  knn_grid<K><<<ceil_div(n_nodes, KNN_BLOCK), KNN_BLOCK, 0, st>>>(
      ws.pts, ws.cell_start, ws.row_frame, ws.fg, frame_ptr, n_nodes, kk, eps2, mode, ws.knn_idx,
      ws.knn_cnt, ball_degree, ws.bits, W, ws.redo, ws.kth);
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
  size_t need = graph_ws_layout(n_nodes, n_frames, max_frame_nodes, k, mode, &ws,
                                (char*)workspace);
  RG_REQUIRE(workspace_bytes >= need, RG_ERR_ARG,
             "rg_build_graph: workspace %zu < required %zu", workspace_bytes, need);
  if (n_nodes == 0) {
    RG_CHECK_HIP(hipMemsetAsync(row_ptr, 0, sizeof(int), st));
    RG_CHECK_HIP(hipMemsetAsync(n_edges_out, 0, sizeof(int), st));
    return RG_OK;
  }
  const int W = (max_frame_nodes + 31) / 32;
  const bool rad_coop = RG_RADIUS_COOP && mode == RG_GRAPH_RADIUS;
  // the cooperative selection zeroes its own bitset rows; the radius path has none
  if (!(RG_KNN_COOP && mode == RG_GRAPH_KNN) && !rad_coop)
    RG_CHECK_HIP(hipMemsetAsync(ws.bits, 0, (size_t)n_nodes * W * sizeof(uint32_t), st));
  build_init<<<ceil_div(max((long)n_nodes, ws.n_cells), 256), 256, 0, st>>>(
      frame_ptr, n_frames, ws.row_base, ws.row_frame, n_nodes, ws.redo, ws.n_cells, ws.cell_cnt,
      ws.cursor, ws.cursor_t);
  // bucket every frame's points into its grid (cell order = frame order, so the scan of
  // all cells gives absolute positions inside each frame's row range)
  grid_setup<<<n_frames, GS_T, 0, st>>>(px, py, frame_ptr, ws.cpf, ws.fg);
  grid_count<<<ceil_div(n_nodes, 256), 256, 0, st>>>(px, py, ws.row_frame, ws.fg, n_nodes,
                                                     ws.cell_of, ws.cell_cnt);
  RG_LAUNCH_CHECK();
  int rc0 = exclusive_scan(ws.cell_cnt, ws.n_cells, ws.cell_start, ws.cell_start + ws.n_cells,
                           ws.scan_ws, st);
  if (rc0) return rc0;
  grid_scatter<<<ceil_div(n_nodes, 256), 256, 0, st>>>(px, py, ws.row_base, ws.cell_of, n_nodes,
                                                       ws.cursor, ws.pts, ws.cell_start);
  RG_LAUNCH_CHECK();
  // the column-major copy of the same grid
  grid_transpose_counts<<<ceil_div(ws.n_cells, 256), 256, 0, st>>>(ws.fg, ws.cpf, ws.n_cells,
                                                                    ws.cell_cnt, ws.cell_cnt_t);
  RG_LAUNCH_CHECK();
  rc0 = exclusive_scan(ws.cell_cnt_t, ws.n_cells, ws.cell_start_t, ws.cell_start_t + ws.n_cells,
                       ws.scan_ws, st);
  if (rc0) return rc0;
  grid_scatter_t<<<ceil_div(n_nodes, 256), 256, 0, st>>>(px, py, ws.row_base, ws.row_frame, ws.fg,
                                                         ws.cell_of, n_nodes, ws.cursor_t, ws.pts_t,
                                                         ws.cell_start_t);
  RG_LAUNCH_CHECK();
  if (rad_coop) {
    radius_count_coop<<<ceil_div(n_nodes, CO_ROWS), KNN_BLOCK, 0, st>>>(
        ws.pts, ws.cell_start, ws.pts_t, ws.cell_start_t, ws.row_frame, ws.fg, frame_ptr, n_nodes,
        eps2, ball_degree, ws.cnt);
    RG_LAUNCH_CHECK();
    int rc = exclusive_scan(ws.cnt, n_nodes, row_ptr, n_edges_out, ws.scan_ws, st);
    if (rc) return rc;
    radius_emit_coop<<<ceil_div(n_nodes, CO_ROWS), KNN_BLOCK, 0, st>>>(
        ws.pts, ws.cell_start, ws.pts_t, ws.cell_start_t, ws.row_frame, ws.fg, frame_ptr, n_nodes,
        eps2, row_ptr, col, col_capacity);
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  switch (K) {
    case 1: launch_knn<1>(st, px, py, frame_ptr, n_nodes, 1, eps2, mode, ws, ball_degree, W); break;
    case 2: launch_knn<2>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 4: launch_knn<4>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 8: launch_knn<8>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 11: launch_knn<11>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 16: launch_knn<16>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 17: launch_knn<17>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 24: launch_knn<24>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 32: launch_knn<32>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 33: launch_knn<33>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 48: launch_knn<48>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    case 64: launch_knn<64>(st, px, py, frame_ptr, n_nodes, kk, eps2, mode, ws, ball_degree, W); break;
    default: RG_REQUIRE(false, RG_ERR_UNSUPPORTED, "knn list %d", K);
  }
  RG_LAUNCH_CHECK();
  if (mode != RG_GRAPH_RADIUS) {
    long tot = (long)n_nodes * K;
    node_key_pack<<<ceil_div(n_nodes, 256), 256, 0, st>>>(px, py, ws.kth, n_nodes, ws.nkey);
    knn_mark<<<ceil_div(tot, 256), 256, 0, st>>>(ws.row_base, ws.knn_idx, ws.knn_cnt, ws.nkey,
                                                  K, n_nodes, ws.bits, W);
    RG_LAUNCH_CHECK();
  }
  row_count<<<ceil_div(n_nodes, 16), 256, 0, st>>>(ws.row_base, frame_ptr, ws.bits, W, n_nodes,
                                                   ws.cnt);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(ws.cnt, n_nodes, row_ptr, n_edges_out, ws.scan_ws, st);
  if (rc) return rc;
  row_emit<<<ceil_div(n_nodes, 16), 256, 0, st>>>(ws.row_base, ws.bits, W, n_nodes, row_ptr, col,
                                                 col_capacity);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ------------------------------------------------------------- proposal clustering
struct GridWs {
  int* row_base;
  int* row_frame;
  FrameGrid* fg;
  int* cell_cnt;
  int* cell_start;
  int* cursor;
  int* cell_of;
  float4* pts;
  void* scan_ws;
  int cpf;
  long n_cells;
};

static size_t grid_ws_layout(int n_nodes, int n_frames, int max_frame_nodes, GridWs* ws,
                             char* base) {
  const int cpf = cells_per_frame(max_frame_nodes);
  const long n_cells = (long)n_frames * cpf;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += align_up(bytes);
    return p;
  };
  char* p_rb = take((size_t)n_nodes * sizeof(int));
  char* p_rf = take((size_t)n_nodes * sizeof(int));
  char* p_fg = take((size_t)n_frames * sizeof(FrameGrid));
  char* p_cc = take((size_t)n_cells * sizeof(int));
  char* p_cs = take((size_t)(n_cells + 1) * sizeof(int));
  char* p_cu = take((size_t)n_cells * sizeof(int));
  char* p_co = take((size_t)n_nodes * sizeof(int));
  char* p_pt = take((size_t)n_nodes * sizeof(float4));
  char* p_sc = take(scan_workspace_bytes(max((long)n_nodes, n_cells)));
  if (ws) {
    ws->row_base = (int*)p_rb;
    ws->row_frame = (int*)p_rf;
    ws->fg = (FrameGrid*)p_fg;
    ws->cell_cnt = (int*)p_cc;
    ws->cell_start = (int*)p_cs;
    ws->cursor = (int*)p_cu;
    ws->cell_of = (int*)p_co;
    ws->pts = (float4*)p_pt;
    ws->scan_ws = p_sc;
    ws->cpf = cpf;
    ws->n_cells = n_cells;
  }
  return off;
}

extern "C" size_t rg_cluster_radius_workspace_size(int n_nodes, int n_frames, int max_frame_nodes) {
  return grid_ws_layout(n_nodes, n_frames, max_frame_nodes, nullptr, nullptr);
}

extern "C" int rg_cluster_radius(const float* px, const float* py, const int* frame_ptr,
                                 int n_nodes, int n_frames, int max_frame_nodes, float eps2,
                                 int* labels, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_nodes >= 0 && n_frames >= 1 && max_frame_nodes >= 0, RG_ERR_ARG,
             "rg_cluster_radius: bad sizes");
  if (n_nodes == 0) return RG_OK;
  GridWs ws;
  const size_t need = grid_ws_layout(n_nodes, n_frames, max_frame_nodes, &ws, (char*)workspace);
  RG_REQUIRE(workspace_bytes >= need, RG_ERR_ARG, "rg_cluster_radius: workspace %zu < %zu",
             workspace_bytes, need);
  row_frame_base<<<ceil_div(n_nodes, 256), 256, 0, st>>>(frame_ptr, n_frames, ws.row_base,
                                                         ws.row_frame, n_nodes);
  grid_setup<<<n_frames, GS_T, 0, st>>>(px, py, frame_ptr, ws.cpf, ws.fg);
  RG_CHECK_HIP(hipMemsetAsync(ws.cell_cnt, 0, (size_t)ws.n_cells * sizeof(int), st));
  grid_count<<<ceil_div(n_nodes, 256), 256, 0, st>>>(px, py, ws.row_frame, ws.fg, n_nodes,
                                                     ws.cell_of, ws.cell_cnt);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(ws.cell_cnt, ws.n_cells, ws.cell_start, ws.cell_start + ws.n_cells,
                          ws.scan_ws, st);
  if (rc) return rc;
  RG_CHECK_HIP(hipMemcpyAsync(ws.cursor, ws.cell_start, (size_t)ws.n_cells * sizeof(int),
                              hipMemcpyDeviceToDevice, st));
  grid_scatter<<<ceil_div(n_nodes, 256), 256, 0, st>>>(px, py, ws.row_base, ws.cell_of, n_nodes,
                                                       ws.cursor, ws.pts);
  cc_init<<<ceil_div(n_nodes, 256), 256, 0, st>>>(labels, n_nodes);
  cc_radius_hook<<<ceil_div(n_nodes, KNN_BLOCK), KNN_BLOCK, 0, st>>>(
      ws.pts, ws.cell_start, ws.row_frame, ws.fg, frame_ptr, n_nodes, eps2, labels);
  cc_compress<<<ceil_div(n_nodes, 256), 256, 0, st>>>(labels, n_nodes);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_cluster_pairs(const float* px, const float* py, const int* pair_src,
                                const int* pair_dst, const int* n_pairs_dev, long n_pairs,
                                const float* link_logits, int ld_logits, float eps, int n_nodes,
                                int* labels, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_nodes >= 0 && n_pairs >= 0 && ld_logits >= 2, RG_ERR_ARG,
             "rg_cluster_pairs: bad sizes");
  if (n_nodes == 0) return RG_OK;
  cc_init<<<ceil_div(n_nodes, 256), 256, 0, st>>>(labels, n_nodes);
  if (n_pairs > 0)
    cc_pairs_hook<<<ceil_div(n_pairs, 256), 256, 0, st>>>(px, py, pair_src, pair_dst, n_pairs_dev,
                                                          n_pairs, link_logits, ld_logits, eps,
                                                          labels);
  cc_compress<<<ceil_div(n_nodes, 256), 256, 0, st>>>(labels, n_nodes);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
