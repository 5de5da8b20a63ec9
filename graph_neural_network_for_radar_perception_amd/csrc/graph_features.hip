// Node / edge input features, link pairs, destination-major CSR, tensorization helpers.
//
//   rg_node_features  <- compute_node_features   graph_features.py:117-144 (+ normalize_time :47-55)
//   rg_edge_features  <- compute_edge_features   graph_features.py:147-164
//   rg_link_pairs     <- edge_formation triu/nonzero gnn_blocks.py:295-296
//   rg_csr_by_dst     <- PyG's gather/scatter indexing of edge_index[1] (gnn_blocks.py:106)
//   rg_dense_adjacency<- the dense adj_matrix / distance_mat of graph_features.py:80-84
#include "rg_common.h"
#include "scan.h"

// numpy semantics: every f32/f64 operation rounds on its own -- never contract
// a*b+c into an FMA in this file (hipcc's default is -ffp-contract=fast)
#pragma clang fp contract(off)

namespace rg {

// ------------------------------------------------------------------ node features
// Blocks (chunk c = blockIdx.x, frame f = blockIdx.y): every block reduces its frame's
// min/max timestamp (an L2-resident re-read; a frame of one block would serialise a
// 20 000-node frame's f64 atan2 work on one CU), then computes the nodes of chunks
// c, c + gridDim.x, ... of the frame.
// Arithmetic follows numpy-2 promotion of the reference expressions:
//   t_norm     = float64(t - tmin) / float64(tmax - tmin)      (int64 / int64 -> f64)
//   degree/10  = float64(deg) / 10
//   r          = sqrtf(px*px + py*py)                           (float32)
//   range_conf = (float64(r) - max_range) / (min_range - max_range)   (np.float64 scalars)
//   th         = |atan2(py, px)| rounded to float32
//   azi_conf   = (th - f32(max_az)) / f32(min_az - max_az)     (python-float scalars: weak -> f32)
// OutT = float: the tensorized float32 features (datagen_gnn.py:122); OutT = double: the
// float64 array compute_node_features itself returns (np.stack promotes the float32
// columns exactly; t_norm, degree / 10 and range_conf are float64 computations)
template <typename OutT>
__global__ __launch_bounds__(256) void node_features_kernel(
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ vr,
    const float* __restrict__ rcs, const int64_t* __restrict__ ts, const int* __restrict__ deg,
    const int* __restrict__ frame_ptr, double min_r, double max_r, float az_den, float max_az,
    OutT* __restrict__ out) {
  const int f = blockIdx.y;
  const int b = frame_ptr[f], e = frame_ptr[f + 1];
  if (b + (int)blockIdx.x * 256 >= e) return;  // block-uniform: no chunk of this frame
  __shared__ long long smin[256], smax[256];
  long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000ULL;
  // eight loads in flight per thread (a one-load loop over a 20 000-node frame waited 79
  // L2 round trips per thread)
  int i0 = b + threadIdx.x;
  for (; i0 + 7 * 256 < e; i0 += 8 * 256) {
    long long t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = ts[i0 + u * 256];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      mn = t[u] < mn ? t[u] : mn;
      mx = t[u] > mx ? t[u] : mx;
    }
  }
  for (int i = i0; i < e; i += 256) {
    const long long t = ts[i];
    mn = t < mn ? t : mn;
    mx = t > mx ? t : mx;
  }
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = min(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = max(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  const long long tmin = smin[0], tmax = smax[0];
  const double span = (double)(tmax - tmin);
  for (int i = b + (int)blockIdx.x * 256 + threadIdx.x; i < e; i += 256 * gridDim.x) {
    const double tn = tmax == tmin ? (double)(ts[i] - tmin) : (double)(ts[i] - tmin) / span;
    const double dg = (double)deg[i] / 10.0;
    const float x = px[i], y = py[i];
    const float r = sqrt_rn(((x * x) + (y * y)));
    const double rc = ((double)r - max_r) / (min_r - max_r);
    const float th = fabsf((float)atan2((double)y, (double)x));
    const float az = div_rn((th - max_az), az_den);
    OutT* o = out + (size_t)i * 6;
    o[0] = (OutT)vr[i];
    o[1] = (OutT)rcs[i];
    o[2] = (OutT)tn;
    o[3] = (OutT)dg;
    o[4] = (OutT)rc;
    o[5] = (OutT)az;
  }
}

// ------------------------------------------------------------------ edge features
// One thread per edge (src -> dst).  graph_features.py:153-161 in float32
// (dx/10, dl = sqrt(dx^2+dy^2)/10, ...) and dt = float64(t_s - t_d) * 1e-6,
// all cast to float32 as the tensorization does (datagen_gnn.py:121).
// x / 10 correctly rounded to f32 without a division: x = M 2^E (24-bit M), so x / 10
// is either exactly representable or at least 2^-27 (relative) away from every f32
// rounding midpoint (the distance is 2^(e-1) |M 2^j - 10 (2k+1)| / 10 with a nonzero
// integer numerator), while the f64 product x * 0.1 is within 2^-52 of x / 10: rounding
// it to f32 gives the correctly rounded quotient (numpy's float32 x / 10) for every x.
__device__ __forceinline__ float div10_rn(float x) { return (float)((double)x * 0.1); }

__global__ __launch_bounds__(256) void edge_features_kernel(
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ vx,
    const float* __restrict__ vy, const int64_t* __restrict__ ts, const int* __restrict__ src,
    const int* __restrict__ dst, const int* __restrict__ n_edges_dev, long n_edges,
    float* __restrict__ out) {
  // rows of 7 floats (28 B) written per lane would touch every cache line of the block's
  // output seven times with partial writes: the block stages its 256 x 7 values in LDS
  // (stride 7 words: conflict-free) and writes them back as contiguous 16-B vectors
  __shared__ float4 stage4[256 * 7 / 4];
  float* stage = (float*)stage4;
  const long E = min(n_edges_dev ? (long)*n_edges_dev : n_edges, n_edges);
  for (long b0 = (long)blockIdx.x * 256; b0 < E; b0 += (long)gridDim.x * 256) {
    const long p = b0 + threadIdx.x;
    if (p < E) {
      const int s = src[p];
      const int d = dst[p];
      const float dx = div10_rn((px[s] - px[d]));
      const float dy = div10_rn((py[s] - py[d]));
      const float dl = div10_rn(sqrt_rn(((dx * dx) + (dy * dy))));
      const float dvx = (vx[s] - vx[d]);
      const float dvy = (vy[s] - vy[d]);
      const float dv = sqrt_rn(((dvx * dvx) + (dvy * dvy)));
      const float dt = (float)((double)(ts[s] - ts[d]) * 1e-6);
      float* o = stage + threadIdx.x * 7;
      o[0] = dx; o[1] = dy; o[2] = dl; o[3] = dvx; o[4] = dvy; o[5] = dv; o[6] = dt;
    }
    __syncthreads();
    const int n = (int)min(256L, E - b0) * 7;  // floats of this block; b0 * 7 * 4 B is 16-B aligned
    const int n4 = ((uintptr_t)out & 15) == 0 ? n / 4 : 0;  // a caller's unaligned view: dwords
    float4* o4 = (float4*)(out + (size_t)b0 * 7);
    for (int i = threadIdx.x; i < n4; i += 256) o4[i] = stage4[i];
    for (int i = 4 * n4 + threadIdx.x; i < n; i += 256) out[(size_t)b0 * 7 + i] = stage[i];
    __syncthreads();
  }
}

// compute_edge_features' own float64 result (graph_features.py:147-164): columns 0-5 are
// float32 computations promoted exactly by np.stack; dt = (t_s - t_d) * 1e-6 is int64 x
// python float = float64
__global__ __launch_bounds__(256) void edge_features_f64_kernel(
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ vx,
    const float* __restrict__ vy, const int64_t* __restrict__ ts, const int* __restrict__ src,
    const int* __restrict__ dst, long n_edges, double* __restrict__ out) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n_edges; p += (long)gridDim.x * 256) {
    const int s = src[p];
    const int d = dst[p];
    const float dx = div10_rn((px[s] - px[d]));
    const float dy = div10_rn((py[s] - py[d]));
    const float dl = div10_rn(sqrt_rn(((dx * dx) + (dy * dy))));
    const float dvx = (vx[s] - vx[d]);
    const float dvy = (vy[s] - vy[d]);
    const float dv = sqrt_rn(((dvx * dvx) + (dvy * dvy)));
    double* o = out + (size_t)p * 7;
    o[0] = dx; o[1] = dy; o[2] = dl; o[3] = dvx; o[4] = dvy; o[5] = dv;
    o[6] = (double)(ts[s] - ts[d]) * 1e-6;
  }
}

// The same from node kinematics packed as float4 (px, py, vx, vy): two gathers per
// endpoint (the float4 and the timestamp) instead of five separate arrays (the kernel
// above is bound by its ten gathered loads per edge).
__global__ __launch_bounds__(256) void pack_kinematics_kernel(
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ vx,
    const float* __restrict__ vy, int n, float4* __restrict__ kin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) kin[i] = make_float4(px[i], py[i], vx[i], vy[i]);
}

__global__ __launch_bounds__(256) void edge_features_packed_kernel(
    const float4* __restrict__ kin, const int64_t* __restrict__ ts, const int* __restrict__ src,
    const int* __restrict__ dst, const int* __restrict__ n_edges_dev, long n_edges,
    float* __restrict__ out) {
  __shared__ float4 stage4[256 * 7 / 4];
  float* stage = (float*)stage4;
  const long E = min(n_edges_dev ? (long)*n_edges_dev : n_edges, n_edges);
  for (long b0 = (long)blockIdx.x * 256; b0 < E; b0 += (long)gridDim.x * 256) {
    const long p = b0 + threadIdx.x;
    if (p < E) {
      const int s = src[p];
      const int d = dst[p];
      const float4 ks = kin[s], kd = kin[d];
      const int64_t tsd = ts[s] - ts[d];
      const float dx = div10_rn((ks.x - kd.x));
      const float dy = div10_rn((ks.y - kd.y));
      const float dl = div10_rn(sqrt_rn(((dx * dx) + (dy * dy))));
      const float dvx = (ks.z - kd.z);
      const float dvy = (ks.w - kd.w);
      const float dv = sqrt_rn(((dvx * dvx) + (dvy * dvy)));
      const float dt = (float)((double)tsd * 1e-6);
      float* o = stage + threadIdx.x * 7;
      o[0] = dx; o[1] = dy; o[2] = dl; o[3] = dvx; o[4] = dvy; o[5] = dv; o[6] = dt;
    }
    __syncthreads();
    const int n = (int)min(256L, E - b0) * 7;
    const int n4 = ((uintptr_t)out & 15) == 0 ? n / 4 : 0;
    float4* o4 = (float4*)(out + (size_t)b0 * 7);
    for (int i = threadIdx.x; i < n4; i += 256) o4[i] = stage4[i];
    for (int i = 4 * n4 + threadIdx.x; i < n; i += 256) out[(size_t)b0 * 7 + i] = stage[i];
    __syncthreads();
  }
}

// ------------------------------------------------------------------ link pairs
__global__ void pairs_count(const int* __restrict__ row_ptr, const int* __restrict__ col,
                            int n_nodes, int* __restrict__ cnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  int lo = row_ptr[i], hi = row_ptr[i + 1];  // first position with col > i
  const int end = hi;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (col[mid] <= i) lo = mid + 1; else hi = mid;
  }
  cnt[i] = end - lo;
}

__global__ __launch_bounds__(256) void pairs_emit(const int* __restrict__ row_ptr,
                                                  const int* __restrict__ col, int n_nodes,
                                                  const int* __restrict__ pair_ptr,
                                                  int* __restrict__ ps, int* __restrict__ pd,
                                                  long cap) {
  // 16 lanes per row (a kNN row has ~k/2 + a few pairs: a wave per row left most idle)
  const int lane = threadIdx.x & 15;
  const int nw = gridDim.x * 16;
  for (int row = blockIdx.x * 16 + (threadIdx.x >> 4); row < n_nodes; row += nw) {
    const int e = row_ptr[row + 1];
    const int q0 = pair_ptr[row], q1 = pair_ptr[row + 1];
    if ((long)q1 > cap) continue;
    const int n = q1 - q0;
    const int start = e - n;  // cols > row are the row's suffix
    for (int t = lane; t < n; t += 16) {
      ps[q0 + t] = row;
      pd[q0 + t] = col[start + t];
    }
  }
}

// ------------------------------------------------------------------ CSR by destination
__global__ void dst_count(const int64_t* __restrict__ ei, long E, int n_nodes,
                          int* __restrict__ cnt, int* __restrict__ bad) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  const int64_t s = ei[p], d = ei[E + p];
  if (s < 0 || s >= n_nodes || d < 0 || d >= n_nodes) {
    atomicOr(bad, 1);
    return;
  }
  atomicAdd(cnt + d, 1);
}

__global__ void dst_fill(const int64_t* __restrict__ ei, long E, int n_nodes,
                         const int* __restrict__ dst_ptr, int* __restrict__ cursor,
                         int* __restrict__ perm) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  const int64_t s = ei[p], d = ei[E + p];
  if (s < 0 || s >= n_nodes || d < 0 || d >= n_nodes) return;
  const int slot = atomicAdd(cursor + d, 1);
  perm[dst_ptr[d] + slot] = (int)p;
}

// order each destination segment by (src, reference position): insertion sort,
// segments are short (node degree)
__global__ void dst_sort(const int64_t* __restrict__ ei, int n_nodes, const int* __restrict__ dst_ptr,
                         int* __restrict__ perm, int* __restrict__ src_sorted) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_nodes) return;
  const int b = dst_ptr[d], e = dst_ptr[d + 1];
  for (int i = b + 1; i < e; ++i) {
    const int v = perm[i];
    const int64_t kv = ei[v];
    int j = i - 1;
    while (j >= b) {
      const int u = perm[j];
      const int64_t ku = ei[u];
      if (ku < kv || (ku == kv && u < v)) break;
      perm[j + 1] = u;
      --j;
    }
    perm[j + 1] = v;
  }
  for (int i = b; i < e; ++i) src_sorted[i] = (int)ei[perm[i]];
}

// ------------------------------------------------------------------ dense views
__global__ void dense_adj_kernel(const float* __restrict__ px, const float* __restrict__ py,
                                 const int* __restrict__ row_ptr, const int* __restrict__ col,
                                 int n, uint8_t* __restrict__ adj, float* __restrict__ dist) {
  const int i = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  if (dist) {
    float dx = (px[i] - px[j]), dy = (py[i] - py[j]);
    dist[(size_t)i * n + j] = ((dx * dx) + (dy * dy));
  }
  if (adj) adj[(size_t)i * n + j] = 0;
}

__global__ void dense_adj_set(const int* __restrict__ row_ptr, const int* __restrict__ col, int n,
                              uint8_t* __restrict__ adj) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int p = row_ptr[i]; p < row_ptr[i + 1]; ++p) adj[(size_t)i * n + col[p]] = 1;
}

// CSR row id of every position (edge_index[0] of the np.where order, or the
// destination of each destination-major edge)
__global__ __launch_bounds__(256) void csr_rows_kernel(const int* __restrict__ row_ptr, int n_rows,
                                                       int* __restrict__ out) {
  // 16 lanes per row: graph rows hold tens of edges, so a 64-lane wave per row idled most lanes
  const int lane = threadIdx.x & 15;
  const int nw = gridDim.x * 16;
  for (int row = blockIdx.x * 16 + (threadIdx.x >> 4); row < n_rows; row += nw) {
    const int b = row_ptr[row], e = row_ptr[row + 1];
    for (int p = b + lane; p < e; p += 16) out[p] = row;
  }
}

// link pairs of an arbitrary edge_index: positions p with ei[0][p] < ei[1][p], in order
__global__ void pair_flags(const int64_t* __restrict__ ei, long E, int* __restrict__ flag) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < E) flag[p] = ei[p] < ei[E + p] ? 1 : 0;
}
__global__ void pair_scatter(const int64_t* __restrict__ ei, long E, const int* __restrict__ pos,
                             int* __restrict__ ps, int* __restrict__ pd) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= E) return;
  const int64_t s = ei[p], d = ei[E + p];
  if (s < d) {
    ps[pos[p]] = (int)s;
    pd[pos[p]] = (int)d;
  }
}

__global__ void i32_to_i64_kernel(const int* __restrict__ in, long n, int64_t* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i];
}

__global__ void gather_rows_kernel(const float* __restrict__ in, const int* __restrict__ idx,
                                   long rows, int w, float* __restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * w) return;
  const long r = t / w;
  const int c = (int)(t % w);
  out[t] = in[(size_t)idx[r] * w + c];
}

}  // namespace rg

using namespace rg;

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

extern "C" int rg_node_features(const float* px, const float* py, const float* vr,
                                const float* rcs, const int64_t* timestamp, const int* ball_degree,
                                const int* frame_ptr, int n_nodes, int n_frames, double min_range,
                                double max_range, double min_azimuth, double max_azimuth,
                                float* out, void* stream) {
  RG_REQUIRE(n_frames >= 1 && n_nodes >= 0, RG_ERR_ARG, "rg_node_features: bad sizes");
  if (n_nodes == 0) return RG_OK;
  // chunks of 256 nodes per frame at the mean frame size (larger frames stride)
  const int chunks = max(1, min(1024, (int)((n_nodes / n_frames + 255) / 256)));
  node_features_kernel<float><<<dim3(chunks, n_frames), 256, 0, (hipStream_t)stream>>>(
      px, py, vr, rcs, timestamp, ball_degree, frame_ptr, min_range, max_range,
      (float)(min_azimuth - max_azimuth), (float)max_azimuth, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_node_features_f64(const float* px, const float* py, const float* vr,
                                    const float* rcs, const int64_t* timestamp,
                                    const int* ball_degree, const int* frame_ptr, int n_nodes,
                                    int n_frames, double min_range, double max_range,
                                    double min_azimuth, double max_azimuth, double* out,
                                    void* stream) {
  RG_REQUIRE(n_frames >= 1 && n_nodes >= 0, RG_ERR_ARG, "rg_node_features_f64: bad sizes");
  if (n_nodes == 0) return RG_OK;
  const int chunks = max(1, min(1024, (int)((n_nodes / n_frames + 255) / 256)));
  node_features_kernel<double><<<dim3(chunks, n_frames), 256, 0, (hipStream_t)stream>>>(
      px, py, vr, rcs, timestamp, ball_degree, frame_ptr, min_range, max_range,
      (float)(min_azimuth - max_azimuth), (float)max_azimuth, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_edge_features_f64(const float* px, const float* py, const float* vx,
                                    const float* vy, const int64_t* timestamp, const int* src,
                                    const int* dst, long n_edges, double* out, void* stream) {
  if (n_edges <= 0) return RG_OK;
  long blocks = (n_edges + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  edge_features_f64_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(px, py, vx, vy, timestamp, src,
                                                                    dst, n_edges, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_edge_features(const float* px, const float* py, const float* vx, const float* vy,
                                const int64_t* timestamp, const int* src, const int* dst,
                                const int* n_edges_dev, long n_edges, float* out, void* stream) {
  if (n_edges <= 0) return RG_OK;
  long blocks = (n_edges + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  edge_features_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(px, py, vx, vy, timestamp, src, dst,
                                                                n_edges_dev, n_edges, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_pack_kinematics(const float* px, const float* py, const float* vx,
                                  const float* vy, int n_nodes, void* kin, void* stream) {
  RG_REQUIRE(n_nodes >= 0 && ((uintptr_t)kin & 15) == 0, RG_ERR_ARG,
             "rg_pack_kinematics: n_nodes=%d, kin must be 16-B aligned", n_nodes);
  if (n_nodes == 0) return RG_OK;
  pack_kinematics_kernel<<<ceil_div(n_nodes, 256), 256, 0, (hipStream_t)stream>>>(
      px, py, vx, vy, n_nodes, (float4*)kin);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_edge_features_packed(const void* kin, const int64_t* timestamp, const int* src,
                                       const int* dst, const int* n_edges_dev, long n_edges,
                                       float* out, void* stream) {
  if (n_edges <= 0) return RG_OK;
  long blocks = (n_edges + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  edge_features_packed_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(
      (const float4*)kin, timestamp, src, dst, n_edges_dev, n_edges, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_link_pairs_workspace_size(int n_nodes) {
  return align256((size_t)n_nodes * sizeof(int)) + align256(scan_workspace_bytes(n_nodes));
}

extern "C" int rg_link_pairs(const int* row_ptr, const int* col, int n_nodes, int* pair_ptr,
                             int* pair_src, int* pair_dst, long pair_capacity, int* n_pairs,
                             void* workspace, size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(workspace_bytes >= rg_link_pairs_workspace_size(n_nodes), RG_ERR_ARG,
             "rg_link_pairs: workspace too small");
  if (n_nodes == 0) {
    RG_CHECK_HIP(hipMemsetAsync(pair_ptr, 0, sizeof(int), st));
    RG_CHECK_HIP(hipMemsetAsync(n_pairs, 0, sizeof(int), st));
    return RG_OK;
  }
  int* cnt = (int*)workspace;
  void* sws = (char*)workspace + align256((size_t)n_nodes * sizeof(int));
  pairs_count<<<ceil_div(n_nodes, 256), 256, 0, st>>>(row_ptr, col, n_nodes, cnt);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(cnt, n_nodes, pair_ptr, n_pairs, sws, st);
  if (rc) return rc;
  int blocks = ceil_div(n_nodes, 16);
  if (blocks > 8192) blocks = 8192;
  pairs_emit<<<blocks, 256, 0, st>>>(row_ptr, col, n_nodes, pair_ptr, pair_src, pair_dst,
                                     pair_capacity);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_csr_by_dst_workspace_size(int n_nodes, long n_edges) {
  (void)n_edges;
  return 2 * align256((size_t)n_nodes * sizeof(int)) + align256(sizeof(int) * 64) +
         align256(scan_workspace_bytes(n_nodes));
}

extern "C" int rg_csr_by_dst(const int64_t* edge_index, long n_edges, int n_nodes, int* dst_ptr,
                             int* perm, int* src_sorted, void* workspace, size_t workspace_bytes,
                             void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(workspace_bytes >= rg_csr_by_dst_workspace_size(n_nodes, n_edges), RG_ERR_ARG,
             "rg_csr_by_dst: workspace too small");
  char* w = (char*)workspace;
  int* cnt = (int*)w;
  w += align256((size_t)n_nodes * sizeof(int));
  int* cursor = (int*)w;
  w += align256((size_t)n_nodes * sizeof(int));
  int* bad = (int*)w;
  w += align256(sizeof(int) * 64);
  void* sws = w;
  RG_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)n_nodes * sizeof(int), st));
  RG_CHECK_HIP(hipMemsetAsync(cursor, 0, (size_t)n_nodes * sizeof(int), st));
  RG_CHECK_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
  if (n_edges > 0) {
    dst_count<<<ceil_div(n_edges, 256), 256, 0, st>>>(edge_index, n_edges, n_nodes, cnt, bad);
    RG_LAUNCH_CHECK();
  }
  int rc = exclusive_scan(cnt, n_nodes, dst_ptr, nullptr, sws, st);
  if (rc) return rc;
  if (n_edges > 0) {
    dst_fill<<<ceil_div(n_edges, 256), 256, 0, st>>>(edge_index, n_edges, n_nodes, dst_ptr, cursor,
                                                     perm);
    RG_LAUNCH_CHECK();
    dst_sort<<<ceil_div(n_nodes, 256), 256, 0, st>>>(edge_index, n_nodes, dst_ptr, perm,
                                                     src_sorted);
    RG_LAUNCH_CHECK();
  }
  return RG_OK;
}

extern "C" int rg_dense_adjacency(const float* px, const float* py, const int* row_ptr,
                                  const int* col, int n_nodes, uint8_t* adj, float* dist,
                                  void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n_nodes == 0) return RG_OK;
  dim3 grid(ceil_div(n_nodes, 256), n_nodes);
  dense_adj_kernel<<<grid, 256, 0, st>>>(px, py, row_ptr, col, n_nodes, adj, dist);
  RG_LAUNCH_CHECK();
  if (adj) {
    dense_adj_set<<<ceil_div(n_nodes, 256), 256, 0, st>>>(row_ptr, col, n_nodes, adj);
    RG_LAUNCH_CHECK();
  }
  return RG_OK;
}

extern "C" int rg_i32_to_i64(const int* in, long n, int64_t* out, void* stream) {
  if (n <= 0) return RG_OK;
  i32_to_i64_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(in, n, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gather_rows_f32(const float* in, const int* idx, long rows, int w, float* out,
                                  void* stream) {
  if (rows <= 0 || w <= 0) return RG_OK;
  gather_rows_kernel<<<ceil_div(rows * w, 256), 256, 0, (hipStream_t)stream>>>(in, idx, rows, w,
                                                                                out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_csr_rows(const int* row_ptr, int n_rows, int* out, void* stream) {
  if (n_rows <= 0) return RG_OK;
  int blocks = ceil_div(n_rows, 16);
  if (blocks > 16384) blocks = 16384;
  csr_rows_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(row_ptr, n_rows, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Capacity guard of a radius graph built into a capacity that was not checked on the host
// first: need[0] = the true edge count; when it exceeds cap, the CSR is cut at the last row
// boundary <= cap / 2 (rows past cap were not written by row_emit; and a cut graph is no
// longer symmetric, so its i < j link pairs are bounded only by its edge count, while the
// pair arrays hold cap / 2 + 1) and n_edges = that boundary, so every consumer stays
// inside its arrays.  One workgroup.
__global__ __launch_bounds__(1024) void csr_clamp_kernel(int* __restrict__ row_ptr, int n,
                                                          int* __restrict__ n_edges, long cap,
                                                          int* __restrict__ need) {
  __shared__ int cut;
  const int E = *n_edges;
  if (threadIdx.x == 0) need[0] = E;
  if ((long)E <= cap) return;  // uniform
  if (threadIdx.x == 0) {
    int lo = 0, hi = n;  // the largest j with row_ptr[j] <= cap / 2 (row_ptr[0] = 0)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((long)row_ptr[mid] <= cap / 2) lo = mid;
      else hi = mid - 1;
    }
    cut = row_ptr[lo];
  }
  __syncthreads();
  for (int i = threadIdx.x; i <= n; i += blockDim.x)
    if (row_ptr[i] > cut) row_ptr[i] = cut;
  if (threadIdx.x == 0) *n_edges = cut;
}

extern "C" int rg_csr_clamp(int* row_ptr, int n_rows, int* n_edges_dev, long capacity,
                            int* need_out, void* stream) {
  RG_REQUIRE(row_ptr && n_edges_dev && need_out && n_rows >= 0, RG_ERR_ARG,
             "rg_csr_clamp: null argument");
  csr_clamp_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(row_ptr, n_rows, n_edges_dev, capacity,
                                                       need_out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_pairs_from_edge_index_workspace_size(long n_edges) {
  return 2 * align256((size_t)(n_edges + 1) * sizeof(int)) + align256(scan_workspace_bytes(n_edges));
}

// edge_formation's pairs from a dense adjacency (gnn_blocks.py:295-296: torch.nonzero(
// torch.triu(adj, 1)), row-major) in two passes over the rows, one wave per row: count
// the set entries right of the diagonal, exclusive scan of the row counts (the caller sizes
// the pair arrays from the total), then emit each row's pairs in column order (ballot +
// popcount prefix per 64-column chunk).  Workspace O(n), not O(n^2).
__global__ __launch_bounds__(256) void dense_pair_row_count(const uint8_t* __restrict__ adj,
                                                             int n, int* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int i = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (i >= n) return;  // wave-uniform
  const uint8_t* row = adj + (size_t)i * n;
  int c = 0;
  for (int j = i + 1 + lane; j < n; j += 64) c += row[j] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) cnt[i] = c;
}
__global__ __launch_bounds__(256) void dense_pair_row_emit(const uint8_t* __restrict__ adj, int n,
                                                            const int* __restrict__ row_ptr,
                                                            int* __restrict__ ps,
                                                            int* __restrict__ pd) {
  const int lane = threadIdx.x & 63;
  const int i = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (i >= n) return;  // wave-uniform
  const uint8_t* row = adj + (size_t)i * n;
  int pos = row_ptr[i];
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int j0 = i + 1; j0 < n; j0 += 64) {
    const int j = j0 + lane;
    const bool set = j < n && row[j] != 0;
    const unsigned long long m = __ballot(set);
    if (set) {
      const int p = pos + __popcll(m & below);
      ps[p] = i;
      pd[p] = j;
    }
    pos += __popcll(m);
  }
}
// out[r] = x[idx0[r]] + x[idx1[r]] (float32, one rounding: the reference's x[i] + x[j])
__global__ void pair_add_rows_kernel(const float* __restrict__ x, int ldx, int w,
                                     const int* __restrict__ i0, const int* __restrict__ i1,
                                     long rows, float* __restrict__ out, int ldo) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * w) return;
  const long r = t / w;
  const int c = (int)(t - r * w);
  out[r * ldo + c] = x[(size_t)i0[r] * ldx + c] + x[(size_t)i1[r] * ldx + c];
}

extern "C" size_t rg_dense_pair_rows_workspace_size(int n_nodes) {
  return align256((size_t)(n_nodes + 1) * sizeof(int)) + scan_workspace_bytes(n_nodes);
}

extern "C" int rg_dense_pair_rows(const void* adj, int n_nodes, int* row_ptr, int* n_pairs,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_nodes >= 0 && n_nodes <= 46340, RG_ERR_ARG,
             "rg_dense_pair_rows: n_nodes=%d outside 0..46340", n_nodes);
  RG_REQUIRE(adj || n_nodes == 0, RG_ERR_ARG, "rg_dense_pair_rows: null adjacency");
  RG_REQUIRE(workspace_bytes >= rg_dense_pair_rows_workspace_size(n_nodes), RG_ERR_ARG,
             "rg_dense_pair_rows: workspace too small");
  if (n_nodes == 0) {
    RG_CHECK_HIP(hipMemsetAsync(row_ptr, 0, sizeof(int), st));
    RG_CHECK_HIP(hipMemsetAsync(n_pairs, 0, sizeof(int), st));
    return RG_OK;
  }
  char* w = (char*)workspace;
  int* cnt = (int*)w;
  w += align256((size_t)(n_nodes + 1) * sizeof(int));
  dense_pair_row_count<<<ceil_div((long)n_nodes * 64, 256), 256, 0, st>>>((const uint8_t*)adj,
                                                                           n_nodes, cnt);
  RG_LAUNCH_CHECK();
  return exclusive_scan(cnt, n_nodes, row_ptr, n_pairs, w, st);
}

extern "C" int rg_dense_pair_emit(const void* adj, int n_nodes, const int* row_ptr, int* pair_src,
                                  int* pair_dst, void* stream) {
  RG_REQUIRE(n_nodes >= 0 && n_nodes <= 46340, RG_ERR_ARG,
             "rg_dense_pair_emit: n_nodes=%d outside 0..46340", n_nodes);
  if (n_nodes == 0) return RG_OK;
  RG_REQUIRE(adj && row_ptr && pair_src && pair_dst, RG_ERR_ARG, "rg_dense_pair_emit: null argument");
  dense_pair_row_emit<<<ceil_div((long)n_nodes * 64, 256), 256, 0, (hipStream_t)stream>>>(
      (const uint8_t*)adj, n_nodes, row_ptr, pair_src, pair_dst);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_pair_add_rows_f32(const float* x, int ldx, int w, const int* idx0,
                                    const int* idx1, long rows, float* out, int ld_out,
                                    void* stream) {
  RG_REQUIRE(w >= 0 && rows >= 0, RG_ERR_ARG, "rg_pair_add_rows_f32: bad sizes");
  if (rows == 0 || w == 0) return RG_OK;
  pair_add_rows_kernel<<<ceil_div(rows * w, 256), 256, 0, (hipStream_t)stream>>>(
      x, ldx, w, idx0, idx1, rows, out, ld_out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_pairs_from_edge_index(const int64_t* edge_index, long n_edges, int* pair_src,
                                        int* pair_dst, int* n_pairs, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(workspace_bytes >= rg_pairs_from_edge_index_workspace_size(n_edges), RG_ERR_ARG,
             "rg_pairs_from_edge_index: workspace too small");
  if (n_edges <= 0) {
    RG_CHECK_HIP(hipMemsetAsync(n_pairs, 0, sizeof(int), st));
    return RG_OK;
  }
  char* w = (char*)workspace;
  int* flag = (int*)w;
  w += align256((size_t)(n_edges + 1) * sizeof(int));
  int* pos = (int*)w;
  w += align256((size_t)(n_edges + 1) * sizeof(int));
  pair_flags<<<ceil_div(n_edges, 256), 256, 0, st>>>(edge_index, n_edges, flag);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(flag, n_edges, pos, n_pairs, w, st);
  if (rc) return rc;
  pair_scatter<<<ceil_div(n_edges, 256), 256, 0, st>>>(edge_index, n_edges, pos, pair_src, pair_dst);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
