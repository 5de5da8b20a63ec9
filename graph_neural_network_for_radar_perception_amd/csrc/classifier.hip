// Graph build of the cluster-level classifier GNN.
//
//   compute_edge_index (datagen_classifier.py:124-133): the block-diagonal union of
//     complete graphs, one per object (cluster of n measurements), self loops
//     removed, edge_index = np.nonzero(adj) -- row-major: source ascending, then
//     destination ascending.  Node i of object c (rows [off_c, off_c + n_c)) has the
//     n_c - 1 neighbours off_c .. off_c + n_c - 1 except itself, so the CSR is closed
//     form: row_ptr[i] = Epref_c + (i - off_c) (n_c - 1), Epref = prefix sum of
//     n (n - 1).  The graph is symmetric, so this CSR is also the destination-major
//     view the aggregation reads (segment i = sources of target i, ascending).
//
//   object row ranges of classifier Model_Inference.forward (classifier.py:60-68):
//     startidx[0] = 0, startidx[i] = object_size[i-1], endidx = cumsum(object_size);
//     object i pools rows [startidx[i], endidx[i]).  (startidx is NOT a cumulative
//     offset in the reference -- for i >= 2 the pooled range starts at the previous
//     object's SIZE -- and the drop-in reproduces exactly that.)
#include "rg_common.h"
#include "scan.h"

namespace rg {

static size_t align256_c(size_t v) { return (v + 255) & ~(size_t)255; }

__global__ void object_sizes_kernel(const int64_t* __restrict__ object_size, int n_obj,
                                    int* __restrict__ sz, int* __restrict__ pairs) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_obj) return;
  const int n = (int)object_size[c];
  sz[c] = n;
  if (pairs) pairs[c] = n * (n - 1);
}

// one thread per node: its object by binary search over the node offsets, then its
// n_c - 1 neighbours in ascending order
__global__ void complete_rows_kernel(const int* __restrict__ node_off, const int* __restrict__ edge_off,
                                     int n_obj, int n_nodes, int* __restrict__ row_ptr,
                                     int* __restrict__ col, int64_t* __restrict__ edge_index,
                                     long n_edges) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) row_ptr[n_nodes] = edge_off[n_obj];
  if (i >= n_nodes) return;
  if (i >= node_off[n_obj]) {  // past the last object: no edges
    row_ptr[i] = edge_off[n_obj];
    return;
  }
  int lo = 0, hi = n_obj - 1;   // last c with node_off[c] <= i (empty objects skipped)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (node_off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  const int c = lo, off = node_off[c], n = node_off[c + 1] - off;
  int p = edge_off[c] + (i - off) * (n - 1);
  row_ptr[i] = p;
  for (int j = off; j < off + n; ++j) {
    if (j == i) continue;
    if (col) col[p] = j;
    if (edge_index) {
      edge_index[p] = i;
      edge_index[n_edges + p] = j;
    }
    ++p;
  }
}

// object c of sample s (objects [sobj[s], sobj[s+1]), rows from nbase[s]):
//   begin = nbase[s] + (c == first ? 0 : object_size[c-1]),
//   end   = nbase[s] + (node_off[c+1] - node_off[first])   (cumsum within the sample)
__global__ void object_ranges_kernel(const int64_t* __restrict__ object_size,
                                     const int* __restrict__ node_off, int n_obj,
                                     const int* __restrict__ sobj, const int* __restrict__ nbase,
                                     int n_samples, int* __restrict__ begin,
                                     int* __restrict__ end) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_obj) return;
  int first = 0, base = 0;
  if (sobj) {
    int lo = 0, hi = n_samples - 1;   // last s with sobj[s] <= c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sobj[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    first = sobj[lo];
    base = nbase[lo];
  }
  begin[c] = base + (c == first ? 0 : (int)object_size[c - 1]);
  end[c] = base + (node_off[c + 1] - node_off[first]);
}

}  // namespace rg

using namespace rg;

extern "C" size_t rg_object_graph_workspace_size(int n_obj) {
  return 4 * align256_c(((size_t)n_obj + 1) * sizeof(int)) + align256_c(scan_workspace_bytes(n_obj));
}

extern "C" int rg_object_complete_graph(const int64_t* object_size, int n_obj, int n_nodes,
                                        long n_edges, int* row_ptr, int* col, int64_t* edge_index,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  RG_REQUIRE(n_obj >= 0 && n_nodes >= 0 && n_edges >= 0 && row_ptr, RG_ERR_ARG,
             "rg_object_complete_graph: bad arguments");
  RG_REQUIRE(workspace_bytes >= rg_object_graph_workspace_size(n_obj), RG_ERR_ARG,
             "rg_object_complete_graph: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (n_obj == 0) {
    RG_CHECK_HIP(hipMemsetAsync(row_ptr, 0, ((size_t)n_nodes + 1) * sizeof(int), st));
    return RG_OK;
  }
  char* w = (char*)workspace;
  const size_t a = align256_c(((size_t)n_obj + 1) * sizeof(int));
  int* sz = (int*)w;
  int* pairs = (int*)(w + a);
  int* node_off = (int*)(w + 2 * a);
  int* edge_off = (int*)(w + 3 * a);
  void* sws = w + 4 * a;
  object_sizes_kernel<<<ceil_div(n_obj, 256), 256, 0, st>>>(object_size, n_obj, sz, pairs);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(sz, n_obj, node_off, nullptr, sws, st);
  if (rc) return rc;
  rc = exclusive_scan(pairs, n_obj, edge_off, nullptr, sws, st);
  if (rc) return rc;
  complete_rows_kernel<<<ceil_div((long)n_nodes + 1, 256), 256, 0, st>>>(
      node_off, edge_off, n_obj, n_nodes, row_ptr, col, edge_index, n_edges);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_object_row_ranges(const int64_t* object_size, int n_obj,
                                    const int* sample_obj_ptr, const int* sample_node_base,
                                    int n_samples, int* begin, int* end, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  RG_REQUIRE(!sample_obj_ptr || (sample_node_base && n_samples >= 1), RG_ERR_ARG,
             "rg_object_row_ranges: sample_obj_ptr needs sample_node_base and n_samples >= 1");
  RG_REQUIRE(workspace_bytes >= rg_object_graph_workspace_size(n_obj), RG_ERR_ARG,
             "rg_object_row_ranges: workspace too small");
  if (n_obj <= 0) return RG_OK;
  hipStream_t st = (hipStream_t)stream;
  char* w = (char*)workspace;
  const size_t a = align256_c(((size_t)n_obj + 1) * sizeof(int));
  int* sz = (int*)w;
  int* node_off = (int*)(w + 2 * a);
  void* sws = w + 4 * a;
  object_sizes_kernel<<<ceil_div(n_obj, 256), 256, 0, st>>>(object_size, n_obj, sz, nullptr);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(sz, n_obj, node_off, nullptr, sws, st);
  if (rc) return rc;
  object_ranges_kernel<<<ceil_div(n_obj, 256), 256, 0, st>>>(
      object_size, node_off, n_obj, sample_obj_ptr, sample_node_base, n_samples, begin, end);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ---------------------------------------------------------------------------
// classifier Loss (classifier/loss.py:5-14, lossfunc.py:52-60): torchvision
// sigmoid_focal_loss(x, t, alpha=-1 (no alpha weighting), gamma=2) with one-hot t,
//   ce = max(x, 0) - x t + log1p(exp(-|x|)),  p = sigmoid(x),
//   p_t = p t + (1 - p)(1 - t),  loss = ce (1 - p_t)^2,
// summed over the classes, then sum / n.
// ---------------------------------------------------------------------------
namespace rg {

__global__ __launch_bounds__(256) void object_focal_loss_kernel(const float* __restrict__ logits,
                                                                int ld,
                                                                const int64_t* __restrict__ labels,
                                                                int n, int nc, float* __restrict__ out) {
  __shared__ double part[256];
  double acc = 0.0;
  for (int r = threadIdx.x; r < n; r += 256) {
    const int64_t lab = labels[r];
    float row = 0.f;
    for (int c = 0; c < nc; ++c) {
      const float x = logits[(size_t)r * ld + c];
      const float t = c == lab ? 1.f : 0.f;
      const float p = 1.f / (1.f + expf(-x));
      const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
      const float pt = p * t + (1.f - p) * (1.f - t);
      const float m = 1.f - pt;
      row += ce * (m * m);
    }
    acc += (double)row;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(part[0] / (double)n);
}

}  // namespace rg

extern "C" int rg_object_focal_loss(const float* logits, int ld, const int64_t* labels, int n,
                                    int nc, float* out, void* stream) {
  RG_REQUIRE(n > 0 && nc > 0 && ld >= nc, RG_ERR_ARG, "rg_object_focal_loss: n=%d nc=%d ld=%d",
             n, nc, ld);
  object_focal_loss_kernel<<<1, 256, 0, (hipStream_t)stream>>>(logits, ld, labels, n, nc, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ---------------------------------------------------------------------------
// Backward of the classifier loss and of its pooling (Model_Training + loss.backward(),
// classifier/training.py).
//
// d loss / d x for the focal loss above, scaled by g / n (g = upstream gradient of the
// scalar loss, on the device):
//   d ce / dx = p - t,  d p_t / dx = (2t - 1) p (1 - p),
//   d [ce (1 - p_t)^2] / dx = (p - t) m^2 - 2 ce m (2t - 1) p (1 - p),  m = 1 - p_t.
// ---------------------------------------------------------------------------
namespace rg {

__global__ __launch_bounds__(256) void object_focal_loss_backward_kernel(
    const float* __restrict__ logits, int ld, const int64_t* __restrict__ labels, int n, int nc,
    const float* __restrict__ g_loss, float* __restrict__ d_logits, int ldd) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n * nc) return;
  const int r = (int)(i / nc), c = (int)(i % nc);
  const float x = logits[(size_t)r * ld + c];
  const float t = c == labels[r] ? 1.f : 0.f;
  const float p = 1.f / (1.f + expf(-x));
  const float ce = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float m = 1.f - pt;
  const float d = (p - t) * (m * m) - 2.f * ce * m * (2.f * t - 1.f) * p * (1.f - p);
  d_logits[(size_t)r * ldd + c] = d * (g_loss[0] / (float)n);
}

// torch.max(x[begin:end], dim=0) backward (classifier/blocks.py:171-176): the gradient
// of object o, channel c goes to the FIRST row of [begin[o], end[o]) holding the maximum
// (torch's index for ties); ranges overlap (classifier.py:60-62), so rows accumulate
// with atomics.  One thread per (object, channel), rows scanned in order.
__global__ __launch_bounds__(256) void range_max_backward_kernel(
    const float* __restrict__ x, int ldx, int C, const int* __restrict__ begin,
    const int* __restrict__ end, int n_obj, const float* __restrict__ d_pooled, int ldp,
    float* __restrict__ dx, int lddx) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n_obj * C) return;
  const int o = (int)(i / C), c = (int)(i % C);
  const int b = begin[o], e = end[o];
  if (b >= e) return;
  int arg = b;
  float best = x[(size_t)b * ldx + c];
  for (int r = b + 1; r < e; ++r) {
    const float v = x[(size_t)r * ldx + c];
    if (v > best || (v != v && best == best)) { best = v; arg = r; }  // NaN wins, as torch.max
  }
  atomicAdd(dx + (size_t)arg * lddx + c, d_pooled[(size_t)o * ldp + c]);
}

}  // namespace rg

extern "C" int rg_object_focal_loss_backward(const float* logits, int ld, const int64_t* labels,
                                             int n, int nc, const float* g_loss, float* d_logits,
                                             int ldd, void* stream) {
  RG_REQUIRE(n > 0 && nc > 0 && ld >= nc && ldd >= nc, RG_ERR_ARG,
             "rg_object_focal_loss_backward: n=%d nc=%d", n, nc);
  const long tot = (long)n * nc;
  object_focal_loss_backward_kernel<<<(tot + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      logits, ld, labels, n, nc, g_loss, d_logits, ldd);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_range_max_backward(const float* x, int ldx, int C, const int* begin,
                                     const int* end, int n_obj, const float* d_pooled, int ldp,
                                     float* dx, int lddx, void* stream) {
  RG_REQUIRE(n_obj >= 0 && C > 0, RG_ERR_ARG, "rg_range_max_backward: n_obj=%d C=%d", n_obj, C);
  if (n_obj == 0) return RG_OK;
  const long tot = (long)n_obj * C;
  range_max_backward_kernel<<<(tot + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      x, ldx, C, begin, end, n_obj, d_pooled, ldp, dx, lddx);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// PyG aggr='max' (scatter_reduce amax, include_self=False, classifier/blocks.py:62-66)
// backward over a destination-major CSR whose position p IS the message row: torch's
// amax backward splits the gradient evenly among the messages equal to the maximum.
// One thread per (segment, channel); empty segments have no messages.
namespace rg {
__global__ __launch_bounds__(256) void segment_amax_backward_kernel(
    const float* __restrict__ msg, int ldm, int C, const int* __restrict__ seg_ptr, int n_seg,
    const float* __restrict__ d_agg, int ldd, float* __restrict__ d_msg, int ldo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n_seg * C) return;
  const int s = (int)(i / C), c = (int)(i % C);
  const int b = seg_ptr[s], e = seg_ptr[s + 1];
  if (b >= e) return;
  float m = msg[(size_t)b * ldm + c];
  int cnt = 1;
  for (int p = b + 1; p < e; ++p) {
    const float v = msg[(size_t)p * ldm + c];
    if (v > m) { m = v; cnt = 1; } else if (v == m) { ++cnt; }
  }
  const float g = d_agg[(size_t)s * ldd + c] / (float)cnt;
  for (int p = b; p < e; ++p)
    d_msg[(size_t)p * ldo + c] = msg[(size_t)p * ldm + c] == m ? g : 0.f;
}
}  // namespace rg

extern "C" int rg_segment_amax_backward(const float* msg, int ldm, int C, const int* seg_ptr,
                                        int n_seg, const float* d_agg, int ldd, float* d_msg,
                                        int ldo, void* stream) {
  RG_REQUIRE(n_seg >= 0 && C > 0, RG_ERR_ARG, "rg_segment_amax_backward: n_seg=%d C=%d", n_seg, C);
  if (n_seg == 0) return RG_OK;
  const long tot = (long)n_seg * C;
  segment_amax_backward_kernel<<<(tot + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      msg, ldm, C, seg_ptr, n_seg, d_agg, ldd, d_msg, ldo);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
