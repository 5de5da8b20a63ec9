// Proposal branch of Model_Inference (gnn_detector.py:164-187) around the clustering
// kernels of graph_build.hip:
//   rg_proposal_centres : unnormalize_gt_offsets (compute_offsets.py:13-17) and
//                         other_features[:, :2] + deltas (gnn_detector.py:165-167);
//   rg_cluster_lists    : component labels (root = lowest node index) -> cluster ids in
//                         the reference's order (ascending lowest index, per frame, frames
//                         concatenated) and the member lists, each ascending
//                         (np.nonzero(meas_to_cluster_id == i), gnn_detector.py:181-184),
//                         as a CSR: cluster_ptr / cluster_idx.
#include "rg_common.h"
#include "scan.h"

#include <hipcub/hipcub.hpp>

// the f32 operation order of the reference (torch in-place mul then add, no FMA)
#pragma clang fp contract(off)

namespace rg {
namespace prop {

__global__ void centres_kernel(const float* __restrict__ off, int ld_off,
                               const float* __restrict__ xy, int ld_xy, int n, float mu_x,
                               float mu_y, float sg_x, float sg_y, float* __restrict__ cx,
                               float* __restrict__ cy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float dx = (off[(size_t)i * ld_off + 0] * sg_x) + mu_x;
  const float dy = (off[(size_t)i * ld_off + 1] * sg_y) + mu_y;
  cx[i] = xy[(size_t)i * ld_xy + 0] + dx;
  cy[i] = xy[(size_t)i * ld_xy + 1] + dy;
}

__global__ void root_flags(const int* __restrict__ labels, int n, int* __restrict__ flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = labels[i] == i ? 1 : 0;
}

// cluster id of a node = rank of its root among all roots; members counted per cluster
__global__ void cluster_ids(const int* __restrict__ labels, const int* __restrict__ root_rank,
                            int n, int* __restrict__ cluster_of, int* __restrict__ count,
                            int* __restrict__ node_iota) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = root_rank[labels[i]];
  cluster_of[i] = c;
  node_iota[i] = i;
  atomicAdd(count + c, 1);
}

struct ListWs {
  int* flag;
  int* rank;
  int* count;
  int* iota;
  int* keys_out;
  void* scan_ws;
  void* sort_ws;
  size_t sort_bytes;
};

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

static size_t sort_temp_bytes(int n) {
  size_t bytes = 0;
  const hipError_t e = hipcub::DeviceRadixSort::SortPairs(
      nullptr, bytes, (const int*)nullptr, (int*)nullptr, (const int*)nullptr, (int*)nullptr, n, 0,
      32);
  return e == hipSuccess ? bytes : (size_t)n * 16 + (1 << 20);
}

static size_t list_ws_layout(int n, ListWs* ws, char* base) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += align_up(bytes);
    return p;
  };
  char* p_fl = take((size_t)n * sizeof(int));
  char* p_rk = take((size_t)(n + 1) * sizeof(int));
  char* p_ct = take((size_t)(n + 1) * sizeof(int));
  char* p_io = take((size_t)n * sizeof(int));
  char* p_ko = take((size_t)n * sizeof(int));
  char* p_sc = take(scan_workspace_bytes(n + 1));
  const size_t sb = sort_temp_bytes(n);
  char* p_so = take(sb);
  if (ws) {
    ws->flag = (int*)p_fl;
    ws->rank = (int*)p_rk;
    ws->count = (int*)p_ct;
    ws->iota = (int*)p_io;
    ws->keys_out = (int*)p_ko;
    ws->scan_ws = p_sc;
    ws->sort_ws = p_so;
    ws->sort_bytes = sb;
  }
  return off;
}

}  // namespace prop
}  // namespace rg

using namespace rg;
using namespace rg::prop;

extern "C" int rg_proposal_centres(const float* offsets, int ld_off, const float* xy, int ld_xy,
                                   int n_nodes, float mu_x, float mu_y, float sigma_x,
                                   float sigma_y, float* cx, float* cy, void* stream) {
  RG_REQUIRE(n_nodes >= 0 && ld_off >= 2 && ld_xy >= 2, RG_ERR_ARG, "rg_proposal_centres: sizes");
  if (n_nodes == 0) return RG_OK;
  centres_kernel<<<ceil_div(n_nodes, 256), 256, 0, (hipStream_t)stream>>>(
      offsets, ld_off, xy, ld_xy, n_nodes, mu_x, mu_y, sigma_x, sigma_y, cx, cy);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_cluster_lists_workspace_size(int n_nodes) {
  return list_ws_layout(n_nodes, nullptr, nullptr);
}

extern "C" int rg_cluster_lists(const int* labels, int n_nodes, int* cluster_of, int* cluster_ptr,
                                int* cluster_idx, int* n_clusters, void* workspace,
                                size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_nodes >= 0, RG_ERR_ARG, "rg_cluster_lists: n_nodes");
  if (n_nodes == 0) {
    RG_CHECK_HIP(hipMemsetAsync(n_clusters, 0, sizeof(int), st));
    RG_CHECK_HIP(hipMemsetAsync(cluster_ptr, 0, sizeof(int), st));
    return RG_OK;
  }
  ListWs ws;
  const size_t need = list_ws_layout(n_nodes, &ws, (char*)workspace);
  RG_REQUIRE(workspace_bytes >= need, RG_ERR_ARG, "rg_cluster_lists: workspace %zu < %zu",
             workspace_bytes, need);
  root_flags<<<ceil_div(n_nodes, 256), 256, 0, st>>>(labels, n_nodes, ws.flag);
  int rc = exclusive_scan(ws.flag, n_nodes, ws.rank, n_clusters, ws.scan_ws, st);
  if (rc) return rc;
  RG_CHECK_HIP(hipMemsetAsync(ws.count, 0, (size_t)(n_nodes + 1) * sizeof(int), st));
  cluster_ids<<<ceil_div(n_nodes, 256), 256, 0, st>>>(labels, ws.rank, n_nodes, cluster_of,
                                                      ws.count, ws.iota);
  RG_LAUNCH_CHECK();
  // cluster_ptr = exclusive scan of the member counts (clusters beyond n_clusters are empty)
  rc = exclusive_scan(ws.count, n_nodes + 1, cluster_ptr, nullptr, ws.scan_ws, st);
  if (rc) return rc;
  // members grouped by cluster, ascending inside each: a stable radix sort of the node
  // indices (already ascending) keyed by cluster id
  int bits = 1;
  while ((1 << bits) < n_nodes + 1 && bits < 31) ++bits;
  size_t sb = ws.sort_bytes;
  RG_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(ws.sort_ws, sb, cluster_of, ws.keys_out,
                                                  ws.iota, cluster_idx, n_nodes, 0, bits, st));
  return RG_OK;
}
