// Fused residual_graph_conv_block (gnn_blocks.py:96-113) for the shipped widths
// (C = 64 node / edge channels, msg MLP 192 -> 128 -> 64, update 128 -> 64, aggr add
// or mean), bf16 operands, f32 accumulation.  One launch per layer replaces
// message chain + scatter-aggregate + update chain; messages and aggregates never
// touch HBM.
//
// Work unit = a block of 8 destination nodes and all their incoming edges (the
// destination-major CSR makes them one contiguous edge range).  A wave
//   0. computes P[node] = W1[:, :C] x[node] + b1 for the block's nodes (the x_i = x[dst]
//      third of the first message layer is shared by all edges into a node) into LDS;
//   1. streams the block's edges in tiles of 32: accumulators start from P[dst], the
//      x[src] and e rows go straight into MFMA B fragments for the remaining 2/3 of
//      the first layer, then the rest of the message MLP (32x32x16 MFMAs,
//      channel_normalization + LeakyReLU in-lane, layers chained in registers)
//      -> message tile M [64 features x 32 edges], lane = edge;
//   2. transposes M through a wave-private, XOR-swizzled LDS tile (8-B row stores,
//      hardware transposed reads ds_read_b64_tr_b16, both bank-conflict free) and
//      accumulates Agg[64 x 8 nodes] += M . S with S the one-hot (edge -> destination slot)
//      matrix: the segmented scatter-add as 4 MFMAs per tile, summed in edge order
//      with f32 accumulation (sources ascending within a destination = the
//      reference scatter_add_ order; bf16-rounded messages as in the unfused path);
//   3. after the block's last tile: Agg (lane = node) is already the B operand of
//      the update MLP (k-steps 4..7); x[node] provides k-steps 0..3; update +
//      norm + act + residual, store x_new[node].
// Workgroups (8 waves, 2 per SIMD) are persistent and pull node blocks from an
// atomic counter; all weights (81 KiB packed bf16 + biases) sit in LDS.
#include "rg_common.h"
#include "scan.h"

#define RG_HALF_F16 0
#define RG_CONV_NS conv
#include "conv_fused_impl.h"
#undef RG_HALF_F16
#undef RG_CONV_NS
#define RG_HALF_F16 1
#define RG_CONV_NS conv_f16
#include "conv_fused_impl.h"
#undef RG_HALF_F16
#undef RG_CONV_NS


using namespace rg;
using namespace rg::conv;

// Each XCD's share of the blocks (the fused kernel's ranges [n*x/NQ, n*(x+1)/NQ) of the
// dequeue order) sorted by tile count, largest first: the waves then finish on the
// smallest blocks (greedy longest-first), instead of on whatever blocks come last in node
// order -- a 20 000-node frame is only ~2.3 blocks of 1-4 tiles per wave, and its launch
// tail (waves idle until the last block ends) was a third of the wave time.  Order within
// a size class is arbitrary: every node's result is independent of the schedule.
__global__ __launch_bounds__(256) void conv_blocks_lpt(const int* __restrict__ bounds,
                                                       const int* __restrict__ seg_ptr,
                                                       const int* __restrict__ n_blocks_dev,
                                                       int* __restrict__ pairs) {
  constexpr int NBIN = 64;
  __shared__ int hist[NBIN];
  const int nb = *n_blocks_dev;
  const int lo = (int)((long)nb * blockIdx.x / NQ), hi = (int)((long)nb * (blockIdx.x + 1) / NQ);
  if (threadIdx.x < NBIN) hist[threadIdx.x] = 0;
  __syncthreads();
  auto bin = [&](int b) {  // bin 0 = the most tiles
    const int t = (seg_ptr[bounds[b + 1]] - seg_ptr[bounds[b]] + 31) / 32;
    return NBIN - 1 - min(t, NBIN - 1);
  };
  for (int b = lo + threadIdx.x; b < hi; b += blockDim.x) atomicAdd(&hist[bin(b)], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NBIN; ++i) {
      const int c = hist[i];
      hist[i] = acc;
      acc += c;
    }
  }
  __syncthreads();
  for (int b = lo + threadIdx.x; b < hi; b += blockDim.x) {
    const int pos = lo + atomicAdd(&hist[bin(b)], 1);
    pairs[2 * pos] = bounds[b];
    pairs[2 * pos + 1] = bounds[b + 1];
  }
}

extern "C" size_t rg_conv_blocks_workspace_size(int n_nodes) {
  const long nb8 = ((long)n_nodes + NB - 1) / NB;
  return 2 * ((size_t)((nb8 + 1) * sizeof(int) + 255) / 256 * 256) +
         ((size_t)((n_nodes + 1) * sizeof(int)) + 255) / 256 * 256 + scan_workspace_bytes(nb8);
}

extern "C" int rg_conv_blocks(const int* seg_ptr, int n_nodes, int* blk_nodes, int* n_blocks,
                              void* workspace, size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_nodes >= 1, RG_ERR_ARG, "rg_conv_blocks: n_nodes must be >= 1");
  RG_REQUIRE(workspace_bytes >= rg_conv_blocks_workspace_size(n_nodes), RG_ERR_ARG,
             "rg_conv_blocks: workspace too small");
  const int nb8 = (n_nodes + NB - 1) / NB;
  const size_t arr = ((size_t)(nb8 + 1) * sizeof(int) + 255) / 256 * 256;
  int* cnt = (int*)workspace;                 // sub-blocks per 8-node run
  int* off = (int*)((char*)workspace + arr);  // their exclusive scan
  int* bounds = (int*)((char*)workspace + 2 * arr);  // block boundaries in node order
  void* sws = (char*)workspace + 2 * arr + ((size_t)((n_nodes + 1) * sizeof(int)) + 255) / 256 * 256;
  // block edge cap max(cap_min, E / cap_div): a same-box sweep (scripts/experiments/
  // gpu_c5_cap.sh) put C5's conv at 0.055 ms here and at min 64; 0.061 at E / 2048, at min
  // 256 and at (64, E / 8192); 0.080 at 32-edge blocks
  constexpr int cap_min = CAP_MIN, cap_div = 4096;
  conv_blocks_kernel<false><<<(nb8 + 255) / 256, 256, 0, st>>>(seg_ptr, n_nodes, cnt, nullptr,
                                                                nullptr, cap_min, cap_div);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(cnt, nb8, off, n_blocks, sws, st);
  if (rc) return rc;
  conv_blocks_kernel<true><<<(nb8 + 255) / 256, 256, 0, st>>>(seg_ptr, n_nodes, nullptr, off,
                                                               bounds, cap_min, cap_div);
  RG_LAUNCH_CHECK();
  conv_blocks_lpt<<<NQ, 256, 0, st>>>(bounds, seg_ptr, n_blocks, blk_nodes);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

static_assert((rg::conv::CTR_STRIDE * rg::conv::NQ + 1) * sizeof(int) <= 2048, "conv workspace");
extern "C" size_t rg_conv_layer_workspace_size(void) { return 2048; }

extern "C" int rg_conv_layer_fused_blocks(const rg_layer* msg_layers, const rg_layer* upd_layer,
                                          int aggr, const void* x, int ldx, const void* e,
                                          int lde, const int* seg_ptr, const int* src,
                                          const int* dst, int n_nodes, void* x_out, int ld_out,
                                          const int* blk_nodes, const int* n_blocks_dev,
                                          void* workspace, void* stream) {
  // bf16 or fp16 operands by the packed weights (RG_LAYER_F16: rg_pack_linear with RG_PACK_F16)
  const int f16 = msg_layers[0].flags & msg_layers[1].flags & upd_layer->flags & RG_LAYER_F16;
  RG_REQUIRE(f16 || !((msg_layers[0].flags | msg_layers[1].flags | upd_layer->flags) & RG_LAYER_F16),
             RG_ERR_ARG, "rg_conv_layer_fused: every layer packed with the same 16-bit type");
  auto fn = f16 ? rg::conv_f16::conv_fused_entry : rg::conv::conv_fused_entry;
  return fn(msg_layers, upd_layer, aggr, x, ldx, e, lde, seg_ptr, src, dst, n_nodes, x_out, ld_out,
            blk_nodes, n_blocks_dev, nullptr, 0, workspace, stream);
}

extern "C" int rg_conv_wave_nodes(const int* seg_ptr, int n_nodes, int n_waves, int* wave_nodes,
                                  void* stream) {
  RG_REQUIRE(seg_ptr && wave_nodes && n_nodes >= 1 && n_waves >= 1, RG_ERR_ARG,
             "rg_conv_wave_nodes: bad argument");
  constexpr int cost = rg::conv::WAVE_NODE_COST;  // (4, 7 or 10 edge units: same within noise)
  conv_wave_nodes_kernel<<<(n_waves + 1 + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      seg_ptr, n_nodes, n_waves, cost, wave_nodes);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_conv_layer_fused_waves(const rg_layer* msg_layers, const rg_layer* upd_layer,
                                         int aggr, const void* x, int ldx, const void* e, int lde,
                                         const int* seg_ptr, const int* src, const int* dst,
                                         int n_nodes, void* x_out, int ld_out,
                                         const int* wave_nodes, int n_waves, void* workspace,
                                         void* stream) {
  RG_REQUIRE(wave_nodes, RG_ERR_ARG, "rg_conv_layer_fused_waves: wave_nodes from rg_conv_wave_nodes");
  const int f16 = msg_layers[0].flags & msg_layers[1].flags & upd_layer->flags & RG_LAYER_F16;
  RG_REQUIRE(f16 || !((msg_layers[0].flags | msg_layers[1].flags | upd_layer->flags) & RG_LAYER_F16),
             RG_ERR_ARG, "rg_conv_layer_fused: every layer packed with the same 16-bit type");
  auto fn = f16 ? rg::conv_f16::conv_fused_entry : rg::conv::conv_fused_entry;
  return fn(msg_layers, upd_layer, aggr, x, ldx, e, lde, seg_ptr, src, dst, n_nodes, x_out, ld_out,
            nullptr, nullptr, wave_nodes, n_waves, workspace, stream);
}

extern "C" int rg_conv_layer_fused(const rg_layer* msg_layers, const rg_layer* upd_layer, int aggr,
                                   const void* x, int ldx, const void* e, int lde,
                                   const int* seg_ptr, const int* src, const int* dst,
                                   int n_nodes, void* x_out, int ld_out, void* workspace,
                                   void* stream) {
  return rg_conv_layer_fused_blocks(msg_layers, upd_layer, aggr, x, ldx, e, lde, seg_ptr, src,
                                    dst, n_nodes, x_out, ld_out, nullptr, nullptr, workspace,
                                    stream);
}

#if RG_CONV_STAMP
// diagnostic build only (not in radar_gnn.h): read and reset the per-phase stamp sums
extern "C" int rg_debug_conv_stamps(int f16, unsigned long long* out_host) {
  return f16 ? rg::conv_f16::conv_stamps(out_host) : rg::conv::conv_stamps(out_host);
}
#endif
