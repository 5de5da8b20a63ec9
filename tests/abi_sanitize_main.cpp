// Host-side sanitizer driver for the C ABI (include/radar_gnn.h), run by
// tests/test_native_lib.py::test_abi_host_code_under_asan_ubsan on the CPU.
//
// The library's host code (argument checks, workspace-size arithmetic, launch set-up) is
// compiled with -fsanitize=address,undefined (host side only: -Xarch_host; device code is
// untouched) and linked into this executable.  It calls every *_workspace_size / *_bytes
// query at the sizes of the BASELINE configurations (M: 64 x 3000 nodes, 2.42 M edges; C3: 64 x
// 3000 nodes, 7.28 M edges; C5: 20 000 nodes, 400 k edges) and past them, and the
// null / negative / too-small-workspace / unsupported-shape paths of the entry points, which
// must return an RG_ERR_* code with a message before touching any device memory.  No GPU is
// needed: nothing here reaches a kernel launch.  Any sanitizer report fails the test (the
// runtime aborts with a nonzero exit status), as does a failed CHECK.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "radar_gnn.h"

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

// an entry point rejected its arguments: an error code and a message
static void expect_error(int rc, const char* what) {
  const char* msg = rg_last_error();
  if (rc == RG_OK || !msg || !msg[0]) {
    std::fprintf(stderr, "%s: expected an error, got rc %d (%s)\n", what, rc, msg ? msg : "null");
    ++g_fail;
  }
}

struct Size {
  const char* name;
  int nodes, frames, frame_nodes, k;
  long edges;
};

int main() {
  CHECK(rg_version() >= 1);
  const Size sizes[] = {
      {"one node", 1, 1, 1, 1, 0},
      {"small", 300, 1, 300, 10, 3600},
      {"M", 64 * 3000, 64, 3000, 10, 2422792},
      {"C3", 64 * 3000, 64, 3000, 32, 7284502},
      {"C5", 20000, 1, 20000, 10, 398000},
      {"C5b", 8 * 20000, 8, 20000, 10, 3184000},
      {"large", 1 << 22, 512, 8192, 32, 1L << 28},
  };
  for (const Size& s : sizes) {
    for (int mode = RG_GRAPH_KNN; mode <= RG_GRAPH_KNN_RADIUS; ++mode) {
      const size_t b = rg_build_graph_workspace_size(s.nodes, s.frames, s.frame_nodes, s.k, mode);
      CHECK(b >= (size_t)s.nodes * sizeof(int));
    }
    const size_t x3 = rg_conv_layer_x3_workspace_size(s.nodes);
    CHECK(x3 >= (size_t)s.nodes * 64 * sizeof(float));
    // the edge launch's wave table: one node boundary per wave + the end (a fixed size)
    CHECK(rg_conv_x3_blocks_bytes(s.nodes) >= 2 * sizeof(int));
    CHECK(rg_conv_layer_f32_workspace_size(s.nodes) > 0);
    CHECK(rg_conv_blocks_workspace_size(s.nodes) > 0);
    CHECK(rg_csr_by_dst_workspace_size(s.nodes, s.edges) > 0);
    CHECK(rg_pairs_from_edge_index_workspace_size(s.edges) > 0 || s.edges == 0);
    CHECK(rg_dense_pair_rows_workspace_size(s.nodes) > 0);
    CHECK(rg_link_pairs_workspace_size(s.nodes) > 0);
    CHECK(rg_frame_norm_workspace_size(s.nodes, 4) > 0);
    CHECK(rg_frame_norm_backward_workspace_size(s.nodes, 4) > 0);
    (void)rg_segment_reduce_ranges_workspace_size(s.edges, 64, RG_F32);
    CHECK(rg_object_graph_workspace_size(s.nodes / 8 + 1) > 0);
    CHECK(rg_frontend_labels_workspace_size(s.nodes / 16 + 1) > 0);
    CHECK(rg_frontend_select_workspace_size(s.nodes) > 0);
    CHECK(rg_cluster_radius_workspace_size(s.nodes, s.frames, s.frame_nodes) > 0);
    CHECK(rg_cluster_lists_workspace_size(s.nodes) > 0);
    CHECK(rg_linear_grad_workspace_size(s.edges, 64, 192) > 0 || s.edges == 0);
    CHECK(rg_incidence_workspace_size(s.nodes, s.edges) > 0);
    CHECK(rg_loss_workspace_size(s.nodes, s.edges / 2, s.nodes / 10) > 0);
  }
  (void)rg_conv_layer_workspace_size();
  (void)rg_segment_order_workspace_size();
  (void)rg_ffn_backward_workspace_size();
  // packed sizes of every layer shape of the yml architecture, every format
  const int shapes[][2] = {{7, 256}, {256, 128}, {128, 128}, {128, 64}, {6, 256},
                           {192, 128}, {128, 64},  {64, 256},  {64, 7},   {1, 1}};
  const int fmts[] = {RG_F32, RG_BF16, RG_PACK_FAST_IN, RG_PACK_FAST_CHAIN, RG_PACK_F32_FAST,
                      RG_PACK_FAST_IN | RG_PACK_X3, RG_PACK_FAST_CHAIN | RG_PACK_X3,
                      RG_PACK_FAST_IN | RG_PACK_F16};
  for (const auto& sh : shapes)
    for (int f : fmts) CHECK(rg_packed_linear_bytes(sh[0], sh[1], f) > 0);

  // ---- argument errors, caught before any device access
  expect_error(rg_build_graph(nullptr, nullptr, nullptr, 3000, 1, 3000, 10, 25.f, RG_GRAPH_KNN,
                              nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr),
               "rg_build_graph workspace too small");
  expect_error(rg_build_graph(nullptr, nullptr, nullptr, 10, 1, 10, 100, 25.f, RG_GRAPH_KNN,
                              nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr),
               "rg_build_graph k > frame size");
  rg_layer none[1];
  std::memset(none, 0, sizeof(none));
  expect_error(rg_mlp_chain(RG_F32, none, 0, 10, nullptr, RG_IN_DENSE, RG_F32, nullptr, 0, 0,
                            nullptr, 0, 0, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, 0, nullptr,
                            0, 0, nullptr),
               "rg_mlp_chain n_layers 0");
  expect_error(rg_mlp_chain(RG_F32, none, RG_MAX_LAYERS + 1, 10, nullptr, RG_IN_DENSE, RG_F32,
                            nullptr, 0, 0, nullptr, 0, 0, nullptr, 0, 0, nullptr, nullptr, nullptr,
                            0, 0, nullptr, 0, 0, nullptr),
               "rg_mlp_chain too many layers");
  rg_layer big[1];
  std::memset(big, 0, sizeof(big));
  big[0].w_packed = (const void*)16;
  big[0].in_dim = 300;
  big[0].out_dim = 8;
  expect_error(rg_mlp_chain(RG_F32, big, 1, 10, nullptr, RG_IN_DENSE, RG_F32, (const void*)16,
                            300, 300, nullptr, 0, 0, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, 0,
                            (void*)16, 8, 0, nullptr),
               "rg_mlp_chain width > 256");
  // the fp32 conv layer: wrong widths, wrong aggregation, aliasing, short workspace
  rg_layer conv[3];
  std::memset(conv, 0, sizeof(conv));
  const float one = 1.f;
  const int dims[3][2] = {{64, 128}, {128, 64}, {128, 64}};
  for (int l = 0; l < 3; ++l) {
    conv[l].w_packed = (const void*)64;
    conv[l].norm_mu = &one;
    conv[l].norm_std = &one;
    conv[l].in_dim = dims[l][0];
    conv[l].out_dim = dims[l][1];
    conv[l].act = RG_ACT_LEAKY;
  }
  float* fake = (float*)(size_t)256;
  expect_error(rg_conv_layer_x3(conv, nullptr, RG_REDUCE_MAX, fake, 64, fake, 64, fake, nullptr,
                                nullptr, nullptr, 100, fake + 64, 64, nullptr, fake, 1 << 20,
                                nullptr),
               "rg_conv_layer_x3 max aggregation");
  expect_error(rg_conv_layer_x3(conv, nullptr, RG_REDUCE_SUM, fake, 64, fake, 64, fake, nullptr,
                                nullptr, nullptr, 100, fake, 64, nullptr, fake, 1 << 20, nullptr),
               "rg_conv_layer_x3 x_out aliases x");
  expect_error(rg_conv_layer_x3(conv, nullptr, RG_REDUCE_SUM, fake, 64, fake, 64, fake, nullptr,
                                nullptr, nullptr, 64 * 3000, fake + 64, 64, nullptr, fake, 16,
                                nullptr),
               "rg_conv_layer_x3 workspace too small");
  expect_error(rg_conv_layer_x3(conv, nullptr, RG_REDUCE_SUM, fake, 66, fake, 64, fake, nullptr,
                                nullptr, nullptr, 100, fake + 64, 64, nullptr, fake, 1 << 20,
                                nullptr),
               "rg_conv_layer_x3 unaligned row stride");
  expect_error(rg_conv_layer_x3(conv, conv, RG_REDUCE_SUM, fake, 64, fake, 64, fake, nullptr,
                                nullptr, nullptr, 100, fake + 64, 64, nullptr, fake, 1 << 20,
                                nullptr),
               "rg_conv_layer_x3 next_pq without pq_out");
  conv[1].out_dim = 32;
  expect_error(rg_conv_layer_x3(conv, nullptr, RG_REDUCE_SUM, fake, 64, fake, 64, fake, nullptr,
                                nullptr, nullptr, 100, fake + 64, 64, nullptr, fake, 1 << 20,
                                nullptr),
               "rg_conv_layer_x3 unsupported widths");
  conv[1].out_dim = 64;
  expect_error(rg_conv_x3_blocks(nullptr, 100, nullptr, nullptr), "rg_conv_x3_blocks null table");
  // RANSAC: null lists, iteration count out of range
  expect_error(rg_frontend_gate_lists(nullptr, nullptr, 4, nullptr, nullptr, nullptr),
               "rg_frontend_gate_lists null arguments");
  expect_error(rg_frontend_ransac(fake, fake, (const int*)fake, 4, (const int*)fake,
                                  (const int*)fake, (const int*)fake, 0, 2, 0.25, 10, 0.6,
                                  (uint8_t*)fake, (double*)fake, (uint8_t*)fake, nullptr),
               "rg_frontend_ransac zero iterations");
  expect_error(rg_frontend_ransac(fake, fake, (const int*)fake, 4, (const int*)fake,
                                  (const int*)fake, (const int*)fake, 30, 2, 0.25, 10, 0.6,
                                  nullptr, nullptr, nullptr, nullptr),
               "rg_frontend_ransac null outputs");
  expect_error(rg_ransac_consensus_sets(nullptr, nullptr, nullptr, 4, 30, 2, 10, nullptr),
               "rg_ransac_consensus_sets null arguments");
  {  // a draw over a real state: 3 scans, the middle one below the minimum
    uint32_t key[624];
    for (int i = 0; i < 624; ++i) key[i] = 0x9e3779b9u * (uint32_t)(i + 1);
    int pos = 624, cnt[3] = {40, 7, 13}, sets[3 * 30 * 2];
    CHECK(rg_ransac_consensus_sets(key, &pos, cnt, 3, 30, 2, 10, sets) == RG_OK);
    for (int i = 0; i < 3 * 30 * 2; ++i) CHECK(sets[i] >= 0 && sets[i] < 40);
    CHECK(pos >= 0 && pos <= 624);
  }
  expect_error(rg_conv_layer_x3_blocks(conv, nullptr, RG_REDUCE_SUM, fake, 64, fake, 64, fake,
                                       nullptr, nullptr, nullptr, 100, fake + 64, 64, nullptr,
                                       nullptr, fake, 1 << 20, nullptr),
               "rg_conv_layer_x3_blocks without a table");
  expect_error(rg_segment_reduce(nullptr, RG_F32, 6, nullptr, nullptr, 4, 6, RG_REDUCE_SUM,
                                 nullptr, RG_F32, 6, nullptr),
               "rg_segment_reduce width 6");
  expect_error(rg_segment_reduce_sched(nullptr, RG_F32, 64, nullptr, nullptr, 4, 64,
                                       RG_REDUCE_SUM, nullptr, RG_F32, 64, 3, 5, 0, nullptr),
               "rg_segment_reduce_sched schedule not compiled");
  return g_fail ? 1 : 0;
}
