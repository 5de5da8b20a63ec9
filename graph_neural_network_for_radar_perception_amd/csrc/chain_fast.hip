// Register-resident bf16 MLP chains for the shapes of the shipped architecture.
//
// Same semantics as rg_mlp_chain (ffn_block chains: Linear -> channel_normalization
// -> activation, common.py:185-220, gnn_blocks.py:19-389) but every width is a
// compile-time constant, so the whole chain is unrolled:
//
//  * one wave = 32 rows; v_mfma_f32_32x32x16_bf16 computes Y^T = W . X^T, so lane
//    (r = lane&31, h = lane>>5) holds row r's features {32m + 8(q>>2) + 4h + (q&3)}
//    in accumulator register q of M-tile m;
//  * channel_normalization statistics = in-lane sum + ONE xor-32 exchange;
//  * a layer's accumulators become the next layer's B operand IN REGISTERS
//    (registers 8s'..8s'+7 of a tile, packed to bf16, are k-step s'; the next
//    layer's weights are packed with that k permutation, rg_pack_linear format
//    RG_PACK_FAST_CHAIN), so activations never touch LDS or HBM between layers;
//  * the first layer's B fragments are loaded straight from HBM/L2 into
//    registers: dense rows, concatenations (update MLP, gnn_blocks.py:108), the
//    gathered cat(x_i, x_j, e) of MessagePassing.message (gnn_blocks.py:113) or the
//    pair sum x_i + x_j of edge_formation (gnn_blocks.py:297);
//  * every layer's packed weights + bias live in LDS for the whole (persistent)
//    workgroup: 8 waves, two per SIMD, share them; one 1-KiB ds_read_b128 feeds a
//    32-cycle MFMA.
#include "rg_common.h"

#define RG_HALF_F16 0
#define RG_HALF_CODE RG_BF16
#define RG_FAST_NS fast
#include "chain_fast_impl.h"
#undef RG_HALF_F16
#undef RG_HALF_CODE
#undef RG_FAST_NS
#define RG_HALF_F16 1
#define RG_HALF_CODE RG_F16
#define RG_FAST_NS fast_f16
#include "chain_fast_impl.h"
#undef RG_HALF_F16
#undef RG_HALF_CODE
#undef RG_FAST_NS

// bf16 or fp16 operands by the packed weights (RG_LAYER_F16: rg_pack_linear with RG_PACK_F16)
extern "C" int rg_mlp_chain_fast(const rg_layer* layers, int n_layers, long rows,
                                 const int* rows_dev, int in_mode, int in_dtype, const void* in0,
                                 int ld0, int w0, const void* in1, int ld1, int w1,
                                 const void* in2, int ld2, int w2, const int* idx0,
                                 const int* idx1, const void* residual, int ld_res, int res_dtype,
                                 void* out, int ld_out, int out_dtype, void* stream) {
  RG_REQUIRE(n_layers >= 1 && layers, RG_ERR_ARG, "rg_mlp_chain_fast: layers");
  const bool f16 = (layers[0].flags & RG_LAYER_F16) != 0;
  for (int l = 1; l < n_layers; ++l)
    RG_REQUIRE(((layers[l].flags & RG_LAYER_F16) != 0) == f16, RG_ERR_ARG,
               "rg_mlp_chain_fast: every layer packed with the same 16-bit type");
  auto fn = f16 ? rg::fast_f16::chain_fast_entry : rg::fast::chain_fast_entry;
  return fn(layers, n_layers, rows, rows_dev, in_mode, in_dtype, in0, ld0, w0, in1, ld1, w1, in2, ld2,
            w2, idx0, idx1, residual, ld_res, res_dtype, out, ld_out, out_dtype, stream);
}
