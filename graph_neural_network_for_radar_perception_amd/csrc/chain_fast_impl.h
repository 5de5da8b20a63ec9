// Register-resident 16-bit MLP chains: the body of chain_fast.hip, compiled once per
// operand type (RG_HALF_F16 = 0: bf16 in namespace rg::fast; 1: IEEE fp16 in rg::fast_f16).
// No include guard: chain_fast.hip includes it twice.
namespace rg {
namespace RG_FAST_NS {

using HT = ::rg::H16<RG_HALF_F16 != 0>;  // the 16-bit operand type (bf16 / fp16)

typedef HT::v8 bf16x8_t;  // (named for the bf16 build; fp16 lanes in the fp16 build)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Workgroup size is per shape: 512 threads (2 waves per SIMD) for register-heavy
// chains, 768 / 1024 (3 / 4 per SIMD) where the chain fits 170 / 128 VGPRs -- one
// workgroup per CU shares one LDS copy of the weights, so more waves per workgroup is
// the only way to more latency hiding.
static constexpr float NORM_EPS = 1e-5f;
#ifndef RG_PAIR_SPLIT
#define RG_PAIR_SPLIT 1  // PAIRADD chains: the MFMAs add the pair (see Input::PAIR_SPLIT)
#endif
static constexpr int FUSE01 = 0x100;  // kernel MODE flag: run_chain01 for layers 0+1

// the chains' MFMA (bf16 or fp16 by HT)
__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return HT::mfma(a, b, c);
}

struct FLayer {
  const void* src;  // packed weights (+bias) in global memory
  const float* mu;
  const float* sd;
  int woff;   // byte offset of the layer in the LDS image
  int bytes;  // packed bytes
  int out;    // real output width
  int act;
  int centered;  // RG_LAYER_CENTERED
};

struct FArgs {
  FLayer L[RG_MAX_LAYERS];
  int nl;
  int total_bytes;
  long rows;
  const int* rows_dev;
  const void* in0;
  const void* in1;
  const void* in2;
  int ld0, ld1, ld2;
  int in_f32;   // in0 is float32 (DENSE only)
  int w0real;   // real width of a float32 DENSE input
  const int* idx0;
  const int* idx1;
  const void* res;
  int ld_res, res_f32;
  void* out;
  int ld_out, out_f32, out_real;
  int out_vec;  // row stride allows 4-wide vector stores
};

__device__ __forceinline__ uint32_t bf2(float a, float b) { return HT::pack2(a, b); }

__device__ __forceinline__ bf16x8_t ld_bf8(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *(const u32x4*)p);
}

__device__ __forceinline__ bf16x8_t zero_bf8() {
  return __builtin_bit_cast(bf16x8_t, (u32x4){0u, 0u, 0u, 0u});
}

// x_i + x_j of two bf16x8 rows, added in f32 and rounded once
__device__ __forceinline__ bf16x8_t add_bf8(bf16x8_t a, bf16x8_t b) {
  const u32x4 ua = __builtin_bit_cast(u32x4, a), ub = __builtin_bit_cast(u32x4, b);
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a0 = HT::lo(ua[i]), a1 = HT::hi(ua[i]);
    const float b0 = HT::lo(ub[i]), b1 = HT::hi(ub[i]);
    o[i] = bf2(__fadd_rn(a0, b0), __fadd_rn(a1, b1));
  }
  return __builtin_bit_cast(bf16x8_t, o);
}

// ----------------------------------------------------------------- layer-0 operands
// k-step s, lane half h: features [16s + 8h, 16s + 8h + 8) of the row's input vector
template <int MODE, bool IN_F32, int W0, int W1>
struct Input {
  static constexpr int K0 = MODE == RG_IN_GATHER3 ? 2 * W0 + W1
                          : (MODE == RG_IN_CONCAT2 ? W0 + W1 : W0);
  static constexpr int KS = (K0 + 15) / 16;
  // B fragments handed to layer 0: PAIRADD keeps x[i] and x[j] apart (KS each) and lets
  // the MFMAs add them, W (x_i + x_j) = W x_i + W x_j, instead of ~28 VALU per fragment
  // to unpack, add and repack the pair in bf16 (the chain is VALU-bound)
  static constexpr bool PAIR_SPLIT = MODE == RG_IN_PAIRADD && RG_PAIR_SPLIT;
  static constexpr int KSB = PAIR_SPLIT ? 2 * KS : KS;

  static __device__ __forceinline__ void load(const FArgs& a, long row, bool valid, int h,
                                              bf16x8_t (&b)[KSB], float pre = 1.f) {
    if (!valid) {
#pragma unroll
      for (int s = 0; s < KSB; ++s) b[s] = zero_bf8();
      return;
    }
    if constexpr (MODE == RG_IN_DENSE && IN_F32) {
      const float* p = (const float*)a.in0 + (size_t)row * a.ld0;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int f = 16 * s + 8 * h + j;
          v[j] = f < a.w0real ? p[f] * pre : 0.f;
        }
        b[s] = __builtin_bit_cast(bf16x8_t, (u32x4){bf2(v[0], v[1]), bf2(v[2], v[3]),
                                                    bf2(v[4], v[5]), bf2(v[6], v[7])});
      }
    } else if constexpr (MODE == RG_IN_DENSE) {
      static_assert(W0 % 16 == 0, "bf16 dense input width must be a multiple of 16");
      const uint16_t* p = (const uint16_t*)a.in0 + (size_t)row * a.ld0 + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) b[s] = ld_bf8(p + 16 * s);
    } else if constexpr (MODE == RG_IN_CONCAT2) {
      static_assert(W0 % 16 == 0 && W1 % 16 == 0, "concat widths must be multiples of 16");
      const uint16_t* p0 = (const uint16_t*)a.in0 + (size_t)row * a.ld0 + 8 * h;
      const uint16_t* p1 = (const uint16_t*)a.in1 + (size_t)row * a.ld1 + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        b[s] = s < W0 / 16 ? ld_bf8(p0 + 16 * s) : ld_bf8(p1 + 16 * (s - W0 / 16));
    } else if constexpr (MODE == RG_IN_GATHER3) {
      static_assert(W0 % 16 == 0 && W1 % 16 == 0, "gather widths must be multiples of 16");
      const int ri = a.idx0[row], rj = a.idx1[row];
      const uint16_t* pi = (const uint16_t*)a.in0 + (size_t)ri * a.ld0 + 8 * h;
      const uint16_t* pj = (const uint16_t*)a.in0 + (size_t)rj * a.ld0 + 8 * h;
      const uint16_t* pe = (const uint16_t*)a.in2 + (size_t)row * a.ld2 + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (s < W0 / 16) b[s] = ld_bf8(pi + 16 * s);
        else if (s < 2 * W0 / 16) b[s] = ld_bf8(pj + 16 * (s - W0 / 16));
        else b[s] = ld_bf8(pe + 16 * (s - 2 * W0 / 16));
      }
    } else {  // RG_IN_PAIRADD
      static_assert(W0 % 16 == 0, "pair width must be a multiple of 16");
      const int ri = a.idx0[row], rj = a.idx1[row];
      const uint16_t* pi = (const uint16_t*)a.in0 + (size_t)ri * a.ld0 + 8 * h;
      const uint16_t* pj = (const uint16_t*)a.in0 + (size_t)rj * a.ld0 + 8 * h;
      if constexpr (PAIR_SPLIT) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          b[s] = ld_bf8(pi + 16 * s);
          b[KS + s] = ld_bf8(pj + 16 * s);
        }
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) b[s] = add_bf8(ld_bf8(pi + 16 * s), ld_bf8(pj + 16 * s));
      }
    }
  }
};

// ----------------------------------------------------------------- one layer
template <int KS, int MT>
__device__ __forceinline__ void mfma_layer(const bf16x8_t (&b)[KS], f32x16 (&acc)[MT],
                                           const char* w, int lane) {
  const int h = lane >> 5;
  const float* bias = (const float*)(w + (size_t)MT * KS * 1024);
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    acc[m] = ld_bias_frag(bias, m, h);  // accumulator-order bias: 4 x ds_read_b128
  }
  // software pipeline: the A fragments of k-step s+1 are read from LDS while the
  // MFMAs of step s issue; a scheduling fence per step keeps the compiler from
  // hoisting every fragment of the layer (register blow-up)
  const char* wl = w + lane * 16;
  bf16x8_t acur[MT], anxt[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acur[m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KS) * 1024));
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + 1 < KS) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        anxt[m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KS + s + 1) * 1024));
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
      acc[m] = mfma32(acur[m], b[s], acc[m]);
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < KS) {
#pragma unroll
      for (int m = 0; m < MT; ++m) acur[m] = anxt[m];
    }
  }
}

// layer 0 of a split pair: REP x KS B fragments against the same KS weight k-steps
// (acc = bias + W b[0..KS) + W b[KS..2KS)), fragments of step s+1 read during step s
template <int KS, int MT, int REP>
__device__ __forceinline__ void mfma_layer_rep(const bf16x8_t (&b)[REP * KS], f32x16 (&acc)[MT],
                                               const char* w, int lane) {
  const int h = lane >> 5;
  const float* bias = (const float*)(w + (size_t)MT * KS * 1024);
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = ld_bias_frag(bias, m, h);
  const char* wl = w + lane * 16;
  bf16x8_t acur[MT], anxt[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acur[m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KS) * 1024));
#pragma unroll
  for (int s = 0; s < REP * KS; ++s) {
    if (s + 1 < REP * KS) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        anxt[m] = ld_bf8((const uint16_t*)(wl + (size_t)(m * KS + (s + 1) % KS) * 1024));
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma32(acur[m], b[s], acc[m]);
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < REP * KS) {
#pragma unroll
      for (int m = 0; m < MT; ++m) acur[m] = anxt[m];
    }
  }
}

// packed bytes of a fast-format Linear(K -> N): MT x KS fragments of 1 KiB + the
// bias padded to N (rg_packed_linear_bytes, mlp_chain.hip); layer images are
// 16-B aligned and back to back, so every LDS offset is a compile-time constant
__host__ __device__ constexpr int fast_bytes(int K, int N) {
  return (N / 32) * ((K + 15) / 16) * 1024 + N * 4;
}
template <int N, int... Rest> struct FirstOf { static constexpr int value = N; };
template <int K, int... Ns> struct Offsets;
template <int K> struct Offsets<K> {
  static constexpr int get(int) { return 0; }
};
template <int K, int N, int... Rest> struct Offsets<K, N, Rest...> {
  static constexpr int get(int l) {
    return l == 0 ? 0 : ((fast_bytes(K, N) + 15) & ~15) + Offsets<N, Rest...>::get(l - 1);
  }
};

// Padded output features (beyond L.out) need no masking: their weight rows and bias are
// packed as zeros, so they are exactly 0 before normalisation (normalised layers are
// never padded, checked on the host) and act(0) = 0; only the LAST layer may be padded
// and store_out never writes those columns.
//
// SPEC >= 0 fixes the chain's epilogues at compile time: bits 0-7 the hidden activation,
// bit 8 + l = layer l is normalised (and packed RG_PACK_CENTERED), bit 16 + l = layer l
// applies the activation (else identity) -- checked against the layer descriptors on
// the host.  SPEC < 0: the descriptors decide at run time.
constexpr int spec(int act, int norm_mask, int act_mask) {
  return act | (norm_mask << 8) | (act_mask << 16);
}
// nrm: the layers' channel_normalization (mu, sd) staged in LDS at kernel start
template <int SPEC, int LI, int MT>
__device__ __forceinline__ void epilogue(f32x16 (&acc)[MT], const FLayer& L, const float* nrm) {
  if constexpr (SPEC >= 0) {
    constexpr bool NORM = ((SPEC >> (8 + LI)) & 1) != 0, ACTV = ((SPEC >> (16 + LI)) & 1) != 0;
#ifndef RG_NO_FUSED_LEAKY
    if constexpr (NORM && ACTV && (SPEC & 0xff) == ACT_LEAKY) {  // centred: two fmas
      channel_norm_leaky_centered<MT>(acc, nrm[2 * LI], nrm[2 * LI + 1], NORM_EPS);
      return;
    }
#endif
    if constexpr (NORM)  // normalised => centred (host-checked)
      channel_norm_pk_centered<MT>(acc, nrm[2 * LI], nrm[2 * LI + 1], NORM_EPS);
    if constexpr (ACTV) act_pk_all<(SPEC & 0xff), MT>(acc);
  } else {
    norm_act_rows<-1, MT>(acc, L.mu != nullptr, nrm[2 * LI], nrm[2 * LI + 1], L.act, NORM_EPS,
                          L.centered != 0);
  }
}

template <int MT>
__device__ __forceinline__ void pack_next(const f32x16 (&acc)[MT], bf16x8_t (&nb)[2 * MT]) {
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int q = 8 * hf;
      nb[2 * m + hf] = __builtin_bit_cast(
          bf16x8_t, (u32x4){bf2(acc[m][q + 0], acc[m][q + 1]), bf2(acc[m][q + 2], acc[m][q + 3]),
                            bf2(acc[m][q + 4], acc[m][q + 5]), bf2(acc[m][q + 6], acc[m][q + 7])});
    }
}

// SPEC bit 30: the launch checked on the host that the output is bf16 with 4-wide
// vector rows, full width and no residual (the encoders' x and e), so the epilogue is
// plain packed stores -- no run-time branches or kernel arguments live across the tile
static constexpr int SPEC_PLAIN_OUT = 1 << 30;

#ifndef RG_FAST_ENC_BUF
#define RG_FAST_ENC_BUF 1  // plain outputs by branch-free buffer stores (a row past the end dropped
                           // by the hardware) and the encoders' next-tile rows loaded
                           // unconditionally, masked at use: the compiler counts these stores, so
                           // the loop-top wait for the prefetched rows does not also drain them
#endif

template <int MT, bool PLAIN = false>
__device__ __forceinline__ void store_out(const f32x16 (&acc)[MT], const FArgs& a, long row,
                                          int h) {
  if constexpr (PLAIN) {
    uint16_t* o = (uint16_t*)a.out + (size_t)row * a.ld_out;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 w;
        w.x = bf2(acc[m][4 * g], acc[m][4 * g + 1]);
        w.y = bf2(acc[m][4 * g + 2], acc[m][4 * g + 3]);
        *(uint2*)(o + 32 * m + 8 * g + 4 * h) = w;
      }
    return;
  }
  const int out = a.out_real;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * m + 8 * g + 4 * h;
      if (f0 >= out) continue;
      float v[4] = {acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2], acc[m][4 * g + 3]};
      if (f0 + 4 <= out && a.out_vec) {
        if (a.res) {
          if (a.res_f32) {
            const f32x4 r = *(const f32x4*)((const float*)a.res + (size_t)row * a.ld_res + f0);
            v[0] = __fadd_rn(r.x, v[0]); v[1] = __fadd_rn(r.y, v[1]);
            v[2] = __fadd_rn(r.z, v[2]); v[3] = __fadd_rn(r.w, v[3]);
          } else {
            const uint2 r = *(const uint2*)((const uint16_t*)a.res + (size_t)row * a.ld_res + f0);
            v[0] = __fadd_rn(HT::lo(r.x), v[0]);
            v[1] = __fadd_rn(HT::hi(r.x), v[1]);
            v[2] = __fadd_rn(HT::lo(r.y), v[2]);
            v[3] = __fadd_rn(HT::hi(r.y), v[3]);
          }
        }
        if (a.out_f32) {
          *(f32x4*)((float*)a.out + (size_t)row * a.ld_out + f0) = (f32x4){v[0], v[1], v[2], v[3]};
        } else {
          uint2 w;
          w.x = bf2(v[0], v[1]);
          w.y = bf2(v[2], v[3]);
          *(uint2*)((uint16_t*)a.out + (size_t)row * a.ld_out + f0) = w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int f = f0 + e;
          if (f < out) {
            float x = v[e];
            if (a.res)
              x = __fadd_rn(a.res_f32 ? ((const float*)a.res)[(size_t)row * a.ld_res + f]
                                      : HT::to_f32(((const uint16_t*)a.res)[(size_t)row * a.ld_res + f]),
                            x);
            if (a.out_f32) ((float*)a.out)[(size_t)row * a.ld_out + f] = x;
            else ((uint16_t*)a.out)[(size_t)row * a.ld_out + f] = HT::from_f32(x);
          }
        }
      }
    }
}

// a finished tile's rows: plain outputs (host-checked 32-bit byte offsets, plain_out) by buffer
// stores for every lane, an invalid row's offset past the buffer; else store_out per valid row
template <int MT, bool PLAIN>
__device__ __forceinline__ void store_tile(const f32x16 (&acc)[MT], const FArgs& a, long row,
                                           bool valid, int h) {
  if constexpr (PLAIN && RG_FAST_ENC_BUF) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        a.out, 0, (int)(((a.rows - 1) * a.ld_out + 32 * MT) * 2), 0x00020000);
    const int off = valid ? (int)((row * a.ld_out + 4 * h) * 2) : 0x7ffff000;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t w = {bf2(acc[m][4 * g], acc[m][4 * g + 1]), bf2(acc[m][4 * g + 2], acc[m][4 * g + 3])};
        __builtin_amdgcn_raw_buffer_store_b64(w, rs, off + (32 * m + 8 * g) * 2, 0, 0);
      }
  } else {
    if (valid) store_out<MT, PLAIN>(acc, a, row, h);
  }
}

template <int SPEC, int OFF, int LI, int K, int N, int... Rest>
__device__ __forceinline__ void run_chain(const FArgs& a, const bf16x8_t (&b)[(K + 15) / 16],
                                          const char* lds, const float* nrm, long row, bool valid,
                                          int lane) {
  constexpr int KS = (K + 15) / 16;
  constexpr int MT = N / 32;
  static_assert(N % 32 == 0, "padded widths are multiples of 32");
  f32x16 acc[MT];
  mfma_layer<KS, MT>(b, acc, lds + OFF, lane);
  epilogue<SPEC, LI, MT>(acc, a.L[LI], nrm);
  if constexpr (sizeof...(Rest) > 0) {
    bf16x8_t nb[2 * MT];
    pack_next<MT>(acc, nb);
    run_chain<SPEC, OFF + ((fast_bytes(K, N) + 15) & ~15), LI + 1, N, Rest...>(a, nb, lds, nrm,
                                                                             row, valid, lane);
  } else {
    store_tile<MT, SPEC >= 0 && (SPEC & SPEC_PLAIN_OUT) != 0>(acc, a, row, valid, lane >> 5);
  }
}

// A tile-fused first layer with a compile-time LeakyReLU runs on PRESCALED operands:
// the kernel multiplies its float32 inputs and its staged bias by 0.505 (LEAKY_PRE), so
// the accumulator holds y' = 0.505 y and leaky(y) = 0.505 y + 0.495 |y| = y' + c |y'| is
// ONE fma with a free |.| source modifier instead of a multiply and a max (the encoders
// apply it to 256 features per row).
constexpr bool pre_scaled_l0(int spec_) {
  return spec_ >= 0 && ((spec_ >> 16) & 1) != 0 && (spec_ & 0xff) == ACT_LEAKY;
}

// a chain whose layer 0 takes a split pair (Input::PAIR_SPLIT): layer 0 over 2 KS
// fragments, then the rest of the chain as usual
template <int SPEC, int K, int N, int... Rest>
__device__ __forceinline__ void run_chain_pair(const FArgs& a,
                                               const bf16x8_t (&b)[2 * ((K + 15) / 16)],
                                               const char* lds, const float* nrm, long row,
                                               bool valid, int lane) {
  constexpr int KS = (K + 15) / 16;
  constexpr int MT = N / 32;
  f32x16 acc[MT];
  mfma_layer_rep<KS, MT, 2>(b, acc, lds, lane);
  epilogue<SPEC, 0, MT>(acc, a.L[0], nrm);
  if constexpr (sizeof...(Rest) > 0) {
    bf16x8_t nb[2 * MT];
    pack_next<MT>(acc, nb);
    run_chain<SPEC, ((fast_bytes(K, N) + 15) & ~15), 1, N, Rest...>(a, nb, lds, nrm, row, valid,
                                                                    lane);
  } else {
    store_tile<MT, SPEC >= 0 && (SPEC & SPEC_PLAIN_OUT) != 0>(acc, a, row, valid, lane >> 5);
  }
}

// Layers 0 and 1 fused tile by tile, for a first layer WITHOUT normalisation (the
// encoders' first ffn_block, gnn_blocks.py:31): each 32-wide output tile of layer 0 is
// activated, packed to bf16 and consumed at once as layer 1's k-steps 2m0, 2m0+1, so
// layer 0's N0-wide activation never exists in full (the 7 -> 256 edge encoder would
// otherwise hold 128 accumulators + 64 packed registers and spill).
template <int SPEC, int K0, int N0, int N1, int... Rest>
__device__ __forceinline__ void run_chain01(const FArgs& a, const bf16x8_t (&b)[(K0 + 15) / 16],
                                            const char* lds, const float* nrm, long row,
                                            bool valid, int lane) {
  constexpr int KS0 = (K0 + 15) / 16, MT0 = N0 / 32, KS1 = N0 / 16, MT1 = N1 / 32;
  constexpr int OFF1 = (fast_bytes(K0, N0) + 15) & ~15;
  constexpr bool PRE0 = pre_scaled_l0(SPEC);
  constexpr int OFF2 = OFF1 + ((fast_bytes(N0, N1) + 15) & ~15);
  static_assert(N0 % 32 == 0 && N1 % 32 == 0, "padded widths are multiples of 32");
  const int h = lane >> 5;
  const char* w0 = lds + lane * 16;
  const char* w1 = lds + OFF1 + lane * 16;
  const float* bias0 = (const float*)(lds + MT0 * KS0 * 1024);
  const float* bias1 = (const float*)(lds + OFF1 + MT1 * KS1 * 1024);
  f32x16 acc[MT1];
#pragma unroll
  for (int m = 0; m < MT1; ++m)
    acc[m] = ld_bias_frag(bias1, m, h);  // accumulator-order bias: 4 x ds_read_b128
  // skewed by one layer-0 tile: the layer-0 MFMA + activation of tile m0+1 are
  // independent of the 2*MT1 layer-1 MFMAs of tile m0, so the scheduler can issue that
  // VALU work while the matrix pipe runs (MFMA / VALU co-execution inside one wave)
  auto l0_tile = [&](auto A, int m0, bf16x8_t (&nb)[2]) {
    f32x16 t = ld_bias_frag(bias0, m0, h);  // accumulator-order bias: 4 x ds_read_b128
#pragma unroll
    for (int s = 0; s < KS0; ++s)
      t = mfma32(ld_bf8((const uint16_t*)(w0 + (m0 * KS0 + s) * 1024)), b[s], t);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      f32x2 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (PRE0) {  // prescaled layer 0: leaky(y) = y' + c |y'|, one fma each
          const f32x2 y = pair(t, 4 * hf + j);
          v[j] = (f32x2){fmaf(fabsf(y.x), LEAKY_C, y.x), fmaf(fabsf(y.y), LEAKY_C, y.y)};
        } else {
          v[j] = act_pk<decltype(A)::value>(pair(t, 4 * hf + j));
        }
      }
      nb[hf] = __builtin_bit_cast(bf16x8_t, (u32x4){bf2(v[0].x, v[0].y), bf2(v[1].x, v[1].y),
                                                    bf2(v[2].x, v[2].y), bf2(v[3].x, v[3].y)});
    }
  };
  // layer-1 A fragments of layer-0 tile m0: 2*MT1 contiguous fragments, read one tile
  // ahead (double-buffered) so no MFMA waits on its LDS read
  auto l1_frags = [&](int m0, bf16x8_t (&f)[2 * MT1]) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int m = 0; m < MT1; ++m)
        f[hf * MT1 + m] = ld_bf8((const uint16_t*)(w1 + (m * KS1 + 2 * m0 + hf) * 1024));
  };
  auto body = [&](auto A) {
    bf16x8_t ncur[2], nnxt[2];
    bf16x8_t fcur[2 * MT1], fnxt[2 * MT1];
    l1_frags(0, fcur);
    l0_tile(A, 0, ncur);
#pragma unroll
    for (int m0 = 0; m0 < MT0; ++m0) {
      if (m0 + 1 < MT0) {
        l1_frags(m0 + 1, fnxt);
        l0_tile(A, m0 + 1, nnxt);
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int m = 0; m < MT1; ++m)
          acc[m] = mfma32(fcur[hf * MT1 + m], ncur[hf], acc[m]);
      // interleave: the next tile's activation VALU between this tile's layer-1 MFMAs
#pragma unroll
      for (int i = 0; i < 2 * MT1; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // 4 VALU
      }
      __builtin_amdgcn_sched_barrier(0);  // two layer-0 tiles in flight: bounded registers
      if (m0 + 1 < MT0) {
        ncur[0] = nnxt[0];
        ncur[1] = nnxt[1];
#pragma unroll
        for (int i = 0; i < 2 * MT1; ++i) fcur[i] = fnxt[i];
      }
    }
  };
  if constexpr (SPEC >= 0) {
    if constexpr (((SPEC >> 16) & 1) != 0) body(std::integral_constant<int, (SPEC & 0xff)>{});
    else body(std::integral_constant<int, ACT_NONE>{});
  } else {
    act_dispatch(a.L[0].act, body);
  }
  epilogue<SPEC, 1, MT1>(acc, a.L[1], nrm);
  if constexpr (sizeof...(Rest) > 0) {
    bf16x8_t nb[2 * MT1];
    pack_next<MT1>(acc, nb);
    run_chain<SPEC, OFF2, 2, N1, Rest...>(a, nb, lds, nrm, row, valid, lane);
  } else {
    store_tile<MT1, SPEC >= 0 && (SPEC & SPEC_PLAIN_OUT) != 0>(acc, a, row, valid, h);
  }
}

template <int MODE, bool IN_F32, int W0, int W1, int SPEC, int FT, int... Ns>
__global__ __launch_bounds__(FT) void fast_chain_kernel(FArgs a) {
  constexpr int FW = FT / 64;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ float nrm[2 * RG_MAX_LAYERS];
  using In = Input<MODE & ~FUSE01, IN_F32, W0, W1>;
  if (threadIdx.x == 0) {  // static layer indices: a dynamic a.L[i] would copy a to scratch
#pragma unroll
    for (int l = 0; l < RG_MAX_LAYERS; ++l) {
      const bool n = l < a.nl && a.L[l].mu;
      nrm[2 * l] = n ? *a.L[l].mu : 0.f;
      nrm[2 * l + 1] = n ? *a.L[l].sd : 0.f;
    }
  }
  // stage all layers' packed weights + biases (static layer indices: no scratch copy)
#pragma unroll
  for (int l = 0; l < RG_MAX_LAYERS; ++l) {
    if (l < a.nl) {
      stage_lds<FT>(lds + a.L[l].woff, a.L[l].src, a.L[l].bytes);
    }
  }
  __syncthreads();
  constexpr bool PRE0 = (MODE & FUSE01) != 0 && pre_scaled_l0(SPEC);
  if constexpr (PRE0) {  // layer 0's bias, scaled like its inputs (run_chain01)
    constexpr int N0 = FirstOf<Ns...>::value;
    float* b0 = (float*)(lds + (N0 / 32) * In::KS * 1024);
    for (int i = threadIdx.x; i < N0; i += FT) b0[i] *= LEAKY_PRE;
    __syncthreads();
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long rows = a.rows_dev ? min((long)*a.rows_dev, a.rows) : a.rows;
  const long ntiles = (rows + 31) / 32;
  const long tstride = (long)gridDim.x * FW;
  auto run = [&](const bf16x8_t (&b)[In::KSB], long row, bool valid) {
    if constexpr ((MODE & FUSE01) != 0)  // un-normalised first layer: tile-fused layers 0+1
      run_chain01<SPEC, In::K0, Ns...>(a, b, lds, nrm, row, valid, lane);
    else if constexpr (In::PAIR_SPLIT)
      run_chain_pair<SPEC, In::K0, Ns...>(a, b, lds, nrm, row, valid, lane);
    else
      run_chain<SPEC, 0, 0, In::K0, Ns...>(a, b, lds, nrm, row, valid, lane);
  };
#ifdef RG_ENC_NOPF
  if constexpr (false) {
#else
  if constexpr ((MODE & ~FUSE01) == RG_IN_DENSE && IN_F32 && In::KS == 1) {
#endif
    // float32 encoder inputs (<= 8 features per row): the next tile's row is loaded
    // while this tile runs its chain, so no tile waits for an HBM round trip; lanes of
    // the upper half (features 8..15) only supply zeros
    const int h = lane >> 5;
    float nx[8];
    auto fetch = [&](long t, float (&v)[8]) {
      const long r = t * 32 + (lane & 31);
      if constexpr (RG_FAST_ENC_BUF) {  // unconditional: a row past the end reads row 0
        const float* p = (const float*)a.in0 + (size_t)(r < rows ? r : 0) * a.ld0;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = p[min(j, a.w0real - 1)];
      } else {
        const float* p = (const float*)a.in0 + (size_t)r * a.ld0;
        const bool ok = h == 0 && t < ntiles && r < rows;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ok && j < a.w0real ? p[j] : 0.f;
      }
    };
    long tile = (long)blockIdx.x * FW + wave;
    if constexpr (RG_FAST_ENC_BUF) {
      if (tile < ntiles) fetch(tile, nx);
      // nothing in flight at the loop entry: the loop-top wait for the prefetched rows is counted
      __builtin_amdgcn_s_waitcnt(0x0f70);
    } else {
      fetch(tile, nx);
    }
    for (; tile < ntiles; tile += tstride) {
      bf16x8_t b[1];
      if constexpr (RG_FAST_ENC_BUF) {  // the mask of this tile's prefetched rows
        const bool ok = h == 0 && tile * 32 + (lane & 31) < rows;
#pragma unroll
        for (int j = 0; j < 8; ++j) nx[j] = ok && j < a.w0real ? nx[j] : 0.f;
      }
      if constexpr (PRE0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) nx[j] *= LEAKY_PRE;
      }
      b[0] = __builtin_bit_cast(bf16x8_t, (u32x4){bf2(nx[0], nx[1]), bf2(nx[2], nx[3]),
                                                  bf2(nx[4], nx[5]), bf2(nx[6], nx[7])});
      fetch(tile + tstride, nx);
      const long row = tile * 32 + (lane & 31);
      run(b, row, row < rows);
    }
  } else {
    for (long tile = (long)blockIdx.x * FW + wave; tile < ntiles; tile += tstride) {
      const long row = tile * 32 + (lane & 31);
      const bool valid = row < rows;
      bf16x8_t b[In::KSB];
      In::load(a, row, valid, lane >> 5, b, PRE0 ? LEAKY_PRE : 1.f);
      run(b, row, valid);
    }
  }
}

template <int MODE, bool IN_F32, int W0, int W1, int SPEC, int FT, int... Ns>
static int launch(const FArgs& a, hipStream_t st) {
  constexpr int FW = FT / 64;
  using In = Input<MODE & ~FUSE01, IN_F32, W0, W1>;
  // the host-side LDS image must be the layout the kernel assumes
  using Off = Offsets<In::K0, Ns...>;
  for (int l = 0; l < a.nl; ++l)
    RG_REQUIRE(a.L[l].woff == Off::get(l), RG_ERR_ARG, "rg_mlp_chain_fast: LDS layout of layer %d", l);
  auto kern = fast_chain_kernel<MODE, IN_F32, W0, W1, SPEC, FT, Ns...>;
  RG_ENSURE_LDS(kern, DYN_LDS_MAX);
  const long tiles = (a.rows + 31) / 32;
  long blocks = (tiles + FW - 1) / FW;
  const int per_cu = (FT == 512 && a.total_bytes <= 76 * 1024) ? 2 : 1;
  if (blocks > 256L * per_cu) blocks = 256L * per_cu;
  if (blocks < 1) blocks = 1;
  kern<<<blocks, FT, a.total_bytes, st>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// shape key: mode, f32 input, widths, epilogue spec (-1: run-time), padded outputs
struct Key {
  int mode, in_f32, w0, w1, spec, nl;
  int n[RG_MAX_LAYERS];
};

static bool match(const Key& k, int mode, int in_f32, int w0, int w1,
                  std::initializer_list<int> ns) {
  if (k.mode != mode || k.in_f32 != in_f32 || k.w0 != w0 || k.w1 != w1 ||
      k.nl != (int)ns.size())
    return false;
  int i = 0;
  for (int v : ns)
    if (k.n[i++] != v) return false;
  return true;
}

#ifndef RG_ENC_FT
#define RG_ENC_FT 768  // edge-encoder workgroup: 3 waves/SIMD (167 VGPRs, 13 dwords spilled) beat 2 (179) by 4 %
#endif
// output of width nl written as bf16 rows of 4-wide vectors, no residual
static bool plain_out(const FArgs& a, int nl) {
  return !a.res && !a.out_f32 && a.out_vec && a.out_real == nl &&
         (!RG_FAST_ENC_BUF || (double)a.rows * a.ld_out * 2 <= 0x7ff00000);  // 32-bit offsets
}

// instantiations: the yml / BASELINE architecture (C = 64, encoders 256/128, heads 7 / 2)
static int dispatch(const Key& k, const FArgs& a, hipStream_t st) {
#define RG_FAST(FT, SP, MODE, F32, W0, W1, ...)                                           \
  if (match(k, MODE, F32, W0, W1, {__VA_ARGS__}))                                        \
    return k.spec == (SP) ? launch<MODE, F32, W0, W1, (SP), FT, __VA_ARGS__>(a, st)       \
                          : launch<MODE, F32, W0, W1, -1, 512, __VA_ARGS__>(a, st);
  // the same with a plain bf16 output epilogue when the call allows it (SPEC_PLAIN_OUT)
#define RG_FAST_P(FT, SP, MODE, F32, W0, W1, NL, ...)                                      \
  if (match(k, MODE, F32, W0, W1, {__VA_ARGS__}) && k.spec == (SP) && plain_out(a, NL))  \
    return launch<MODE, F32, W0, W1, (SP) | SPEC_PLAIN_OUT, FT, __VA_ARGS__>(a, st);
  constexpr int L = ACT_LEAKY;
  // node / edge encoders (graph_feature_encoding, gnn_blocks.py:19-42: block 0 is not
  // normalised)
  RG_FAST_P(512, spec(L, 0b110, 0b111), RG_IN_DENSE | FUSE01, 1, 6, 0, 64, 256, 128, 64)
  RG_FAST_P(RG_ENC_FT, spec(L, 0b1110, 0b1111), RG_IN_DENSE | FUSE01, 1, 7, 0, 64, 256, 128, 128,
            64)
  RG_FAST(512, spec(L, 0b110, 0b111), RG_IN_DENSE | FUSE01, 1, 6, 0, 256, 128, 64)
  RG_FAST(RG_ENC_FT, spec(L, 0b1110, 0b1111), RG_IN_DENSE | FUSE01, 1, 7, 0, 256, 128, 128, 64)
  // message MLP on cat(x_i, x_j, e) and update MLP on cat(x, agg) (msg_mlp_hidden_dim 128)
  RG_FAST(512, spec(L, 0b11, 0b11), RG_IN_GATHER3, 0, 64, 64, 128, 64)
  RG_FAST(1024, spec(L, 0b1, 0b1), RG_IN_CONCAT2, 0, 64, 64, 64)
  // heads: 3-block stems + FFN_TaskSpecificHead (ffn + bare Linear -> 7 / 2)
  RG_FAST(1024, spec(L, 0b1111, 0b1111), RG_IN_DENSE, 0, 64, 0, 64, 64, 64, 64, 32)
  RG_FAST(1024, spec(L, 0b1111, 0b1111), RG_IN_PAIRADD, 0, 64, 0, 64, 64, 64, 64, 32)
  RG_FAST(768, spec(L, 0b1, 0b1), RG_IN_DENSE, 0, 64, 0, 64)
  RG_FAST(768, spec(L, 0b111, 0b111), RG_IN_DENSE, 0, 64, 0, 64, 64, 64)
  RG_FAST(1024, spec(L, 0b01, 0b01), RG_IN_DENSE, 0, 64, 0, 64, 32)
  // cluster-level classifier GNN (classifier/blocks.py, classifier yml: C = 128, no
  // normalisation): encoder 5 -> 256 -> 128 -> 128, message MLP on cat(x_i, x_j),
  // update on cat(x, agg), pooled stem 3 x 128 + head (ffn 128 + Linear -> 7)
  RG_FAST(512, spec(L, 0b000, 0b111), RG_IN_DENSE | FUSE01, 1, 5, 0, 256, 128, 128)
  RG_FAST(512, spec(L, 0b00, 0b11), RG_IN_GATHER3, 0, 128, 0, 128, 128)
  RG_FAST(512, spec(L, 0b0, 0b1), RG_IN_CONCAT2, 0, 128, 128, 128)
  RG_FAST(512, spec(L, 0b00000, 0b01111), RG_IN_DENSE, 0, 128, 0, 128, 128, 128, 128, 32)
#undef RG_FAST
  return RG_ERR_UNSUPPORTED;
}

// the C-ABI entry of this operand type (rg_mlp_chain_fast dispatches on RG_LAYER_F16)
static int chain_fast_entry(const rg_layer* layers, int n_layers, long rows,
                                 const int* rows_dev, int in_mode, int in_dtype, const void* in0,
                                 int ld0, int w0, const void* in1, int ld1, int w1,
                                 const void* in2, int ld2, int w2, const int* idx0,
                                 const int* idx1, const void* residual, int ld_res, int res_dtype,
                                 void* out, int ld_out, int out_dtype, void* stream) {
  RG_REQUIRE(n_layers >= 1 && n_layers <= RG_MAX_LAYERS, RG_ERR_ARG, "rg_mlp_chain_fast: n_layers");
  Key k;
  memset(&k, 0, sizeof(k));
  k.mode = in_mode;
  k.in_f32 = in_dtype == RG_F32 ? 1 : 0;
  RG_REQUIRE(in_dtype == RG_F32 || in_dtype == RG_HALF_CODE, RG_ERR_ARG, "rg_mlp_chain_fast: in_dtype");
  RG_REQUIRE(out_dtype == RG_F32 || out_dtype == RG_HALF_CODE, RG_ERR_ARG, "rg_mlp_chain_fast: out_dtype");
  RG_REQUIRE(!residual || res_dtype == RG_F32 || res_dtype == RG_HALF_CODE, RG_ERR_ARG, "rg_mlp_chain_fast: res_dtype");
  RG_REQUIRE(in_mode == RG_IN_DENSE || in_dtype == RG_HALF_CODE, RG_ERR_UNSUPPORTED,
             "rg_mlp_chain_fast: gathered / concatenated inputs must be bf16");
  k.w0 = w0;
  k.w1 = in_mode == RG_IN_GATHER3 ? w2 : (in_mode == RG_IN_CONCAT2 ? w1 : 0);
  k.nl = n_layers;
  FArgs a;
  memset(&a, 0, sizeof(a));
  int off = 0;
  for (int l = 0; l < n_layers; ++l) {
    const rg_layer& s = layers[l];
    RG_REQUIRE(s.w_packed, RG_ERR_ARG, "rg_mlp_chain_fast: layer %d weights", l);
    if (s.save_pre || s.save_out) return RG_ERR_UNSUPPORTED;  // tapes: the f32 generic chain
    RG_REQUIRE(!s.norm_mu || (s.norm_std && s.out_dim >= 2), RG_ERR_ARG, "norm params");
    k.n[l] = (s.out_dim + 31) / 32 * 32;
    if (l > 0)
      RG_REQUIRE(s.in_dim == layers[l - 1].out_dim, RG_ERR_ARG, "rg_mlp_chain_fast: widths");
    a.L[l].src = s.w_packed;
    a.L[l].mu = s.norm_mu;
    a.L[l].sd = s.norm_std;
    a.L[l].woff = off;
    a.L[l].bytes = (int)rg_packed_linear_bytes(s.in_dim, s.out_dim,
                                               l == 0 ? RG_PACK_FAST_IN : RG_PACK_FAST_CHAIN);
    a.L[l].out = s.out_dim;
    a.L[l].act = s.act;
    a.L[l].centered = (s.flags & RG_LAYER_CENTERED) ? 1 : 0;
    off += (a.L[l].bytes + 15) & ~15;
    // chained layers: the previous padded width is the next K (zero columns beyond out)
    if (l > 0 && layers[l - 1].out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
  }
  if (off > DYN_LDS_MAX) return RG_ERR_UNSUPPORTED;
  a.nl = n_layers;
  a.total_bytes = off;
  a.rows = rows;
  a.rows_dev = rows_dev;
  a.in0 = in0; a.in1 = in1; a.in2 = in2;
  a.ld0 = ld0; a.ld1 = ld1; a.ld2 = ld2;
  a.in_f32 = k.in_f32;
  a.w0real = w0;
  a.idx0 = idx0; a.idx1 = idx1;
  a.res = residual; a.ld_res = ld_res; a.res_f32 = res_dtype == RG_F32;
  a.out = out; a.ld_out = ld_out; a.out_f32 = out_dtype == RG_F32;
  a.out_real = layers[n_layers - 1].out_dim;
  // vector paths need 16-B (bf16 x8) aligned rows
  RG_REQUIRE(in_mode == RG_IN_DENSE && k.in_f32 ? true : (ld0 % 8 == 0 && (!in1 || ld1 % 8 == 0) &&
                                                         (!in2 || ld2 % 8 == 0)),
             RG_ERR_UNSUPPORTED, "rg_mlp_chain_fast: row strides must be multiples of 8");
  a.out_vec = (ld_out % 4 == 0) && (!residual || ld_res % 4 == 0);
  if (in_mode == RG_IN_DENSE && k.in_f32) {
    if (w0 > 8) return RG_ERR_UNSUPPORTED;
    k.w0 = w0;
    // encoders: the first ffn_block has no normalisation (gnn_blocks.py:31)
    if (n_layers >= 2 && !layers[0].norm_mu) k.mode |= FUSE01;
  }
  // compile-time epilogues: the yml activation (LeakyReLU,
  // configuration_radarscenes_gnn.yml:50) or identity per layer, norm per layer
  {
    int nm = 0, am = 0;
    bool ok = true;
    for (int l = 0; l < n_layers; ++l) {
      if (layers[l].norm_mu) nm |= 1 << l;
      if (layers[l].norm_mu && !(layers[l].flags & RG_LAYER_CENTERED)) ok = false;
      if (layers[l].act == ACT_LEAKY) am |= 1 << l;
      else if (layers[l].act != ACT_NONE) ok = false;
    }
    k.spec = ok ? spec(ACT_LEAKY, nm, am) : -1;
  }
  // normalised layers must be unpadded (epilogue statistics run over 32*MT features)
  for (int l = 0; l < n_layers; ++l)
    if (layers[l].norm_mu && layers[l].out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
  if (rows <= 0) return RG_OK;
  return dispatch(k, a, (hipStream_t)stream);
}

}  // namespace RG_FAST_NS
}  // namespace rg

