// Float32 encoders (graph_feature_encoding, gnn_blocks.py:19-42: ffn_block chains
// Linear -> channel_normalization -> LeakyReLU, common.py:185-220) on the bf16 matrix cores
// with the exact three-term operand splits of x3_common.h, the weights STREAMED THROUGH AN
// LDS RING shared by the workgroup.
//
// The edge encoder 7 -> 256 -> 128 -> 128 -> 64 holds 361 KiB of split weights; chain_x3.hip
// keeps 153 KiB of them in LDS and has every wave read the other 208 KiB from L2 straight
// into registers, once per 64 rows: four copies of the same fragment stream per CU, and the
// waves spent 42 % of their time waiting (SQ_WAIT_INST_ANY, profiles/r02g_sq_counters.txt).
// Here the workgroup's waves run in step over one chunk sequence:
//  * layer 0 (<= 8 inputs, no norm; 24 KiB) and every bias stay resident in LDS;
//  * layers 1.. are cut into 24-KiB chunks (two k-steps of a 128-wide layer, four of a
//    64-wide one: the three planes of every M-tile of those k-steps); chunk q + 1 is copied
//    global -> LDS by the workgroup (global_load_lds_dwordx4: no registers, one 1-KiB
//    fragment block per wave instruction) while chunk q is consumed (two ring slots, one
//    barrier per chunk); fragments are read from the slot with ds_read_b128;
//  * layer 0 is fused tile by tile into layer 1 (its 32-wide output tile m0 = layer 1's
//    k-steps 2 m0, 2 m0 + 1 = layer 1's chunk m0), activations stay in registers between
//    layers, a normalised layer's scale + LeakyReLU is applied in the next layer's B
//    operand (split_acc_pend), the next k-step's B operand is split beside the MFMAs.
// A CU reads each weight byte from L2 once per 32 * RT * W rows instead of once per 32 * RT.
// Same arithmetic and the same summation order per output as chain_x3.hip's encoders.
#include "x3_common.h"

namespace rg {
namespace encx3 {

using namespace ::rg::x3;

typedef __attribute__((address_space(3))) void* lds_as3;

static constexpr int SLOT = 24 * 1024;  // one chunk
#ifndef RG_ENC_NSLOT
#define RG_ENC_NSLOT 3  // 3: chunk q + 1 is already visible while chunk q is consumed, so the
                        // first fragments of the next chunk are read before its boundary
#endif
static constexpr int NSLOT = RG_ENC_NSLOT;
static constexpr bool XPF = NSLOT >= 3;  // cross-chunk fragment prefetch

constexpr int spec(int norm_mask, int act_mask, bool centred) {
  return norm_mask | (act_mask << 8) | (centred ? 1 << 16 : 0);
}
constexpr bool sp_norm(int sp, int l) { return ((sp >> l) & 1) != 0; }
constexpr bool sp_act(int sp, int l) { return ((sp >> (8 + l)) & 1) != 0; }
constexpr bool sp_cent(int sp) { return ((sp >> 16) & 1) != 0; }

template <int K0, int... Ns>
struct Sh {
  static constexpr int NL = sizeof...(Ns);
  static constexpr int N[NL] = {Ns...};
  static constexpr int K(int l) { return l == 0 ? K0 : N[l - 1]; }
  static constexpr int MT(int l) { return N[l] / 32; }
  static constexpr int KS(int l) { return l == 0 ? 1 : K(l) / 16; }
  static constexpr int KPC(int l) { return 8 / MT(l); }  // k-steps per chunk (MT * 3 KiB each)
  static constexpr int CH(int l) { return KS(l) / KPC(l); }
  static constexpr int C0(int l) {  // first chunk of layer l >= 1
    int c = 0;
    for (int i = 1; i < l; ++i) c += CH(i);
    return c;
  }
  static constexpr int NCH = C0(NL);
  static constexpr int pl(int l) { return plane_bytes(K(l), N[l]); }
  // LDS: ring, layer 0's three planes, every bias, the norm scalars
  static constexpr int W0_OFF = NSLOT * SLOT;
  static constexpr int B_OFF = W0_OFF + 3 * plane_bytes(K0, N[0]);
  static constexpr int boff(int l) {
    int o = B_OFF;
    for (int i = 0; i < l; ++i) o += N[i] * 4;
    return o;
  }
  static constexpr int NRM_OFF = boff(NL);
  static constexpr int LDS = NRM_OFF + 2 * NL * 4;
};

struct Args {
  const char* w[RG_MAX_LAYERS];  // x3 images (global)
  const float* mu[RG_MAX_LAYERS];
  const float* sd[RG_MAX_LAYERS];
  long rows;
  const int* rows_dev;
  const float* in0;
  int ld0, w0real;
  float* out;
  int ld_out;
};

// The workgroup's weight stream: chunk q of it holds chunk q % NCH of the chain
template <typename S, int W>
struct Ring {
  const char* w[S::NL];  // the layers' x3 images
  char* lds;
  const char* slot;  // current chunk's slot + lane * 16
  const char* nslot; // the next chunk's slot + lane * 16 (visible when XPF)
  long q;            // next chunk to consume
  long total;        // chunks this workgroup consumes
  int wave, lane;

  // chunk q into slot q % NSLOT: 24 fragment blocks of 1 KiB, block b = (j MT + m) 3 + p
  // (k-step j of the chunk, M-tile m, plane p) copied by wave b % W
  __device__ __forceinline__ void issue(long qq) const {
    if (qq >= total) return;
    const int c = (int)(qq % S::NCH);
    char* dst = lds + (int)(qq % NSLOT) * SLOT;
    int mt = 0, ks = 0, c0 = 0, pl = 0;
    const char* src = nullptr;
#pragma unroll
    for (int i = 1; i < S::NL; ++i)
      if (c >= S::C0(i)) {
        mt = S::MT(i);
        ks = S::KS(i);
        c0 = S::C0(i);
        pl = S::pl(i);
        src = w[i];
      }
    const int kpc = 8 / mt;
    const int s0 = (c - c0) * kpc;
#pragma unroll
    for (int i = 0; i < 24 / W; ++i) {
      const int b = wave + W * i;
      const int j = b / (3 * mt), rem = b - j * 3 * mt;
      const int m = rem / 3, p = rem - 3 * m;
      const char* g = src + p * pl + (m * ks + s0 + j) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_as3)(dst + b * 1024), 16, 0, 0);
    }
  }
  // chunk boundary of chunk q: this wave's copies issued so far are complete (vmcnt 0: chunk
  // q + NSLOT - 2, which makes chunk q ready with two slots and q + 1 ready with three), the
  // barrier makes every wave's copies visible and frees the slot of chunk q - 1 (every wave
  // is past it); then chunk q + NSLOT - 1 is issued into that slot.  hook() runs between the
  // barrier and the issue (register work whose loads must not wait for the new copies),
  // after() behind it.
  template <typename Hook, typename After>
  __device__ __forceinline__ void begin(Hook&& hook, After&& after) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    hook();
    issue(q + NSLOT - 1);
    after();
    slot = lds + (int)(q % NSLOT) * SLOT + lane * 16;
    nslot = lds + (int)((q + 1) % NSLOT) * SLOT + lane * 16;
    ++q;
  }
  // fragment (k-step j of the chunk, M-tile m, plane p) of the current / the next chunk
  template <int MT>
  __device__ __forceinline__ bf16x8_t frag(int j, int m, int p) const {
    return ld_bf8(slot + ((j * MT + m) * 3 + p) * 1024);
  }
  template <int MT>
  __device__ __forceinline__ bf16x8_t frag_next(int j, int m, int p) const {
    return ld_bf8(nslot + ((j * MT + m) * 3 + p) * 1024);
  }
};

struct Nop {
  __device__ __forceinline__ void operator()() const {}
};

template <int SPEC, int l, int MT>
__device__ __forceinline__ void epilogue(f32x16 (&acc)[MT], const float* nrm) {
  if constexpr (sp_norm(SPEC, l) && sp_act(SPEC, l)) {
    norm_leaky<MT, sp_cent(SPEC)>(acc, nrm[2 * l], nrm[2 * l + 1]);
  } else if constexpr (sp_norm(SPEC, l)) {
    norm_only<MT, sp_cent(SPEC)>(acc, nrm[2 * l], nrm[2 * l + 1]);
  } else if constexpr (sp_act(SPEC, l)) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[m][q] = act_t<ACT_LEAKY>(acc[m][q]);
  }
}
template <int SPEC, int l>
constexpr int pend_kind() {
  return (sp_norm(SPEC, l) && sp_act(SPEC, l)) ? 1 : sp_norm(SPEC, l) ? 2 : 0;
}
template <int SPEC, int l, int MT, int RT>
__device__ __forceinline__ void epilogue_pend(f32x16 (&acc)[RT][MT], const float* nrm, Pend (&pn)[RT]) {
  constexpr int K = pend_kind<SPEC, l>();
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    if constexpr (K == 1) {
      pn[t] = pend_norm_leaky<MT, sp_cent(SPEC)>(acc[t], nrm[2 * l], nrm[2 * l + 1]);
    } else if constexpr (K == 2) {
      pn[t] = pend_norm_only<MT, sp_cent(SPEC)>(acc[t], nrm[2 * l], nrm[2 * l + 1]);
    } else {
      epilogue<SPEC, l, MT>(acc[t], nrm);
      pn[t] = Pend{0.f, 0.f};
    }
  }
}

// layer l >= 2 from the ring; prev = layer l - 1's accumulators with its norm / act pending
// (PEND); the last layer's rows land in outv.  last() runs behind the stream's last chunk
// issue of this pass (the next pass's input loads).
template <typename S, int SPEC, int W, int l, int RT, int PMT, int PEND, typename Last>
__device__ __forceinline__ void run_rest(Ring<S, W>& ring, const f32x16 (&prev)[RT][PMT],
                                         const Pend (&pend)[RT], const char* lds, const float* nrm,
                                         f32x16 (&outv)[RT][S::MT(S::NL - 1)], Last&& last) {
  constexpr int MT = S::MT(l), KS = S::KS(l), KPC = S::KPC(l);
  static_assert(S::K(l) == 32 * PMT, "chained width");
  static_assert(MT == 2 || MT == 4, "24-KiB chunks hold 2 or 4 k-steps");
  const int h = ring.lane >> 5;
  const float* bias = (const float*)(lds + S::boff(l));
  f32x16 acc[RT][MT];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = ld_bias_frag(bias, m, h);
  auto bop = [&](int s, int t) { return split_acc_pend<PEND>(prev[t][s >> 1], s & 1, pend[t]); };
  X3 bq[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) bq[t] = bop(0, t);
  bf16x8_t Ab[2][MT][3];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int j = s % KPC;
    if (j == 0) {
      if constexpr (l + 1 == S::NL) {
        if (s + KPC == KS) ring.begin(Nop{}, last);
        else ring.begin(Nop{}, Nop{});
      } else {
        ring.begin(Nop{}, Nop{});
      }
      if (s == 0 || !XPF) {  // else read during the previous chunk's last k-step
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int p = 0; p < 3; ++p) Ab[s & 1][m][p] = ring.template frag<MT>(j, m, p);
      }
    }
    if (j + 1 < KPC) {  // the next k-step's fragments from the same slot
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int p = 0; p < 3; ++p) Ab[(s + 1) & 1][m][p] = ring.template frag<MT>(j + 1, m, p);
    } else if (XPF && s + 1 < KS) {  // the next chunk's first k-step (visible already)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int p = 0; p < 3; ++p) Ab[(s + 1) & 1][m][p] = ring.template frag_next<MT>(0, m, p);
    }
    X3 bn[RT];
    if (s + 1 < KS) {
#pragma unroll
      for (int t = 0; t < RT; ++t) bn[t] = bop(s + 1, t);
    }
    const bf16x8_t(&A)[MT][3] = Ab[s & 1];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const X3 b = bq[t];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][2], b.p0, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][1], b.p1, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][0], b.p2, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][1], b.p0, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][0], b.p1, acc[t][m]);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = mf(A[m][0], b.p0, acc[t][m]);
    }
    if (s + 1 < KS) {
#pragma unroll
      for (int t = 0; t < RT; ++t) bq[t] = bn[t];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (l + 1 < S::NL) {
    Pend pn[RT];
    epilogue_pend<SPEC, l, MT, RT>(acc, nrm, pn);
    run_rest<S, SPEC, W, l + 1, RT, MT, pend_kind<SPEC, l>()>(ring, acc, pn, lds, nrm, outv, last);
  } else {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      epilogue<SPEC, l, MT>(acc[t], nrm);
#pragma unroll
      for (int m = 0; m < MT; ++m) outv[t][m] = acc[t][m];
    }
  }
}

template <int SPEC, int W, int RT, int K0, int... Ns>
__global__ __launch_bounds__(64 * W) void enc_ring_kernel(Args a) {
  using S = Sh<K0, Ns...>;
  constexpr int NL = S::NL, NCH = S::NCH, FT = 64 * W;
  static_assert(NL >= 3, "layer 0 + layer 1 + at least one ring layer after them");
  static_assert(S::N[0] / 32 == S::CH(1) && S::KPC(1) == 2, "layer-0 tile m0 = layer-1 chunk m0");
  static_assert(24 % W == 0, "fragment blocks per chunk over the waves");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;

  // layer 0's planes, every bias, the norm scalars: resident
  stage_lds<FT>(lds + S::W0_OFF, a.w[0], 3 * S::pl(0));
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const u32x4* bs = (const u32x4*)(a.w[l] + 3 * S::pl(l));
    u32x4* bd = (u32x4*)(lds + S::boff(l));
    for (int i = threadIdx.x; i < S::N[l] / 4; i += FT) bd[i] = bs[i];
  }
  float* nrm = (float*)(lds + S::NRM_OFF);
  if (threadIdx.x < NL) {
    nrm[2 * threadIdx.x] = a.mu[threadIdx.x] ? *a.mu[threadIdx.x] : 0.f;
    nrm[2 * threadIdx.x + 1] = a.sd[threadIdx.x] ? *a.sd[threadIdx.x] : 0.f;
  }

  const long rows = a.rows_dev ? min((long)*a.rows_dev, a.rows) : a.rows;
  constexpr int PROWS = 32 * RT * W;  // rows per workgroup pass
  const long npass = (rows + PROWS - 1) / PROWS;
  const long my_pass = npass > (long)blockIdx.x ? (npass - 1 - blockIdx.x) / gridDim.x + 1 : 0;

  Ring<S, W> ring;
#pragma unroll
  for (int l = 0; l < NL; ++l) ring.w[l] = a.w[l];
  ring.lds = lds;
  ring.slot = lds;
  ring.nslot = lds;
  ring.q = 0;
  ring.total = my_pass * NCH;
  ring.wave = wave;
  ring.lane = lane;
  __syncthreads();  // the resident images are staged
#pragma unroll
  for (int i = 0; i + 1 < NSLOT; ++i) ring.issue(i);
  const WLds W0{lds + S::W0_OFF + lane * 16, S::pl(0)};

  // the next pass's inputs (lane r = row; lanes h = 0 hold the <= 8 features)
  float vin[RT][8];
  auto load_in = [&](long pass) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const long row = pass * PROWS + (long)wave * 32 * RT + 32 * t + r;
      const bool ok = row < rows && h == 0;
      const float* p = a.in0 + (size_t)(ok ? row : 0) * a.ld0;
#pragma unroll
      for (int j = 0; j < 8; ++j) vin[t][j] = (ok && j < a.w0real) ? p[j] : 0.f;
    }
  };
  constexpr int MTL = S::MT(NL - 1);
  f32x16 outv[RT][MTL];  // the last layer's rows, stored behind the next chunk boundary
  long out_row0 = -1;
  auto store_out = [&]() {
    if (out_row0 < 0) return;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const long row = out_row0 + 32 * t + r;
      if (row >= rows) continue;
      float* o = a.out + (size_t)row * a.ld_out;
#pragma unroll
      for (int m = 0; m < MTL; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *(f32x4*)(o + 32 * m + 8 * g + 4 * h) = (f32x4){outv[t][m][4 * g], outv[t][m][4 * g + 1],
                                                           outv[t][m][4 * g + 2], outv[t][m][4 * g + 3]};
    }
    out_row0 = -1;
  };

  if (my_pass > 0) load_in(blockIdx.x);
  constexpr int MT0 = S::MT(0), MT1 = S::MT(1);
  const float* bias0 = (const float*)(lds + S::boff(0));
  const float* bias1 = (const float*)(lds + S::boff(1));
  for (long pass = blockIdx.x; pass < npass; pass += gridDim.x) {
    const long row0 = pass * PROWS + (long)wave * 32 * RT;
    X3 b0[RT];
    // ---- layer 0 fused into layer 1: chunk m0 = layer-1 k-steps 2 m0, 2 m0 + 1
    f32x16 acc1[RT][MT1];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int m = 0; m < MT1; ++m) acc1[t][m] = ld_bias_frag(bias1, m, h);
    bf16x8_t An[MT1][3];  // XPF: the next chunk's first-k-step fragments
#pragma unroll
    for (int m0 = 0; m0 < MT0; ++m0) {
      if (m0 == 0) {
        ring.begin(
            [&] {
#pragma unroll
              for (int t = 0; t < RT; ++t)
                b0[t] = split8((f32x4){vin[t][0], vin[t][1], vin[t][2], vin[t][3]},
                               (f32x4){vin[t][4], vin[t][5], vin[t][6], vin[t][7]});
            },
            store_out);
      } else {
        ring.begin(Nop{}, Nop{});
      }
      bf16x8_t A[2][MT1][3];
#pragma unroll
      for (int m = 0; m < MT1; ++m)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          A[0][m][p] = (XPF && m0 > 0) ? An[m][p] : ring.template frag<MT1>(0, m, p);
      f32x16 y[RT][1];
#pragma unroll
      for (int t = 0; t < RT; ++t) y[t][0] = ld_bias_frag(bias0, m0, h);
      layer_x3<1, 1, MT0, RT>(y, W0, m0, [&](int, int t) { return b0[t]; });
      if constexpr (sp_act(SPEC, 0)) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int qq = 0; qq < 16; ++qq) y[t][0][qq] = act_t<ACT_LEAKY>(y[t][0][qq]);
      }
#pragma unroll
      for (int m = 0; m < MT1; ++m)
#pragma unroll
        for (int p = 0; p < 3; ++p) A[1][m][p] = ring.template frag<MT1>(1, m, p);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (XPF && hf == 1 && m0 + 1 < MT0) {  // the next chunk's first k-step (visible)
#pragma unroll
          for (int m = 0; m < MT1; ++m)
#pragma unroll
            for (int p = 0; p < 3; ++p) An[m][p] = ring.template frag_next<MT1>(0, m, p);
        }
#pragma unroll
        for (int t = 0; t < RT; ++t) {
          const X3 b = split_acc(y[t][0], hf);
#pragma unroll
          for (int m = 0; m < MT1; ++m) acc1[t][m] = mf(A[hf][m][2], b.p0, acc1[t][m]);
#pragma unroll
          for (int m = 0; m < MT1; ++m) acc1[t][m] = mf(A[hf][m][1], b.p1, acc1[t][m]);
#pragma unroll
          for (int m = 0; m < MT1; ++m) acc1[t][m] = mf(A[hf][m][0], b.p2, acc1[t][m]);
#pragma unroll
          for (int m = 0; m < MT1; ++m) acc1[t][m] = mf(A[hf][m][1], b.p0, acc1[t][m]);
#pragma unroll
          for (int m = 0; m < MT1; ++m) acc1[t][m] = mf(A[hf][m][0], b.p1, acc1[t][m]);
#pragma unroll
          for (int m = 0; m < MT1; ++m) acc1[t][m] = mf(A[hf][m][0], b.p0, acc1[t][m]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    Pend pn[RT];
    epilogue_pend<SPEC, 1, MT1, RT>(acc1, nrm, pn);
    const long next = pass + gridDim.x;
    run_rest<S, SPEC, W, 2, RT, MT1, pend_kind<SPEC, 1>()>(ring, acc1, pn, lds, nrm, outv, [&] {
      if (next < npass) load_in(next);  // behind the pass's last chunk boundary
    });
    out_row0 = row0;
  }
  store_out();
}

template <int SPEC, int W, int RT, int K0, int... Ns>
static int launch(const Args& a, hipStream_t st) {
  using S = Sh<K0, Ns...>;
  static_assert(S::LDS <= DYN_LDS_MAX, "enc_x3 LDS");
  auto kern = enc_ring_kernel<SPEC, W, RT, K0, Ns...>;
  RG_ENSURE_LDS(kern, S::LDS);
  constexpr int PROWS = 32 * RT * W;
  const long npass = (a.rows + PROWS - 1) / PROWS;
  // persistent: one workgroup per CU (the ring + resident images take ~75 KiB, the
  // registers one wave per SIMD at RT = 2)
  long blocks = npass < 256L ? npass : 256L;
  if (blocks < 1) blocks = 1;
  kern<<<blocks, 64 * W, S::LDS, st>>>(a);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

}  // namespace encx3
}  // namespace rg

using namespace rg;
using namespace rg::encx3;

#ifndef RG_ENC_W
#define RG_ENC_W 4  // waves per workgroup (one per SIMD at RT = 2)
#endif
#ifndef RG_ENC_RT
#define RG_ENC_RT 2  // 32-row tiles per wave
#endif

// The encoder shapes of rg_mlp_chain_x3 (IN_SMALL: <= 8 float32 inputs, layer 0 neither
// normalised nor anything but LeakyReLU / none); RG_ERR_UNSUPPORTED for any other chain.
// Called by rg_mlp_chain_x3 (chain_x3.hip) before its own dispatch; RG_X3_RING=0 disables.
int rg_enc_ring_x3(const rg_layer* layers, int n_layers, long rows, const int* rows_dev,
                   const float* in0, int ld0, int w0, float* out, int ld_out, int norm_mask,
                   int act_mask, int centred, void* stream) {
  const char* knob = getenv("RG_X3_RING");  // read per call (tests switch it)
  const bool on = knob && atoi(knob) != 0;  // off until measured on the GPU
  if (!on || n_layers < 3 || w0 > 8) return RG_ERR_UNSUPPORTED;
  if (ld_out % 4 != 0) return RG_ERR_UNSUPPORTED;
  if (layers[n_layers - 1].out_dim % 32 != 0) return RG_ERR_UNSUPPORTED;
  Args a;
  memset(&a, 0, sizeof(a));
  for (int l = 0; l < n_layers; ++l) {
    a.w[l] = (const char*)layers[l].w_packed;
    a.mu[l] = layers[l].norm_mu;
    a.sd[l] = layers[l].norm_std;
  }
  a.rows = rows;
  a.rows_dev = rows_dev;
  a.in0 = in0;
  a.ld0 = ld0;
  a.w0real = w0;
  a.out = out;
  a.ld_out = ld_out;
  if (rows <= 0) return RG_OK;
  const hipStream_t st = (hipStream_t)stream;
  auto is = [&](int k0, std::initializer_list<int> ns) {
    if (w0 != k0 || (int)ns.size() != n_layers) return false;
    int i = 0;
    for (int v : ns)
      if (layers[i++].out_dim != v) return false;
    return true;
  };
  // edge encoder 7 -> 256 -> 128 -> 128 -> 64, node encoder 6 -> 256 -> 128 -> 64
  // (gnn_blocks.py:19-42: block 0 without norm, every block LeakyReLU)
#define RG_ENC(K0, NM, AM, ...)                                                          \
  if (is(K0, {__VA_ARGS__}) && norm_mask == NM && act_mask == AM) {                   \
    if (centred) return launch<spec(NM, AM, true), RG_ENC_W, RG_ENC_RT, K0, __VA_ARGS__>(a, st); \
    return launch<spec(NM, AM, false), RG_ENC_W, RG_ENC_RT, K0, __VA_ARGS__>(a, st);   \
  }
  RG_ENC(7, 0b1110, 0b1111, 256, 128, 128, 64)
  RG_ENC(6, 0b110, 0b111, 256, 128, 64)
#undef RG_ENC
  return RG_ERR_UNSUPPORTED;
}
