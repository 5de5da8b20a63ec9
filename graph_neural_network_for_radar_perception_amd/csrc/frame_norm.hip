// layer_normalization / group_normalization (modules/neural_net/common.py:223-253) for a
// batch of frames: the reference normalises a WHOLE tensor -- every row of one frame's
// nodes, edges, link pairs or clusters -- with
//   layer:  mean / unbiased std over all rows x all C features,
//   group:  x.reshape(N, G, C/G), mean / std over dims (0, 2): per group g, all rows x the
//           C/G features of g,
// then y = std_param * (x - mean) / (std + eps) + mu_param and the block's activation.
// The chain kernels fuse only per-row statistics, so a layer followed by a frame-wide
// norm ends its chain launch (writing z = x W^T + b) and this file finishes it:
//   1. partial sums: grid (CHUNKS, n_seg), each workgroup sums a contiguous slice of its
//      segment's rows per group in float64 (sum, sum of squares);
//   2. finalize: per (segment, group) the CHUNKS partials in fixed order -> mean and
//      unbiased std (float64, rounded to float32 once: the statistics the reference
//      computes in float32, to within an ulp);
//   3. apply: y = act(s (z - mean) / (std + eps) + m) in float32, the reference's op order.
// Deterministic (fixed reduction orders, no atomics).  Segments are row ranges
// [seg_ptr[s], seg_ptr[s+1]) of device int32 offsets.
#include "rg_common.h"

namespace rg {
namespace fnorm {

static constexpr int CHUNKS = 32;   // workgroups per segment
static constexpr int BT = 256;
static constexpr int MAXG = 64;     // groups per layer
static constexpr float NORM_EPS = 1e-5f;

__device__ __forceinline__ void seg_rows(const int* seg_ptr, int s, int chunk, long& r0, long& r1) {
  const long b = seg_ptr[s], e = seg_ptr[s + 1];
  const long n = e - b;
  r0 = b + n * chunk / CHUNKS;
  r1 = b + n * (chunk + 1) / CHUNKS;
}

// partial[s][chunk][g] = (sum, sum of squares) of z over the chunk's rows, group g
__global__ __launch_bounds__(BT) void partial_kernel(const float* __restrict__ z, int ldz, int C,
                                                     int G, const int* __restrict__ seg_ptr,
                                                     double* __restrict__ partial) {
  const int chunk = blockIdx.x, s = blockIdx.y;
  long r0, r1;
  seg_rows(seg_ptr, s, chunk, r0, r1);
  const int cg = C / G;
  __shared__ double sh_s[BT], sh_q[BT];
  for (int g = 0; g < G; ++g) {
    double a = 0.0, q = 0.0;
    const long n = (r1 - r0) * cg;
    for (long t = threadIdx.x; t < n; t += BT) {
      const long r = r0 + t / cg;
      const int c = g * cg + (int)(t % cg);
      const double v = (double)z[(size_t)r * ldz + c];
      a += v;
      q += v * v;
    }
    sh_s[threadIdx.x] = a;
    sh_q[threadIdx.x] = q;
    __syncthreads();
    for (int w = BT / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) {
        sh_s[threadIdx.x] += sh_s[threadIdx.x + w];
        sh_q[threadIdx.x] += sh_q[threadIdx.x + w];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      double* p = partial + (((size_t)s * CHUNKS + chunk) * G + g) * 2;
      p[0] = sh_s[0];
      p[1] = sh_q[0];
    }
    __syncthreads();
  }
}

// stats[s][g] = (mean, std) as float32
__global__ void finalize_kernel(const double* __restrict__ partial, const int* __restrict__ seg_ptr,
                                int n_seg, int C, int G, float* __restrict__ stats) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_seg * G) return;
  const int s = t / G, g = t % G;
  double a = 0.0, q = 0.0;
  for (int c = 0; c < CHUNKS; ++c) {
    const double* p = partial + (((size_t)s * CHUNKS + c) * G + g) * 2;
    a += p[0];
    q += p[1];
  }
  const double n = (double)(seg_ptr[s + 1] - seg_ptr[s]) * (C / G);
  const double mean = a / n;
  const double var = (q - a * mean) / (n - 1.0);  // torch.std: unbiased (NaN for n = 1)
  stats[2 * t] = (float)mean;
  stats[2 * t + 1] = (float)sqrt(var > 0.0 ? var : (var == var ? 0.0 : var));
}

template <int ACT>
__global__ __launch_bounds__(BT) void apply_kernel(const float* __restrict__ z, int ldz, int C, int G,
                                                   const int* __restrict__ seg_ptr,
                                                   const float* __restrict__ stats,
                                                   const float* __restrict__ mu_p,
                                                   const float* __restrict__ sd_p,
                                                   const float* __restrict__ res, int ldr,
                                                   float* __restrict__ out, int ldo) {
  const int chunk = blockIdx.x, s = blockIdx.y;
  long r0, r1;
  seg_rows(seg_ptr, s, chunk, r0, r1);
  const int cg = C / G;
  const float mu = *mu_p, sd = *sd_p;
  const long n = (r1 - r0) * C;
  for (long t = threadIdx.x; t < n; t += BT) {
    const long r = r0 + t / C;
    const int c = (int)(t % C);
    const float* st = stats + 2 * ((size_t)s * G + c / cg);
    const float x = z[(size_t)r * ldz + c];
    // reference order: (x - mean) / (std + eps), then std_param * x + mu_param
    const float y = __fadd_rn(__fmul_rn(sd, div_rn(x - st[0], st[1] + NORM_EPS)), mu);
    const float v = act_t<ACT>(y);
    out[(size_t)r * ldo + c] = res ? __fadd_rn(res[(size_t)r * ldr + c], v) : v;
  }
}

// ------------------------------------------------------------------ backward
// Training through layer / group normalisation (the reference's loss.backward() over
// common.py:223-253).  Per segment s and group g with n = rows x C/G elements, from the
// saved pre-norm rows z and the output gradient da:
//   d = z - mean,  r = 1 / (std + eps),  n_ = d r,  y = s n_ + m,  gy = da act'(y),
//   gn = s gy;   d_std_param += sum gy n_,  d_mu_param += sum gy   (over every element)
//   dz = r (gn - mean(gn)) - r^2 (sum gn d) d / ((n - 1) std)     (torch.std: unbiased)
// Pass 1 recomputes the statistics as the forward does; pass 2 sums (gn, gn d, d) per
// (segment, chunk, group) and (gy n_, gy) per (segment, chunk) in float64; a finalize
// turns them into per-(segment, group) coefficients and the two parameter gradients
// (fixed order); pass 3 writes dz.  Deterministic.
__device__ __forceinline__ float act_grad_y(float y, int act) {
  if (act == ACT_LEAKY) return y > 0.f ? 1.f : 0.01f;  // torch: self > 0 ? grad : grad * slope
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == ACT_SWISH) {
    const float sg = 1.f / (1.f + expf(-y));
    return sg * (1.f + y * (1.f - sg));
  }
  return 1.f;
}

__global__ __launch_bounds__(BT) void bpartial_kernel(const float* __restrict__ z, int ldz,
                                                      const float* __restrict__ da, int ldda,
                                                      int C, int G, const int* __restrict__ seg_ptr,
                                                      const float* __restrict__ stats,
                                                      const float* __restrict__ mu_p,
                                                      const float* __restrict__ sd_p, int act,
                                                      double* __restrict__ gpart,
                                                      double* __restrict__ ppart) {
  const int chunk = blockIdx.x, s = blockIdx.y;
  long r0, r1;
  seg_rows(seg_ptr, s, chunk, r0, r1);
  const int cg = C / G;
  const float mu = *mu_p, sd = *sd_p;
  __shared__ double sh[3][BT];
  double pn = 0.0, pm = 0.0;  // sum gy n_, sum gy over every group of the chunk
  for (int g = 0; g < G; ++g) {
    const float mean = stats[2 * ((size_t)s * G + g)];
    const float sdev = stats[2 * ((size_t)s * G + g) + 1];
    double a = 0.0, b = 0.0, c = 0.0;
    const long n = (r1 - r0) * cg;
    for (long t = threadIdx.x; t < n; t += BT) {
      const long r = r0 + t / cg;
      const int col = g * cg + (int)(t % cg);
      const float x = z[(size_t)r * ldz + col];
      const float d = x - mean;
      const float nn = div_rn(d, sdev + NORM_EPS);
      const float y = __fadd_rn(__fmul_rn(sd, nn), mu);
      const float gy = da[(size_t)r * ldda + col] * act_grad_y(y, act);
      const float gn = sd * gy;
      a += (double)gn;
      b += (double)gn * (double)d;
      c += (double)d;
      pn += (double)gy * (double)nn;
      pm += (double)gy;
    }
    sh[0][threadIdx.x] = a;
    sh[1][threadIdx.x] = b;
    sh[2][threadIdx.x] = c;
    __syncthreads();
    for (int w = BT / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w)
        for (int k = 0; k < 3; ++k) sh[k][threadIdx.x] += sh[k][threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      double* p = gpart + (((size_t)s * CHUNKS + chunk) * G + g) * 3;
      p[0] = sh[0][0];
      p[1] = sh[1][0];
      p[2] = sh[2][0];
    }
    __syncthreads();
  }
  sh[0][threadIdx.x] = pn;
  sh[1][threadIdx.x] = pm;
  __syncthreads();
  for (int w = BT / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + w];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    ppart[((size_t)s * CHUNKS + chunk) * 2] = sh[0][0];
    ppart[((size_t)s * CHUNKS + chunk) * 2 + 1] = sh[1][0];
  }
}

// coef[s][g] = (r, r mean(gn), r^2 (sum gn d) / ((n - 1) std) - ... folded: see apply);
// the parameter gradients over every (segment, chunk) in a fixed order (one thread)
__global__ void bfinal_kernel(const double* __restrict__ gpart, const double* __restrict__ ppart,
                              const int* __restrict__ seg_ptr, int n_seg, int C, int G,
                              const float* __restrict__ stats, float* __restrict__ coef,
                              float* __restrict__ d_mu, float* __restrict__ d_sd) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n_seg * G) {
    const int s = t / G, g = t % G;
    double a = 0.0, b = 0.0, c = 0.0;
    for (int k = 0; k < CHUNKS; ++k) {
      const double* p = gpart + (((size_t)s * CHUNKS + k) * G + g) * 3;
      a += p[0];
      b += p[1];
      c += p[2];
    }
    const double n = (double)(seg_ptr[s + 1] - seg_ptr[s]) * (C / G);
    const double sdev = (double)stats[2 * t + 1];
    const double r = 1.0 / (double)(stats[2 * t + 1] + NORM_EPS);
    // a constant segment / group (std = 0): torch's std backward masks its 1 / std to zero
    // (FunctionsManual.cpp std_backward: masked_fill_(result == 0, 0)), so the reference's
    // gradient is finite, r (gn - mean(gn)) -- k2 = 0 here gives exactly that; n = 1 makes
    // std NaN in the forward (torch.std's 0 / 0), and r = NaN carries it into dz
    const double k2 = sdev > 0.0 ? r * r * b / ((n - 1.0) * sdev) : 0.0;
    // dz = r gn - k2 d - mean(r gn - k2 d) = r gn - k2 d - (r a - k2 c) / n
    coef[3 * t] = (float)r;
    coef[3 * t + 1] = (float)k2;
    coef[3 * t + 2] = (float)((r * a - k2 * c) / n);
  }
  if (t == 0 && d_mu && d_sd) {
    double pn = 0.0, pm = 0.0;
    for (long k = 0; k < (long)n_seg * CHUNKS; ++k) {
      pn += ppart[2 * k];
      pm += ppart[2 * k + 1];
    }
    *d_sd += (float)pn;
    *d_mu += (float)pm;
  }
}

__global__ __launch_bounds__(BT) void bapply_kernel(const float* __restrict__ z, int ldz,
                                                    const float* __restrict__ da, int ldda, int C,
                                                    int G, const int* __restrict__ seg_ptr,
                                                    const float* __restrict__ stats,
                                                    const float* __restrict__ coef,
                                                    const float* __restrict__ mu_p,
                                                    const float* __restrict__ sd_p, int act,
                                                    float* __restrict__ dz, int lddz) {
  const int chunk = blockIdx.x, s = blockIdx.y;
  long r0, r1;
  seg_rows(seg_ptr, s, chunk, r0, r1);
  const int cg = C / G;
  const float mu = *mu_p, sd = *sd_p;
  const long n = (r1 - r0) * C;
  for (long t = threadIdx.x; t < n; t += BT) {
    const long r = r0 + t / C;
    const int col = (int)(t % C);
    const size_t sg = (size_t)s * G + col / cg;
    const float mean = stats[2 * sg], sdev = stats[2 * sg + 1];
    const float x = z[(size_t)r * ldz + col];
    const float d = x - mean;
    const float nn = div_rn(d, sdev + NORM_EPS);
    const float y = __fadd_rn(__fmul_rn(sd, nn), mu);
    const float gn = sd * (da[(size_t)r * ldda + col] * act_grad_y(y, act));
    const float* k = coef + 3 * sg;
    dz[(size_t)r * lddz + col] = k[0] * gn - k[1] * d - k[2];
  }
}

}  // namespace fnorm
}  // namespace rg

using namespace rg;
using namespace rg::fnorm;

extern "C" size_t rg_frame_norm_workspace_size(int n_seg, int groups) {
  const size_t a = ((size_t)n_seg * CHUNKS * groups * 2 * sizeof(double) + 255) & ~(size_t)255;
  return a + (size_t)n_seg * groups * 2 * sizeof(float);
}

extern "C" int rg_frame_norm(const float* z, int ldz, int C, int groups, const int* seg_ptr,
                             int n_seg, const float* norm_mu, const float* norm_std, int act,
                             const float* residual, int ld_res, float* out, int ld_out,
                             void* workspace, size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(C >= 1 && groups >= 1 && groups <= MAXG && C % groups == 0, RG_ERR_ARG,
             "rg_frame_norm: C=%d groups=%d (C must be a multiple of groups <= %d)", C, groups,
             MAXG);
  RG_REQUIRE(n_seg >= 0 && norm_mu && norm_std, RG_ERR_ARG, "rg_frame_norm: arguments");
  RG_REQUIRE(workspace_bytes >= rg_frame_norm_workspace_size(n_seg, groups), RG_ERR_ARG,
             "rg_frame_norm: workspace too small");
  if (n_seg == 0) return RG_OK;
  double* partial = (double*)workspace;
  float* stats = (float*)((char*)workspace +
                          (((size_t)n_seg * CHUNKS * groups * 2 * sizeof(double) + 255) & ~(size_t)255));
  const dim3 grid(CHUNKS, n_seg);
  partial_kernel<<<grid, BT, 0, st>>>(z, ldz, C, groups, seg_ptr, partial);
  RG_LAUNCH_CHECK();
  finalize_kernel<<<ceil_div((long)n_seg * groups, 256), 256, 0, st>>>(partial, seg_ptr, n_seg, C,
                                                                       groups, stats);
  RG_LAUNCH_CHECK();
  auto kern = act == ACT_LEAKY ? apply_kernel<ACT_LEAKY>
              : act == ACT_RELU  ? apply_kernel<ACT_RELU>
              : act == ACT_SWISH ? apply_kernel<ACT_SWISH>
                                 : apply_kernel<ACT_NONE>;
  kern<<<grid, BT, 0, st>>>(z, ldz, C, groups, seg_ptr, stats, norm_mu, norm_std, residual, ld_res,
                            out, ld_out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

extern "C" size_t rg_frame_norm_backward_workspace_size(int n_seg, int groups) {
  return rg_frame_norm_workspace_size(n_seg, groups) +
         al256((size_t)n_seg * CHUNKS * groups * 3 * sizeof(double)) +
         al256((size_t)n_seg * CHUNKS * 2 * sizeof(double)) +
         al256((size_t)n_seg * groups * 3 * sizeof(float));
}

extern "C" int rg_frame_norm_backward(const float* z, int ldz, const float* da, int ldda, int C,
                                      int groups, const int* seg_ptr, int n_seg,
                                      const float* norm_mu, const float* norm_std, int act,
                                      float* dz, int lddz, float* d_mu, float* d_std,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(C >= 1 && groups >= 1 && groups <= MAXG && C % groups == 0, RG_ERR_ARG,
             "rg_frame_norm_backward: C=%d groups=%d", C, groups);
  RG_REQUIRE(n_seg >= 0 && norm_mu && norm_std && z && da && dz, RG_ERR_ARG,
             "rg_frame_norm_backward: arguments");
  RG_REQUIRE(act >= ACT_NONE && act <= ACT_SWISH, RG_ERR_ARG, "rg_frame_norm_backward: act %d", act);
  RG_REQUIRE(workspace_bytes >= rg_frame_norm_backward_workspace_size(n_seg, groups), RG_ERR_ARG,
             "rg_frame_norm_backward: workspace too small");
  if (n_seg == 0) return RG_OK;
  char* w = (char*)workspace;
  double* partial = (double*)w;
  float* stats = (float*)(w + al256((size_t)n_seg * CHUNKS * groups * 2 * sizeof(double)));
  w += rg_frame_norm_workspace_size(n_seg, groups);
  double* gpart = (double*)w;
  w += al256((size_t)n_seg * CHUNKS * groups * 3 * sizeof(double));
  double* ppart = (double*)w;
  w += al256((size_t)n_seg * CHUNKS * 2 * sizeof(double));
  float* coef = (float*)w;
  const dim3 grid(CHUNKS, n_seg);
  partial_kernel<<<grid, BT, 0, st>>>(z, ldz, C, groups, seg_ptr, partial);
  RG_LAUNCH_CHECK();
  finalize_kernel<<<ceil_div((long)n_seg * groups, 256), 256, 0, st>>>(partial, seg_ptr, n_seg, C,
                                                                       groups, stats);
  RG_LAUNCH_CHECK();
  bpartial_kernel<<<grid, BT, 0, st>>>(z, ldz, da, ldda, C, groups, seg_ptr, stats, norm_mu,
                                       norm_std, act, gpart, ppart);
  RG_LAUNCH_CHECK();
  bfinal_kernel<<<ceil_div((long)n_seg * groups, 256), 256, 0, st>>>(
      gpart, ppart, seg_ptr, n_seg, C, groups, stats, coef, d_mu, d_std);
  RG_LAUNCH_CHECK();
  bapply_kernel<<<grid, BT, 0, st>>>(z, ldz, da, ldda, C, groups, seg_ptr, stats, coef, norm_mu,
                                     norm_std, act, dz, lddz);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ------------------------------------------------------------------ segment bounds
__global__ void gather_i32_kernel(const int* __restrict__ table, const int* __restrict__ idx, int n,
                                  int* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = table[idx[t]];
}

__global__ void lower_bound_kernel(const int* __restrict__ sorted, const int* __restrict__ n_dev,
                                   long n, const int* __restrict__ q, int nq, int* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nq) return;
  long lo = 0, hi = n_dev ? min((long)*n_dev, n) : n;
  const int v = q[t];
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (sorted[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  out[t] = (int)lo;
}

extern "C" int rg_gather_i32(const int* table, const int* idx, int n, int* out, void* stream) {
  if (n <= 0) return RG_OK;
  gather_i32_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(table, idx, n, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_lower_bound_i32(const int* sorted, const int* n_sorted_dev, long n_sorted,
                                  const int* queries, int n_queries, int* out, void* stream) {
  if (n_queries <= 0) return RG_OK;
  lower_bound_kernel<<<ceil_div(n_queries, 256), 256, 0, (hipStream_t)stream>>>(
      sorted, n_sorted_dev, n_sorted, queries, n_queries, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
