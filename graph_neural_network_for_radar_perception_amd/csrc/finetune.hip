// Object-classifier finetuning (Model_Object_Classifier_Finetuning, gnn_detector.py:481-519):
//  * the per-proposal ground truth torch.argmax(torch.bincount(node_gt_class[members]))
//    (gnn_detector.py:511-513): one thread per cluster, a class histogram in registers,
//    first maximum (torch.argmax's tie rule);
//  * Loss_Object_Class (loss.py:79-89): cross entropy with one-hot targets, summed and
//    divided by the number of proposals, + compute_accuracy (gnn_detector.py:24-28) --
//    one workgroup, fixed-order float64 sum (the no-grad / validation path; the training
//    path runs the object head through the native training engine).
#include "rg_common.h"

namespace rg {
namespace finetune {

static constexpr int MAXC = 32;  // classes (the detector has 7)

__global__ void majority_kernel(const int64_t* __restrict__ labels, const int* __restrict__ cptr,
                                const int* __restrict__ cidx, int ncl, int n_classes,
                                int64_t* __restrict__ out, int* __restrict__ bad) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncl) return;
  int hist[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) hist[k] = 0;
  for (int p = cptr[c]; p < cptr[c + 1]; ++p) {
    const int64_t l = labels[cidx[p]];
    if (l < 0 || l >= n_classes) {
      atomicExch(bad, 1);
      continue;
    }
#pragma unroll
    for (int k = 0; k < MAXC; ++k) hist[k] += (k == (int)l) ? 1 : 0;
  }
  int best = 0;
#pragma unroll
  for (int k = 1; k < MAXC; ++k)
    if (hist[k] > hist[best]) best = k;
  out[c] = best;
}

__global__ __launch_bounds__(256) void cross_entropy_kernel(const float* __restrict__ logits, int ld,
                                                            const int64_t* __restrict__ labels,
                                                            int n, int nc, float* __restrict__ loss,
                                                            float* __restrict__ acc) {
  __shared__ double sl[256];
  __shared__ int sa[256];
  double l = 0.0;
  int a = 0;
  for (int r = threadIdx.x; r < n; r += 256) {
    const float* x = logits + (size_t)r * ld;
    float m = x[0];
    int am = 0;
    for (int k = 1; k < nc; ++k)
      if (x[k] > m) {
        m = x[k];
        am = k;
      }
    double s = 0.0;
    for (int k = 0; k < nc; ++k) s += exp((double)x[k] - (double)m);
    const int64_t t = labels[r];
    l += log(s) + (double)m - (double)x[t];
    a += am == (int)t ? 1 : 0;
  }
  sl[threadIdx.x] = l;
  sa[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sl[threadIdx.x] += sl[threadIdx.x + w];
      sa[threadIdx.x] += sa[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = (float)(sl[0] / (double)n);
    acc[0] = (float)((double)sa[0] / (double)n);
  }
}

// d logits[r][k] = g * (softmax(logits[r])[k] - [k == label_r]) / n
__global__ void cross_entropy_backward_kernel(const float* __restrict__ logits, int ld,
                                              const int64_t* __restrict__ labels, int n, int nc,
                                              const float* __restrict__ g, float* __restrict__ d,
                                              int ldd) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* x = logits + (size_t)r * ld;
  float m = x[0];
  for (int k = 1; k < nc; ++k) m = fmaxf(m, x[k]);
  double s = 0.0;
  for (int k = 0; k < nc; ++k) s += exp((double)x[k] - (double)m);
  const double scale = (double)*g / (double)n;
  const int64_t t = labels[r];
  for (int k = 0; k < nc; ++k) {
    const double p = exp((double)x[k] - (double)m) / s;
    d[(size_t)r * ldd + k] = (float)(scale * (p - (k == (int)t ? 1.0 : 0.0)));
  }
}

}  // namespace finetune
}  // namespace rg

using namespace rg;
using namespace rg::finetune;

extern "C" int rg_cluster_majority_label(const int64_t* node_labels, const int* cluster_ptr,
                                         const int* cluster_idx, int n_clusters, int n_classes,
                                         int64_t* out, int* bad_label, void* stream) {
  RG_REQUIRE(n_classes >= 1 && n_classes <= MAXC, RG_ERR_ARG,
             "rg_cluster_majority_label: n_classes=%d outside 1..%d", n_classes, MAXC);
  if (n_clusters <= 0) return RG_OK;
  majority_kernel<<<ceil_div(n_clusters, 256), 256, 0, (hipStream_t)stream>>>(
      node_labels, cluster_ptr, cluster_idx, n_clusters, n_classes, out, bad_label);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_cross_entropy(const float* logits, int ld, const int64_t* labels, int n, int nc,
                                float* loss, float* accuracy, void* stream) {
  RG_REQUIRE(n >= 1 && nc >= 1, RG_ERR_ARG, "rg_cross_entropy: n=%d nc=%d", n, nc);
  cross_entropy_kernel<<<1, 256, 0, (hipStream_t)stream>>>(logits, ld, labels, n, nc, loss,
                                                           accuracy);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_cross_entropy_backward(const float* logits, int ld, const int64_t* labels, int n,
                                         int nc, const float* g, float* d_logits, int ld_d,
                                         void* stream) {
  RG_REQUIRE(n >= 0 && nc >= 1 && g, RG_ERR_ARG, "rg_cross_entropy_backward: arguments");
  if (n == 0) return RG_OK;
  cross_entropy_backward_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(
      logits, ld, labels, n, nc, g, d_logits, ld_d);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
