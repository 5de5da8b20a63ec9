// Real-data front-end: the step before the graph build, for a
// window of radar scans already in HBM (the .h5 reading of read_data.py stays on the
// host).  Replaces, per window:
//   read_data.extract_and_sync_radar_data (read_data.py:227-303) and extract_frame
//   (:442-486): per scan the stationary gate identify_stationary_measurements
//   (meas_selection.py:22-70,169-200; ransac off, configuration_radarscenes_gnn.yml:11),
//   vr_cartesian_vf (meas_sync.py:15-20) and ego_compensate_radar_frames_list
//   (meas_sync.py:23-103) into the last scan's vehicle frame, cast to float32;
//   compute_ground_truth (compute_node_labels.py:50-105): class labels and per-track
//   offsets to the track mean;
//   grid_properties.select_meas_within_the_grid (grid_features.py:162-174) and
//   select_moving_data (graph_features.py:167-182) as ONE order-preserving compaction.
// One thread per measurement; the per-scan transforms are recomputed per thread from
// the scan's float64 pose (a few flops).  Arithmetic follows the reference's numpy
// promotion (comments at each step); transcendental functions of float32 arrays are
// evaluated in float32 as numpy does.
#include "rg_common.h"
#include <vector>
#include "scan.h"

// numpy evaluates every product and sum separately
#pragma clang fp contract(off)

namespace rg {

struct ScanPose {  // per scan, float64: mount (tx, ty, yaw), odometry (x, y, yaw, vx, yaw_rate)
  double tx, ty, myaw, ox, oy, oyaw, ovx, oyr;
};

__device__ __forceinline__ int scan_of(const int* __restrict__ scan_ptr, int n_scans, int i) {
  int lo = 0, hi = n_scans;  // scan_ptr[lo] <= i < scan_ptr[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (scan_ptr[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ ScanPose load_pose(const double* __restrict__ mount,
                                              const double* __restrict__ odo, int s) {
  ScanPose p;
  p.tx = mount[3 * s]; p.ty = mount[3 * s + 1]; p.myaw = mount[3 * s + 2];
  p.ox = odo[5 * s]; p.oy = odo[5 * s + 1]; p.oyaw = odo[5 * s + 2];
  p.ovx = odo[5 * s + 3]; p.oyr = odo[5 * s + 4];
  return p;
}

__global__ __launch_bounds__(256) void frontend_sync_kernel(
    const float* __restrict__ x_cc, const float* __restrict__ y_cc,
    const float* __restrict__ azimuth, const float* __restrict__ vr,
    const float* __restrict__ vr_comp, const int* __restrict__ scan_ptr, int n_scans,
    const int* __restrict__ scan_ref, const double* __restrict__ mount,
    const double* __restrict__ odo, float gamma, int n,
    float* __restrict__ px, float* __restrict__ py, float* __restrict__ vx,
    float* __restrict__ vy, uint8_t* __restrict__ stationary) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = scan_of(scan_ptr, n_scans, i);
  const ScanPose p = load_pose(mount, odo, s);
  const float az = azimuth[i];
  // ---- stationary gate (meas_selection.py:22-70): the sensor-frame ego velocity is
  // float64 (odometry scalars are np.float64), cos / sin of the float32 azimuths are
  // float32, their products with the float64 scalars float64
  const double vxs0 = p.ovx - p.oyr * p.ty;
  const double vys0 = 0.0 + p.oyr * p.tx;
  const double c = cos(-p.myaw), sn = sin(-p.myaw);
  const double vxs = vxs0 * c - vys0 * sn;
  const double vys = vxs0 * sn + vys0 * c;
  const double vr_pred = -((vxs * (double)cosf(az)) + (vys * (double)sinf(az)));
  const double err = vr_pred - (double)vr[i];
  stationary[i] = fabs(err) <= (double)gamma ? 1 : 0;
  // ---- vr_cartesian_vf (meas_sync.py:15-20): float32 array + python-float mount yaw
  // stays float32 (NEP 50 weak scalar); products float32
  const float ang = az + (float)p.myaw;
  const float v = vr_comp[i];
  vx[i] = v * cosf(ang);
  vy[i] = v * sinf(ang);
  // ---- ego compensation (meas_sync.py:52-71): T = T_curr^-1 T_prev in float64,
  // position R p + t, velocities unchanged; extract_frame casts to float32
  // the window's current scan (a batch of windows: each scan names its own)
  const ScanPose q = load_pose(mount, odo, scan_ref ? scan_ref[s] : n_scans - 1);
  const double cc = cos(q.oyaw), sc = sin(q.oyaw), cp = cos(p.oyaw), sp = sin(p.oyaw);
  const double r00 = cc * cp + sc * sp, r01 = -(cc * sp) + sc * cp;
  const double r10 = -(sc * cp) + cc * sp, r11 = sc * sp + cc * cp;
  const double dx = p.ox - q.ox, dy = p.oy - q.oy;
  const double t0 = cc * dx + sc * dy, t1 = -(sc * dx) + cc * dy;
  const double x = (double)x_cc[i], y = (double)y_cc[i];
  px[i] = (float)((r00 * x + r01 * y) + t0);
  py[i] = (float)((r10 * x + r11 * y) + t1);
}

// class labels (compute_node_labels.py:70-86) and per-track float64 sums for the offsets
__global__ __launch_bounds__(256) void frontend_labels_kernel(
    const int* __restrict__ track_key, const int64_t* __restrict__ label_id,
    const uint8_t* __restrict__ stationary, const int* __restrict__ old_to_new, int n_old,
    const float* __restrict__ px, const float* __restrict__ py, int n,
    float* __restrict__ cls, double* __restrict__ tsum, int* __restrict__ tcnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = track_key[i];
  float c;
  if (k > 0) {  // valid object: reassigned label id
    const int64_t o = label_id[i];
    c = (o >= 0 && o < n_old) ? (float)old_to_new[o] : -1.f;
    atomicAdd(tsum + 2 * k, (double)px[i]);
    atomicAdd(tsum + 2 * k + 1, (double)py[i]);
    atomicAdd(tcnt + k, 1);
  } else {      // no track: clutter 'FALSE' (6) or static environment 'STATIC' (7)
    c = stationary[i] ? 7.f : 6.f;
  }
  cls[i] = c;
}

// offsets to the track mean (compute_node_labels.py:50-67): mean in float64 from exact
// sums, rounded once to float32 (numpy's float32 pairwise mean is within an ulp), minus
// the float32 position in float32; untracked measurements keep 0
__global__ __launch_bounds__(256) void frontend_offsets_kernel(
    const int* __restrict__ track_key, const float* __restrict__ px,
    const float* __restrict__ py, const double* __restrict__ tsum,
    const int* __restrict__ tcnt, int n, float* __restrict__ offx, float* __restrict__ offy) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = track_key[i];
  if (k > 0) {
    const double m = (double)tcnt[k];
    offx[i] = (float)(tsum[2 * k] / m) - px[i];
    offy[i] = (float)(tsum[2 * k + 1] / m) - py[i];
  } else {
    offx[i] = 0.f;
    offy[i] = 0.f;
  }
}

// keep = inside [min_x, max_x) x [min_y, max_y) and class != STATIC
__global__ __launch_bounds__(256) void frontend_keep_kernel(
    const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ cls,
    float min_x, float max_x, float min_y, float max_y, float static_id, int n,
    int* __restrict__ keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = px[i], y = py[i];
  keep[i] = (x >= min_x && x < max_x && y >= min_y && y < max_y && cls[i] != static_id) ? 1 : 0;
}

__global__ __launch_bounds__(256) void frontend_index_kernel(const int* __restrict__ keep,
                                                             const int* __restrict__ pos, int n,
                                                             int* __restrict__ index) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (keep[i]) index[pos[i]] = i;
}

// the dynamic frames of a batch of windows: frame w = selected rows
// [pos[win_ptr[w]], pos[win_ptr[w + 1]]) (pos[n] = the total)
__global__ void frontend_frame_ptr_kernel(const int* __restrict__ pos,
                                          const int* __restrict__ win_ptr, int n_windows,
                                          int* __restrict__ frame_ptr) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w <= n_windows) frame_ptr[w] = pos[win_ptr[w]];
}

// ---- RANSAC stationary-measurement rejection (meas_selection.py:96-166, applied per scan to
// the gated measurements by identify_stationary_measurements, :188-199)
//
// The gated measurements of each scan, in order: one workgroup per scan, 256 at a time,
// positions from the waves' ballots.  gated_idx holds measurement indices at the scan's own
// offset scan_ptr[s]; gated_cnt[s] their count.
__global__ __launch_bounds__(256) void frontend_gate_lists_kernel(
    const uint8_t* __restrict__ stationary, const int* __restrict__ scan_ptr,
    int* __restrict__ gated_idx, int* __restrict__ gated_cnt) {
  __shared__ int wsum[4];
  const int s = blockIdx.x, a = scan_ptr[s], b = scan_ptr[s + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int base = 0;
  for (int c = a; c < b; c += 256) {
    const int i = c + threadIdx.x;
    const bool g = i < b && stationary[i];
    const uint64_t m = __ballot(g);
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    if (g) gated_idx[a + off + __popcll(m & ((1ull << lane) - 1ull))] = i;
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) gated_cnt[s] = base;
}

// The least-squares sensor velocity of a consensus set (meas_selection.py:72-93): normal
// equations summed in float64 over float32 cos / sin (numpy's float32 scalars: c ** 2,
// sin(2 t), c * vr, s * vr in float32), then inv(A) @ b.  numpy's float32 cos / sin (and its
// scalar c ** 2 in ~0.1 % of cases) are not correctly rounded and differ from cosf / sinf in
// the last place for some inputs, so a fit can differ from numpy's by ~1e-7 relative: an
// inlier decision then moves only for an error within ~1e-6 of the margin
__device__ void ransac_fit(const float* __restrict__ az, const float* __restrict__ vr,
                           const int* __restrict__ gi, const int* __restrict__ set, int k,
                           double& vx, double& vy) {
  double a00 = 0.0, a01 = 0.0, b0 = 0.0, b1 = 0.0;
  for (int j = 0; j < k; ++j) {
    const int m = gi[set[j]];
    const float t = az[m], v = vr[m];
    const float c = cosf(t), sn = sinf(t), s2 = sinf(2.f * t);
    a00 += (double)(c * c);
    a01 += (double)s2;
    b0 -= (double)(c * v);
    b1 -= (double)(sn * v);
  }
  a01 = 0.5 * a01;
  const double a10 = a01, a11 = (double)k - a00;
  // np.linalg.inv = LAPACK gesv against the identity: getrf (row pivot on |a10| > |a00|, the
  // multiplier scaled by the pivot's reciprocal), getrs (L, then U: y0 - u01 x1 in one fused
  // step, times the reciprocal); then numpy's matmul x_i = fma(inv_i0, b0, inv_i1 b1) --
  // bit-identical to numpy on this image's OpenBLAS for the fits of two samples
  const bool piv = fabs(a10) > fabs(a00);
  const double u00 = piv ? a10 : a00, u01 = piv ? a11 : a01;
  const double q0 = piv ? a00 : a10, q1 = piv ? a01 : a11;
  const double r0 = 1.0 / u00, l = q0 * r0, u11 = q1 - l * u01, r1 = 1.0 / u11;
  const double xa1 = (-l) * r1, xa0 = fma(-u01, xa1, 1.0) * r0;  // right-hand side (1, 0) / P
  const double xb1 = r1, xb0 = (-u01 * r1) * r0;                  // (0, 1) / P
  const double i00 = piv ? xb0 : xa0, i10 = piv ? xb1 : xa1;
  const double i01 = piv ? xa0 : xb0, i11 = piv ? xa1 : xb1;
  vx = fma(i00, b0, i01 * b1);
  vy = fma(i10, b0, i11 * b1);
}

__device__ __forceinline__ bool ransac_inlier(float t, float v, double vx, double vy,
                                              double margin) {
  const double pred = -(vx * (double)cosf(t) + vy * (double)sinf(t));
  return fabs((double)v - pred) <= margin;
}

// One workgroup per scan: every consensus set's fit and its inlier count over the test set
// (all gated measurements but the set's own), the first best, then the flags of the gated
// measurements from that fit.  Scans with <= min_meas gated measurements: no inliers.
constexpr int RANSAC_MAX_ITERS = 256;
__global__ __launch_bounds__(256) void frontend_ransac_kernel(
    const float* __restrict__ az, const float* __restrict__ vr, const int* __restrict__ scan_ptr,
    const int* __restrict__ gated_idx, const int* __restrict__ gated_cnt,
    const int* __restrict__ sets, int n_iter, int k, double margin, int min_meas,
    double ratio_thresh, uint8_t* __restrict__ stationary, double* __restrict__ in_ratio,
    uint8_t* __restrict__ is_valid) {
  __shared__ int cnt_it[RANSAC_MAX_ITERS];
  __shared__ int part[4];
  __shared__ double best_v[2];
  const int s = blockIdx.x, a = scan_ptr[s], n = gated_cnt[s];
  const int* gi = gated_idx + a;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (n <= min_meas) {
    for (int j = threadIdx.x; j < n; j += 256) stationary[gi[j]] = 0;
    if (threadIdx.x == 0) {
      in_ratio[s] = 0.0;
      is_valid[s] = 0;
    }
    return;
  }
  for (int it = 0; it < n_iter; ++it) {
    const int* set = sets + ((size_t)s * n_iter + it) * k;
    double vx, vy;
    ransac_fit(az, vr, gi, set, k, vx, vy);
    int c = 0;
    for (int j = threadIdx.x; j < n; j += 256) {
      const int m = gi[j];
      c += ransac_inlier(az[m], vr[m], vx, vy, margin) ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) part[wave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = part[0] + part[1] + part[2] + part[3];
      for (int j = 0; j < k; ++j) {  // the consensus set is not in the test set
        const int m = gi[set[j]];
        tot -= ransac_inlier(az[m], vr[m], vx, vy, margin) ? 1 : 0;
      }
      cnt_it[it] = tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int best = 0;
    for (int it = 1; it < n_iter; ++it)
      if (cnt_it[it] > cnt_it[best]) best = it;  // np.argmax: the first maximum
    double vx, vy;
    ransac_fit(az, vr, gi, sets + ((size_t)s * n_iter + best) * k, k, vx, vy);
    best_v[0] = vx;
    best_v[1] = vy;
    const double r = ((double)cnt_it[best] + (double)k) / (double)n;
    in_ratio[s] = r;
    is_valid[s] = r >= ratio_thresh ? 1 : 0;
  }
  __syncthreads();
  const double vx = best_v[0], vy = best_v[1];
  for (int j = threadIdx.x; j < n; j += 256) {
    const int m = gi[j];
    stationary[m] = ransac_inlier(az[m], vr[m], vx, vy, margin) ? 1 : 0;
  }
}

}  // namespace rg

using namespace rg;

// ---- the RANSAC consensus draws, host side (no device work): numpy's legacy generator
// (RandomState: MT19937, mtrand.pyx shuffle -> _shuffle_raw + random_interval of
// distributions.c) restated, so the draws numpy.random.shuffle would make -- and the state
// it would leave -- come out of one native loop instead of one Python call per shuffle
namespace {
constexpr int MT_N = 624, MT_M = 397;
void mt_refill(uint32_t* key) {
  int i = 0;
  for (; i < MT_N - MT_M; ++i) {
    const uint32_t y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
    key[i] = key[i + MT_M] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  for (; i < MT_N - 1; ++i) {
    const uint32_t y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
    key[i] = key[i + (MT_M - MT_N)] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  const uint32_t y = (key[MT_N - 1] & 0x80000000u) | (key[0] & 0x7fffffffu);
  key[MT_N - 1] = key[MT_M - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}
uint32_t mt_next32(uint32_t* key, int& pos) {
  if (pos >= MT_N) {
    mt_refill(key);
    pos = 0;
  }
  uint32_t y = key[pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
// a uniform integer in [0, mx] by masked rejection (random_interval, mx < 2^32)
uint32_t mt_interval(uint32_t* key, int& pos, uint32_t mx) {
  if (mx == 0) return 0;
  uint32_t mask = mx;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t v;
  while ((v = (mt_next32(key, pos) & mask)) > mx) {
  }
  return v;
}
}  // namespace

extern "C" int rg_ransac_consensus_sets(uint32_t* mt_key, int* mt_pos, const int* gated_cnt,
                                        int n_scans, int n_iter, int n_samples, int min_num_meas,
                                        int* consensus_sets) {
  RG_REQUIRE(mt_key && mt_pos && gated_cnt && consensus_sets && n_scans >= 0 && n_iter >= 1 &&
                 n_samples >= 1 && *mt_pos >= 0 && *mt_pos <= MT_N,
             RG_ERR_ARG, "rg_ransac_consensus_sets: bad argument");
  int pos = *mt_pos;
  std::vector<int> order;
  for (int s = 0; s < n_scans; ++s) {
    const int c = gated_cnt[s];
    int* out = consensus_sets + (size_t)s * n_iter * n_samples;
    if (c <= min_num_meas) {  // no draws (ransac's size check), sets unused
      for (int q = 0; q < n_iter * n_samples; ++q) out[q] = 0;
      continue;
    }
    RG_REQUIRE(n_samples <= c, RG_ERR_ARG, "rg_ransac_consensus_sets: %d samples of %d",
               n_samples, c);
    order.resize(c);
    for (int i = 0; i < c; ++i) order[i] = i;      // meas_idx = np.arange(n)
    for (int it = 0; it < n_iter; ++it) {          // np.random.shuffle(meas_idx), in place
      for (int i = c - 1; i >= 1; --i) {
        const int j = (int)mt_interval(mt_key, pos, (uint32_t)i);
        const int t = order[i];
        order[i] = order[j];
        order[j] = t;
      }
      for (int q = 0; q < n_samples; ++q) out[it * n_samples + q] = order[q];
    }
  }
  *mt_pos = pos;
  return RG_OK;
}

extern "C" int rg_frontend_gate_lists(const uint8_t* stationary, const int* scan_ptr, int n_scans,
                                      int* gated_idx, int* gated_cnt, void* stream) {
  RG_REQUIRE(n_scans >= 1 && stationary && scan_ptr && gated_idx && gated_cnt, RG_ERR_ARG,
             "rg_frontend_gate_lists: bad argument");
  frontend_gate_lists_kernel<<<n_scans, 256, 0, (hipStream_t)stream>>>(stationary, scan_ptr,
                                                                       gated_idx, gated_cnt);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_frontend_ransac(const float* azimuth_sc, const float* vr, const int* scan_ptr,
                                  int n_scans, const int* gated_idx, const int* gated_cnt,
                                  const int* consensus_sets, int n_iter, int n_samples,
                                  double error_margin, int min_num_meas, double ratio_threshold,
                                  uint8_t* stationary, double* in_ratio, uint8_t* is_valid,
                                  void* stream) {
  RG_REQUIRE(n_scans >= 1 && n_iter >= 1 && n_iter <= RANSAC_MAX_ITERS && n_samples >= 1 &&
                 n_samples <= min_num_meas + 1,
             RG_ERR_ARG, "rg_frontend_ransac: n_iter %d (<= %d), n_samples %d", n_iter,
             RANSAC_MAX_ITERS, n_samples);
  RG_REQUIRE(azimuth_sc && vr && scan_ptr && gated_idx && gated_cnt && consensus_sets &&
                 stationary && in_ratio && is_valid,
             RG_ERR_ARG, "rg_frontend_ransac: null argument");
  frontend_ransac_kernel<<<n_scans, 256, 0, (hipStream_t)stream>>>(
      azimuth_sc, vr, scan_ptr, gated_idx, gated_cnt, consensus_sets, n_iter, n_samples,
      error_margin, min_num_meas, ratio_threshold, stationary, in_ratio, is_valid);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_frontend_sync(const float* x_cc, const float* y_cc, const float* azimuth_sc,
                                const float* vr, const float* vr_compensated,
                                const int* scan_ptr, int n_scans, const int* scan_ref,
                                const double* mount, const double* odometry,
                                float gamma_stationary, int n_meas,
                                float* px, float* py, float* vx, float* vy,
                                uint8_t* stationary, void* stream) {
  RG_REQUIRE(n_scans >= 1 && n_meas >= 0, RG_ERR_ARG, "rg_frontend_sync: n_scans=%d n_meas=%d",
             n_scans, n_meas);
  if (n_meas == 0) return RG_OK;
  frontend_sync_kernel<<<ceil_div(n_meas, 256), 256, 0, (hipStream_t)stream>>>(
      x_cc, y_cc, azimuth_sc, vr, vr_compensated, scan_ptr, n_scans, scan_ref, mount, odometry,
      gamma_stationary, n_meas, px, py, vx, vy, stationary);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_frontend_labels_workspace_size(int n_tracks) {
  return ((size_t)(n_tracks + 1) * 2 * sizeof(double) + 255) / 256 * 256 +
         ((size_t)(n_tracks + 1) * sizeof(int) + 255) / 256 * 256;
}

extern "C" int rg_frontend_labels(const int* track_key, int n_tracks, const int64_t* label_id,
                                  const uint8_t* stationary, const int* old_to_new, int n_old,
                                  const float* px, const float* py, int n_meas, float* cls,
                                  float* offset_x, float* offset_y, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(n_tracks >= 0 && n_meas >= 0, RG_ERR_ARG, "rg_frontend_labels: bad sizes");
  RG_REQUIRE(workspace_bytes >= rg_frontend_labels_workspace_size(n_tracks), RG_ERR_ARG,
             "rg_frontend_labels: workspace too small");
  if (n_meas == 0) return RG_OK;
  double* tsum = (double*)workspace;
  int* tcnt = (int*)((char*)workspace +
                     ((size_t)(n_tracks + 1) * 2 * sizeof(double) + 255) / 256 * 256);
  RG_CHECK_HIP(hipMemsetAsync(workspace, 0, rg_frontend_labels_workspace_size(n_tracks), st));
  frontend_labels_kernel<<<ceil_div(n_meas, 256), 256, 0, st>>>(
      track_key, label_id, stationary, old_to_new, n_old, px, py, n_meas, cls, tsum, tcnt);
  frontend_offsets_kernel<<<ceil_div(n_meas, 256), 256, 0, st>>>(track_key, px, py, tsum, tcnt,
                                                                   n_meas, offset_x, offset_y);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" size_t rg_frontend_select_workspace_size(int n_meas) {
  return 2 * (((size_t)(n_meas + 1) * sizeof(int) + 255) / 256 * 256) +
         scan_workspace_bytes(n_meas);
}

extern "C" int rg_frontend_select(const float* px, const float* py, const float* cls, int n_meas,
                                  float min_x, float max_x, float min_y, float max_y,
                                  float static_id, const int* win_ptr, int n_windows,
                                  int* frame_ptr, int* index, int* n_selected, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RG_REQUIRE(workspace_bytes >= rg_frontend_select_workspace_size(n_meas), RG_ERR_ARG,
             "rg_frontend_select: workspace too small");
  if (n_meas == 0) {
    RG_CHECK_HIP(hipMemsetAsync(n_selected, 0, sizeof(int), st));
    return RG_OK;
  }
  const size_t arr = ((size_t)(n_meas + 1) * sizeof(int) + 255) / 256 * 256;
  int* keep = (int*)workspace;
  int* pos = (int*)((char*)workspace + arr);
  void* sws = (char*)workspace + 2 * arr;
  frontend_keep_kernel<<<ceil_div(n_meas, 256), 256, 0, st>>>(px, py, cls, min_x, max_x, min_y,
                                                                max_y, static_id, n_meas, keep);
  RG_LAUNCH_CHECK();
  int rc = exclusive_scan(keep, n_meas, pos, n_selected, sws, st);
  if (rc) return rc;
  frontend_index_kernel<<<ceil_div(n_meas, 256), 256, 0, st>>>(keep, pos, n_meas, index);
  if (win_ptr && frame_ptr)
    frontend_frame_ptr_kernel<<<ceil_div(n_windows + 1, 256), 256, 0, st>>>(pos, win_ptr,
                                                                             n_windows, frame_ptr);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
