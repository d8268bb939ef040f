// rsl_scene.hip — the configs[3] per-frame call pattern on MI355X: per-cube peak selection for the
// robust DoA and the analyser's cross-frame association, batched over a whole sequence.
//
// Reference (results/ground_truth_comparison/radarscenes_complete_analysis.py):
//   per (frame, sensor) cube: extract_range_doppler_peaks(rds, threshold_db=-25) (:171) then
//   RobustAngleEstimator.process_targets_robust (:174-176), whose selection is
//     peaks = [p for p in peaks if p['power_db'] > -25.0]; peaks.sort(key=power_db, reverse=True);
//     peaks = peaks[:max_targets]                         (robust_angle_estimation.py:362-369)
//   -> k_topk_entries: one workgroup per cube, radix select of the max_targets-th largest key over the cube's peak
//      entries, then the selected entries sorted by (power desc, entry order asc) = Python's stable reverse sort;
//   per frame: _create_target_associations (:274-305): for every current target in order, the previous target with
//     the smallest sqrt((r - r')^2 + (az - az')^2) under a strict '<' against the running minimum AND '< 5.0'
//     (metres and radians mixed, no exclusion of used targets), and angle(s_cur[0] * conj(s_prev[0]))
//   -> k_associate_nearest: one thread per current target of every frame of the batch.
#include <climits>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

constexpr int kTopkThreads = 256;
constexpr int kTopkMax = 256;  // max_targets supported by the in-LDS sort

// Orderable key of an f32: larger float <=> larger unsigned key (NaN never occurs: dB of a finite power)
RSL_DEV unsigned f32_key(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Entries of cube k are [entry_base[k], entry_base[k + 1]) (the chain's global exclusive offsets, clamped to the
// capacity).  Outputs per cube k, slots k * kmax .. k * kmax + kmax - 1: the selected entries' global indices, their
// frame (= cube) and rc = range_bin * C + doppler_bin (a DoA cell list; unused slots hold cell (k, 0) and entry -1),
// and sel_n[k] = the number selected.
__global__ __launch_bounds__(kTopkThreads) void k_topk_entries(const long long* __restrict__ entry_base,
                                                              long long entry_cap, const unsigned* __restrict__ e_coord,
                                                              const float* __restrict__ e_pdb, float thr_db, int kmax,
                                                              int C, int* __restrict__ sel_entry,
                                                              int* __restrict__ sel_frame, int* __restrict__ sel_rc,
                                                              int* __restrict__ sel_n) {
  __shared__ int hist[256];
  __shared__ int s_cnt[kTopkThreads];
  __shared__ unsigned long long s_sort[kTopkMax];
  __shared__ unsigned s_prefix, s_need;
  const int t = threadIdx.x;
  const int k = blockIdx.x;
  long long b0 = entry_base[k], b1 = entry_base[k + 1];
  if (b0 > entry_cap) b0 = entry_cap;
  if (b1 > entry_cap) b1 = entry_cap;
  const long long n = b1 > b0 ? b1 - b0 : 0;
  // contiguous chunk per thread: thread order then chunk order = entry order (stable compaction below)
  const long long per = (n + kTopkThreads - 1) / kTopkThreads;
  const long long c0 = b0 + (long long)t * per;
  const long long c1 = min(b1, c0 + per);
  // valid entries: power_db > thr (robust_angle_estimation.py:362; the detection already applied this threshold, so
  // it removes nothing after extract_range_doppler_peaks(threshold_db = thr))
  int nvalid = 0;
  for (long long e = c0; e < c1; ++e) nvalid += e_pdb[e] > thr_db;
  s_cnt[t] = nvalid;
  if (t == 0) s_prefix = 0u;
  __syncthreads();
  int total = 0;
  for (int i = 0; i < kTopkThreads; ++i) total += s_cnt[i];  // LDS broadcast reads
  const int want = min(kmax, total);
  unsigned prefix = 0u, need = (unsigned)want;
  if (want > 0 && want < total) {
    // MSB-first radix select of the want-th largest key: 4 passes of 8-bit digits over the entries matching the prefix
    for (int d = 3; d >= 0; --d) {
      hist[t] = 0;
      __syncthreads();
      const unsigned hmask = d == 3 ? 0u : (0xFFFFFFFFu << (8 * (d + 1)));
      for (long long e = c0; e < c1; ++e) {
        const float v = e_pdb[e];
        if (!(v > thr_db)) continue;
        const unsigned key = f32_key(v);
        if ((key & hmask) == (prefix & hmask)) atomicAdd(&hist[(key >> (8 * d)) & 255u], 1);
      }
      __syncthreads();
      if (t == 0) {
        unsigned acc = 0u;
        int b = 255;
        for (; b > 0; --b) {
          if (acc + (unsigned)hist[b] >= need) break;
          acc += (unsigned)hist[b];
        }
        s_prefix = prefix | ((unsigned)b << (8 * d));
        s_need = need - acc;
      }
      __syncthreads();
      prefix = s_prefix;
      need = s_need;
      __syncthreads();
    }
  } else {
    prefix = 0u;  // everything valid is selected (key >= 0 for all)
    need = 0u;
  }
  // selected: key > T, plus the first `need` entries (entry order) with key == T (T = prefix when want < total)
  const bool all = !(want > 0 && want < total);
  int n_gt = 0, n_eq = 0;
  for (long long e = c0; e < c1; ++e) {
    const float v = e_pdb[e];
    if (!(v > thr_db)) continue;
    const unsigned key = f32_key(v);
    if (all || key > prefix) ++n_gt;
    else if (key == prefix) ++n_eq;
  }
  // exclusive scans of the per-thread counts (thread order = entry order)
  __syncthreads();
  s_cnt[t] = n_eq;
  __syncthreads();
  int eq_before = 0;
  for (int i = 0; i < t; ++i) eq_before += s_cnt[i];
  __syncthreads();
  const int eq_take = all ? 0 : max(0, min(n_eq, (int)need - eq_before));
  s_cnt[t] = n_gt + eq_take;
  __syncthreads();
  int slot = 0;
  for (int i = 0; i < t; ++i) slot += s_cnt[i];
  int taken_eq = 0;
  for (long long e = c0; e < c1; ++e) {
    const float v = e_pdb[e];
    if (!(v > thr_db)) continue;
    const unsigned key = f32_key(v);
    bool sel = all || key > prefix;
    if (!sel && key == prefix && taken_eq < eq_take) {
      sel = true;
      ++taken_eq;
    }
    if (sel) {
      // composite sort key: power descending, then entry order ascending (stable reverse sort)
      const unsigned idx = (unsigned)(e - b0);
      s_sort[slot++] = ((unsigned long long)key << 32) | (0xFFFFFFFFu - idx);
    }
  }
  __syncthreads();
  // bitonic sort (descending) of the want selected keys, padded with zeros to kTopkMax
  for (int i = want + t; i < kTopkMax; i += kTopkThreads) s_sort[i] = 0ull;
  __syncthreads();
  for (int size = 2; size <= kTopkMax; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < kTopkMax; i += kTopkThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const unsigned long long a = s_sort[i], b = s_sort[j];
          const bool desc = (i & size) == 0;
          if (desc ? (a < b) : (a > b)) {
            s_sort[i] = b;
            s_sort[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int r = t; r < kmax; r += kTopkThreads) {
    const size_t o = (size_t)k * kmax + r;
    if (r < want) {
      const long long e = b0 + (long long)(0xFFFFFFFFu - (unsigned)(s_sort[r] & 0xFFFFFFFFull));
      const unsigned cd = e_coord[e];
      sel_entry[o] = (int)e;
      sel_frame[o] = k;
      sel_rc[o] = (int)(((cd >> 13) & 0x1FFFu) * (unsigned)C + (cd & 0x1FFFu));
    } else {
      sel_entry[o] = -1;
      sel_frame[o] = k;
      sel_rc[o] = 0;
    }
  }
  if (t == 0) sel_n[k] = want;
}

hipError_t launch_topk_entries(hipStream_t st, const long long* entry_base, long long entry_cap, int ncube,
                               const unsigned* e_coord, const float* e_pdb, float thr_db, int kmax, int C,
                               int* sel_entry, int* sel_frame, int* sel_rc, int* sel_n) {
  if (ncube <= 0) return hipSuccess;
  if (kmax < 1 || kmax > kTopkMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_topk_entries, dim3((unsigned)ncube), dim3(kTopkThreads), 0, st, entry_base, entry_cap, e_coord,
                     e_pdb, thr_db, kmax, C, sel_entry, sel_frame, sel_rc, sel_n);
  return hipGetLastError();
}

// One thread per current target i of frame f (targets of frame f are [off[f], off[f + 1]) in the concatenated
// arrays; the previous frame's are [off[f - 1], off[f]); frame 0 has no previous frame).  Exact float64 arithmetic in
// the reference's operation order (no FMA contraction): range_diff**2 + azimuth_diff**2, sqrt, strict '<'.
__global__ __launch_bounds__(256) void k_associate_nearest(const double* __restrict__ range_m,
                                                           const double* __restrict__ az_rad,
                                                           const double2* __restrict__ s0, const long long* __restrict__ off,
                                                           int nframes, double thr, int* __restrict__ match,
                                                           double* __restrict__ dist, double* __restrict__ phase) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n = off[nframes];
  if (i >= n) return;
  // frame of target i: binary search over the offsets
  int lo = 0, hi = nframes - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  const int f = lo;
  int bj = -1;
  double bd = INFINITY;
  if (f > 0) {
    const double r = range_m[i], a = az_rad[i];
    for (long long j = off[f - 1]; j < off[f]; ++j) {
      const double dr = __dsub_rn(r, range_m[j]), da = __dsub_rn(a, az_rad[j]);
      const double d = __dsqrt_rn(__dadd_rn(__dmul_rn(dr, dr), __dmul_rn(da, da)));
      if (d < bd && d < thr) {
        bd = d;
        bj = (int)(j - off[f - 1]);
      }
    }
  }
  match[i] = bj;
  dist[i] = bd;
  if (bj >= 0) {
    // angle(c * conj(p)) of the two targets' first signature components (radarscenes_complete_analysis.py:296)
    const double2 c = s0[i], p = s0[off[f - 1] + bj];
    const double re = __dadd_rn(__dmul_rn(c.x, p.x), __dmul_rn(c.y, p.y));
    const double im = __dsub_rn(__dmul_rn(c.y, p.x), __dmul_rn(c.x, p.y));
    phase[i] = atan2(im, re);
  } else {
    phase[i] = 0.0;
  }
}

hipError_t launch_associate_nearest(hipStream_t st, const double* range_m, const double* az_rad, const double2* s0,
                                    const long long* off, int nframes, long long ntargets, double thr, int* match,
                                    double* dist, double* phase) {
  if (nframes <= 0 || ntargets <= 0) return hipSuccess;
  const long long nb = (ntargets + 255) / 256;
  hipLaunchKernelGGL(k_associate_nearest, dim3((unsigned)nb), dim3(256), 0, st, range_m, az_rad, s0, off, nframes,
                     thr, match, dist, phase);
  return hipGetLastError();
}

}  // namespace rsl
