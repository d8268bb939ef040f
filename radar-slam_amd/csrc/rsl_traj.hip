// rsl_traj.hip — trajectory reduction: device prefix scans of the per-frame ego-motion (fp64).
//
// Replaces (reference src/pose_integration/pose_integration.py):
//   integrate_translational_velocity :67-111 (trapezoidal / euler rule, before smoothing),
//   integrate_angular_velocity :113-167 (R_i = R_{i-1} * exp(omega_{i-1} dt_{i-1}), as quaternions),
//   smoothing uniform_filter1d(size, mode='nearest') :105-109.
//
// The sequential recurrences are associative, so each is a block-wide inclusive scan: positions are the prefix
// sum of the per-step increments, orientations the ordered prefix product of the per-step rotation quaternions
// (q_i = q_{i-1} (x) exp(omega_{i-1} dt / 2)).  One wave (k_traj_scan_wave, blocks up to 65536 frames) or one
// 1024-thread workgroup (k_traj_scan, longer blocks) scans one frame block: each thread
// reduces a contiguous chunk serially, the chunk totals are scanned in LDS, then each chunk is rewritten with
// its exclusive prefix.  Frames sharded over GPUs are stitched by rsl/traj.py from 16-double block summaries.
#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

struct Quat {
  double w, x, y, z;
};

RSL_DEV Quat qmul(const Quat& a, const Quat& b) {  // Hamilton product a (x) b
  return Quat{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
              a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x, a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}

// Rotation.from_rotvec(axis * angle) with the reference's |omega| > 1e-12 gate (pose_integration.py:139-151).
RSL_DEV Quat rotvec_quat(double wx, double wy, double wz, double dt) {
  const double m = sqrt(wx * wx + wy * wy + wz * wz);
  if (!(m > 1e-12)) return Quat{1.0, 0.0, 0.0, 0.0};
  const double ang = m * dt;
  const double s = sin(0.5 * ang) / m, c = cos(0.5 * ang);
  return Quat{c, wx * s, wy * s, wz * s};
}

constexpr int kTrajThreads = 1024;

// vel [F][vstride] (first nv components = v_x, v_y[, v_z]); om [F][ostride] (3 comps) nullable;
// ts [F] nullable (then uniform dt); method 0 = trapezoidal, 1 = euler.
// Outputs: pos [F][3] with pos[0] = 0, quat [F][4] (w, x, y, z) with quat[0] = identity,
// summary [16] = {pos[F-1] (3), quat[F-1] (4), v[F-1] (3), v[0] (3), omega[F-1] (3)}.
__global__ __launch_bounds__(kTrajThreads) void k_traj_scan(const double* __restrict__ vel, int vstride, int nv,
                                                             const double* __restrict__ om, int ostride,
                                                             const double* __restrict__ ts, double dt, long F,
                                                             int method, double* __restrict__ pos,
                                                             double* __restrict__ quat, double* __restrict__ summary) {
  __shared__ double sp[kTrajThreads][3];
  __shared__ double sq[kTrajThreads][4];
  const int t = threadIdx.x;
  const long per = (F + kTrajThreads - 1) / kTrajThreads;
  const long b = t * per, e = min(F, b + per);
  auto V = [&](long i, int a) -> double { return a < nv ? vel[i * vstride + a] : 0.0; };
  auto W = [&](long i, int a) -> double { return om ? om[i * ostride + a] : 0.0; };
  auto DT = [&](long i) -> double { return ts ? ts[i + 1] - ts[i] : dt; };  // np.diff(timestamps)[i]
  // pass 1: chunk totals (increments for frames i in [b, e), i >= 1 use step i-1 -> i)
  double p[3] = {0.0, 0.0, 0.0};
  Quat q{1.0, 0.0, 0.0, 0.0};
  for (long i = max(b, 1L); i < e; ++i) {
    const double d = DT(i - 1);
    for (int a = 0; a < 3; ++a)
      p[a] += method == 0 ? 0.5 * d * (V(i - 1, a) + V(i, a)) : d * V(i - 1, a);
    q = qmul(q, rotvec_quat(W(i - 1, 0), W(i - 1, 1), W(i - 1, 2), d));
  }
  for (int a = 0; a < 3; ++a) sp[t][a] = p[a];
  sq[t][0] = q.w;
  sq[t][1] = q.x;
  sq[t][2] = q.y;
  sq[t][3] = q.z;
  __syncthreads();
  // inclusive scan over chunks (Hillis-Steele; quaternion products keep left-to-right order)
  for (int off = 1; off < kTrajThreads; off <<= 1) {
    double pp[3] = {0.0, 0.0, 0.0};
    Quat qq{1.0, 0.0, 0.0, 0.0};
    const bool has = t >= off;
    if (has) {
      for (int a = 0; a < 3; ++a) pp[a] = sp[t - off][a];
      qq = Quat{sq[t - off][0], sq[t - off][1], sq[t - off][2], sq[t - off][3]};
    }
    __syncthreads();
    if (has) {
      for (int a = 0; a < 3; ++a) sp[t][a] += pp[a];
      const Quat cur{sq[t][0], sq[t][1], sq[t][2], sq[t][3]};
      const Quat r = qmul(qq, cur);
      sq[t][0] = r.w;
      sq[t][1] = r.x;
      sq[t][2] = r.y;
      sq[t][3] = r.z;
    }
    __syncthreads();
  }
  // pass 2: rewrite each chunk from its exclusive prefix
  double ep[3] = {0.0, 0.0, 0.0};
  Quat eq{1.0, 0.0, 0.0, 0.0};
  if (t > 0) {
    for (int a = 0; a < 3; ++a) ep[a] = sp[t - 1][a];
    eq = Quat{sq[t - 1][0], sq[t - 1][1], sq[t - 1][2], sq[t - 1][3]};
  }
  for (long i = b; i < e; ++i) {
    if (i >= 1) {
      const double d = DT(i - 1);
      for (int a = 0; a < 3; ++a) ep[a] += method == 0 ? 0.5 * d * (V(i - 1, a) + V(i, a)) : d * V(i - 1, a);
      eq = qmul(eq, rotvec_quat(W(i - 1, 0), W(i - 1, 1), W(i - 1, 2), d));
    }
    for (int a = 0; a < 3; ++a) pos[i * 3 + a] = ep[a];
    quat[i * 4 + 0] = eq.w;
    quat[i * 4 + 1] = eq.x;
    quat[i * 4 + 2] = eq.y;
    quat[i * 4 + 3] = eq.z;
  }
  if (t == kTrajThreads - 1 && summary) {
    for (int a = 0; a < 3; ++a) summary[a] = sp[t][a];
    for (int a = 0; a < 4; ++a) summary[3 + a] = sq[t][a];
    for (int a = 0; a < 3; ++a) {
      summary[7 + a] = V(F - 1, a);
      summary[10 + a] = V(0, a);
      summary[13 + a] = W(F - 1, a);
    }
  }
}

// The same scan by ONE wave (64 lanes, no LDS, no barrier), for blocks of up to kTrajWaveMax frames (the bench's
// 2000-frame batches): lane t reduces its contiguous chunk serially, the 64 chunk totals are scanned across lanes by
// __shfl_up (Hillis-Steele; quaternion products keep left-to-right order), then each chunk is rewritten from its
// exclusive prefix.  A 64-thread launch needs one free wave slot anywhere on the chip, so on a third stream it starts
// at once beside the other batch's kernels; the 1024-thread form waited for a whole CU to drain (k_traj_scan: 24 us
// to 5.7 ms in the r3f trace, 2.8 ms average).
constexpr long kTrajWaveMax = 1L << 16;
__global__ __launch_bounds__(64) void k_traj_scan_wave(const double* __restrict__ vel, int vstride, int nv,
                                                       const double* __restrict__ om, int ostride,
                                                       const double* __restrict__ ts, double dt, long F, int method,
                                                       double* __restrict__ pos, double* __restrict__ quat,
                                                       double* __restrict__ summary) {
  const int t = threadIdx.x;
  const long per = (F + 63) / 64;
  const long b = t * per, e = min(F, b + per);
  auto V = [&](long i, int a) -> double { return a < nv ? vel[i * vstride + a] : 0.0; };
  auto W = [&](long i, int a) -> double { return om ? om[i * ostride + a] : 0.0; };
  auto DT = [&](long i) -> double { return ts ? ts[i + 1] - ts[i] : dt; };  // np.diff(timestamps)[i]
  double p[3] = {0.0, 0.0, 0.0};
  Quat q{1.0, 0.0, 0.0, 0.0};
  for (long i = max(b, 1L); i < e; ++i) {
    const double d = DT(i - 1);
    for (int a = 0; a < 3; ++a) p[a] += method == 0 ? 0.5 * d * (V(i - 1, a) + V(i, a)) : d * V(i - 1, a);
    q = qmul(q, rotvec_quat(W(i - 1, 0), W(i - 1, 1), W(i - 1, 2), d));
  }
  // inclusive scan of the chunk totals across the wave
  for (int off = 1; off < 64; off <<= 1) {
    double pp[3];
    for (int a = 0; a < 3; ++a) pp[a] = __shfl_up(p[a], off);
    const Quat qq{__shfl_up(q.w, off), __shfl_up(q.x, off), __shfl_up(q.y, off), __shfl_up(q.z, off)};
    if (t >= off) {
      for (int a = 0; a < 3; ++a) p[a] += pp[a];
      q = qmul(qq, q);
    }
  }
  // exclusive prefix = the inclusive value of lane t - 1
  double ep[3];
  for (int a = 0; a < 3; ++a) ep[a] = __shfl_up(p[a], 1);
  Quat eq{__shfl_up(q.w, 1), __shfl_up(q.x, 1), __shfl_up(q.y, 1), __shfl_up(q.z, 1)};
  if (t == 0) {
    ep[0] = ep[1] = ep[2] = 0.0;
    eq = Quat{1.0, 0.0, 0.0, 0.0};
  }
  for (long i = b; i < e; ++i) {
    if (i >= 1) {
      const double d = DT(i - 1);
      for (int a = 0; a < 3; ++a) ep[a] += method == 0 ? 0.5 * d * (V(i - 1, a) + V(i, a)) : d * V(i - 1, a);
      eq = qmul(eq, rotvec_quat(W(i - 1, 0), W(i - 1, 1), W(i - 1, 2), d));
    }
    for (int a = 0; a < 3; ++a) pos[i * 3 + a] = ep[a];
    quat[i * 4 + 0] = eq.w;
    quat[i * 4 + 1] = eq.x;
    quat[i * 4 + 2] = eq.y;
    quat[i * 4 + 3] = eq.z;
  }
  if (t == 63 && summary) {
    for (int a = 0; a < 3; ++a) summary[a] = p[a];
    summary[3] = q.w;
    summary[4] = q.x;
    summary[5] = q.y;
    summary[6] = q.z;
    for (int a = 0; a < 3; ++a) {
      summary[7 + a] = V(F - 1, a);
      summary[10 + a] = V(0, a);
      summary[13 + a] = W(F - 1, a);
    }
  }
}

// pos[i] += base_p ; quat[i] = base_q (x) quat[i]   (base [7] device: p (3), q (4))
__global__ __launch_bounds__(256) void k_traj_apply(double* __restrict__ pos, double* __restrict__ quat, long F,
                                                    const double* __restrict__ base) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= F) return;
  for (int a = 0; a < 3; ++a) pos[i * 3 + a] += base[a];
  const Quat bq{base[3], base[4], base[5], base[6]};
  const Quat c{quat[i * 4], quat[i * 4 + 1], quat[i * 4 + 2], quat[i * 4 + 3]};
  const Quat r = qmul(bq, c);
  quat[i * 4] = r.w;
  quat[i * 4 + 1] = r.x;
  quat[i * 4 + 2] = r.y;
  quat[i * 4 + 3] = r.z;
}

// uniform_filter1d(x, size, mode='nearest') on each of the ncol columns of x [F][ncol] (scipy.ndimage):
// out[i] = mean of x[clamp(i + j)] for j in [-(size//2), size - size//2 - 1].
__global__ __launch_bounds__(256) void k_traj_smooth(const double* __restrict__ x, long F, int ncol, int size,
                                                     double* __restrict__ out) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= F * ncol) return;
  const long i = g / ncol;
  const int c = (int)(g - i * ncol);
  const int lo = -(size / 2), hi = size - size / 2 - 1;
  double s = 0.0;
  for (int j = lo; j <= hi; ++j) {
    long k = i + j;
    k = k < 0 ? 0 : (k >= F ? F - 1 : k);
    s += x[k * ncol + c];
  }
  out[g] = s / size;
}

// Block stitching (one thread): summaries [R][16] of consecutive frame blocks (rank order), running state
// [16] = {pos (3), quat (4), v_last (3), omega_last (3), started, -, -}.  Writes base [7] of block `rank` and
// advances the state past the last block (every rank computes the same state).
__global__ void k_traj_stitch(const double* __restrict__ summ, int R, int rank, double dt, int method,
                              double* __restrict__ state, double* __restrict__ base) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double p[3] = {state[0], state[1], state[2]};
  Quat q{state[3], state[4], state[5], state[6]};
  double vl[3] = {state[7], state[8], state[9]};
  double wl[3] = {state[10], state[11], state[12]};
  bool started = state[13] != 0.0;
  for (int r = 0; r < R; ++r) {
    const double* s = summ + 16 * r;
    if (started) {  // the step from the previous block's last frame to this block's first frame
      for (int a = 0; a < 3; ++a) p[a] += method == 0 ? 0.5 * dt * (vl[a] + s[10 + a]) : dt * vl[a];
      q = qmul(q, rotvec_quat(wl[0], wl[1], wl[2], dt));
    }
    if (r == rank) {
      for (int a = 0; a < 3; ++a) base[a] = p[a];
      base[3] = q.w;
      base[4] = q.x;
      base[5] = q.y;
      base[6] = q.z;
    }
    for (int a = 0; a < 3; ++a) p[a] += s[a];
    q = qmul(q, Quat{s[3], s[4], s[5], s[6]});
    for (int a = 0; a < 3; ++a) {
      vl[a] = s[7 + a];
      wl[a] = s[13 + a];
    }
    started = true;
  }
  for (int a = 0; a < 3; ++a) state[a] = p[a];
  state[3] = q.w;
  state[4] = q.x;
  state[5] = q.y;
  state[6] = q.z;
  for (int a = 0; a < 3; ++a) {
    state[7 + a] = vl[a];
    state[10 + a] = wl[a];
  }
  state[13] = 1.0;
}

hipError_t launch_traj_stitch(hipStream_t st, const double* summ, int R, int rank, double dt, int method,
                              double* state, double* base) {
  hipLaunchKernelGGL(k_traj_stitch, dim3(1), dim3(64), 0, st, summ, R, rank, dt, method, state, base);
  return hipGetLastError();
}

hipError_t launch_traj_scan(hipStream_t st, const double* vel, int vstride, int nv, const double* om, int ostride,
                            const double* ts, double dt, long F, int method, double* pos, double* quat,
                            double* summary) {
  if (F <= 0) return hipSuccess;
  if (F <= kTrajWaveMax) {
    hipLaunchKernelGGL(k_traj_scan_wave, dim3(1), dim3(64), 0, st, vel, vstride, nv, om, ostride, ts, dt, F, method,
                       pos, quat, summary);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_traj_scan, dim3(1), dim3(kTrajThreads), 0, st, vel, vstride, nv, om, ostride, ts, dt, F,
                     method, pos, quat, summary);
  return hipGetLastError();
}

hipError_t launch_traj_apply(hipStream_t st, double* pos, double* quat, long F, const double* base) {
  if (F <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_traj_apply, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, st, pos, quat, F, base);
  return hipGetLastError();
}

hipError_t launch_traj_smooth(hipStream_t st, const double* x, long F, int ncol, int size, double* out) {
  if (F <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_traj_smooth, dim3((unsigned)((F * ncol + 255) / 256)), dim3(256), 0, st, x, F, ncol, size,
                     out);
  return hipGetLastError();
}

}  // namespace rsl
