// rsl_eval.hip — pose-error evaluation (APE / RTE with Umeyama alignment) on the device, fp64.  gfx950.
//
// Replaces evaluation/compute_pose_error.py of the reference (PoseErrorEvaluator.align_trajectories :51-96,
// _umeyama_alignment :98-140, _align_orientations :142-169, compute_ape :171-236, compute_rte :238-306,
// _find_segment_end :308-322, _compute_relative_transformation :324-343, _compute_transformation_error :345-361).
// Poses are f64 [N][7] = (x, y, z, q0, q1, q2, q3); the reference reads q as scipy quaternions (scalar LAST,
// Rotation.from_quat normalises them), whatever its docstring says, and so does this file.
//
// Work per pose is a handful of 3x3 / quaternion products: every kernel is a streaming pass over the pose arrays
// (56 B per pose per array) or a block reduction of fp64 partials, so the evaluation is HBM / latency bound and
// O(N); the only serial work is one 3x3 SVD (one-sided Jacobi) and one 4x4 symmetric eigenproblem (cyclic Jacobi)
// per alignment, in one thread.
#include <cmath>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

namespace {
constexpr int kPeThreads = 256;

struct Q {  // scipy order: x, y, z, w
  double x, y, z, w;
};
RSL_DEV Q qnorm(Q a) {
  const double n = sqrt(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w);
  return {a.x / n, a.y / n, a.z / n, a.w / n};
}
RSL_DEV Q qmul(Q p, Q q) {  // Hamilton product p (x) q = scipy Rotation p * q
  return {p.w * q.x + q.w * p.x + (p.y * q.z - p.z * q.y), p.w * q.y + q.w * p.y + (p.z * q.x - p.x * q.z),
          p.w * q.z + q.w * p.z + (p.x * q.y - p.y * q.x), p.w * q.w - (p.x * q.x + p.y * q.y + p.z * q.z)};
}
RSL_DEV Q qinv(Q a) { return {-a.x, -a.y, -a.z, a.w}; }
RSL_DEV void qmat(Q q, double (&m)[3][3]) {  // unit quaternion -> rotation matrix
  const double x = q.x, y = q.y, z = q.z, w = q.w;
  m[0][0] = 1 - 2 * (y * y + z * z); m[0][1] = 2 * (x * y - z * w); m[0][2] = 2 * (x * z + y * w);
  m[1][0] = 2 * (x * y + z * w); m[1][1] = 1 - 2 * (x * x + z * z); m[1][2] = 2 * (y * z - x * w);
  m[2][0] = 2 * (x * z - y * w); m[2][1] = 2 * (y * z + x * w); m[2][2] = 1 - 2 * (x * x + y * y);
}
RSL_DEV Q load_q(const double* p) { return qnorm({p[3], p[4], p[5], p[6]}); }

// Block sum of K doubles per thread into part[blockIdx.x * K + k] (wave shuffles, then LDS).
template <int K>
RSL_DEV void block_sum(double (&v)[K], double* part) {
  __shared__ double red[kPeThreads / 64][K];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double x = v[k];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
    if (lane == 0) red[w][k] = x;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += kPeThreads) {
    double s = 0;
#pragma unroll
    for (int j = 0; j < kPeThreads / 64; ++j) s += red[j][k];
    part[(size_t)blockIdx.x * K + k] = s;
  }
}

// Every thread: the sum over NB blocks of the K partials (NB <= a few hundred: a redundant read per block).
template <int K>
RSL_DEV void sum_parts(const double* part, int nb, double (&out)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = 0;
  for (int b = 0; b < nb; ++b)
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] += part[(size_t)b * K + k];
}

// Pass 1: sums of the estimated and ground-truth positions (means of :112-113).
__global__ __launch_bounds__(kPeThreads) void k_pe_sums(const double* __restrict__ est,
                                                        const double* __restrict__ gt, long n,
                                                        double* __restrict__ part) {
  double v[6] = {0, 0, 0, 0, 0, 0};
  for (long i = blockIdx.x * (long)kPeThreads + threadIdx.x; i < n; i += (long)gridDim.x * kPeThreads) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[k] += est[7 * i + k];
      v[3 + k] += gt[7 * i + k];
    }
  }
  block_sum<6>(v, part);
}

// Pass 2: centred cross-covariance H = S_c^T T_c (:116) and the quaternion-mean matrix K = sum r r^T of the relative
// rotations r = gt (x) est^-1 (:160-163, Rotation.mean).
__global__ __launch_bounds__(kPeThreads) void k_pe_moments(const double* __restrict__ est,
                                                           const double* __restrict__ gt, long n,
                                                           const double* __restrict__ part1, int nb,
                                                           double* __restrict__ part) {
  double m[6];
  sum_parts<6>(part1, nb, m);
#pragma unroll
  for (int k = 0; k < 6; ++k) m[k] /= (double)n;
  double v[19];
#pragma unroll
  for (int k = 0; k < 19; ++k) v[k] = 0;
  for (long i = blockIdx.x * (long)kPeThreads + threadIdx.x; i < n; i += (long)gridDim.x * kPeThreads) {
    double s[3], t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      s[k] = est[7 * i + k] - m[k];
      t[k] = gt[7 * i + k] - m[3 + k];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) v[3 * a + b] += s[a] * t[b];
    const Q r = qmul(load_q(gt + 7 * i), qinv(load_q(est + 7 * i)));
    const double q4[4] = {r.x, r.y, r.z, r.w};
    int o = 9;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = a; b < 4; ++b) v[o++] += q4[a] * q4[b];
  }
  block_sum<19>(v, part);
}

// 3x3 SVD H = U diag(s) V^T by one-sided Jacobi on the columns of H; singular values in descending order.
RSL_DEV void svd3(const double (&H)[3][3], double (&U)[3][3], double (&s)[3], double (&V)[3][3]) {
  double A[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      A[i][j] = H[i][j];
      V[i][j] = i == j ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      double al = 0, be = 0, ga = 0;
      for (int i = 0; i < 3; ++i) {
        al += A[i][p] * A[i][p];
        be += A[i][q] * A[i][q];
        ga += A[i][p] * A[i][q];
      }
      if (ga == 0.0) continue;
      const double den = sqrt(al * be);
      if (den > 0) off = fmax(off, fabs(ga) / den);
      if (fabs(ga) <= 1e-17 * den) continue;
      const double zeta = (be - al) / (2 * ga);
      const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
      const double c = 1 / sqrt(1 + t * t), sn = c * t;
      for (int i = 0; i < 3; ++i) {
        const double ap = A[i][p], aq = A[i][q];
        A[i][p] = c * ap - sn * aq;
        A[i][q] = sn * ap + c * aq;
        const double vp = V[i][p], vq = V[i][q];
        V[i][p] = c * vp - sn * vq;
        V[i][q] = sn * vp + c * vq;
      }
    }
    if (off < 1e-16) break;
  }
  double sv[3];
  for (int j = 0; j < 3; ++j) sv[j] = sqrt(A[0][j] * A[0][j] + A[1][j] * A[1][j] + A[2][j] * A[2][j]);
  int o[3] = {0, 1, 2};  // descending order of the singular values
  for (int a = 0; a < 3; ++a)
    for (int b = a + 1; b < 3; ++b)
      if (sv[o[b]] > sv[o[a]]) {
        const int tmp = o[a];
        o[a] = o[b];
        o[b] = tmp;
      }
  double Vs[3][3];
  for (int k = 0; k < 3; ++k) {
    s[k] = sv[o[k]];
    for (int i = 0; i < 3; ++i) {
      Vs[i][k] = V[i][o[k]];
      U[i][k] = s[k] > 0 ? A[i][o[k]] / s[k] : 0.0;
    }
  }
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) V[i][k] = Vs[i][k];
  const double tiny = 1e-13 * (s[0] > 0 ? s[0] : 1.0);
  if (!(s[0] > 0)) {  // H = 0: U = I
    for (int i = 0; i < 3; ++i)
      for (int k = 0; k < 3; ++k) U[i][k] = i == k ? 1.0 : 0.0;
  } else {
    if (!(s[1] > tiny)) {  // rank 1: complete U with a unit vector orthogonal to u0
      double e[3] = {0, 0, 0};
      const int m = fabs(U[0][0]) < fabs(U[1][0]) ? (fabs(U[0][0]) < fabs(U[2][0]) ? 0 : 2)
                                                  : (fabs(U[1][0]) < fabs(U[2][0]) ? 1 : 2);
      e[m] = 1.0;
      double d = 0;
      for (int i = 0; i < 3; ++i) d += e[i] * U[i][0];
      double nn = 0;
      for (int i = 0; i < 3; ++i) {
        U[i][1] = e[i] - d * U[i][0];
        nn += U[i][1] * U[i][1];
      }
      nn = sqrt(nn);
      for (int i = 0; i < 3; ++i) U[i][1] /= nn;
    }
    if (!(s[2] > tiny)) {  // rank <= 2: u2 = u0 x u1 (its sign is fixed by the det correction below)
      U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
      U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
      U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
    }
  }
}

RSL_DEV double det3(const double (&R)[3][3]) {
  return R[0][0] * (R[1][1] * R[2][2] - R[1][2] * R[2][1]) - R[0][1] * (R[1][0] * R[2][2] - R[1][2] * R[2][0]) +
         R[0][2] * (R[1][0] * R[2][1] - R[1][1] * R[2][0]);
}

// Largest-eigenvalue eigenvector of a symmetric 4x4 (cyclic Jacobi, fp64).
RSL_DEV void eig4_top(double (&K)[4][4], double (&v)[4]) {
  double E[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) E[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0, diag = 0;
    for (int i = 0; i < 4; ++i) {
      diag += K[i][i] * K[i][i];
      for (int j = i + 1; j < 4; ++j) off += K[i][j] * K[i][j];
    }
    if (off <= 1e-32 * diag || off == 0.0) break;
    for (int p = 0; p < 3; ++p)
      for (int q = p + 1; q < 4; ++q) {
        if (K[p][q] == 0.0) continue;
        const double th = (K[q][q] - K[p][p]) / (2 * K[p][q]);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
        const double c = 1 / sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 4; ++k) {  // K <- J^T K J
          const double kp = K[k][p], kq = K[k][q];
          K[k][p] = c * kp - s * kq;
          K[k][q] = s * kp + c * kq;
        }
        for (int k = 0; k < 4; ++k) {
          const double kp = K[p][k], kq = K[q][k];
          K[p][k] = c * kp - s * kq;
          K[q][k] = s * kp + c * kq;
        }
        for (int k = 0; k < 4; ++k) {
          const double ep = E[k][p], eq = E[k][q];
          E[k][p] = c * ep - s * eq;
          E[k][q] = s * ep + c * eq;
        }
      }
  }
  int best = 0;
  for (int i = 1; i < 4; ++i)
    if (K[i][i] > K[best][best]) best = i;
  double n = 0;
  for (int k = 0; k < 4; ++k) n += E[k][best] * E[k][best];
  n = sqrt(n);
  const double sg = E[3][best] < 0 ? -1.0 : 1.0;  // canonical sign: w >= 0 (the reference's is LAPACK's choice)
  for (int k = 0; k < 4; ++k) v[k] = sg * E[k][best] / n;
}

// Solve the alignment: align f64 [32] = R (9, row-major), t (3), Rq (9), qbar (4, x y z w), scale (1), means (6).
__global__ void k_pe_solve(const double* __restrict__ part1, const double* __restrict__ part2, int nb, long n,
                           double* __restrict__ align) {
  if (threadIdx.x != 0) return;
  double m[6], v[19];
  sum_parts<6>(part1, nb, m);
  sum_parts<19>(part2, nb, v);
  for (int k = 0; k < 6; ++k) m[k] /= (double)n;
  double H[3][3], U[3][3], s[3], V[3][3], R[3][3];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) H[a][b] = v[3 * a + b];
  svd3(H, U, s, V);
  for (int pass = 0; pass < 2; ++pass) {  // R = Vt.T @ U.T; det < 0 -> Vt[-1, :] *= -1 (:121-127)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R[i][j] = V[i][0] * U[j][0] + V[i][1] * U[j][1] + V[i][2] * U[j][2];
    if (pass == 0 && det3(R) < 0) {
      for (int i = 0; i < 3; ++i) V[i][2] = -V[i][2];
    } else {
      break;
    }
  }
  double K[4][4];
  int o = 9;
  for (int a = 0; a < 4; ++a)
    for (int b = a; b < 4; ++b) K[a][b] = K[b][a] = v[o++];
  double qb[4];
  eig4_top(K, qb);
  double Rq[3][3];
  qmat({qb[0], qb[1], qb[2], qb[3]}, Rq);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      align[3 * i + j] = R[i][j];
      align[12 + 3 * i + j] = Rq[i][j];
    }
  for (int i = 0; i < 3; ++i) align[9 + i] = m[3 + i] - (R[i][0] * m[0] + R[i][1] * m[1] + R[i][2] * m[2]);
  for (int k = 0; k < 4; ++k) align[21 + k] = qb[k];
  align[25] = cbrt(det3(R));  // alignment_info['scale_factor'] (:89)
  for (int k = 0; k < 6; ++k) align[26 + k] = m[k];
}

// Apply the alignment (:133, :166) and the APE errors (:195-209): aligned f64 [N][7] (quaternion scalar last, as
// Rotation.as_quat), err f64 [3][N] = position, orientation (rotation angle of gt (x) aligned^-1), combined.
__global__ __launch_bounds__(kPeThreads) void k_pe_apply(const double* __restrict__ est,
                                                         const double* __restrict__ gt, long n,
                                                         const double* __restrict__ align,
                                                         double* __restrict__ aligned, double* __restrict__ err) {
  const long i = blockIdx.x * (long)kPeThreads + threadIdx.x;
  if (i >= n) return;
  double R[9], t[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = align[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = align[9 + k];
  const Q qb = {align[21], align[22], align[23], align[24]};
  const double* e = est + 7 * i;
  const double* g = gt + 7 * i;
  double p[3], d2 = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    p[a] = R[3 * a] * e[0] + R[3 * a + 1] * e[1] + R[3 * a + 2] * e[2] + t[a];
    const double d = p[a] - g[a];
    d2 += d * d;
  }
  const Q aq = qmul(load_q(e), qb);
  const Q rel = qmul(load_q(g), qinv(aq));
  const double ang = 2 * atan2(sqrt(rel.x * rel.x + rel.y * rel.y + rel.z * rel.z), fabs(rel.w));
  double* o = aligned + 7 * i;
  o[0] = p[0];
  o[1] = p[1];
  o[2] = p[2];
  o[3] = aq.x;
  o[4] = aq.y;
  o[5] = aq.z;
  o[6] = aq.w;
  const double pe = sqrt(d2);
  err[i] = pe;
  err[n + i] = ang;
  err[2 * n + i] = sqrt(pe * pe + ang * ang);
}

// Travelled distance of the aligned estimate, d[0] = 0, d[i] = sum_{k<i} |p_{k+1} - p_k| (:261-262): one block,
// each thread a contiguous chunk, exclusive scan of the chunk sums.
__global__ __launch_bounds__(1024) void k_pe_distance(const double* __restrict__ aligned, long n,
                                                      double* __restrict__ d) {
  __shared__ double sc[1024];
  const int t = threadIdx.x;
  const long per = (n + 1023) / 1024;
  const long b = t * per, e = b + per < n ? b + per : n;
  auto step = [&](long k) {  // |p_{k+1} - p_k|
    const double* p = aligned + 7 * k;
    const double dx = p[7] - p[0], dy = p[8] - p[1], dz = p[9] - p[2];
    return sqrt(dx * dx + dy * dy + dz * dz);
  };
  double s = 0;
  for (long k = b; k < e; ++k)
    if (k + 1 < n) s += step(k);
  sc[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const double v = t >= off ? sc[t - off] : 0.0;
    __syncthreads();
    sc[t] += v;
    __syncthreads();
  }
  double run = sc[t] - s;
  for (long k = b; k < e; ++k) {
    d[k] = run;
    if (k + 1 < n) run += step(k);
  }
}

// RTE errors (:270-292) for segment length L = len[l]: start i is valid when searchsorted(d, d[i] + L) < n and > i
// (for L > 0: d[i] + L <= d[n-1], a prefix of the starts); err[l][i] = sqrt(|t_err|^2 + |R1^T R2 - I|_F^2) with
// R1 / R2 = the relative rotations of the aligned estimate / ground truth and t_err their translation difference
// (= the norm of inv(T1) T2's translation).  cnt[l] = number of valid starts (the valid prefix's length).
__global__ __launch_bounds__(kPeThreads) void k_pe_rte(const double* __restrict__ aligned,
                                                       const double* __restrict__ gt, long n,
                                                       const double* __restrict__ d,
                                                       const double* __restrict__ len, double* __restrict__ err,
                                                       unsigned long long* __restrict__ cnt) {
  const int l = blockIdx.y;
  const long i = blockIdx.x * (long)kPeThreads + threadIdx.x;
  const double L = len[l];
  bool ok = false;
  long end = 0;
  if (i < n) {
    const double target = d[i] + L;
    long lo = 0, hi = n;  // first index with d >= target (numpy searchsorted, side 'left')
    while (lo < hi) {
      const long mid = (lo + hi) >> 1;
      if (d[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    end = lo;
    ok = end < n && end > i;
  }
  if (ok) {
    const double* a0 = aligned + 7 * i;
    const double* a1 = aligned + 7 * end;
    const double* g0 = gt + 7 * i;
    const double* g1 = gt + 7 * end;
    double dt2 = 0;
    for (int k = 0; k < 3; ++k) {
      const double dd = (g1[k] - g0[k]) - (a1[k] - a0[k]);
      dt2 += dd * dd;
    }
    double Ma[3][3], Mb[3][3], Ga[3][3], Gb[3][3];
    qmat(load_q(a0), Ma);
    qmat(load_q(a1), Mb);
    qmat(load_q(g0), Ga);
    qmat(load_q(g1), Gb);
    double R1[3][3], R2[3][3];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        R1[r][c] = Mb[r][0] * Ma[c][0] + Mb[r][1] * Ma[c][1] + Mb[r][2] * Ma[c][2];  // rot2 * rot1.inv()
        R2[r][c] = Gb[r][0] * Ga[c][0] + Gb[r][1] * Ga[c][1] + Gb[r][2] * Ga[c][2];
      }
    double re = 0;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        const double x = R1[0][r] * R2[0][c] + R1[1][r] * R2[1][c] + R1[2][r] * R2[2][c] - (r == c ? 1.0 : 0.0);
        re += x * x;
      }
    err[(size_t)l * n + i] = sqrt(dt2 + re);
  }
  const unsigned long long b = __ballot(ok);
  if ((threadIdx.x & 63) == 0 && b) atomicMax(cnt + l, (unsigned long long)(i - (threadIdx.x & 63)) + 64 - __clzll(b));
}

// Statistics of nser series (series s = x[s * stride .. + len_s), len_s = lens ? lens[s] : n) (:216-227, :296-301):
// pass 1 per-block sum, sum of squares and max; pass 2 sum of squared deviations from the mean; final per series
// {rmse, mean, std (population, as np.std), max, count}.
__global__ __launch_bounds__(kPeThreads) void k_pe_stats1(const double* __restrict__ x, long stride, long n,
                                                          const unsigned long long* __restrict__ lens,
                                                          double* __restrict__ part) {
  const int s = blockIdx.y;
  const long m = lens ? (long)lens[s] : n;
  double v[2] = {0, 0};
  double mx = -INFINITY;
  for (long i = blockIdx.x * (long)kPeThreads + threadIdx.x; i < m; i += (long)gridDim.x * kPeThreads) {
    const double a = x[(size_t)s * stride + i];
    v[0] += a;
    v[1] += a * a;
    mx = fmax(mx, a);
  }
  __shared__ double red[kPeThreads / 64][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    v[0] += __shfl_xor(v[0], d);
    v[1] += __shfl_xor(v[1], d);
    mx = fmax(mx, __shfl_xor(mx, d));
  }
  if (lane == 0) {
    red[w][0] = v[0];
    red[w][1] = v[1];
    red[w][2] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0, c = -INFINITY;
    for (int j = 0; j < kPeThreads / 64; ++j) {
      a += red[j][0];
      b += red[j][1];
      c = fmax(c, red[j][2]);
    }
    double* o = part + ((size_t)s * gridDim.x + blockIdx.x) * 4;
    o[0] = a;
    o[1] = b;
    o[2] = c;
  }
}

__global__ __launch_bounds__(kPeThreads) void k_pe_stats2(const double* __restrict__ x, long stride, long n,
                                                          const unsigned long long* __restrict__ lens,
                                                          double* __restrict__ part) {
  const int s = blockIdx.y;
  const long m = lens ? (long)lens[s] : n;
  double mean = 0;
  for (unsigned b = 0; b < gridDim.x; ++b) mean += part[((size_t)s * gridDim.x + b) * 4];
  mean = m > 0 ? mean / (double)m : 0.0;
  double v[1] = {0};
  for (long i = blockIdx.x * (long)kPeThreads + threadIdx.x; i < m; i += (long)gridDim.x * kPeThreads) {
    const double a = x[(size_t)s * stride + i] - mean;
    v[0] += a * a;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v[0] += __shfl_xor(v[0], d);
  __shared__ double red[kPeThreads / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v[0];
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0;
    for (int j = 0; j < kPeThreads / 64; ++j) a += red[j];
    part[((size_t)s * gridDim.x + blockIdx.x) * 4 + 3] = a;
  }
}

__global__ void k_pe_stats3(const double* __restrict__ part, int nb, long n,
                            const unsigned long long* __restrict__ lens, double* __restrict__ stats) {
  const int s = threadIdx.x;
  if (s >= (int)blockDim.x) return;
  const long m = lens ? (long)lens[s] : n;
  double a = 0, b = 0, c = -INFINITY, dv = 0;
  for (int k = 0; k < nb; ++k) {
    const double* p = part + ((size_t)s * nb + k) * 4;
    a += p[0];
    b += p[1];
    c = fmax(c, p[2]);
    dv += p[3];
  }
  double* o = stats + 5 * s;
  const double mm = m > 0 ? (double)m : 1.0;
  o[0] = sqrt(b / mm);
  o[1] = a / mm;
  o[2] = sqrt(dv / mm);
  o[3] = c;
  o[4] = (double)m;
}

int pe_blocks(long n) {
  long b = (n + kPeThreads - 1) / kPeThreads;
  if (b > 256) b = 256;
  return (int)(b < 1 ? 1 : b);
}
}  // namespace

long long pose_error_scratch_doubles(long long n, int nlen) {
  // partials: sums 256 x 6, moments 256 x 19, stats 256 x 4 x max(3, nlen); distance n
  const long long ns = nlen > 3 ? nlen : 3;
  return 256LL * 6 + 256LL * 19 + 256LL * 4 * ns + n + 64;
}

hipError_t launch_pose_align(hipStream_t st, const double* est, const double* gt, long n, double* scratch,
                             double* align, double* aligned, double* ape_err, double* ape_stats) {
  const int nb = pe_blocks(n);
  double* p1 = scratch;
  double* p2 = p1 + 256 * 6;
  double* ps = p2 + 256 * 19;
  hipLaunchKernelGGL(k_pe_sums, dim3(nb), dim3(kPeThreads), 0, st, est, gt, n, p1);
  hipLaunchKernelGGL(k_pe_moments, dim3(nb), dim3(kPeThreads), 0, st, est, gt, n, p1, nb, p2);
  hipLaunchKernelGGL(k_pe_solve, dim3(1), dim3(64), 0, st, p1, p2, nb, n, align);
  hipLaunchKernelGGL(k_pe_apply, dim3((unsigned)((n + kPeThreads - 1) / kPeThreads)), dim3(kPeThreads), 0, st, est,
                     gt, n, align, aligned, ape_err);
  if (ape_stats) {
    hipLaunchKernelGGL(k_pe_stats1, dim3(nb, 3), dim3(kPeThreads), 0, st, ape_err, n, n, nullptr, ps);
    hipLaunchKernelGGL(k_pe_stats2, dim3(nb, 3), dim3(kPeThreads), 0, st, ape_err, n, n, nullptr, ps);
    hipLaunchKernelGGL(k_pe_stats3, dim3(1), dim3(3), 0, st, ps, nb, n, nullptr, ape_stats);
  }
  return hipGetLastError();
}

hipError_t launch_pose_rte(hipStream_t st, const double* aligned, const double* gt, long n, const double* len,
                           int nlen, double* scratch, double* err, unsigned long long* cnt, double* stats) {
  const int nb = pe_blocks(n);
  double* ps = scratch + 256 * 6 + 256 * 19;
  double* d = ps + 256 * 4 * (nlen > 3 ? nlen : 3);
  hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * nlen, st);
  hipLaunchKernelGGL(k_pe_distance, dim3(1), dim3(1024), 0, st, aligned, n, d);
  hipLaunchKernelGGL(k_pe_rte, dim3((unsigned)((n + kPeThreads - 1) / kPeThreads), nlen), dim3(kPeThreads), 0, st,
                     aligned, gt, n, d, len, err, cnt);
  hipLaunchKernelGGL(k_pe_stats1, dim3(nb, nlen), dim3(kPeThreads), 0, st, err, n, n, cnt, ps);
  hipLaunchKernelGGL(k_pe_stats2, dim3(nb, nlen), dim3(kPeThreads), 0, st, err, n, n, cnt, ps);
  hipLaunchKernelGGL(k_pe_stats3, dim3(1), dim3(nlen), 0, st, ps, nb, n, cnt, stats);
  return hipGetLastError();
}

}  // namespace rsl
