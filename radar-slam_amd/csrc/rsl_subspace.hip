// rsl_subspace.hip — MUSIC and ESPRIT with an arbitrary num_sources (reference angle_estimation.py:109-154,
// :178-225 with num_sources != 1), fp64.  gfx950.
//
// The reference's covariance is rank-1 (R = s s^H, :127), so its eigenvectors are s (eigenvalue |s|^2) and ANY
// orthonormal basis of s-perp (eigenvalue 0, ordered by LAPACK round-off).  With num_sources = 1 that freedom cancels
// (den = |a|^2 - |a^H s|^2 / |s|^2, the closed form of the batched path); with num_sources = K != 1 the noise subspace
// V[:, K:] mixes s-perp vectors that LAPACK picks by round-off, so the reference's spectrum for 2 <= K < M is not a
// function of s alone.  This file fixes the basis deterministically: V = [s / |s|, the Householder completion of s]
// (P e_j, P the reflector with P s = alpha e_1), so |a^H v_j| = |(P a)_j| and den(K) = sum over the noise columns of
// |(P a)_j|^2.  Every case the reference determines is reproduced: K = 1 (closed form), K >= M (no noise subspace:
// den = 0, spectrum 0), a zero signature (eigh(0) = identity, descending order = reversed columns), negative K
// (Python slicing: the last -K columns).  ESPRIT: U = [left singular vectors of X = [s[:-1], s[1:]] in descending
// order, their Householder completion], Us = U[:, :K] (Python slicing), Phi = pinv(Us[:-1]) Us[1:], and the angle
// of Phi's first eigenvalue; an empty Phi raises in the reference (IndexError on eigvals(...)[0]) and returns 0.0.
// The first eigenvalue's order is LAPACK's for K >= 2; here it is the first diagonal entry of the Schur form from
// a Wilkinson-shifted complex QR iteration on Phi.  One thread per (cell, grid point) or per cell:
// these are per-call drop-in paths (estimate_angle_music / _esprit with num_sources != 1), not the batched chain.
#include <cmath>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

namespace {
constexpr int kMaxM = 16;

struct Z {
  double r, i;
};
RSL_DEV Z zmul(Z a, Z b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
RSL_DEV Z zcmul(Z a, Z b) { return {a.r * b.r + a.i * b.i, a.r * b.i - a.i * b.r}; }  // conj(a) b
RSL_DEV Z zadd(Z a, Z b) { return {a.r + b.r, a.i + b.i}; }
RSL_DEV Z zsub(Z a, Z b) { return {a.r - b.r, a.i - b.i}; }
RSL_DEV Z zscale(Z a, double s) { return {a.r * s, a.i * s}; }
RSL_DEV double zabs2(Z a) { return a.r * a.r + a.i * a.i; }
RSL_DEV Z zdiv(Z a, Z b) {
  const double d = b.r * b.r + b.i * b.i;
  return {(a.r * b.r + a.i * b.i) / d, (a.i * b.r - a.r * b.i) / d};
}
RSL_DEV Z zsqrt(Z a) {
  const double m = sqrt(sqrt(zabs2(a)));
  const double th = 0.5 * atan2(a.i, a.r);
  return {m * cos(th), m * sin(th)};
}

// Householder reflector of x (length n): P = I - 2 w w^H / (w^H w) with P x = alpha e_1 (alpha = -e^{i arg x_0} |x|).
// Returns false when x = 0 (P = I).  w is written in place of w[0..n).
RSL_DEV bool householder(const Z* x, int n, Z* w, double* wn) {
  double nx = 0;
  for (int k = 0; k < n; ++k) nx += zabs2(x[k]);
  nx = sqrt(nx);
  if (!(nx > 0)) return false;
  const double a0 = sqrt(zabs2(x[0]));
  const Z ph = a0 > 0 ? Z{x[0].r / a0, x[0].i / a0} : Z{1.0, 0.0};
  const Z alpha = zscale(ph, -nx);
  for (int k = 0; k < n; ++k) w[k] = x[k];
  w[0] = zsub(w[0], alpha);
  double s = 0;
  for (int k = 0; k < n; ++k) s += zabs2(w[k]);
  *wn = s;
  return s > 0;
}
// y = P v
RSL_DEV void hh_apply(const Z* w, double wn, int n, const Z* v, Z* y) {
  Z d = {0, 0};
  for (int k = 0; k < n; ++k) d = zadd(d, zcmul(w[k], v[k]));
  const Z f = zscale(d, 2.0 / wn);
  for (int k = 0; k < n; ++k) y[k] = zsub(v[k], zmul(w[k], f));
}
}  // namespace

// MUSIC spectrum 1 / den (0 where den <= 1e-12, :149-152), den = sum over the noise columns j of |(P a)_j|^2.
__global__ __launch_bounds__(256) void k_music_subspace(const double* __restrict__ sigs, long n, int M, int K,
                                                        const double* __restrict__ steer, int G,
                                                        double* __restrict__ spec) {
  const long idx = blockIdx.x * 256L + threadIdx.x;
  if (idx >= n * (long)G) return;
  const long c = idx / G;
  const int g = (int)(idx - c * G);
  Z s[kMaxM], a[kMaxM], w[kMaxM], pa[kMaxM];
  for (int m = 0; m < M; ++m) {
    s[m] = {sigs[2 * (c * M + m)], sigs[2 * (c * M + m) + 1]};
    a[m] = {steer[2 * ((long)g * M + m)], steer[2 * ((long)g * M + m) + 1]};
  }
  // noise columns [lo, M) of V (Python slice V[:, K:])
  const int lo = K >= 0 ? (K < M ? K : M) : (M + K > 0 ? M + K : 0);
  double wn = 0;
  double den = 0;
  if (householder(s, M, w, &wn)) {
    hh_apply(w, wn, M, a, pa);  // |a^H v_j| = |(P a)_j|, v_0 = P e_1 ∝ s
    for (int j = lo; j < M; ++j) den += zabs2(pa[j]);
  } else {  // R = 0: eigh -> identity, descending (all-equal) order reverses the columns: v_j = e_{M-1-j}
    for (int j = lo; j < M; ++j) den += zabs2(a[M - 1 - j]);
  }
  spec[c * (long)G + g] = den > 1e-12 ? 1.0 / den : 0.0;
}

namespace {
// Eigenvalues of a small complex matrix (n <= kMaxM, row-major) by the shifted QR iteration: per step the Givens QR
// of A - mu I (left rotations, recorded), then A <- R Q + mu I; Wilkinson shift from the trailing 2x2; deflation
// when the last row's off-diagonal part is negligible.  ev[k] = the converged diagonal (Schur form) entries.
RSL_DEV void zeig(Z (*A)[kMaxM], int n, Z* ev) {
  int hi = n - 1;
  for (int it = 0; hi > 0 && it < 200 * n; ++it) {
    double off = 0, dg = sqrt(zabs2(A[hi][hi]));
    for (int k = 0; k < hi; ++k) off = fmax(off, sqrt(zabs2(A[hi][k])));
    if (off <= 1e-15 * (dg + sqrt(zabs2(A[hi - 1][hi - 1]))) || off == 0.0) {
      --hi;
      continue;
    }
    const Z a = A[hi - 1][hi - 1], b = A[hi - 1][hi], cc = A[hi][hi - 1], d = A[hi][hi];
    const Z tr = zadd(a, d), det = zsub(zmul(a, d), zmul(b, cc));
    const Z disc = zsqrt(zsub(zmul(tr, tr), zscale(det, 4.0)));
    const Z l1 = zscale(zadd(tr, disc), 0.5), l2 = zscale(zsub(tr, disc), 0.5);
    Z mu = zabs2(zsub(l1, d)) < zabs2(zsub(l2, d)) ? l1 : l2;
    if (it % 17 == 16) mu = zadd(mu, Z{0.5 * off, 0.0});  // exceptional shift against cycling
    for (int k = 0; k <= hi; ++k) A[k][k] = zsub(A[k][k], mu);
    Z gc[kMaxM * kMaxM / 2], gs[kMaxM * kMaxM / 2];
    int gj[kMaxM * kMaxM / 2];
    int ng = 0;
    for (int k = 0; k < hi; ++k)
      for (int j = hi; j > k; --j) {  // zero A[j][k] with rows (j-1, j): G = [c^H s^H; -s c]
        const Z x = A[j - 1][k], y = A[j][k];
        const double r = sqrt(zabs2(x) + zabs2(y));
        if (r == 0.0 || zabs2(y) == 0.0) continue;
        const Z c = {x.r / r, x.i / r}, sn = {y.r / r, y.i / r};
        for (int m = 0; m <= hi; ++m) {
          const Z u = A[j - 1][m], v = A[j][m];
          A[j - 1][m] = zadd(zcmul(c, u), zcmul(sn, v));
          A[j][m] = zsub(zmul(c, v), zmul(sn, u));
        }
        gc[ng] = c;
        gs[ng] = sn;
        gj[ng] = j;
        ++ng;
      }
    for (int g = 0; g < ng; ++g) {  // R Q: right-multiply by each G^H = [c -s^H; s c^H] on columns (j-1, j)
      const Z c = gc[g], sn = gs[g];
      const int j = gj[g];
      for (int m = 0; m <= hi; ++m) {
        const Z u = A[m][j - 1], v = A[m][j];
        A[m][j - 1] = zadd(zmul(u, c), zmul(v, sn));
        A[m][j] = zsub(zmul(v, Z{c.r, -c.i}), zmul(u, Z{sn.r, -sn.i}));
      }
    }
    for (int k = 0; k <= hi; ++k) A[k][k] = zadd(A[k][k], mu);
  }
  for (int k = 0; k < n; ++k) ev[k] = A[k][k];
}
}  // namespace

// ESPRIT angle for num_sources K (see the file comment); deg f64 [n], 0.0 where the reference raises.
__global__ __launch_bounds__(64) void k_esprit_subspace(const double* __restrict__ sigs, long n, int M, int K,
                                                        double esprit_scale, double* __restrict__ deg) {
  const long c = blockIdx.x * 64L + threadIdx.x;
  if (c >= n) return;
  const int L = M - 1;  // rows of X
  Z s[kMaxM];
  for (int m = 0; m < M; ++m) s[m] = {sigs[2 * (c * M + m)], sigs[2 * (c * M + m) + 1]};
  // Python slice U[:, :K] of the (L x L) U
  const int kk = K >= 0 ? (K < L ? K : L) : (L + K > 0 ? L + K : 0);
  if (kk == 0 || L < 2) {  // empty Phi: eigvals(...)[0] raises -> 0.0
    deg[c] = 0.0;
    return;
  }
  // left singular vectors of X = [x0, x1] (L x 2), x0 = s[:-1], x1 = s[1:]: eigen of the 2x2 Hermitian X^H X
  double a = 0, cc = 0;
  Z b = {0, 0};
  for (int m = 0; m < L; ++m) {
    a += zabs2(s[m]);
    cc += zabs2(s[m + 1]);
    b = zadd(b, zcmul(s[m], s[m + 1]));
  }
  const double hd = 0.5 * (a - cc), rt = sqrt(hd * hd + zabs2(b));
  const double lam[2] = {0.5 * (a + cc) + rt, 0.5 * (a + cc) - rt};
  Z U[kMaxM][kMaxM];
  int nu = 0;
  auto push = [&](Z* u) {  // Gram-Schmidt (two passes) against the columns so far; keep it if independent
    for (int rep = 0; rep < 2; ++rep)
      for (int p = 0; p < nu; ++p) {
        Z d = {0, 0};
        for (int q = 0; q < L; ++q) d = zadd(d, zcmul(U[q][p], u[q]));
        for (int q = 0; q < L; ++q) u[q] = zsub(u[q], zmul(U[q][p], d));
      }
    double nn = 0;
    for (int m = 0; m < L; ++m) nn += zabs2(u[m]);
    if (nn > 1e-24) {
      nn = sqrt(nn);
      for (int m = 0; m < L; ++m) U[m][nu] = zscale(u[m], 1.0 / nn);
      ++nu;
    }
  };
  for (int e = 0; e < 2; ++e) {  // u_e = X v_e, v_e the eigenvector of X^H X for lam[e] (descending)
    Z v0, v1;
    if (a >= cc) {
      v0 = {lam[e] - cc, 0};
      v1 = {b.r, -b.i};
    } else {
      v0 = b;
      v1 = {lam[e] - a, 0};
    }
    if (zabs2(v0) + zabs2(v1) == 0.0) {
      v0 = {e == 0 ? 1.0 : 0.0, 0};
      v1 = {e == 0 ? 0.0 : 1.0, 0};
    }
    Z u[kMaxM];
    for (int m = 0; m < L; ++m) u[m] = zadd(zmul(s[m], v0), zmul(s[m + 1], v1));
    push(u);
  }
  // orthonormal completion of U against e_0, e_1, ... (the reference's null-space columns are LAPACK's)
  for (int e = 0; e < L && nu < L; ++e) {
    Z u[kMaxM];
    for (int m = 0; m < L; ++m) u[m] = {m == e ? 1.0 : 0.0, 0};
    push(u);
  }
  // Phi = pinv(U1) U2, U1 = Us[:-1], U2 = Us[1:] ((L-1) x kk): normal equations (U1^H U1) Phi = U1^H U2 when
  // kk <= L-1 (full column rank), else the minimum-norm form U1^H (U1 U1^H)^-1 U2
  const int r = L - 1;
  Z Phi[kMaxM][kMaxM];
  if (kk <= r) {
    Z Nm[kMaxM][2 * kMaxM];
    for (int p = 0; p < kk; ++p)
      for (int q = 0; q < kk; ++q) {
        Z x = {0, 0}, y = {0, 0};
        for (int m = 0; m < r; ++m) {
          x = zadd(x, zcmul(U[m][p], U[m][q]));
          y = zadd(y, zcmul(U[m][p], U[m + 1][q]));
        }
        Nm[p][q] = x;
        Nm[p][kk + q] = y;
      }
    for (int p = 0; p < kk; ++p) {  // Gauss-Jordan with partial pivoting
      int piv = p;
      for (int q = p + 1; q < kk; ++q)
        if (zabs2(Nm[q][p]) > zabs2(Nm[piv][p])) piv = q;
      if (piv != p)
        for (int q = 0; q < 2 * kk; ++q) {
          const Z t = Nm[p][q];
          Nm[p][q] = Nm[piv][q];
          Nm[piv][q] = t;
        }
      const Z d = Nm[p][p];
      if (zabs2(d) == 0.0) {
        deg[c] = 0.0;  // singular: numpy's pinv would still return; treated as the reference's failure value
        return;
      }
      for (int q = 0; q < 2 * kk; ++q) Nm[p][q] = zdiv(Nm[p][q], d);
      for (int o = 0; o < kk; ++o) {
        if (o == p) continue;
        const Z f = Nm[o][p];
        for (int q = 0; q < 2 * kk; ++q) Nm[o][q] = zsub(Nm[o][q], zmul(f, Nm[p][q]));
      }
    }
    for (int p = 0; p < kk; ++p)
      for (int q = 0; q < kk; ++q) Phi[p][q] = Nm[p][kk + q];
  } else {
    // W = (U1 U1^H)^-1 U2 (r x kk), Phi = U1^H W
    Z Nm[kMaxM][2 * kMaxM];
    for (int p = 0; p < r; ++p) {
      for (int q = 0; q < r; ++q) {
        Z x = {0, 0};
        for (int m = 0; m < kk; ++m) x = zadd(x, zmul(U[p][m], Z{U[q][m].r, -U[q][m].i}));
        Nm[p][q] = x;
      }
      for (int q = 0; q < kk; ++q) Nm[p][r + q] = U[p + 1][q];
    }
    for (int p = 0; p < r; ++p) {
      int piv = p;
      for (int q = p + 1; q < r; ++q)
        if (zabs2(Nm[q][p]) > zabs2(Nm[piv][p])) piv = q;
      if (piv != p)
        for (int q = 0; q < r + kk; ++q) {
          const Z t = Nm[p][q];
          Nm[p][q] = Nm[piv][q];
          Nm[piv][q] = t;
        }
      const Z d = Nm[p][p];
      if (zabs2(d) == 0.0) {
        deg[c] = 0.0;
        return;
      }
      for (int q = 0; q < r + kk; ++q) Nm[p][q] = zdiv(Nm[p][q], d);
      for (int o = 0; o < r; ++o) {
        if (o == p) continue;
        const Z f = Nm[o][p];
        for (int q = 0; q < r + kk; ++q) Nm[o][q] = zsub(Nm[o][q], zmul(f, Nm[p][q]));
      }
    }
    for (int p = 0; p < kk; ++p)
      for (int q = 0; q < kk; ++q) {
        Z x = {0, 0};
        for (int m = 0; m < r; ++m) x = zadd(x, zcmul(U[m][p], Nm[m][r + q]));
        Phi[p][q] = x;
      }
  }
  Z ev[kMaxM];
  if (kk == 1) {
    ev[0] = Phi[0][0];
  } else {
    zeig(Phi, kk, ev);
  }
  const double ph = atan2(ev[0].i, ev[0].r);
  deg[c] = asin(ph * esprit_scale) * (180.0 / M_PI);  // NaN outside [-1, 1], as np.arcsin
}

hipError_t launch_music_subspace(hipStream_t st, const double* sigs, long n, int M, int K, const double* steer,
                                 int G, double* spec) {
  const long tot = n * (long)G;
  hipLaunchKernelGGL(k_music_subspace, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, sigs, n, M, K, steer,
                     G, spec);
  return hipGetLastError();
}

hipError_t launch_esprit_subspace(hipStream_t st, const double* sigs, long n, int M, int K, double esprit_scale,
                                  double* deg) {
  hipLaunchKernelGGL(k_esprit_subspace, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, sigs, n, M, K,
                     esprit_scale, deg);
  return hipGetLastError();
}

}  // namespace rsl
