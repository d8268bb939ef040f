// rsl_aux.hip — per-call kernels behind the reference's fine-grained methods.  gfx950.
//
//  k_preprocess_rows : dechirp_signal / apply_window / remove_dc / process_chirp (dechirp.py:85-166):
//                      rows * table, then optional complex-mean removal.
//  k_phase_model     : compute_phase_difference_model + cost_function (velocity_solver.py:65-176,
//                      velocity_solver_improved.py:173-266 with the wrap and ridge), general 6-DoF.
//  k_bvls            : two_step_optimization (velocity_solver.py:178-307) for arbitrary positions /
//                      angles: the model k (v + w x p).d = k [d, p x d] . [v; w] is linear in the 6
//                      unknowns, so the DE box problem is a bounded linear least-squares problem, solved
//                      exactly by an active-set (Stark-Parker BVLS) on the 6x6 normal equations in fp64.
#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

__global__ __launch_bounds__(256) void k_preprocess_rows(const float2* __restrict__ in, int S,
                                                         const float2* __restrict__ table, int dc,
                                                         float2* __restrict__ out) {
  const long r = blockIdx.x;
  const float2* src = in + (size_t)r * S;
  float2* dst = out + (size_t)r * S;
  double ax = 0.0, ay = 0.0;  // fp64 mean accumulation
  for (int s = threadIdx.x; s < S; s += 256) {
    const float2 v = cmul(src[s], table[s]);
    dst[s] = v;
    ax += v.x;
    ay += v.y;
  }
  if (!dc) return;
  for (int off = 32; off > 0; off >>= 1) {
    ax += __shfl_down(ax, off);
    ay += __shfl_down(ay, off);
  }
  __shared__ double dx[4], dy[4];
  if ((threadIdx.x & 63) == 0) {
    dx[threadIdx.x >> 6] = ax;
    dy[threadIdx.x >> 6] = ay;
  }
  __syncthreads();
  const double mx = (dx[0] + dx[1] + dx[2] + dx[3]) / S, my = (dy[0] + dy[1] + dy[2] + dy[3]) / S;
  for (int s = threadIdx.x; s < S; s += 256) {
    const float2 v = dst[s];
    dst[s] = make_float2((float)(v.x - mx), (float)(v.y - my));
  }
}

hipError_t launch_preprocess_rows(hipStream_t st, const float2* in, long rows, int S, const float2* table, int dc,
                                  float2* out) {
  if (rows <= 0 || S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_preprocess_rows, dim3((unsigned)rows), dim3(256), 0, st, in, S, table, dc, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
RSL_DEV void jacobian_row(const double* pos, const double* ang, double* J) {
  const double az = ang[0], el = ang[1];
  const double ce = cos(el);
  const double d0 = ce * cos(az), d1 = ce * sin(az), d2 = sin(el);
  // (w x p).d = w . (p x d)
  const double px = pos[0], py = pos[1], pz = pos[2];
  J[0] = d0;
  J[1] = d1;
  J[2] = d2;
  J[3] = py * d2 - pz * d1;
  J[4] = pz * d0 - px * d2;
  J[5] = px * d1 - py * d0;
}

// pos f64 [N,3], ang f64 [N,2], x f64 [6] (v, w); y f64 [N] nullable; out_pred/out_resid nullable;
// cost_out f64 [1] = sum r^2 (+ ridge |x|^2), r wrapped to (-pi, pi] when wrap != 0.  One block.
__global__ __launch_bounds__(256) void k_phase_model(const double* __restrict__ pos, const double* __restrict__ ang,
                                                     long n, const double* __restrict__ x, double k,
                                                     const double* __restrict__ y, int wrap, double ridge,
                                                     double* __restrict__ pred, double* __restrict__ resid,
                                                     double* __restrict__ cost_out) {
  __shared__ double sh[4];
  double acc = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) {
    double J[6];
    jacobian_row(pos + 3 * i, ang + 2 * i, J);
    double p = 0.0;
    for (int c = 0; c < 6; ++c) p += J[c] * x[c];
    p *= k;
    if (pred) pred[i] = p;
    if (y) {
      double r = y[i] - p;
      if (wrap) r = atan2(sin(r), cos(r));
      if (resid) resid[i] = r;
      acc += r * r;
    }
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0 && cost_out) {
    double reg = 0.0;
    for (int c = 0; c < 6; ++c) reg += x[c] * x[c];
    cost_out[0] = sh[0] + sh[1] + sh[2] + sh[3] + ridge * reg;
  }
}

hipError_t launch_phase_model(hipStream_t st, const double* pos, const double* ang, long n, const double* x, double k,
                              const double* y, int wrap, double ridge, double* pred, double* resid, double* cost) {
  hipLaunchKernelGGL(k_phase_model, dim3(1), dim3(256), 0, st, pos, ang, n, x, k, y, wrap, ridge, pred, resid, cost);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Solve H_FF z = g_F for the free set F (n <= 6) by Gaussian elimination with partial pivoting;
// singular directions (pivot <= eps * scale) get 0 (minimum-norm on exactly-null columns).
RSL_DEV void solve_free(const double H[6][6], const double* g, const int* freev, int nf, double* z) {
  double M[6][7];
  double scale = 0.0;
  for (int a = 0; a < nf; ++a) scale = fmax(scale, fabs(H[freev[a]][freev[a]]));
  for (int a = 0; a < nf; ++a) {
    for (int b = 0; b < nf; ++b) M[a][b] = H[freev[a]][freev[b]];
    M[a][nf] = g[a];
  }
  int piv_ok[6];
  for (int col = 0; col < nf; ++col) {
    int best = col;
    for (int r = col + 1; r < nf; ++r)
      if (fabs(M[r][col]) > fabs(M[best][col])) best = r;
    if (best != col)
      for (int c = 0; c <= nf; ++c) {
        const double t = M[col][c];
        M[col][c] = M[best][c];
        M[best][c] = t;
      }
    piv_ok[col] = fabs(M[col][col]) > 1e-13 * (scale > 0 ? scale : 1.0);
    if (!piv_ok[col]) continue;
    for (int r = col + 1; r < nf; ++r) {
      const double f = M[r][col] / M[col][col];
      for (int c = col; c <= nf; ++c) M[r][c] -= f * M[col][c];
    }
  }
  for (int col = nf - 1; col >= 0; --col) {
    if (!piv_ok[col]) {
      z[col] = 0.0;
      continue;
    }
    double s = M[col][nf];
    for (int c = col + 1; c < nf; ++c) s -= M[col][c] * z[c];
    z[col] = s / M[col][col];
  }
}

// One block: normal equations of min |y - k J x|^2 + ridge |x|^2 over nv (3 or 6) unknowns, then BVLS.
// out f64 [nv + 1] = x, cost.
__global__ __launch_bounds__(256) void k_bvls(const double* __restrict__ pos, const double* __restrict__ ang, long n,
                                              const double* __restrict__ y, double k, int nv, double ridge,
                                              const double* __restrict__ lo, const double* __restrict__ hi,
                                              double* __restrict__ out) {
  __shared__ double red[4][28];
  double acc[28];
  for (int c = 0; c < 28; ++c) acc[c] = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) {
    double J[6];
    jacobian_row(pos + 3 * i, ang + 2 * i, J);
    for (int c = 0; c < 6; ++c) J[c] *= k;
    int t = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 6; ++b) acc[t++] += J[a] * J[b];  // 21
    for (int a = 0; a < 6; ++a) acc[21 + a] += J[a] * y[i];  // 6
    acc[27] += y[i] * y[i];
  }
  for (int c = 0; c < 28; ++c) {
    double v = acc[c];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][c] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double H[6][6], b[6], yy;
  {
    double m[28];
    for (int c = 0; c < 28; ++c) m[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    int t = 0;
    for (int a = 0; a < 6; ++a)
      for (int c = a; c < 6; ++c) {
        H[a][c] = H[c][a] = m[t++];
      }
    for (int a = 0; a < 6; ++a) {
      b[a] = m[21 + a];
      H[a][a] += ridge;
    }
    yy = m[27];
  }
  // BVLS (Stark & Parker): state 0 free, -1 at lower, +1 at upper.  Start with all at bound nearest 0
  // (0 itself when inside the box: treat as free start).
  double x[6];
  int state[6];
  for (int a = 0; a < nv; ++a) {
    x[a] = fmin(fmax(0.0, lo[a]), hi[a]);
    state[a] = 0;
  }
  for (int it = 0; it < 100; ++it) {
    // solve on the free set with bound variables fixed
    int freev[6], nf = 0;
    for (int a = 0; a < nv; ++a)
      if (state[a] == 0) freev[nf++] = a;
    double g[6], z[6];
    for (int ai = 0; ai < nf; ++ai) {
      const int a = freev[ai];
      double s = b[a];
      for (int c = 0; c < nv; ++c)
        if (state[c] != 0) s -= H[a][c] * x[c];
      g[ai] = s;
    }
    solve_free(H, g, freev, nf, z);
    // move toward z; stop at the first bound crossed
    double alpha = 1.0;
    int hit = -1, hit_state = 0;
    for (int ai = 0; ai < nf; ++ai) {
      const int a = freev[ai];
      const double d = z[ai] - x[a];
      if (z[ai] < lo[a]) {
        const double t = (lo[a] - x[a]) / d;
        if (t < alpha) { alpha = t; hit = a; hit_state = -1; }
      } else if (z[ai] > hi[a]) {
        const double t = (hi[a] - x[a]) / d;
        if (t < alpha) { alpha = t; hit = a; hit_state = 1; }
      }
    }
    if (alpha < 0) alpha = 0;
    for (int ai = 0; ai < nf; ++ai) {
      const int a = freev[ai];
      x[a] = x[a] + alpha * (z[ai] - x[a]);
    }
    if (hit >= 0) {
      x[hit] = hit_state < 0 ? lo[hit] : hi[hit];
      state[hit] = hit_state;
      continue;
    }
    // KKT: gradient of 0.5|r|^2 wrt x is -(b - H x); release the bound variable that violates most
    int rel = -1;
    double worst = 0.0;
    for (int a = 0; a < nv; ++a) {
      if (state[a] == 0) continue;
      double gr = b[a];
      for (int c = 0; c < nv; ++c) gr -= H[a][c] * x[c];  // descent direction component
      const double viol = state[a] < 0 ? gr : -gr;          // at lower: wants to increase if gr > 0
      if (viol > worst * (1.0 + 1e-12) && viol > 1e-12 * (fabs(b[a]) + 1.0)) {
        worst = viol;
        rel = a;
      }
    }
    if (rel < 0) break;
    state[rel] = 0;
  }
  double xHx = 0.0, bx = 0.0, reg = 0.0;
  for (int a = 0; a < nv; ++a) {
    bx += b[a] * x[a];
    reg += x[a] * x[a];
    for (int c = 0; c < nv; ++c) xHx += x[a] * H[a][c] * x[c];
  }
  for (int a = 0; a < nv; ++a) out[a] = x[a];
  out[nv] = yy - 2.0 * bx + xHx;  // includes ridge |x|^2 via H's diagonal
  (void)reg;
}

hipError_t launch_bvls(hipStream_t st, const double* pos, const double* ang, long n, const double* y, double k, int nv,
                       double ridge, const double* lo, const double* hi, double* out) {
  hipLaunchKernelGGL(k_bvls, dim3(1), dim3(256), 0, st, pos, ang, n, y, k, nv, ridge, lo, hi, out);
  return hipGetLastError();
}

}  // namespace rsl
