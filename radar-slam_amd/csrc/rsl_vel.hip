// rsl_vel.hip — K8: batched box-constrained (ridge) least-squares velocity solve, fp64.  gfx950.
//
// Replaces VelocitySolver.two_step_optimization (reference src/velocity_solver/velocity_solver.py:178-307),
// which runs differential_evolution (seed 42) over cost = sum (y - 4 pi dt / lambda * (v + w x p).d)^2
// (velocity_solver.py:65-176).  With elevation 0 and p = r d (velocity_solver.py:334-339), (w x p).d = 0 and
// d_z = 0: only (v_x, v_y) enter, linearly.  The cost is a convex quadratic over the box
// [-50,50]^2, so its exact minimiser is the interior normal-equation solution when feasible, else the
// best of the four edge minimisers (1-D clamp).  ``ridge`` adds ridge*(vx^2+vy^2)
// (velocity_solver_improved.py:261 without the wrap).  Items carry a multiplicity (popcount of the
// antenna mask of a deduplicated cell) so duplicate per-antenna detections count as in the reference.
#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

__device__ double block_sum(double v, double* sh) {
  const int t = threadIdx.x;
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
  __syncthreads();
  if ((t & 63) == 0) sh[t >> 6] = v;
  __syncthreads();
  double r = 0.0;
  if (t == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r += sh[w];
  __syncthreads();
  return r;  // valid on thread 0
}

__device__ double block_max(double v, double* sh) {
  const int t = threadIdx.x;
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off));
  __syncthreads();
  if ((t & 63) == 0) sh[t >> 6] = v;
  __syncthreads();
  double r = -1.0;
  if (t == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmax(r, sh[w]);
  __syncthreads();
  return r;
}

__device__ double qcost(double vx, double vy, double k, double ridge, const double* m) {
  // m: [n, cc, cs, ss, cy, sy, yy]
  const double kx = k * vx, ky = k * vy;
  return m[6] - 2.0 * (kx * m[4] + ky * m[5]) + kx * kx * m[1] + 2.0 * kx * ky * m[2] + ky * ky * m[3] +
         ridge * (vx * vx + vy * vy);
}

constexpr int kVelU = 8;

// kVelU cells i0 + u * blockDim.x (u < kVelU) of one thread; cells at or past e read as weight 0, grid index 0
RSL_DEV void vel_load(long long i0, long long e, const int* __restrict__ gidx, const double* __restrict__ y,
                      const unsigned* __restrict__ amask, int (&gv)[kVelU], double (&yv)[kVelU],
                      unsigned (&mv)[kVelU]) {
#pragma unroll
  for (int u = 0; u < kVelU; ++u) {
    const long long i = i0 + (long long)u * blockDim.x;
    const bool ok = i < e;
    const long long ii = ok ? i : i0;  // i0 < e: always a valid address
    gv[u] = gidx[ii];
    yv[u] = y[ii];
    mv[u] = amask ? amask[ii] : 1u;
    if (!ok) {
      gv[u] = 0;
      yv[u] = 0.0;
      mv[u] = 0u;
    }
  }
}

// Order-preserving key of a finite or infinite double (NaN never enters): min / max of keys = min / max of values.
RSL_DEV unsigned long long okey(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
RSL_DEV double unkey(unsigned long long k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// One workgroup per frame.  gidx path (the chain): one pass over the cells.  Besides the 7 moments it keeps, per grid
// index g, the smallest and largest phase of the cells with weight > 0 (LDS min / max on order-preserving keys:
// exact and order-independent).  All cells of index g share the prediction p_g = k (vx c_g + vy s_g), so the
// residual y - p_g of largest magnitude is that of the group's smallest or largest y: max |residual| comes from 2G
// values instead of a second pass over the cells (bit-identical: same p_g, same subtraction).  The residual sum
// of squares is the quadratic form of the moments; it is used when its terms do not cancel (R2 >= 1e-6 of their
// magnitude sum, i.e. < 1e-9 relative rounding), else (a near-perfect fit) R2 is summed per cell in a second pass,
// as it is for the az path and whenever per-cell residuals / predictions are requested.
__global__ __launch_bounds__(512) void k_velocity(const double* __restrict__ az, const int* __restrict__ gidx,
                                                  const double* __restrict__ az_table, int G,
                                                  const double* __restrict__ y, const unsigned* __restrict__ amask,
                                                  const long long* __restrict__ seg, long long nmax, double k, double ridge,
                                                  double lx, double hx, double ly, double hy,
                                                  double* __restrict__ out, double* __restrict__ resid,
                                                  double* __restrict__ pred) {
  __shared__ double sh[8];
  __shared__ double mom[7];
  __shared__ double sol[3];
  extern __shared__ double cs_tab[];  // [2G] cos, sin of the grid azimuths, then [2G] min / max phase keys (gidx path)
  const bool tab = gidx != nullptr;
  const bool grp = tab;  // per-group extremes: 32 G B of LDS (rsl_velocity admits G <= 2048)
  unsigned long long* ymn = reinterpret_cast<unsigned long long*>(cs_tab + 2 * G);
  unsigned long long* ymx = ymn + G;
  if (tab) {
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
      sincos(az_table[g], &cs_tab[G + g], &cs_tab[g]);
      if (grp) {
        ymn[g] = ~0ull;
        ymx[g] = 0ull;  // no key is 0 (that would be a NaN's bits): 0 marks an empty group
      }
    }
    __syncthreads();
  }
  const long f = blockIdx.x;
  // segment bounds clamped to the arrays' length (an overflowed capacity-sized list ends at its capacity)
  const long long b = seg[f] < nmax ? seg[f] : nmax, e = seg[f + 1] < nmax ? seg[f + 1] : nmax;
  double n = 0, cc = 0, cs = 0, ss = 0, cy = 0, sy = 0, yy = 0;
  auto acc1 = [&](double w, double c, double s, double yi) {
    n += w;
    cc += w * c * c;
    cs += w * c * s;
    ss += w * s * s;
    cy += w * c * yi;
    sy += w * s * yi;
    yy += w * yi * yi;
  };
  const long long step = (long long)blockDim.x * kVelU;
  if (tab) {
    // kVelU cells per thread per trip, all loads issued first: the loop is HBM-latency bound otherwise
    for (long long i0 = b + threadIdx.x; i0 < e; i0 += step) {
      int gv[kVelU];
      double yv[kVelU];
      unsigned mv[kVelU];
      vel_load(i0, e, gidx, y, amask, gv, yv, mv);
#pragma unroll
      for (int u = 0; u < kVelU; ++u) {
        acc1((double)__popc(mv[u]), cs_tab[gv[u]], cs_tab[G + gv[u]], yv[u]);
        if (grp && mv[u] != 0u && yv[u] == yv[u]) {  // weight > 0, not NaN (fmax ignores a NaN residual)
          const unsigned long long kk = okey(yv[u]);
          atomicMin(&ymn[gv[u]], kk);
          atomicMax(&ymx[gv[u]], kk);
        }
      }
    }
  } else {
    for (long long i = b + threadIdx.x; i < e; i += blockDim.x) {
      double s, c;
      sincos(az[i], &s, &c);
      acc1(amask ? (double)__popc(amask[i]) : 1.0, c, s, y[i]);
    }
  }
  const double vals[7] = {n, cc, cs, ss, cy, sy, yy};
  for (int v = 0; v < 7; ++v) {
    const double r = block_sum(vals[v], sh);
    if (threadIdx.x == 0) mom[v] = r;
  }
  if (threadIdx.x == 0) {
    const double* m = mom;
    const double H00 = k * k * m[1] + ridge, H01 = k * k * m[2], H11 = k * k * m[3] + ridge;
    const double b0 = k * m[4], b1 = k * m[5];
    const double det = H00 * H11 - H01 * H01;
    double bx = 0.0, by = 0.0;
    bool done = false;
    if (det > 1e-300) {
      const double vx = (H11 * b0 - H01 * b1) / det, vy = (H00 * b1 - H01 * b0) / det;
      if (vx >= lx && vx <= hx && vy >= ly && vy <= hy) {
        bx = vx;
        by = vy;
        done = true;
      }
    }
    if (!done) {
      double bc = INFINITY;
      for (int edge = 0; edge < 4; ++edge) {
        const int fix = edge >> 1;  // 0: vx fixed, 1: vy fixed
        const double val = (fix == 0) ? ((edge & 1) ? hx : lx) : ((edge & 1) ? hy : ly);
        double x;
        if (fix == 0) {
          x = H11 > 0 ? (b1 - H01 * val) / H11 : 0.0;
          x = fmin(fmax(x, ly), hy);
        } else {
          x = H00 > 0 ? (b0 - H01 * val) / H00 : 0.0;
          x = fmin(fmax(x, lx), hx);
        }
        const double vx = fix == 0 ? val : x, vy = fix == 0 ? x : val;
        const double cst = qcost(vx, vy, k, ridge, m);
        if (cst < bc) {
          bc = cst;
          bx = vx;
          by = vy;
        }
      }
    }
    sol[0] = bx;
    sol[1] = by;
    // residual sum of squares from the moments, kept when its terms do not cancel (gidx path only)
    const double kx = k * bx, ky = k * by;
    const double q = m[6] - 2.0 * (kx * m[4] + ky * m[5]) + kx * kx * m[1] + 2.0 * kx * ky * m[2] + ky * ky * m[3];
    const double mag = m[6] + 2.0 * (fabs(kx * m[4]) + fabs(ky * m[5])) + kx * kx * m[1] + 2.0 * fabs(kx * ky * m[2]) +
                       ky * ky * m[3];
    sol[2] = (grp && q >= 1e-6 * mag) ? q : -1.0;
  }
  __syncthreads();
  const double vx = sol[0], vy = sol[1], r2m = sol[2];
  double r2 = 0.0, rmax = 0.0;
  auto acc2 = [&](long long i, double w, double c, double s, double yi) {
    const double pr = k * (vx * c + vy * s);
    const double r = yi - pr;
    r2 += w * r * r;
    if (w > 0) rmax = fmax(rmax, fabs(r));
    if (resid) resid[i] = r;
    if (pred) pred[i] = pr;
  };
  if (tab) {
    if (!grp || r2m < 0.0 || resid || pred) {
      for (long long i0 = b + threadIdx.x; i0 < e; i0 += step) {
        int gv[kVelU];
        double yv[kVelU];
        unsigned mv[kVelU];
        vel_load(i0, e, gidx, y, amask, gv, yv, mv);
#pragma unroll
        for (int u = 0; u < kVelU; ++u)
          if (i0 + (long long)u * blockDim.x < e)
            acc2(i0 + (long long)u * blockDim.x, (double)__popc(mv[u]), cs_tab[gv[u]], cs_tab[G + gv[u]], yv[u]);
      }
    }
    if (grp) rmax = 0.0;  // from the per-group extremes (same values as the per-cell maximum)
    for (int g = threadIdx.x; grp && g < G; g += blockDim.x) {
      const unsigned long long hi = ymx[g];
      if (hi == 0ull) continue;
      const double pr = k * (vx * cs_tab[g] + vy * cs_tab[G + g]);
      rmax = fmax(rmax, fmax(fabs(unkey(ymn[g]) - pr), fabs(unkey(hi) - pr)));
    }
  } else {
    for (long long i = b + threadIdx.x; i < e; i += blockDim.x) {
      double s, c;
      sincos(az[i], &s, &c);
      acc2(i, amask ? (double)__popc(amask[i]) : 1.0, c, s, y[i]);
    }
  }
  const double R2s = block_sum(r2, sh);
  const double R2 = r2m >= 0.0 ? r2m : R2s;
  const double RM = block_max(rmax, sh);
  if (threadIdx.x == 0) {
    double* o = out + f * 8;
    o[0] = vx;
    o[1] = vy;
    o[2] = R2 + ridge * (vx * vx + vy * vy);               // cost at the optimum
    o[3] = mom[0] > 0 ? sqrt(R2 / mom[0]) : 0.0;           // rmse (velocity_solver.py:283)
    o[4] = RM;                                             // max |residual| (velocity_solver.py:284)
    o[5] = mom[0];                                         // number of targets (with multiplicity)
    o[6] = mom[1] * mom[3] - mom[2] * mom[2];              // normal-matrix determinant / k^4
    o[7] = 0.0;
  }
}

hipError_t launch_velocity(hipStream_t st, const double* az, const int* gidx, const double* az_table, int G,
                           const double* y, const unsigned* amask, const long long* seg, long long n, int F, double k, double ridge,
                           const double* bounds4, double* out, double* resid, double* pred) {
  if (F <= 0) return hipSuccess;
  const size_t lds = gidx ? sizeof(double) * 4 * (size_t)G : 0;
  hipLaunchKernelGGL(k_velocity, dim3(F), dim3(512), lds, st, az, gidx, az_table, G, y, amask, seg, n, k, ridge,
                     bounds4[0], bounds4[1], bounds4[2], bounds4[3], out, resid, pred);
  return hipGetLastError();
}

}  // namespace rsl
