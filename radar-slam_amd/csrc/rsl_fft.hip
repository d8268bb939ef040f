// rsl_fft.hip — K1 (dechirp*window + range FFT + DC) and K2 (Doppler FFT + fftshift) for gfx950.
//
// Replaces SignalPreprocessor.generate_range_doppler_spectrum (reference src/radar_signal/dechirp.py:168-213):
//   per chirp  y = x * conj(ref) * w ; y -= mean(y)      (dechirp.py:156-164)
//   rds = fftshift(fft2(y^T, axes=(1,2)), axes=(1,2))     (dechirp.py:193-211)
// DC removal is folded into the range FFT: FFT(y - mean y)[k] = FFT(y)[k] for k != 0 and 0 for k = 0,
// so the kernel zeroes range bin 0 instead of reducing a mean (exact in real arithmetic).
// conj(ref)*w is precomputed on the host in fp64 (the chirp phase reaches 2.5e7 rad) and passed as a c64 table.
#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

constexpr int kThreads = 256;

// Rows per workgroup for an N-point FFT held in LDS (~32 KiB of row data).
constexpr int rows_for(int N) {
  int r = 4096 / N;
  if (r < 1) r = 1;
  if (r > 64) r = 64;
  return r;
}

// ---------------------------------------------------------------------------------------------
// K1: range FFT.  One workgroup = CB consecutive chirp rows of one (frame, antenna).
// Rows are contiguous S-sample vectors: loads/stores are fully coalesced 16-B accesses.
// ---------------------------------------------------------------------------------------------
template <int S>
__global__ __launch_bounds__(kThreads) void k_range_fft(const float2* __restrict__ cube, int A, int Ct, int c0,
                                                         int C, const float2* __restrict__ table,
                                                         const float2* __restrict__ tw, int dc,
                                                         float2* __restrict__ work) {
  constexpr int CB = rows_for(S);
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* buf = sm + S;
  const int tid = threadIdx.x;
  const int ncb = (C + CB - 1) / CB;
  const int cb = blockIdx.x % ncb;
  const long fa = blockIdx.x / ncb;  // frame * A + antenna
  const int cbeg = cb * CB;
  const int nrows = min(CB, C - cbeg);
  for (int k = tid; k < S; k += kThreads) tws[k] = tw[k];
  const float2* src = cube + ((size_t)fa * Ct + c0 + cbeg) * S;
  if constexpr (S % 2 == 0) {
    const float4* src4 = reinterpret_cast<const float4*>(src);
    const float4* tab4 = reinterpret_cast<const float4*>(table);
    float4* buf4 = reinterpret_cast<float4*>(buf);
    for (int idx = tid; idx < CB * S / 2; idx += kThreads) {
      const int r = idx / (S / 2), s2 = idx - r * (S / 2);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < nrows) {
        const float4 x = src4[(size_t)r * (S / 2) + s2];
        const float4 t = tab4[s2];
        const float2 lo = cmul(make_float2(x.x, x.y), make_float2(t.x, t.y));
        const float2 hi = cmul(make_float2(x.z, x.w), make_float2(t.z, t.w));
        v = make_float4(lo.x, lo.y, hi.x, hi.y);
      }
      buf4[idx] = v;
    }
  } else {
    for (int idx = tid; idx < CB * S; idx += kThreads) {
      const int r = idx / S, s = idx - r * S;
      buf[idx] = (r < nrows) ? cmul(src[(size_t)r * S + s], table[s]) : make_float2(0.f, 0.f);
    }
  }
  __syncthreads();
  fft_rows<S, CB, kThreads, S>(buf, tws, tid);
  if (dc) {
    if (tid < CB) buf[tid * S] = make_float2(0.f, 0.f);
    __syncthreads();
  }
  float2* dst = work + ((size_t)fa * C + cbeg) * S;
  if constexpr (S % 2 == 0) {
    float4* dst4 = reinterpret_cast<float4*>(dst);
    const float4* buf4 = reinterpret_cast<const float4*>(buf);
    for (int idx = tid; idx < nrows * S / 2; idx += kThreads) dst4[idx] = buf4[idx];
  } else {
    for (int idx = tid; idx < nrows * S; idx += kThreads) dst[idx] = buf[idx];
  }
}

// ---------------------------------------------------------------------------------------------
// K2: Doppler FFT.  One workgroup = KB consecutive (unshifted) range bins of one (frame, antenna):
// reads C segments of KB contiguous complex values (KB*8 bytes each), transposes into LDS rows of
// C points (odd stride C+1: conflict-free column writes), FFTs, and writes each shifted range row of
// the RDS [A, S, C] contiguously with the Doppler fftshift folded into the store index.
// ---------------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(kThreads) void k_doppler_fft(const float2* __restrict__ work, int S,
                                                           const float2* __restrict__ tw, float2* __restrict__ rds) {
  constexpr int KB = rows_for(C);
  constexpr int LD = (KB == 1) ? C : C + 1;
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* buf = sm + C;
  const int tid = threadIdx.x;
  const int nkb = (S + KB - 1) / KB;
  const int kb = blockIdx.x % nkb;
  const long fa = blockIdx.x / nkb;
  const int k0 = kb * KB;
  const int nk = min(KB, S - k0);
  for (int k = tid; k < C; k += kThreads) tws[k] = tw[k];
  const float2* src = work + (size_t)fa * C * S + k0;
  for (int idx = tid; idx < C * KB; idx += kThreads) {
    const int c = idx / KB, kk = idx - c * KB;
    buf[kk * LD + c] = (kk < nk) ? src[(size_t)c * S + kk] : make_float2(0.f, 0.f);
  }
  __syncthreads();
  fft_rows<C, KB, kThreads, LD>(buf, tws, tid);
  float2* dst = rds + (size_t)fa * S * C;
  const int hs = S / 2, hc = C / 2;
  for (int idx = tid; idx < nk * C; idx += kThreads) {
    const int kk = idx / C, j = idx - kk * C;
    const int k = k0 + kk;
    int i = k + hs;
    if (i >= S) i -= S;
    int d = j - hc;  // out[j] = X[(j - C//2) mod C]
    if (d < 0) d += C;
    dst[(size_t)i * C + j] = buf[kk * LD + d];
  }
}

template <int S>
static hipError_t launch_k1(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C,
                            const float2* table, const float2* tw, int dc, float2* work) {
  constexpr int CB = rows_for(S);
  const long nblk = (long)F * A * ((C + CB - 1) / CB);
  const size_t lds = sizeof(float2) * (S + (size_t)CB * S);
  hipLaunchKernelGGL(k_range_fft<S>, dim3((unsigned)nblk), dim3(kThreads), lds, st, cube, A, Ct, c0, C, table, tw,
                     dc, work);
  return hipGetLastError();
}

template <int C>
static hipError_t launch_k2(hipStream_t st, const float2* work, int F, int A, int S, const float2* tw,
                            float2* rds) {
  constexpr int KB = rows_for(C);
  const long nblk = (long)F * A * ((S + KB - 1) / KB);
  const size_t lds = sizeof(float2) * (C + (size_t)KB * ((KB == 1) ? C : C + 1));
  hipLaunchKernelGGL(k_doppler_fft<C>, dim3((unsigned)nblk), dim3(kThreads), lds, st, work, S, tw, rds);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Any-length fallback (sizes whose prime factors are not all in {2,3,5,7}, e.g. a chirp_subset of 59
// chirps): direct DFT from LDS with the fp64-accurate twiddle table, O(N) per output point.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_range_dft(const float2* __restrict__ cube, int Ct, int c0, int C, int S,
                                                        const float2* __restrict__ table,
                                                        const float2* __restrict__ tw, int dc,
                                                        float2* __restrict__ work) {
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* row = sm + S;
  const long r = blockIdx.x;  // (f*A + a)*C + c
  const long fa = r / C;
  const int c = (int)(r - fa * C);
  const float2* src = cube + ((size_t)fa * Ct + c0 + c) * S;
  for (int k = threadIdx.x; k < S; k += kThreads) {
    tws[k] = tw[k];
    row[k] = cmul(src[k], table[k]);
  }
  __syncthreads();
  float2* dst = work + (size_t)r * S;
  for (int k = threadIdx.x; k < S; k += kThreads) {
    float2 acc = make_float2(0.f, 0.f);
    int idx = 0;
    for (int n = 0; n < S; ++n) {
      acc = cadd(acc, cmul(row[n], tws[idx]));
      idx += k;
      if (idx >= S) idx -= S;
    }
    dst[k] = (dc && k == 0) ? make_float2(0.f, 0.f) : acc;
  }
}

__global__ __launch_bounds__(kThreads) void k_doppler_dft(const float2* __restrict__ work, int C, int S,
                                                          const float2* __restrict__ tw, float2* __restrict__ rds) {
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* col = sm + C;
  const long r = blockIdx.x;  // (f*A + a)*S + k
  const long fa = r / S;
  const int k = (int)(r - fa * S);
  const float2* src = work + (size_t)fa * C * S + k;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    tws[c] = tw[c];
    col[c] = src[(size_t)c * S];
  }
  __syncthreads();
  int i = k + S / 2;
  if (i >= S) i -= S;
  float2* dst = rds + ((size_t)fa * S + i) * C;
  for (int j = threadIdx.x; j < C; j += kThreads) {
    int d = j - C / 2;
    if (d < 0) d += C;
    float2 acc = make_float2(0.f, 0.f);
    int idx = 0;
    for (int n = 0; n < C; ++n) {
      acc = cadd(acc, cmul(col[n], tws[idx]));
      idx += d;
      if (idx >= C) idx -= C;
    }
    dst[j] = acc;
  }
}

hipError_t launch_range_dft(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C, int S,
                            const float2* table, const float2* tw, int dc, float2* work) {
  const long nblk = (long)F * A * C;
  hipLaunchKernelGGL(k_range_dft, dim3((unsigned)nblk), dim3(kThreads), sizeof(float2) * 2 * (size_t)S, st, cube, Ct,
                     c0, C, S, table, tw, dc, work);
  return hipGetLastError();
}

hipError_t launch_doppler_dft(hipStream_t st, const float2* work, int F, int A, int C, int S, const float2* tw,
                              float2* rds) {
  const long nblk = (long)F * A * S;
  hipLaunchKernelGGL(k_doppler_dft, dim3((unsigned)nblk), dim3(kThreads), sizeof(float2) * 2 * (size_t)C, st, work, C,
                     S, tw, rds);
  return hipGetLastError();
}

#define RSL_FFT_SIZES(X) \
  X(8) X(16) X(32) X(64) X(128) X(256) X(512) X(1024) X(2048) X(4096) X(25) X(50) X(100) X(200) X(400) X(800) X(1600)

hipError_t launch_range_fft(hipStream_t st, const float2* cube, int F, int A, int Ct, int chirp0, int C, int S,
                            const float2* table, const float2* tw_S, int dc, float2* work, bool* supported) {
  *supported = true;
  if (F <= 0 || A <= 0 || C <= 0) return hipSuccess;
  switch (S) {
#define CASE(n) \
  case n:       \
    return launch_k1<n>(st, cube, F, A, Ct, chirp0, C, table, tw_S, dc, work);
    RSL_FFT_SIZES(CASE)
#undef CASE
    default:
      if (S > 4096) {
        *supported = false;
        return hipSuccess;
      }
      return launch_range_dft(st, cube, F, A, Ct, chirp0, C, S, table, tw_S, dc, work);
  }
}

hipError_t launch_doppler_fft(hipStream_t st, const float2* work, int F, int A, int C, int S, const float2* tw_C,
                              float2* rds, bool* supported) {
  *supported = true;
  if (F <= 0 || A <= 0 || S <= 0) return hipSuccess;
  switch (C) {
#define CASE(n) \
  case n:       \
    return launch_k2<n>(st, work, F, A, S, tw_C, rds);
    RSL_FFT_SIZES(CASE)
#undef CASE
    default:
      if (C > 4096) {
        *supported = false;
        return hipSuccess;
      }
      return launch_doppler_dft(st, work, F, A, C, S, tw_C, rds);
  }
}

}  // namespace rsl
