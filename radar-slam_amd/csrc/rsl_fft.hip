// rsl_fft.hip — K1 (dechirp*window + range FFT + DC) and K2 (Doppler FFT + fftshift) for gfx950.
//
// Replaces SignalPreprocessor.generate_range_doppler_spectrum (reference src/radar_signal/dechirp.py:168-213):
//   per chirp  y = x * conj(ref) * w ; y -= mean(y)      (dechirp.py:156-164)
//   rds = fftshift(fft2(y^T, axes=(1,2)), axes=(1,2))     (dechirp.py:193-211)
// DC removal is folded into the range FFT: FFT(y - mean y)[k] = FFT(y)[k] for k != 0 and 0 for k = 0,
// so the kernel zeroes range bin 0 instead of reducing a mean (exact in real arithmetic).
// conj(ref)*w is precomputed on the host in fp64 (the chirp phase reaches 2.5e7 rad) and passed as a c64 table.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

constexpr int kThreads = 256;

// K1 work queues (RSL_RF_DYN): per launch slot, 8 per-XCD dequeue heads and 8 exit counters, each on its own 128-B
// line. The last workgroup of an XCD to leave resets its pair, so a slot is clean for its next launch; the host
// hands slots round-robin, so up to kRfSlots K1 launches may be in flight at once (on any streams).
constexpr int kRfSlots = 8;
__device__ unsigned g_rf_q[kRfSlots][2][8][32];

// Global accesses with an optional non-temporal hint (`nt`: streamed once, not kept in L2 / MALL).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
template <bool NTH>
RSL_DEV float4 ld16(const float4* p) {
  if constexpr (NTH) {
    return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p)));
  } else {
    return *p;
  }
}
template <bool NTH>
RSL_DEV void st16(float4* p, float4 x) {
  if constexpr (NTH) {
    f4v v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
  } else {
    *p = x;
  }
}
template <bool NTH>
RSL_DEV float2 ld8(const float2* p) {
  if constexpr (NTH) {
    return __builtin_bit_cast(float2, __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p)));
  } else {
    return *p;
  }
}
template <bool NTH>
RSL_DEV void st8(float2* p, float2 x) {
  if constexpr (NTH) {
    f2v v = {x.x, x.y};
    __builtin_nontemporal_store(v, reinterpret_cast<f2v*>(p));
  } else {
    *p = x;
  }
}

// Packed `work` (the fused RDS + detection path, RSL_WORK_PACK): every range-spectrum component is a 24-bit two's-
// complement mantissa and each block of 8 chirps x kPkG range bins (one K1 tile's rows of one group) shares one
// exponent, so a complex value takes 6 B instead of 8 (the K1 -> K2 round trip is 3/4 of the bytes).  Rows keep the
// [fa][C][S] order (row pitch 6 S bytes); the int8 exponents follow the packed rows as [fa][S / kPkG][C / 8] (a K2
// tile's exponents are one 16-B load).  A value v of a block whose largest component magnitude m has frexp exponent
// e (m < 2^e) is stored as rint(v 2^(23-e)): error <= 2^(e-24) <= m 2^-23, i.e. within one fp32 ulp of the block's
// largest value.  A strong target raises the exponent of its own range bins' blocks only.
constexpr int kPkG = 16;
typedef unsigned u3v __attribute__((ext_vector_type(3)));
typedef unsigned u2a __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
RSL_DEV unsigned pk_q(float v, int e) {
  const float s = fminf(fmaxf(rintf(ldexpf(v, 23 - e)), -8388607.f), 8388607.f);
  return (unsigned)(int)s;
}
// four values (two complex) -> three dwords
RSL_DEV u3v pk_pack(float2 lo, float2 hi, int e) {
  const unsigned a = pk_q(lo.x, e), b = pk_q(lo.y, e), c = pk_q(hi.x, e), d = pk_q(hi.y, e);
  u3v w;
  w.x = (a & 0xFFFFFFu) | (b << 24);
  w.y = ((b >> 8) & 0xFFFFu) | (c << 16);
  w.z = ((c >> 16) & 0xFFu) | (d << 8);
  return w;
}
// dword index of complex k of a packed row, and the two dwords holding it (odd k starts 2 B into the first)
RSL_DEV unsigned pk_word(unsigned k) { return (3u * k) >> 1; }
RSL_DEV float2 pk_unpack(u2a w, unsigned k, int e) {
  const unsigned long long v = ((((unsigned long long)w.y) << 32) | w.x) >> ((k & 1u) ? 16 : 0);
  const int re = ((int)((unsigned)v << 8)) >> 8;
  const int im = ((int)((unsigned)(v >> 24) << 8)) >> 8;
  return make_float2(ldexpf((float)re, e - 23), ldexpf((float)im, e - 23));
}

// Grid of a persistent kernel: resident workgroups only (occupancy x CUs), at most ntile.
static long resident_grid(const void* kern, size_t lds, long ntile) {
  int nb = 0, dev = 0, ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kThreads, lds) != hipSuccess || nb < 1) nb = 1;
  if (nb > 8) nb = 8;
  if (const char* e = getenv("RSL_RF_BPC"))  // blocks-per-CU cap (pipelined chain: room for a concurrent kernel)
    if (atoi(e) > 0 && atoi(e) < nb) nb = atoi(e);
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long g = (long)nb * ncu;
  return g < ntile ? g : (ntile > 0 ? ntile : 1);
}

// The largest float t <= thr: for a float p, (double)p > thr  <=>  p > t.
float threshold_as_float(double thr) {
  float t = (float)thr;
  if ((double)t > thr) t = nextafterf(t, -INFINITY);
  return t;
}

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
  constexpr int LD = lp_row(S);
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
    for (int idx = tid; idx < CB * S / 2; idx += kThreads) {
      const int r = idx / (S / 2), s2 = idx - r * (S / 2);
      float2 lo = make_float2(0.f, 0.f), hi = lo;
      if (r < nrows) {
        const float4 x = src4[(size_t)r * (S / 2) + s2];
        const float4 t = tab4[s2];
        lo = cmul(make_float2(x.x, x.y), make_float2(t.x, t.y));
        hi = cmul(make_float2(x.z, x.w), make_float2(t.z, t.w));
      }
      buf[r * LD + lp(2 * s2)] = lo;
      buf[r * LD + lp(2 * s2 + 1)] = hi;
    }
  } else {
    for (int idx = tid; idx < CB * S; idx += kThreads) {
      const int r = idx / S, s = idx - r * S;
      buf[r * LD + lp(s)] = (r < nrows) ? cmul(src[(size_t)r * S + s], table[s]) : make_float2(0.f, 0.f);
    }
  }
  __syncthreads();
  fft_rows<S, CB, kThreads, LD>(buf, tws, tid);
  if (dc) {
    if (tid < CB) buf[tid * LD] = make_float2(0.f, 0.f);
    __syncthreads();
  }
  float2* dst = work + ((size_t)fa * C + cbeg) * S;
  if constexpr (S % 2 == 0) {
    float4* dst4 = reinterpret_cast<float4*>(dst);
    for (int idx = tid; idx < nrows * S / 2; idx += kThreads) {
      const int r = idx / (S / 2), s2 = idx - r * (S / 2);
      const float2 lo = buf[r * LD + lp(2 * s2)], hi = buf[r * LD + lp(2 * s2 + 1)];
      dst4[idx] = make_float4(lo.x, lo.y, hi.x, hi.y);
    }
  } else {
    for (int idx = tid; idx < nrows * S; idx += kThreads) {
      const int r = idx / S, s = idx - r * S;
      dst[idx] = buf[r * LD + lp(s)];
    }
  }
}

// Persistent K1: the grid holds only resident workgroups; each loops over (frame, antenna, chirp-block) tiles
// and issues the next tile's 16-B global loads into registers before running the current tile's LDS FFT, so
// HBM latency overlaps the FFT instead of stalling every tile's load phase.  Requires even S with
// rows_for(S) * S / 2 a multiple of the block size (every power-of-two S >= 16).
// CP (cache policy) bit 0: nt cube loads, bit 1: nt work stores, bit 2: masked loads (A/B).
// PD: tiles in flight per workgroup (1: the next tile's loads during this tile's FFT; 2: the next two, in two register
// sets used in turn, registers capped for 3 waves per SIMD (9 dwords spilled); 3: as 2, uncapped, 2 waves per SIMD).
// Measured (tools/rf_pd.py, tools/cpb.sh): depth 2 is faster before the plain Doppler kernel (1.55 vs 1.68 ms per 1000
// cfg2 frames) but not in the chain (1.63 vs 1.63 ms; 178.9 vs 178.5 k frames/s), so depth 1 stays the default.
template <int S, int CB, int DBG = 0, int CP = 0, int PD = 1, bool DYN = false, bool PK = false>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(PD == 2 ? 3 : 1))) void k_range_fft_p(const float2* __restrict__ cube, int A, int Ct, int c0,
                                                           int C, long ntile, const float2* __restrict__ table,
                                                           const float2* __restrict__ tw, int dc,
                                                           float2* __restrict__ work, int slot,
                                                           signed char* __restrict__ wexp) {
  static_assert(!PK || (S / 2 == kThreads && CB == 8), "packed work: S = 512, one bin pair per thread");
  constexpr int LD = lp_row(S);
  constexpr int H = S / 2;                 // float4 (2 complex) per row
  constexpr int PF = CB * H / kThreads;    // float4 per thread per tile
  static_assert((CB * H) % kThreads == 0, "tile must split evenly over the block");
  static_assert(PD >= 1 && PD <= 3, "prefetch variant 1, 2 or 3");
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* buf = sm + lp_row(S);
  const int tid = threadIdx.x;
  const int ncb = (C + CB - 1) / CB;
  const long G = gridDim.x;
  for (int k = tid; k < S; k += kThreads) tws[lp(k)] = tw[k];
  const float4* tab4 = reinterpret_cast<const float4*>(table);
  // the thread's table entries (one float4 when the block spans whole rows: every q hits the same samples)
  constexpr int NTAB = (kThreads % H == 0) ? 1 : PF;
  float4 tab[NTAB];
#pragma unroll
  for (int q = 0; q < NTAB; ++q) tab[q] = tab4[(tid + q * kThreads) % H];
  auto load = [&](float4(&nx)[PF], long t) {
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    const int nrows = min(CB, C - cb * CB);
    const float4* src4 = reinterpret_cast<const float4*>(cube + ((size_t)fa * Ct + c0 + cb * CB) * S);
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int idx = tid + q * kThreads;
      const int r = idx / H;
      // unconditional (clamped) load, rows past nrows zeroed at consumption (a select on the loaded value here
      // would wait for it); CP bit 2: the masked-load form
      if constexpr ((CP & 4) != 0)
        nx[q] = (r < nrows) ? src4[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
      else
        nx[q] = ld16<(CP & 1) != 0>(src4 + (r < nrows ? idx : 0));
    }
  };
  // one tile: stage nx (x conj(ref) w) in LDS, refill nx with tile t + PD G, FFT, DC bin, store
  // DYN: workgroup b serves XCD x = b % 8 (dispatch order) and walks that XCD's tile range [lo, hi): its first two
  // tiles are static, every later one comes from the XCD's dequeue head, claimed one tile ahead (the atomic returns
  // during a whole tile), so workgroups that start late (CUs held by a concurrent kernel) take fewer tiles
  __shared__ long s_nn;
  const int xcd = blockIdx.x & 7;
  const long gx = (G - xcd + 7) / 8;
  const long lo = DYN ? xcd * ntile / 8 : 0, hi = DYN ? (xcd + 1) * ntile / 8 : ntile;
  unsigned* head = &g_rf_q[slot][0][xcd][0];
  auto body = [&](float4(&nx)[PF], long t, long tn) {
    unsigned claim = 0;
    if (DYN && tid == 0) claim = atomicAdd(head, 1u);
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    const int nrows = min(CB, C - cb * CB);
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int idx = tid + q * kThreads;
      const int r = idx / H, s2 = idx - r * H;
      float4 x = nx[q];
      const float4 tb = tab[NTAB == 1 ? 0 : q];
      if constexpr ((CP & 4) == 0)
        if (r >= nrows) x = make_float4(0.f, 0.f, 0.f, 0.f);
      buf[r * LD + lp(2 * s2)] = cmul(make_float2(x.x, x.y), make_float2(tb.x, tb.y));
      buf[r * LD + lp(2 * s2 + 1)] = cmul(make_float2(x.z, x.w), make_float2(tb.z, tb.w));
    }
    __syncthreads();
    if (tn < hi) load(nx, tn);  // in flight during the FFT below (and the next PD - 1 tiles)
    if constexpr (DBG != 1) fft_rows<S, CB, kThreads, LD, true>(buf, tws, tid);  // DBG 1: no FFT (ablation)
    if (dc) {
      if (tid < CB) buf[tid * LD] = make_float2(0.f, 0.f);
      __syncthreads();
    }
    float4* dst4 = reinterpret_cast<float4*>(work + ((size_t)fa * C + cb * CB) * S);
    if constexpr (PK) {
      // H == kThreads: thread tid holds bin pair s2 = tid of every row q of the tile.  One exponent per (tile, group
      // of kPkG bins): the max over the thread's 8 rows, then over the group's 8 lanes by DPP (quad_perm [1,0,3,2],
      // [2,3,0,1], row_half_mirror)
      float2 lo[PF], hi[PF];
      float m = 0.f;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        lo[q] = buf[q * LD + lp(2 * tid)];
        hi[q] = buf[q * LD + lp(2 * tid + 1)];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(lo[q].x), fabsf(lo[q].y)), fmaxf(fabsf(hi[q].x), fabsf(hi[q].y))));
      }
      m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0xB1, 0xF, 0xF, true)));
      m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x4E, 0xF, 0xF, true)));
      m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x141, 0xF, 0xF, true)));
      int e;
      (void)frexpf(m, &e);
      // three dwords per (row, bin pair) at 12-B steps (a u3v is 16-B sized: no u3v pointer arithmetic)
      unsigned* dst3 = reinterpret_cast<unsigned*>(work) + ((size_t)fa * C + cb * CB) * (3 * S / 2) + 3 * tid;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        if (q < nrows) {
          const u3v w = pk_pack(lo[q], hi[q], e);
          unsigned* d3 = dst3 + q * (3 * S / 2);
          if constexpr ((CP & 2) != 0) {
            __builtin_nontemporal_store(w.x, d3);
            __builtin_nontemporal_store(w.y, d3 + 1);
            __builtin_nontemporal_store(w.z, d3 + 2);
          } else {
            d3[0] = w.x;
            d3[1] = w.y;
            d3[2] = w.z;
          }
        }
      }
      // exponents [fa][group][chirp block]
      if ((tid & 7) == 0) wexp[((size_t)fa * (S / kPkG) + (tid >> 3)) * (C / CB) + cb] = (signed char)e;
    }
#pragma unroll
    for (int q = 0; q < PF && !PK; ++q) {
      const int idx = tid + q * kThreads;
      const int r = idx / H, s2 = idx - r * H;
      if (r < nrows) {
        const float2 lo = buf[r * LD + lp(2 * s2)], hi = buf[r * LD + lp(2 * s2 + 1)];
        if constexpr ((CP & 2) != 0)
          st16<true>(dst4 + idx, make_float4(lo.x, lo.y, hi.x, hi.y));
        else
          dst4[idx] = make_float4(lo.x, lo.y, hi.x, hi.y);
      }
    }
    if (DYN && tid == 0) s_nn = lo + 2 * gx + (long)claim;
    __syncthreads();  // buf is rewritten by the next tile
  };
  if constexpr (DYN) {
    static_assert(PD == 1, "dequeue variant: one tile in flight");
    long t = lo + (blockIdx.x >> 3), tn = t + gx;
    float4 nx[PF];
    if (t < hi) load(nx, t);
    while (t < hi) {
      body(nx, t, tn);
      t = tn;
      tn = s_nn;  // written before body's last barrier, rewritten only after the next body's first one
    }
    // every dequeue of this workgroup has returned: the XCD's last leaver resets the slot for its next launch
    if (tid == 0 && atomicAdd(&g_rf_q[slot][1][xcd][0], 1u) == (unsigned)gx - 1u) {
      atomicExch(head, 0u);
      atomicExch(&g_rf_q[slot][1][xcd][0], 0u);
    }
    return;
  }
  long t = blockIdx.x;
  if constexpr (PD == 1) {
    float4 nx[PF];
    if (t < ntile) load(nx, t);
    for (; t < ntile; t += G) body(nx, t, t + G);
  } else {
    float4 na[PF], nb[PF];
    if (t < ntile) load(na, t);
    if (t + G < ntile) load(nb, t + G);
    for (; t < ntile; t += 2 * G) {
      body(na, t, t + 2 * G);
      if (t + G < ntile) body(nb, t + G, t + 3 * G);
    }
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
  constexpr int LD = lp_row(C) | 1;  // odd: conflict-free transposed (column) writes
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
    buf[kk * LD + lp(c)] = (kk < nk) ? src[(size_t)c * S + kk] : make_float2(0.f, 0.f);
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
    dst[(size_t)i * C + j] = buf[kk * LD + lp(d)];
  }
}

// Tile body after the LDS fill (and its barrier): Doppler FFT, shifted RDS store, |X|^2 tile, 3x3 detection.
template <int C, int KB, int NT, bool PAD, int DBG>
RSL_DEV void dd_tile_compute(float2* buf, const float2* tws, int S, int k0, unsigned fa, float2* __restrict__ rds,
                             float thr_f, int i_lo, int i_hi, unsigned long long* __restrict__ mask,
                             int* __restrict__ row_count, float* __restrict__ dbmap, float* __restrict__ pk_pow) {
  constexpr int NR = KB + 2;
  constexpr int LD = lp_rowp<PAD>(C) | 1;
  constexpr int W = (C + 63) / 64;
  constexpr int PER = (NR * C + NT - 1) / NT;
  const int tid = threadIdx.x;
  if constexpr (DBG != 1) fft_rows<C, NR, NT, LD, false, PAD>(buf, tws, tid);  // DBG 1: no FFT (ablation)
  const int hs = S / 2, hc = C / 2;
  int i0 = k0 + hs;  // shifted row of LDS row 1
  if (i0 >= S) i0 -= S;
  float2* dst = rds + ((size_t)fa * S + i0) * C;
  // one pass over the tile: shifted RDS stores (interior rows) and |X|^2 kept in registers
  float pr[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = tid + q * NT;
    pr[q] = 0.f;
    if (idx < NR * C) {
      const int r = idx / C, j = idx - r * C;  // j: shifted doppler index
      int d = j - hc;                          // out[j] = X[(j - C//2) mod C]
      if (d < 0) d += C;
      const float2 z = buf[r * LD + lpp<PAD>(d)];
      if (DBG != 2 && r >= 1 && r <= KB) dst[(size_t)(r - 1) * C + j] = z;  // DBG 2: no RDS store
      pr[q] = cabs2(z);
    }
  }
  __syncthreads();
  float* pw = reinterpret_cast<float*>(buf);  // power tile [NR][C], shifted doppler order
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = tid + q * NT;
    if (idx < NR * C) pw[idx] = pr[q];
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  for (int kk = wave; kk < (DBG == 3 ? 0 : KB); kk += NT / 64) {  // DBG 3: no detection
    const int i = i0 + kk;
    const bool gate = (i >= i_lo && i <= i_hi);
    const bool has_up = i > 0, has_dn = i + 1 < S;
    const float* up = pw + kk * C;
    const float* mid = up + C;
    const float* dn = mid + C;
    const size_t row = (size_t)fa * S + i;
    int cnt = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int j = w * 64 + lane;
      bool pk = false;
      float p = 0.f;
      if (j < C) {
        // 3x3 window max with 'reflect' edges (an out-of-range neighbour repeats an in-window cell)
        const int jl = j > 0 ? j - 1 : j, jr = j + 1 < C ? j + 1 : j;
        p = mid[j];
        float m = fmaxf(fmaxf(mid[jl], p), mid[jr]);
        if (has_up) m = fmaxf(m, fmaxf(fmaxf(up[jl], up[j]), up[jr]));
        if (has_dn) m = fmaxf(m, fmaxf(fmaxf(dn[jl], dn[j]), dn[jr]));
        pk = gate && (p > thr_f) && (p >= m);
        if (dbmap) dbmap[row * C + j] = 10.f * log10f(p + 1e-12f);
      }
      const unsigned long long b = __ballot(pk);
      if (lane == 0) mask[row * W + w] = b;
      if (pk_pow && pk) pk_pow[row * C + cnt + __popcll(b & ((1ull << lane) - 1ull))] = p;
      cnt += __popcll(b);
    }
    if (lane == 0) row_count[row] = cnt;
  }
}

// Register form of the tile body for C = 64 NCH and KB = 8 NRH with NCH * NRH waves: wave (ch, rh) owns Doppler
// columns 64 ch + lane and interior rows 8 rh + 1 .. 8 rh + 8.  Each lane reads its 10 LDS values once (8 rows +
// halo), stores the shifted RDS rows (coalesced), takes the vertical 3-max in registers and the horizontal one
// from neighbouring lanes (LDS only for the wave-edge columns), and ballots the peaks: no power tile in LDS and
// no 9-read window per cell.  Same decisions as the general body (max is separable: 3x3 max = max of the
// column-wise 3-max over j-1, j, j+1; 'reflect' edges repeat the in-window cell).
template <int C, int KB, int NT>
constexpr bool dd_reg_ok() {
  return C % 64 == 0 && KB % 8 == 0 && (C / 64) * (KB / 8) * 64 == NT && KB * (C / 64) <= 64;
}

template <int C, int KB, int NT, int DBG = 0, int CP = 0>
RSL_DEV void dd_tile_compute_reg(const float2* buf, float* xch, int S, int k0, unsigned fa, float2* __restrict__ rds,
                                 float thr_f, int i_lo, int i_hi, unsigned long long* __restrict__ mask,
                                 int* __restrict__ row_count, float* __restrict__ dbmap,
                                 float* __restrict__ pk_pow, int tid_in = -1) {
  constexpr int LD = lp_row(C) | 1;
  constexpr int NCH = C / 64;
  // tid_in: a laundered thread index from a persistent caller (keeps per-thread addresses out of its tile loop)
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = wave % NCH, rh = wave / NCH;
  const int j = ch * 64 + lane;  // shifted Doppler column: out[j] = X[(j - C//2) mod C]
  int d = j - C / 2;
  if (d < 0) d += C;
  int i0 = k0 + S / 2;  // shifted range row of LDS row 1
  if (i0 >= S) i0 -= S;
  const int rb = rh * 8;  // LDS rows rb .. rb + 9; interior rows rb + 1 .. rb + 8
  float p[10];
  const float2* col = buf + lp(d);
  float2* dst = rds + ((size_t)fa * S + i0 + rb) * C + j;
  float2 zp = make_float2(0.f, 0.f);  // CP bit 4: the first row of the current row pair
  const bool odd = (lane & 1) != 0;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const float2 z = col[(rb + r) * LD];
    p[r] = cabs2(z);
    if constexpr ((CP & 16) != 0) {
      // 16-B stores: lane pairs swap one value per row pair (DPP quad_perm [1,0,3,2]), then the even lane stores
      // row r - 2 at columns (j, j + 1) and the odd lane row r - 1 at (j - 1, j)
      if (r == 1 || r == 3 || r == 5 || r == 7) zp = z;
      if (r == 2 || r == 4 || r == 6 || r == 8) {
        const float2 snd = odd ? zp : z;
        float2 rcv;
        rcv.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd.x), 0xB1, 0xF, 0xF, true));
        rcv.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd.y), 0xB1, 0xF, 0xF, true));
        const float4 v = odd ? make_float4(rcv.x, rcv.y, z.x, z.y) : make_float4(zp.x, zp.y, rcv.x, rcv.y);
        float2* q = dst + (size_t)(r - 2 + (odd ? 1 : 0)) * C - (odd ? 1 : 0);
        st16<(CP & 2) != 0>(reinterpret_cast<float4*>(q), v);
      }
    } else if (r >= 1 && r <= 8) {
      if constexpr ((CP & 2) != 0)
        st8<true>(dst + (size_t)(r - 1) * C, z);
      else
        dst[(size_t)(r - 1) * C] = z;
    }
  }
  float vm[8];
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) {
    const int i = i0 + rb + rr;
    float m = p[rr + 1];
    if (i > 0) m = fmaxf(m, p[rr]);          // 'reflect' at the shifted range edges: no neighbour
    if (i + 1 < S) m = fmaxf(m, p[rr + 2]);
    vm[rr] = m;
  }
  // wave-edge columns for the horizontal neighbours: xch[(rh * 8 + rr) * 2 NCH + 2 ch + {0: lane 0, 1: lane 63}]
  float* ex = xch + (rb + 0) * 2 * NCH;
  if (lane == 0 || lane == 63) {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) ex[rr * 2 * NCH + 2 * ch + (lane == 63)] = vm[rr];
  }
  __syncthreads();
  unsigned long long* wb = reinterpret_cast<unsigned long long*>(xch + KB * 2 * NCH);  // [KB][NCH] ballots
  bool pkv[8];
  unsigned long long bal[8];  // this wave's ballot word of each of its rows (wave-uniform)
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) {
    // neighbour lanes by DPP wavefront shifts (wave_shr:1 / wave_shl:1, one VALU op each) instead of ds_bpermute
    // round trips through the LDS unit; lanes 0 / 63 take their outside neighbour from the exchange words below
    float l, r;
    if constexpr ((CP & 64) != 0) {
      l = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(vm[rr]), 0x138, 0xF, 0xF, false));
      r = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(vm[rr]), 0x130, 0xF, 0xF, false));
    } else {
      l = __shfl_up(vm[rr], 1);
      r = __shfl_down(vm[rr], 1);
    }
    if (lane == 0) l = ch > 0 ? ex[rr * 2 * NCH + 2 * (ch - 1) + 1] : vm[rr];
    if (lane == 63) r = ch + 1 < NCH ? ex[rr * 2 * NCH + 2 * (ch + 1)] : vm[rr];
    const float m = fmaxf(fmaxf(l, vm[rr]), r);
    const int i = i0 + rb + rr;
    const float pc = p[rr + 1];
    const bool pk = (i >= i_lo && i <= i_hi) && (pc > thr_f) && (pc >= m);
    pkv[rr] = pk;
    const unsigned long long b = __ballot(pk);
    bal[rr] = b;
    if (lane == 0) wb[(rb + rr) * NCH + ch] = b;
    if (dbmap) dbmap[((size_t)fa * S + i) * C + j] = 10.f * log10f(pc + 1e-12f);
  }
  __syncthreads();
  // peak powers compact over the tile's KB rows (one contiguous run from the tile's first row slot): an exclusive
  // scan of the tile's KB * NCH <= 64 ballot-word popcounts (one word per lane) gives every word's offset; each row
  // reads its word's offset with one v_readlane (the word index is wave-uniform) and ranks its lanes in its ballot
  const unsigned long long myw = lane < KB * NCH ? wb[lane] : 0ull;
  const int cw = __popcll(myw);
  int incl = cw;
  if constexpr ((CP & 64) != 0) {
    incl = wave_incl_scan(incl);
  } else {
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const int v = __shfl_up(incl, dd);
      if (lane >= dd) incl += v;
    }
  }
  const int excl = incl - cw;
  float* tile_pk = pk_pow ? pk_pow + ((size_t)fa * S + i0) * C : nullptr;
  const unsigned long long lt = (1ull << lane) - 1ull;
  if constexpr ((CP & 8) != 0) {
    // CP bit 3: stage the tile's compacted peak powers in the (now dead) LDS tile, then one block-wide contiguous
    // store of the whole run instead of 8 partial-line stores per wave
    float* stg = reinterpret_cast<float*>(const_cast<float2*>(buf));
    const int total = __builtin_amdgcn_readlane(incl, 63);
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int off = __builtin_amdgcn_readlane(excl, (rb + rr) * NCH + ch);
      if (pkv[rr]) stg[off + __popcll(bal[rr] & lt)] = p[rr + 1];
    }
    __syncthreads();
    if (DBG != 4 && tile_pk)
      for (int k = tid; k < total; k += NT) tile_pk[k] = stg[k];
  } else {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int off = __builtin_amdgcn_readlane(excl, (rb + rr) * NCH + ch);
      if (DBG != 4 && tile_pk && pkv[rr]) tile_pk[off + __popcll(bal[rr] & lt)] = p[rr + 1];
    }
  }
  // the tile's mask words and row counts from the ballots in LDS, one coalesced store each (the tile's shifted rows
  // i0 .. i0 + KB - 1 are contiguous), instead of single-lane stores per row and wave
  if (DBG != 5) {  // DBG 5: no mask / count stores (ablation)
    const size_t row0 = (size_t)fa * S + i0;
    if (tid < KB * NCH) mask[row0 * NCH + tid] = wb[tid];
    if (tid < KB) {
      int cnt = 0;
#pragma unroll
      for (int c = 0; c < NCH; ++c) cnt += __popcll(wb[tid * NCH + c]);
      row_count[row0 + tid] = cnt;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K2+K3 fused: Doppler FFT, fftshift, RDS store AND peak detection (dechirp.py:208-271) in one pass.
// The block FFTs KB interior range bins plus one halo bin on each side (KB+2 rows), writes the KB shifted
// RDS rows, overwrites the LDS tile with |X|^2, and runs the 3x3 'reflect' local-max test, threshold and
// range gate on the interior rows.  Halo rows are neighbours in shifted range space except across the
// shifted edges i = 0 / S-1, where 'reflect' means "no neighbour".  Saves k_detect's full RDS re-read.
// Requires S % KB == 0 and (S/2) % KB == 0 (each block's shifted rows contiguous).
// ---------------------------------------------------------------------------------------------
// CP (cache policy) bit 0: nt interior loads, bit 1: nt RDS stores, bit 2: nt halo loads; register body: bit 3 LDS-staged
// peak powers, bit 4 16-B RDS stores, bit 5 16-B interior loads, bit 6 DPP neighbour lanes and wave scan
template <int C, int KB, int NT, bool PAD, int DBG = 0, int CP = 0, bool PK = false>
__global__ __launch_bounds__(NT) void k_doppler_detect(const float2* __restrict__ work, int S,
                                                             const float2* __restrict__ tw, float2* __restrict__ rds,
                                                             float thr_f, int i_lo, int i_hi,
                                                             unsigned long long* __restrict__ mask,
                                                             int* __restrict__ row_count, float* __restrict__ dbmap,
                                                             float* __restrict__ pk_pow, int xcd,
                                                             const signed char* __restrict__ wexp) {
  constexpr int NR = KB + 2;
  constexpr int LD = lp_rowp<PAD>(C) | 1;  // odd: conflict-free transposed (column) writes
    constexpr int PER = (NR * C + NT - 1) / NT;
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* buf = sm + C;
  const int tid = threadIdx.x;
  const unsigned nkb = (unsigned)(S / KB);
  const unsigned tile = xcd ? (unsigned)xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  const int kb = (int)(tile % nkb);
  const unsigned fa = tile / nkb;
  const int k0 = kb * KB;
  const float2* src = work + (size_t)fa * C * S;
  // all of the thread's loads in flight before the first LDS write (a rolled loop waits on each load in turn);
  // the twiddles first, so their LDS copy waits only on them
  constexpr int TWP = (C + NT - 1) / NT;
  float2 twv[TWP];
#pragma unroll
  for (int q = 0; q < TWP; ++q)
    if (C % NT == 0 || tid + q * NT < C) twv[q] = tw[tid + q * NT];
  // structured map: thread = (interior range bin ri, chirp slot cs), chirps cs + CS q at a constant stride
  // (one address add per load, 128-B aligned row segments), then the two halo rows spread over all threads
  constexpr int CS = NT / KB;
  constexpr bool STRUCT = (NT % KB == 0) && (C % (NT / KB) == 0) && ((NT / KB) % 8 == 0) && (C / (NT / KB) <= 16);
  // CP bit 5: interior rows as 16-B loads (a lane reads two adjacent range bins of one chirp: half the load
  // instructions); thread = (bin pair rp, chirp slot cs2), chirps cs2 + CS2 q
  constexpr int CS2 = NT / (KB / 2);
  constexpr bool WIDE = ((CP & 32) != 0) && (KB % 2 == 0) && (NT % (KB / 2) == 0) && (C % CS2 == 0);
  static_assert(!PK || (STRUCT && !WIDE), "packed work: structured tile map");
  if constexpr (PK) {
    // packed rows (see pk_pack): a lane reads one bin pair (2 p, 2 p + 1) of a chirp row as one aligned 12-B load
    // (dwords 3 p .. 3 p + 2 of the row); thread = (pair rp, chirp slot cs2), chirps cs2 + 32 q.  KB == kPkG: the tile
    // is one exponent group, whose C / 8 chirp-block exponents are one 16-B load; the halo values take their
    // neighbour group's exponent byte
    static_assert(KB == kPkG && C == 128 && CS2 == 32, "packed work: C = 128, KB = 16");
    constexpr int PI = C / CS2, PH = (2 * C + NT - 1) / NT;
    const unsigned rw = 3u * (unsigned)S / 2u;  // dwords per packed row
    const unsigned* srcw = reinterpret_cast<const unsigned*>(work) + (size_t)fa * C * rw;
    const signed char* ex = wexp + (size_t)fa * (unsigned)(S / kPkG) * (C / 8);
    const int rp = tid % (KB / 2), cs = tid / (KB / 2);
    u3v lw[PI];
    const unsigned* p = srcw + cs * rw + 3u * (unsigned)(k0 / 2 + rp);
#pragma unroll
    for (int q = 0; q < PI; ++q) {
      const unsigned* a = p + (unsigned)(q * CS2) * rw;
      lw[q] = u3v{a[0], a[1], a[2]};
    }
    const uint4 eg = *reinterpret_cast<const uint4*>(ex + (unsigned)(k0 / kPkG) * (C / 8));
    int kl = k0 - 1, kh = k0 + KB;
    if (kl < 0) kl += S;
    if (kh >= S) kh -= S;
    u2a hw[PH];
    int he[PH];
    unsigned hk[PH];
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        hk[h] = (unsigned)(side ? kh : kl);
        hw[h] = *reinterpret_cast<const u2a*>(srcw + c * rw + pk_word(hk[h]));
        he[h] = ex[(hk[h] / kPkG) * (C / 8) + c / 8];
      }
    }
#pragma unroll
    for (int q = 0; q < TWP; ++q)
      if (C % NT == 0 || tid + q * NT < C) tws[tid + q * NT] = twv[q];
    float2* row0 = buf + (2 * rp + 1) * LD + lpp<PAD>(cs);
    // chirp cs + 32 q is in block cs / 8 + 4 q: byte cs / 8 of dword q
    const unsigned bsh = (unsigned)(cs >> 3) * 8u;
#pragma unroll
    for (int q = 0; q < PI; ++q) {
      const unsigned dw = q == 0 ? eg.x : q == 1 ? eg.y : q == 2 ? eg.z : eg.w;
      const int e = (int)(signed char)(dw >> bsh);
      row0[lpp<PAD>(q * CS2)] = pk_unpack(u2a{lw[q].x, lw[q].y}, 0u, e);
      row0[LD + lpp<PAD>(q * CS2)] = pk_unpack(u2a{lw[q].y, lw[q].z}, 1u, e);
    }
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        buf[(side ? NR - 1 : 0) * LD + lpp<PAD>(c)] = pk_unpack(hw[h], hk[h], he[h]);
      }
    }
  } else if constexpr (WIDE) {
    constexpr int PI = C / CS2, PH = (2 * C + NT - 1) / NT;
    const int rp = tid % (KB / 2), cs = tid / (KB / 2);
    float4 ld[PI];
    float2 lh[PH];
    const float4* p = reinterpret_cast<const float4*>(src + (unsigned)(cs * S + k0 + 2 * rp));
#pragma unroll
    for (int q = 0; q < PI; ++q) ld[q] = p[(unsigned)(q * CS2 * S / 2)];
    int kl = k0 - 1, kh = k0 + KB;
    if (kl < 0) kl += S;
    if (kh >= S) kh -= S;
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        lh[h] = src[(unsigned)(c * S + (side ? kh : kl))];
      }
    }
#pragma unroll
    for (int q = 0; q < TWP; ++q)
      if (C % NT == 0 || tid + q * NT < C) tws[tid + q * NT] = twv[q];
    float2* row0 = buf + (2 * rp + 1) * LD + lpp<PAD>(cs);
#pragma unroll
    for (int q = 0; q < PI; ++q) {
      row0[lpp<PAD>(q * CS2)] = make_float2(ld[q].x, ld[q].y);
      row0[LD + lpp<PAD>(q * CS2)] = make_float2(ld[q].z, ld[q].w);
    }
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        buf[(side ? NR - 1 : 0) * LD + lpp<PAD>(c)] = lh[h];
      }
    }
  } else if constexpr (STRUCT) {
    constexpr int PI = C / CS, PH = (2 * C + NT - 1) / NT;
    const int ri = tid % KB, cs = tid / KB;
    float2 ld[PI + PH];
    const float2* p = src + (unsigned)(cs * S + k0 + ri);
#pragma unroll
    for (int q = 0; q < PI; ++q) {
      if constexpr ((CP & 1) != 0)
        ld[q] = ld8<true>(p + (unsigned)(q * CS * S));
      else
        ld[q] = p[(unsigned)(q * CS * S)];
    }
    int kl = k0 - 1, kh = k0 + KB;  // halo range bins (periodic: reflect is applied in the detect stage)
    if (kl < 0) kl += S;
    if (kh >= S) kh -= S;
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        if constexpr ((CP & 4) != 0)
          ld[PI + h] = ld8<true>(src + (unsigned)(c * S + (side ? kh : kl)));
        else
          ld[PI + h] = src[(unsigned)(c * S + (side ? kh : kl))];
      }
    }
#pragma unroll
    for (int q = 0; q < TWP; ++q)
      if (C % NT == 0 || tid + q * NT < C) tws[tid + q * NT] = twv[q];
    float2* row = buf + (ri + 1) * LD + lpp<PAD>(cs);
#pragma unroll
    for (int q = 0; q < PI; ++q) row[lpp<PAD>(q * CS)] = ld[q];
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        buf[(side ? NR - 1 : 0) * LD + lpp<PAD>(c)] = ld[PI + h];
      }
    }
  } else {
    float2 ld[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = tid + q * NT;
      if ((NR * C) % NT == 0 || idx < NR * C) {
        const int c = idx / NR, r = idx - c * NR;
        int k = k0 - 1 + r;  // unshifted range bin of LDS row r
        k = k < 0 ? k + S : (k >= S ? k - S : k);
        ld[q] = src[(unsigned)(c * S + k)];
      }
    }
#pragma unroll
    for (int q = 0; q < TWP; ++q)
      if (C % NT == 0 || tid + q * NT < C) tws[tid + q * NT] = twv[q];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = tid + q * NT;
      if ((NR * C) % NT == 0 || idx < NR * C) {
        const int c = idx / NR, r = idx - c * NR;
        buf[r * LD + lpp<PAD>(c)] = ld[q];
      }
    }
  }
  __syncthreads();
  if constexpr (PAD && (DBG == 0 || DBG >= 4) && dd_reg_ok<C, KB, NT>()) {
    fft_rows<C, NR, NT, LD, false, PAD>(buf, tws, tid);
    dd_tile_compute_reg<C, KB, NT, DBG, CP>(buf, reinterpret_cast<float*>(buf + NR * LD), S, k0, fa, rds, thr_f, i_lo, i_hi,
                                   mask, row_count, dbmap, pk_pow);
  } else {
    dd_tile_compute<C, KB, NT, PAD, DBG>(buf, tws, S, k0, fa, rds, thr_f, i_lo, i_hi, mask, row_count, dbmap,
                                         pk_pow);
  }
}

// Persistent K2+K3: the grid holds only resident workgroups.  Each XCD walks a contiguous range of tiles
// (workgroup b serves XCD b % 8, tiles slot, slot + nb8, ... of that range: neighbouring tiles, whose halo rows
// share cache lines, run back to back in one L2), and every workgroup issues the next tile's global loads into
// registers right after staging the current tile in LDS, so HBM latency overlaps the FFT / store / detect phases.
template <int C, int KB, int NT>
__global__ __launch_bounds__(NT) void k_doppler_detect_p(const float2* __restrict__ work, int S,
                                                         const float2* __restrict__ tw, float2* __restrict__ rds,
                                                         float thr_f, int i_lo, int i_hi,
                                                         unsigned long long* __restrict__ mask,
                                                         int* __restrict__ row_count, float* __restrict__ dbmap,
                                                         float* __restrict__ pk_pow, long ntile) {
  constexpr int NR = KB + 2;
  constexpr int LD = lp_row(C) | 1;
  constexpr int CS = NT / KB;
  static_assert((NT % KB == 0) && (C % (NT / KB) == 0) && ((NT / KB) % 8 == 0) && (C / (NT / KB) <= 16),
                "structured tile map required");
  constexpr int PI = C / CS, PH = (2 * C + NT - 1) / NT;
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* buf = sm + C;
  const int tid = threadIdx.x;
  const int ri = tid % KB, cs = tid / KB;
  for (int k = tid; k < C; k += NT) tws[k] = tw[k];
  const unsigned nkb = (unsigned)(S / KB);
  const long nb8 = gridDim.x >> 3;  // grid is a multiple of 8
  const long x = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const long per = (ntile + 7) >> 3;
  const long lo = x * per, hi = min(ntile, lo + per);
  float2 ld[PI + PH];
  auto issue = [&](long tile) {
    const int kb = (int)((unsigned)tile % nkb);
    const unsigned fa = (unsigned)tile / nkb;
    const int k0 = kb * KB;
    const float2* src = work + (size_t)fa * C * S;
    const float2* p = src + (unsigned)(cs * S + k0 + ri);
#pragma unroll
    for (int q = 0; q < PI; ++q) ld[q] = p[(unsigned)(q * CS * S)];
    int kl = k0 - 1, kh = k0 + KB;
    if (kl < 0) kl += S;
    if (kh >= S) kh -= S;
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        ld[PI + h] = src[(unsigned)(c * S + (side ? kh : kl))];
      }
    }
  };
  long t = lo + slot;
  if (t < hi) issue(t);
  for (; t < hi; t += nb8) {
    float2* row = buf + (ri + 1) * LD + lp(cs);
#pragma unroll
    for (int q = 0; q < PI; ++q) row[lp(q * CS)] = ld[q];
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        buf[(side ? NR - 1 : 0) * LD + lp(c)] = ld[PI + h];
      }
    }
    __syncthreads();
    if (t + nb8 < hi) issue(t + nb8);  // in flight during this tile's FFT, stores and detection
    const int kb = (int)((unsigned)t % nkb);
    if constexpr (dd_reg_ok<C, KB, NT>()) {  // the register body (tile-compact peak powers, as K2)
      // a laundered thread index: the per-thread LDS addresses of the FFT stages and the detection are recomputed
      // per tile instead of being hoisted out of the loop (held across tiles they cost ~70 VGPRs)
      int tl = tid;
      asm volatile("" : "+v"(tl));
      fft_rows<C, NR, NT, LD, false, true>(buf, tws, tl);
      dd_tile_compute_reg<C, KB, NT, 0, 10>(buf, reinterpret_cast<float*>(buf + NR * LD), S, kb * KB,
                                            (unsigned)t / nkb, rds, thr_f, i_lo, i_hi, mask, row_count, dbmap,
                                            pk_pow, tl);
    } else {
      dd_tile_compute<C, KB, NT, true, 0>(buf, tws, S, kb * KB, (unsigned)t / nkb, rds, thr_f, i_lo, i_hi, mask,
                                          row_count, dbmap, pk_pow);
    }
    __syncthreads();  // the detection reads the LDS tile; the next tile's staging overwrites it
  }
}

// XCD-grouped tile order (default on; RSL_DD_XCD=0 for the dispatch order, A/B tuning)
static int dd_xcd() {
  const char* e = getenv("RSL_DD_XCD");
  return e ? atoi(e) != 0 : 1;
}

template <int C, int KB>
static hipError_t launch_k2d_kb(hipStream_t st, const float2* work, int F, int A, int S, const float2* tw,
                                float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask,
                                int* row_count, float* dbmap, float* pk_pow, int* pk_group,
                                const signed char* wexp) {
  *pk_group = 1;  // row-compact, except the register tile body (tile-compact: KB rows)
  const long ntile = (long)F * A * (S / KB);
  // padded LDS rows; RSL_DD_PAD=0 selects plain rows (smaller tile: measured slower, 2.14 vs 1.98 ms per 1000
  // cfg2 frames, also with the registers capped for 8 resident workgroups per CU)
  const char* pe = getenv("RSL_DD_PAD");
  const bool pad = !pe || atoi(pe) != 0;
  // + the register body's exchange area (edge columns and ballots: 16 B per row per 64 columns)
  size_t lds = sizeof(float2) * (C + (size_t)(KB + 2) * ((pad ? lp_row(C) : C) | 1)) + (size_t)KB * (C / 64) * 16;
  if (const char* e = getenv("RSL_DD_LDS"))  // LDS reserved per workgroup (fewer per CU: room for another kernel; A/B)
    if ((size_t)atol(e) > lds) lds = (size_t)atol(e);
  const float thr_f = threshold_as_float(thr_p);
  // one tile per workgroup: a persistent variant with a register prefetch of the next tile measured slower
  // (4.7 vs 3.2 ms per 1000 cfg2 frames; the prefetch registers cost occupancy); rebuilt on the register tile body
  // with a laundered thread index (93 VGPRs, 5 workgroups per CU): still 5.0-5.25 vs 3.85 ms per 2000 frames
  // (tools/ring_ab.py, RSL_DD_PERSIST=1; outputs bit-identical)
  // 256 threads (a 320-thread block that runs each radix-8 stage of the 18-row KB-16 tile in one pass measured
  // slower: 2.72 vs 2.48 ms per 1000 cfg2 frames)
  constexpr int NT = 256;
  // nt RDS stores (the product output, not re-read by this stage; tools/cp_ab.py: 1.68 vs 1.70 ms per 1000 frames);
  // peak powers staged in LDS and stored block-wide (tools/pkb.sh: 187.2-188.5 k vs 184.1-185.2 k frames/s)
  // DPP neighbour lanes and wave scan in the register tile body (CP bit 6; RSL_DD_CP=10 for the ds_bpermute form):
  // tools/ring_ab.py, one call, K2 3.52 vs 3.76 ms per 2000 cfg2 frames, outputs bit-identical
  auto kern = pad ? k_doppler_detect<C, KB, NT, true, 0, 74> : k_doppler_detect<C, KB, NT, false>;
  if (const char* e = getenv("RSL_DD_DBG")) {  // ablation variants (timing only: results are wrong)
    const int v = atoi(e);
    if (v == 1) kern = k_doppler_detect<C, KB, NT, true, 1, 10>;
    if (v == 2) kern = k_doppler_detect<C, KB, NT, true, 2, 10>;
    if (v == 3) kern = k_doppler_detect<C, KB, NT, true, 3, 10>;
    if (v == 4) kern = k_doppler_detect<C, KB, NT, true, 4, 10>;
    if (v == 5) kern = k_doppler_detect<C, KB, NT, true, 5, 10>;
  }
  if constexpr (C == 128 && KB == 16) {
    if (const char* e = getenv("RSL_DD_CP")) {  // cache-policy variants (A/B tuning)
      const int v = atoi(e);
      if (v == 0) kern = k_doppler_detect<C, KB, NT, true, 0, 0>;
      if (v == 1) kern = k_doppler_detect<C, KB, NT, true, 0, 1>;
      if (v == 2) kern = k_doppler_detect<C, KB, NT, true, 0, 2>;
      if (v == 3) kern = k_doppler_detect<C, KB, NT, true, 0, 3>;
      if (v == 4) kern = k_doppler_detect<C, KB, NT, true, 0, 4>;
      if (v == 7) kern = k_doppler_detect<C, KB, NT, true, 0, 7>;
      if (v == 10) kern = k_doppler_detect<C, KB, NT, true, 0, 10>;
      if (v == 26) kern = k_doppler_detect<C, KB, NT, true, 0, 26>;
      if (v == 42) kern = k_doppler_detect<C, KB, NT, true, 0, 42>;  // 10 + 16-B interior loads
      if (v == 74) kern = k_doppler_detect<C, KB, NT, true, 0, 74>;  // 10 + DPP neighbour lanes
      // measured with the DPP body (tools/ring_ab.py, one call): nt interior loads 3.58-3.59, nt interior + halo
      // loads 3.92, 16-B RDS stores 3.59 vs 3.55-3.56 ms per 2000 frames
      if (v == 106) kern = k_doppler_detect<C, KB, NT, true, 0, 106>;  // 10 + 16-B loads + DPP
    }
  }
  if constexpr ((NT % KB == 0) && (C % (NT / KB) == 0) && ((NT / KB) % 8 == 0) && (C / (NT / KB) <= 16)) {
    const char* ep = getenv("RSL_DD_PERSIST");
    if (pad && ep && atoi(ep) != 0 && !getenv("RSL_DD_DBG")) {
      auto pk = k_doppler_detect_p<C, KB, NT>;
      long nblk = resident_grid(reinterpret_cast<const void*>(pk), lds, ntile) & ~7L;
      if (nblk >= 8) {
        if (dd_reg_ok<C, KB, NT>()) *pk_group = KB;
        hipLaunchKernelGGL(pk, dim3((unsigned)nblk), dim3(NT), lds, st, work, S, tw, rds, thr_f, i_lo, i_hi, mask,
                           row_count, dbmap, pk_pow, ntile);
        return hipGetLastError();
      }
    }
  }
  if (pad && dd_reg_ok<C, KB, NT>()) {
    const char* ed = getenv("RSL_DD_DBG");
    const int v = ed ? atoi(ed) : 0;
    if (v == 0 || v >= 4) *pk_group = KB;
  }
  if constexpr (C == 128 && KB == kPkG) {
    if (wexp) kern = k_doppler_detect<C, KB, NT, true, 0, 74, true>;  // packed work (work_pack_ok checked the rest)
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)ntile), dim3(NT), lds, st, work, S, tw, rds, thr_f, i_lo, i_hi, mask,
                     row_count, dbmap, pk_pow, dd_xcd(), wexp);
  return hipGetLastError();
}

// range bins per Doppler/detect tile: rows_for(C), or RSL_DD_KB (16 / 32 / 64) when it tiles S/2
static int dd_kb(int C, int S) {
  // ~20 KiB tiles: measured fastest at C = 128 (KB 16: 2.42 ms vs KB 32: 3.23 ms per 1000 cfg2 frames; more
  // resident workgroups hide the per-tile load -> FFT -> store phases)
  int kb = 2048 / C < 1 ? 1 : 2048 / C;
  if (kb > rows_for(C) || (S / 2) % kb != 0 || S % kb != 0) kb = rows_for(C);
  if (const char* e = getenv("RSL_DD_KB")) {
    const int v = atoi(e);
    if ((v == 8 || v == 16 || v == 32 || v == 64) && (S / 2) % v == 0 && (size_t)(v + 2) * (lp_row(C) | 1) * 8 <= 60 * 1024)
      kb = v;
  }
  return kb;
}

template <int C>
static hipError_t launch_k2d(hipStream_t st, const float2* work, int F, int A, int S, const float2* tw, float2* rds,
                             double thr_p, int i_lo, int i_hi, unsigned long long* mask, int* row_count, float* dbmap,
                             float* pk_pow, int* pk_group, const signed char* wexp) {
  constexpr int K0 = rows_for(C);
  constexpr int K1 = (2048 / C) < 1 ? 1 : (2048 / C) > K0 ? K0 : (2048 / C);
  const int kb = dd_kb(C, S);
#define K2D(KBV) \
  return launch_k2d_kb<C, KBV>(st, work, F, A, S, tw, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group, \
                               wexp)
  if (kb == K1) K2D(K1);
  if constexpr (C == 128) {  // tuning variants (RSL_DD_KB)
    if (kb == 8) K2D(8);
    if (kb == 64) K2D(64);
  }
  K2D(K0);
#undef K2D
}

template <int S>
static hipError_t launch_k1(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C,
                            const float2* table, const float2* tw, int dc, float2* work, signed char* wexp) {
  constexpr int CB = rows_for(S);
  const char* enp = getenv("RSL_RF_NP");  // 1: one tile per workgroup (interleaves with a concurrent kernel)
  if constexpr (S % 2 == 0 && (CB * (S / 2)) % kThreads == 0) {
    if (!(enp && atoi(enp) != 0)) {
    auto go = [&](auto cbc) -> hipError_t {
      constexpr int CBX = decltype(cbc)::value;
      const long ntile = (long)F * A * ((C + CBX - 1) / CBX);
      const size_t lds = sizeof(float2) * (lp_row(S) + (size_t)CBX * lp_row(S));
      // nt cube loads and nt work stores (both streamed once per batch; tools/cp_ab.py, tools/cpb.sh: 1.48-1.57 vs
      // 1.57-1.64 ms per 1000 cfg2 frames in the pipelined bench)
      auto kern = k_range_fft_p<S, CBX, 0, 3>;
      if constexpr (S == 512) {
        if (const char* e = getenv("RSL_RF_PD")) {  // two tiles in flight per workgroup (A/B)
          if (atoi(e) == 2) kern = k_range_fft_p<S, CBX, 0, 3, 2>;
        }
      }
      if (const char* e = getenv("RSL_RF_DBG"))  // ablation (timing only: results are wrong)
        if (atoi(e) == 1) kern = k_range_fft_p<S, CBX, 1>;
      if constexpr (S == 512) {
        if (const char* e = getenv("RSL_RF_CP")) {  // cache-policy variants (A/B tuning)
          const int v = atoi(e);
          if (v == 0) kern = k_range_fft_p<S, CBX, 0, 0>;
          if (v == 1) kern = k_range_fft_p<S, CBX, 0, 1>;
          if (v == 2) kern = k_range_fft_p<S, CBX, 0, 2>;
          if (v == 4) kern = k_range_fft_p<S, CBX, 0, 4>;
          if (v == 6) kern = k_range_fft_p<S, CBX, 0, 6>;
        }
      }
      long nblk = resident_grid(reinterpret_cast<const void*>(kern), lds, ntile);
      int slot = 0;
      // per-XCD dequeue of tiles (every XCD needs a workgroup; RSL_RF_DYN=0: the static walk): tools/dyn.sh, one call,
      // K1 alone 1.499 vs 1.667 ms per 1000 cfg2 frames, outputs bit-identical; bench 187.8-189.0 vs 186.9-188.7 k
      {
        const char* e = getenv("RSL_RF_DYN");
        if ((!e || atoi(e) != 0) && nblk >= 8 && !getenv("RSL_RF_DBG") && !getenv("RSL_RF_PD") && !getenv("RSL_RF_CP")) {
          kern = k_range_fft_p<S, CBX, 0, 3, 1, true>;
          if constexpr (S == 512 && CBX == 8)
            if (wexp) kern = k_range_fft_p<S, CBX, 0, 3, 1, true, true>;
          static std::atomic<int> next_slot{0};
          slot = next_slot.fetch_add(1) % kRfSlots;
        } else if constexpr (S == 512 && CBX == 8) {
          if (wexp) kern = k_range_fft_p<S, CBX, 0, 3, 1, false, true>;
        }
      }
      hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(kThreads), lds, st, cube, A, Ct, c0, C, ntile, table, tw,
                         dc, work, slot, wexp);
      return hipGetLastError();
    };
    if constexpr (S == 512) {  // RSL_RF_CB: chirp rows per tile (4 / 8 / 16) for tuning
      // 16 rows (78 KiB LDS, 16 float4 in flight per thread) is faster alone (1.53 vs 1.63 ms per 1000 cfg2 frames,
      // tools/rf_ab.py) but leaves no LDS for the previous batch's DoA blocks in the pipelined chain (153 k vs
      // 171 k frames/s), so 8 rows stay the default
      const char* e = getenv("RSL_RF_CB");
      const int v = e ? atoi(e) : CB;
      if (v == 4) return go(std::integral_constant<int, 4>{});
      if (v == 16) return go(std::integral_constant<int, 16>{});
    }
    return go(std::integral_constant<int, CB>{});
    }
  }
  const long nblk = (long)F * A * ((C + CB - 1) / CB);
  const size_t lds = sizeof(float2) * (S + (size_t)CB * lp_row(S));
  hipLaunchKernelGGL(k_range_fft<S>, dim3((unsigned)nblk), dim3(kThreads), lds, st, cube, A, Ct, c0, C, table, tw,
                     dc, work);
  return hipGetLastError();
}

template <int C>
static hipError_t launch_k2(hipStream_t st, const float2* work, int F, int A, int S, const float2* tw,
                            float2* rds) {
  constexpr int KB = rows_for(C);
  const long nblk = (long)F * A * ((S + KB - 1) / KB);
  const size_t lds = sizeof(float2) * (C + (size_t)KB * (lp_row(C) | 1));
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

// Packed `work` between K1 and K2 (see pk_pack): opt-in (RSL_WORK_PACK=1) where both kernels take their packed forms:
// S = 512 (one bin pair per K1 thread), C = 128 (KB = 16 Doppler tiles), no tuning overrides.  Measured neutral
// (tools/pack_ab.sh, one call, 2 rounds: 197.9-198.1 k vs 197.3-198.4 k frames/s; K1 2.83-2.87 vs 2.90-2.95 ms,
// K2 3.61-3.63 vs 3.50 ms per 2000 cfg2 frames): 25 % fewer `work` bytes do not shorten kernels bound by requests
// in flight, and the c64 rows keep fp32 rounding, so c64 stays the default.
bool work_pack_ok(int C, int S) {
  const char* en = getenv("RSL_WORK_PACK");
  if (!en || atoi(en) == 0) return false;
  for (const char* v : {"RSL_RF_NP", "RSL_RF_DBG", "RSL_RF_PD", "RSL_RF_CP", "RSL_RF_CB", "RSL_DD_PERSIST", "RSL_DD_DBG",
                        "RSL_DD_CP", "RSL_DD_KB", "RSL_DD_PAD"})
    if (getenv(v)) return false;
  return S == 512 && C == 128 && doppler_detect_supported(C, S) && dd_kb(C, S) == kPkG;
}

bool doppler_detect_supported(int C, int S) {
  if (!fft_supported(C) || (C & (C - 1)) != 0 || C < 8 || C > 1024 || (S & 1)) return false;  // LDS <= 64 KiB
  const int KB = dd_kb(C, S);
  return S % KB == 0 && (S / 2) % KB == 0;
}

hipError_t launch_doppler_detect(hipStream_t st, const float2* work, int F, int A, int C, int S, const float2* tw_C,
                                 float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask,
                                 int* row_count, float* dbmap, float* pk_pow, bool* supported, int* pk_group,
                                 const signed char* wexp) {
  *pk_group = 1;
  *supported = doppler_detect_supported(C, S);
  if (!*supported || F <= 0 || A <= 0) return hipSuccess;
  switch (C) {
#define CASE(n) \
  case n:       \
    return launch_k2d<n>(st, work, F, A, S, tw_C, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group, \
                          wexp);
    CASE(8) CASE(16) CASE(32) CASE(64) CASE(128) CASE(256) CASE(512) CASE(1024)
#undef CASE
    default:
      *supported = false;
      return hipSuccess;
  }
}

hipError_t launch_range_fft(hipStream_t st, const float2* cube, int F, int A, int Ct, int chirp0, int C, int S,
                            const float2* table, const float2* tw_S, int dc, float2* work, bool* supported,
                            signed char* wexp) {
  *supported = true;
  if (F <= 0 || A <= 0 || C <= 0) return hipSuccess;
  switch (S) {
#define CASE(n) \
  case n:       \
    return launch_k1<n>(st, cube, F, A, Ct, chirp0, C, table, tw_S, dc, work, wexp);
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


// ---------------------------------------------------------------------------------------------
// K12 ring: range FFT and Doppler FFT + detection in ONE persistent launch, with the `work` intermediate kept in the
// XCD's L2 instead of making an HBM round trip (8.4 MB per cfg2 frame written by K1 and read back by K2).
//
// A slab (frame, antenna) is the transpose unit: its C x S range spectra (512 KiB at cfg2) are produced by NP = C / CB
// range tiles (K1's body: CB chirps x S) and consumed by NC = S / KB Doppler tiles (K2's body: KB range bins x C
// chirps + 2 halo bins).  Every XCD owns the slabs s = x + 8 k of the launch (x = the XCD's HW_REG_XCC_ID) and a ring
// of R slab buffers at the front of `work`, and its workgroups dequeue that XCD's items in the order
//     P(0) .. P(L-1) | C(0) P(L) | C(1) P(L+1) | ...      (P(k): the NP range tiles of slab k, C(k): its NC tiles)
// so a slab's range spectra are produced L slabs ahead of their Doppler tiles.  Hand-offs stay inside one XCD's L2:
//   - a range tile stores its rows (plain stores: the lines stay in L2), waits vmcnt(0) in every wave, and after a
//     workgroup barrier one lane adds 1 to prod[x][k % R];
//   - a Doppler tile polls prod[x][k % R] >= NP (k / R + 1) with an L2-served (sc1) load, then loads its rows with
//     L1-bypassing (nt) loads, so no L1 line of an earlier use of the ring slot can be read; after the rows are in LDS
//     one lane adds 1 to cons[x][k % R];
//   - the range tiles of slab k >= R wait for cons[x][k % R] >= NC (k / R) (the slot's previous slab fully read).
// Counters only grow within a launch (uses of a slot are ordered by those waits) and the last workgroup to leave
// resets the launch slot.  Every dependency points to an item dequeued earlier, and an item is dequeued only by a
// running workgroup, so the smallest unfinished item can always run: no residency assumption, no deadlock.  The
// queues are chosen by the XCD each workgroup actually runs on (HW_REG_XCC_ID), so producer and consumer of a slab
// always share an L2 whatever the placement; the host enables the path only on an 8-XCC device.
//
// Measured (tools/ring_ab.py, 2000 cfg2 frames, outputs bit-identical to K1 + K2): 7.3 ms per launch (4-chirp range
// tiles, R 8, L 5) vs 6.6-6.9 ms for K1 + K2 in the same processes, so the path is opt-in (RSL_RING=1).  The hand-off
// itself is cheap (waits ~5 % of workgroup time at 3 workgroups per CU, RSL_RING_PROF) and keeping the slabs in L2
// barely matters (own-address slabs, no reuse: 7.9 ms); the launch is bound by its single register / LDS budget.
// With 8-chirp range tiles the range role needs 42 KiB of LDS (and, before the thread index was laundered, 157
// VGPRs), capping the Doppler role at 3 workgroups per CU where K2 alone runs 7 (7.4-8.3 ms); 4-chirp tiles fit 6 per
// CU but then the ring slots are waited on (range-tile waits 11-14 % of workgroup time).
// ---------------------------------------------------------------------------------------------
constexpr int kRingSlots = 8;  // launches in flight (round-robin, as K1's queues)
constexpr int kRingMaxR = 16;  // ring slabs per XCD (counter slots)
struct RingSync {
  unsigned head[8][32];                 // per-XCD dequeue heads (each counter on its own 128-B line)
  unsigned prod[8][kRingMaxR][32];      // range tiles finished, per (XCD, ring slot)
  unsigned cons[8][kRingMaxR][32];      // Doppler tiles that have read their rows, per (XCD, ring slot)
  unsigned exit_[32];                   // workgroups that have left
};
__device__ RingSync g_ring[kRingSlots];
__device__ unsigned g_ring_faults;  // launches that left a queue undrained, or whose waits timed out
__device__ unsigned long long g_ring_prof[8];  // RSL_RING_PROF: clock sums over workgroups (A/B diagnostics)

unsigned ring_faults() {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ring_faults), sizeof(v)) != hipSuccess) return ~0u;
  return v;
}

RSL_DEV unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}

RSL_DEV unsigned ld_relaxed(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane waits for *p >= target (bounded: ~2 s of polling, then the launch goes on and the outputs are wrong rather
// than the GPU hung); the caller's barrier broadcasts the wait.
RSL_DEV void ring_wait(const unsigned* p, unsigned target) {
  unsigned it = 0;
  for (; ld_relaxed(p) < target && it < (1u << 21); ++it) __builtin_amdgcn_s_sleep(8);
  if (it == (1u << 21)) atomicAdd(&g_ring_faults, 1u);
}

template <int S, int C, int CB, int KB, int WPE = 0, int CT = 1>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1))) void k_rds_ring(const float2* __restrict__ cube, int A, int Ct, int c0,
                                                      long nfa, const float2* __restrict__ table,
                                                      const float2* __restrict__ twS, const float2* __restrict__ twC,
                                                      int dc, float2* __restrict__ work, int R, int L, int ring, int Q,
                                                      float2* __restrict__ rds, float thr_f, int i_lo, int i_hi,
                                                      unsigned long long* __restrict__ mask, int* __restrict__ row_count,
                                                      float* __restrict__ pk_pow, int slot, int prof) {
  constexpr int NT = kThreads;
  constexpr int NP = C / CB, NC = S / KB / CT;  // items per slab
  unsigned long long t_all = prof ? clock64() : 0, t_p = 0, t_c = 0, w_p = 0, w_c = 0, n_p = 0, n_c = 0;
  constexpr int LDS_S = lp_row(S);         // range rows (padded)
  constexpr int H = S / 2;
  constexpr int PF = CB * H / NT;          // float4 per thread per range tile
  constexpr int NR = KB + 2;
  constexpr int LDC = lp_row(C) | 1;       // Doppler rows (padded, odd)
  constexpr int CS = NT / KB, PI = C / CS, PH = (2 * C + NT - 1) / NT;
  static_assert(C % CB == 0 && S % KB == 0 && (S / 2) % KB == 0 && (S / KB) % CT == 0, "tiles must divide the slab");
  static_assert((CB * H) % NT == 0 && NT % KB == 0 && C % CS == 0 && CS % 8 == 0, "tile maps");
  static_assert(dd_reg_ok<C, KB, NT>(), "register Doppler body");
  extern __shared__ float2 sm[];
  float2* tS = sm;                 // S twiddles at padded positions
  float2* tC = sm + LDS_S;         // C twiddles
  float2* buf = tC + C;            // range tile [CB][LDS_S] or Doppler tile [NR][LDC] + exchange words
  __shared__ unsigned s_next;
  const int tid = threadIdx.x;
  for (int k = tid; k < S; k += NT) tS[lp(k)] = twS[k];
  for (int k = tid; k < C; k += NT) tC[k] = twC[k];
  const unsigned x = xcc_id();
  RingSync& sy = g_ring[slot];
  const unsigned nk = nfa > (long)x ? (unsigned)((nfa - (long)x + 7) / 8) : 0u;  // slabs of this XCD
  const unsigned total = nk * (NP + NC);
  const unsigned Lp = (unsigned)L < nk ? (unsigned)L : nk;
  const unsigned nfull = nk > (unsigned)L ? nk - (unsigned)L : 0u;
  const float4* tab4 = reinterpret_cast<const float4*>(table);
  const size_t slab = (size_t)C * S;
  unsigned* head = &sy.head[x][0];
  // the queue hands out runs of Q consecutive items (one atomic per run); the next run is claimed one ahead
  unsigned claim = 0;
  if (tid == 0) s_next = atomicAdd(head, 1u);
  __syncthreads();
  unsigned run = __builtin_amdgcn_readfirstlane(s_next);
  while (run * (unsigned)Q < total) {
    if (tid == 0) claim = atomicAdd(head, 1u);
    const unsigned iend = min(total, (run + 1) * (unsigned)Q);
    for (unsigned it = run * (unsigned)Q; it < iend; ++it) {
    // a laundered thread index: per-thread addresses are recomputed per item instead of held across the loop
    int tidv = tid;
    asm volatile("" : "+v"(tidv));
    // decode: role, slab k of this XCD, tile j
    bool prod_role;
    unsigned k, j;
    if (it < Lp * NP) {
      prod_role = true; k = it / NP; j = it % NP;
    } else {
      const unsigned m = it - Lp * NP;
      if (m < nfull * (NP + NC)) {
        const unsigned b = m / (NP + NC), q = m % (NP + NC);
        if (q < NC) { prod_role = false; k = b; j = q; }
        else { prod_role = true; k = b + (unsigned)L; j = q - NC; }
      } else {
        const unsigned m2 = m - nfull * (NP + NC);
        prod_role = false; k = nfull + m2 / NC; j = m2 % NC;
      }
    }
    const unsigned r = k % (unsigned)R, use = k / (unsigned)R;
    const long fa = (long)x + 8L * k;
    float2* wslab = work + (ring ? (size_t)(x * (unsigned)R + r) : (size_t)fa) * slab;
    const unsigned long long t0 = prof ? clock64() : 0;
    if (prod_role) {
      // ---- range tile: chirps j CB .. j CB + CB - 1 of slab fa (K1's body) ----
      const float4* src4 = reinterpret_cast<const float4*>(cube + ((size_t)fa * Ct + c0 + j * CB) * S);
      float4 nx[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) nx[q] = ld16<true>(src4 + tidv + q * NT);
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int idx = tidv + q * NT;
        const int rr = idx / H, s2 = idx - rr * H;
        const float4 tb = tab4[s2];
        buf[rr * LDS_S + lp(2 * s2)] = cmul(make_float2(nx[q].x, nx[q].y), make_float2(tb.x, tb.y));
        buf[rr * LDS_S + lp(2 * s2 + 1)] = cmul(make_float2(nx[q].z, nx[q].w), make_float2(tb.z, tb.w));
      }
      __syncthreads();
      fft_rows<S, CB, NT, LDS_S, true>(buf, tS, tidv);
      if (dc) {
        if (tidv < CB) buf[tidv * LDS_S] = make_float2(0.f, 0.f);
      }
      const unsigned long long tw0 = prof ? clock64() : 0;
      if (tidv == 0 && use > 0) ring_wait(&sy.cons[x][r][0], (unsigned)NC * use);  // the slot's previous slab is read
      __syncthreads();
      if (prof) w_p += clock64() - tw0;
      float4* dst4 = reinterpret_cast<float4*>(wslab + (size_t)j * CB * S);
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int idx = tidv + q * NT;
        const int rr = idx / H, s2 = idx - rr * H;
        const float2 lo = buf[rr * LDS_S + lp(2 * s2)], hi = buf[rr * LDS_S + lp(2 * s2 + 1)];
        dst4[idx] = make_float4(lo.x, lo.y, hi.x, hi.y);  // plain stores: the lines stay in this XCD's L2
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tidv == 0) atomicAdd(&sy.prod[x][r][0], 1u);
      if (prof) { t_p += clock64() - t0; ++n_p; }
    } else {
      // ---- Doppler item: CT tiles of KB range bins (+ halo) of slab fa (K2's body); the loads of all CT tiles are in
      // flight together (memory-level parallelism at the kernel's low occupancy) ----
      if (tidv == 0) ring_wait(&sy.prod[x][r][0], (unsigned)NP * (use + 1));
      __syncthreads();
      if (prof) w_c += clock64() - t0;
      const int ri = tidv % KB, cs = tidv / KB;
      float2 ld[CT][PI + PH];
#pragma unroll
      for (int u = 0; u < CT; ++u) {
        const int k0 = (int)(j * CT + u) * KB;
        const float2* p = wslab + (unsigned)(cs * S + k0 + ri);
#pragma unroll
        for (int q = 0; q < PI; ++q) ld[u][q] = ld8<true>(p + (unsigned)(q * CS * S));
        int kl = k0 - 1, kh = k0 + KB;
        if (kl < 0) kl += S;
        if (kh >= S) kh -= S;
#pragma unroll
        for (int h = 0; h < PH; ++h) {
          const int e = tidv + h * NT;
          if ((2 * C) % NT == 0 || e < 2 * C) {
            const int side = e / C, c = e - side * C;
            ld[u][PI + h] = ld8<true>(wslab + (unsigned)(c * S + (side ? kh : kl)));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < CT; ++u) {
        const int k0 = (int)(j * CT + u) * KB;
        float2* row = buf + (ri + 1) * LDC + lp(cs);
#pragma unroll
        for (int q = 0; q < PI; ++q) row[lp(q * CS)] = ld[u][q];
#pragma unroll
        for (int h = 0; h < PH; ++h) {
          const int e = tidv + h * NT;
          if ((2 * C) % NT == 0 || e < 2 * C) {
            const int side = e / C, c = e - side * C;
            buf[(side ? NR - 1 : 0) * LDC + lp(c)] = ld[u][PI + h];
          }
        }
        if (u == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every tile's rows are in registers
        __syncthreads();
        if (u == 0 && tidv == 0) atomicAdd(&sy.cons[x][r][0], 1u);  // the slot may be refilled
        fft_rows<C, NR, NT, LDC, false, true>(buf, tC, tidv);
        dd_tile_compute_reg<C, KB, NT, 0, 10>(buf, reinterpret_cast<float*>(buf + NR * LDC), S, k0, (unsigned)fa, rds,
                                              thr_f, i_lo, i_hi, mask, row_count, nullptr, pk_pow, tidv);
        __syncthreads();
      }
      if (prof) { t_c += clock64() - t0; ++n_c; }
    }
    }
    if (tid == 0) s_next = claim;
    __syncthreads();
    run = __builtin_amdgcn_readfirstlane(s_next);
  }
  if (prof && tid == 0) {
    const unsigned long long v[7] = {clock64() - t_all, t_p, t_c, w_p, w_c, n_p, n_c};
    for (int q = 0; q < 7; ++q) atomicAdd(&g_ring_prof[q], v[q]);
  }
  // every claim of this workgroup has returned; the last workgroup to leave checks that every XCD's queue was
  // drained (an XCD without workgroups would leave its slabs unprocessed: counted in g_ring_faults) and resets the
  // launch slot
  if (tid == 0 && atomicAdd(&sy.exit_[0], 1u) == gridDim.x - 1u) {
    for (int q = 0; q < 8; ++q) {
      const unsigned nq = nfa > (long)q ? (unsigned)((nfa - (long)q + 7) / 8) : 0u;
      if (ld_relaxed(&sy.head[q][0]) * (unsigned)Q < nq * (NP + NC)) atomicAdd(&g_ring_faults, 1u);  // NC: items
    }
    for (int q = 0; q < 8; ++q) {
      atomicExch(&sy.head[q][0], 0u);
      for (int rr = 0; rr < kRingMaxR; ++rr) {
        atomicExch(&sy.prod[q][rr][0], 0u);
        atomicExch(&sy.cons[q][rr][0], 0u);
      }
    }
    atomicExch(&sy.exit_[0], 0u);
    if (prof) {
      unsigned long long v[7];
      for (int q = 0; q < 7; ++q) v[q] = atomicExch(&g_ring_prof[q], 0ull);
      printf("RINGPROF grid %u all %llu p %llu c %llu wait_p %llu wait_c %llu n_p %llu n_c %llu\n", gridDim.x, v[0],
             v[1], v[2], v[3], v[4], v[5], v[6]);
    }
  }
}

// Device check for the ring path: 8 XCCs (the queues are indexed by HW_REG_XCC_ID & 7).
static bool ring_device_ok() {
  static int ok = -1;
  if (ok < 0) {
    int dev = 0, nx = 0;
    (void)hipGetDevice(&dev);
    ok = (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, dev) == hipSuccess && nx == 8) ? 1 : 0;
  }
  return ok == 1;
}

bool rds_ring_supported(int C, int S) { return C == 128 && S == 512; }

// RSL_RING_R / RSL_RING_L: ring slabs per XCD and lead (slabs); RSL_RING_BPC: workgroups per CU; RSL_RING_Q: items per
// dequeue; RSL_RING_PROF: clock breakdown printed by the last workgroup (A/B diagnostics)
template <int CB, int WPE, int CT>
static hipError_t launch_rds_ring_t(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0,
                                    const float2* table, const float2* twS, const float2* twC, int dc, float2* work,
                                    float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask,
                                    int* row_count, float* pk_pow, int* pk_group) {
  constexpr int SS = 512, CC = 128, KB = 16;
  auto kern = k_rds_ring<SS, CC, CB, KB, WPE, CT>;
  constexpr int LDS_S = lp_row(SS), NR = KB + 2, LDC = lp_row(CC) | 1;
  constexpr int BUF = (CB * LDS_S > NR * LDC + KB * (CC / 64) * 2) ? CB * LDS_S : NR * LDC + KB * (CC / 64) * 2;
  const size_t lds = sizeof(float2) * (size_t)(LDS_S + CC + BUF);
  const long nfa = (long)F * A;
  int R = 8, L = 5;  // fastest measured (tools/ring_ab.py)
  if (const char* e = getenv("RSL_RING_R")) R = atoi(e);
  if (const char* e = getenv("RSL_RING_L")) L = atoi(e);
  // a Doppler tile may only wait for items dequeued before it (L >= 1), and a range tile only for the slot's previous
  // slab (L < R): then the smallest unfinished item can always run
  if (R < 2) R = 2;
  if (R > kRingMaxR) R = kRingMaxR;
  if (L < 1) L = 1;
  // a batch smaller than the ring (or RSL_RING_OWN=1, A/B) uses its own slab addresses; the slot waits stay (they
  // keep the per-slot counters exact)
  int ring = nfa >= 8L * R ? 1 : 0;
  if (const char* e = getenv("RSL_RING_OWN"))
    if (atoi(e) != 0) ring = 0;
  if (L > R - 1) L = R - 1;
  const int prof = getenv("RSL_RING_PROF") ? 1 : 0;
  int Q = 1;  // items per dequeue
  if (const char* e = getenv("RSL_RING_Q")) Q = atoi(e) < 1 ? 1 : (atoi(e) > 16 ? 16 : atoi(e));
  int nb = 0, dev = 0, ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kThreads, lds) != hipSuccess || nb < 1) nb = 1;
  if (nb > 8) nb = 8;
  if (const char* e = getenv("RSL_RING_BPC"))
    if (atoi(e) > 0 && atoi(e) < nb) nb = atoi(e);
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // the whole chip (every XCD needs workgroups for its queue; extra ones leave at once)
  const long grid = (long)nb * ncu;
  static std::atomic<int> next_slot{0};
  const int slot = next_slot.fetch_add(1) % kRingSlots;
  *pk_group = KB;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kThreads), lds, st, cube, A, Ct, c0, nfa, table, twS, twC, dc,
                     work, R, L, ring, Q, rds, threshold_as_float(thr_p), i_lo, i_hi, mask, row_count, pk_pow, slot, prof);
  return hipGetLastError();
}

hipError_t launch_rds_ring(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C, int S,
                           const float2* table, const float2* twS, const float2* twC, int dc, float2* work,
                           float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask, int* row_count,
                           float* pk_pow, int* pk_group, bool* supported) {
  *supported = rds_ring_supported(C, S) && ring_device_ok();
  if (!*supported || F <= 0) return hipSuccess;
  const char* e = getenv("RSL_RING_CT");  // Doppler tiles per item (1 or 2; A/B)
  const char* cb = getenv("RSL_RING_CB");  // chirps per range tile (4: 26 KiB of LDS, 6 workgroups per CU; or 8)
  if (e && atoi(e) == 2)
    return launch_rds_ring_t<8, 0, 2>(st, cube, F, A, Ct, c0, table, twS, twC, dc, work, rds, thr_p, i_lo, i_hi,
                                      mask, row_count, pk_pow, pk_group);
  if (cb && atoi(cb) == 8)
    return launch_rds_ring_t<8, 0, 1>(st, cube, F, A, Ct, c0, table, twS, twC, dc, work, rds, thr_p, i_lo, i_hi,
                                      mask, row_count, pk_pow, pk_group);
  return launch_rds_ring_t<4, 0, 1>(st, cube, F, A, Ct, c0, table, twS, twC, dc, work, rds, thr_p, i_lo, i_hi, mask,
                                    row_count, pk_pow, pk_group);
}

}  // namespace rsl
