// rsl_rds_fused.hip — single-pass range-Doppler spectrum + Doppler-direction detection for gfx950 (K12), and the
// range-direction detection finish (K3').
//
// Replaces SignalPreprocessor.generate_range_doppler_spectrum + extract_range_doppler_peaks (reference
// src/radar_signal/dechirp.py:143-166, 168-213, 215-278) for the shapes it is instantiated for (S = 512, C = 128).
//
// Why: the two-kernel path (K1 range FFT -> `work` -> K2 Doppler FFT) moves the 4 MiB per-frame intermediate out to
// HBM and back.  A whole (frame, antenna) slab (C x S c64 = 512 KiB at cfg2) does not fit one CU's LDS, so the slab is
// split by RANGE CLASS instead: block q of a slab owns the range bins k = 4 k' + q.  Decimation in frequency gives
//     X_c[4 k' + q] = FFT_{S/4}( y_c )[k'],   y_c[n] = sum_{j<4} h_q[n + j S/4] x_c[n + j S/4],
//     h_q[s] = conj(ref)[s] w[s] W_S^{s q}
// so each block reads the whole slab (the 4 class blocks of a slab run back to back on one XCD: 3 of the 4 reads
// hit L2), but does a quarter of the range FFT work and holds a quarter of the spectrum: a 128 x 128 c64 LDS tile
// (range FFT in place, chirp rows).  Thread (k', u) of S = 512 then reads chirps c = 4 i + u of range bin k' into
// registers; the Doppler FFT is an in-register FFT over i (C/4 points), a twiddle W_C^{u e}, and a radix-4 across the
// 4 lanes of the quad (two DPP radix-2 stages).  The 3x3 local-max test is separable: the Doppler-direction 3-max `hm` (the
// quad's 4 contiguous Doppler blocks) is taken here, and the candidate bit (threshold, range gate, p >= both Doppler
// neighbours) is stored with hm; the range neighbours live in the other 3 class blocks, so k_detect_finish compares
// hm of the rows above and below.  HBM per frame: cube 4 MiB in, RDS 4 MiB + hm 2 MiB out, hm 2 MiB back in (the
// two-kernel path: 16 MiB).  Detection decisions are those of k_doppler_detect (max is exact and separable).
#include <cstdlib>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

RSL_DEV float dpp_xor1(float v) {  // quad_perm [1,0,3,2]
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
RSL_DEV float dpp_xor2(float v) {  // quad_perm [2,3,0,1]
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
}

// In-register forward FFT of N = N1 N2 points (natural order in and out), i = N2 i1 + i2, e = e1 + N1 e2.
// tw[t k] = W_N^k (an LDS table of a longer transform, stride t): broadcast reads.
template <int N1, int N2>
RSL_DEV void fft_reg(float2 (&v)[N1 * N2], const float2* tw, int t) {
  float2 a[N2][N1];
#pragma unroll
  for (int i2 = 0; i2 < N2; ++i2) {
#pragma unroll
    for (int i1 = 0; i1 < N1; ++i1) a[i2][i1] = v[N2 * i1 + i2];
    Dft<N1>::run(a[i2]);
  }
#pragma unroll
  for (int i2 = 1; i2 < N2; ++i2)
#pragma unroll
    for (int e1 = 1; e1 < N1; ++e1) a[i2][e1] = cmul(a[i2][e1], tw[t * i2 * e1]);
#pragma unroll
  for (int e1 = 0; e1 < N1; ++e1) {
    float2 b[N2];
#pragma unroll
    for (int i2 = 0; i2 < N2; ++i2) b[i2] = a[i2][e1];
    Dft<N2>::run(b);
#pragma unroll
    for (int e2 = 0; e2 < N2; ++e2) v[e1 + N1 * e2] = b[e2];
  }
}

template <int CU>
struct RegFft;
template <>
struct RegFft<32> {
  RSL_DEV static void run(float2 (&v)[32], const float2* tw, int t) { fft_reg<8, 4>(v, tw, t); }
};
template <>
struct RegFft<16> {
  RSL_DEV static void run(float2 (&v)[16], const float2*, int) { Dft<16>::run(v); }
};

// Lane (within the quad) that holds shifted Doppler block sb: block m = u1 + 2 u0 is stored at sb = (m + 2) & 3.
RSL_DEV int quad_lane_of_block(int sb) {
  const int m = (sb + 2) & 3;
  return (m >> 1) | ((m & 1) << 1);
}

// K12.  Work item = (slab = frame * A + antenna, range class q); S threads.  Writes the shifted RDS [slab][S][C], the
// Doppler-direction 3-max hm [slab][S][C] (f32, shifted order, 'reflect' edges) and the candidate bits
// cand [slab][S][C/32] (u32; bit e of word sb = shifted Doppler 32 sb + e).
// Persistent: the grid holds resident workgroups only (a multiple of 32).  Workgroup b serves XCD x = b % 8
// (round-robin placement), class q = (b / 8) % 4 and slab lane lg = b / 32, i.e. slabs x + 8 (lg + NLG t): the 4 class
// blocks of a slab are resident together on one XCD and advance in step, so their 4 reads of the slab share one L2.
// The next chirp group's 16-B loads (the next slab's first group during the Doppler phase) are in flight while the
// current group is combined and transformed.
template <int S, int C, int G>
__global__ __launch_bounds__(S) void k_rds_fused(const float2* __restrict__ cube, int Ct, int c0, long nslab,
                                                 const float2* __restrict__ table, const float2* __restrict__ twS,
                                                 const float2* __restrict__ twC, int dc, float2* __restrict__ rds,
                                                 float* __restrict__ hm_out, unsigned* __restrict__ cand,
                                                 float thr_f, int i_lo, int i_hi) {
  constexpr int NT = S;
  constexpr int NK = S / 4;        // range bins of a class
  constexpr int CU = C / 4;        // Doppler inputs per thread
  constexpr int NG = C / G;        // chirp groups
  constexpr int LDR = lp_row(NK);  // padded LDS row of the NK-point range FFT
  constexpr int PAIRS = NK / 2;    // float4 per (chirp, j)
  constexpr int CPR = NT / PAIRS;  // chirps per load round
  constexpr int LR = G / CPR;      // load rounds per group
  constexpr int RP = 32;           // range bins per store pass
  constexpr int NPASS = NK / RP;
  constexpr int BS = CU + 2, RS = 4 * BS;  // RDS staging: padded Doppler blocks (float2)
  constexpr int HB = CU + 4, HS = 4 * HB;  // hm staging (float)
  static_assert(G % CPR == 0 && G % 4 == 0 && C % G == 0, "chirp groups");
  static_assert(CU == 32 || CU == 16, "C / 4 Doppler points per thread");
  static_assert((size_t)RP * (RS * 8 + HS * 4) <= (size_t)C * LDR * 8, "the store staging fits in the tile");
  extern __shared__ float2 sm[];
  float2* twk = sm;         // W_NK^k at padded positions lp(k)
  float2* twc = twk + LDR;  // W_C^k
  float2* buf = twc + C;    // the class tile: C chirp rows x LDR (range FFT in place); then the store staging
  float* hst = reinterpret_cast<float*>(buf + RP * RS);
  const int tid = threadIdx.x;
  const int x = (int)(blockIdx.x & 7), q = (int)((blockIdx.x >> 3) & 3), lg = (int)(blockIdx.x >> 5);
  const long sstep = 8L * (long)(gridDim.x >> 5);
  for (int k = tid; k < NK; k += NT) twk[lp(k)] = twS[4 * k];
  for (int k = tid; k < C; k += NT) twc[k] = twC[k];
  const int p = tid % PAIRS, g0 = tid / PAIRS;
  float2 hq[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int s = 2 * p + e + NK * j;
      hq[j][e] = cmul(table[s], twS[(s * q) & (S - 1)]);
    }
  const int kq = tid >> 2, u = tid & 3, lane = tid & 63;
  float4 ld[LR][4];
  auto load = [&](long slab, int grp) {
    const float4* src = reinterpret_cast<const float4*>(cube + ((size_t)slab * Ct + c0) * S);
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const float4* row = src + (size_t)(grp * G + g0 + CPR * r) * (S / 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) ld[r][j] = row[p + PAIRS * j];
    }
  };
  long slab = x + 8L * lg;
  if (slab < nslab) load(slab, 0);
  for (; slab < nslab; slab += sstep) {
    __syncthreads();  // the tile is free: the previous slab's store staging has been read out
#pragma unroll 1
    for (int grp = 0; grp < NG; ++grp) {
      float2* rows = buf + grp * G * LDR;
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        float2 y0 = make_float2(0.f, 0.f), y1 = y0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 xv = ld[r][j];
          y0 = cadd(y0, cmul(make_float2(xv.x, xv.y), hq[j][0]));
          y1 = cadd(y1, cmul(make_float2(xv.z, xv.w), hq[j][1]));
        }
        float2* dst = rows + (g0 + CPR * r) * LDR;
        dst[lp(2 * p)] = y0;
        dst[lp(2 * p + 1)] = y1;
      }
      if (grp + 1 < NG) {
        load(slab, grp + 1);  // in flight during this group's FFT
      } else if (slab + sstep < nslab) {
        load(slab + sstep, 0);  // in flight during the Doppler phase below
      }
      __syncthreads();
      fft_rows<NK, G, NT, LDR, true>(rows, twk, tid);  // ends with a barrier
    }
    float2 dv[CU];  // chirps c = 4 i + u of range bin k' (one tile column)
#pragma unroll
    for (int i = 0; i < CU; ++i) dv[i] = buf[(4 * i + u) * LDR + lp(kq)];
    if (dc && q == 0 && kq == 0) {  // DC removal: range bin 0 of every chirp is zero (dechirp.py:110-120)
#pragma unroll
      for (int i = 0; i < CU; ++i) dv[i] = make_float2(0.f, 0.f);
    }
    // Doppler FFT: F_u[e] over i, twiddle W_C^{u e}, radix-4 over the quad's lanes u = u0 + 2 u1
    RegFft<CU>::run(dv, twc, C / CU);
#pragma unroll
    for (int e = 1; e < CU; ++e) dv[e] = cmul(dv[e], twc[u * e]);
    {
      const int u0 = u & 1, u1 = u >> 1;
      const float s1 = u1 ? -1.f : 1.f, s0 = u0 ? -1.f : 1.f;
      const bool rot = (u0 & u1) != 0;
#pragma unroll
      for (int e = 0; e < CU; ++e) {
        const float bx = fmaf(s1, dv[e].x, dpp_xor2(dv[e].x));
        const float by = fmaf(s1, dv[e].y, dpp_xor2(dv[e].y));
        const float rx = rot ? by : bx, ry = rot ? -bx : by;  // x (-i) on lane (1, 1)
        dv[e].x = fmaf(s0, rx, dpp_xor1(rx));
        dv[e].y = fmaf(s0, ry, dpp_xor1(ry));
      }
    }
    // lane (u0, u1) holds Doppler bins CU (u1 + 2 u0) + e; fftshift: shifted block sb = (m + 2) & 3
    const int m = (u >> 1) + 2 * (u & 1);
    const int sb = (m + 2) & 3;
    const int k = 4 * kq + q;
    const int i = k + S / 2 < S ? k + S / 2 : k - S / 2;  // shifted range row
    float hm[CU];  // |X|^2, then (in place) the Doppler 3-max
#pragma unroll
    for (int e = 0; e < CU; ++e) hm[e] = cabs2(dv[e]);
    const int qb = lane & ~3;
    const float le = __shfl(hm[CU - 1], qb | quad_lane_of_block((sb + 3) & 3));
    const float re = __shfl(hm[0], qb | quad_lane_of_block((sb + 1) & 3));
    const bool gate = i >= i_lo && i <= i_hi;
    unsigned bits = 0;
    float prev = 0.f;
#pragma unroll
    for (int e = 0; e < CU; ++e) {
      const float pc = hm[e];
      const float l = e > 0 ? prev : (sb > 0 ? le : pc);  // 'reflect' at the shifted edges: no neighbour
      const float r = e + 1 < CU ? hm[e + 1] : (sb < 3 ? re : pc);
      const float mx = fmaxf(fmaxf(l, pc), r);
      bits |= (unsigned)(gate && pc > thr_f && pc >= mx) << e;
      prev = pc;
      hm[e] = mx;
    }
    cand[((size_t)slab * S + i) * (C / 32) + sb] = bits;
    // stores through LDS: RP range bins per pass, whole 1 KiB RDS rows per wave instruction
#pragma unroll 1
    for (int P = 0; P < NPASS; ++P) {
      __syncthreads();
      if (kq / RP == P) {
        const int rr = kq - RP * P;
        float2* d = buf + rr * RS + sb * BS;
#pragma unroll
        for (int e = 0; e < CU; e += 2)
          *reinterpret_cast<float4*>(d + e) = make_float4(dv[e].x, dv[e].y, dv[e + 1].x, dv[e + 1].y);
        float* hd = hst + rr * HS + sb * HB;
#pragma unroll
        for (int e = 0; e < CU; e += 4)
          *reinterpret_cast<float4*>(hd + e) = make_float4(hm[e], hm[e + 1], hm[e + 2], hm[e + 3]);
      }
      __syncthreads();
#pragma unroll
      for (int z = 0; z < RP * C / 2 / NT; ++z) {
        const int idx = tid + NT * z;
        const int rr = idx / (C / 2), j = 2 * (idx % (C / 2));
        const int kk = 4 * (RP * P + rr) + q;
        const int ii = kk + S / 2 < S ? kk + S / 2 : kk - S / 2;
        const float4 v = *reinterpret_cast<const float4*>(buf + rr * RS + (j / CU) * BS + (j % CU));
        *reinterpret_cast<float4*>(rds + ((size_t)slab * S + ii) * C + j) = v;
      }
#pragma unroll
      for (int z = 0; z < RP * C / 4 / NT; ++z) {
        const int idx = tid + NT * z;
        const int rr = idx / (C / 4), j = 4 * (idx % (C / 4));
        const int kk = 4 * (RP * P + rr) + q;
        const int ii = kk + S / 2 < S ? kk + S / 2 : kk - S / 2;
        const float4 v = *reinterpret_cast<const float4*>(hst + rr * HS + (j / CU) * HB + (j % CU));
        *reinterpret_cast<float4*>(hm_out + ((size_t)slab * S + ii) * C + j) = v;
      }
    }
  }
}

// K3'.  Range-direction finish of the 3x3 test on K12's Doppler 3-max: a candidate (p > thr, in gate, p >= its
// Doppler neighbours, so p = hm) is a peak when hm >= hm of the shifted rows above and below ('reflect': no
// neighbour past the shifted edges).  Tile = KB shifted rows of one slab; wave (ch, rh) owns Doppler columns
// 64 ch + lane and rows 8 rh .. 8 rh + 7.  Outputs as k_doppler_detect's register body: mask words, row counts and
// tile-compact peak powers (peak_pow_group = KB).
template <int C>
__global__ __launch_bounds__(256) void k_detect_finish(const float* __restrict__ hm,
                                                       const unsigned long long* __restrict__ cand, int S,
                                                       unsigned long long* __restrict__ mask,
                                                       int* __restrict__ row_count, float* __restrict__ pk_pow) {
  constexpr int NCH = C / 64;
  constexpr int KB = 8 * (4 / NCH);
  __shared__ unsigned long long wb[KB * NCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = wave % NCH, rh = wave / NCH;
  const unsigned nkb = (unsigned)(S / KB);
  const unsigned tile = (unsigned)xcd_tile(blockIdx.x, gridDim.x);
  const unsigned fa = tile / nkb;
  const int i0 = (int)(tile % nkb) * KB;
  const int rb = 8 * rh;
  const int j = 64 * ch + lane;
  const float* col = hm + ((size_t)fa * S) * C + j;
  float h[10];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const int i = i0 + rb + r - 1;
    h[r] = (i >= 0 && i < S) ? col[(size_t)i * C] : 0.f;
  }
  unsigned long long cw[8];
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) cw[rr] = cand[((size_t)fa * S + i0 + rb + rr) * NCH + ch];
  bool pkv[8];
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) {
    const int i = i0 + rb + rr;
    const bool c = (cw[rr] >> lane) & 1ull;
    const bool pk = c && (i == 0 || h[rr + 1] >= h[rr]) && (i + 1 == S || h[rr + 1] >= h[rr + 2]);
    pkv[rr] = pk;
    const unsigned long long bm = __ballot(pk);
    if (lane == 0) wb[(rb + rr) * NCH + ch] = bm;
  }
  __syncthreads();
  int pre = 0;
  for (int x = 0; x < rb * NCH; ++x) pre += __popcll(wb[x]);
  float* tile_pk = pk_pow ? pk_pow + ((size_t)fa * S + i0) * C : nullptr;
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) {
    const size_t row = (size_t)fa * S + i0 + rb + rr;
    int off = pre, cnt = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int pc = __popcll(wb[(rb + rr) * NCH + c]);
      off += c < ch ? pc : 0;
      cnt += pc;
    }
    pre += cnt;
    const unsigned long long bm = wb[(rb + rr) * NCH + ch];
    if (lane == 0) {
      mask[row * NCH + ch] = bm;
      if (ch == 0) row_count[row] = cnt;
    }
    if (tile_pk && pkv[rr]) tile_pk[off + __popcll(bm & ((1ull << lane) - 1ull))] = h[rr + 1];
  }
}

// Opt-in (RSL_FUSED=1): measured slower than K1 + K2 on MI355X.  Per 1000 cfg2 frames K12 takes 4.0-4.5 ms + K3' 0.7 ms
// against 1.6 + 1.9 ms, although its HBM traffic is lower as designed (PMC: 5.1 MiB read + 6.1 MiB written per frame,
// the 4 class blocks' slab reads hit L2).  The 128 KiB class state (registers or LDS tile) leaves one 512-thread
// workgroup per CU, so the barrier-separated load / FFT / transpose phases run with 8 waves and little overlap.
bool rds_fused_supported(int C, int S) {
  const char* e = getenv("RSL_FUSED");
  return e && atoi(e) != 0 && S == 512 && C == 128;
}

hipError_t launch_rds_fused(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C, int S,
                            const float2* table, const float2* tw_S, const float2* tw_C, int dc, float2* rds,
                            void* work, double thr_p, int i_lo, int i_hi) {
  constexpr int SS = 512, CC = 128, G = 32;
  if (S != SS || C != CC) return hipErrorInvalidValue;
  const long nslab = (long)F * A;
  float* hmv = reinterpret_cast<float*>(work);
  unsigned* cand = reinterpret_cast<unsigned*>(hmv + (size_t)nslab * SS * CC);
  const size_t lds = sizeof(float2) * (lp_row(SS / 4) + CC + (size_t)CC * lp_row(SS / 4));
  auto kern = k_rds_fused<SS, CC, G>;
  // resident workgroups only, a multiple of 32 (8 XCDs x 4 range classes), no more than the slabs need
  int nb = 0, dev = 0, ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, SS, lds) != hipSuccess || nb < 1) nb = 1;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  long nblk = ((long)nb * ncu) & ~31L;
  const long need = ((nslab + 7) / 8) * 32;
  if (nblk > need) nblk = need;
  if (nblk < 32) nblk = 32;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(SS), lds, st, cube, Ct, c0, nslab, table,
                     tw_S, tw_C, dc, rds, hmv, cand, threshold_as_float(thr_p), i_lo, i_hi);
  return hipGetLastError();
}

hipError_t launch_detect_finish(hipStream_t st, const void* work, int F, int A, int C, int S,
                                unsigned long long* mask, int* row_count, float* pk_pow, int* pk_group) {
  constexpr int CC = 128, KB = 16;
  if (C != CC || S % KB != 0) return hipErrorInvalidValue;
  const long nslab = (long)F * A;
  const float* hmv = reinterpret_cast<const float*>(work);
  const unsigned long long* cand = reinterpret_cast<const unsigned long long*>(hmv + (size_t)nslab * S * CC);
  *pk_group = KB;
  const long ntile = nslab * (S / KB);
  hipLaunchKernelGGL(k_detect_finish<CC>, dim3((unsigned)ntile), dim3(256), 0, st, hmv, cand, S, mask, row_count,
                     pk_pow);
  return hipGetLastError();
}

}  // namespace rsl
