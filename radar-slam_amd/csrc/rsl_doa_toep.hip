// rsl_doa_toep.hip — K5 fast path: steering-scan argmax (MUSIC / beamforming) through the Toeplitz form of
// |a^H s|^2 on f16 MFMA with a hi/lo split that keeps fp32-class accuracy.  gfx950 / CDNA4.
//
// Replaces (reference src/angle_estimation/angle_estimation.py):
//   music_spectrum :109-154 + estimate_angle_music :156-176 (argmax only),
//   estimate_angle_beamforming :227-251; robust_angle_estimation.py estimate_angle_robust :236-245.
//
// For a uniform linear array a_m(theta) = a_0 e^{j m phi(theta)} (angle_estimation.py:92-107, positions
// arange(M) d), so with r_k = sum_n s_{n+k} conj(s_n) (the signature's autocorrelation, k = 0..M-1)
//     P(theta) = |a^H s|^2 = r_0 + 2 sum_{k>=1} (Re r_k cos k phi + Im r_k sin k phi).
// That is ONE real dot product of length 2M-1 per (grid point, cell): half the rows of the [Re; Im] GEMM,
// and no |.|^2 in the epilogue.  The contraction T[G x 2M-1] . R[2M-1 x cells] runs on
// v_mfma_f32_32x32x16_f16 (16x the f32 MFMA rate).  fp16 alone would leave 2^-11 relative error, so both
// operands are split, x = x_hi + x_lo (each fp16), and three products are accumulated in fp32:
//     P ~= T_lo r_hi + T_hi r_lo + T_hi r_hi      (dropped T_lo r_lo ~ 2^-22 |T r|)
// f16 x f16 products are exact in fp32, so the result is within ~1e-6 |T||r| of the fp32 scan.  The r
// entries are scaled by 2^8 (exact) so the lo halves stay out of the fp16 subnormal range.
//
// MUSIC rule (angle_estimation.py:149-152): the spectrum is 1/(M - P) if M - P > 1e-12 else 0.  That can
// only change the argmax when max P is within rounding of M (s equal to a steering vector).  Such cells
// are re-scanned exactly in fp64 from the reference's fp64 steering table (rare, lane-divergent path).
#include <climits>
#include <cstdlib>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr float kToepScale = 256.f;

// The Toeplitz B column of one cell: e = [r0, Re r1, Im r1, ..., Re r_{M-1}, Im r_{M-1}, 0...] of the unit-norm
// signature, scaled by 2^8 (exact), fp32.
// Autocorrelation of the raw signature, r_k = sum_n s_{n+k} conj(s_n) (k = 0..MA-1; r_0 = |s|^2 real): shared by the
// Toeplitz column, ESPRIT and (through s) the spatial phase.
template <int MA>
RSL_DEV void acf(const float2 (&s)[MA], float (&ar)[MA], float (&ai)[MA]) {
  float pw = 0.f;
#pragma unroll
  for (int m = 0; m < MA; ++m) pw = fmaf(s[m].x, s[m].x, fmaf(s[m].y, s[m].y, pw));
  ar[0] = pw;
  ai[0] = 0.f;
#pragma unroll
  for (int k = 1; k < MA; ++k) {
    float re = 0.f, im = 0.f;
#pragma unroll
    for (int n = 0; n + k < MA; ++n) {  // s_{n+k} conj(s_n)
      re = fmaf(s[n + k].x, s[n].x, fmaf(s[n + k].y, s[n].y, re));
      im = fmaf(s[n + k].y, s[n].x, fmaf(-s[n + k].x, s[n].y, im));
    }
    ar[k] = re;
    ai[k] = im;
  }
}

// The Toeplitz B column of one cell: e = [r0, Re r1, Im r1, ..., Re r_{M-1}, Im r_{M-1}, 0...] of the unit-norm
// signature, scaled by 2^8 (exact), fp32.  inv = 2^8 / |s|^2 (0 for a zero signature).
template <int MA, int KB>
RSL_DEV void toep_entries(const float (&ar)[MA], const float (&ai)[MA], float inv, float (&e)[16 * KB]) {
  // angle_estimation.py:86-88 (unit-norm s).  v_rcp_f32 (1 ulp): a common scale of all of a cell's grid values
  // cannot move its argmax, and the MUSIC degeneracy test has a 1e-4 margin
  e[0] = ar[0] > 0.f ? kToepScale : 0.f;
#pragma unroll
  for (int k = 1; k < MA; ++k) {
    e[2 * k - 1] = ar[k] * inv;
    e[2 * k] = ai[k] * inv;
  }
#pragma unroll
  for (int x = 2 * MA - 1; x < 16 * KB; ++x) e[x] = 0.f;
}

// ESPRIT (angle_estimation.py:178-225) for a full array (A = M) from the autocorrelation: the 2x2 Gram matrix of
// X = [s[:-1], s[1:]] is [[r0 - |s_{M-1}|^2, r1], [conj r1, r0 - |s_0|^2]], and with u_m = v0 s_m + v1 s_{m+1} the
// sums phi = sum_{m<M-2} conj(u_m) u_{m+1} and d = sum_{m<M-2} |u_m|^2 expand into r0, r1, r2 and edge products:
//   phi = |v0|^2 (r1 - conj(s_{M-2}) s_{M-1}) + conj(v0) v1 r2 + conj(v1) v0 (r0 - |s_0|^2 - |s_{M-1}|^2)
//         + |v1|^2 (r1 - conj(s_0) s_1)
//   d   = |v0|^2 (r0 - |s_{M-2}|^2 - |s_{M-1}|^2) + |v1|^2 (r0 - |s_0|^2 - |s_{M-1}|^2)
//         + 2 Re(conj(v0) v1 (r1 - conj(s_{M-2}) s_{M-1}))
// (O(1) work instead of esprit_phi's O(M) passes; all terms share the scale sc, which cancels in angle(phi)).
template <int MA>
RSL_DEV void esprit_acf(const float2 (&s)[MA], const float (&ar)[MA], const float (&ai)[MA], float sc, float& nr,
                        float& ni, float& dd) {
  static_assert(MA >= 3, "ESPRIT from the autocorrelation needs M >= 3");
  const float2 s0 = s[0], s1 = s[1], sl = s[MA - 1], sl2 = s[MA - 2];
  const float r0 = ar[0] * sc, r1r = ar[1] * sc, r1i = ai[1] * sc, r2r = ar[2] * sc, r2i = ai[2] * sc;
  const float e0 = cabs2(s0) * sc, el = cabs2(sl) * sc, el2 = cabs2(sl2) * sc;
  // conj(s_{M-2}) s_{M-1}, conj(s_0) s_1
  const float tr = (sl2.x * sl.x + sl2.y * sl.y) * sc, ti = (sl2.x * sl.y - sl2.y * sl.x) * sc;
  const float hr = (s0.x * s1.x + s0.y * s1.y) * sc, hi = (s0.x * s1.y - s0.y * s1.x) * sc;
  const float a = r0 - el, cc = r0 - e0, br = r1r, bi = r1i;
  const float hd = 0.5f * (a - cc);
  // v_sqrt_f32 directly (1 ulp; the ESPRIT tolerance is 1e-3 rad): the IEEE sqrtf expansion is ~15 VALU per cell
  const float l1 = 0.5f * (a + cc) + __builtin_amdgcn_sqrtf(hd * hd + br * br + bi * bi);
  float v0r, v0i, v1r, v1i;
  if (a >= cc) {  // v = [l1 - c, conj(b)]
    v0r = l1 - cc; v0i = 0.f; v1r = br; v1i = -bi;
  } else {        // v = [b, l1 - a]
    v0r = br; v0i = bi; v1r = l1 - a; v1i = 0.f;
  }
  const float n0 = v0r * v0r + v0i * v0i, n1 = v1r * v1r + v1i * v1i;
  const float cr = v0r * v1r + v0i * v1i, ci = v0r * v1i - v0i * v1r;  // conj(v0) v1
  const float sar = r1r - tr, sai = r1i - ti;                          // r1 - conj(s_{M-2}) s_{M-1}
  const float scc = r0 - e0 - el;
  const float sdr = r1r - hr, sdi = r1i - hi;                          // r1 - conj(s_0) s_1
  nr = n0 * sar + (cr * r2r - ci * r2i) + cr * scc + n1 * sdr;         // conj(v1) v0 = conj(conj(v0) v1)
  ni = n0 * sai + (cr * r2i + ci * r2r) - ci * scc + n1 * sdi;
  dd = n0 * (r0 - el2 - el) + n1 * scc + 2.f * (cr * sar - ci * sai);
}

// fp16 hi/lo split of 8 consecutive entries, packed two halves per dword (4 + 4 dwords).
RSL_DEV void split8(const float* v, uint4& hi, uint4& lo) {
  unsigned h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const _Float16 h0 = (_Float16)v[2 * j], h1 = (_Float16)v[2 * j + 1];
    const _Float16 l0 = (_Float16)(v[2 * j] - (float)h0), l1 = (_Float16)(v[2 * j + 1] - (float)h1);
    h[j] = (unsigned)__builtin_bit_cast(unsigned short, h0) | ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
    l[j] = (unsigned)__builtin_bit_cast(unsigned short, l0) | ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

// The same hi/lo split straight from the unscaled autocorrelation, two entries per packed dword pair: entry x of the
// Toeplitz column is v_x * g_x (v = r0-flag, Re r1, Im r1, ...; g = 1 for the first, inv for the others, 0 past
// 2 MA - 1), and v_fma_mix{lo,hi}_f16 write the halves in place (hi = f16(v g), lo = f16(v g - hi), both halves of
// a dword by one instruction each, no shift / or packing).  Values equal to toep_entries + split8.
template <int MA, int KB>
RSL_DEV void toep_split(const float (&ar)[MA], const float (&ai)[MA], float inv, uint4 (&hi)[2 * KB],
                        uint4 (&lo)[2 * KB]) {
  auto val = [&](int x) { return x == 0 ? (ar[0] > 0.f ? kToepScale : 0.f) : x < 2 * MA - 1 ? ((x & 1) ? ar[(x + 1) >> 1] : ai[x >> 1]) : 0.f; };
  auto scl = [&](int x) { return x == 0 ? 1.f : x < 2 * MA - 1 ? inv : 0.f; };
#pragma unroll
  for (int q = 0; q < 2 * KB; ++q) {
    unsigned h[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = 8 * q + 2 * j;
      asm("v_fma_mixlo_f16 %0, %2, %3, 0\n\t"
          "v_fma_mixhi_f16 %0, %4, %5, 0\n\t"
          "v_fma_mixlo_f16 %1, %2, %3, -%0 op_sel_hi:[0,0,1]\n\t"
          "v_fma_mixhi_f16 %1, %4, %5, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
          : "=&v"(h[j]), "=&v"(l[j])
          : "v"(val(x)), "v"(scl(x)), "v"(val(x + 1)), "v"(scl(x + 1)));
    }
    hi[q] = make_uint4(h[0], h[1], h[2], h[3]);
    lo[q] = make_uint4(l[0], l[1], l[2], l[3]);
  }
}

// atan2 for the fused extras: |t| = min / max reduced to [0, 1], atan(t) = t + t z P(z) (z = t^2, P of degree 7,
// least-squares fit, max error 9e-8 rad in fp32 evaluation) and the octant / quadrant fixes.  About half the VALU of
// the library atan2f (no frexp-scaled division, no inf / nan cases: the inputs are finite); within 1e-7 rad of it,
// four orders below the 1e-3 rad DoA tolerance.  atan2(+-0, x < 0) = +-pi, atan2(y, +-0) as atan2f except y = x = 0
// (0 here).
RSL_DEV float atan2_fast(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  const float t = mx > 0.f ? mn * __builtin_amdgcn_rcpf(mx) : 0.f;
  const float z = t * t;
  float p = 0.00262275873683393f;
  p = fmaf(p, z, -0.015134590677917004f);
  p = fmaf(p, z, 0.041125182062387466f);
  p = fmaf(p, z, -0.07366984337568283f);
  p = fmaf(p, z, 0.10574059933423996f);
  p = fmaf(p, z, -0.14186006784439087f);
  p = fmaf(p, z, 0.19990399479866028f);
  p = fmaf(p, z, -0.3333298861980438f);
  float a = fmaf(t * z, p, t);
  a = ay > ax ? 1.57079632679489662f - a : a;
  a = x < 0.f ? 3.14159265358979324f - a : a;
  return copysignf(a, y);
}

// v_permlane32_swap on each dword: the upper 32 lanes of a are exchanged with the lower 32 lanes of b.
RSL_DEV void swap32_u4(uint4& a, uint4& b) {
  unsigned av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto r = __builtin_amdgcn_permlane32_swap(av[j], bv[j], false, false);
    av[j] = r[0];
    bv[j] = r[1];
  }
  a = make_uint4(av[0], av[1], av[2], av[3]);
  b = make_uint4(bv[0], bv[1], bv[2], bv[3]);
}

// The cell's (frame, range * C + doppler) pair; past the end: cell 0 (its results are never stored).  Cell indices are
// 32-bit (the launchers check counts < 2^31 - 64): 64-bit per-lane indices pushed the scan loop past 128 VGPRs, and the
// spills' reloads (s_waitcnt vmcnt(0)) waited out the signature prefetch of the next pass.
RSL_DEV int2 load_cell(const int* __restrict__ cfr, const int* __restrict__ crc, int c, bool ok) {
  const unsigned cc = ok ? (unsigned)c : 0u;
  return make_int2(cfr[cc], crc[cc]);
}

// Signature of a cell from its (frame, rc) pair; antennas past A (A < MA, wave-uniform) are clamped to A-1 and zeroed.
template <int MA>
RSL_DEV void load_sig_at(const float2* __restrict__ rds, int2 fr, int A, size_t plane, size_t fstride, float2 (&s)[MA]) {
  const float2* base = rds + (size_t)fr.x * fstride + fr.y;
  if (A >= MA) {
#pragma unroll
    for (int m = 0; m < MA; ++m) s[m] = base[(size_t)m * plane];
  } else {
#pragma unroll
    for (int m = 0; m < MA; ++m) {
      const float2 z = base[(size_t)(m < A ? m : A - 1) * plane];
      s[m] = m < A ? z : make_float2(0.f, 0.f);
    }
  }
}

template <int MA>
RSL_DEV void load_sig_c(const float2* __restrict__ rds, const int* __restrict__ cfr, const int* __restrict__ crc,
                        int c, bool ok, int A, size_t plane, size_t fstride, float2 (&s)[MA]) {
  load_sig_at<MA>(rds, load_cell(cfr, crc, c, ok), A, plane, fstride, s);
}

// Max of one 32x32 tile's 16 values held by this lane, as signed-integer max3 on the float bits (v_max3_i32):
// order-preserving for non-negative floats, and a tile max is one of its inputs exactly.  P = |a^H s|^2 >= 0; a
// rounding-negative value can only lose to a positive one, and a tile whose values are all <= 0 never holds the
// spectrum maximum of a non-zero signature.  (fmaxf on MFMA outputs costs NaN-canonicalising v_max_f32 ops.)
RSL_DEV float tile_max(const floatx16& a, float lo = __int_as_float(INT_MIN)) {
  int v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = __float_as_int(a[i]);
  auto mx3 = [](int x, int y, int z) { return max(max(x, y), z); };
  const int m0 = mx3(v[0], v[1], v[2]), m1 = mx3(v[3], v[4], v[5]), m2 = mx3(v[6], v[7], v[8]);
  const int m3 = mx3(v[9], v[10], v[11]), m4 = mx3(v[12], v[13], v[14]);
  return __int_as_float(mx3(mx3(m0, m1, m2), mx3(m3, m4, v[15]), __float_as_int(lo)));
}

// Record-tile copy for the lanes that set a new record: 8 v_pk_mov_b32 (64-bit pairs) under the branch's exec mask
// instead of 16 v_cndmask_b32 on every tile.  Volatile asm also keeps the compiler from speculating the branch into
// per-value selects.
template <int NCOPY = 8>  // NCOPY < 8: ablation (timing only)
RSL_DEV void copy_tile(double (&dst)[8], const floatx16& src) {
  typedef double doublex8 __attribute__((ext_vector_type(8)));
  const doublex8 s = __builtin_bit_cast(doublex8, src);
#pragma unroll
  for (int k = 0; k < NCOPY; ++k) asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[0,1]" : "=v"(dst[k]) : "v"(s[k]));
}

// Ambiguity bound of the f16 hi/lo scan, relative to a cell's maximum: a cell whose best grid value is not at least
// this far above every other grid value (its top-2 gap) is re-scanned exactly in fp64 (k_doa_fixup), so that the grid
// index is the fp64 argmax of the cell's own fp32 signature (no scan-caused flips).  The scan's
// error is far smaller: the dropped T_lo r_lo term is <= 2^-22 sum |T_k| |r_k| and the fp32 autocorrelation and MFMA
// accumulation add a few fp32 ulps of that sum (measured against the fp64 scan of the same signatures:
// tests/test_gpu_spectrum.py::test_toeplitz_spectrum_matches_f32_scan, max 3.8e-6 of M on den = M - P; the flips the
// round-3 build made had gaps <= 8.6e-8).  What decides a flip is the f16 deficit of the fp64 argmax against the f16
// maximum: <= 2.4e-7 relative in a CPU emulation of the split (M 4 / 8 / 16, two grids, 140 k cells).  1e-6 marks
// 0.17 % of cfg2 cells (2e-6: 0.31 %), and over 142 M cfg2 cells it gave the same indices as 2e-6
// (tools/doa_bound_study.py, gpurun_out/r4m_bound.log).  The bound is relative and the worst case of the dropped term
// is absolute (about 2^-22 (2M - 1) r0): for weak, flat cells whose best value is only a few r0 that worst case would
// exceed it, so exactness here is statistical (the emulation, the 142 M-cell study and the weak two-lobe cells of
// tests/test_gpu_doa_exact.py), not a proof.  An absolute term max(kAmbRel best, 2^-21 (2M - 1) r0) would make it
// one, at the price of marking most noise cells (best ~ r0 to 2 r0: a bound of ~7e-6 of best at M = 8).
constexpr float kAmbRel = 1e-6f;

// Ties of the exact scan: keys within this relative distance count as equal and the lower grid index wins, as
// np.argmax does on an exact tie.  Such keys are equal in exact arithmetic up to fp64 rounding (the reference's own
// fp64 noise decides between them, e.g. the identical steering vectors of -90 and +90 degrees at d = lambda / 2),
// and the parity tests treat gaps <= 1e-13 as ties (tests/parity.py OWN_TIE_RGAP).  fp64 rounding of the 2M-term
// sums is ~1e-15 relative: 1e-13 still covers the +-90 degree alias pair (identical to 5.6e-15) without treating
// real gaps of 1e-13..1e-12 as ties.
constexpr double kTieRel = 1e-13;

// Exact fp64 scan of ONE cell over grid points [g0, g1) by the whole wave (wave-uniform cell c): the key is P if
// M - P > 1e-12 (MUSIC, angle_estimation.py:149-152) else -1, P for beamforming; first index of the maximum key, as
// np.argmax (ties within kTieRel).  P = |a^H s|^2 / |s|^2 from the reference's fp64 steering table [G][A].  Lane =
// (grid point p = lane >> 3 of 8 per step, antenna m = lane & 7, and m + 8 for A > 8): each steering load is one
// 16-B complex of a row, so a step's 64 lanes read 8 consecutive rows as contiguous 128-B runs (lanes splitting the
// grid points with a whole row each read 16 lines per instruction: 16x the L2 requests); the sum over the antennas
// is three xor shuffles inside the 8-lane group.  Returns (index, P at it) on every lane.
// One wave = 64 cells per pass: lane (n, h) = (l & 31, l >> 5) loads, normalises and owns cell 64 ch + 32 h + n.
// The two 32-cell halves are the two column tiles of v_mfma_f32_32x32x16_f16 (B: lane holds K rows 8h..8h+7 of
// column n), so each lane computes the Toeplitz column of its own cell once and swaps the other K half with
// lane l ^ 32 (no redundant loads or autocorrelations), and the fused ESPRIT / phase work of a pass is spread
// over all 64 lanes.  Per grid tile (32 grid points) the two column tiles are two independent accumulator chains.
template <int MA, int KB, bool MUSIC, bool GMAX, bool EXTRAS, int DBG = 0, int NTC = 0, bool SKEW = false,
          bool SPEC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MA <= 8 ? 4 : (SPEC ? 1 : 3)))) void k_doa_toep(const float2* __restrict__ rds, int A, int S, int C,
                                                  const int* __restrict__ cfr, const int* __restrict__ crc,
                                                  const long long* __restrict__ ncell_dev, long long ncell_host,
                                                  const uint4* __restrict__ ttab, int ntiles, int G,
                                                  const double* __restrict__ steer64, int* __restrict__ out_idx,
                                                  float* __restrict__ out_gmax, float esprit_scale, int esprit_clamp,
                                                  double* __restrict__ out_esprit, double* __restrict__ out_phase,
                                                  float* __restrict__ out_spec) {
  extern __shared__ uint4 tt[];  // the whole Toeplitz operand table (<= 64 KiB)
  __shared__ float sstg[SPEC ? 4 * 512 : 1];  // SPEC: per-wave store stage
  {
    const long long nc = list_count(ncell_dev, ncell_host);
    if ((long long)blockIdx.x * 256 >= nc) return;  // a block past the cells (capacity-sized grids): no table load
  }
  const int nvec = ntiles * KB * 2 * 64;
  for (int x = threadIdx.x; x < nvec; x += 256) tt[x] = ttab[x];
  __syncthreads();
  const int ncell = (int)list_count(ncell_dev, ncell_host);
  // the wave index is wave-uniform: in an SGPR, the pass index ch and everything derived from it are scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const size_t plane = (size_t)S * C, fstride = (size_t)A * plane;
  const int nch = (ncell + 63) >> 6;
  const int stride = (int)gridDim.x * 4;
  int ch = (int)blockIdx.x * 4 + wave;
  const float mthr = ((float)A - 1e-4f) * kToepScale;
  // Two-level prefetch: the signature of the next pass is loaded during this pass from cell indices that were loaded
  // one pass earlier (index loads followed at once by the dependent signature loads stalled every pass for a full
  // memory round trip).
  // The next pass's signatures land in s itself, issued once this pass's prologue (the autocorrelation and the fused
  // extras) has consumed s: no second signature array, and no register copies between passes (a separate prefetch
  // array cost 16 64-bit moves per pass); the tile loop and the epilogue still cover the loads' latency.
  float2 s[MA];
  int2 nidx = make_int2(0, 0);
  if (ch < nch) {
    const int c = ch * 64 + lane;
    if constexpr (DBG == 3) {
#pragma unroll
      for (int m = 0; m < MA; ++m) s[m] = make_float2(0.1f * (lane + m), 0.2f * m - lane * 0.01f);
    } else {
      load_sig_c<MA>(rds, cfr, crc, c, c < ncell, A, plane, fstride, s);
      const int c2 = (ch + stride) * 64 + lane;
      if (ch + stride < nch) nidx = load_cell(cfr, crc, c2, c2 < ncell);
    }
  }
  // The argmax (and gmax) of a pass is stored at the start of the NEXT pass, after the wait for that pass's prefetched
  // signatures: stored at the end of its own pass it sat in front of that wait (stores count in vmcnt, and a store
  // under a branch makes the compiler wait for vmcnt(0)), so every pass waited out a store round trip.
  // pending store of the previous pass (wave-uniform flag; its cell is (ch - stride) 64 + lane, recomputed rather
  // than kept in a register across the tile loop)
  int pc = -1;  // pending store: cell (-1: none; cell counts < 2^31, checked by the launcher), grid index, gmax
  int pidx = 0;
  float pgv = 0.f;
  for (; ch < nch; ch += stride) {
    if (pc >= 0) {
      out_idx[pc] = pidx;
      if constexpr (GMAX) out_gmax[pc] = pgv;
    }
    const int c = ch * 64 + lane;  // this lane's own cell
    const int nx = ch + stride;
    float ar[MA], ai[MA];
    acf<MA>(s, ar, ai);
    const float inv = ar[0] > 0.f ? kToepScale * __builtin_amdgcn_rcpf(ar[0]) : 0.f;
    if constexpr (EXTRAS) {
      // fused K6 (k_cell_extras) for the own cell, before the scan so its registers are dead during the MFMA
      // loop: ESPRIT (angle_estimation.py:178-225) and the spatial phase angle(s1 conj(s0)) (velocity_solver.py
      // :136); fp32 closed forms from the fp32 signature (both invariant to its scale).
      if (c < ncell) {
        if (out_esprit) {
          float nr, ni, dd;
          if (A == MA) {
            esprit_acf<MA>(s, ar, ai, inv * (1.f / kToepScale), nr, ni, dd);
          } else {  // fewer antennas than the template width: the general per-element form
            float sr[MA], si[MA];
            const float sc = ar[0] > 0.f ? __builtin_amdgcn_rsqf(ar[0]) : 1.f;
#pragma unroll
            for (int m = 0; m < MA; ++m) {
              sr[m] = s[m].x * sc;
              si[m] = s[m].y * sc;
            }
            esprit_phi<MA>(sr, si, A, nr, ni, dd);
          }
          const float ang = dd > 0.f ? atan2_fast(ni, nr) : 0.f;
          // fp32 asin (the input angle is fp32 already; tolerance 1e-3 rad).  For d >= lambda/2 the reference's
          // argument never exceeds 1 (|angle| <= pi): clamp the fp32 rounding of pi * scale there; for d < lambda/2
          // |x| > 1 gives NaN as in the reference.
          float x = ang * esprit_scale;
          if (esprit_clamp) x = fminf(fmaxf(x, -1.f), 1.f);
          out_esprit[c] = (double)(asinf(x) * 57.2957795130823208768f);
        }
        if (out_phase)
          out_phase[c] = (double)atan2_fast(s[1].y * s[0].x - s[1].x * s[0].y, s[1].x * s[0].x + s[1].y * s[0].y);
      }
    }
    // Prefetch into s: the next pass's signatures, the pass after's cell indices.  Unconditional: after the last pass
    // nidx still holds this pass's cells (valid addresses, just read: cache hits), and a load under the loop-exit test
    // would make s a phi of the loaded and the old values, i.e. a second register set and 16 copies per pass.
    // The register barrier ends s's last uses (the compiler sinks the autocorrelation's tail below the extras, which
    // kept s live beside its own prefetch: 16 copies at the loop latch).
#pragma unroll
    for (int k = 0; k < MA; ++k) asm volatile("" : "+v"(ar[k]), "+v"(ai[k])::"memory");
    if constexpr (DBG != 3) {
      if constexpr (DBG == 10) nidx = make_int2(0, nidx.y & 2047);  // ablation: L2-resident signatures
      load_sig_at<MA>(rds, nidx, A, plane, fstride, s);
      const int c3 = (nx + stride) * 64 + lane;
      if (nx + stride < nch) nidx = load_cell(cfr, crc, c3, c3 < ncell);
    }
    // B operands of the two column tiles: own K half from the own cell, the other half from lane ^ 32
    uint4 b0h[KB], b0l[KB], b1h[KB], b1l[KB];
    {
      uint4 eh[2 * KB], el[2 * KB];
      toep_split<MA, KB>(ar, ai, inv, eh, el);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        // E0 / E1 = the own cell's K rows 16 kb .. +7 / +8 .. +15.  Column tile 0 (cells of lanes 0-31) needs
        // [E0 of lanes 0-31 | E1 of lanes 0-31 moved up], column tile 1 [E0 of lanes 32-63 moved down | E1 of lanes
        // 32-63]: exactly what v_permlane32_swap does to the pair (E0, E1), one instruction per dword
        uint4 h0h = eh[2 * kb], h0l = el[2 * kb], h1h = eh[2 * kb + 1], h1l = el[2 * kb + 1];
        swap32_u4(h0h, h1h);
        swap32_u4(h0l, h1l);
        b0h[kb] = h0h;
        b0l[kb] = h0l;
        b1h[kb] = h1h;
        b1l[kb] = h1l;
      }
    }
    // Argmax epilogue per column tile: the tile max (v_max3 tree), a strict '>' record test and a conditional
    // copy of the record tile's 16 values; the in-tile index is resolved once per pass.  Tiles ascend in g and
    // in-tile values ascend in row ((i&3) + 8(i>>2) + 4h): the first index wins as in np.argmax.  Rows past G
    // replicate row G-1 and so never win.
    float best0 = -INFINITY, best1 = -INFINITY;
    float second0 = __int_as_float(INT_MIN), second1 = __int_as_float(INT_MIN);  // below every value as ints
    int bt01 = 0;  // record tile of column tile 0 (bits 0-15) and 1 (bits 16-31): one register
    auto set_bt = [&](int sh, int t) { bt01 = (bt01 & ~(0xFFFF << sh)) | (t << sh); };
    double sv0[8], sv1[8];  // record tiles as 64-bit register pairs (copied with v_pk_mov_b32)
#pragma unroll
    for (int k = 0; k < 8; ++k) sv0[k] = sv1[k] = 0.0;
    auto mma = [&](int t, floatx16& acc0, floatx16& acc1) {
      acc0 = floatx16{};
      acc1 = floatx16{};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const half8 ah = __builtin_bit_cast(half8, tt[(((t * KB + kb) * 2) + 0) * 64 + lane]);
        const half8 al = __builtin_bit_cast(half8, tt[(((t * KB + kb) * 2) + 1) * 64 + lane]);
        const half8 x0h = __builtin_bit_cast(half8, b0h[kb]), x0l = __builtin_bit_cast(half8, b0l[kb]);
        const half8 x1h = __builtin_bit_cast(half8, b1h[kb]), x1l = __builtin_bit_cast(half8, b1l[kb]);
        if constexpr (DBG == 2) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            acc0[i] += (float)ah[i & 7] * (float)x0h[(i + 1) & 7];
            acc1[i] += (float)al[i & 7] * (float)x1l[(i + 3) & 7];
          }
        } else {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, x0h, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, x1h, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, x0l, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, x1l, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, x0h, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, x1h, acc1, 0, 0, 0);
        }
      }
    };
    // record tiles: a real branch (exec-masked 64-bit register copies for the lanes that set a record) instead of
    // a v_cndmask per value
    auto record = [&](int t, const floatx16& acc0, const floatx16& acc1) {
      const float m0 = tile_max(acc0), m1 = tile_max(acc1);
      if (NTC > 0 && t == 0) {  // unrolled: the first tile is always the record (no branch, no initial copies)
        typedef double doublex8 __attribute__((ext_vector_type(8)));
        const doublex8 d0 = __builtin_bit_cast(doublex8, acc0), d1 = __builtin_bit_cast(doublex8, acc1);
        best0 = m0;
        best1 = m1;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          sv0[k] = d0[k];
          sv1[k] = d1[k];
        }
        return;
      }
      // second*: the largest tile maximum of the other tiles (ambiguity test at the end of the pass)
      if (m0 > best0) {
        second0 = best0;
        best0 = m0;
        set_bt(0, t);
        if constexpr (DBG == 7) copy_tile<1>(sv0, acc0);
        else if constexpr (DBG != 1) copy_tile(sv0, acc0);
      } else {
        second0 = fmaxf(second0, m0);
      }
      if (m1 > best1) {
        second1 = best1;
        best1 = m1;
        set_bt(16, t);
        if constexpr (DBG == 7) copy_tile<1>(sv1, acc1);
        else if constexpr (DBG != 1) copy_tile(sv1, acc1);
      } else {
        second1 = fmaxf(second1, m1);
      }
    };
    // SPEC: the whole spectrum of both column tiles, cell-blocked f32 [ceil(n / 32)][G][32] (RSL_DOA_SPEC_BLOCKED):
    // MUSIC 1/(M - P) with the reference's den > 1e-12 rule (angle_estimation.py:149-152; a zero signature has
    // den = M - 1: its eigenvectors are the identity) or the beamforming P (:227-251), P = acc / 2^8.  Lane (n, h)
    // holds rows (i & 3) + 8 (i >> 2) + 4 h of column n, so each store instruction writes two 128-B runs.
    bool zc0 = false, zc1 = false;  // zero signature of column tile 0 / 1's cell n
    if constexpr (SPEC) {
      const bool zown = !(ar[0] > 0.f);
      const bool zoth = __shfl_xor((int)zown, 32) != 0;
      zc0 = h ? zoth : zown;
      zc1 = h ? zown : zoth;
    }
    // Stores go through a per-wave 2 KiB LDS stage, half a tile (16 grid points x 32 cells) at a time, so that each
    // store instruction writes 1 KiB (8 whole 128-B lines, consecutive grid points) instead of two 128-B runs.
    auto spec_tile = [&](int t, const floatx16& acc, int ct) {
      if constexpr (SPEC) {
        if (ch * 64 + 32 * ct >= ncell) return;  // a column tile past the cells (wave-uniform)
        const bool zc = ct ? zc1 : zc0;
        const float Mf = (float)A;
        float* stw = sstg + wave * 512;
        float* dst = out_spec + ((size_t)(2 * ch + ct) * G) * 32;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int ii = 0; ii < 8; ++ii) {
            const int i = 8 * half + ii;
            const int r = (i & 3) + 8 * ((i >> 2) & 1) + 4 * h;  // row within the half (0..15)
            const float P = acc[i] * (1.f / kToepScale);
            float v = P;
            if constexpr (MUSIC) {
              const float d = zc ? Mf - 1.f : Mf - P;
              v = d > 1e-12f ? __builtin_amdgcn_rcpf(d) : 0.f;
            }
            stw[r * 32 + (lane & 31)] = v;
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int r = (lane >> 3) + 8 * q;
            const float4 v = reinterpret_cast<const float4*>(stw)[r * 8 + (lane & 7)];
            const int g = 32 * t + 16 * half + r;
            // non-temporal stores: the 51 MB per frame are written once and never re-read by the chain (1-2 % faster
            // than plain stores in every allocation of gpurun_out/r6f_nt*)
            if (g < G) {
              typedef float f4v_t __attribute__((ext_vector_type(4)));
              __builtin_nontemporal_store(f4v_t{v.x, v.y, v.z, v.w},
                                          reinterpret_cast<f4v_t*>(dst + (size_t)g * 32) + (lane & 7));
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
      }
    };
      if constexpr (SKEW && NTC > 0 && KB == 1 && (DBG == 0 || DBG == 1 || DBG == 3 || DBG >= 8)) {
      // Skewed schedule: the two column tiles' MFMA chains run half a tile apart, so each chain's epilogue (tile max,
      // record test, record copy) issues while the other chain's MFMAs execute instead of waiting for them; the A
      // operands of tile t + 1 are read from LDS during tile t's first epilogue.  Same products and record order.
      const half8 x0h = __builtin_bit_cast(half8, b0h[0]), x0l = __builtin_bit_cast(half8, b0l[0]);
      const half8 x1h = __builtin_bit_cast(half8, b1h[0]), x1l = __builtin_bit_cast(half8, b1l[0]);
      half8 ah, al;
      floatx16 acc0, acc1;
      auto lda = [&](int t) {
        ah = __builtin_bit_cast(half8, tt[(t * 2 + 0) * 64 + lane]);
        al = __builtin_bit_cast(half8, tt[(t * 2 + 1) * 64 + lane]);
      };
      auto chain = [&](floatx16& acc, const half8& xh, const half8& xl) {
        acc = floatx16{};
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh, acc, 0, 0, 0);
      };
      auto rec = [&](int t, const floatx16& acc, float& best, float& second, int sh, double (&sv)[8]) {
        if constexpr (DBG == 8) {  // no epilogue: one max per tile keeps the accumulator live
          best = fmaxf(best, acc[t & 15]);
          return;
        }
        if (t == 0) {
          typedef double doublex8 __attribute__((ext_vector_type(8)));
          const doublex8 d = __builtin_bit_cast(doublex8, acc);
          best = tile_max(acc);
#pragma unroll
          for (int k = 0; k < 8; ++k) sv[k] = d[k];
          return;
        }
        // the running SECOND joins the max tree (same 8 v_max3): m2 = max(second, tile max); since second <= best,
        // m2 > best <=> the tile max > best.  A record moves best to second; otherwise second = m2 (the largest tile
        // maximum of the other tiles: the end-of-pass ambiguity test)
        if constexpr (DBG == 13) {  // timing ablation: no second tracking (the old record test, best folded in)
          const float mb = tile_max(acc, best);
          const bool r = mb > best;
          best = mb;
          if (r) {
            set_bt(sh, t);
            copy_tile(sv, acc);
          }
          return;
        }
        if constexpr (DBG == 15) {  // variant: second = min(best, m2) (one op), best moved under the record branch
          const float m2 = tile_max(acc, second);
          const bool r = m2 > best;
          second = __int_as_float(min(__float_as_int(best), __float_as_int(m2)));
          if (r) {
            best = m2;
            set_bt(sh, t);
            copy_tile(sv, acc);
          }
          return;
        }
        // branch-free top-2: a record (m2 > best) leaves second = the old best, otherwise second = m2 -- both are
        // min(best, m2); best = max(best, m2).  Only the record tile's index and copy sit under the branch.
        // (integer min / max on the bit patterns, as in tile_max: the values are non-negative, and fminf / fmaxf
        // would add an IEEE canonicalising v_max per operand)
        const float m2 = tile_max(acc, second);
        const bool r = m2 > best;
        const int bb = __float_as_int(best), mb = __float_as_int(m2);
        second = __int_as_float(min(bb, mb));
        best = __int_as_float(max(bb, mb));
        if (r) {
          set_bt(sh, t);
          if constexpr (DBG != 1) copy_tile(sv, acc);
        }
      };
      if constexpr (DBG == 9) {  // no tile loop (prologue, loads and the index resolution only)
        best0 = __builtin_bit_cast(float, b0h[0].x ^ b1l[0].y);
        best1 = __builtin_bit_cast(float, b1h[0].z ^ b0l[0].w);
      } else {
      lda(0);
      chain(acc0, x0h, x0l);
      chain(acc1, x1h, x1l);
#pragma unroll
      for (int t = 0; t < NTC; ++t) {
        if (t + 1 < NTC) lda(t + 1);
        __builtin_amdgcn_sched_barrier(0);
        rec(t, acc0, best0, second0, 0, sv0);
        spec_tile(t, acc0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < NTC) chain(acc0, x0h, x0l);
        __builtin_amdgcn_sched_barrier(0);
        rec(t, acc1, best1, second1, 16, sv1);
        spec_tile(t, acc1, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < NTC) chain(acc1, x1h, x1l);
      }
      }
    } else {
      const int ntl = NTC ? NTC : ntiles;  // NTC: compile-time tile count (fully unrolled loop)
#pragma unroll
      for (int t = 0; t < ntl; ++t) {
        floatx16 acc0, acc1;
        mma(t, acc0, acc1);
        record(t, acc0, acc1);
        spec_tile(t, acc0, 0);
        spec_tile(t, acc1, 1);
      }
    }
    // Index resolution and ambiguity, per column tile: theta = best (1 - kAmbRel); i = the first of the record tile's
    // 16 values >= theta, n = how many there are.  n == 1: that value is the lane's maximum and every other value of
    // the lane is below theta, so i is its exact argmax; n >= 2, a tile maximum of another tile >= theta, or a
    // non-positive best (a zero signature): ambiguous, re-scanned in fp64 below.
    // (any / two as lane masks: scalar ALU work, only the compares and the index selects are vector instructions)
    constexpr float kAmb = DBG == 16 ? 5e-7f : kAmbRel;  // DBG 16 (development study): a tighter bound
    int i0 = 15, i1 = 15;
    bool any0 = false, two0 = false, any1 = false, two1 = false;
    {
      const floatx16 r0 = __builtin_bit_cast(floatx16, sv0), r1 = __builtin_bit_cast(floatx16, sv1);
      const float th0 = best0 * (1.f - kAmb), th1 = best1 * (1.f - kAmb);
#pragma unroll
      for (int i = 15; i >= 0; --i) {
        const bool g0 = r0[i] >= th0, g1 = r1[i] >= th1;
        i0 = g0 ? i : i0;
        i1 = g1 ? i : i1;
        if constexpr (DBG != 14) {  // DBG 14 (timing ablation): no count of the values >= theta
          two0 = two0 || (any0 && g0);
          two1 = two1 || (any1 && g1);
        }
        any0 = any0 || g0;
        any1 = any1 || g1;
      }
    }
    bool amb0 = !any0 || two0 || second0 >= best0 * (1.f - kAmb) || !(best0 > 0.f);
    bool amb1 = !any1 || two1 || second1 >= best1 * (1.f - kAmb) || !(best1 > 0.f);
    int g0 = 32 * (bt01 & 0xFFFF) + 4 * h + (i0 & 3) + 8 * (i0 >> 2);
    int g1 = 32 * (bt01 >> 16) + 4 * h + (i1 & 3) + 8 * (i1 >> 2);
    // merge the two K-half lanes of each column (first index wins on ties); ambiguous if the winner is, or if the
    // loser's maximum is within the bound of the winner's (an exact tie included)
    // Window of the exact re-scan: the record tiles of the two K halves when no other tile of either half came within
    // the bound (then every value >= theta lies in those one or two tiles), else the whole grid.
    bool loc0, loc1;
    int pbt;
    {
      const float ob0 = __shfl_xor(best0, 32), ob1 = __shfl_xor(best1, 32);
      const int og0 = __shfl_xor(g0, 32), og1 = __shfl_xor(g1, 32);
      const bool oa0 = __shfl_xor((int)amb0, 32) != 0, oa1 = __shfl_xor((int)amb1, 32) != 0;
      const float os0 = __shfl_xor(second0, 32), os1 = __shfl_xor(second1, 32);
      const int obt = __shfl_xor(bt01, 32) ^ bt01;
      const bool tk0 = (ob0 > best0) | ((ob0 == best0) & (og0 < g0));
      const bool tk1 = (ob1 > best1) | ((ob1 == best1) & (og1 < g1));
      const float lo0 = tk0 ? best0 : ob0, lo1 = tk1 ? best1 : ob1;
      best0 = tk0 ? ob0 : best0;
      g0 = tk0 ? og0 : g0;
      amb0 = (tk0 ? oa0 : amb0) || lo0 >= best0 * (1.f - kAmb);
      best1 = tk1 ? ob1 : best1;
      g1 = tk1 ? og1 : g1;
      amb1 = (tk1 ? oa1 : amb1) || lo1 >= best1 * (1.f - kAmb);
      loc0 = fmaxf(second0, os0) < best0 * (1.f - kAmb);
      loc1 = fmaxf(second1, os1) < best1 * (1.f - kAmb);
      pbt = obt ^ bt01;  // the partner K half's record tiles
    }
    float best = h ? best1 : best0;  // own cell = column tile h
    int bidx = h ? g1 : g0;
    bool amb = h ? amb1 : amb0;
    bool loc = h ? loc1 : loc0;
    if (bidx >= G) bidx = G - 1;
    float gval = best * (1.0f / kToepScale);
    // MUSIC: the reference's den > 1e-12 rule can only matter when the maximum is within rounding of M
    if constexpr (MUSIC) {
      const bool nearm = best >= mthr;  // the key rule may move the argmax anywhere: whole grid
      amb = amb || nearm;
      loc = loc && !nearm;
    }
    // ambiguous: marked -1 - index for k_doa_fixup (the exact fp64 re-scan, launched right after this kernel; kept
    // out of this kernel so that its register allocation stays that of the scan loop)
    if (amb) {
      const int sh = h ? 16 : 0;
      const int ta = (bt01 >> sh) & 0xFFFF, tb = (pbt >> sh) & 0xFFFF;
      bidx = -1 - (loc ? (1 << 28) | (ta << 14) | tb : 0);  // k_doa_fixup's window code
    }
    pc = c < ncell ? c : -1;
    pidx = bidx;
    pgv = gval;
  }
  if (pc >= 0) {
    out_idx[pc] = pidx;
    if constexpr (GMAX) out_gmax[pc] = pgv;
  }
}

// Exact fp64 argmax of the cells a scan marked ambiguous (out_idx = -1 - code; k_doa_toep: its f16 top-2 gap inside
// kAmbRel, or a MUSIC maximum within rounding of M; k_doa_argmax / k_doa_scan: the f32 top-2 gap).  code bit 28 set:
// re-scan the 32-point tiles (code >> 14) & 0x3FFF and code & 0x3FFF (the two K halves' record tiles, when every
// value within the bound lies in them), else the whole grid.
// A wave reads the indices of kFixCells cells (coalesced 16-B loads, 256 cells per step) and queues its marked
// cells in LDS; 8 queued cells at a time, the lanes (cell, antenna) load the cells' signatures into LDS together (one
// memory round trip for 8 cells), then each cell is re-scanned by the whole wave with one grid point per lane
// (lanes 0-31 / 32-63 = the two window tiles, or 64 grid points per pass over the whole grid) from the transposed
// fp64 table steerT[m][g] (a lane's antenna loads are 16 B of consecutive grid points: each load instruction reads
// one or two contiguous runs), and a wave argmax with the tie rule.
constexpr int kFixCells = 2048;
constexpr int kFixQ = 256 + 8;  // queue entries per wave: a step adds at most 256

template <int MA, bool MUSIC>
__global__ __launch_bounds__(256) void k_doa_fixup(const float2* __restrict__ rds, int A, int S, int C,
                                                   const int* __restrict__ cfr, const int* __restrict__ crc,
                                                   const long long* __restrict__ ncell_dev, long long ncell_host, int G,
                                                   const double2* __restrict__ steerT, int* __restrict__ out_idx,
                                                   float* __restrict__ out_gmax) {
  __shared__ int2 q[4][kFixQ];        // (cell - base, marked index)
  __shared__ float2 sig[4][8][MA];    // the signatures of the 8 cells being re-scanned
  __shared__ int qn[4];
  const long long ncell = list_count(ncell_dev, ncell_host);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long base = ((long long)blockIdx.x * 4 + wave) * kFixCells;
  const size_t plane = (size_t)S * C, fstride = (size_t)A * plane;
  const bool al = (reinterpret_cast<size_t>(out_idx) & 15) == 0;
  auto lds_sync = [] {  // this wave's LDS writes visible to its own later LDS reads
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
  };
  if (lane == 0) qn[wave] = 0;
  lds_sync();
  auto rescan = [&](int n) {  // the queued cells, 8 per round
    for (int e0 = 0; e0 < n; e0 += 8) {
      {  // signatures of up to 8 cells: lane (e, m) loads antennas m and m + 8 of cell e0 + e
        const int e = e0 + (lane >> 3), m = lane & 7;
        if (e < n) {
          const long long cell = base + q[wave][e].x;
          const float2* sb = rds + (size_t)cfr[cell] * fstride + crc[cell];
          sig[wave][lane >> 3][m] = m < A ? sb[(size_t)m * plane] : make_float2(0.f, 0.f);
          if constexpr (MA > 8) sig[wave][lane >> 3][m + 8] = m + 8 < A ? sb[(size_t)(m + 8) * plane] : make_float2(0.f, 0.f);
        }
      }
      lds_sync();
      const int ne = min(8, n - e0);
      for (int e = 0; e < ne; ++e) {  // wave-uniform
        const int2 en = q[wave][e0 + e];
        const long long cell = base + en.x;
        const int code = -1 - en.y;
        double sr[MA], si[MA], pw = 0.0;
#pragma unroll
        for (int m = 0; m < MA; ++m) {
          const float2 z = sig[wave][e][m];
          sr[m] = z.x;
          si[m] = z.y;
          pw += sr[m] * sr[m] + si[m] * si[m];
        }
        const double sc2 = pw > 0.0 ? 1.0 / pw : 1.0;  // unit-norm signature (angle_estimation.py:86-88)
        double best = -2.0, bp = 0.0;  // below every key (keys are P >= 0 or -1)
        int bi = G;
        auto point = [&](int g) {  // ascending g per lane: a later g must beat the tie tolerance
          double zr = 0.0, zi = 0.0;
#pragma unroll
          for (int m = 0; m < MA; ++m)
            if (m < A) {
              const double2 a = steerT[(size_t)m * G + g];
              zr += a.x * sr[m] + a.y * si[m];  // conj(a) s
              zi += a.x * si[m] - a.y * sr[m];
            }
          const double pv = (zr * zr + zi * zi) * sc2;
          const double key = MUSIC ? (((double)A - pv > 1e-12) ? pv : -1.0) : pv;
          if (key > best + kTieRel * fabs(best)) {
            best = key;
            bi = g;
            bp = pv;
          }
        };
        if ((code >> 28) & 1) {
          int ta = (code >> 14) & 0x3FFF, tb = code & 0x3FFF;
          if (tb < ta) {
            const int t = ta;
            ta = tb;
            tb = t;
          }
          const int t = lane < 32 ? ta : tb;
          const int g = 32 * t + (lane & 31);
          if (g < G && (lane < 32 || tb != ta)) point(g);
        } else {
#pragma unroll 1
          for (int g = lane; g < G; g += 64) point(g);
        }
        // wave argmax: larger key beyond the tie tolerance, else lower index
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const double ok = __shfl_xor(best, off), op = __shfl_xor(bp, off);
          const int oi = __shfl_xor(bi, off);
          const double tol = kTieRel * fmax(fabs(ok), fabs(best));
          if (ok > best + tol || (fabs(ok - best) <= tol && oi < bi)) {
            best = ok;
            bi = oi;
            bp = op;
          }
        }
        if (lane == 0) {
          out_idx[cell] = bi;
          if (out_gmax) out_gmax[cell] = (float)bp;
        }
      }
      lds_sync();  // the next round overwrites sig
    }
  };
  constexpr int NST = kFixCells / 256;
  int4 vv[NST];
#pragma unroll
  for (int j = 0; j < NST; ++j) {  // every index load in flight at once
    const long long c0 = base + j * 256 + 4 * lane;
    if (al && c0 + 3 < ncell) {
      vv[j] = *reinterpret_cast<const int4*>(out_idx + c0);
    } else {
      vv[j].x = c0 < ncell ? out_idx[c0] : 0;
      vv[j].y = c0 + 1 < ncell ? out_idx[c0 + 1] : 0;
      vv[j].z = c0 + 2 < ncell ? out_idx[c0 + 2] : 0;
      vv[j].w = c0 + 3 < ncell ? out_idx[c0 + 3] : 0;
    }
  }
  // Phase 1: queue the marked cells of all NST steps (the index registers die before any re-scan: interleaving the
  // re-scans with the steps kept them live through it, 122 VGPRs and 4 waves per SIMD); phase 2: re-scan the queue.
#pragma unroll
  for (int j = 0; j < NST; ++j) {
    const int v[4] = {vv[j].x, vv[j].y, vv[j].z, vv[j].w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (v[k] < 0) {
        const int slot = atomicAdd(&qn[wave], 1);
        if (slot < kFixQ) q[wave][slot] = make_int2(j * 256 + 4 * lane + k, v[k]);
      }
  }
  lds_sync();
  const int nq = qn[wave];
  rescan(min(nq, kFixQ));
  if (nq > kFixQ) {  // more marked cells than the queue holds (wave-uniform; rare): the rest in rounds
    __threadfence();  // the re-scanned cells' indices are written: the reloads below see them fixed (>= 0)
    if (lane == 0) qn[wave] = 0;
    lds_sync();
#pragma unroll 1
    for (int st = 0; st < kFixCells; st += 256) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long long c = base + st + 4 * lane + k;
        const int v = c < ncell ? __hip_atomic_load(out_idx + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        if (v < 0) q[wave][atomicAdd(&qn[wave], 1)] = make_int2(st + 4 * lane + k, v);
      }
      lds_sync();
      const int n = qn[wave];
      if (n >= 8 || st + 256 >= kFixCells) {
        rescan(n);
        if (lane == 0) qn[wave] = 0;
        lds_sync();
      }
    }
  }
}

hipError_t launch_doa_fixup(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                            const int* c_rc, const long long* ncell_dev, long long ncell_host, int G, int music,
                            const double* steerT, int* out_idx, float* out_gmax) {
  if (A < 1 || A > 16 || G >= (1 << 24) || !steerT) return hipErrorInvalidValue;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_DOA_NOFIX"))  // measurement only: marked cells keep -1 - code
    if (atoi(e) == 1) return hipSuccess;
#endif
  long long fb = (ncell_host + 4LL * kFixCells - 1) / (4LL * kFixCells);  // kFixCells cells per wave
  if (fb < 1) fb = 1;
  // steerT = the transposed fp64 table [A][G], built once with the steering tables (rsl_steer_table_build)
  auto kern = A <= 8 ? (music ? k_doa_fixup<8, true> : k_doa_fixup<8, false>)
                     : (music ? k_doa_fixup<16, true> : k_doa_fixup<16, false>);
  hipLaunchKernelGGL(kern, dim3((unsigned)fb), dim3(256), 0, st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, G,
                     reinterpret_cast<const double2*>(steerT), out_idx, out_gmax);
  return hipGetLastError();
}

template <int MA, int KB, bool MUSIC, bool GMAX, bool EXTRAS, bool SPEC = false>
static hipError_t launch_toep_t(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                                const int* c_rc, const long long* ncell_dev, long long ncell_host, const uint4* tab,
                                int ntiles, int G, const double* steer64, int* out_idx, float* out_gmax,
                                double esprit_scale, double* out_esprit, double* out_phase, int max_blocks,
                                float* out_spec = nullptr) {
  auto kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 0, 0, false, SPEC>;
  if constexpr (MA == 8 && !SPEC) {  // the 0.5-degree grid (G = 361: 12 tiles of 32): unrolled tile loop
    // skewed column-tile chains: tools/doa_var_ab.py, one call, 3.77-3.78 vs 3.83-3.87 ms per 2000 cfg2 frames,
    // outputs bit-identical (the spectrum scan keeps the rolled tile loop: the unrolled one spills with the stores)
    if (ntiles == 12) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 0, 12, true>;
  }
  if constexpr (MA == 16 && !SPEC) {  // 16 antennas (KB = 2): the tile loop unrolled, no skew (that needs KB = 1)
    if (ntiles == 12) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 0, 12, false>;
  }
#ifdef RSL_DEV_KNOBS
  if constexpr (MUSIC && !GMAX && !SPEC && MA == 8) {  // RSL_DOA_DBG: ablation variants of the skewed kernel (timing)
    if (const char* e = getenv("RSL_DOA_DBG")) {
      const int v = atoi(e);
      if (ntiles == 12) {
        if (v == 1) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 1, 12, true>;  // no record-tile copies
        if (v == 3) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 3, 12, true>;  // no signature loads
        if (v == 8) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 8, 12, true>;  // no argmax epilogue
        if (v == 9) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 9, 12, true>;  // no tile loop
        if (v == 10) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 10, 12, true>;  // L2-resident signatures
        if (v == 13) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 13, 12, true>;  // no second tracking
        if (v == 14) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 14, 12, true>;  // no in-tile count
        if (v == 15) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 15, 12, true>;  // second by one min
        if (v == 16) kern = k_doa_toep<MA, KB, MUSIC, GMAX, EXTRAS, 16, 12, true>;  // bound 5e-7 (study)
      }
    }
  }
#endif
  size_t lds = (size_t)ntiles * KB * 2 * 64 * sizeof(uint4);
  if (lds > 64 * 1024) return hipErrorInvalidValue;  // caller checks toep_table_fits()
  (void)max_blocks;
#ifdef RSL_DEV_KNOBS
  // RSL_DOA_WGPC: at most this many workgroups per CU (extra dynamic LDS), i.e. waves per SIMD (occupancy study)
  if (const char* e = getenv("RSL_DOA_WGPC")) {
    const int w = atoi(e);
    if (w > 0 && (size_t)(160 * 1024) / w > lds) lds = (size_t)(160 * 1024) / w - 256;
  }
#endif
  // Grid sized from the cell count (the capacity when the count is on the device; blocks past the cells exit before
  // loading the table) with ~8 passes per wave, instead of a persistent grid of resident blocks: measured 1.52-1.56
  // vs 1.71-1.79 ms per 1000 cfg2 frames (4 or 16 passes per wave: no better, tools/ppw_ab.sh).
  constexpr long long ppw = 8;
  long long blocks = (ncell_host + 256LL * ppw - 1) / (256LL * ppw);
  if (blocks < 1) blocks = 1;
#ifdef RSL_DEV_KNOBS
  // RSL_DOA_GRID: at most this many workgroups (the pass loop is grid-strided): a persistent share of the CUs, so
  // that the scan co-runs with the other batch's memory-bound kernels instead of taking whole CUs (study)
  if (const char* e = getenv("RSL_DOA_GRID")) {
    const long long g = atoll(e);
    if (g > 0 && blocks > g) blocks = g;
  }
#endif
  // ESPRIT's asin argument is clamped to [-1, 1] for d >= lambda / 2, where the reference's argument never exceeds 1
  // (|angle| <= pi) and only the fp32 rounding of pi * scale can; for d < lambda / 2, |x| > 1 gives NaN as in the
  // reference
  const int clamp = esprit_scale * 3.14159265358979323846 <= 1.0 + 1e-9;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, rds, A, S, C, c_frame, c_rc, ncell_dev,
                     ncell_host, tab, ntiles, G, steer64, out_idx, out_gmax, (float)esprit_scale, clamp, out_esprit,
                     out_phase, out_spec);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  // the exact re-scan of the marked cells
  return launch_doa_fixup(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, G, MUSIC, steer64, out_idx,
                          out_gmax);
}

hipError_t launch_doa_toep(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                           const int* c_rc, const long long* ncell_dev, long long ncell_host, const void* toep_tab,
                           int ntiles32, int G, int music, const double* steer64, int* out_idx, float* out_gmax,
                           double esprit_scale, double* out_esprit, double* out_phase, float* out_spec) {
  if (A < 1 || A > 16 || (ntiles32 & 1) || ncell_host >= (1LL << 31) - 64) return hipErrorInvalidValue;
  if (!steer64) return hipErrorInvalidValue;  // steerT: the exact fp64 re-scan of ambiguous cells
  if ((out_esprit || out_phase) && A < 2) return hipErrorInvalidValue;
  const long long max_blocks = ncell_dev ? 0 : (ncell_host + 255) / 256;  // 4 waves x 64 cells
  if (!ncell_dev && ncell_host <= 0) return hipSuccess;
  const uint4* tab = reinterpret_cast<const uint4*>(toep_tab);
  const bool gm = out_gmax != nullptr, ex = out_esprit || out_phase;
#define ARGS                                                                                                     \
  st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, tab, ntiles32, G, steer64, out_idx, out_gmax,          \
      esprit_scale, out_esprit, out_phase, (int)max_blocks
#define GO(MA, KB)                                                                                               \
  if (music) {                                                                                                   \
    if (gm) return ex ? launch_toep_t<MA, KB, true, true, true>(ARGS) : launch_toep_t<MA, KB, true, true, false>(ARGS); \
    return ex ? launch_toep_t<MA, KB, true, false, true>(ARGS) : launch_toep_t<MA, KB, true, false, false>(ARGS);     \
  }                                                                                                              \
  if (gm) return ex ? launch_toep_t<MA, KB, false, true, true>(ARGS) : launch_toep_t<MA, KB, false, true, false>(ARGS); \
  return ex ? launch_toep_t<MA, KB, false, false, true>(ARGS) : launch_toep_t<MA, KB, false, false, false>(ARGS);
  if (out_spec) {  // the spectrum-writing scan (cell-blocked layout), no GMAX
    if (gm) return hipErrorInvalidValue;
#define GOS(MA, KB)                                                                                              \
  if (music) return ex ? launch_toep_t<MA, KB, true, false, true, true>(ARGS, out_spec)                          \
                       : launch_toep_t<MA, KB, true, false, false, true>(ARGS, out_spec);                        \
  return ex ? launch_toep_t<MA, KB, false, false, true, true>(ARGS, out_spec)                                    \
            : launch_toep_t<MA, KB, false, false, false, true>(ARGS, out_spec);
    if (A <= 8) {
      GOS(8, 1)
    }
    GOS(16, 2)
#undef GOS
  }
  if (A <= 8) {
    GO(8, 1)
  }
  GO(16, 2)
#undef GO
#undef ARGS
}

bool toep_table_fits(int G, int M) {
  const int KB = M <= 8 ? 1 : 2;
  int nt = (G + 31) / 32;
  nt += nt & 1;
  return (size_t)nt * KB * 2 * 64 * 16 <= 64 * 1024;
}

// Host: Toeplitz operand table in MFMA A-operand order.  Returns 0 if the steering matrix is not a uniform
// linear array (then only the f32 path applies).  Layout: [tile t][k-block kb][part hi/lo][lane][8 halves],
// lane l = row (l & 31) of the tile, k = 16 kb + 8 (l >> 5) + j.  Tiles are padded to an even count with
// copies of row G-1.
int toep_table_build(const double* steer, int G, int M, uint16_t* out, int* ntiles32_out) {
  const int KB = M <= 8 ? 1 : 2;
  int nt = (G + 31) / 32;
  nt += nt & 1;
  if (ntiles32_out) *ntiles32_out = nt;
  if (M < 2) return 0;
  // uniformity: a[g][m] = a[g][0] * (a[g][1] conj(a[g][0]))^m, |a| = 1
  for (int g = 0; g < G; ++g) {
    const double* a = steer + (size_t)g * M * 2;
    const double a0r = a[0], a0i = a[1];
    if (fabs(a0r * a0r + a0i * a0i - 1.0) > 1e-9) return 0;
    const double er = a[2] * a0r + a[3] * a0i, ei = a[3] * a0r - a[2] * a0i;  // a1 conj(a0)
    double pr = a0r, pi = a0i;
    for (int m = 1; m < M; ++m) {
      const double nr = pr * er - pi * ei, ni = pr * ei + pi * er;
      pr = nr;
      pi = ni;
      if (fabs(pr - a[2 * m]) > 1e-9 || fabs(pi - a[2 * m + 1]) > 1e-9) return 0;
    }
  }
  for (int t = 0; t < nt; ++t)
    for (int kb = 0; kb < KB; ++kb)
      for (int lane = 0; lane < 64; ++lane) {
        int g = 32 * t + (lane & 31);
        if (g >= G) g = G - 1;
        const double* a = steer + (size_t)g * M * 2;
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * kb + 8 * (lane >> 5) + j;
          double v = 0.0;
          if (k == 0) {
            v = 1.0;
          } else if (k < 2 * M - 1) {
            const int q = (k + 1) / 2;  // e^{j q phi} = a_q conj(a_0)
            const double cr = a[2 * q] * a[0] + a[2 * q + 1] * a[1];
            const double ci = a[2 * q + 1] * a[0] - a[2 * q] * a[1];
            v = 2.0 * ((k & 1) ? cr : ci);
          }
          const _Float16 hi = (_Float16)v;
          const _Float16 lo = (_Float16)(v - (double)(float)hi);
          const size_t base = ((((size_t)t * KB + kb) * 2) * 64 + lane) * 8 + j;
          out[base] = __builtin_bit_cast(uint16_t, hi);
          out[base + 64 * 8] = __builtin_bit_cast(uint16_t, lo);
        }
      }
  return 1;
}

}  // namespace rsl
