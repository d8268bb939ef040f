// rsl_doa.hip — K4..K7: signature gather, MFMA steering scan (MUSIC / beamforming argmax), ESPRIT,
// spatial phase, robust confidence.  gfx950 / CDNA4.
//
// Replaces (reference src/angle_estimation/angle_estimation.py):
//   extract_spatial_signature :67-90, music_spectrum :109-154, estimate_angle_music :156-176,
//   estimate_angle_esprit :178-225, estimate_angle_beamforming :227-251,
// and robust_angle_estimation.py compute_angle_confidence :88-138, estimate_angle_robust :220-272.
//
// MUSIC in the reference is rank-1 (R = s s^H from one normalised snapshot), so with E_n the M-1
// noise eigenvectors, |a^H E_n E_n^H a| = M - |a^H s|^2 exactly; MUSIC and beamforming share the one
// dense contraction G = |A^H S|^2 (A: [G x M] steering table, S: [M x cells]).  It is run as a real
// GEMM on v_mfma_f32_16x16x4_f32 (exact fp32, bitwise an fmaf chain): steering rows are stacked
// [Re; Im] per grid point ([ar, ai] and [-ai, ar] against the column [sr; si]), so lane (q, col)
// of a 16x16 accumulator holds Re/Im of two grid points of one cell and folds |.|^2 + argmax
// in registers.  The steering operand lives in LDS in per-lane MFMA order (one ds_read_b128 per
// tile); 32 cells per wave per pass give two independent accumulator chains.
#include <cstdlib>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

// Loads the B operand (unit-normalised [Re; Im] signature column) of one 16-cell tile for this lane:
// lane (q, jj) holds S'[k = 4 s + q][cell jj], s < KS.  FAST: A == 2*KS, so the two complex loads for
// antennas q + 4s' (s' < KS/2) give both the real (slot s') and imaginary (slot s' + KS/2) parts.
template <int KS, bool FAST>
RSL_DEV void load_sig(const float2* __restrict__ rds, const int* __restrict__ cfr, const int* __restrict__ crc,
                      long long c, bool ok, int A, int q, size_t plane, size_t fstride, float (&b)[KS]) {
  const float2* base = rds;
  if (ok) base = rds + (size_t)cfr[c] * fstride + crc[c];
  if constexpr (FAST) {
#pragma unroll
    for (int s = 0; s < KS / 2; ++s) {
      float2 z = make_float2(0.f, 0.f);
      if (ok) z = base[(size_t)(4 * s + q) * plane];
      b[s] = z.x;
      b[s + KS / 2] = z.y;
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + q;
      float v = 0.f;
      if (ok && k < 2 * A) {
        const int m = k < A ? k : k - A;
        const float2 z = base[(size_t)m * plane];
        v = k < A ? z.x : z.y;
      }
      b[s] = v;
    }
  }
}

// Ambiguity bound of the f32 scans (relative top-2 gap): the [Re; Im] products are exact fp32 fmaf chains of <= 32
// terms, so P = re^2 + im^2 is within a few fp32 ulps of the fp64 value of the same fp32 signature; a cell whose
// best grid value is not this far above every other one (or, MUSIC, whose maximum is within rounding of M, where
// the reference's den > 1e-12 rule may move the argmax) is marked -1 (k_doa_fixup code 0) and re-scanned over the whole
// grid in fp64 by k_doa_fixup (rsl_doa_toep.hip), so that no grid index differs from the fp64 argmax of the cell's
// own signature by the scan's rounding.
constexpr float kAmbRel32 = 4e-6f;

RSL_DEV int mark_amb(int g, float best, float second, bool music, float Mf) {
  const bool amb = second >= best * (1.f - kAmbRel32) || !(best > 0.f) || (music && best >= Mf - 1e-4f);
  return amb ? -1 : g;  // k_doa_fixup code 0: the whole grid
}

// One wave = 32 cells (two 16-column MFMA tiles) per pass over all grid tiles; the next pass's signature
// loads are issued before the current pass's MFMAs (software prefetch).  Grid = resident workgroups only
// (occupancy query), grid-striding over 32-cell chunks, so no tail wave of late workgroups.
template <int KS, bool FAST, bool MUSIC, bool SPEC, bool GMAX>
__global__ __launch_bounds__(256) void k_doa_scan(const float2* __restrict__ rds, int A, int S, int C,
                                                  const int* __restrict__ cfr, const int* __restrict__ crc,
                                                  const long long* __restrict__ ncell_dev, long long ncell_host,
                                                  const float4* __restrict__ steer, int ntiles, int G, int use_lds,
                                                  int* __restrict__ out_idx, float* __restrict__ out_gmax,
                                                  float* __restrict__ out_spec, long long spec_ld) {
  constexpr int KSG = (KS + 3) / 4;
  extern __shared__ float4 sst[];
  __shared__ float4 sstage[SPEC ? 4 * 64 : 1];  // per wave: one tile's 8 grid points x 32 cells (grid-major stores)
  const float4* st = steer;
  if (use_lds) {
    for (int x = threadIdx.x; x < ntiles * KSG * 64; x += 256) sst[x] = steer[x];
    __syncthreads();
    st = sst;
  }
  const long long ncell = list_count(ncell_dev, ncell_host);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, jj = lane & 15;
  const size_t plane = (size_t)S * C, fstride = (size_t)A * plane;
  const float Mf = (float)A;
  const long long nch = (ncell + 31) >> 5;
  const long long stride = (long long)gridDim.x * 4;
  long long ch = (long long)blockIdx.x * 4 + wave;
  float nb[2][KS];
  if (ch < nch) {
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const long long c = ch * 32 + t2 * 16 + jj;
      load_sig<KS, FAST>(rds, cfr, crc, c, c < ncell, A, q, plane, fstride, nb[t2]);
    }
  }
  for (; ch < nch; ch += stride) {
    float b[2][KS];
    float pz[2];
    long long cidx[2];
    bool ok[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      cidx[t2] = ch * 32 + t2 * 16 + jj;
      ok[t2] = cidx[t2] < ncell;
      float acc = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        b[t2][s] = nb[t2][s];
        acc = fmaf(b[t2][s], b[t2][s], acc);
      }
      acc += __shfl_xor(acc, 16);
      acc += __shfl_xor(acc, 32);
      pz[t2] = acc;
      const float sc = acc > 0.f ? 1.0f / sqrtf(acc) : 1.0f;  // angle_estimation.py:86-88
#pragma unroll
      for (int s = 0; s < KS; ++s) b[t2][s] *= sc;
    }
    // prefetch the next chunk's signatures while this chunk's scan runs
    const long long nx = ch + stride;
    if (nx < nch) {
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const long long c = nx * 32 + t2 * 16 + jj;
        load_sig<KS, FAST>(rds, cfr, crc, c, c < ncell, A, q, plane, fstride, nb[t2]);
      }
    }
    float best[2] = {-INFINITY, -INFINITY}, second[2] = {-INFINITY, -INFINITY};
    float bestg[2] = {0.f, 0.f};
    int bidx[2] = {0, 0};
    for (int t = 0; t < ntiles; ++t) {
      float a[KSG * 4];
#pragma unroll
      for (int sg = 0; sg < KSG; ++sg) {
        const float4 v = st[(t * KSG + sg) * 64 + lane];
        a[4 * sg + 0] = v.x;
        a[4 * sg + 1] = v.y;
        a[4 * sg + 2] = v.z;
        a[4 * sg + 3] = v.w;
      }
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[0][s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[1][s], acc1, 0, 0, 0);
      }
      const int g0 = 8 * t + 2 * q;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
        const floatx4 acc = t2 ? acc1 : acc0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int g = g0 + h;
          const float re = acc[2 * h], im = acc[2 * h + 1];
          const float gv = fmaf(re, re, im * im);
          float key = gv;
          if constexpr (MUSIC) key = (Mf - gv > 1e-12f) ? gv : -1.f;  // den <= 1e-12 -> spectrum 0
          if (g < G) {
            if (key > best[t2]) {
              second[t2] = best[t2];
              best[t2] = key;
              bidx[t2] = g;
              if constexpr (GMAX) bestg[t2] = gv;
            } else {
              second[t2] = fmaxf(second[t2], key);
            }
          }
          if constexpr (SPEC) {
            float val = gv;
            if constexpr (MUSIC) {
              const float d = (pz[t2] > 0.f) ? Mf - gv : (Mf - 1.f);
              val = (d > 1e-12f) ? __builtin_amdgcn_rcpf(d) : 0.f;  // angle_estimation.py:149-152 (v_rcp_f32: 1 ulp)
            }
            if (spec_ld != 0) {
              // grid-major / cell-blocked: stage the tile (8 grid points x 32 cells) in LDS, stored below as 128-B runs
              reinterpret_cast<float*>(sstage + wave * 64)[(2 * q + h) * 32 + t2 * 16 + jj] = val;
            } else if (ok[t2] && g < G) {  // cell-major [n][G] (the reference's per-target spectrum rows)
              out_spec[(size_t)cidx[t2] * G + g] = val;
            }
          }
        }
      }
      if constexpr (SPEC) {
        if (spec_ld != 0) {
          __builtin_amdgcn_wave_barrier();
          const int r = lane >> 3, c4 = lane & 7;  // grid point 8 t + r, cells 4 c4 .. 4 c4 + 3 of the chunk
          const float4 v = sstage[wave * 64 + r * 8 + c4];
          __builtin_amdgcn_wave_barrier();
          const int g = 8 * t + r;
          const long long c0 = ch * 32 + 4 * c4;
          if (g < G && spec_ld < 0) {
            // cell-blocked [ceil(n / 32)][G][32]: a tile is one contiguous 1 KiB run, a pass one 46 KiB block
            *reinterpret_cast<float4*>(out_spec + ((size_t)ch * G + g) * 32 + 4 * c4) = v;
          } else if (g < G) {
            float* dst = out_spec + (size_t)g * spec_ld + c0;
            if (c0 + 3 < ncell && (spec_ld & 3) == 0) {
              *reinterpret_cast<float4*>(dst) = v;
            } else {
              if (c0 < ncell) dst[0] = v.x;
              if (c0 + 1 < ncell) dst[1] = v.y;
              if (c0 + 2 < ncell) dst[2] = v.z;
              if (c0 + 3 < ncell) dst[3] = v.w;
            }
          }
        }
      }
    }
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float ob = __shfl_xor(best[t2], off), os = __shfl_xor(second[t2], off);
        const int oi = __shfl_xor(bidx[t2], off);
        float og = 0.f;
        if constexpr (GMAX) og = __shfl_xor(bestg[t2], off);
        const bool take = ob > best[t2] || (ob == best[t2] && oi < bidx[t2]);  // first index wins (np.argmax)
        second[t2] = fmaxf(fmaxf(second[t2], os), take ? best[t2] : ob);
        if (take) {
          best[t2] = ob;
          bidx[t2] = oi;
          if constexpr (GMAX) bestg[t2] = og;
        }
      }
      if (q == 0 && ok[t2]) {
        out_idx[cidx[t2]] = mark_amb(bidx[t2], best[t2], second[t2], MUSIC, Mf);
        if constexpr (GMAX) out_gmax[cidx[t2]] = bestg[t2];
      }
    }
  }
}

// Argmax-only fast path (no spectrum output).  Per tile and cell column the epilogue is
//   g0 = re0^2 + im0^2, g1 = re1^2 + im1^2, c = g1 > g0, m = c ? g1 : g0, i = c ? 2t+1 : 2t,
//   u = m > best, best = u ? m : best, idx = u ? i : idx
// (10 VALU per 4 MFMA outputs; strict compares keep the first index, as np.argmax).  MUSIC's rule
// "den = M - g <= 1e-12 -> spectrum 0" can only matter when max g >= M in fp32 (a perfect steering
// match); such chunks are detected after the scan and re-run with the exact MUSIC key (slow path).
// NCT = 16-cell column tiles per wave (independent MFMA accumulator chains).
template <int KS, bool FAST, int NCT, bool KEYED>
RSL_DEV void argmax_scan(const float4* __restrict__ st, int ntiles, int G, float Mf, int q,
                         const float (&b)[NCT][KS], float (&best)[NCT], float (&second)[NCT], int (&bidx)[NCT]) {
  constexpr int KSG = (KS + 3) / 4;
#pragma unroll
  for (int t2 = 0; t2 < NCT; ++t2) {
    best[t2] = -INFINITY;
    second[t2] = -INFINITY;
    bidx[t2] = 0;
  }
#pragma unroll 2
  for (int t = 0; t < ntiles; ++t) {
    float a[KSG * 4];
#pragma unroll
    for (int sg = 0; sg < KSG; ++sg) {
      const float4 v = st[(t * KSG + sg) * 64 + (threadIdx.x & 63)];
      a[4 * sg + 0] = v.x;
      a[4 * sg + 1] = v.y;
      a[4 * sg + 2] = v.z;
      a[4 * sg + 3] = v.w;
    }
    floatx4 acc[NCT];
#pragma unroll
    for (int t2 = 0; t2 < NCT; ++t2) acc[t2] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t2 = 0; t2 < NCT; ++t2) acc[t2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[t2][s], acc[t2], 0, 0, 0);
    const int i0 = 8 * t + 2 * q;
    const bool last = (t == ntiles - 1);
#pragma unroll
    for (int t2 = 0; t2 < NCT; ++t2) {
      float g0 = fmaf(acc[t2][0], acc[t2][0], acc[t2][1] * acc[t2][1]);
      float g1 = fmaf(acc[t2][2], acc[t2][2], acc[t2][3] * acc[t2][3]);
      if constexpr (KEYED) {  // exact MUSIC key: points with M - g <= 1e-12 never win
        g0 = (Mf - g0 > 1e-12f) ? g0 : -1.f;
        g1 = (Mf - g1 > 1e-12f) ? g1 : -1.f;
      }
      if (last) {  // zero-padded rows of the last tile never win
        if (i0 >= G) g0 = -INFINITY;
        if (i0 + 1 >= G) g1 = -INFINITY;
      }
      const bool c = g1 > g0;
      const float m = c ? g1 : g0, lo = c ? g0 : g1;
      const int ii = c ? i0 + 1 : i0;
      const bool u = m > best[t2];
      second[t2] = u ? fmaxf(best[t2], lo) : fmaxf(second[t2], m);  // top-2 of everything this lane has seen
      best[t2] = u ? m : best[t2];
      bidx[t2] = u ? ii : bidx[t2];
    }
  }
}

template <int KS, bool FAST, int NCT, bool MUSIC, bool GMAX>
__global__ __launch_bounds__(256) void k_doa_argmax(const float2* __restrict__ rds, int A, int S, int C,
                                                    const int* __restrict__ cfr, const int* __restrict__ crc,
                                                    const long long* __restrict__ ncell_dev, long long ncell_host,
                                                    const float4* __restrict__ steer, int ntiles, int G, int use_lds,
                                                    int* __restrict__ out_idx, float* __restrict__ out_gmax) {
  constexpr int KSG = (KS + 3) / 4;
  constexpr int CPW = 16 * NCT;  // cells per wave per pass
  extern __shared__ float4 sst[];
  const float4* st = steer;
  if (use_lds) {
    for (int x = threadIdx.x; x < ntiles * KSG * 64; x += 256) sst[x] = steer[x];
    __syncthreads();
    st = sst;
  }
  const long long ncell = list_count(ncell_dev, ncell_host);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, jj = lane & 15;
  const size_t plane = (size_t)S * C, fstride = (size_t)A * plane;
  const float Mf = (float)A;
  const long long nch = (ncell + CPW - 1) / CPW;
  const long long stride = (long long)gridDim.x * 4;
  long long ch = (long long)blockIdx.x * 4 + wave;
  float nb[NCT][KS];
  if (ch < nch) {
#pragma unroll
    for (int t2 = 0; t2 < NCT; ++t2) {
      const long long c = ch * CPW + t2 * 16 + jj;
      load_sig<KS, FAST>(rds, cfr, crc, c, c < ncell, A, q, plane, fstride, nb[t2]);
    }
  }
  for (; ch < nch; ch += stride) {
    float b[NCT][KS];
#pragma unroll
    for (int t2 = 0; t2 < NCT; ++t2) {
      float acc = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        b[t2][s] = nb[t2][s];
        acc = fmaf(b[t2][s], b[t2][s], acc);
      }
      acc += __shfl_xor(acc, 16);
      acc += __shfl_xor(acc, 32);
      const float sc = acc > 0.f ? 1.0f / sqrtf(acc) : 1.0f;  // angle_estimation.py:86-88
#pragma unroll
      for (int s = 0; s < KS; ++s) b[t2][s] *= sc;
    }
    const long long nx = ch + stride;
    if (nx < nch) {
#pragma unroll
      for (int t2 = 0; t2 < NCT; ++t2) {
        const long long c = nx * CPW + t2 * 16 + jj;
        load_sig<KS, FAST>(rds, cfr, crc, c, c < ncell, A, q, plane, fstride, nb[t2]);
      }
    }
    float best[NCT], second[NCT];
    int bidx[NCT];
    argmax_scan<KS, FAST, NCT, false>(st, ntiles, G, Mf, q, b, best, second, bidx);
    if constexpr (MUSIC) {
      bool hit = false;
#pragma unroll
      for (int t2 = 0; t2 < NCT; ++t2) hit |= !(Mf - best[t2] > 1e-12f);
      if (__ballot(hit)) argmax_scan<KS, FAST, NCT, true>(st, ntiles, G, Mf, q, b, best, second, bidx);  // rare
    }
#pragma unroll
    for (int t2 = 0; t2 < NCT; ++t2) {
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {
        const float ob = __shfl_xor(best[t2], off), os = __shfl_xor(second[t2], off);
        const int oi = __shfl_xor(bidx[t2], off);
        const bool take = (ob > best[t2]) | ((ob == best[t2]) & (oi < bidx[t2]));  // first index wins
        second[t2] = fmaxf(fmaxf(second[t2], os), take ? best[t2] : ob);
        best[t2] = take ? ob : best[t2];
        bidx[t2] = take ? oi : bidx[t2];
      }
      const long long c = ch * CPW + t2 * 16 + jj;
      if (q == 0 && c < ncell) {
        out_idx[c] = mark_amb(bidx[t2], best[t2], second[t2], MUSIC, Mf);
        if constexpr (GMAX) out_gmax[c] = best[t2];
      }
    }
  }
}

template <int KS, bool FAST, bool MUSIC, bool GMAX>
static hipError_t launch_argmax_t(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                                  const int* c_rc, const long long* ncell_dev, long long ncell_host, const float4* stp,
                                  int ntiles, int G, int use_lds, size_t lds, int* out_idx, float* out_gmax,
                                  int max_blocks) {
  constexpr int NCT = 4;
  auto kern = k_doa_argmax<KS, FAST, NCT, MUSIC, GMAX>;
  static int per_cu[2] = {-1, -1};
  int& occ = per_cu[use_lds ? 1 : 0];
  if (occ < 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, lds) != hipSuccess || nb < 1) nb = 1;
    occ = nb;
  }
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  long long blocks = (long long)occ * ncu;
  if (max_blocks > 0) {
    const long long need = (max_blocks * 128LL + 16 * NCT * 4 - 1) / (16 * NCT * 4);  // max_blocks was for 128 cells
    if (blocks > need) blocks = need;
  }
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, rds, A, S, C, c_frame, c_rc, ncell_dev,
                     ncell_host, stp, ntiles, G, use_lds, out_idx, out_gmax);
  return hipGetLastError();
}

template <int KS, bool FAST, bool MUSIC, bool SPEC, bool GMAX>
static hipError_t launch_scan_t(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                                const int* c_rc, const long long* ncell_dev, long long ncell_host, const float4* stp,
                                int ntiles, int G, int use_lds, size_t lds, int* out_idx, float* out_gmax,
                                float* out_spec, long long spec_ld, int max_blocks) {
  auto kern = k_doa_scan<KS, FAST, MUSIC, SPEC, GMAX>;
  static int per_cu[2] = {-1, -1};  // occupancy per CU for the LDS / no-LDS variants
  int& occ = per_cu[use_lds ? 1 : 0];
  if (occ < 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, lds) != hipSuccess || nb < 1) nb = 1;
    occ = nb;
  }
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  long long blocks = (long long)occ * ncu;
  if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, rds, A, S, C, c_frame, c_rc, ncell_dev,
                     ncell_host, stp, ntiles, G, use_lds, out_idx, out_gmax, out_spec, spec_ld);
  return hipGetLastError();
}

template <int KS, bool FAST>
static hipError_t launch_scan_f(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                                const int* c_rc, const long long* ncell_dev, long long ncell_host, const float4* stp,
                                int ntiles, int G, int music, int use_lds, size_t lds, int* out_idx, float* out_gmax,
                                float* out_spec, long long spec_ld, int max_blocks) {
  const bool spec = out_spec != nullptr, gmax = out_gmax != nullptr;
#define L(M, SP, GM)                                                                                               \
  return launch_scan_t<KS, FAST, M, SP, GM>(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, stp, ntiles, G, \
                                            use_lds, lds, out_idx, out_gmax, out_spec, spec_ld, max_blocks)
  if (music) {
    if (spec) { if (gmax) L(true, true, true); else L(true, true, false); }
    else { if (gmax) L(true, false, true); else L(true, false, false); }
  } else {
    if (spec) { if (gmax) L(false, true, true); else L(false, true, false); }
    else { if (gmax) L(false, false, true); else L(false, false, false); }
  }
#undef L
}

hipError_t launch_doa_scan(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                           const int* c_rc, const long long* ncell_dev, long long ncell_host, const float* steer_tab,
                           int ntiles, int G, int music, int* out_idx, float* out_gmax, float* out_spec,
                           long long spec_ld, int grid_blocks) {
  const int KS = (2 * A + 3) / 4;
  const int KSG = (KS + 3) / 4;
  const size_t tab_bytes = (size_t)ntiles * KSG * 64 * sizeof(float4);
  const int use_lds = tab_bytes <= 60 * 1024;
  const size_t lds = use_lds ? tab_bytes : 0;
  const float4* stp = reinterpret_cast<const float4*>(steer_tab);
  const bool fast = (A == 2 * KS);
  if (!out_spec) {  // argmax-only fast path
    const bool gm = out_gmax != nullptr;
#define AM(n, F_)                                                                                                  \
  return music ? (gm ? launch_argmax_t<n, F_, true, true>(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host,  \
                                                          stp, ntiles, G, use_lds, lds, out_idx, out_gmax,         \
                                                          grid_blocks)                                             \
                     : launch_argmax_t<n, F_, true, false>(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, \
                                                           stp, ntiles, G, use_lds, lds, out_idx, out_gmax,        \
                                                           grid_blocks))                                           \
               : (gm ? launch_argmax_t<n, F_, false, true>(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, \
                                                           stp, ntiles, G, use_lds, lds, out_idx, out_gmax,        \
                                                           grid_blocks)                                            \
                     : launch_argmax_t<n, F_, false, false>(st, rds, A, S, C, c_frame, c_rc, ncell_dev,            \
                                                            ncell_host, stp, ntiles, G, use_lds, lds, out_idx,     \
                                                            out_gmax, grid_blocks))
    switch (KS) {
      case 2: if (fast) AM(2, true); AM(2, false);
      case 4: if (fast) AM(4, true); AM(4, false);
      case 6: if (fast) AM(6, true); AM(6, false);
      case 8: if (fast) AM(8, true); AM(8, false);
      case 1: AM(1, false);
      case 3: AM(3, false);
      case 5: AM(5, false);
      case 7: AM(7, false);
      default: return hipErrorInvalidValue;
    }
#undef AM
  }
#define CASE(n)                                                                                                    \
  case n:                                                                                                          \
    if (fast && (n % 2 == 0))                                                                                      \
      return launch_scan_f<n, (n % 2 == 0)>(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, stp, ntiles, G, \
                                            music, use_lds, lds, out_idx, out_gmax, out_spec, spec_ld,             \
                                            grid_blocks);                                                          \
    return launch_scan_f<n, false>(st, rds, A, S, C, c_frame, c_rc, ncell_dev, ncell_host, stp, ntiles, G, music,   \
                                   use_lds, lds, out_idx, out_gmax, out_spec, spec_ld, grid_blocks);
  switch (KS) {
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    default:
      return hipErrorInvalidValue;
  }
#undef CASE
}

// ---------------------------------------------------------------------------------------------
// Per-cell extras in fp64 from the fp32 RDS: normalised signature (angle_estimation.py:83-88),
// ESPRIT closed form (angle_estimation.py:178-225), spatial phase angle(s1 conj(s0))
// (velocity_solver.py:136), azimuth lookup from the argmax grid index.
//
// ESPRIT: svd of X = [s[:-1], s[1:]] -> U[:,0] = u ∝ X v with v the principal eigenvector of the
// 2x2 Hermitian X^H X; pinv(U1) U2 = u[:-1]^H u[1:] / u[:-1]^H u[:-1]; the scale/phase of u cancels.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxA = 32;

// NA > 0: antenna count fixed at compile time (registers only); NA == 0: runtime A (<= kMaxA).
template <int NA>
__global__ __launch_bounds__(256) void k_cell_extras(const float2* __restrict__ rds, int A_rt, int S, int C,
                                                     const int* __restrict__ cfr, const int* __restrict__ crc,
                                                     const long long* __restrict__ ncell_dev, long long ncell_host,
                                                     double esprit_scale, const int* __restrict__ gidx,
                                                     const double* __restrict__ az_table, float2* __restrict__ sig_out,
                                                     double* __restrict__ esprit_deg, double* __restrict__ phase,
                                                     double* __restrict__ az_out) {
  constexpr int MA = NA > 0 ? NA : kMaxA;
  const int A = NA > 0 ? NA : A_rt;
  const long long ncell = list_count(ncell_dev, ncell_host);
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  if (c >= ncell) return;
  const size_t plane = (size_t)S * C;
  const float2* base = rds + (size_t)cfr[c] * A * plane + crc[c];
  float2 zf[MA];
#pragma unroll
  for (int m = 0; m < MA; ++m)
    if (m < A) zf[m] = base[(size_t)m * plane];
  double sr[MA], si[MA];
  double pw = 0.0;
#pragma unroll
  for (int m = 0; m < MA; ++m) {
    if (m < A) {
      sr[m] = zf[m].x;
      si[m] = zf[m].y;
      pw += sr[m] * sr[m] + si[m] * si[m];
    }
  }
  if (pw > 0.0) {
    const double sc = 1.0 / sqrt(pw);
#pragma unroll
    for (int m = 0; m < MA; ++m)
      if (m < A) {
        sr[m] *= sc;
        si[m] *= sc;
      }
  }
  if (sig_out) {
#pragma unroll
    for (int m = 0; m < MA; ++m)
      if (m < A) sig_out[(size_t)c * A + m] = make_float2((float)sr[m], (float)si[m]);
  }
  if (phase) {
    // s1 * conj(s0)
    const double re = sr[1] * sr[0] + si[1] * si[0];
    const double im = si[1] * sr[0] - sr[1] * si[0];
    phase[c] = atan2(im, re);
  }
  if (az_out && gidx) az_out[c] = az_table[gidx[c]];
  if (esprit_deg) {
    double nr, ni, dd;
    esprit_phi<MA>(sr, si, A, nr, ni, dd);
    const double ang = dd > 0.0 ? atan2(ni, nr) : 0.0;
    esprit_deg[c] = asin(ang * esprit_scale) * (180.0 / 3.14159265358979323846);
  }
}

hipError_t launch_cell_extras(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                              const int* c_rc, const long long* ncell_dev, long long ncell_host, double esprit_scale,
                              const int* gidx, const double* az_table, float2* sig_out, double* esprit_deg,
                              double* phase, double* az_out) {
  if (A > kMaxA || A < 2) return hipErrorInvalidValue;
  if (ncell_host <= 0) return hipSuccess;
  const long long nb = (ncell_host + 255) / 256;
#define GO(NA)                                                                                                   \
  hipLaunchKernelGGL(k_cell_extras<NA>, dim3((unsigned)nb), dim3(256), 0, st, rds, A, S, C, c_frame, c_rc,      \
                     ncell_dev, ncell_host, esprit_scale, gidx, az_table, sig_out, esprit_deg, phase, az_out)
  if (A == 8) GO(8);
  else if (A == 16) GO(16);
  else if (A == 4) GO(4);
  else GO(0);
#undef GO
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Robust confidence (robust_angle_estimation.py:88-138), one thread per (cell, grid index):
//   0.4 |a^H s|/||s|| + 0.3 exp(-mean |wrap(arg s - arg a)|) + 0.3 min(1, log10(mean p / pct20(p)) / 3)
// clipped to [0, 1]; percentile is numpy 'linear' (index 0.2 (M-1)).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_confidence(const float2* __restrict__ rds, int A, int S, int C,
                                                    const int* __restrict__ cfr, const int* __restrict__ crc,
                                                    long long n, const int* __restrict__ gidx,
                                                    const double* __restrict__ steer,  // complex [G][A]
                                                    const double* __restrict__ sphase,  // [G][A] np.angle(a)
                                                    double* __restrict__ conf_out) {
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  if (c >= n) return;
  const size_t plane = (size_t)S * C;
  const float2* base = rds + (size_t)cfr[c] * A * plane + crc[c];
  double sr[kMaxA], si[kMaxA], p[kMaxA];
  double pw = 0.0;
  for (int m = 0; m < A; ++m) {
    const float2 z = base[(size_t)m * plane];
    sr[m] = z.x;
    si[m] = z.y;
    pw += sr[m] * sr[m] + si[m] * si[m];
  }
  if (pw > 0.0) {  // process_targets_robust normalises first (robust_angle_estimation.py:374-377)
    const double sc = 1.0 / sqrt(pw);
    for (int m = 0; m < A; ++m) {
      sr[m] *= sc;
      si[m] *= sc;
    }
  }
  const int g = gidx[c];
  const double* a = steer + (size_t)g * A * 2;
  const double* ap = sphase + (size_t)g * A;
  double cr = 0, ci = 0, sp = 0, perr = 0, pm = 0;
  for (int m = 0; m < A; ++m) {
    const double ar = a[2 * m], ai = a[2 * m + 1];
    cr += ar * sr[m] + ai * si[m];
    ci += ar * si[m] - ai * sr[m];
    p[m] = sr[m] * sr[m] + si[m] * si[m];
    sp += p[m];
    pm += p[m];
    double d = atan2(si[m], sr[m]) - ap[m];
    d = atan2(sin(d), cos(d));  // np.angle(np.exp(1j*d))
    perr += fabs(d);
  }
  const double corr = sqrt(cr * cr + ci * ci);
  const double ncorr = sp > 0 ? corr / sqrt(sp) : 0.0;
  const double pc = exp(-perr / A);
  // percentile 20, linear: sort p ascending (insertion sort, A <= 32)
  for (int i = 1; i < A; ++i) {
    const double v = p[i];
    int j = i - 1;
    while (j >= 0 && p[j] > v) {
      p[j + 1] = p[j];
      --j;
    }
    p[j + 1] = v;
  }
  const double vi = 0.2 * (A - 1);
  const int lo = (int)floor(vi);
  const int hi = lo + 1 < A ? lo + 1 : A - 1;
  const double tfr = vi - lo;
  double nf = (tfr >= 0.5) ? p[hi] - (p[hi] - p[lo]) * (1.0 - tfr) : p[lo] + (p[hi] - p[lo]) * tfr;
  double snrc = 0.0;
  if (nf > 0) {
    snrc = log10((pm / A) / nf) / 3.0;
    if (snrc > 1.0) snrc = 1.0;
  }
  double conf = ncorr * 0.4 + pc * 0.3 + snrc * 0.3;
  conf = fmin(1.0, fmax(0.0, conf));
  conf_out[c] = conf;
}

hipError_t launch_confidence(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                             const int* c_rc, long long n, const int* gidx, const double* steer_c128,
                             const double* steer_phase, double* conf_out) {
  if (A > kMaxA) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_confidence, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rds, A, S, C, c_frame, c_rc,
                     n, gidx, steer_c128, steer_phase, conf_out);
  return hipGetLastError();
}

}  // namespace rsl
