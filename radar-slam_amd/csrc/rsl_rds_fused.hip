// rsl_rds_fused.hip — single-pass range-Doppler spectrum + Doppler-direction detection for gfx950 (K12), and the
// range-direction detection finish (K3').
//
// Replaces SignalPreprocessor.generate_range_doppler_spectrum + extract_range_doppler_peaks (reference
// src/radar_signal/dechirp.py:143-166, 168-213, 215-278) for S = 512, C = 128 (configs[1..2]).
//
// Why: the two-kernel path (K1 range FFT -> `work` -> K2 Doppler FFT) moves the 4 MiB per-frame intermediate out to
// HBM and back (16 MiB per frame against 8 MiB of algorithmic traffic).  A whole (frame, antenna) slab (C x S c64 =
// 512 KiB) does not fit one CU's LDS, so the slab is split by RANGE CLASS: block q of a slab owns the range bins
// k = 8 k' + q (k' < 64).  Decimation in frequency by 8 gives
//     X_c[8 k' + q] = FFT64_n( y_c )[k'],   y_c[n] = sum_{j<8} g_q[n + 64 j] x_c[n + 64 j],
//     g_q[s] = conj(ref)[s] w[s] W_512^{s q}            (dechirp.py:139 and :108 folded into one table)
// so each of the 8 class blocks reads the whole slab but holds 1/8 of its spectrum: a 64 x 128 c64 LDS state (64 KiB,
// two blocks per CU).  The 8 class blocks of a slab are dispatched back to back on one XCD (block b serves XCD b % 8,
// class (b / 8) % 8), so 7 of the 8 slab reads are L2 hits: HBM sees the cube once.
//   Phase A (chirps -> range spectrum): a wave handles two chirps at a time, lane (h, p) owns y_c[2 p' + e] (e = 0, 1;
//     p' = bitrev5(p)): eight coalesced 16-B loads, 16 complex MACs, then the 64-point FFT as two 32-point radix-2
//     DIT FFTs across the 32 lanes of the chirp (xor partners: DPP quad permutes, ds_swizzle) and one in-lane radix-2.
//     Lane p ends with range bins k' = p and p + 32 of its chirp: written to the LDS state (XOR-swizzled columns,
//     conflict-free for both phases).  The next chirp pair's loads are in flight during the transform.
//   Phase B (Doppler): thread (k', u) reads chirps u + 8 i (i < 16), an in-register 16-point DFT, the twiddle
//     W_128^{u e} and a radix-8 DIF across the 8 lanes u: lane u holds the 16 contiguous Doppler bins 16 bitrev3(u) +
//     e.  fftshift on both axes is an index map.  Detection, first half: |X|^2, the Doppler-direction 3-max hm
//     ('reflect' at the shifted edges) and the candidate bit (threshold, range gate, p >= both Doppler neighbours).
//   Stores: RDS rows (1 KiB, one per wave instruction) and the hm rows, staged through the dead LDS state in two
//     halves.  The range neighbours of a row live in the other class blocks, so K3' (k_detect_finish) completes the
//     3x3 test from hm.  HBM per frame: cube 4 MiB in, RDS 4 MiB + hm 2 MiB + candidate bits out, hm back in.
#include <algorithm>
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
// value of lane (lane ^ D), D < 32: DPP quad permutes for 1 and 2, ds_swizzle bitmask mode (xor within 32 lanes)
typedef float f4v_t __attribute__((ext_vector_type(4)));
template <bool NTH>
RSL_DEV float4 ldq(const float4* p) {
  if constexpr (NTH) return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f4v_t*>(p)));
  else return *p;
}
template <bool NTH>
RSL_DEV void stq(float4* p, float4 x) {
  if constexpr (NTH) {
    f4v_t v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<f4v_t*>(p));
  } else {
    *p = x;
  }
}
// 16-B store with the sc1 bit: written through to memory without keeping the line in the XCD's L2
// (MI355X_MICROARCH.md: plain / nt stores keep it), so the streamed outputs do not evict the cube lines that the
// sibling class blocks are about to re-read.
RSL_DEV void st_sc1(float4* p, float4 x) {
  f4v_t v = {x.x, x.y, x.z, x.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}
template <int D>
RSL_DEV float xlane(float v) {
  if constexpr (D == 1) return dpp_xor1(v);
  else if constexpr (D == 2) return dpp_xor2(v);
  else return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (D << 10) | 0x1F));
}
template <int D>
RSL_DEV float2 xlane2(float2 v) { return make_float2(xlane<D>(v.x), xlane<D>(v.y)); }

// radix-2 butterfly across lanes (lane ^ D): lower lane (bit D clear) -> a + W b, upper -> a - W b (DIT, the upper
// lane pre-multiplies its own value by W; the lower lane's W is 1).
template <int D>
RSL_DEV float2 dit2(float2 own, float2 w, float sg) {
  const float2 z = cmul(own, w);
  const float2 zp = xlane2<D>(z);
  return make_float2(fmaf(sg, z.x, zp.x), fmaf(sg, z.y, zp.y));
}
// radix-2 DIF butterfly across lanes: lower -> a + b, upper -> (a - b) W
template <int D>
RSL_DEV float2 dif2(float2 own, float2 w, float sg) {
  const float2 pt = xlane2<D>(own);
  return cmul(make_float2(fmaf(sg, own.x, pt.x), fmaf(sg, own.y, pt.y)), w);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global loads (the
// __syncthreads lowering drains vmcnt too, which stalled the next slab's prefetched loads at every phase boundary).
RSL_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

RSL_DEV int brev5(int x) { return (int)(__brev((unsigned)x) >> 27); }
RSL_DEV int brev3(int x) { return (int)(__brev((unsigned)x) >> 29); }

// LDS state of a class block: row = range bin k' (64), column = chirp, then Doppler (128), c64.  Column XOR swizzle
// P(row): Phase A writes 16 consecutive rows of one column per 16-lane group (P mod 16 is a bijection of row mod 16)
// and Phase B reads 4 aligned rows x 8 columns u + 8 i per 32-lane group (P bits 3-4 = row & 3).
RSL_DEV int sx(int row, int col) {
  const int P = ((row & 1) << 3) | ((row >> 1) & 7) | (((row >> 1) & 1) << 4);
  return row * 128 + (col ^ P);
}

// K12.  Block = (slab = frame * A + antenna, range class q), 512 threads.  Writes the shifted RDS [slab][S][C], the
// Doppler-direction 3-max hm [slab][S][C] (f32, shifted order) and the candidate bits cand [slab][S][C/64] (u64; bit
// j % 64 of word j / 64 = shifted Doppler j).  CP: bit 0 nt cube loads, bit 1 nt RDS stores, bit 2 sc1 RDS stores, bit 3 sc1 hm stores; ablations: bit 4 no loads,
// bit 5 no Phase A compute, bit 6 no Phase B compute, bit 7 no global stores; bit 8 no cross-slab prefetch, bit 9
// natural-order loads with the lane FFT in DIF form.
template <int CP>
__global__ __launch_bounds__(512, 4) void k_rds_class(const float2* __restrict__ cube, int Ct, int c0, long nslab,
                                                      const float2* __restrict__ table,
                                                      const float2* __restrict__ twS,
                                                      const float2* __restrict__ twC, int dc,
                                                      float2* __restrict__ rds, float* __restrict__ hm_out,
                                                      unsigned long long* __restrict__ cand, float thr_f, int i_lo,
                                                      int i_hi, int map, int skew) {
  constexpr int S = 512, C = 128, NK = 64;
  __shared__ float2 st[NK * C];  // 64 KiB: the class state, then the store staging
  __shared__ float2 twc[C];
  __shared__ float4 gq[S / 2];  // g_q[s] pairs (s = 2 t, 2 t + 1)
  __shared__ float2 tw5[6][32];  // Phase A twiddles per lane p: 5 DIT stages (1 on lower lanes), then W_64^p
  const int tid = threadIdx.x, w = tid >> 6;
  // persistent: sibling group = the 8 class blocks b = 64 g1 + 8 q + x (same XCD x under round-robin placement);
  // they start together and do identical work per slab, so they read each slab line within a short window
  const long b = blockIdx.x;
  int q;
  long grp;
  const long ngrp = (long)(gridDim.x >> 3);
  if (map == 1 && gridDim.x == 512) {
    // 2 blocks per CU, block b and b + 256 on one CU (observed): make them siblings (classes 2 j, 2 j + 1), so the
    // second block's slab lines are fresh in the CU's L1
    const int sl = (int)(b >> 8), r = (int)(b & 255), x = r & 7, m = r >> 3;
    q = sl + 2 * (m & 3);
    grp = x + 8 * (m >> 2);
  } else {
    q = (int)((b >> 3) & 7);
    grp = ((b >> 6) << 3) + (b & 7);
  }
  if (grp >= nslab) return;
  {
    // skew > 0: de-phase the second block of each CU by `skew` clocks; skew < 0: stagger the siblings, class q
    // starting q * |skew| clocks late (so a sibling re-reads a line after its first reader's miss has filled L2)
    const long long d = skew > 0 ? (b >= (long)(gridDim.x >> 1) ? skew : 0) : (long long)q * (-skew);
    if (d > 0) {
      const long long t0 = clock64();
      while (clock64() - t0 < d) __builtin_amdgcn_s_sleep(8);
    }
  }
  for (int k = tid; k < C; k += 512) twc[k] = twC[k];
  for (int t = tid; t < S / 2; t += 512) {
    const float2 g0 = cmul(table[2 * t], twS[(2 * t * q) & (S - 1)]);
    const float2 g1 = cmul(table[2 * t + 1], twS[((2 * t + 1) * q) & (S - 1)]);
    gq[t] = make_float4(g0.x, g0.y, g1.x, g1.y);
  }
  for (int t = tid; t < 6 * 32; t += 512) {
    const int s = t >> 5, pp = t & 31, m = 1 << s;
    tw5[s][pp] = s == 5 ? twS[8 * pp] : ((pp & m) ? twS[(pp & (m - 1)) * (S / (2 * m))] : make_float2(1.f, 0.f));
  }

  // The slab loop recomputes every per-lane index from a laundered thread id: hoisted out of the loop, they stayed
  // live across both phases and spilled.
  auto lane_id = [&]() {
    int t = tid;
    asm volatile("" : "+v"(t));
    return t;
  };
  float4 va[8], vb[8];
  auto ld = [&](float4 (&v)[8], long sl, int cp, int t) {
    if (map == 2) sl = 0;                              // ablation: every block reads slab 0 (L2-resident)
    else if (map == 3) sl = (sl * 8 + q) % nslab;      // ablation: siblings read different slabs (no sharing)
    const int h = (t >> 5) & 1, pr = (CP & 512) ? (t & 31) : brev5(t & 31);
    const float4* r = reinterpret_cast<const float4*>(cube + ((size_t)sl * Ct + c0 + 2 * cp + h) * S) + pr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr ((CP & 16) != 0) v[j] = make_float4((float)j, 0.f, 0.f, (float)sl);  // ablation: no loads
      else v[j] = ldq<(CP & 1) != 0>(r + 32 * j);
    }
  };
  if constexpr ((CP & 256) == 0) ld(va, grp, w, tid);
  for (long slab = grp; slab < nslab; slab += ngrp) {
  lds_barrier();  // the previous slab's store staging is read out (first slab: the tables are written)
  {
    // ---- Phase A: lane (h, p) of wave w, chirp pairs w + 8 it ----
    const int t = lane_id();
    const int wv = t >> 6, h = (t >> 5) & 1, p = t & 31, pr = (CP & 512) ? p : brev5(p);
    const bool zero_dc = dc && q == 0 && p == 0;
    auto sg = [&](int s) { return (p >> s) & 1 ? -1.f : 1.f; };
    auto body = [&](const float4 (&cur)[8], int it) {
      if constexpr ((CP & 32) != 0) {  // ablation: no Phase A compute
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) a += cur[j].x + cur[j].y + cur[j].z + cur[j].w;
        st[sx(t & 31, 2 * ((t >> 6) + 8 * it) + ((t >> 5) & 1))] = make_float2(a, a);
        return;
      }
      // per-call laundered LDS indices: the table reads are loop-invariant, and hoisted they cost 44 VGPRs
      int pq = pr, p = t & 31;
      asm volatile("" : "+v"(pq), "+v"(p));
      float2 E = make_float2(0.f, 0.f), O = E;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 gv = gq[32 * j + pq];
        E = cadd(E, cmul(make_float2(cur[j].x, cur[j].y), make_float2(gv.x, gv.y)));
        O = cadd(O, cmul(make_float2(cur[j].z, cur[j].w), make_float2(gv.z, gv.w)));
      }
      int k1 = p;  // the range bin pair (k1, k1 + 32) this lane ends with
      if constexpr ((CP & 512) != 0) {
        // natural-order loads (each lane quad reads one 64-B run: the bit-reversed lane order of the DIT form broke
        // the L1's quad coalescing), radix-2 DIF across the lanes, output in bit-reversed lane order
        E = dif2<16>(E, tw5[4][p], sg(4));
        O = dif2<16>(O, tw5[4][p], sg(4));
        E = dif2<8>(E, tw5[3][p], sg(3));
        O = dif2<8>(O, tw5[3][p], sg(3));
        E = dif2<4>(E, tw5[2][p], sg(2));
        O = dif2<4>(O, tw5[2][p], sg(2));
        E = dif2<2>(E, tw5[1][p], sg(1));
        O = dif2<2>(O, tw5[1][p], sg(1));
        E = dif2<1>(E, tw5[0][p], sg(0));
        O = dif2<1>(O, tw5[0][p], sg(0));
        k1 = brev5(p);
      } else {
        E = dit2<1>(E, tw5[0][p], sg(0));
        O = dit2<1>(O, tw5[0][p], sg(0));
        E = dit2<2>(E, tw5[1][p], sg(1));
        O = dit2<2>(O, tw5[1][p], sg(1));
        E = dit2<4>(E, tw5[2][p], sg(2));
        O = dit2<4>(O, tw5[2][p], sg(2));
        E = dit2<8>(E, tw5[3][p], sg(3));
        O = dit2<8>(O, tw5[3][p], sg(3));
        E = dit2<16>(E, tw5[4][p], sg(4));
        O = dit2<16>(O, tw5[4][p], sg(4));
      }
      const float2 wo = cmul(O, tw5[5][k1]);
      float2 x0 = cadd(E, wo);
      const float2 x1 = csub(E, wo);
      if (zero_dc) x0 = make_float2(0.f, 0.f);  // DC removal = range bin 0 (dechirp.py:110-120)
      const int c = 2 * (wv + 8 * it) + h;
      st[sx(k1, c)] = x0;
      st[sx(k1 + 32, c)] = x1;
    };
    // every load is unconditional (the last slab re-loads its own first pair): with a conditional load the compiler
    // cannot count the loads in flight and drains all of them (vmcnt(0)) before each use
    const long nxt = slab + ngrp < nslab ? slab + ngrp : slab;
    if constexpr ((CP & 256) != 0) {  // no cross-slab prefetch: the slab's first pair is loaded here
      ld(va, slab, wv, t);
#pragma unroll
      for (int it2 = 0; it2 < 4; ++it2) {
        ld(vb, slab, wv + 8 * (2 * it2 + 1), t);
        body(va, 2 * it2);
        if (it2 < 3) ld(va, slab, wv + 8 * (2 * it2 + 2), t);
        body(vb, 2 * it2 + 1);
      }
    } else {
#pragma unroll 1
      for (int it2 = 0; it2 < 4; ++it2) {
        ld(vb, slab, wv + 8 * (2 * it2 + 1), t);
        body(va, 2 * it2);
        const bool last = it2 == 3;  // the next slab's first chirp pair: in flight during Phase B and the stores
        ld(va, last ? nxt : slab, last ? wv : wv + 8 * (2 * it2 + 2), t);
        body(vb, 2 * it2 + 1);
      }
    }
  }
  lds_barrier();

  // ---- Phase B: Doppler FFT of range bin kp over 8 lanes u ----
  const int t = lane_id();
  const int lane = t & 63, w = t >> 6;
  const int kk = lane >> 3, u = lane & 7, kp = 8 * w + kk;
  float2 X[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) X[i] = st[sx(kp, u + 8 * i)];
  if constexpr ((CP & 64) == 0) {
  Dft<16>::run(X);
#pragma unroll
  for (int e = 1; e < 16; ++e) X[e] = cmul(X[e], twc[u * e]);
  {
    const bool u4 = (u & 4) != 0, u2 = (u & 2) != 0, u1 = (u & 1) != 0;
    const float2 w8 = tw5[2][u];  // lanes 4..7: W_8^{u - 4}; lanes 0..3: 1
    const float2 w4 = (u2 && u1) ? make_float2(0.f, -1.f) : make_float2(1.f, 0.f);
    const float s4 = u4 ? -1.f : 1.f, s2 = u2 ? -1.f : 1.f, s1 = u1 ? -1.f : 1.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      X[e] = dif2<4>(X[e], w8, s4);
      X[e] = dif2<2>(X[e], w4, s2);
      const float2 pt = xlane2<1>(X[e]);
      X[e] = make_float2(fmaf(s1, X[e].x, pt.x), fmaf(s1, X[e].y, pt.y));
    }
  }
  }
  // lane u holds Doppler d = e + 16 v, v = bitrev3(u); shifted block vs = (v + 4) % 8
  const int v = brev3(u), vs = (v + 4) & 7;
  const int k = 8 * kp + q;
  const int i = (k + S / 2) & (S - 1);  // shifted range row
  const bool gate = i >= i_lo && i <= i_hi;
  const int gb = lane & ~7;
  // Doppler neighbours across the lane's block edges ('reflect' at the shifted Doppler edges)
  float le = __shfl(cabs2(X[15]), gb | brev3((v + 7) & 7));
  float re = __shfl(cabs2(X[0]), gb | brev3((v + 1) & 7));
  if (vs == 0) le = cabs2(X[0]);
  if (vs == 7) re = cabs2(X[15]);
  // hm[e] = max(p[e-1], p[e], p[e+1]), recomputed from X where needed (not kept in registers)
  auto hmax = [&](int e) {
    const float pl = e > 0 ? cabs2(X[e - 1]) : le;
    const float pr2 = e < 15 ? cabs2(X[e + 1]) : re;
    return fmaxf(fmaxf(pl, cabs2(X[e])), pr2);
  };
  unsigned bits = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float pc = cabs2(X[e]);
    bits |= (unsigned)(gate && pc > thr_f && pc >= hmax(e)) << e;
  }
  // ---- stores through the dead state, rows kp in [32 P, 32 P + 32) per pass ----
  constexpr int RST = C + C / 8;   // RDS staging row (float2): 2 pad slots per 16 Doppler bins
  constexpr int HST = C + C / 4;   // hm staging row (float): 4 pad slots per 16
  float2* srds = st;
  float* shm = reinterpret_cast<float*>(st + 32 * RST);
  unsigned short* scand = reinterpret_cast<unsigned short*>(shm + 32 * HST);
#pragma unroll 1
  for (int P = 0; P < 2; ++P) {
    lds_barrier();  // the state (pass 0) or the previous pass's staging is read out
    if ((w >> 2) == P) {
      const int rr = kp - 32 * P;
      float2* d = srds + rr * RST + 18 * vs;
#pragma unroll
      for (int e = 0; e < 16; e += 2)
        *reinterpret_cast<float4*>(d + e) = make_float4(X[e].x, X[e].y, X[e + 1].x, X[e + 1].y);
      float* hd = shm + rr * HST + 20 * vs;
#pragma unroll
      for (int e = 0; e < 16; e += 4)
        *reinterpret_cast<float4*>(hd + e) = make_float4(hmax(e), hmax(e + 1), hmax(e + 2), hmax(e + 3));
      scand[rr * 8 + vs] = (unsigned short)bits;
    }
    lds_barrier();
#pragma unroll
    for (int z = 0; z < 4; ++z) {  // 32 rows x 64 float4: one 1 KiB row per wave instruction
      const int idx = tid + 512 * z;
      const int rr = idx >> 6, c4 = idx & 63;
      const int kk2 = 8 * (32 * P + rr) + q;
      const int ii = (kk2 + S / 2) & (S - 1);
      const float4 val = *reinterpret_cast<const float4*>(srds + rr * RST + 2 * c4 + 2 * (c4 >> 3));
      float4* dst = reinterpret_cast<float4*>(rds + ((size_t)slab * S + ii) * C) + c4;
      if constexpr ((CP & 128) != 0) { if (val.x == 12345.f) *dst = val; }  // ablation: no stores
      else if constexpr ((CP & 4) != 0) st_sc1(dst, val);
      else stq<(CP & 2) != 0>(dst, val);
    }
#pragma unroll
    for (int z = 0; z < 2; ++z) {  // 32 rows x 32 float4
      const int idx = tid + 512 * z;
      const int rr = idx >> 5, c4 = idx & 31;
      const int kk2 = 8 * (32 * P + rr) + q;
      const int ii = (kk2 + S / 2) & (S - 1);
      const float4 val = *reinterpret_cast<const float4*>(shm + rr * HST + 4 * c4 + 4 * (c4 >> 2));
      float4* hdst = reinterpret_cast<float4*>(hm_out + ((size_t)slab * S + ii) * C) + c4;
      if constexpr ((CP & 128) != 0) { if (val.x == 12345.f) *hdst = val; }
      else if constexpr ((CP & 8) != 0) st_sc1(hdst, val);
      else *hdst = val;
    }
    if (tid < 64) {
      const int rr = tid >> 1, wd = tid & 1;
      const int kk2 = 8 * (32 * P + rr) + q;
      const int ii = (kk2 + S / 2) & (S - 1);
      const unsigned short* cs = scand + rr * 8 + 4 * wd;
      const unsigned long long word = (unsigned long long)cs[0] | ((unsigned long long)cs[1] << 16) |
                                      ((unsigned long long)cs[2] << 32) | ((unsigned long long)cs[3] << 48);
      cand[((size_t)slab * S + ii) * 2 + wd] = word;
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

// Opt-in (RSL_FUSED=1), S = 512, C = 128: measured slower than K1 + K2.  RSL_FUSED_CP: variant bits
// of k_rds_class (default 770 = natural-order loads, DIF across lanes, no cross-slab prefetch, nt RDS stores).
bool rds_fused_supported(int C, int S) {
  const char* e = getenv("RSL_FUSED");
  return e && atoi(e) != 0 && S == 512 && C == 128;
}

hipError_t launch_rds_fused(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C, int S,
                            const float2* table, const float2* tw_S, const float2* tw_C, int dc, float2* rds,
                            void* work, double thr_p, int i_lo, int i_hi) {
  if (S != 512 || C != 128) return hipErrorInvalidValue;
  const long nslab = (long)F * A;
  float* hmv = reinterpret_cast<float*>(work);
  unsigned long long* cand = reinterpret_cast<unsigned long long*>(hmv + (size_t)nslab * S * C);
  // persistent grid: resident blocks only (2 per CU), a multiple of 64 (8 XCDs x 8 range classes), no more sibling
  // groups than slabs
  static const long resident = [] {
    int dev = 0, ncu = 256, nb = 2;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rds_class<2>, 512, 0) != hipSuccess || nb < 1) nb = 1;
    const char* e = getenv("RSL_FUSED_BPC");
    if (e && atoi(e) > 0 && atoi(e) < nb) nb = atoi(e);
    return std::max(64L, ((long)nb * ncu) & ~63L);
  }();
  const long nblk = std::min(resident, ((nslab + 7) / 8) * 64);
  static const int cp = [] {
    const char* e = getenv("RSL_FUSED_CP");
    return e ? atoi(e) : 770;
  }();
  const float thr = threshold_as_float(thr_p);
  static const int map = [] {
    const char* e = getenv("RSL_FUSED_MAP");
    return e ? atoi(e) : 0;
  }();
  static const int skew = [] {
    const char* e = getenv("RSL_FUSED_SKEW");
    return e ? atoi(e) : 0;
  }();
#define RSL_KRC(CPV)                                                                                              \
  hipLaunchKernelGGL(k_rds_class<CPV>, dim3((unsigned)nblk), dim3(512), 0, st, cube, Ct, c0, nslab, table, tw_S, \
                     tw_C, dc, rds, hmv, cand, thr, i_lo, i_hi, map, skew)
  switch (cp) {  // variants kept for re-measuring (tools/k12_ab.py): bits as documented at k_rds_class
    case 2: RSL_KRC(2); break;      // DIT, bit-reversed lane loads, cross-slab prefetch
    case 514: RSL_KRC(514); break;  // DIF natural-order loads, cross-slab prefetch
    case 994: RSL_KRC(994); break;  // ablation: loads only (no Phase A / B compute, no stores)
    case 786: RSL_KRC(786); break;  // ablation: no loads
    case 898: RSL_KRC(898); break;  // ablation: no global stores
    default: RSL_KRC(770); break;   // DIF natural-order loads, no cross-slab prefetch
  }
#undef RSL_KRC
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
