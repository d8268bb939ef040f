// rsl_detect.hip — K3 peak detection and order-preserving compaction for gfx950.
//
// Replaces SignalPreprocessor.extract_range_doppler_peaks (reference src/radar_signal/dechirp.py:215-278):
//   db = 10 log10(|rds|^2 + 1e-12); peak = (maximum_filter(db, 3, mode='reflect') == db) & (db > thr)
//   & (min_range <= range_m[i] <= max_range); peaks listed antenna -> range -> doppler (np.where order).
// The 3x3 test runs on fp32 power p (log10 is monotone); 'reflect' boundary duplicates the edge cell,
// so out-of-range neighbours simply do not take part.  The threshold is evaluated as
// (double)p > 10^(thr/10) - 1e-12 and the range gate as an index interval, both precomputed in fp64.
// Per-antenna 64-bit ballots give one mask word per 64 Doppler cells; a per-frame scan then turns
// row counts into entry offsets (antenna-major) and union-cell offsets (range-major), and the emit
// kernel writes both lists in reference order without any sort.
#include <cstdlib>

#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

constexpr int kDetRows = 16;  // shifted range rows per workgroup

__global__ __launch_bounds__(256) void k_detect(const float2* __restrict__ rds, int S, int C, int W, double thr_p,
                                                int i_lo, int i_hi, unsigned long long* __restrict__ mask,
                                                int* __restrict__ row_count, float* __restrict__ dbmap,
                                                float* __restrict__ pk_pow) {
  extern __shared__ float pw[];  // (kDetRows + 2) x C power values
  const int nib = (S + kDetRows - 1) / kDetRows;
  const int ib = blockIdx.x % nib;
  const long fa = blockIdx.x / nib;
  const int i0 = ib * kDetRows;
  const int nrows = min(kDetRows, S - i0);
  const float2* base = rds + (size_t)fa * S * C;
  for (int idx = threadIdx.x; idx < (nrows + 2) * C; idx += 256) {
    const int r = idx / C, j = idx - r * C;
    const int i = i0 - 1 + r;
    pw[idx] = (i >= 0 && i < S) ? cabs2(base[(size_t)i * C + j]) : -1.f;  // -1: outside (no neighbour)
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = wave; r < nrows; r += 4) {
    const int i = i0 + r;
    const bool gate = (i >= i_lo && i <= i_hi);
    const float* up = pw + r * C;
    const float* mid = up + C;
    const float* dn = mid + C;
    int cnt = 0;
    for (int w = 0; w < W; ++w) {
      const int j = w * 64 + lane;
      bool pk = false;
      if (j < C) {
        const float p = mid[j];
        pk = gate && ((double)p > thr_p);
        const bool hasl = j > 0, hasr = j + 1 < C;
        float m = fmaxf(up[j], dn[j]);
        if (hasl) m = fmaxf(m, fmaxf(mid[j - 1], fmaxf(up[j - 1], dn[j - 1])));
        if (hasr) m = fmaxf(m, fmaxf(mid[j + 1], fmaxf(up[j + 1], dn[j + 1])));
        pk = pk && (p >= m);
        if (dbmap) dbmap[((size_t)fa * S + i) * C + j] = 10.f * log10f(p + 1e-12f);
      }
      const unsigned long long b = __ballot(pk);
      if (lane == 0) mask[((size_t)fa * S + i) * W + w] = b;
      if (pk_pow && pk)  // row-compact peak powers: slot = rank of the peak within its row
        pk_pow[((size_t)fa * S + i) * C + cnt + lanes_below(b)] = mid[j];
      cnt += __popcll(b);
    }
    if (lane == 0) row_count[(size_t)fa * S + i] = cnt;
  }
}

// Exclusive scan of one value per thread over an NT-thread block (wave shuffles + one LDS round); *total = the sum.
template <int NT>
__device__ long long block_exscan(long long v, long long* lds, long long* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  long long inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const long long u = __shfl_up(inc, d);
    if (lane >= d) inc += u;
  }
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  long long base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    const long long x = lds[k];
    base += k < w ? x : 0;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// Exclusive scan of n ints (global) into out (global) by one NT-thread block; returns total.
template <int NT>
__device__ long long block_scan_global(const int* in, int* out, int n, long long* lds) {
  const int t = threadIdx.x;
  const int per = (n + NT - 1) / NT;
  const int b = t * per, e = min(n, b + per);
  long long total;
  if (per % 4 == 0 && n % per == 0 && ((reinterpret_cast<size_t>(in) | reinterpret_cast<size_t>(out)) & 15) == 0) {
    // whole 16-B runs per thread (e.g. the A * S = 4096 row counts of a cfg2 frame: 4 int4 per thread, each thread's
    // 64-B segment read and written by 16-B accesses instead of 16 lane-strided 4-B ones)
    const int4* in4 = reinterpret_cast<const int4*>(in);
    int4* out4 = reinterpret_cast<int4*>(out);
    const int q0 = b >> 2, nq = (e - b) >> 2;
    int4 v[8];
    long long s = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < nq) {
        v[q] = in4[q0 + q];
        s += (long long)v[q].x + v[q].y + v[q].z + v[q].w;
      }
    for (int q = 8; q < nq; ++q) {  // long runs (per > 32): a second pass over the rest
      const int4 x = in4[q0 + q];
      s += (long long)x.x + x.y + x.z + x.w;
    }
    long long run = block_exscan<NT>(s, lds, &total);
    auto put = [&](int q, const int4& x) {
      int4 o;
      o.x = (int)run; run += x.x;
      o.y = (int)run; run += x.y;
      o.z = (int)run; run += x.z;
      o.w = (int)run; run += x.w;
      out4[q0 + q] = o;
    };
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < nq) put(q, v[q]);
    for (int q = 8; q < nq; ++q) put(q, in4[q0 + q]);
    return total;
  }
  long long s = 0;
  for (int k = b; k < e; ++k) s += in[k];
  long long run = block_exscan<NT>(s, lds, &total);
  for (int k = b; k < e; ++k) {
    const int v = in[k];
    out[k] = (int)run;
    run += v;
  }
  return total;
}

// One block per frame: entry offsets over (antenna, range) rows and union-cell offsets over range rows.  NT = 256:
// small blocks get CU slots between the long-lived DoA blocks of the other batch in the pipelined chain (a 1024-thread
// block waits for a whole CU to drain).
template <int NT>
__global__ __launch_bounds__(NT) void k_offsets(const unsigned long long* __restrict__ mask,
                                                const int* __restrict__ row_count, int A, int S, int W,
                                                int* __restrict__ entry_row_off, int* __restrict__ cell_row_off,
                                                int* __restrict__ cell_row_cnt, long long* __restrict__ frame_counts,
                                                unsigned long long* __restrict__ umask) {
  __shared__ long long lds[NT / 64];
  const long f = blockIdx.x;
  const long long te = block_scan_global<NT>(row_count + f * A * S, entry_row_off + f * A * S, A * S, lds);
  const unsigned long long* mf = mask + (size_t)f * A * S * W;
  if (W == 2) {  // C = 65..128 (cfg2): a row's two words as one 16-B load / store
    const ulonglong2* mf2 = reinterpret_cast<const ulonglong2*>(mf);
    ulonglong2* um2 = umask ? reinterpret_cast<ulonglong2*>(umask + (size_t)f * S * 2) : nullptr;
    for (int i = threadIdx.x; i < S; i += NT) {
      ulonglong2 u = make_ulonglong2(0ull, 0ull);
#pragma unroll 8
      for (int a = 0; a < A; ++a) {
        const ulonglong2 x = mf2[(size_t)a * S + i];
        u.x |= x.x;
        u.y |= x.y;
      }
      if (um2) um2[i] = u;
      cell_row_cnt[f * S + i] = __popcll(u.x) + __popcll(u.y);
    }
  } else
  for (int i = threadIdx.x; i < S; i += NT) {
    int c = 0;
    for (int w = 0; w < W; ++w) {
      unsigned long long u = 0;
      for (int a = 0; a < A; ++a) u |= mf[((size_t)a * S + i) * W + w];
      c += __popcll(u);
      if (umask) umask[((size_t)f * S + i) * W + w] = u;
    }
    cell_row_cnt[f * S + i] = c;
  }
  __syncthreads();
  const long long tc = block_scan_global<NT>(cell_row_cnt + f * S, cell_row_off + f * S, S, lds);
  if (threadIdx.x == 0) {
    frame_counts[2 * f] = te;
    frame_counts[2 * f + 1] = tc;
  }
}

// One block: exclusive scan over frames -> entry_base[F+1], cell_base[F+1].
template <int NT>
__global__ __launch_bounds__(NT) void k_frame_scan(const long long* __restrict__ frame_counts, int F,
                                                   long long* __restrict__ entry_base,
                                                   long long* __restrict__ cell_base) {
  __shared__ long long lds[NT / 64];
  const int t = threadIdx.x;
  const int per = (F + NT - 1) / NT;
  const int b = t * per, e = min(F, b + per);
  long long se = 0, sc = 0;
  for (int k = b; k < e; ++k) {
    se += frame_counts[2 * k];
    sc += frame_counts[2 * k + 1];
  }
  long long tot_e, tot_c;
  long long re = block_exscan<NT>(se, lds, &tot_e);
  long long rc = block_exscan<NT>(sc, lds, &tot_c);
  for (int k = b; k < e; ++k) {
    entry_base[k] = re;
    cell_base[k] = rc;
    re += frame_counts[2 * k];
    rc += frame_counts[2 * k + 1];
  }
  if (t == 0) {
    entry_base[F] = tot_e;
    cell_base[F] = tot_c;
  }
}

// One wave per (frame, range row): lane j of word w owns Doppler cell 64 w + j.  Ranks inside a word are
// popcounts of the lower lanes' bits, so every entry/cell index is computed without serial loops and the
// per-entry stores and RDS reads (power_db) are coalesced across the wave.
__global__ __launch_bounds__(256) void k_emit(const float2* __restrict__ rds, const unsigned long long* __restrict__ mask,
                                              int F, int A, int S, int C, int W,
                                              const int* __restrict__ entry_row_off, const int* __restrict__ cell_row_off,
                                              const long long* __restrict__ entry_base,
                                              const long long* __restrict__ cell_base, long long entry_cap,
                                              long long cell_cap, unsigned* __restrict__ e_coord,
                                              int* __restrict__ e_cell, float* __restrict__ e_pdb,
                                              int* __restrict__ c_frame,
                                              int* __restrict__ c_rc, unsigned* __restrict__ c_amask) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // f * S + i
  if (row >= (long)F * S) return;
  const int lane = threadIdx.x & 63;
  const long f = row / S;
  const int i = (int)(row - f * S);
  const unsigned long long* mf = mask + (size_t)f * A * S * W;
  const float2* rf = rds + (size_t)f * A * S * C;
  long long cnext = cell_base[f] + cell_row_off[row];
  const long long e0 = entry_base[f];
  for (int w = 0; w < W; ++w) {
    unsigned long long u = 0;
    for (int a = 0; a < A; ++a) u |= mf[((size_t)a * S + i) * W + w];
    if (u == 0) continue;  // wave-uniform
    const int j = w * 64 + lane;
    const bool has = (u >> lane) & 1ull;
    const long long c = cnext + lanes_below(u);
    unsigned am = 0;
    for (int a = 0; a < A; ++a) {
      const unsigned long long m = mf[((size_t)a * S + i) * W + w];
      if (!m) continue;  // wave-uniform
      const bool hb = (m >> lane) & 1ull;
      if (hb) {
        am |= 1u << a;
        const unsigned long long* mrow = mf + ((size_t)a * S + i) * W;
        long long e = e0 + entry_row_off[(size_t)f * A * S + (size_t)a * S + i] + lanes_below(m);
        for (int ww = 0; ww < w; ++ww) e += __popcll(mrow[ww]);
        if (e < entry_cap) {
          e_coord[e] = ((unsigned)a << 26) | ((unsigned)i << 13) | (unsigned)j;
          e_cell[e] = (int)c;
          if (e_pdb) {
            const float p = cabs2(rf[((size_t)a * S + i) * C + j]);
            e_pdb[e] = (float)(10.0 * log10((double)p + 1e-12));
          }
        }
      }
    }
    if (has && c < cell_cap) {
      c_frame[c] = (int)f;
      c_rc[c] = i * C + j;
      c_amask[c] = am;
    }
    cnext += __popcll(u);
  }
}

// Stream compaction of the peak / cell bit masks: 256 consecutive mask words per block produce one contiguous run of
// entries (or cells).  Phase 1: per-word popcounts, a block scan, and one packed (word, bit) code per item in
// LDS.  Phase 2: item k of the block is written by lane k % 256, so every store instruction is coalesced
// (consecutive lanes -> consecutive addresses); scattered 4-byte stores from a per-word set-bit loop would cost
// one memory request per lane.  Entries follow dechirp.py:257 (np.where order: antenna -> range -> doppler);
// cells are range-major unions over antennas.  power_db comes from the row-compact peak powers of k_detect
// (no RDS re-read), 10 log10 in fp32 (the powers are fp32), stored as float64 like power_spectrum_db.  A block with more than kEmitCap items
// runs phases 1-2 in rounds of kEmitCap (a per-word store loop would scatter 4-byte stores: measured 2.9x HBM write
// amplification on the 54%-dense cell unions of cfg2).
constexpr int kEmitCap = 2048;
constexpr int kEmitU = 4;  // phase-2 items per lane per trip

RSL_DEV int block_exclusive_scan(int v, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = wave_incl_scan(v);
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int pre = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ws = wsum[k];
    if (k < wave) pre += ws;
    total += ws;
  }
  return pre + x - v;
}

// WPE: minimum waves per SIMD the register allocation must allow (0: unconstrained; A/B knob RSL_EMIT_WPE).
// (Non-temporal entry stores were measured slower: 0.53 vs 0.48 ms per 1000 cfg2 frames.)
// CELLS = false: an entries-only launch (the cells go to k_emit_cells): no antenna-mask buffer in LDS (14 instead of 22
// KiB) and no cell path in the registers.
template <int W, int MAXA, int WPE = 0, bool CELLS = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1))) void k_emit_block(const unsigned long long* __restrict__ mask,
                                                    const unsigned long long* __restrict__ umask,
                                                    const float* __restrict__ pk_pow, int pk_group, long long F,
                                                    int A, int S, int C, const int* __restrict__ entry_row_off,
                                                    const int* __restrict__ cell_row_off,
                                                    const long long* __restrict__ entry_base,
                                                    const long long* __restrict__ cell_base, long long entry_cap,
                                                    long long cell_cap, long long nblk_e,
                                                    unsigned* __restrict__ e_coord, int* __restrict__ e_cell,
                                                    float* __restrict__ e_pdb,
                                                    int* __restrict__ c_frame, int* __restrict__ c_rc,
                                                    unsigned* __restrict__ c_amask) {
  static_assert(64 % W == 0, "a mask row must lie within one wave");
  __shared__ unsigned pk[kEmitCap];                  // item code: (word << 6) | bit
  __shared__ unsigned pam[CELLS ? kEmitCap : 1];  // cells: antenna mask of the item
  __shared__ int wsum[4];
  __shared__ int s_cw[256], s_fi[256];
  __shared__ long long s_pkb[256];  // entries: peak_pow index of the word's item 0 minus its block rank
  __shared__ unsigned long long s_u[256];
  __shared__ long long s_first;
  const int t = threadIdx.x, lane = t & 63;
  const bool entries = !CELLS || blockIdx.x < nblk_e;
  const long long nent = F * A * S * W, ncw = F * S * W;
  const long long gw0 = (entries ? (long long)blockIdx.x : (long long)blockIdx.x - nblk_e) * 256;  // row-aligned
  const long long nw = entries ? nent : ncw;
  const bool valid = gw0 + t < nw;
  const long long gw = valid ? gw0 + t : gw0;  // past-the-end words alias the block's first word (then m = 0)
  // word -> (row, w); entries: row = (f*A + a)*S + i, cells: row = f*S + i  (divisions once per word)
  const long long row = gw / W;
  const int w = (int)(gw - row * W);
  const long long q = row / S;  // entries: f*A + a ; cells: f
  const int i = (int)(row - q * S);
  const long long f = entries ? q / A : q;
  const int a = entries ? (int)(q - f * A) : 0;
  // every global load of the word is issued here, independent of its value (one memory round trip)
  unsigned long long m = entries ? mask[gw] : umask[gw];
  long long fst = 0;  // thread 0: the block's first item index (the block starts a row: no earlier words)
  if (t == 0) fst = entries ? entry_base[f] + entry_row_off[row] : cell_base[f] + cell_row_off[row];
  unsigned long long u = 0;  // entries: the union word of (f, i, w)
  long long cwb = 0;
  int cwo = 0;
  int gof = 0;  // entries: peaks of the earlier rows of the row's peak_pow group
  if (entries) {
    const int ig = i - i % pk_group;
    if (ig != i) gof = entry_row_off[row] - entry_row_off[row - (i - ig)];
    const unsigned long long* urow = umask + ((size_t)f * S + i) * W;
    u = urow[w];
    cwb = cell_base[f] + cell_row_off[f * S + i];
#pragma unroll
    for (int ww = 0; ww < W; ++ww)
      if (ww < w) cwo += __popcll(urow[ww]);
  }
  unsigned long long ma[CELLS ? MAXA : 1];  // cells: the antennas' peak words of (f, i, w)
  if (CELLS && !entries) {
#pragma unroll
    for (int aa = 0; aa < MAXA; ++aa) ma[aa] = aa < A ? mask[(((size_t)f * A + aa) * S + i) * W + w] : 0ull;
  }
  if (!valid) m = 0;
  const int cnt = __popcll(m);
  int total;
  const int loc = block_exclusive_scan(cnt, wsum, total);
  // entries: peaks of the earlier words of this row (the row's words are lanes lane-w .. lane of this wave)
  const int r0 = loc - __shfl(loc, lane - w);
  if (t == 0) s_first = fst;
  s_cw[t] = (int)(cwb + cwo);
  s_u[t] = u;
  s_fi[t] = entries ? ((a << 16) | i) : (int)f;
  // the row's group starts at row - i % pk_group; item k of the block reads peak_pow[s_pkb + base + k] (divisions once
  // per word instead of 64-bit divisions per item)
  if (entries) s_pkb[t] = (row - i % pk_group) * (long long)C + (r0 + gof) - loc;
  // rounds of kEmitCap items (one round unless the block is dense, e.g. the cell union at high peak density)
  for (int base = 0; base < total; base += kEmitCap) {
    // phase 1: packed (word, bit) codes (+ the cell's antenna mask) of this round's items, in LDS
    if (loc < base + kEmitCap && loc + cnt > base) {
      unsigned long long mm = m;
      int o = loc;
      while (mm && o < base + kEmitCap) {
        const int b = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        if (o >= base) {
          pk[o - base] = ((unsigned)t << 6) | (unsigned)b;
          if constexpr (CELLS) {
            if (!entries) {
              unsigned am = 0;
#pragma unroll
              for (int aa = 0; aa < MAXA; ++aa) am |= (unsigned)((ma[aa] >> b) & 1ull) << aa;
              pam[o - base] = am;
            }
          }
        }
        ++o;
      }
    }
    __syncthreads();
    const long long first = s_first + base;
    const int nk = total - base < kEmitCap ? total - base : kEmitCap;
    // phase 2: coalesced stores, lane k % 256 writes item k; kEmitU items per trip with their peak-power
    // gathers issued first (a rolled loop waits on each gather in turn)
    for (int k0 = t; k0 < nk; k0 += 256 * kEmitU) {
      if (entries) {
        float pw[kEmitU];
#pragma unroll
        for (int uu = 0; uu < kEmitU; ++uu) {
          const int k = k0 + 256 * uu;
          pw[uu] = 0.f;
          if (k < nk && e_pdb) {
            pw[uu] = pk_pow[s_pkb[pk[k] >> 6] + base + k];
          }
        }
#pragma unroll
        for (int uu = 0; uu < kEmitU; ++uu) {
          const int k = k0 + 256 * uu;
          const long long e = first + k;
          if (k < nk && e < entry_cap) {
            const unsigned code = pk[k];
            const int tt = (int)(code >> 6), b = (int)(code & 63);
            const int ww = (int)((gw0 + tt) % W);
            const int ai = s_fi[tt];
            e_coord[e] = ((unsigned)(ai >> 16) << 26) | ((unsigned)(ai & 0xffff) << 13) | (unsigned)(ww * 64 + b);
            e_cell[e] = s_cw[tt] + __popcll(s_u[tt] & ((1ull << b) - 1ull));
            if (e_pdb) e_pdb[e] = 10.0f * log10f(pw[uu] + 1e-12f);  // dechirp.py:235-236
          }
        }
      } else if constexpr (CELLS) {
#pragma unroll
        for (int uu = 0; uu < kEmitU; ++uu) {
          const int k = k0 + 256 * uu;
          const long long e = first + k;
          if (k < nk && e < cell_cap) {
            const unsigned code = pk[k];
            const int tt = (int)(code >> 6), b = (int)(code & 63);
            const long long g2 = gw0 + tt;
            const long long rw = g2 / W;
            const int ww = (int)(g2 - rw * W);
            c_frame[e] = s_fi[tt];
            c_rc[e] = (int)(rw - (long long)s_fi[tt] * S) * C + ww * 64 + b;
            c_amask[e] = pam[k];
          }
        }
      }
    }
    __syncthreads();  // pk / pam reused by the next round
  }
}

// Cell-list compaction (union masks, ~54 % dense at cfg2): 4 threads per mask word (16-bit slices), 64 words per
// block, so every block's items (at most 4096) are expanded in one round and no thread walks more than 16 set bits
// (k_emit_block's word-per-thread cells path walked ~35 bits per word, up to 5 rounds of 2048 per block).
// Blocks are row- and frame-aligned ((S * W) % 64 == 0): one contiguous run of cells from cell_base[f] + row offset.
constexpr int kCellWords = 64;
constexpr int kCellCap = kCellWords * 64;

template <int W, int MAXA>
__global__ __launch_bounds__(256) void k_emit_cells(const unsigned long long* __restrict__ mask,
                                                    const unsigned long long* __restrict__ umask, long long F, int A,
                                                    int S, int C, const int* __restrict__ cell_row_off,
                                                    const long long* __restrict__ cell_base, long long cell_cap,
                                                    int* __restrict__ c_frame, int* __restrict__ c_rc,
                                                    unsigned* __restrict__ c_amask) {
  // item code (thread << 4) | bit within the thread's 16-bit slice (12 bits); for MAXA <= 16 the cell's antenna mask
  // is packed above it (16 KiB of LDS instead of 32: 5 workgroups per CU instead of 4)
  constexpr bool PACK = MAXA <= 16;
  __shared__ unsigned pk[kCellCap];
  __shared__ unsigned pam[PACK ? 1 : kCellCap];
  __shared__ int wsum[4];
  __shared__ long long s_first;
  const int t = threadIdx.x;
  const long long ncw = F * S * W;
  const long long gw0 = (long long)blockIdx.x * kCellWords;
  const int wl = t >> 2, sl = t & 3;
  const bool valid = gw0 + wl < ncw;
  const long long gw = valid ? gw0 + wl : gw0;
  const long long row = gw / W;  // f * S + i
  const int w = (int)(gw - row * W);
  const long long f = row / S;
  const int i = (int)(row - f * S);
  unsigned long long m = valid ? umask[gw] : 0ull;
  unsigned long long ma[MAXA];
#pragma unroll
  for (int aa = 0; aa < MAXA; ++aa) ma[aa] = aa < A ? mask[(((size_t)f * A + aa) * S + i) * W + w] : 0ull;
  if (t == 0) s_first = cell_base[f] + cell_row_off[row];
  const unsigned sm16 = (unsigned)(m >> (16 * sl)) & 0xffffu;
  unsigned sa[MAXA];  // this thread's 16-bit slice of every antenna's word: 32-bit bit extracts per cell below
#pragma unroll
  for (int aa = 0; aa < MAXA; ++aa) sa[aa] = (unsigned)(ma[aa] >> (16 * sl)) & 0xffffu;
  int total;
  const int loc = block_exclusive_scan(__popc(sm16), wsum, total);
  {
    unsigned mm = sm16;
    int o = loc;
    while (mm) {
      const int b = __ffs(mm) - 1;
      mm &= mm - 1;
      unsigned am = 0;
#pragma unroll
      for (int aa = 0; aa < MAXA; ++aa) am |= ((sa[aa] >> b) & 1u) << aa;
      if constexpr (PACK) {
        pk[o] = ((unsigned)t << 4) | (unsigned)b | (am << 12);
      } else {
        pk[o] = ((unsigned)t << 4) | (unsigned)b;
        pam[o] = am;
      }
      ++o;
    }
  }
  __syncthreads();
  const long long first = s_first;
  for (int k = t; k < total; k += 256) {
    const long long e = first + k;
    if (e < cell_cap) {
      const unsigned code = pk[k];
      const int tt = (int)((code >> 4) & 0xffu);
      const long long g2 = gw0 + (tt >> 2);
      const long long rw = g2 / W;
      const int ww = (int)(g2 - rw * W);
      // the block lies in one frame (launch condition (S * W) % 64 == 0): every item's frame is this thread's f, so
      // no 64-bit division by S per item
      c_frame[e] = (int)f;
      c_rc[e] = (int)(rw - f * S) * C + ww * 64 + 16 * (tt & 3) + (int)(code & 15);
      c_amask[e] = PACK ? code >> 12 : pam[k];
    }
  }
}

hipError_t launch_emit2(hipStream_t st, const unsigned long long* mask, const unsigned long long* umask,
                        const float* pk_pow, int pk_group, int F, int A, int S, int C, const int* entry_row_off,
                        const int* cell_row_off, const long long* entry_base, const long long* cell_base,
                        long long entry_cap, long long cell_cap, unsigned* e_coord, int* e_cell, float* e_pdb,
                        int* c_frame, int* c_rc, unsigned* c_amask) {
  if (F <= 0) return hipSuccess;
  if (A > 32) return hipErrorInvalidValue;
  const int W = (C + 63) / 64;
  const long long nbe = ((long long)F * A * S * W + 255) / 256;
  // cells: k_emit_cells when its frame-aligned blocks tile the cell words, else the word-per-thread path
  const bool cells4 = ((long long)S * W) % kCellWords == 0;
  const long long nbc = cells4 ? 0 : ((long long)F * S * W + 255) / 256;
  const unsigned nb = (unsigned)(nbe + nbc);
  if (cells4) {
    const unsigned nbc4 = (unsigned)(((long long)F * S * W) / kCellWords);
#define GOC(WW)                                                                                                  \
  hipLaunchKernelGGL((A <= 8 ? k_emit_cells<WW, 8> : A <= 16 ? k_emit_cells<WW, 16> : k_emit_cells<WW, 32>),      \
                     dim3(nbc4), dim3(256), 0, st, mask,                                                        \
                     umask, (long long)F, A, S, C, cell_row_off, cell_base, cell_cap, c_frame, c_rc, c_amask);
    switch (W) {
      case 1: GOC(1) break;
      case 2: GOC(2) break;
      case 4: GOC(4) break;
      case 8: GOC(8) break;
      case 16: GOC(16) break;
      case 32: GOC(32) break;
      case 64: GOC(64) break;
      default: return hipErrorInvalidValue;
    }
#undef GOC
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  // registers capped for 7 waves per SIMD (72 VGPRs, no spill; 7 workgroups per CU as the LDS allows, instead of 6):
  // emit 0.45-0.47 vs 0.46-0.48 ms per 1000 cfg2 frames (tools/cpb.sh); the entries-only instance (cells by
  // k_emit_cells) holds 14 KiB of LDS and is capped for 8 waves per SIMD
  constexpr int EWPE = 8;
#define GO(WW)                                                                                                   \
  hipLaunchKernelGGL((cells4 ? k_emit_block<WW, 8, EWPE, false> /* entries only: MAXA unused */                 \
                             : (A <= 8 ? k_emit_block<WW, 8, 7> : k_emit_block<WW, 32>)),                         \
                     dim3(nb), dim3(256), 0, st, mask,                                                           \
                     umask, pk_pow, pk_group, (long long)F, A, S, C, entry_row_off, cell_row_off, entry_base, cell_base,     \
                     entry_cap, cell_cap, nbe, e_coord, e_cell, e_pdb, c_frame, c_rc, c_amask);
  switch (W) {
    case 1: GO(1) break;
    case 2: GO(2) break;
    case 4: GO(4) break;
    case 8: GO(8) break;
    case 16: GO(16) break;
    case 32: GO(32) break;
    case 64: GO(64) break;
    default: return hipErrorInvalidValue;
  }
#undef GO
  return hipGetLastError();
}

hipError_t launch_detect(hipStream_t st, const float2* rds, int F, int A, int S, int C, double thr_p, int i_lo,
                         int i_hi, unsigned long long* mask, int* row_count, float* dbmap, float* pk_pow) {
  if (F <= 0 || A <= 0 || S <= 0 || C <= 0) return hipSuccess;
  const int W = (C + 63) / 64;
  const long nblk = (long)F * A * ((S + kDetRows - 1) / kDetRows);
  const size_t lds = sizeof(float) * (kDetRows + 2) * (size_t)C;
  hipLaunchKernelGGL(k_detect, dim3((unsigned)nblk), dim3(256), lds, st, rds, S, C, W, thr_p, i_lo, i_hi, mask,
                     row_count, dbmap, pk_pow);
  return hipGetLastError();
}

hipError_t launch_offsets(hipStream_t st, const unsigned long long* mask, const int* row_count, int F, int A, int S,
                          int C, int* entry_row_off, int* cell_row_off, int* cell_row_cnt, long long* entry_base,
                          long long* cell_base, long long* frame_counts, unsigned long long* umask) {
  if (F <= 0) return hipSuccess;
  const int W = (C + 63) / 64;
  // 256-thread blocks: 1024-thread ones waited for a whole CU to drain behind the other batch's DoA blocks
  hipLaunchKernelGGL(k_offsets<256>, dim3(F), dim3(256), 0, st, mask, row_count, A, S, W, entry_row_off, cell_row_off,
                     cell_row_cnt, frame_counts, umask);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_frame_scan<256>, dim3(1), dim3(256), 0, st, frame_counts, F, entry_base, cell_base);
  return hipGetLastError();
}

hipError_t launch_emit(hipStream_t st, const float2* rds, const unsigned long long* mask, int F, int A, int S, int C,
                       const int* entry_row_off, const int* cell_row_off, const long long* entry_base,
                       const long long* cell_base, long long entry_cap, long long cell_cap, unsigned* e_coord,
                       int* e_cell, float* e_pdb, int* c_frame, int* c_rc, unsigned* c_amask) {
  if (F <= 0) return hipSuccess;
  const int W = (C + 63) / 64;
  const long rows = (long)F * S;
  hipLaunchKernelGGL(k_emit, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, rds, mask, F, A, S, C, W,
                     entry_row_off, cell_row_off, entry_base, cell_base, entry_cap, cell_cap, e_coord,
                     e_cell, e_pdb, c_frame, c_rc, c_amask);
  return hipGetLastError();
}

}  // namespace rsl
