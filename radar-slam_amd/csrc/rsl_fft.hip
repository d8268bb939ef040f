// rsl_fft.hip — K1 (dechirp*window + range FFT + DC) and K2 (Doppler FFT + fftshift) for gfx950.
//
// Replaces SignalPreprocessor.generate_range_doppler_spectrum (reference src/radar_signal/dechirp.py:168-213):
//   per chirp  y = x * conj(ref) * w ; y -= mean(y)      (dechirp.py:156-164)
//   rds = fftshift(fft2(y^T, axes=(1,2)), axes=(1,2))     (dechirp.py:193-211)
// DC removal is folded into the range FFT: FFT(y - mean y)[k] = FFT(y)[k] for k != 0 and 0 for k = 0,
// so the kernel zeroes range bin 0 instead of reducing a mean (exact in real arithmetic).
// conj(ref)*w is precomputed on the host in fp64 (the chirp phase reaches 2.5e7 rad) and passed as a c64 table.
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <cstdlib>
#include <type_traits>

// No packed-FP32 VALU (v_pk_add / v_pk_mul / v_pk_fma_f32) in the FFT kernels: both recorded pipelined-mode wrong
// results (round 3 in K2, round 4 in K1) sit in a packed-FP32 instruction whose source register pair the
// very next packed instruction overwrites, and the round-4 values fit, on all 16 lanes of the pass to fp32 rounding,
// that instruction reading its source AFTER the next one wrote it (tools/transient_fit.py).  Scalar fp32 ops compute
// the same roundings (fma for fma, mul for mul), so the outputs are bit-identical.  The device pass only: the feature
// is unknown to the host target.
#if defined(__HIP_DEVICE_COMPILE__)
#pragma clang attribute push(__attribute__((target("no-packed-fp32-ops"))), apply_to = function)
#endif
#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

constexpr int kThreads = 256;

// K1 work queues (RSL_RF_DYN): per (handle, stream), 8 per-XCD dequeue heads and 8 exit counters, each on its own
// 128-B line ([2][8][32] unsigned, 2 KiB of device memory allocated on the handle's device and zeroed on the stream's
// first K1 launch through that handle).  The last workgroup of an XCD to leave resets its pair, so the queue is clean
// for the stream's next launch; launches on one stream run in order, so no two K1 launches in flight ever share a
// queue.  The set lives in the handle (rsl_context::rfq) and rsl_destroy frees it: handles share no mutable state
// (rsl.h).  Round 5 kept one process-global map keyed by the stream handle alone, so two devices' null streams (both
// handle 0, what torch reports for a default stream) shared one queue on the first device.
constexpr size_t kRfQueueBytes = 2 * 8 * 32 * sizeof(unsigned);

struct RfQueues {
  int device = 0;
  std::mutex mu;
  std::unordered_map<hipStream_t, unsigned*> q;  // a destroyed stream's address may come back on this handle's device:
};                                               // its queue is clean between launches, so reuse is safe

RfQueues* rf_queues_new(int device) {
  RfQueues* s = new RfQueues();
  s->device = device;
  return s;
}

void rf_queues_free(RfQueues* s) {
  if (!s) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(s->device);
  for (auto& kv : s->q) (void)hipFree(kv.second);  // hipFree waits for the device: no K1 still reads the queue
  (void)hipSetDevice(cur);
  delete s;
}

// The queue of stream `st` in the set, allocated at its first use.  hipErrorStreamCaptureUnsupported when that first
// use is inside a graph capture (hipMalloc is not capturable: run one uncaptured K1 launch on the stream first, and
// never replay one captured K1 concurrently on two streams, which would share the captured queue); hipErrorInvalidDevice
// when the stream belongs to another device than the handle.
static hipError_t rf_queue(RfQueues* s, hipStream_t st, unsigned** out) {
  *out = nullptr;
  if (!s) return hipErrorInvalidValue;
  std::lock_guard<std::mutex> lock(s->mu);
  auto it = s->q.find(st);
  if (it != s->q.end()) {
    *out = it->second;
    return hipSuccess;
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
    return hipErrorStreamCaptureUnsupported;
  hipDevice_t sd = 0;
  if (st && hipStreamGetDevice(st, &sd) == hipSuccess && (int)sd != s->device) return hipErrorInvalidDevice;
  unsigned* q = nullptr;
  hipError_t e = hipMalloc(&q, kRfQueueBytes);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(q, 0, kRfQueueBytes, st);  // ordered before the stream's first K1
  if (e != hipSuccess) {
    (void)hipFree(q);
    return e;
  }
  s->q.emplace(st, q);
  *out = q;
  return hipSuccess;
}

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

// Packed `work` (K1 -> K2 at S = 512, C = 128).  Per K1 tile (frame, antenna, 8-chirp block cb)
// a 24 KiB block of 6 planes x 256 bin pairs x 16 B: planes 0-2 hold the even bin 2p of pair p, planes 3-5 the odd
// bin 2p + 1, each bin's 8 rows x (re, im) as 16 fields of 23 bits plus the bin's exponent (12 dwords, 3 x 16 B).
// Every K1 store and every K2 load is a 16-B access: a K1 wave stores 1 KiB runs (lane = pair), a K2 lane loads the 3
// chunks of one (bin, chirp block) and a wave's loads cover whole 128-B lines (16 bins = 8 pairs of one plane, or the
// other plane).  Each bin of a tile has its own exponent e (int8); a field is n = rint(v 2^(22 - e)), |n| < 2^22, stored
// offset-binary (the low 23 bits of the f32 1.5 2^23 + n: every such f32 has exponent 2^23), so the value's error is
// <= 2^(e - 23) = two fp32 ulps of the bin's largest component, fp32-class for the RDS (1e-5 max-relative tolerance)
// and the peak decisions.  The exponent byte sits in the 4 spare bits of the first two field groups (round 3; it was
// a separate [tile][512] byte array before, 0.26 GB of extra K1 writes and K2 byte loads per 2000 frames, and the
// fields were 24-bit with the 24th bit always 0: the same values, bit for bit).
// 6 B per value instead of 8: K1 + K2 move 14.0 instead of 16.8 MB per cfg2 frame.
constexpr float kPkMagic = 12582912.0f;  // 1.5 * 2^23
constexpr int kPkPlane = 4096;           // bytes per plane of one tile (256 pairs x 16 B)
constexpr int kPkTile = 6 * kPkPlane;    // bytes per tile
constexpr int kR128Pitch = 128 + 7;      // k_doppler_detect_r128 tile row pitch (float2)
constexpr int kR128Skew = 1;             // ... and the upper halo row's extra offset
// frexp exponent of the largest |component| (abs bits), clamped so that both scale factors are normal floats
RSL_DEV int pk_exp(unsigned mbits) {
  const int e = (int)((mbits >> 23) & 0xFFu) - 126;
  return e < -100 ? -100 : (e > 127 ? 127 : e);
}
RSL_DEV float pk_pow2(int k) { return __uint_as_float((unsigned)(127 + k) << 23); }
// 16 fields (8 complex) of one bin with its exponent e -> 12 dwords: field group g (u0..u3, 23 bits each) and a nibble
// x_g in 96 bits, u0 | u1 << 23, u1 >> 9 | u2 << 14, u2 >> 18 | u3 << 5 | x_g << 28; x_0 / x_1 = the low / high nibble
// of the int8 e, x_2 = x_3 = 0
RSL_DEV void pk_pack16(const float (&f)[16], int e, uint4 (&o)[3]) {
  const float s = pk_pow2(22 - e);
  const rsl_f2v s2 = {s, s}, mg = {kPkMagic, kPkMagic};
  unsigned u[16], d[12];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    // fma rounds v s to the nearest integer (|v s| < 2^22; one packed fma per complex value); the min keeps a value
    // that rounds up to 2^22 in range
    const rsl_f2v q = __builtin_elementwise_fma((rsl_f2v){f[c], f[c + 1]}, s2, mg);
    u[c] = min(__float_as_uint(q.x), 0x4B7FFFFFu) & 0x7FFFFFu;
    u[c + 1] = min(__float_as_uint(q.y), 0x4B7FFFFFu) & 0x7FFFFFu;
  }
  const unsigned eb = (unsigned)e & 0xFFu;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const unsigned x = g == 0 ? (eb & 0xFu) : (g == 1 ? (eb >> 4) : 0u);
    d[3 * g] = u[4 * g] | (u[4 * g + 1] << 23);
    d[3 * g + 1] = (u[4 * g + 1] >> 9) | (u[4 * g + 2] << 14);
    d[3 * g + 2] = (u[4 * g + 2] >> 18) | (u[4 * g + 3] << 5) | (x << 28);
  }
  o[0] = make_uint4(d[0], d[1], d[2], d[3]);
  o[1] = make_uint4(d[4], d[5], d[6], d[7]);
  o[2] = make_uint4(d[8], d[9], d[10], d[11]);
}
RSL_DEV void pk_unpack16(const uint4 (&w)[3], float (&f)[16]) {
  const unsigned d[12] = {w[0].x, w[0].y, w[0].z, w[0].w, w[1].x, w[1].y, w[1].z, w[1].w,
                          w[2].x, w[2].y, w[2].z, w[2].w};
  const int e = (int)(signed char)((d[2] >> 28) | ((d[5] >> 28) << 4));
  const float s = pk_pow2(e - 22);
  const float off = -kPkMagic * s;
  const rsl_f2v s2 = {s, s}, o2 = {off, off};
  // (field & 0x7FFFFF) | 0x4B000000 as one bit-field insert; the two fields of a complex value decoded by one packed fma
  auto m = [](unsigned x) { return __uint_as_float(__builtin_amdgcn_ubfe(x, 0, 23) | 0x4B000000u); };
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const unsigned u0 = d[3 * g];
    const unsigned u1 = __builtin_amdgcn_alignbit(d[3 * g + 1], d[3 * g], 23);
    const unsigned u2 = __builtin_amdgcn_alignbit(d[3 * g + 2], d[3 * g + 1], 14);
    const unsigned u3 = d[3 * g + 2] >> 5;
    // 0x4B000000 | u = 2^23 + u = 1.5 2^23 + n exactly; (that - 1.5 2^23) s in one rounding (exact: n s)
    const rsl_f2v a = __builtin_elementwise_fma((rsl_f2v){m(u0), m(u1)}, s2, o2);
    const rsl_f2v b = __builtin_elementwise_fma((rsl_f2v){m(u2), m(u3)}, s2, o2);
    f[4 * g] = a.x;
    f[4 * g + 1] = a.y;
    f[4 * g + 2] = b.x;
    f[4 * g + 3] = b.y;
  }
}

// Grid of a persistent kernel: resident workgroups only (occupancy x CUs), at most ntile.
static long resident_grid(const void* kern, size_t lds, long ntile, int nt = kThreads) {
  int nb = 0, dev = 0, ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, nt, lds) != hipSuccess || nb < 1) nb = 1;
  if (nb > 8) nb = 8;
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
// CB * S / 2 a multiple of the block size (every power-of-two S >= 16).  Cube loads and `work` stores are
// non-temporal (`nt`: both streamed once per batch; tools/cp_ab.py: 1.48-1.57 vs 1.57-1.64 ms per 1000 cfg2 frames).
// DYN: workgroup b serves XCD x = b % 8 (dispatch order) and walks that XCD's tile range [lo, hi): its first two tiles
// are static, every later one comes from the XCD's dequeue head, claimed one tile ahead (the atomic returns during a
// whole tile), so workgroups that start late (CUs held by a concurrent kernel) take fewer tiles (tools/dyn.sh: K1 alone
// 1.499 vs 1.667 ms per 1000 cfg2 frames for the static walk, outputs bit-identical).  Without DYN (grids of fewer
// than 8 workgroups) the walk is static.  DBG (development builds only; ablations with wrong results): 1 no FFT,
// 2 no cube loads (constant tiles), 3 loads and LDS staging only (no FFT, no stores).
template <int S, int CB, bool DYN, int DBG = 0>
__global__ __launch_bounds__(kThreads) void k_range_fft_p(const float2* __restrict__ cube, int A, int Ct, int c0,
                                                           int C, long ntile, const float2* __restrict__ table,
                                                           const float2* __restrict__ tw, int dc,
                                                           float2* __restrict__ work, unsigned* __restrict__ rfq,
                                                           unsigned char* __restrict__ wexp) {
  (void)wexp;
  constexpr int LD = lp_row(S);
  constexpr int H = S / 2;                 // float4 (2 complex) per row
  constexpr int PF = CB * H / kThreads;    // float4 per thread per tile
  static_assert((CB * H) % kThreads == 0, "tile must split evenly over the block");
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
      // would wait for it)
      if constexpr (DBG == 2)
        nx[q] = make_float4((float)tid, (float)q, (float)r, 1.f);
      else
        nx[q] = ld16<true>(src4 + (r < nrows ? idx : 0));
    }
  };
  __shared__ long s_nn;
  const int xcd = blockIdx.x & 7;
  const long gx = (G - xcd + 7) / 8;
  const long lo = DYN ? xcd * ntile / 8 : 0, hi = DYN ? (xcd + 1) * ntile / 8 : ntile;
  unsigned* head = rfq + xcd * 32;  // this XCD's dequeue head (the exit counter: + 256)
  // one tile: stage nx (x conj(ref) w) in LDS, refill nx with tile tn, FFT, DC bin, store
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
      if (r >= nrows) x = make_float4(0.f, 0.f, 0.f, 0.f);
      buf[r * LD + lp(2 * s2)] = cmul(make_float2(x.x, x.y), make_float2(tb.x, tb.y));
      buf[r * LD + lp(2 * s2 + 1)] = cmul(make_float2(x.z, x.w), make_float2(tb.z, tb.w));
    }
    __syncthreads();
    if (tn < hi) load(nx, tn);  // in flight during the FFT below
    if constexpr (DBG == 3) {  // loads only: keep the staged tile live, skip the FFT and the stores
      if (buf[tid * 2].x == 1.2345e30f) work[tid] = buf[tid * 2];
      if (DYN && tid == 0) s_nn = lo + 2 * gx + (long)claim;
      __syncthreads();
      return;
    }
    if constexpr (DBG != 1) fft_rows<S, CB, kThreads, LD, true>(buf, tws, tid);
    if (dc) {
      if (tid < CB) buf[tid * LD] = make_float2(0.f, 0.f);
      __syncthreads();
    }
    float4* dst4 = reinterpret_cast<float4*>(work + ((size_t)fa * C + cb * CB) * S);
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int idx = tid + q * kThreads;
      const int r = idx / H, s2 = idx - r * H;
      if (r < nrows) {
        const float2 lo2 = buf[r * LD + lp(2 * s2)], hi2 = buf[r * LD + lp(2 * s2 + 1)];
        st16<true>(dst4 + idx, make_float4(lo2.x, lo2.y, hi2.x, hi2.y));
      }
    }
    if (DYN && tid == 0) s_nn = lo + 2 * gx + (long)claim;
    __syncthreads();  // buf is rewritten by the next tile
  };
  if constexpr (DYN) {
    long t = lo + (blockIdx.x >> 3), tn = t + gx;
    float4 nx[PF];
    if (t < hi) load(nx, t);
    while (t < hi) {
      body(nx, t, tn);
      t = tn;
      tn = s_nn;  // written before body's last barrier, rewritten only after the next body's first one
    }
    // every dequeue of this workgroup has returned: the XCD's last leaver resets the slot for its next launch
    if (tid == 0 && atomicAdd(head + 8 * 32, 1u) == (unsigned)gx - 1u) {
      atomicExch(head, 0u);
      atomicExch(head + 8 * 32, 0u);
    }
    return;
  }
  long t = blockIdx.x;
  float4 nx[PF];
  if (t < ntile) load(nx, t);
  for (; t < ntile; t += G) body(nx, t, t + G);
}

// ---------------------------------------------------------------------------------------------
// K1 for S = 512 with packed `work` (the cfg2 shape): the range FFT as 16 x 32 in registers instead of three radix-8
// Stockham passes through LDS.  The LDS FFT was LDS-bound (SQ_LDS_IDX_ACTIVE ~70 % of the kernel's cycles, 21 % of wave
// time waiting on LDS issue, 42 % extra bank-conflict cycles): staging + 3 stage writes + 3 stage reads + the output
// read.  Here a tile (8 chirp rows of one (frame, antenna)) takes two LDS exchanges, both conflict-free:
//   a tile is chirp class c of one (frame, antenna): the 8 chirps c + 16 q (q < 8; C = 128, c < 16), so that the
//   Doppler transform's radix-8 step over q (and its W128^(c k1) twiddle) runs here, in registers, at the packed
//   store; K2 (k_doppler_detect_r128) does the 16-point step over the classes;
//   x[n], n = j + 32 m (j < 32, m < 16), thread t = (row q = t / 32, j = t % 32) loads x[j + 32 m] of chirp c + 16 q
//   (8-B loads, two 256-B runs per wave instruction) and multiplies by conj(ref) w;
//   stage 1: V[j][k1] = DFT16_m x[j + 32 m]  (registers), times W512^(j k1) (LDS table, 17-float2 pitch per j);
//   exchange: V' -> xbuf[row][k1][j] (pitch 34: the stage-2 reads of 32 lanes hit 64 distinct banks);
//   stage 2: thread t = (row, k1 = (t / 2) % 16, h = t % 2) takes j = 2 i + h: E or O = DFT16_i (registers); lane
//   pairs swap halves by DPP and form X[k1 + 16 k2] = E + W32^k2 O, X[k1 + 16 (k2 + 16)] = E - W32^k2 O;
//   output: X -> obuf[row][b + 8 (b / 256)] (the b >= 256 half shifted by 8: conflict-free writes), then thread p
//   reads bins 2p, 2p + 1 of the 8 rows (16-B reads), takes W128^(c k1) DFT8_q of each and stores them packed.
// X[k1 + 16 k2'] = sum_j W512^(j k1) W32^(j k2') sum_m x[j + 32 m] W16^(m k1): the 512-point DFT exactly.
// DBG (development builds only; wrong results): 2 no cube loads, 3 loads only.
constexpr int kR512Pitch = 34;             // xbuf pitch per (row, k1): 32 j + 2 pad
constexpr int kR512Obuf = 520;             // obuf row pitch (512 bins + 8 shift)
constexpr int kR512TwPitch = 17;           // ldtw pitch per j
RSL_DEV float2 w32(int k) {                // exp(-2 pi i k / 32), k < 16
  constexpr float c[16] = {1.f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f,
                           0.70710678118654757f, 0.55557023301960229f, 0.38268343236508984f, 0.19509032201612833f,
                           0.f, -0.19509032201612819f, -0.38268343236508973f, -0.55557023301960196f,
                           -0.70710678118654746f, -0.83146961230254535f, -0.92387953251128674f, -0.98078528040323043f};
  return make_float2(c[k], c[(k + 8) & 15] * (k < 8 ? 1.f : -1.f));  // -sin(2 pi k / 32)
}

template <bool DYN, int DBG = 0, bool NTW = true>
__global__ __launch_bounds__(kThreads) void k_range_fft_r512(const float2* __restrict__ cube, int A, int Ct, int c0,
                                                              int C, long ntile, const float2* __restrict__ table,
                                                              const float2* __restrict__ tw, int dc,
                                                              float2* __restrict__ work, unsigned* __restrict__ rfq,
                                                              unsigned char* __restrict__ wexp) {
  constexpr int S = 512, CB = 8;
  (void)wexp;  // the exponents travel inside the packed units (pk_pack16)
  __shared__ float2 ldtab[S];
  __shared__ float2 ldtw[32 * kR512TwPitch];
  __shared__ float2 xbuf[CB * 16 * kR512Pitch];  // stage exchange; aliased by the output buffer
  static_assert(CB * kR512Obuf <= CB * 16 * kR512Pitch, "output buffer must fit in the exchange buffer");
  float2* obuf = xbuf;
  const int tid = threadIdx.x;
  const int row = tid >> 5, j = tid & 31;
  const int k1b = (tid >> 1) & 15, h = tid & 1;
  constexpr int ncb = 128 / CB;  // C = 128 wherever this kernel runs (work_packed_supported): tile index math by shifts
  (void)C;
  const long G = gridDim.x;
  for (int k = tid; k < S; k += kThreads) ldtab[k] = table[k];
  for (int k = tid; k < 32 * 16; k += kThreads) {
    const int jj = k >> 4, kk = k & 15;
    ldtw[jj * kR512TwPitch + kk] = tw[jj * kk];  // W512^(j k1), j k1 <= 465
  }
  auto load = [&](float2(&nx)[16], long t) {
    t = (long)__builtin_amdgcn_readfirstlane((int)t);  // the tile index is workgroup-uniform (ntile < 2^31)
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    const float2* src = cube + ((size_t)fa * Ct + c0 + cb + 16 * row) * S + j;  // chirp class cb, row q = row
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if constexpr (DBG == 2)
        nx[m] = make_float2((float)tid, (float)m);
      else
        nx[m] = ld8<true>(src + 32 * m);
    }
  };
  __shared__ long s_nn;
  const int xcd = blockIdx.x & 7;
  const long gx = (G - xcd + 7) / 8;
  const long lo = DYN ? xcd * ntile / 8 : 0, hi = DYN ? (xcd + 1) * ntile / 8 : ntile;
  unsigned* head = rfq + xcd * 32;  // this XCD's dequeue head (the exit counter: + 256)
  __syncthreads();
  auto body = [&](float2(&nx)[16], long t, long tn) {
    // workgroup-uniform tile indices (read from LDS or derived from blockIdx; ntile < 2^31, checked by the launcher):
    // scalar, so the tile's address arithmetic runs on the SALU
    t = (long)__builtin_amdgcn_readfirstlane((int)t);
    tn = (long)__builtin_amdgcn_readfirstlane((int)tn);
    unsigned claim = 0;
    if (DYN && tid == 0) claim = atomicAdd(head, 1u);
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = cmul(nx[m], ldtab[j + 32 * m]);
    // in flight during this tile's transforms and stores; unconditional (past the range: this tile again, an L2 hit
    // once per workgroup), which spares a copy of the 32 loaded registers per tile
    load(nx, tn < hi ? tn : t);
    if constexpr (DBG == 3) {
      if (v[0].x == 1.2345e30f) work[tid] = v[1];
      if (DYN && tid == 0) s_nn = lo + 2 * gx + (long)claim;
      __syncthreads();
      return;
    }
    // stage 1: DFT16 over m, twiddle W512^(j k1)
    Dft<16>::run(v);
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], ldtw[j * kR512TwPitch + k]);
    float2* xw = xbuf + row * 16 * kR512Pitch + j;
#pragma unroll
    for (int k = 0; k < 16; ++k) xw[k * kR512Pitch] = v[k];
    __syncthreads();
    // stage 2: DFT16 over i of V'[2 i + h][k1], then the radix-2 combine across the lane pair (h = 0, 1)
    const float2* xr = xbuf + (row * 16 + k1b) * kR512Pitch + h;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = xr[2 * i];
    Dft<16>::run(v);
    // lane h = 0 holds E[k], lane h = 1 holds O[k]: u = E[k] or W32^k O[k], swapped with the partner lane by DPP;
    // bin k1 + 16 k = E + W O on h = 0 (u + recv), bin k1 + 16 (k + 16) = E - W O on h = 1 (recv - u): one packed
    // fma with a per-lane sign (+1 / -1) instead of selecting operands and both sums
    float2 xo[16];
    const rsl_f2v sgn = h ? (rsl_f2v){-1.f, -1.f} : (rsl_f2v){1.f, 1.f};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float2 u = h ? cmul(v[k], w32(k)) : v[k];
      float2 recv;
      recv.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(u.x), 0xB1, 0xF, 0xF, true));
      recv.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(u.y), 0xB1, 0xF, 0xF, true));
      xo[k] = cf(__builtin_elementwise_fma(sgn, cv(u), cv(recv)));
    }
    if (dc && k1b == 0 && h == 0) xo[0] = make_float2(0.f, 0.f);  // DC removal = zero range bin 0
    __syncthreads();  // xbuf reads done: obuf aliases it
    float2* ow = obuf + row * kR512Obuf + k1b + 264 * h;  // bin k1 + 16 k + 256 h at position bin + 8 h
#pragma unroll
    for (int k = 0; k < 16; ++k) ow[16 * k] = xo[k];
    __syncthreads();
    // thread tid holds bins 2 tid, 2 tid + 1 of the 8 rows (chirps cb + 16 q): the Doppler transform's first step,
    // Y[k1] = W128^(cb k1) DFT8_q, here in registers (K2 starts from the 16-point step)
    float2 y0[8], y1[8];
    const int pos = 2 * tid + (tid >= 128 ? 8 : 0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 ab = *reinterpret_cast<const float4*>(obuf + q * kR512Obuf + pos);
      y0[q] = make_float2(ab.x, ab.y);
      y1[q] = make_float2(ab.z, ab.w);
    }
    Dft<8>::run(y0);
    Dft<8>::run(y1);
    const int cbs = __builtin_amdgcn_readfirstlane(cb);  // the tile is workgroup-uniform
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float2 wk = tw[4 * cbs * k];  // W128^(cb k) = W512^(4 cb k), 4 cb k <= 420 (workgroup-uniform: scalar loads)
      y0[k] = cmul(y0[k], wk);
      y1[k] = cmul(y1[k], wk);
    }
    // packed store
    float f0[16], f1[16];
    unsigned m0 = 0u, m1 = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      f0[2 * q] = y0[q].x;
      f0[2 * q + 1] = y0[q].y;
      f1[2 * q] = y1[q].x;
      f1[2 * q + 1] = y1[q].y;
      m0 = max(m0, max(__float_as_uint(y0[q].x) & 0x7FFFFFFFu, __float_as_uint(y0[q].y) & 0x7FFFFFFFu));
      m1 = max(m1, max(__float_as_uint(y1[q].x) & 0x7FFFFFFFu, __float_as_uint(y1[q].y) & 0x7FFFFFFFu));
    }
    const int e0 = pk_exp(m0), e1 = pk_exp(m1);
    uint4 w0[3], w1[3];
    pk_pack16(f0, e0, w0);
    pk_pack16(f1, e1, w1);
    const size_t tile = (size_t)fa * ncb + cb;
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(work) + tile * kPkTile) + tid;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      st16<NTW>(reinterpret_cast<float4*>(dst + jj * (kPkPlane / 16)), __builtin_bit_cast(float4, w0[jj]));
      st16<NTW>(reinterpret_cast<float4*>(dst + (jj + 3) * (kPkPlane / 16)), __builtin_bit_cast(float4, w1[jj]));
    }
    if (DYN && tid == 0) s_nn = lo + 2 * gx + (long)claim;
    __syncthreads();  // obuf is read above; the next tile's exchange writes overwrite it
  };
  if constexpr (DYN) {
    long t = lo + (blockIdx.x >> 3), tn = t + gx;
    float2 nx[16];
    if (t < hi) load(nx, t);
    while (t < hi) {
      body(nx, t, tn);
      t = tn;
      tn = s_nn;
    }
    if (tid == 0 && atomicAdd(head + 8 * 32, 1u) == (unsigned)gx - 1u) {
      atomicExch(head, 0u);
      atomicExch(head + 8 * 32, 0u);
    }
    return;
  }
  long t = blockIdx.x;
  float2 nx[16];
  if (t < ntile) load(nx, t);
  for (; t < ntile; t += G) body(nx, t, t + G);
}

// ---------------------------------------------------------------------------------------------
// K1 for S = 1024 with packed `work` (the configs[4] shape: C = 256): k_range_fft_r512's design at
// twice the length, on 512 threads.  A tile is chirp class c of one (frame, antenna), the 8 chirps c + 32 q (q < 8,
// c < 32), so that the radix-8 step of the 256-point Doppler transform over q, with its W256^(c k1) twiddle, runs here
// and K2 (k_doppler_detect_r256) does the 32-point step over the classes.  One wave per chirp row:
//   x[n], n = j + 64 m (j < 64, m < 16): lane j of wave q loads x[j + 64 m] (8-B loads, 512-B runs), x conj(ref) w
//   (the dechirp table is read through L1: in LDS it would not leave room for two workgroups per CU);
//   stage 1: V[j][k1] = DFT16_m, times W1024^(j k1) (LDS, 16 per j, XOR-swizzled: k1 ^ ((j >> 1) & 15));
//   exchange: V -> xbuf[q][k1][j ^ 4 k1] (the stage-2 reads of 32 lanes then hit 64 distinct banks, the writes 32);
//   stage 2: lane (k1 = lane / 4, h = lane % 4) takes j = 4 i + h: F_h = DFT16_i, u_h = W64^(h k') F_h[k'], and the
//   radix-4 step over h across the lane quad by two DPP swaps (h ^ 2, then h ^ 1 after the W4 twiddle), after which
//   lane h holds Y[k' + 16 s], s = (h >> 1) | 2 (h & 1): bin k1 + 16 k' + 256 s;
//   output: -> obuf[q][bin ^ 4 s] (conflict-free 16-lane writes), then thread p reads bins 2p, 2p + 1 of the 8 rows
//   (16-B reads), takes W256^(c k1) DFT8_q and stores both bins packed (pk_pack16; planes of 512 pairs x 16 B).
// LDS: xbuf 64 KiB (aliased by obuf) + twiddles 8 KiB: two workgroups (16 waves) per CU.
constexpr int kR1kThreads = 512;
constexpr int kPkPlane1k = 8 * 1024;        // bytes per plane of one S = 1024 tile (512 pairs x 16 B)
constexpr int kPkTile1k = 6 * kPkPlane1k;   // bytes per tile
// W1024^(j k) in ldtw.  Swizzle (j / 2) ^ (j / 32): the stage-1 reads (lane j, one k) hit 64 distinct banks per 32-lane
// group, and the stage-2 reads of rows j = 16 h (h = lane % 4: swizzles 0, 8, 1, 9) do too; with (j / 2) alone rows
// 0 / 32 and 16 / 48 shared banks (2-way on 15 reads per tile and wave: most of the 17.2 M conflict cycles per 100
// configs[4] frames, gpurun_out/r5aa_ddctr5)
RSL_DEV int r1k_tw(int j, int k) { return j * 16 + (k ^ (((j >> 1) ^ (j >> 5)) & 15)); }

template <bool DYN, int DBG = 0>
__global__ __launch_bounds__(kR1kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_range_fft_r1024(const float2* __restrict__ cube, int A, int Ct,
                                                                  int c0, int C, long ntile,
                                                                  const float2* __restrict__ table,
                                                                  const float2* __restrict__ tw, int dc,
                                                                  float2* __restrict__ work, unsigned* __restrict__ rfq,
                                                                  unsigned char* __restrict__ wexp) {
  constexpr int S = 1024, NT = kR1kThreads, ncb = 32;  // C = 256 wherever this kernel runs (work_packed_supported)
  (void)wexp;
  (void)C;
  (void)A;
  __shared__ float2 ldtab[S];
  __shared__ float2 ldtw[64 * 16];
  __shared__ float2 xbuf[8 * S];  // stage exchange; aliased by the output buffer
  // 80 KiB exactly (two workgroups per CU): the tile hand-off word lives in a twiddle slot no lane reads (k1 = 0 of j = 0)
  long* s_nn = reinterpret_cast<long*>(&ldtw[r1k_tw(0, 0)]);
  float2* obuf = xbuf;
  const int tid = threadIdx.x;
  const long G = gridDim.x;
  for (int k = tid; k < S; k += NT) ldtab[k] = table[k];
  for (int k = tid; k < 64 * 16; k += NT) {
    const int jj = k >> 4, kk = k & 15;
    if (kk) ldtw[r1k_tw(jj, kk)] = tw[jj * kk];  // W1024^(j k1), j k1 <= 945 (k1 = 0: never read)
  }
  auto load = [&](float2(&nx)[16], long t) {
    t = (long)__builtin_amdgcn_readfirstlane((int)t);  // the tile index is workgroup-uniform (ntile < 2^31)
    int lt = tid;
    asm volatile("" : "+v"(lt));
    const int row = __builtin_amdgcn_readfirstlane(lt >> 6), j = lt & 63;  // one wave per chirp row: row is scalar
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    const float2* src = cube + ((size_t)fa * Ct + c0 + cb + 32 * row) * S + j;  // chirp class cb, row q = row
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if constexpr (DBG == 2)
        nx[m] = make_float2((float)tid, (float)m);
      else
        nx[m] = ld8<true>(src + 64 * m);
    }
  };
  const int xcd = blockIdx.x & 7;
  const long gx = (G - xcd + 7) / 8;
  const long lo = DYN ? xcd * ntile / 8 : 0, hi = DYN ? (xcd + 1) * ntile / 8 : ntile;
  unsigned* head = rfq + xcd * 32;  // this XCD's dequeue head (the exit counter: + 256)
  __syncthreads();
  auto body = [&](float2(&nx)[16], long t, long tn) {
    // workgroup-uniform tile indices (read from LDS or derived from blockIdx; ntile < 2^31, checked by the launcher):
    // scalar, so the tile's address arithmetic runs on the SALU
    t = (long)__builtin_amdgcn_readfirstlane((int)t);
    tn = (long)__builtin_amdgcn_readfirstlane((int)tn);
    unsigned claim = 0;
    if (DYN && tid == 0) claim = atomicAdd(head, 1u);
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    // the thread index laundered per tile: otherwise the compiler hoists the tile-invariant table and twiddle reads
    // out of the tile loop (92 registers live across it: 256 VGPRs with spills)
    int lt = tid;
    asm volatile("" : "+v"(lt));
    const int row = __builtin_amdgcn_readfirstlane(lt >> 6), j = lt & 63;  // one wave per chirp row: row is scalar
    const int k1b = (lt >> 2) & 15, h = lt & 3;
    const int s_out = (h >> 1) | ((h & 1) << 1);  // the radix-4 output index lane h ends with
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = cmul(nx[m], ldtab[j + 64 * m]);
    load(nx, tn < hi ? tn : t);  // in flight during this tile's transforms and stores
    if constexpr (DBG == 3) {
      if (v[0].x == 1.2345e30f) work[tid] = v[1];
      if (DYN && tid == 0) *s_nn = lo + 2 * gx + (long)claim;
      __syncthreads();
      return;
    }
    // stage 1: DFT16 over m, twiddle W1024^(j k1)
    Dft<16>::run(v);
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], ldtw[r1k_tw(j, k)]);
    float2* xw = xbuf + row * S;
#pragma unroll
    for (int k = 0; k < 16; ++k) xw[k * 64 + (j ^ ((4 * k) & 63))] = v[k];
    __syncthreads();
    // stage 2: DFT16 over i of V[4 i + h][k1], then the radix-4 step over h across the lane quad
    const float2* xr = xbuf + row * S + k1b * 64;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = xr[4 * (i ^ k1b) + h];
    Dft<16>::run(v);
    const float sg1 = (h & 2) ? -1.f : 1.f, sg2 = (h & 1) ? -1.f : 1.f;
    __syncthreads();  // xbuf reads done: obuf aliases it (the radix-4 step below writes each output as it forms)
    // bin k1 + 16 k + 256 s at (bin ^ 4 s) = ((k1 ^ 4 s) + 256 s) + 16 k: one base, constant offsets
    float2* ow = obuf + row * S + ((k1b ^ (4 * s_out)) + 256 * s_out);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float2 u = v[k];
      // W64^(h k) = W1024^(16 h k); unconditional (lanes h = 0 multiply by W^0 = 1: exact up to the sign of a zero)
      if (k > 0) u = cmul(u, ldtw[r1k_tw(16 * h, k)]);
      // h ^ 2: a = u_h0 +- u_(h0 + 2) (lanes with h & 2 hold the difference)
      float2 r;
      r.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(u.x), 0x4E, 0xF, 0xF, true));
      r.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(u.y), 0x4E, 0xF, 0xF, true));
      float2 a = make_float2(fmaf(sg1, u.x, r.x), fmaf(sg1, u.y, r.y));
      // lanes h0 = 1 take W4^(s0) = (-i)^(h >> 1) before the h ^ 1 swap
      if ((h & 1) && (h & 2)) a = make_float2(a.y, -a.x);
      r.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a.x), 0xB1, 0xF, 0xF, true));
      r.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a.y), 0xB1, 0xF, 0xF, true));
      float2 xo = make_float2(fmaf(sg2, a.x, r.x), fmaf(sg2, a.y, r.y));
      if (k == 0 && dc && k1b == 0 && h == 0) xo = make_float2(0.f, 0.f);  // DC removal = zero range bin 0
      ow[16 * k] = xo;
    }
    __syncthreads();
    // thread tid holds bins 2 tid, 2 tid + 1 of the 8 rows (chirps cb + 32 q): the Doppler transform's first step,
    // Y[k1] = W256^(cb k1) DFT8_q, here in registers (K2 starts from the 32-point step)
    float2 y0[8], y1[8];
    const int pos = (2 * lt) ^ (4 * ((lt >> 7) & 3));
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 ab = *reinterpret_cast<const float4*>(obuf + q * S + pos);
      y0[q] = make_float2(ab.x, ab.y);
      y1[q] = make_float2(ab.z, ab.w);
    }
    Dft<8>::run(y0);
    Dft<8>::run(y1);
    const int cbs = __builtin_amdgcn_readfirstlane(cb);  // the tile is workgroup-uniform
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float2 wk = tw[4 * cbs * k];  // W256^(cb k) = W1024^(4 cb k), 4 cb k <= 868 (workgroup-uniform: scalar loads)
      y0[k] = cmul(y0[k], wk);
      y1[k] = cmul(y1[k], wk);
    }
    float f0[16], f1[16];
    unsigned m0 = 0u, m1 = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      f0[2 * q] = y0[q].x;
      f0[2 * q + 1] = y0[q].y;
      f1[2 * q] = y1[q].x;
      f1[2 * q + 1] = y1[q].y;
      m0 = max(m0, max(__float_as_uint(y0[q].x) & 0x7FFFFFFFu, __float_as_uint(y0[q].y) & 0x7FFFFFFFu));
      m1 = max(m1, max(__float_as_uint(y1[q].x) & 0x7FFFFFFFu, __float_as_uint(y1[q].y) & 0x7FFFFFFFu));
    }
    const int e0 = pk_exp(m0), e1 = pk_exp(m1);
    uint4 w0[3], w1[3];
    pk_pack16(f0, e0, w0);
    pk_pack16(f1, e1, w1);
    const size_t tile = (size_t)fa * ncb + cb;
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(work) + tile * kPkTile1k) + lt;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      st16<true>(reinterpret_cast<float4*>(dst + jj * (kPkPlane1k / 16)), __builtin_bit_cast(float4, w0[jj]));
      st16<true>(reinterpret_cast<float4*>(dst + (jj + 3) * (kPkPlane1k / 16)), __builtin_bit_cast(float4, w1[jj]));
    }
    if (DYN && tid == 0) *s_nn = lo + 2 * gx + (long)claim;
    __syncthreads();  // obuf is read above; the next tile's exchange writes overwrite it
  };
  if constexpr (DYN) {
    long t = lo + (blockIdx.x >> 3), tn = t + gx;
    float2 nx[16];
    if (t < hi) load(nx, t);
    while (t < hi) {
      body(nx, t, tn);
      t = tn;
      tn = *s_nn;
    }
    if (tid == 0 && atomicAdd(head + 8 * 32, 1u) == (unsigned)gx - 1u) {
      atomicExch(head, 0u);
      atomicExch(head + 8 * 32, 0u);
    }
    return;
  }
  long t = blockIdx.x;
  float2 nx[16];
  if (t < ntile) load(nx, t);
  for (; t < ntile; t += G) body(nx, t, t + G);
}

// ---------------------------------------------------------------------------------------------
// K1 for S = 256 with packed `work` (the cfg1 / configs[0] shape: C = 64): the same chirp-class tiles on
// 128 threads.  A tile is chirp class c of one (frame, antenna), the 8 chirps c + 8 q (q < 8, c < 8); K2
// (k_doppler_detect_r64) does the 8-point step over the classes.  16 lanes per chirp row:
//   x[n], n = j + 16 m (j, m < 16): lane j of row q loads x[j + 16 m] (8-B loads, 128-B runs), x conj(ref) w;
//   stage 1: V[j][k1] = DFT16_m, times W256^(j k1) (LDS, XOR-swizzled);
//   exchange: V -> xbuf[q][k1][j ^ k1 ^ (q & 1)] (both rows of a 32-lane read group cover the 64 banks once);
//   stage 2: lane (q, k1) takes the 16 j: X[k1 + 16 k2] = DFT16_j, no cross-lane step;
//   output: -> obuf[q][bin] (aliasing xbuf), then thread p reads bins 2p, 2p + 1 of the 8 rows (16-B reads), takes
//   W64^(c k1) DFT8_q and stores both bins packed (planes of 128 pairs x 16 B).
// LDS 20 KiB: 8 workgroups (16 waves) per CU.
constexpr int kR256Threads = 128;
constexpr int kPkPlane256 = 8 * 256;        // bytes per plane of one S = 256 tile (128 pairs x 16 B)
constexpr int kPkTile256 = 6 * kPkPlane256;
RSL_DEV int r256_tw(int j, int k) { return j * 16 + (k ^ j); }  // W256^(j k) in ldtw

template <int DBG = 0>
__global__ __launch_bounds__(kR256Threads) void k_range_fft_r256(const float2* __restrict__ cube, int A, int Ct, int c0,
                                                                 int C, long ntile, const float2* __restrict__ table,
                                                                 const float2* __restrict__ tw, int dc,
                                                                 float2* __restrict__ work, unsigned* __restrict__ rfq,
                                                                 unsigned char* __restrict__ wexp) {
  constexpr int S = 256, NT = kR256Threads, ncb = 8;  // C = 64 wherever this kernel runs (work_packed_supported)
  (void)wexp;
  (void)C;
  (void)A;
  __shared__ float2 ldtab[S];
  __shared__ float2 ldtw[16 * 16];
  __shared__ float2 xbuf[8 * S];  // stage exchange; aliased by the output buffer
  __shared__ long s_nn;
  float2* obuf = xbuf;
  const int tid = threadIdx.x;
  const long G = gridDim.x;
  for (int k = tid; k < S; k += NT) ldtab[k] = table[k];
  for (int k = tid; k < 16 * 16; k += NT) {
    const int jj = k >> 4, kk = k & 15;
    ldtw[r256_tw(jj, kk)] = tw[jj * kk];  // W256^(j k1), j k1 <= 225
  }
  auto load = [&](float2(&nx)[16], long t) {
    t = (long)__builtin_amdgcn_readfirstlane((int)t);  // the tile index is workgroup-uniform (ntile < 2^31)
    int lt = tid;
    asm volatile("" : "+v"(lt));
    const int row = lt >> 4, j = lt & 15;
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    const float2* src = cube + ((size_t)fa * Ct + c0 + cb + 8 * row) * S + j;  // chirp class cb, row q = row
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if constexpr (DBG == 2)
        nx[m] = make_float2((float)tid, (float)m);
      else
        nx[m] = ld8<true>(src + 16 * m);
    }
  };
  const int xcd = blockIdx.x & 7;
  const long gx = (G - xcd + 7) / 8;
  const long lo = xcd * ntile / 8, hi = (xcd + 1) * ntile / 8;
  unsigned* head = rfq + xcd * 32;  // this XCD's dequeue head (the exit counter: + 256)
  __syncthreads();
  auto body = [&](float2(&nx)[16], long t, long tn) {
    // workgroup-uniform tile indices (read from LDS or derived from blockIdx; ntile < 2^31, checked by the launcher):
    // scalar, so the tile's address arithmetic runs on the SALU
    t = (long)__builtin_amdgcn_readfirstlane((int)t);
    tn = (long)__builtin_amdgcn_readfirstlane((int)tn);
    unsigned claim = 0;
    if (tid == 0) claim = atomicAdd(head, 1u);
    const int cb = (int)(t % ncb);
    const long fa = t / ncb;
    int lt = tid;  // laundered per tile: keeps the tile-invariant table reads inside the tile loop
    asm volatile("" : "+v"(lt));
    const int row = lt >> 4, j = lt & 15, k1 = lt & 15;
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = cmul(nx[m], ldtab[j + 16 * m]);
    load(nx, tn < hi ? tn : t);  // in flight during this tile's transforms and stores
    Dft<16>::run(v);
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], ldtw[r256_tw(j, k)]);
    float2* xw = xbuf + row * S;
    const int rsw = j ^ (row & 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) xw[k * 16 + (rsw ^ k)] = v[k];
    __syncthreads();
    const float2* xr = xbuf + row * S + k1 * 16;
    const int rk = k1 ^ (row & 1);
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = xr[jj ^ rk];
    Dft<16>::run(v);
    if (dc && k1 == 0) v[0] = make_float2(0.f, 0.f);  // DC removal = zero range bin 0
    __syncthreads();  // xbuf reads done: obuf aliases it
    float2* ow = obuf + row * S + k1;
#pragma unroll
    for (int k = 0; k < 16; ++k) ow[16 * k] = v[k];
    __syncthreads();
    // thread lt holds bins 2 lt, 2 lt + 1 of the 8 rows (chirps cb + 8 q): Y[k1] = W64^(cb k1) DFT8_q
    float2 y0[8], y1[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 ab = *reinterpret_cast<const float4*>(obuf + q * S + 2 * lt);
      y0[q] = make_float2(ab.x, ab.y);
      y1[q] = make_float2(ab.z, ab.w);
    }
    Dft<8>::run(y0);
    Dft<8>::run(y1);
    const int cbs = __builtin_amdgcn_readfirstlane(cb);  // the tile is workgroup-uniform
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float2 wk = tw[4 * cbs * k];  // W64^(cb k) = W256^(4 cb k), 4 cb k <= 196 (workgroup-uniform: scalar loads)
      y0[k] = cmul(y0[k], wk);
      y1[k] = cmul(y1[k], wk);
    }
    float f0[16], f1[16];
    unsigned m0 = 0u, m1 = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      f0[2 * q] = y0[q].x;
      f0[2 * q + 1] = y0[q].y;
      f1[2 * q] = y1[q].x;
      f1[2 * q + 1] = y1[q].y;
      m0 = max(m0, max(__float_as_uint(y0[q].x) & 0x7FFFFFFFu, __float_as_uint(y0[q].y) & 0x7FFFFFFFu));
      m1 = max(m1, max(__float_as_uint(y1[q].x) & 0x7FFFFFFFu, __float_as_uint(y1[q].y) & 0x7FFFFFFFu));
    }
    const int e0 = pk_exp(m0), e1 = pk_exp(m1);
    uint4 w0[3], w1[3];
    pk_pack16(f0, e0, w0);
    pk_pack16(f1, e1, w1);
    const size_t tile = (size_t)fa * ncb + cb;
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(work) + tile * kPkTile256) + lt;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      st16<true>(reinterpret_cast<float4*>(dst + jj * (kPkPlane256 / 16)), __builtin_bit_cast(float4, w0[jj]));
      st16<true>(reinterpret_cast<float4*>(dst + (jj + 3) * (kPkPlane256 / 16)), __builtin_bit_cast(float4, w1[jj]));
    }
    if (tid == 0) s_nn = lo + 2 * gx + (long)claim;
    __syncthreads();  // obuf is read above; the next tile's exchange writes overwrite it
  };
  long t = lo + (blockIdx.x >> 3), tn = t + gx;
  float2 nx[16];
  if (t < hi) load(nx, t);
  while (t < hi) {
    body(nx, t, tn);
    t = tn;
    tn = s_nn;
  }
  if (tid == 0 && atomicAdd(head + 8 * 32, 1u) == (unsigned)gx - 1u) {
    atomicExch(head, 0u);
    atomicExch(head + 8 * 32, 0u);
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
      if (pk_pow && pk) pk_pow[row * C + cnt + lanes_below(b)] = p;
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

// Stores: the shifted RDS rows are non-temporal 8-B stores (coalesced 512-B runs per wave and row; 16-B stores by a
// lane-pair DPP swap measured slower, 1.698 vs 1.677 ms per 1000 cfg2 frames); neighbour lanes and the peak-offset scan
// use DPP (wave_shr / wave_shl, row_shr / row_bcast: K2 3.52 vs 3.76 ms per 2000 cfg2 frames against ds_bpermute);
// the tile's compacted peak powers are staged in the dead LDS tile and stored block-wide (tools/pkb.sh).
// DBG (development builds only, ablations with wrong results): 4 no peak-power stores, 5 no mask / count stores,
// 8 no RDS stores, 9 RDS stores only (no detection).
// LD / PADC: the tile's row pitch and whether columns sit at padded positions lp(d) (the LDS Stockham FFT's layout) or
// at d (k_doppler_detect_r128).
// SKL: the last LDS row (NR - 1 = KB + 1, the upper halo row) starts SKL float2 after its pitch position (a bank skew of
// the caller's row writes; k_doppler_detect_r128).
// HSH: columns d >= C / 2 sit HSH float2 later in their row (k_doppler_detect_r256's bank shift).
template <int C, int KB, int NT, int DBG = 0, int LD = lp_row(C) | 1, bool PADC = true, int SKL = 0, int HSH = 0,
          bool UNI = false>
RSL_DEV void dd_tile_compute_reg(const float2* buf, float* xch, int S, int k0, unsigned fa, float2* __restrict__ rds,
                                 float thr_f, int i_lo, int i_hi, unsigned long long* __restrict__ mask,
                                 int* __restrict__ row_count, float* __restrict__ dbmap,
                                 float* __restrict__ pk_pow, int tid_in = -1) {
  constexpr int NCH = C / 64;
  // tid_in: a laundered thread index from a persistent caller (keeps per-thread addresses out of its tile loop)
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, lane = tid & 63;
  // UNI: the wave and tile indices are declared wave-uniform (readfirstlane), so the row index i, the range gate and
  // the 'reflect' edge tests below are scalar instead of per-lane compares and selects: 884 -> 796 static VALU in
  // k_doppler_detect_r128, 2.616-2.621 vs 2.640-2.642 ms per 2000 cfg2 frames (one call, outputs identical); in
  // k_doppler_detect_r256 the same change measured slower (1.164 vs 1.144 ms per 100 configs[4] frames), so it is off
  const int wave = UNI ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int ch = wave % NCH, rh = wave / NCH;
  const int j = ch * 64 + lane;  // shifted Doppler column: out[j] = X[(j - C//2) mod C]
  int d = j - C / 2;
  if (d < 0) d += C;
  if constexpr (UNI) {  // tile-uniform (the callers' tile math reaches here as vector values)
    fa = __builtin_amdgcn_readfirstlane(fa);
    k0 = __builtin_amdgcn_readfirstlane(k0);
  }
  int i0 = k0 + S / 2;  // shifted range row of LDS row 1
  if (i0 >= S) i0 -= S;
  const int rb = rh * 8;  // LDS rows rb .. rb + 9; interior rows rb + 1 .. rb + 8
  float p[10];
  const float2* col = buf + (PADC ? lp(d) : d + (d >= C / 2 ? HSH : 0));
  float2* dst = rds + ((size_t)fa * S + i0 + rb) * C + j;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const float2 z = col[(rb + r) * LD + ((SKL != 0 && r == 9 && rb + r == KB + 1) ? SKL : 0)];
    p[r] = cabs2(z);
    if (DBG != 8 && r >= 1 && r <= 8) st8<true>(dst + (size_t)(r - 1) * C, z);  // DBG 8: no RDS stores
  }
  if constexpr (DBG == 9) {  // DBG 9: RDS stores only, no detection
    if (p[0] == 1.2345e30f) mask[tid] = 0ull;
    return;
  }
  float vm[8];
  if (i0 + rb > 0 && i0 + rb + 8 < S) {  // no row of this wave at a shifted range edge (30 of 32 tiles at cfg2)
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) vm[rr] = fmaxf(fmaxf(p[rr], p[rr + 1]), p[rr + 2]);  // v_max3_f32
  } else {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int i = i0 + rb + rr;
      float m = p[rr + 1];
      if (i > 0) m = fmaxf(m, p[rr]);          // 'reflect' at the shifted range edges: no neighbour
      if (i + 1 < S) m = fmaxf(m, p[rr + 2]);
      vm[rr] = m;
    }
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
    float l = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(vm[rr]), 0x138, 0xF, 0xF, false));
    float r = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(vm[rr]), 0x130, 0xF, 0xF, false));
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
  const int incl = wave_incl_scan(cw);
  const int excl = incl - cw;
  float* tile_pk = pk_pow ? pk_pow + ((size_t)fa * S + i0) * C : nullptr;
  {
    // stage the tile's compacted peak powers in the (now dead) LDS tile, then one block-wide contiguous store of the
    // whole run instead of 8 partial-line stores per wave
    float* stg = reinterpret_cast<float*>(const_cast<float2*>(buf));
    const int total = __builtin_amdgcn_readlane(incl, 63);
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int off = __builtin_amdgcn_readlane(excl, (rb + rr) * NCH + ch);
      if (pkv[rr]) stg[off + lanes_below(bal[rr])] = p[rr + 1];
    }
    __syncthreads();
    if (DBG != 4 && tile_pk)
      for (int k = tid; k < total; k += NT) tile_pk[k] = stg[k];
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
template <int C, int KB, int NT, bool PAD, int DBG = 0>
__global__ __launch_bounds__(NT) void k_doppler_detect(const float2* __restrict__ work, int S,
                                                       const float2* __restrict__ tw, float2* __restrict__ rds,
                                                       float thr_f, int i_lo, int i_hi,
                                                       unsigned long long* __restrict__ mask,
                                                       int* __restrict__ row_count, float* __restrict__ dbmap,
                                                       float* __restrict__ pk_pow,
                                                       const unsigned char* __restrict__ wexp) {
  constexpr int NR = KB + 2;
  constexpr int LD = lp_rowp<PAD>(C) | 1;  // odd: conflict-free transposed (column) writes
  constexpr int PER = (NR * C + NT - 1) / NT;
  extern __shared__ float2 sm[];
  float2* tws = sm;
  float2* buf = sm + C;
  const int tid = threadIdx.x;
  const unsigned nkb = (unsigned)(S / KB);
  // XCD-grouped tile order: neighbouring tiles (which share halo cache lines) meet in one L2
  const unsigned tile = (unsigned)xcd_tile(blockIdx.x, gridDim.x);
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
  if constexpr (STRUCT) {
    constexpr int PI = C / CS, PH = (2 * C + NT - 1) / NT;
    const int ri = tid % KB, cs = tid / KB;
    float2 ld[PI + PH];
    const float2* p = src + (unsigned)(cs * S + k0 + ri);
#pragma unroll
    for (int q = 0; q < PI; ++q) ld[q] = DBG == 6 ? make_float2((float)tid, (float)q) : p[(unsigned)(q * CS * S)];
    int kl = k0 - 1, kh = k0 + KB;  // halo range bins (periodic: reflect is applied in the detect stage)
    if (kl < 0) kl += S;
    if (kh >= S) kh -= S;
#pragma unroll
    for (int h = 0; h < PH; ++h) {
      const int e = tid + h * NT;
      if ((2 * C) % NT == 0 || e < 2 * C) {
        const int side = e / C, c = e - side * C;
        ld[PI + h] = DBG == 6 ? make_float2((float)c, (float)h) : src[(unsigned)(c * S + (side ? kh : kl))];
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
  if constexpr (DBG == 7) {  // loads and LDS staging only
    if (buf[tid].x == 1.2345e30f) rds[tid] = buf[tid];
    return;
  }
  if constexpr (PAD && (DBG == 0 || DBG >= 4) && dd_reg_ok<C, KB, NT>()) {
    fft_rows<C, NR, NT, LD, false, PAD>(buf, tws, tid);
    dd_tile_compute_reg<C, KB, NT, DBG>(buf, reinterpret_cast<float*>(buf + NR * LD), S, k0, fa, rds, thr_f, i_lo, i_hi,
                                   mask, row_count, dbmap, pk_pow);
  } else {
    dd_tile_compute<C, KB, NT, PAD, DBG>(buf, tws, S, k0, fa, rds, thr_f, i_lo, i_hi, mask, row_count, dbmap,
                                         pk_pow);
  }
}

// K2 + K3 for C = 128 with packed `work` (the cfg2 shape): the Doppler FFT as 8 x 16 in registers.  K1 stores chirp
// class c (chirps c + 16 r, r < 8) as one packed tile after the first radix-8 step, Y'_c[k1] = W128^(c k1) DFT8_r
// x[c + 16 r] (k_range_fft_r512), so thread (bin b, class c) = (tid % 16, tid / 16) loads the 8 values of its bin
// (3 x 16 B) and
//   exchange: Y' -> xi[c][k1][b] (interior bins, 128 float2 per class) and, from threads 0-31, the two halo bins'
//   values -> xh[c][k1][side] (17 float2 per class);
//   stage 2: thread t < 128 = (k1 = t / 16, b = t % 16) reads xi[c][k1][b], threads 128-143 = (k1, side) read
//   xh[c][k1][side], for c < 16 (consecutive per instruction); X[k1 + 8 k2] = DFT16_c (registers), written to tile row
//   b2 (b + 1, or the halo rows 0 / 17) at the unshifted Doppler position;
// then the register-form detection (dd_tile_compute_reg) as in k_doppler_detect.  X[k1 + 8 k2] = sum_c W128^(c k1)
// W16^(c k2) sum_r x[c + 16 r] W8^(r k1): the 128-point DFT exactly.  Against the LDS Stockham form (staging + two
// stage passes) a third less LDS traffic.  DBG (development builds only): 6 no work loads, 7 loads only.
// LDS banks (MI355X_MICROARCH §LDS; ds_write_b64: 16-lane groups, bank = dword mod 32; ds_read_b64: 32-lane groups,
// dword mod 64): every exchange and stage-2 access is conflict-free.  The tile rows are C + 7 float2 apart (7 b2 mod 16
// distinct over the 16 interior rows of a k1 group) and the upper halo row sits 1 float2 later (the halo group's rows
// 0 and 17 then fill banks 0-15 and 16-31).  Round 4's map (stage-2 thread t = 18 k1 + b2, rows C + 1 apart, halo
// rows inside the exchange) put (k1, 17) and (k1 + 1, 0) on one bank in 7 of the 9 write groups: 112 conflict
// cycles per tile, 28.7 M per 1000 cfg2 frames, the r4n counter's 29.2 M.
template <int DBG = 0>
__global__ __launch_bounds__(256) void k_doppler_detect_r128(const float2* __restrict__ work, int S_arg,
                                                             const float2* __restrict__ tw, float2* __restrict__ rds,
                                                             float thr_f, int i_lo, int i_hi,
                                                             unsigned long long* __restrict__ mask,
                                                             int* __restrict__ row_count, float* __restrict__ dbmap,
                                                             float* __restrict__ pk_pow,
                                                             const unsigned char* __restrict__ wexp) {
  // S = 512 wherever this kernel runs (work_packed_supported): the tile index math folds to shifts and masks instead of
  // a runtime 32-bit division (≈ 200 SALU per wave before)
  constexpr int KB = 16, C = 128, S = 512, NT = 16 * KB, NR = KB + 2, NCB = 16;
  (void)S_arg;
  (void)tw;
  (void)wexp;  // the exponents travel inside the packed units (pk_unpack16)
  constexpr int LD = kR128Pitch, SKL = kR128Skew;
  constexpr int XPI = 8 * KB, XPH = 17;  // exchange float2 per class: interior [k1][b], halo [k1][side] + 1 pad
  static_assert(NCB * (XPI + XPH) <= NR * LD, "exchange buffer must fit in the tile buffer");
  extern __shared__ float2 sm[];
  float2* buf = sm;
  float2* xi = buf;               // exchange, then the tile rows (aliased: a barrier separates the last read from the
  float2* xh = buf + NCB * XPI;   // first write)
  const int tid = threadIdx.x;
  constexpr unsigned nkb = (unsigned)(S / KB);
  const unsigned tile = (unsigned)__builtin_amdgcn_readfirstlane((int)xcd_tile(blockIdx.x, gridDim.x));
  const unsigned char* wb = reinterpret_cast<const unsigned char*>(work);
  auto unit = [&](size_t tile0, int k, int cls, uint4(&w)[3]) {
    const uint4* src =
        reinterpret_cast<const uint4*>(wb + (tile0 + cls) * kPkTile + (size_t)(3 * (k & 1)) * kPkPlane) + (k >> 1);
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      if constexpr (DBG == 6)
        w[jj] = make_uint4(0x4B4000u + tid, 0x5Au * jj, 0x4B40u + k, 0x12345u);
      else
        w[jj] = src[jj * (kPkPlane / 16)];
    }
  };
  const int b = tid % KB, cls = tid / KB;
  const bool halo = tid < 2 * NCB;  // threads 0-31: (side, class) = (tid / 16, tid % 16)
  const int hside = tid >> 4, hcls = tid & 15;
  const int k0 = (int)(tile % nkb) * KB;
  const unsigned fa = tile / nkb;
  const size_t tile0 = (size_t)fa * NCB;
  // every load issued before the first LDS write
  uint4 wi[3], wh[3];
  unit(tile0, k0 + b, cls, wi);
  if (halo) {
    int kk = hside ? k0 + KB : k0 - 1;  // periodic: 'reflect' is applied in the detect stage
    kk = kk < 0 ? kk + S : (kk >= S ? kk - S : kk);
    unit(tile0, kk, hcls, wh);
  }
  if constexpr (DBG == 7) {
    if (__uint_as_float(wi[0].x ^ wh[1].y) == 1.2345e30f) rds[tid] = make_float2((float)wi[1].z, 0.f);
    return;
  }
  // one unit (K1 stored Y'_c[k1] = W128^(c k1) DFT8_r already): decode, write its 8 values (k1 = 0..7) at stride st
  auto stage1 = [&](const uint4(&w)[3], float2* dst, int st) {
    float f[16];
    pk_unpack16(w, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k * st] = make_float2(f[2 * k], f[2 * k + 1]);
  };
  stage1(wi, xi + cls * XPI + b, KB);
  if (halo) stage1(wh, xh + hcls * XPH + hside, 2);
  __syncthreads();
  // stage 2: DFT16 over the classes
  const bool s2 = tid < 8 * NR;
  const bool hs = tid >= 8 * KB;  // threads 128-143: the halo rows
  const int k1 = hs ? (tid - 8 * KB) >> 1 : tid / KB;
  const int b2 = hs ? ((tid & 1) ? NR - 1 : 0) : (tid % KB) + 1;
  float2 x[16];
  if (s2) {
    const float2* src = hs ? xh + 2 * k1 + (tid & 1) : xi + tid;
    const int cs = hs ? XPH : XPI;
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = src[c * cs];
    Dft<16>::run(x);
  }
  __syncthreads();  // exchange reads done: the tile rows alias it
  if (s2) {
    float2* row = buf + b2 * LD + (b2 == NR - 1 ? SKL : 0);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) row[k1 + 8 * k2] = x[k2];
  }
  __syncthreads();
  dd_tile_compute_reg<C, KB, NT, (DBG == 4 || DBG == 5 || DBG == 8 || DBG == 9) ? DBG : 0, LD, false, SKL, 0, true>(
      buf, reinterpret_cast<float*>(buf + NR * LD), S, k0, fa, rds, thr_f, i_lo, i_hi, mask, row_count, dbmap, pk_pow);
}

// K2 + K3 for C = 256, S = 1024 with packed `work` (the configs[4] shape; K1 = k_range_fft_r1024): the Doppler FFT
// as 8 x 32.  K1 stored chirp class c (chirps c + 32 r, r < 8) after the radix-8 step, Y'_c[k1] = W256^(c k1) DFT8_r,
// so thread (bin b, class c) = (tid % 16, tid / 16) loads its bin's unit (3 x 16 B) and
//   exchange: Y' -> xi[c][(16 k1 + b) ^ 16 (c & 1)] (interior bins) and, from threads 0-63, the halo bins' values
//   -> xh[c][(2 k1 + side) ^ (c & 15)];
//   stage 2: lane (k1, b2, h) takes the classes c = 2 i + h: E or O = DFT16_i (registers), then the lane pair (h = 0, 1)
//   forms X[k1 + 8 k'] = E + W32^k' O and X[k1 + 8 (k' + 16)] = E - W32^k' O by one DPP swap (as K1's radix-2 step at
//   S = 512); 256 lanes for the 16 interior bins, 32 for the two halo bins;
//   tile rows: X -> row b2 at the unshifted Doppler position d, columns d >= 128 one float2 later (HSH = 1) and the
//   upper halo row 1 float2 later (SKL): every exchange and row access is bank-conflict-free except the halo rows';
// then the register-form detection (dd_tile_compute_reg, 16 rows x 4 column waves).  X[k1 + 8 k2] = sum_c W256^(c k1)
// W32^(c k2) sum_r x[c + 32 r] W8^(r k1): the 256-point DFT exactly.  16 bins x 256 chirps on 512 threads, 37 KiB of
// LDS: 4 workgroups (32 waves) per CU.  DBG (development builds only): 6 no work loads, 7 loads only.
constexpr int kR256Pitch = 258;  // tile row pitch (float2): 256 columns + the HSH shift + 1 (516 b2 = 4 b2 mod 32 dwords)
// upper halo row: 6 float2 later, i.e. at 8 mod 16 positions (2 + 6) from row 0, so that each 16-lane group of the
// halo wave's row writes (k1 of one parity x both sides x both h) covers 16 distinct bank pairs (skew 1 with k1 = u / 4:
// 2- to 3-way on all 16 writes, ~76 of the 7.8 M conflict cycles per tile of 100 configs[4] frames, gpurun_out/r5aa_ddctr5)
constexpr int kR256Skew = 6;
constexpr int kR256Gap = 8;  // float2 between the tile rows (+ the skew's overhang) and the detection exchange words
template <int DBG = 0>
__global__ __launch_bounds__(512) void k_doppler_detect_r256(const float2* __restrict__ work, int S_arg,
                                                             const float2* __restrict__ tw, float2* __restrict__ rds,
                                                             float thr_f, int i_lo, int i_hi,
                                                             unsigned long long* __restrict__ mask,
                                                             int* __restrict__ row_count, float* __restrict__ dbmap,
                                                             float* __restrict__ pk_pow,
                                                             const unsigned char* __restrict__ wexp) {
  constexpr int KB = 16, C = 256, S = 1024, NT = 512, NR = KB + 2, NCB = 32;
  (void)S_arg;
  (void)tw;
  (void)wexp;
  constexpr int LD = kR256Pitch, SKL = kR256Skew, HSH = 1;
  constexpr int XPI = 8 * KB, XPH = 16;  // exchange float2 per class: interior [k1][b] (swizzled), halo [k1][side]
  static_assert(NCB * (XPI + XPH) <= NR * LD, "exchange buffer must fit in the tile buffer");
  extern __shared__ float2 sm[];
  float2* buf = sm;
  float2* xi = buf;
  float2* xh = buf + NCB * XPI;
  const int tid = threadIdx.x;
  constexpr unsigned nkb = (unsigned)(S / KB);
  const unsigned tile = (unsigned)xcd_tile(blockIdx.x, gridDim.x);
  const unsigned char* wb = reinterpret_cast<const unsigned char*>(work);
  auto unit = [&](size_t tile0, int k, int cls, uint4(&w)[3]) {
    const uint4* src = reinterpret_cast<const uint4*>(wb + (tile0 + cls) * kPkTile1k +
                                                      (size_t)(3 * (k & 1)) * kPkPlane1k) + (k >> 1);
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      if constexpr (DBG == 6)
        w[jj] = make_uint4(0x4B4000u + tid, 0x5Au * jj, 0x4B40u + k, 0x12345u);
      else
        w[jj] = src[jj * (kPkPlane1k / 16)];
    }
  };
  const int b = tid % KB, cls = tid / KB;
  const bool halo = tid < 2 * NCB;  // threads 0-63: (side, class) = (tid / 32, tid % 32)
  const int hside = tid >> 5, hcls = tid & 31;
  const int k0 = (int)(tile % nkb) * KB;
  const unsigned fa = tile / nkb;
  const size_t tile0 = (size_t)fa * NCB;
  uint4 wi[3], wh[3] = {};
  unit(tile0, k0 + b, cls, wi);
  if (halo) {
    int kk = hside ? k0 + KB : k0 - 1;  // periodic: 'reflect' is applied in the detect stage
    kk = kk < 0 ? kk + S : (kk >= S ? kk - S : kk);
    unit(tile0, kk, hcls, wh);
  }
  if constexpr (DBG == 7) {
    if (__uint_as_float(wi[0].x ^ wh[1].y) == 1.2345e30f) rds[tid] = make_float2((float)wi[1].z, 0.f);
    return;
  }
  {
    float f[16];
    pk_unpack16(wi, f);
    float2* d = xi + cls * XPI;
    const int sw = 16 * (cls & 1);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[(16 * k + b) ^ sw] = make_float2(f[2 * k], f[2 * k + 1]);
  }
  if (halo) {
    float f[16];
    pk_unpack16(wh, f);
    float2* d = xh + hcls * XPH;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[(2 * k + hside) ^ (hcls & 15)] = make_float2(f[2 * k], f[2 * k + 1]);
  }
  __syncthreads();
  // stage 2: DFT32 over the classes as two DFT16 (c = 2 i + h) and one radix-2 step across the lane pair
  const bool s2 = tid < 8 * KB * 2 + 32;
  const bool hs = tid >= 8 * KB * 2;  // threads 256-287: the halo rows
  const int u = tid - 8 * KB * 2;
  const int hh = tid & 1;
  const int k1 = hs ? 2 * ((u >> 2) & 3) + ((u >> 4) & 1) : (tid >> 5);  // halo: one k1 parity per 16-lane group
  const int side = (u >> 1) & 1;
  const int bi = (tid >> 1) & 15;
  const int b2 = hs ? (side ? NR - 1 : 0) : bi + 1;
  float2 x[16];  // defined on the stage-2 lanes only: every use below is under s2
  if (s2) {
    // hs is wave-uniform (waves 0-3: interior lanes only; wave 4: halo lanes 0-31, lanes 32-63 idle): a scalar branch,
    // so that each path's 16 reads are one base address plus immediate offsets instead of both address forms and a
    // select per read
    if (__builtin_amdgcn_readfirstlane((int)hs)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = 2 * i + hh;
        x[i] = xh[c * XPH + ((2 * k1 + side) ^ (c & 15))];
      }
    } else {
      const float2* xb = xi + hh * XPI + ((16 * k1 + bi) ^ (16 * hh));
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = xb[2 * i * XPI];
    }
    Dft<16>::run(x);
  }
  __syncthreads();  // exchange reads done: the tile rows alias it (each output is written as it forms)
  // the radix-2 step under s2 as a whole: waves 5-7 hold no stage-2 lane and skip it (they issued its ~175 VALU for
  // nothing before); the lane pairs (h = 0, 1) of the DPP swap are both inside or both outside s2
  if (s2) {
    const float sg = hh ? -1.f : 1.f;
    float2* rw = buf + b2 * LD + (b2 == NR - 1 ? SKL : 0) + k1 + (C / 2 + HSH) * hh;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float2 uu = hh ? cmul(x[k], w32(k)) : x[k];
      float2 r;
      r.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(uu.x), 0xB1, 0xF, 0xF, true));
      r.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(uu.y), 0xB1, 0xF, 0xF, true));
      rw[8 * k] = make_float2(fmaf(sg, uu.x, r.x), fmaf(sg, uu.y, r.y));
    }
  }
  __syncthreads();
  dd_tile_compute_reg<C, KB, NT, (DBG == 4 || DBG == 5 || DBG == 8 || DBG == 9) ? DBG : 0, LD, false, SKL, HSH>(
      buf, reinterpret_cast<float*>(buf + NR * LD + kR256Gap), S, k0, fa, rds, thr_f, i_lo, i_hi, mask, row_count, dbmap, pk_pow);
}

// K2 + K3 for C = 64, S = 256 with packed `work` (the cfg1 shape; K1 = k_range_fft_r256): the Doppler FFT as 8 x 8.
// K1 stored chirp class c (chirps c + 8 r, r < 8) after the radix-8 step, Y'_c[k1] = W64^(c k1) DFT8_r, so thread
// (bin b, class c) = (tid % 32, tid / 32) loads its bin's unit (3 x 16 B) and decodes it into xi[c][k1][b] (every 16th
// thread a halo unit into xh[c][k1][side]); lane (k1, b) then takes X[k1 + 8 k2] = DFT8_c (registers) for its interior
// bin and threads 0-15 the halo bins' transforms, each written to its tile row (rows C + 1 apart: conflict-free); the
// register-form detection (one column wave x 4 row quarters) follows.  32 bins x 64 chirps on 256 threads, 18 KiB LDS.
template <int DBG = 0>
__global__ __launch_bounds__(256) void k_doppler_detect_r64(const float2* __restrict__ work, int S_arg,
                                                            const float2* __restrict__ tw, float2* __restrict__ rds,
                                                            float thr_f, int i_lo, int i_hi,
                                                            unsigned long long* __restrict__ mask,
                                                            int* __restrict__ row_count, float* __restrict__ dbmap,
                                                            float* __restrict__ pk_pow,
                                                            const unsigned char* __restrict__ wexp) {
  constexpr int KB = 32, C = 64, S = 256, NT = 256, NR = KB + 2, NCB = 8;
  (void)S_arg;
  (void)tw;
  (void)wexp;
  constexpr int LD = C + 1;
  constexpr int XPI = 8 * KB, XPH = 16;  // exchange float2 per class: interior [k1][b], halo [k1][side]
  static_assert(NCB * (XPI + XPH) <= NR * LD, "exchange buffer must fit in the tile buffer");
  extern __shared__ float2 sm[];
  float2* buf = sm;
  float2* xi = buf;
  float2* xh = buf + NCB * XPI;
  const int tid = threadIdx.x;
  constexpr unsigned nkb = (unsigned)(S / KB);
  const unsigned tile = (unsigned)xcd_tile(blockIdx.x, gridDim.x);
  const unsigned char* wb = reinterpret_cast<const unsigned char*>(work);
  auto unit = [&](size_t tile0, int k, int cls, uint4(&w)[3]) {
    const uint4* src = reinterpret_cast<const uint4*>(wb + (tile0 + cls) * kPkTile256 +
                                                      (size_t)(3 * (k & 1)) * kPkPlane256) + (k >> 1);
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      if constexpr (DBG == 6)
        w[jj] = make_uint4(0x4B4000u + tid, 0x5Au * jj, 0x4B40u + k, 0x12345u);
      else
        w[jj] = src[jj * (kPkPlane256 / 16)];
    }
  };
  const int b = tid % KB, cls = tid / KB;
  const bool halo = (tid & 15) == 0;  // 16 halo units, one per 16 threads: (side, class) = (h / 8, h % 8), h = tid / 16
  const int hside = tid >> 7, hcls = (tid >> 4) & 7;
  const int k0 = (int)(tile % nkb) * KB;
  const unsigned fa = tile / nkb;
  const size_t tile0 = (size_t)fa * NCB;
  uint4 wi[3], wh[3] = {};
  unit(tile0, k0 + b, cls, wi);
  if (halo) {
    int kk = hside ? k0 + KB : k0 - 1;  // periodic: 'reflect' is applied in the detect stage
    kk = kk < 0 ? kk + S : (kk >= S ? kk - S : kk);
    unit(tile0, kk, hcls, wh);
  }
  {
    float f[16];
    pk_unpack16(wi, f);
    float2* d = xi + cls * XPI + b;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k * KB] = make_float2(f[2 * k], f[2 * k + 1]);
  }
  if (halo) {
    float f[16];
    pk_unpack16(wh, f);
    float2* d = xh + hcls * XPH + hside;
#pragma unroll
    for (int k = 0; k < 8; ++k) d[2 * k] = make_float2(f[2 * k], f[2 * k + 1]);
  }
  __syncthreads();
  // stage 2: DFT8 over the classes; lane (k1, b) = (tid / 32, tid % 32) for the interior bins, threads 0-15 also
  // (k1, side) = (tid / 2, tid % 2) for the halo bins
  const int k1 = tid / KB;
  float2 x[8], y[8] = {};
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = xi[c * XPI + k1 * KB + b];
  Dft<8>::run(x);
  const bool hs = tid < 16;
  const int hk1 = tid >> 1, hsd = tid & 1;
  if (hs) {
#pragma unroll
    for (int c = 0; c < 8; ++c) y[c] = xh[c * XPH + 2 * hk1 + hsd];
    Dft<8>::run(y);
  }
  __syncthreads();  // exchange reads done: the tile rows alias it
  {
    float2* rw = buf + (b + 1) * LD + k1;
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) rw[8 * k2] = x[k2];
  }
  if (hs) {
    float2* rw = buf + (hsd ? NR - 1 : 0) * LD + hk1;
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) rw[8 * k2] = y[k2];
  }
  __syncthreads();
  dd_tile_compute_reg<C, KB, NT, (DBG == 4 || DBG == 5 || DBG == 8 || DBG == 9) ? DBG : 0, LD, false>(
      buf, reinterpret_cast<float*>(buf + NR * LD), S, k0, fa, rds, thr_f, i_lo, i_hi, mask, row_count, dbmap, pk_pow);
}

static hipError_t launch_k2d_r64(hipStream_t st, const float2* work, int F, int A, int S, float2* rds, double thr_p,
                                 int i_lo, int i_hi, unsigned long long* mask, int* row_count, float* dbmap,
                                 float* pk_pow, int* pk_group, const unsigned char* wexp) {
  constexpr int C = 64, KB = 32, NT = 256;
  static_assert(dd_reg_ok<C, KB, NT>(), "register tile body shape");
  if (S != 256) return hipErrorInvalidValue;  // the kernel's tile math is compiled for S = 256
  const long ntile = (long)F * A * (S / KB);
  const size_t lds = sizeof(float2) * (size_t)(KB + 2) * (C + 1) + (size_t)KB * (C / 64) * 16;
  auto kern = k_doppler_detect_r64<>;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_DD_DBG")) {  // ablation variants (development builds only; results are wrong)
    const int v = atoi(e);
    if (v == 6) kern = k_doppler_detect_r64<6>;
    if (v == 8) kern = k_doppler_detect_r64<8>;
  }
#endif
  *pk_group = KB;
  hipLaunchKernelGGL(kern, dim3((unsigned)ntile), dim3(NT), lds, st, work, S, nullptr, rds, threshold_as_float(thr_p),
                     i_lo, i_hi, mask, row_count, dbmap, pk_pow, wexp);
  return hipGetLastError();
}

static hipError_t launch_k2d_r256(hipStream_t st, const float2* work, int F, int A, int S, float2* rds, double thr_p,
                                  int i_lo, int i_hi, unsigned long long* mask, int* row_count, float* dbmap,
                                  float* pk_pow, int* pk_group, const unsigned char* wexp) {
  constexpr int C = 256, KB = 16, NT = 512;
  static_assert(dd_reg_ok<C, KB, NT>(), "register tile body shape");
  if (S != 1024) return hipErrorInvalidValue;  // the kernel's tile math is compiled for S = 1024
  const long ntile = (long)F * A * (S / KB);
  const size_t lds = sizeof(float2) * ((size_t)(KB + 2) * kR256Pitch + kR256Gap) + (size_t)KB * (C / 64) * 16;
  auto kern = k_doppler_detect_r256<>;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_DD_DBG")) {  // ablation variants (development builds only; results are wrong)
    const int v = atoi(e);
    if (v == 6) kern = k_doppler_detect_r256<6>;
    if (v == 7) kern = k_doppler_detect_r256<7>;
    if (v == 8) kern = k_doppler_detect_r256<8>;
  }
#endif
  *pk_group = KB;
  hipLaunchKernelGGL(kern, dim3((unsigned)ntile), dim3(NT), lds, st, work, S, nullptr, rds, threshold_as_float(thr_p),
                     i_lo, i_hi, mask, row_count, dbmap, pk_pow, wexp);
  return hipGetLastError();
}

template <int C, int KB>
static hipError_t launch_k2d_kb(hipStream_t st, const float2* work, int F, int A, int S, const float2* tw,
                                float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask,
                                int* row_count, float* dbmap, float* pk_pow, int* pk_group,
                                const unsigned char* wexp) {
  constexpr int NT = 256;
  const long ntile = (long)F * A * (S / KB);
  // padded LDS rows (plain rows measured slower: 2.14 vs 1.98 ms per 1000 cfg2 frames) + the register body's exchange
  // area (edge columns and ballots: 16 B per row per 64 columns)
  const size_t lds = sizeof(float2) * (C + (size_t)(KB + 2) * (lp_row(C) | 1)) + (size_t)KB * (C / 64) * 16;
  const float thr_f = threshold_as_float(thr_p);
  // One tile per workgroup, 256 threads.  Measured and not kept: a persistent variant with a register prefetch of the
  // next tile (5.0-5.25 vs 3.85 ms per 2000 cfg2 frames), a 320-thread block (2.72 vs 2.48 ms per 1000 frames).
  auto kern = k_doppler_detect<C, KB, NT, true>;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_DD_DBG")) {  // ablation variants (development builds only; results are wrong)
    const int v = atoi(e);
    if (v == 1) kern = k_doppler_detect<C, KB, NT, true, 1>;
    if (v == 2) kern = k_doppler_detect<C, KB, NT, true, 2>;
    if (v == 3) kern = k_doppler_detect<C, KB, NT, true, 3>;
    if (v == 4) kern = k_doppler_detect<C, KB, NT, true, 4>;
    if (v == 5) kern = k_doppler_detect<C, KB, NT, true, 5>;
    if (v == 6) kern = k_doppler_detect<C, KB, NT, true, 6>;
    if (v == 7) kern = k_doppler_detect<C, KB, NT, true, 7>;
  }
#endif
  // tile-compact peak powers from the register tile body (KB rows per group), row-compact from the general body
  *pk_group = dd_reg_ok<C, KB, NT>() ? KB : 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)ntile), dim3(NT), lds, st, work, S, tw, rds, thr_f, i_lo, i_hi, mask,
                     row_count, dbmap, pk_pow, wexp);
  return hipGetLastError();
}

// range bins per Doppler/detect tile: ~20 KiB tiles (KB 16 at C = 128: 2.42 ms vs KB 32: 3.23 ms per 1000 cfg2
// frames; more resident workgroups hide the per-tile load -> FFT -> store phases), rows_for(C) where that does not
// tile S / 2
static int dd_kb(int C, int S) {
  int kb = 2048 / C < 1 ? 1 : 2048 / C;
  if (kb > rows_for(C) || (S / 2) % kb != 0 || S % kb != 0) kb = rows_for(C);
  return kb;
}

// K2 + K3 on packed work (work_packed_supported: C = 128, S = 512), k_doppler_detect_r128 (16 range bins per tile:
// 2.59 ms per 2000 cfg2 frames against 2.67 for 32 on 512 threads, and 3.10 for two tiles per workgroup; round 3).
static hipError_t launch_k2d_r128(hipStream_t st, const float2* work, int F, int A, int S, float2* rds, double thr_p,
                                  int i_lo, int i_hi, unsigned long long* mask, int* row_count, float* dbmap,
                                  float* pk_pow, int* pk_group, const unsigned char* wexp) {
  constexpr int C = 128, KR = 16, NT = 16 * KR;
  static_assert(dd_reg_ok<C, KR, NT>(), "register tile body shape");
  if (S != 512) return hipErrorInvalidValue;  // the kernel's tile math is compiled for S = 512 (work_packed_supported)
  const long ntile = (long)F * A * (S / KR);
  // the tile rows (the upper halo row skewed inside its pitch) + the register body's exchange area (edge columns and
  // ballots: 16 B per row per 64 columns): 19,952 B, 8 workgroups per CU
  const size_t lds = sizeof(float2) * (size_t)(KR + 2) * kR128Pitch + (size_t)KR * (C / 64) * 16;
  const float thr_f = threshold_as_float(thr_p);
  auto kern = k_doppler_detect_r128<>;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_DD_DBG")) {  // ablation variants (development builds only; results are wrong)
    const int v = atoi(e);
    if (v == 4) kern = k_doppler_detect_r128<4>;
    if (v == 5) kern = k_doppler_detect_r128<5>;
    if (v == 6) kern = k_doppler_detect_r128<6>;
    if (v == 7) kern = k_doppler_detect_r128<7>;
    if (v == 8) kern = k_doppler_detect_r128<8>;
    if (v == 9) kern = k_doppler_detect_r128<9>;
  }
#endif
  *pk_group = KR;  // tile-compact peak powers (dd_tile_compute_reg)
  hipLaunchKernelGGL(kern, dim3((unsigned)ntile), dim3(NT), lds, st, work, S, nullptr, rds, thr_f, i_lo, i_hi, mask,
                     row_count, dbmap, pk_pow, wexp);
  return hipGetLastError();
}


template <int C>
static hipError_t launch_k2d(hipStream_t st, const float2* work, int F, int A, int S, const float2* tw, float2* rds,
                             double thr_p, int i_lo, int i_hi, unsigned long long* mask, int* row_count, float* dbmap,
                             float* pk_pow, int* pk_group, const unsigned char* wexp) {
  if constexpr (C == 128) {
    if (wexp)
      return launch_k2d_r128(st, work, F, A, S, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group, wexp);
  }
  if constexpr (C == 256) {
    if (wexp)
      return launch_k2d_r256(st, work, F, A, S, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group, wexp);
  }
  if constexpr (C == 64) {
    if (wexp)
      return launch_k2d_r64(st, work, F, A, S, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group, wexp);
  }
  constexpr int K0 = rows_for(C);
  constexpr int K1 = (2048 / C) < 1 ? 1 : (2048 / C) > K0 ? K0 : (2048 / C);
  if (dd_kb(C, S) == K1)
    return launch_k2d_kb<C, K1>(st, work, F, A, S, tw, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group,
                                wexp);
  return launch_k2d_kb<C, K0>(st, work, F, A, S, tw, rds, thr_p, i_lo, i_hi, mask, row_count, dbmap, pk_pow, pk_group,
                              wexp);
}

// K1 at S = 1024 on packed work (work_packed_supported): k_range_fft_r1024, one tile per (frame, antenna, class).
static hipError_t launch_k1_r1024(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C,
                                  const float2* table, const float2* tw, int dc, float2* work, unsigned char* wexp,
                                  RfQueues* qs) {
  if (C != 256) return hipErrorInvalidValue;  // its chirp-class tiles are compiled for C = 256
  const long ntile = (long)F * A * 32;
  if (ntile >= (1L << 31)) return hipErrorInvalidValue;  // the kernel's tile indices are 32-bit (readfirstlane)
  auto kern = k_range_fft_r1024<true>;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_RF_DBG")) {  // ablation (development builds only; results are wrong)
    const int v = atoi(e);
    if (v == 2) kern = k_range_fft_r1024<true, 2>;
    if (v == 3) kern = k_range_fft_r1024<true, 3>;
  }
#endif
  // ntile >= 32 (A >= 1, 32 classes) and every CU holds two workgroups: the grid always spans the 8 XCDs, so the
  // per-XCD dequeue always applies (no static-walk instance)
  const long nblk = resident_grid(reinterpret_cast<const void*>(kern), 0, ntile, kR1kThreads);
  if (nblk < 8) return hipErrorInvalidValue;
  unsigned* rfq = nullptr;
  if (hipError_t qe = rf_queue(qs, st, &rfq)) return qe;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(kR1kThreads), 0, st, cube, A, Ct, c0, C, ntile, table, tw, dc,
                     work, rfq, wexp);
  return hipGetLastError();
}

// K1 at S = 256 on packed work (work_packed_supported): k_range_fft_r256, one tile per (frame, antenna, class).
static hipError_t launch_k1_r256(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C,
                                 const float2* table, const float2* tw, int dc, float2* work, unsigned char* wexp,
                                 RfQueues* qs) {
  if (C != 64) return hipErrorInvalidValue;  // its chirp-class tiles are compiled for C = 64
  const long ntile = (long)F * A * 8;
  if (ntile >= (1L << 31)) return hipErrorInvalidValue;  // the kernel's tile indices are 32-bit (readfirstlane)
  auto kern = k_range_fft_r256<>;
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_RF_DBG"))  // ablation (development builds only; results are wrong)
    if (atoi(e) == 2) kern = k_range_fft_r256<2>;
#endif
  // the per-XCD dequeue needs a workgroup on every XCD: tiny batches (F A < 1) do not occur (ntile >= 8)
  const long nblk = resident_grid(reinterpret_cast<const void*>(kern), 0, ntile, kR256Threads);
  if (nblk < 8) return hipErrorInvalidValue;
  unsigned* rfq = nullptr;
  if (hipError_t qe = rf_queue(qs, st, &rfq)) return qe;
  hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(kR256Threads), 0, st, cube, A, Ct, c0, C, ntile, table, tw, dc,
                     work, rfq, wexp);
  return hipGetLastError();
}

template <int S>
static hipError_t launch_k1(hipStream_t st, const float2* cube, int F, int A, int Ct, int c0, int C,
                            const float2* table, const float2* tw, int dc, float2* work, unsigned char* wexp,
                            RfQueues* qs) {
  if constexpr (S == 1024) {
    if (wexp) return launch_k1_r1024(st, cube, F, A, Ct, c0, C, table, tw, dc, work, wexp, qs);
  }
  if constexpr (S == 256) {
    if (wexp) return launch_k1_r256(st, cube, F, A, Ct, c0, C, table, tw, dc, work, wexp, qs);
  }
  constexpr int CB = rows_for(S);
  if constexpr (S % 2 == 0 && (CB * (S / 2)) % kThreads == 0) {
    // 8 chirp rows per tile at S = 512: 16 rows (78 KiB LDS) is faster alone (1.53 vs 1.63 ms per 1000 cfg2 frames)
    // but leaves no LDS for the previous batch's DoA blocks in the pipelined chain (153 k vs 171 k frames/s)
    const long ntile = (long)F * A * ((C + CB - 1) / CB);
    if (ntile >= (1L << 31)) return hipErrorInvalidValue;  // 32-bit tile indices in the tile kernels (readfirstlane)
    const size_t lds = sizeof(float2) * (lp_row(S) + (size_t)CB * lp_row(S));
    auto kern = k_range_fft_p<S, CB, true>;
    size_t lds_k = lds;
    if constexpr (S == 512 && CB == 8) {
      if (wexp) {  // packed work (work_packed_supported): the register-form 16 x 32 transform
        if (C != 128) return hipErrorInvalidValue;  // its chirp-class tiles are compiled for C = 128
        kern = k_range_fft_r512<true>;
        lds_k = 0;  // static LDS only
      }
    }
#ifdef RSL_DEV_KNOBS
    if constexpr (S == 512 && CB == 8) {  // RSL_WORK_TEMPORAL=1: the packed `work` stored without the nt hint (MALL study)
      if (const char* e = getenv("RSL_WORK_TEMPORAL"))
        if (wexp && atoi(e) == 1) kern = k_range_fft_r512<true, 0, false>;
    }
    if (const char* e = getenv("RSL_RF_DBG")) {  // ablation (development builds only; results are wrong)
      const int v = atoi(e);
      if constexpr (S == 512 && CB == 8) {
        if (wexp && v == 2) kern = k_range_fft_r512<true, 2>;
        if (wexp && v == 3) kern = k_range_fft_r512<true, 3>;
      }
      if (!wexp && v == 1) kern = k_range_fft_p<S, CB, true, 1>;
      if (!wexp && v == 2) kern = k_range_fft_p<S, CB, true, 2>;
      if (!wexp && v == 3) kern = k_range_fft_p<S, CB, true, 3>;
    }
#endif
    long nblk = resident_grid(reinterpret_cast<const void*>(kern), lds_k, ntile);
#ifdef RSL_DEV_KNOBS
    if (const char* e = getenv("RSL_K1_WG_PER_CU")) {  // fewer resident K1 workgroups (room for the other stream)
      int dev = 0, ncu = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      const long cap = (long)atoi(e) * ncu;
      if (cap >= 8 && cap < nblk) nblk = cap;
    }
#endif
    unsigned* rfq = nullptr;
    if (nblk >= 8) {  // the per-XCD dequeue needs a workgroup on every XCD
      if (hipError_t qe = rf_queue(qs, st, &rfq)) return qe;
    } else {
      kern = k_range_fft_p<S, CB, false>;
      if constexpr (S == 512 && CB == 8) {
        if (wexp) kern = k_range_fft_r512<false, 0, false>;  // fewer than 8 workgroups: a tiny batch
      }
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(kThreads), lds_k, st, cube, A, Ct, c0, C, ntile, table, tw,
                       dc, work, rfq, wexp);
    return hipGetLastError();
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

// Packed `work` between K1 and K2 (pk_pack16): the K1 tile holds one bin pair per thread and the K2 tile one (bin,
// chirp class) per thread, at the three shapes with register-form kernels: S = 512, C = 128 (k_range_fft_r512,
// k_doppler_detect_r128), S = 1024, C = 256 (k_range_fft_r1024, k_doppler_detect_r256) and S = 256, C = 64
// (k_range_fft_r256, k_doppler_detect_r64).  Development builds:
// RSL_WORK_C64=1 keeps c64 rows (A/B).
bool work_packed_supported(int C, int S) {
#ifdef RSL_DEV_KNOBS
  if (const char* e = getenv("RSL_WORK_C64"))
    if (atoi(e) != 0) return false;
#endif
  return ((S == 512 && C == 128) || (S == 1024 && C == 256) || (S == 256 && C == 64)) &&
         doppler_detect_supported(C, S);
}

bool doppler_detect_supported(int C, int S) {
  if (!fft_supported(C) || (C & (C - 1)) != 0 || C < 8 || C > 1024 || (S & 1)) return false;  // LDS <= 64 KiB
  const int KB = dd_kb(C, S);
  return S % KB == 0 && (S / 2) % KB == 0;
}

hipError_t launch_doppler_detect(hipStream_t st, const float2* work, int F, int A, int C, int S, const float2* tw_C,
                                 float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask,
                                 int* row_count, float* dbmap, float* pk_pow, bool* supported, int* pk_group,
                                 const unsigned char* wexp) {
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
                            RfQueues* queues, unsigned char* wexp) {
  *supported = true;
  if (F <= 0 || A <= 0 || C <= 0) return hipSuccess;
  switch (S) {
#define CASE(n) \
  case n:       \
    return launch_k1<n>(st, cube, F, A, Ct, chirp0, C, table, tw_S, dc, work, wexp, queues);
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

#if defined(__HIP_DEVICE_COMPILE__)
#pragma clang attribute pop
#endif
