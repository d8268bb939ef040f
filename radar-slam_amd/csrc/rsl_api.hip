// rsl_api.hip — C-ABI layer of librsl.so (see include/rsl.h).  No kernels here: argument checks,
// per-size twiddle tables, launch + optional hipEvent timing on the handle's stream.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsl.h"
#include "rsl_common.h"
#include "rsl_internal.h"

struct rsl_context {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::map<int, float2*> tw;  // N -> device table exp(-2 pi i k / N)
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[RSL_K_COUNT];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  double ms[RSL_K_COUNT] = {0};
  long long cnt[RSL_K_COUNT] = {0};
  // per-launch [start, end] in ms after the reference event t0 (recorded by rsl_timing_reset on the handle's stream):
  // the live timeline of the launches since the reset, every stream's launches on one device clock
  hipEvent_t t0 = nullptr;
  std::vector<std::pair<double, double>> span[RSL_K_COUNT];
  rsl::RfQueues* rfq = nullptr;  // K1 tile queues, one per stream this handle launched K1 on (freed by rsl_destroy)
};

namespace {

int fail(rsl_context* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  return code;
}

int hip_check(rsl_context* h, hipError_t e, const char* what) {
  if (e == hipSuccess) return RSL_OK;
  return fail(h, RSL_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct Scope {
  rsl_context* h;
  int kid;
  hipEvent_t a = nullptr, b = nullptr;
  Scope(rsl_context* h_, int kid_) : h(h_), kid(kid_) {
    hipSetDevice(h->device);
    if (h->timing) {
      if (!h->ev_pool.empty()) {
        a = h->ev_pool.back().first;
        b = h->ev_pool.back().second;
        h->ev_pool.pop_back();
      } else {
        hipEventCreate(&a);
        hipEventCreate(&b);
      }
      hipEventRecord(a, h->stream);
    }
  }
  ~Scope() {
    if (a) {
      hipEventRecord(b, h->stream);
      h->ev[kid].push_back({a, b});
    }
  }
};

float2* twiddles(rsl_context* h, int n) {
  auto it = h->tw.find(n);
  if (it != h->tw.end()) return it->second;
  std::vector<float2> t(n);
  for (int k = 0; k < n; ++k) {
    const double ang = -2.0 * M_PI * (double)k / (double)n;
    t[k] = make_float2((float)std::cos(ang), (float)std::sin(ang));
  }
  float2* d = nullptr;
  if (hipMalloc(&d, sizeof(float2) * n) != hipSuccess) return nullptr;
  if (hipMemcpy(d, t.data(), sizeof(float2) * n, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  h->tw[n] = d;
  return d;
}

// Folds the recorded launch events into the per-kernel totals and spans.  t0 is recorded on the stream bound at the
// reset, which need not be the stream of a given launch: it is waited for once, and a span whose elapsed-time query
// fails is dropped (never recorded as a silent (0, 0)); a failed duration query drops the launch from the totals.
void collect(rsl_context* h) {
  const bool t0_ok = h->t0 && hipEventSynchronize(h->t0) == hipSuccess;
  for (int k = 0; k < RSL_K_COUNT; ++k) {
    for (auto& p : h->ev[k]) {
      hipEventSynchronize(p.second);
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
        h->ms[k] += ms;
        h->cnt[k] += 1;
      }
      if (t0_ok) {
        float a = 0.f, b = 0.f;
        if (hipEventElapsedTime(&a, h->t0, p.first) == hipSuccess &&
            hipEventElapsedTime(&b, h->t0, p.second) == hipSuccess)
          h->span[k].push_back({a, b});
      }
      h->ev_pool.push_back(p);
    }
    h->ev[k].clear();
  }
}

}  // namespace

extern "C" {

int rsl_version(void) { return RSL_VERSION; }

// 1: radix-{2,3,4,5,7,8} Stockham FFT in LDS; 2: any other length up to 4096 (direct DFT fallback); 0: no.
int rsl_fft_supported(int n) {
  switch (n) {
    case 8: case 16: case 32: case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096:
    case 25: case 50: case 100: case 200: case 400: case 800: case 1600:
      return 1;
    default:
      return (n >= 1 && n <= 4096) ? 2 : 0;
  }
}

int rsl_create(rsl_handle* out, int device) {
  if (!out) return RSL_ERR_INVALID;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RSL_ERR_HIP;
  rsl_context* h = new rsl_context();
  h->device = device;
  h->rfq = rsl::rf_queues_new(device);
  *out = h;
  return RSL_OK;
}

int rsl_destroy(rsl_handle h) {
  if (!h) return RSL_OK;
  hipSetDevice(h->device);
  for (auto& kv : h->tw) hipFree(kv.second);
  for (int k = 0; k < RSL_K_COUNT; ++k)
    for (auto& p : h->ev[k]) {
      hipEventDestroy(p.first);
      hipEventDestroy(p.second);
    }
  for (auto& p : h->ev_pool) {
    hipEventDestroy(p.first);
    hipEventDestroy(p.second);
  }
  if (h->t0) hipEventDestroy(h->t0);
  rsl::rf_queues_free(h->rfq);
  delete h;
  return RSL_OK;
}

const char* rsl_last_error(rsl_handle h) { return h ? h->err.c_str() : "null handle"; }

int rsl_set_stream(rsl_handle h, void* s) {
  if (!h) return RSL_ERR_INVALID;
  h->stream = reinterpret_cast<hipStream_t>(s);
  return RSL_OK;
}

int rsl_sync(rsl_handle h) {
  if (!h) return RSL_ERR_INVALID;
  hipSetDevice(h->device);
  return hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
}

int rsl_timing_enable(rsl_handle h, int on) {
  if (!h) return RSL_ERR_INVALID;
  h->timing = on != 0;
  return RSL_OK;
}

int rsl_timing_reset(rsl_handle h) {
  if (!h) return RSL_ERR_INVALID;
  collect(h);
  for (int k = 0; k < RSL_K_COUNT; ++k) {
    h->ms[k] = 0;
    h->cnt[k] = 0;
    h->span[k].clear();
  }
  hipSetDevice(h->device);
  if (!h->t0) hipEventCreate(&h->t0);
  hipEventRecord(h->t0, h->stream);
  return RSL_OK;
}

int rsl_timing_spans(rsl_handle h, int kid, int max, double* start_ms, double* end_ms) {
  if (!h || kid < 0 || kid >= RSL_K_COUNT || max < 0) return -1;
  collect(h);
  const int n = (int)h->span[kid].size();
  for (int i = 0; i < n && i < max; ++i) {
    if (start_ms) start_ms[i] = h->span[kid][i].first;
    if (end_ms) end_ms[i] = h->span[kid][i].second;
  }
  return n;
}

int rsl_timing_read(rsl_handle h, int kid, double* total_ms, long long* launches) {
  if (!h || kid < 0 || kid >= RSL_K_COUNT) return RSL_ERR_INVALID;
  collect(h);
  if (total_ms) *total_ms = h->ms[kid];
  if (launches) *launches = h->cnt[kid];
  return RSL_OK;
}

int rsl_rds(rsl_handle h, const void* cube, int F, int A, int C_total, int chirp0, int C, int S, const void* table,
            int dc_removal, void* work, void* rds) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || A <= 0 || S <= 0 || C <= 0 || chirp0 < 0 || chirp0 + C > C_total)
    return fail(h, RSL_ERR_INVALID, "rsl_rds: bad shape");
  if (F == 0) return RSL_OK;  // empty batch: the (zero-size) buffers may be null
  if (!cube || !table || !work || !rds) return fail(h, RSL_ERR_INVALID, "rsl_rds: null pointer");
  if (!rsl_fft_supported(S) || !rsl_fft_supported(C))
    return fail(h, RSL_ERR_UNSUPPORTED, "rsl_rds: FFT size not supported (S=" + std::to_string(S) +
                                            ", C=" + std::to_string(C) + ")");
  hipSetDevice(h->device);
  float2* tS = twiddles(h, S);
  float2* tC = twiddles(h, C);
  if (!tS || !tC) return fail(h, RSL_ERR_HIP, "twiddle table allocation failed");
  bool sup = true;
  hipError_t e;
  {
    Scope sc(h, RSL_K_RANGE_FFT);
    e = rsl::launch_range_fft(h->stream, (const float2*)cube, F, A, C_total, chirp0, C, S, (const float2*)table, tS,
                              dc_removal, (float2*)work, &sup, h->rfq);
  }
  if (int r = hip_check(h, e, "range_fft")) return r;
  {
    Scope sc(h, RSL_K_DOPPLER_FFT);
    e = rsl::launch_doppler_fft(h->stream, (const float2*)work, F, A, C, S, tC, (float2*)rds, &sup);
  }
  return hip_check(h, e, "doppler_fft");
}

int rsl_rds_detect(rsl_handle h, const void* cube, int F, int A, int C_total, int chirp0, int C, int S,
                   const void* table, int dc_removal, void* work, void* rds, double thr_power, int i_lo, int i_hi,
                   void* mask, void* row_count, void* db_map, void* peak_pow, int* peak_pow_group) {
  if (!h) return RSL_ERR_INVALID;
  if (peak_pow_group) *peak_pow_group = 1;
  if (F < 0 || A <= 0 || S <= 0 || C <= 0 || chirp0 < 0 || chirp0 + C > C_total)
    return fail(h, RSL_ERR_INVALID, "rsl_rds_detect: bad shape");
  if (F == 0) return RSL_OK;  // empty batch: the (zero-size) buffers may be null
  if (!mask || !row_count) return fail(h, RSL_ERR_INVALID, "rsl_rds_detect: null pointer");
  if (!rsl::doppler_detect_supported(C, S)) {  // unfused: a7 then a8
    if (int r = rsl_rds(h, cube, F, A, C_total, chirp0, C, S, table, dc_removal, work, rds)) return r;
    return rsl_detect(h, rds, F, A, S, C, thr_power, i_lo, i_hi, mask, row_count, db_map, peak_pow);
  }
  if (!cube || !table || !work || !rds) return fail(h, RSL_ERR_INVALID, "rsl_rds_detect: null pointer");
  if (!rsl_fft_supported(S)) return fail(h, RSL_ERR_UNSUPPORTED, "rsl_rds_detect: FFT size not supported");
  hipSetDevice(h->device);
  float2* tS = twiddles(h, S);
  float2* tC = twiddles(h, C);
  if (!tS || !tC) return fail(h, RSL_ERR_HIP, "twiddle table allocation failed");
  bool sup = true;
  int group = 1;
  hipError_t e;
  // packed range spectra between K1 and K2 (6 B per value, each bin's exponent inside its 48-B unit; the tiles fill
  // the first 3/4 of the c64-sized work buffer the caller provides; wexp is the launchers' packed-path switch)
  unsigned char* wexp =
      rsl::work_packed_supported(C, S) ? (unsigned char*)work + (size_t)F * A * C * S * 6 : nullptr;
  {
    Scope sc(h, RSL_K_RANGE_FFT);
    e = rsl::launch_range_fft(h->stream, (const float2*)cube, F, A, C_total, chirp0, C, S, (const float2*)table, tS,
                              dc_removal, (float2*)work, &sup, h->rfq, wexp);
  }
  if (int r = hip_check(h, e, "range_fft")) return r;
  {
    Scope sc(h, RSL_K_DOPPLER_FFT);
    e = rsl::launch_doppler_detect(h->stream, (const float2*)work, F, A, C, S, tC, (float2*)rds, thr_power, i_lo,
                                   i_hi, (unsigned long long*)mask, (int*)row_count, (float*)db_map,
                                   (float*)peak_pow, &sup, &group, wexp);
  }
  if (peak_pow_group) *peak_pow_group = group;
  return hip_check(h, e, "doppler_detect");
}

int rsl_detect(rsl_handle h, const void* rds, int F, int A, int S, int C, double thr_power, int i_lo, int i_hi,
               void* mask, void* row_count, void* db_map, void* peak_pow) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || A <= 0 || S <= 0 || C <= 0) return fail(h, RSL_ERR_INVALID, "rsl_detect: bad shape");
  if (F == 0) return RSL_OK;
  if (!rds || !mask || !row_count) return fail(h, RSL_ERR_INVALID, "rsl_detect: null pointer");
  if ((size_t)(18 * (size_t)C * 4) > 64 * 1024) return fail(h, RSL_ERR_UNSUPPORTED, "rsl_detect: C too large");
  Scope sc(h, RSL_K_DETECT);
  return hip_check(h,
                   rsl::launch_detect(h->stream, (const float2*)rds, F, A, S, C, thr_power, i_lo, i_hi,
                                      (unsigned long long*)mask, (int*)row_count, (float*)db_map, (float*)peak_pow),
                   "detect");
}

int rsl_peak_offsets(rsl_handle h, const void* mask, const void* row_count, int F, int A, int S, int C,
                     void* entry_row_off, void* cell_row_off, void* scratch, void* entry_base, void* cell_base,
                     void* frame_counts, void* union_mask) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || A <= 0 || S <= 0 || C <= 0 || A > 32) return fail(h, RSL_ERR_INVALID, "rsl_peak_offsets: bad shape");
  if (!entry_base || !cell_base) return fail(h, RSL_ERR_INVALID, "rsl_peak_offsets: null pointer");
  if (F > 0 && (!mask || !row_count || !entry_row_off || !cell_row_off || !scratch || !frame_counts))
    return fail(h, RSL_ERR_INVALID, "rsl_peak_offsets: null pointer");
  if (F == 0) {
    hipSetDevice(h->device);
    long long z = 0;
    hipMemcpyAsync(entry_base, &z, 8, hipMemcpyHostToDevice, h->stream);
    hipMemcpyAsync(cell_base, &z, 8, hipMemcpyHostToDevice, h->stream);
    return hip_check(h, hipStreamSynchronize(h->stream), "offsets(F=0)");
  }
  Scope sc(h, RSL_K_OFFSETS);
  return hip_check(h,
                   rsl::launch_offsets(h->stream, (const unsigned long long*)mask, (const int*)row_count, F, A, S, C,
                                       (int*)entry_row_off, (int*)cell_row_off, (int*)scratch,
                                       (long long*)entry_base, (long long*)cell_base, (long long*)frame_counts,
                                       (unsigned long long*)union_mask),
                   "offsets");
}

int rsl_peak_emit(rsl_handle h, const void* rds, const void* mask, const void* union_mask, const void* peak_pow,
                  int peak_pow_group, int F, int A, int S, int C, const void* entry_row_off, const void* cell_row_off, const void* entry_base,
                  const void* cell_base, long long entry_cap, long long cell_cap, void* e_coord, void* e_cell,
                  void* e_pdb, void* c_frame, void* c_rc, void* c_amask) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || A <= 0 || A > 32 || S <= 0 || C <= 0 || S > 8192 || C > 8192)
    return fail(h, RSL_ERR_INVALID, "rsl_peak_emit: bad shape");
  if (F == 0) return RSL_OK;
  if (!mask || !entry_row_off || !cell_row_off || !entry_base || !cell_base)
    return fail(h, RSL_ERR_INVALID, "rsl_peak_emit: null pointer");
  if ((entry_cap > 0 && (!e_coord || !e_cell)) || (cell_cap > 0 && (!c_frame || !c_rc || !c_amask)))
    return fail(h, RSL_ERR_INVALID, "rsl_peak_emit: null output");
  const int W = (C + 63) / 64;
  if (peak_pow && (peak_pow_group < 1 || S % peak_pow_group != 0))
    return fail(h, RSL_ERR_INVALID, "rsl_peak_emit: peak_pow_group must divide S");
  Scope sc(h, RSL_K_EMIT);
  if (union_mask && (peak_pow || !e_pdb) && (W & (W - 1)) == 0 && W <= 64)
    return hip_check(h,
                     rsl::launch_emit2(h->stream, (const unsigned long long*)mask,
                                       (const unsigned long long*)union_mask, (const float*)peak_pow,
                                       peak_pow_group, F, A, S, C,
                                       (const int*)entry_row_off, (const int*)cell_row_off,
                                       (const long long*)entry_base, (const long long*)cell_base, entry_cap, cell_cap,
                                       (unsigned*)e_coord, (int*)e_cell, (float*)e_pdb,
                                       (int*)c_frame, (int*)c_rc, (unsigned*)c_amask),
                     "emit2");
  if (!rds) return fail(h, RSL_ERR_INVALID, "rsl_peak_emit: rds needed without union_mask / peak_pow");
  return hip_check(h,
                   rsl::launch_emit(h->stream, (const float2*)rds, (const unsigned long long*)mask, F, A, S, C,
                                    (const int*)entry_row_off, (const int*)cell_row_off, (const long long*)entry_base,
                                    (const long long*)cell_base, entry_cap, cell_cap, (unsigned*)e_coord,
                                    (int*)e_cell, (float*)e_pdb, (int*)c_frame, (int*)c_rc,
                                    (unsigned*)c_amask),
                   "emit");
}

static long long steer_f32_floats(int G, int M) {
  const int KS = (2 * M + 3) / 4, KSG = (KS + 3) / 4;
  const long long ntiles = (2LL * G + 15) / 16;
  return ntiles * KSG * 64 * 4;
}

static long long steer_toep_floats(int G, int M) {
  const int KB = M <= 8 ? 1 : 2;
  long long nt = (G + 31) / 32;
  nt += nt & 1;
  return nt * KB * 2 * 64 * 4;
}

// (3) the fp64 steering matrix transposed, steerT[m][g] (double2), for k_doa_fixup's coalesced exact re-scan; at a
// 16-B aligned float offset (both sections before it are multiples of 4 floats)
static long long steer_t64_offset(int G, int M) { return steer_f32_floats(G, M) + steer_toep_floats(G, M); }

long long rsl_steer_table_floats(int G, int M) {
  if (G <= 0 || M <= 0) return 0;
  return steer_t64_offset(G, M) + 4LL * G * M;
}

int rsl_steer_table_build(const double* steer, int G, int M, float* out, int* ntiles_out, int* flags_out) {
  if (!steer || !out || G <= 0 || M <= 0 || M > 16) return RSL_ERR_INVALID;
  const int KS = (2 * M + 3) / 4, KSG = (KS + 3) / 4;
  const int ntiles = (2 * G + 15) / 16;
  for (int t = 0; t < ntiles; ++t)
    for (int sg = 0; sg < KSG; ++sg)
      for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < 4; ++e) {
          const int s = 4 * sg + e;
          const int i = lane & 15, qq = lane >> 4;
          const int k = 4 * s + qq;
          const int g = 8 * t + (i >> 1), part = i & 1;
          double v = 0.0;
          if (s < KS && g < G && k < 2 * M) {
            const int m = k < M ? k : k - M;
            const double ar = steer[((size_t)g * M + m) * 2], ai = steer[((size_t)g * M + m) * 2 + 1];
            if (part == 0) v = k < M ? ar : ai;
            else v = k < M ? -ai : ar;
          }
          out[(((size_t)t * KSG + sg) * 64 + lane) * 4 + e] = (float)v;
        }
  if (ntiles_out) *ntiles_out = ntiles;
  const int uni = rsl::toep_table_build(steer, G, M, reinterpret_cast<uint16_t*>(out + steer_f32_floats(G, M)),
                                        nullptr);
  if (flags_out) *flags_out = (uni && rsl::toep_table_fits(G, M)) ? RSL_STEER_TOEPLITZ : 0;
  double* tT = reinterpret_cast<double*>(out + steer_t64_offset(G, M));
  for (int m = 0; m < M; ++m)
    for (int g = 0; g < G; ++g) {
      tT[((size_t)m * G + g) * 2] = steer[((size_t)g * M + m) * 2];
      tT[((size_t)m * G + g) * 2 + 1] = steer[((size_t)g * M + m) * 2 + 1];
    }
  return RSL_OK;
}

int rsl_doa(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
            const void* ncell_dev, long long ncell, const void* steer_tab, const void* steer_c128, int G, int method,
            void* out_idx, void* out_gmax, void* out_spec) {
  if (!h) return RSL_ERR_INVALID;
  if (A <= 0 || A > 16 || S <= 0 || C <= 0 || G <= 0) return fail(h, RSL_ERR_INVALID, "rsl_doa: bad shape");
  if (!rds || !c_frame || !c_rc || !steer_tab || !out_idx) return fail(h, RSL_ERR_INVALID, "rsl_doa: null pointer");
  const int base_method = method & 0xff;
  const bool toep = (method & RSL_DOA_TOEPLITZ) != 0;
  if (base_method != RSL_METHOD_MUSIC && base_method != RSL_METHOD_BEAMFORMING)
    return fail(h, RSL_ERR_INVALID, "rsl_doa: unknown method");
  const bool music = base_method == RSL_METHOD_MUSIC;
  (void)steer_c128;  // the exact re-scan reads the fp64 copy inside steer_tab (rsl_steer_table_build)
  const double* steerT = reinterpret_cast<const double*>((const float*)steer_tab + steer_t64_offset(G, A));
  if (!ncell_dev && ncell <= 0) return RSL_OK;
  hipSetDevice(h->device);
  Scope sc(h, RSL_K_DOA_SCAN);
  // the Toeplitz f16-MFMA scan: argmax only, or with the whole spectrum in the cell-blocked layout (no gmax there)
  const bool toep_spec = out_spec && (method & RSL_DOA_SPEC_BLOCKED) && !out_gmax;
  if (toep && (!out_spec || toep_spec) && rsl::toep_table_fits(G, A)) {
    int nt32 = (G + 31) / 32;
    nt32 += nt32 & 1;
    const float* tp = (const float*)steer_tab + steer_f32_floats(G, A);
    return hip_check(h,
                     rsl::launch_doa_toep(h->stream, (const float2*)rds, A, S, C, (const int*)c_frame,
                                          (const int*)c_rc, (const long long*)ncell_dev, ncell, tp, nt32, G, music,
                                          steerT, (int*)out_idx, (float*)out_gmax, 0.0,
                                          nullptr, nullptr, toep_spec ? (float*)out_spec : nullptr),
                     "doa_toep");
  }
  long long blocks = 0;  // 0: all resident workgroups (occupancy x CUs)
  if (!ncell_dev) blocks = (ncell + 127) / 128;  // 4 waves x 32 cells
  const int ntiles = (2 * G + 15) / 16;
  if (int r = hip_check(h,
                        rsl::launch_doa_scan(h->stream, (const float2*)rds, A, S, C, (const int*)c_frame,
                                             (const int*)c_rc, (const long long*)ncell_dev, ncell,
                                             (const float*)steer_tab, ntiles, G, music, (int*)out_idx,
                                             (float*)out_gmax, (float*)out_spec,
                                             (method & RSL_DOA_SPEC_BLOCKED) ? -1
                                             : (method & RSL_DOA_SPEC_GMAJOR) ? ncell : 0,
                                             (int)blocks),
                        "doa_scan"))
    return r;
  // the cells the f32 scan marked ambiguous: exact fp64 argmax (rsl_doa_toep.hip k_doa_fixup)
  return hip_check(h,
                   rsl::launch_doa_fixup(h->stream, (const float2*)rds, A, S, C, (const int*)c_frame,
                                         (const int*)c_rc, (const long long*)ncell_dev, ncell, G, music,
                                         steerT, (int*)out_idx, (float*)out_gmax),
                   "doa_fixup");
}

int rsl_doa_extras(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
                   const void* ncell_dev, long long ncell, const void* steer_tab, const void* steer_c128, int G,
                   int method, double esprit_scale, void* out_idx, void* out_gmax, void* esprit_deg, void* phase) {
  if (!h) return RSL_ERR_INVALID;
  if (A < 2 || A > 16 || S <= 0 || C <= 0 || G <= 0) return fail(h, RSL_ERR_INVALID, "rsl_doa_extras: bad shape");
  if (!rds || !c_frame || !c_rc || !steer_tab || !out_idx)
    return fail(h, RSL_ERR_INVALID, "rsl_doa_extras: null pointer");
  if (method != RSL_METHOD_MUSIC && method != RSL_METHOD_BEAMFORMING)
    return fail(h, RSL_ERR_INVALID, "rsl_doa_extras: unknown method");
  const bool music = method == RSL_METHOD_MUSIC;
  (void)steer_c128;  // the exact re-scan reads the fp64 copy inside steer_tab (rsl_steer_table_build)
  const double* steerT = reinterpret_cast<const double*>((const float*)steer_tab + steer_t64_offset(G, A));
  if (!rsl::toep_table_fits(G, A))
    return fail(h, RSL_ERR_UNSUPPORTED, "rsl_doa_extras: grid too large for the Toeplitz path (use rsl_doa)");
  if (!ncell_dev && ncell <= 0) return RSL_OK;
  hipSetDevice(h->device);
  Scope sc(h, RSL_K_DOA_SCAN);
  int nt32 = (G + 31) / 32;
  nt32 += nt32 & 1;
  const float* tp = (const float*)steer_tab + steer_f32_floats(G, A);
  return hip_check(h,
                   rsl::launch_doa_toep(h->stream, (const float2*)rds, A, S, C, (const int*)c_frame, (const int*)c_rc,
                                        (const long long*)ncell_dev, ncell, tp, nt32, G, music,
                                        steerT, (int*)out_idx, (float*)out_gmax, esprit_scale,
                                        (double*)esprit_deg, (double*)phase),
                   "doa_extras");
}

int rsl_cell_extras(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
                    const void* ncell_dev, long long ncell, double esprit_scale, const void* gidx,
                    const void* az_table, void* sig_out, void* esprit_deg, void* phase, void* az_out) {
  if (!h) return RSL_ERR_INVALID;
  if (A <= 0 || A > 32 || S <= 0 || C <= 0) return fail(h, RSL_ERR_INVALID, "rsl_cell_extras: bad shape");
  if (!rds || !c_frame || !c_rc) return fail(h, RSL_ERR_INVALID, "rsl_cell_extras: null pointer");
  if (az_out && (!gidx || !az_table)) return fail(h, RSL_ERR_INVALID, "rsl_cell_extras: az_out needs gidx+table");
  if (ncell <= 0) return RSL_OK;  // ncell is the launch bound (capacity) when ncell_dev is given
  Scope sc(h, RSL_K_CELL_EXTRAS);
  return hip_check(h,
                   rsl::launch_cell_extras(h->stream, (const float2*)rds, A, S, C, (const int*)c_frame,
                                           (const int*)c_rc, (const long long*)ncell_dev, ncell, esprit_scale,
                                           (const int*)gidx, (const double*)az_table, (float2*)sig_out,
                                           (double*)esprit_deg, (double*)phase, (double*)az_out),
                   "cell_extras");
}

int rsl_confidence(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
                   long long n, const void* gidx, const void* steer_c128, const void* steer_phase, void* conf) {
  if (!h) return RSL_ERR_INVALID;
  if (A <= 0 || A > 32 || S <= 0 || C <= 0) return fail(h, RSL_ERR_INVALID, "rsl_confidence: bad shape");
  if (!rds || !c_frame || !c_rc || !gidx || !steer_c128 || !steer_phase || !conf)
    return fail(h, RSL_ERR_INVALID, "rsl_confidence: null pointer");
  Scope sc(h, RSL_K_CONFIDENCE);
  return hip_check(h,
                   rsl::launch_confidence(h->stream, (const float2*)rds, A, S, C, (const int*)c_frame,
                                          (const int*)c_rc, n, (const int*)gidx, (const double*)steer_c128,
                                          (const double*)steer_phase, (double*)conf),
                   "confidence");
}

int rsl_velocity(rsl_handle h, const void* az, const void* gidx, const void* az_table, int G, const void* y,
                 const void* amask, const void* seg, long long n, int F, double k, double ridge, const double* bounds4,
                 void* out, void* resid, void* pred) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || n < 0) return fail(h, RSL_ERR_INVALID, "rsl_velocity: bad argument");
  if (F == 0) return RSL_OK;
  if ((!az && !gidx) || !y || !seg || !bounds4 || !out) return fail(h, RSL_ERR_INVALID, "rsl_velocity: bad argument");
  if (gidx && (!az_table || G <= 0 || G > 2048)) return fail(h, RSL_ERR_INVALID, "rsl_velocity: bad grid table");
  if (!(bounds4[0] <= bounds4[1]) || !(bounds4[2] <= bounds4[3]) || ridge < 0)
    return fail(h, RSL_ERR_INVALID, "rsl_velocity: bad bounds/ridge");
  Scope sc(h, RSL_K_VELOCITY);
  return hip_check(h,
                   rsl::launch_velocity(h->stream, (const double*)az, (const int*)gidx, (const double*)az_table, G,
                                        (const double*)y, (const unsigned*)amask, (const long long*)seg, n, F, k, ridge,
                                        bounds4, (double*)out, (double*)resid, (double*)pred),
                   "velocity");
}

int rsl_preprocess_rows(rsl_handle h, const void* in, long long rows, int S, const void* table, int dc, void* out) {
  if (!h) return RSL_ERR_INVALID;
  if (rows < 0 || S <= 0 || !in || !table || !out) return fail(h, RSL_ERR_INVALID, "rsl_preprocess_rows: bad argument");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h, rsl::launch_preprocess_rows(h->stream, (const float2*)in, rows, S, (const float2*)table, dc,
                                                  (float2*)out),
                   "preprocess_rows");
}

int rsl_phase_model(rsl_handle h, const void* pos, const void* ang, long long n, const void* x, double k,
                    const void* y, int wrap, double ridge, void* pred, void* resid, void* cost) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 0 || !pos || !ang || !x) return fail(h, RSL_ERR_INVALID, "rsl_phase_model: bad argument");
  if ((resid || cost) && !y) return fail(h, RSL_ERR_INVALID, "rsl_phase_model: residual/cost need y");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h, rsl::launch_phase_model(h->stream, (const double*)pos, (const double*)ang, n, (const double*)x,
                                              k, (const double*)y, wrap, ridge, (double*)pred, (double*)resid,
                                              (double*)cost),
                   "phase_model");
}

int rsl_bvls(rsl_handle h, const void* pos, const void* ang, long long n, const void* y, double k, int nv,
             double ridge, const void* lo, const void* hi, void* out) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 0 || (nv != 3 && nv != 6) || !pos || !ang || !y || !lo || !hi || !out || ridge < 0)
    return fail(h, RSL_ERR_INVALID, "rsl_bvls: bad argument");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h, rsl::launch_bvls(h->stream, (const double*)pos, (const double*)ang, n, (const double*)y, k, nv,
                                       ridge, (const double*)lo, (const double*)hi, (double*)out),
                   "bvls");
}

}  // extern "C"

int rsl_associate(rsl_handle h, const void* cur_xy, int nc, const void* prev_xy, int np, double thr, void* scratch,
                  void* match, void* dist) {
  if (!h) return RSL_ERR_INVALID;
  if (nc < 0 || np < 0 || !(thr >= 0)) return fail(h, RSL_ERR_INVALID, "rsl_associate: bad argument");
  if (nc > 0 && (!cur_xy || !match || !dist || (np > 0 && (!prev_xy || !scratch))))
    return fail(h, RSL_ERR_INVALID, "rsl_associate: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_associate(h->stream, (const double*)cur_xy, nc, (const double*)prev_xy, np, thr,
                                         (unsigned*)scratch, (int*)match, (double*)dist),
                   "associate");
}

int rsl_peak_topk(rsl_handle h, const void* entry_base, long long entry_cap, int ncube, const void* e_coord,
                  const void* e_pdb, double thr_db, int kmax, int C, void* sel_entry, void* sel_frame, void* sel_rc,
                  void* sel_n) {
  if (!h) return RSL_ERR_INVALID;
  if (ncube < 0 || entry_cap < 0 || C <= 0 || C > 8192) return fail(h, RSL_ERR_INVALID, "rsl_peak_topk: bad argument");
  if (kmax < 1 || kmax > 256) return fail(h, RSL_ERR_UNSUPPORTED, "rsl_peak_topk: kmax must be 1..256");
  if (ncube == 0) return RSL_OK;
  if (!entry_base || !sel_entry || !sel_frame || !sel_rc || !sel_n || (entry_cap > 0 && (!e_coord || !e_pdb)))
    return fail(h, RSL_ERR_INVALID, "rsl_peak_topk: null pointer");
  hipSetDevice(h->device);
  Scope sc(h, RSL_K_AUX);
  // the reference compares float64 power_db > thr_db; the entries' power_db is f32, so compare against the largest
  // float <= thr_db (identical decisions for every f32 value)
  return hip_check(h,
                   rsl::launch_topk_entries(h->stream, (const long long*)entry_base, entry_cap, ncube,
                                            (const unsigned*)e_coord, (const float*)e_pdb,
                                            rsl::threshold_as_float(thr_db), kmax, C, (int*)sel_entry,
                                            (int*)sel_frame, (int*)sel_rc, (int*)sel_n),
                   "peak_topk");
}

int rsl_associate_nearest(rsl_handle h, const void* range_m, const void* az_rad, const void* s0, const void* off,
                          int nframes, long long ntargets, double thr, void* match, void* dist, void* phase) {
  if (!h) return RSL_ERR_INVALID;
  if (nframes < 0 || ntargets < 0 || !(thr >= 0)) return fail(h, RSL_ERR_INVALID, "rsl_associate_nearest: bad argument");
  if (nframes == 0 || ntargets == 0) return RSL_OK;
  if (!range_m || !az_rad || !s0 || !off || !match || !dist || !phase)
    return fail(h, RSL_ERR_INVALID, "rsl_associate_nearest: null pointer");
  hipSetDevice(h->device);
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_associate_nearest(h->stream, (const double*)range_m, (const double*)az_rad,
                                                 (const double2*)s0, (const long long*)off, nframes, ntargets, thr,
                                                 (int*)match, (double*)dist, (double*)phase),
                   "associate_nearest");
}

long long rsl_wrapped_scratch_bytes(long long n, int grid_n, int nextra) {
  if (n < 0 || grid_n < 0 || nextra < 0) return -1;
  return 8LL * (6 * n + 36 + 8 * ((long long)grid_n * grid_n + nextra));
}

int rsl_wrapped_solve(rsl_handle h, const void* pos, const void* ang, long long n, const void* y, double k, int mode,
                      double w, double vmax, double wmax, const void* prev, const double* lo6, const double* hi6,
                      int nv, int grid_n, const void* extra, int nextra, int iters, void* scratch,
                      long long scratch_bytes, void* out) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 1 || (nv != 3 && nv != 6) || (mode != 0 && mode != 1) || grid_n < 0 || nextra < 0 || iters < 0 ||
      grid_n * (long long)grid_n + nextra < 1)
    return fail(h, RSL_ERR_INVALID, "rsl_wrapped_solve: bad argument");
  if (!pos || !ang || !y || !lo6 || !hi6 || !scratch || !out || (nextra > 0 && !extra))
    return fail(h, RSL_ERR_INVALID, "rsl_wrapped_solve: null pointer");
  for (int a = 0; a < 6; ++a)
    if (!(lo6[a] <= hi6[a])) return fail(h, RSL_ERR_INVALID, "rsl_wrapped_solve: bad bounds");
  if (scratch_bytes < rsl_wrapped_scratch_bytes(n, grid_n, nextra))
    return fail(h, RSL_ERR_INVALID, "rsl_wrapped_solve: scratch too small");
  Scope sc(h, RSL_K_VELOCITY);
  return hip_check(h,
                   rsl::launch_wrapped_solve(h->stream, (const double*)pos, (const double*)ang, n, (const double*)y,
                                             k, mode, w, vmax, wmax, (const double*)prev, lo6, hi6, nv, grid_n,
                                             (const double*)extra, nextra, iters, (double*)scratch, (double*)out),
                   "wrapped_solve");
}

// stage-1 grid of rsl_wrapped_search: ceil(width / spacing) points per axis, at least 1, at most 2^15 (so the grid
// has < 2^30 starts)
static void search_grid(const double* lo6, const double* hi6, double spacing, long long* gx, long long* gy) {
  auto pts = [&](double w) {
    double g = spacing > 0 ? ceil(w / spacing) : 1.0;
    if (!(g >= 1.0)) g = 1.0;
    if (g > 32768.0) g = 32768.0;
    return (long long)g;
  };
  *gx = pts(hi6[0] - lo6[0]);
  *gy = pts(hi6[1] - lo6[1]);
}

long long rsl_wrapped_search_scratch_bytes(long long n, const double* lo6, const double* hi6, double spacing,
                                           int nbest, int nextra) {
  if (n < 0 || !lo6 || !hi6 || nbest < 1 || nextra < 0) return -1;
  long long gx, gy;
  search_grid(lo6, hi6, spacing, &gx, &gy);
  return 8LL * rsl::wrapped_search_scratch_doubles(n, gx * gy, nbest, nextra);
}

int rsl_wrapped_search(rsl_handle h, const void* pos, const void* ang, long long n, const void* y, double k, int mode,
                       double w, double vmax, double wmax, const void* prev, const double* lo6, const double* hi6,
                       int nv, const double* base6, double spacing, int nbest, const void* extra, int nextra, int iters,
                       void* scratch, long long scratch_bytes, void* out) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 1 || (nv != 3 && nv != 6) || (mode != 0 && mode != 1) || !(spacing > 0) || nbest < 1 || nbest > 1024 ||
      nextra < 0 || iters < 0)
    return fail(h, RSL_ERR_INVALID, "rsl_wrapped_search: bad argument");
  if (!pos || !ang || !y || !lo6 || !hi6 || !base6 || !scratch || !out || (nextra > 0 && !extra))
    return fail(h, RSL_ERR_INVALID, "rsl_wrapped_search: null pointer");
  for (int a = 0; a < 6; ++a)
    if (!(lo6[a] <= hi6[a])) return fail(h, RSL_ERR_INVALID, "rsl_wrapped_search: bad bounds");
  if (scratch_bytes < rsl_wrapped_search_scratch_bytes(n, lo6, hi6, spacing, nbest, nextra))
    return fail(h, RSL_ERR_INVALID, "rsl_wrapped_search: scratch too small");
  long long gx, gy;
  search_grid(lo6, hi6, spacing, &gx, &gy);
  hipSetDevice(h->device);
  Scope sc(h, RSL_K_VELOCITY);
  return hip_check(h,
                   rsl::launch_wrapped_search(h->stream, (const double*)pos, (const double*)ang, n, (const double*)y,
                                              k, mode, w, vmax, wmax, (const double*)prev, lo6, hi6, nv, base6, gx,
                                              gy, nbest, (const double*)extra, nextra, iters, (double*)scratch,
                                              (double*)out),
                   "wrapped_search");
}

int rsl_traj_scan(rsl_handle h, const void* vel, int vstride, int nv, const void* omega, int ostride,
                  const void* timestamps, double dt, long long F, int method, void* pos, void* quat, void* summary) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || nv < 0 || nv > 3 || vstride < nv || (omega && ostride < 3) || (method != 0 && method != 1))
    return fail(h, RSL_ERR_INVALID, "rsl_traj_scan: bad argument");
  if (F > 0 && (!vel || !pos || !quat)) return fail(h, RSL_ERR_INVALID, "rsl_traj_scan: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_traj_scan(h->stream, (const double*)vel, vstride, nv, (const double*)omega, ostride,
                                         (const double*)timestamps, dt, F, method, (double*)pos, (double*)quat,
                                         (double*)summary),
                   "traj_scan");
}

int rsl_traj_apply(rsl_handle h, void* pos, void* quat, long long F, const void* base) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || (F > 0 && (!pos || !quat || !base))) return fail(h, RSL_ERR_INVALID, "rsl_traj_apply: bad argument");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h, rsl::launch_traj_apply(h->stream, (double*)pos, (double*)quat, F, (const double*)base),
                   "traj_apply");
}

int rsl_traj_smooth(rsl_handle h, const void* x, long long F, int ncol, int size, void* out) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || ncol < 1 || size < 1 || (F > 0 && (!x || !out)))
    return fail(h, RSL_ERR_INVALID, "rsl_traj_smooth: bad argument");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h, rsl::launch_traj_smooth(h->stream, (const double*)x, F, ncol, size, (double*)out),
                   "traj_smooth");
}

int rsl_traj_stitch(rsl_handle h, const void* summaries, int R, int rank, double dt, int method, void* state,
                    void* base) {
  if (!h) return RSL_ERR_INVALID;
  if (R < 1 || rank < 0 || rank >= R || (method != 0 && method != 1) || !summaries || !state || !base)
    return fail(h, RSL_ERR_INVALID, "rsl_traj_stitch: bad argument");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_traj_stitch(h->stream, (const double*)summaries, R, rank, dt, method, (double*)state,
                                           (double*)base),
                   "traj_stitch");
}

int rsl_synth_pattern(rsl_handle h, const void* scatterers, int n, int A, int S, double fc, double bandwidth,
                      double chirp_duration, double antenna_spacing, void* pattern) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 0 || A <= 0 || S <= 0 || !(fc > 0) || !(chirp_duration > 0))
    return fail(h, RSL_ERR_INVALID, "rsl_synth_pattern: bad arguments");
  if (!pattern || (n > 0 && !scatterers)) return fail(h, RSL_ERR_INVALID, "rsl_synth_pattern: null pointer");
  const double d = antenna_spacing > 0 ? antenna_spacing : 0.5 * 3e8 / fc;
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_synth_pattern(h->stream, (const double*)scatterers, n, A, S, fc, bandwidth,
                                             chirp_duration, d, (double2*)pattern),
                   "synth_pattern");
}

int rsl_synth_cube(rsl_handle h, const void* pattern, int F, int A, int C, int S, double noise_power,
                   unsigned long long seed, long long frame0, void* cube) {
  if (!h) return RSL_ERR_INVALID;
  if (F < 0 || A <= 0 || C <= 0 || S <= 0 || frame0 < 0 || !(noise_power >= 0))
    return fail(h, RSL_ERR_INVALID, "rsl_synth_cube: bad arguments");
  if (S % 2) return fail(h, RSL_ERR_UNSUPPORTED, "rsl_synth_cube: S must be even");
  if (!pattern || !cube) return fail(h, RSL_ERR_INVALID, "rsl_synth_cube: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_synth_cube(h->stream, (const double2*)pattern, F, A, C, S, noise_power, seed, frame0,
                                          (float2*)cube),
                   "synth_cube");
}

long long rsl_pose_error_scratch_bytes(long long n, int nlen) {
  if (n < 0 || nlen < 0) return -1;
  return 8 * rsl::pose_error_scratch_doubles(n, nlen);
}

int rsl_pose_align(rsl_handle h, const void* est, const void* gt, long long n, void* scratch, void* align,
                   void* aligned, void* ape_err, void* ape_stats) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 1) return fail(h, RSL_ERR_INVALID, "rsl_pose_align: need at least one pose");
  if (!est || !gt || !scratch || !align || !aligned || !ape_err)
    return fail(h, RSL_ERR_INVALID, "rsl_pose_align: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_pose_align(h->stream, (const double*)est, (const double*)gt, n, (double*)scratch,
                                          (double*)align, (double*)aligned, (double*)ape_err, (double*)ape_stats),
                   "pose_align");
}

int rsl_pose_rte(rsl_handle h, const void* aligned, const void* gt, long long n, const void* lengths, int nlen,
                 void* scratch, void* err, void* counts, void* stats) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 1 || nlen < 0 || nlen > 1024) return fail(h, RSL_ERR_INVALID, "rsl_pose_rte: bad arguments");
  if (nlen == 0) return RSL_OK;
  if (!aligned || !gt || !lengths || !scratch || !err || !counts || !stats)
    return fail(h, RSL_ERR_INVALID, "rsl_pose_rte: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_pose_rte(h->stream, (const double*)aligned, (const double*)gt, n,
                                        (const double*)lengths, nlen, (double*)scratch, (double*)err,
                                        (unsigned long long*)counts, (double*)stats),
                   "pose_rte");
}

int rsl_music_subspace(rsl_handle h, const void* sigs, long long n, int M, int num_sources, const void* steer_c128,
                       int G, void* spec) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 0 || M < 1 || M > 16 || G < 1) return fail(h, RSL_ERR_INVALID, "rsl_music_subspace: bad shape");
  if (n == 0) return RSL_OK;
  if (!sigs || !steer_c128 || !spec) return fail(h, RSL_ERR_INVALID, "rsl_music_subspace: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_music_subspace(h->stream, (const double*)sigs, n, M, num_sources,
                                              (const double*)steer_c128, G, (double*)spec),
                   "music_subspace");
}

int rsl_esprit_subspace(rsl_handle h, const void* sigs, long long n, int M, int num_sources, double esprit_scale,
                        void* deg) {
  if (!h) return RSL_ERR_INVALID;
  if (n < 0 || M < 1 || M > 16) return fail(h, RSL_ERR_INVALID, "rsl_esprit_subspace: bad shape");
  if (n == 0) return RSL_OK;
  if (!sigs || !deg) return fail(h, RSL_ERR_INVALID, "rsl_esprit_subspace: null pointer");
  Scope sc(h, RSL_K_AUX);
  return hip_check(h,
                   rsl::launch_esprit_subspace(h->stream, (const double*)sigs, n, M, num_sources, esprit_scale,
                                               (double*)deg),
                   "esprit_subspace");
}
