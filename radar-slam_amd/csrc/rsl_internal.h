// rsl_internal.h — launcher declarations shared between the kernel files and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsl {

// Cell count of a capacity-sized list: the device count (written by the emit stage) clamped to the list capacity,
// so an overflowing batch reads and writes only the slots that exist (the host sees the overflow in the count).
__device__ __forceinline__ long long list_count(const long long* dev, long long cap) {
  if (!dev) return cap;
  const long long n = *dev;
  return n < cap ? n : cap;
}

// K1 tile queues of one handle (rsl_fft.hip): one 2 KiB queue per stream the handle launches K1 on, allocated on the
// handle's device at that stream's first K1 launch, freed by rf_queues_free (rsl_destroy).
struct RfQueues;
RfQueues* rf_queues_new(int device);
void rf_queues_free(RfQueues* s);
// K1: dechirp * window (table), range FFT (S points), DC bin zeroing.
// cube c64 [F, A, Ct, S] (chirps chirp0 .. chirp0+C-1 used) -> work c64 [F, A, C, S]
hipError_t launch_range_fft(hipStream_t st, const float2* cube, int F, int A, int Ct, int chirp0, int C, int S,
                            const float2* table, const float2* tw_S, int dc, float2* work, bool* supported,
                            RfQueues* queues, unsigned char* wexp = nullptr);
// K2: Doppler FFT (C points) + fftshift on both axes, transposed store.
// work c64 [F, A, C, S] -> rds c64 [F, A, S, C]
hipError_t launch_doppler_fft(hipStream_t st, const float2* work, int F, int A, int C, int S, const float2* tw_C,
                              float2* rds, bool* supported);

// K2+K3 fused (Doppler FFT + fftshift + RDS store + detection); supported when C is a power of two and the
// block's KB range bins tile both halves of S.
bool doppler_detect_supported(int C, int S);
float threshold_as_float(double thr);  // largest float t <= thr
hipError_t launch_doppler_detect(hipStream_t st, const float2* work, int F, int A, int C, int S, const float2* tw_C,
                                 float2* rds, double thr_p, int i_lo, int i_hi, unsigned long long* mask,
                                 int* row_count, float* dbmap, float* pk_pow, bool* supported, int* pk_group,
                                 const unsigned char* wexp = nullptr);
// wexp non-null (both launches): `work` holds packed rows (rsl_fft.hip pk_pack16: 6 B per value in 24 KiB tiles, each
// bin's int8 exponent inside its 48-B unit; the pointer is only the switch, nothing is stored there) -- only where
// work_packed_supported(C, S).
bool work_packed_supported(int C, int S);
// K3: 3x3 local max (reflect), threshold, range gate -> per-antenna bit masks + row counts.
hipError_t launch_detect(hipStream_t st, const float2* rds, int F, int A, int S, int C, double thr_p, int i_lo,
                         int i_hi, unsigned long long* mask, int* row_count, float* dbmap, float* pk_pow);
// Per-frame offsets of peak entries (antenna-major) and union cells (range-major).
hipError_t launch_offsets(hipStream_t st, const unsigned long long* mask, const int* row_count, int F, int A, int S,
                          int C, int* entry_row_off, int* cell_row_off, int* cell_row_cnt, long long* entry_base,
                          long long* cell_base, long long* frame_counts, unsigned long long* umask);
// Emit compacted entries and cells in reference order.
hipError_t launch_emit(hipStream_t st, const float2* rds, const unsigned long long* mask, int F, int A, int S, int C,
                       const int* entry_row_off, const int* cell_row_off, const long long* entry_base,
                       const long long* cell_base, long long entry_cap, long long cell_cap, unsigned* e_coord,
                       int* e_cell, float* e_pdb, int* c_frame, int* c_rc, unsigned* c_amask);

// Emit from group-compact peak powers (pk_group rows per group, 1 = row-compact) and union masks (no RDS read);
// W = ceil(C/64) must be a power of two <= 64.
hipError_t launch_emit2(hipStream_t st, const unsigned long long* mask, const unsigned long long* umask,
                        const float* pk_pow, int pk_group, int F, int A, int S, int C, const int* entry_row_off,
                        const int* cell_row_off, const long long* entry_base, const long long* cell_base,
                        long long entry_cap, long long cell_cap, unsigned* e_coord, int* e_cell, float* e_pdb,
                        int* c_frame, int* c_rc, unsigned* c_amask);
// K5: steering scan on MFMA (f32 16x16x4), argmax; optional spectrum.
hipError_t launch_doa_scan(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                           const int* c_rc, const long long* ncell_dev, long long ncell_host, const float* steer_tab,
                           int ntiles, int G, int music, int* out_idx, float* out_gmax, float* out_spec,
                           long long spec_ld, int grid_blocks);
// K5 fast path: Toeplitz-form argmax on f16 MFMA with hi/lo split (rsl_doa_toep.hip).
// Exact fp64 re-scan of the cells a DoA scan marked ambiguous (out_idx < 0), rsl_doa_toep.hip k_doa_fixup.
hipError_t launch_doa_fixup(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                            const int* c_rc, const long long* ncell_dev, long long ncell_host, int G, int music,
                            const double* steerT, int* out_idx, float* out_gmax);
hipError_t launch_doa_toep(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                           const int* c_rc, const long long* ncell_dev, long long ncell_host, const void* toep_tab,
                           int ntiles32, int G, int music, const double* steerT, int* out_idx, float* out_gmax,
                           double esprit_scale, double* out_esprit, double* out_phase, float* out_spec = nullptr);
// Host: builds the Toeplitz operand table; returns 1 if the steering matrix is a uniform linear array.
int toep_table_build(const double* steer_c128, int G, int M, uint16_t* out, int* ntiles32_out);
bool toep_table_fits(int G, int M);
// K4/K6: normalised signature, ESPRIT closed form (fp64), spatial phase, azimuth lookup.
hipError_t launch_cell_extras(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                              const int* c_rc, const long long* ncell_dev, long long ncell_host, double esprit_scale,
                              const int* gidx, const double* az_table, float2* sig_out, double* esprit_deg,
                              double* phase, double* az_out);
// K7: robust confidence for (cell, grid index) pairs (fp64).
hipError_t launch_confidence(hipStream_t st, const float2* rds, int A, int S, int C, const int* c_frame,
                             const int* c_rc, long long n, const int* gidx, const double* steer_c128,
                             const double* steer_phase, double* conf_out);
// K8: batched bounded / ridge least squares velocity solve, one segment per frame.
hipError_t launch_velocity(hipStream_t st, const double* az, const int* gidx, const double* az_table, int G,
                           const double* y, const unsigned* amask, const long long* seg, long long n, int F, double k,
                           double ridge,
                           const double* bounds4, double* out, double* resid, double* pred);

// K9: greedy association and wrapped-phase multi-start solve (rsl_wrap.hip).
// configs[3] pattern (rsl_scene.hip): per-cube top-k peak selection and the analyser's nearest association.
hipError_t launch_topk_entries(hipStream_t st, const long long* entry_base, long long entry_cap, int ncube,
                               const unsigned* e_coord, const float* e_pdb, float thr_db, int kmax, int C,
                               int* sel_entry, int* sel_frame, int* sel_rc, int* sel_n);
hipError_t launch_associate_nearest(hipStream_t st, const double* range_m, const double* az_rad, const double2* s0,
                                    const long long* off, int nframes, long long ntargets, double thr, int* match,
                                    double* dist, double* phase);
hipError_t launch_associate(hipStream_t st, const double* cur, int nc, const double* prev, int np, double thr,
                            unsigned* used_scratch, int* match, double* dist);
long wrapped_search_scratch_doubles(long n, long nstart1, int nbest, int nextra);
hipError_t launch_wrapped_search(hipStream_t st, const double* pos, const double* ang, long n, const double* y,
                                 double k, int mode, double w, double vmax, double wmax, const double* prev,
                                 const double* lo, const double* hi, int nv, const double* base6, long gx, long gy,
                                 int nbest, const double* extra, int nextra, int iters, double* scratch, double* out);
hipError_t launch_wrapped_solve(hipStream_t st, const double* pos, const double* ang, long n, const double* y,
                                double k, int mode, double w, double vmax, double wmax, const double* prev,
                                const double* lo, const double* hi, int nv, int gn, const double* extra, int nextra,
                                int iters, double* scratch, double* out);

// Trajectory scans (rsl_traj.hip).
hipError_t launch_traj_scan(hipStream_t st, const double* vel, int vstride, int nv, const double* om, int ostride,
                            const double* ts, double dt, long F, int method, double* pos, double* quat,
                            double* summary);
hipError_t launch_traj_apply(hipStream_t st, double* pos, double* quat, long F, const double* base);
hipError_t launch_traj_stitch(hipStream_t st, const double* summ, int R, int rank, double dt, int method,
                              double* state, double* base);
hipError_t launch_traj_smooth(hipStream_t st, const double* x, long F, int ncol, int size, double* out);
// MUSIC / ESPRIT with num_sources != 1 (rsl_subspace.hip), fp64, per-call drop-in paths.
hipError_t launch_music_subspace(hipStream_t st, const double* sigs, long n, int M, int K, const double* steer,
                                 int G, double* spec);
hipError_t launch_esprit_subspace(hipStream_t st, const double* sigs, long n, int M, int K, double esprit_scale,
                                  double* deg);
// Pose-error evaluation (rsl_eval.hip): Umeyama + quaternion-mean alignment, APE errors / statistics, RTE.
long long pose_error_scratch_doubles(long long n, int nlen);
hipError_t launch_pose_align(hipStream_t st, const double* est, const double* gt, long n, double* scratch,
                             double* align, double* aligned, double* ape_err, double* ape_stats);
hipError_t launch_pose_rte(hipStream_t st, const double* aligned, const double* gt, long n, const double* len,
                           int nlen, double* scratch, double* err, unsigned long long* cnt, double* stats);

}  // namespace rsl

namespace rsl {
hipError_t launch_preprocess_rows(hipStream_t st, const float2* in, long rows, int S, const float2* table, int dc,
                                  float2* out);
hipError_t launch_phase_model(hipStream_t st, const double* pos, const double* ang, long n, const double* x, double k,
                              const double* y, int wrap, double ridge, double* pred, double* resid, double* cost);
hipError_t launch_bvls(hipStream_t st, const double* pos, const double* ang, long n, const double* y, double k, int nv,
                       double ridge, const double* lo, const double* hi, double* out);
// Synthetic cube generator (simulate_raw.py:102-221): fp64 [A, S] pattern, then pattern + Philox noise.
hipError_t launch_synth_pattern(hipStream_t st, const double* sc, int n, int A, int S, double fc, double bandwidth,
                                double Tc, double d, double2* pattern);
hipError_t launch_synth_cube(hipStream_t st, const double2* pattern, int F, int A, int C, int S, double noise_power,
                             unsigned long long seed, long long frame0, float2* cube);

}  // namespace rsl
