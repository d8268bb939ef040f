/* rsl.h — C ABI of the MI355X-native radar signal chain (librsl.so, gfx950 / CDNA4).
 *
 * Drop-in boundary for the per-frame chain of zaidcontractor/radar-slam (snapshot 2025-11-21).
 * The reference is pure Python with no FFI; its boundary is the Python class surface listed per
 * entry point below (file:line in the reference tree).  The Python host layer
 * radar-slam_amd/src/... keeps those module paths and signatures and binds these symbols with
 * ctypes (radar-slam_amd/rsl/_lib.py; binding stubs for other hosts: INTEGRATION.md).
 *
 * Conventions
 *   - every pointer named dev_* / void* data argument is DEVICE memory (hipMalloc / torch tensor);
 *     complex values are interleaved float32 (c64) unless the name says c128 / f64;
 *   - all launches are asynchronous on the handle's stream (rsl_set_stream); rsl_sync waits;
 *   - return 0 (RSL_OK) or an RSL_ERR_* code; rsl_last_error(h) describes the last failure;
 *   - a handle belongs to one device and may launch on any of that device's streams (rsl_set_stream); one thread
 *     drives a handle at a time; handles share no mutable state (the K1 tile queues are per handle and stream,
 *     allocated on the handle's device at a stream's first K1 launch, freed by rsl_destroy);
 *   - graph capture: K1's first launch on a stream allocates that stream's queue, which capture forbids (RSL_ERR_HIP,
 *     "operation not permitted when stream is capturing"): launch once uncaptured first, and never replay one captured
 *     K1 on two streams concurrently (the replays would share the captured queue);
 *   - F = 0 (an empty batch) is valid: nothing is launched (rsl_peak_offsets zeroes the two bases), and
 *     buffers sized by F may be null;
 *   - capacity-sized lists (entries, cells) never overflow in memory: items past the capacity are dropped,
 *     the bases keep the true counts, and the list consumers stop at the capacity.
 */
#ifndef RSL_H
#define RSL_H

#ifdef __cplusplus
extern "C" {
#endif

#define RSL_OK 0
#define RSL_ERR_INVALID 1     /* bad argument (shape, null pointer)        -> Python ValueError   */
#define RSL_ERR_UNSUPPORTED 2 /* FFT size / antenna count not implemented  -> Python ValueError   */
#define RSL_ERR_HIP 3         /* HIP runtime error                          -> Python RuntimeError */

#define RSL_METHOD_BEAMFORMING 0
#define RSL_METHOD_MUSIC 1
/* rsl_doa method flag: use the Toeplitz f16-MFMA argmax path (requires RSL_STEER_TOEPLITZ from the table build) */
#define RSL_DOA_TOEPLITZ 0x100
/* rsl_doa method flag: out_spec is grid-major f32 [G][ncell] (leading dimension = the list capacity ncell) instead of
 * cell-major [n][G]; the batched spectrum path (coalesced stores) */
#define RSL_DOA_SPEC_GMAJOR 0x200
/* rsl_doa method flag: out_spec is cell-blocked f32 [ceil(ncell / 32)][G][32] (cell c, grid point g at
 * ((c / 32) G + g) 32 + c % 32): every store is a contiguous run; the batched chain's spectrum layout */
#define RSL_DOA_SPEC_BLOCKED 0x400
/* rsl_steer_table_build flags */
#define RSL_STEER_TOEPLITZ 1

/* kernel ids for rsl_timing_read */
#define RSL_K_RANGE_FFT 0
#define RSL_K_DOPPLER_FFT 1
#define RSL_K_DETECT 2
#define RSL_K_OFFSETS 3
#define RSL_K_EMIT 4
#define RSL_K_DOA_SCAN 5
#define RSL_K_CELL_EXTRAS 6
#define RSL_K_CONFIDENCE 7
#define RSL_K_VELOCITY 8
#define RSL_K_AUX 9
#define RSL_K_COUNT 10

typedef struct rsl_context* rsl_handle;

/* ABI version returned by rsl_version().
 *   1  rounds 1-4;
 *   2  rsl_rds_detect_chunked removed; rsl_steer_table_floats grew by the 4GM-float fp64 transposed section
 *      (steer_t64_offset) that rsl_doa / rsl_doa_extras now read: tables built or sized by a v1 library must be
 *      rebuilt; K1 tile queues are per handle and stream (freed by rsl_destroy). */
#define RSL_VERSION 2
int rsl_version(void);
int rsl_create(rsl_handle* out, int device);
int rsl_destroy(rsl_handle h);
const char* rsl_last_error(rsl_handle h);
int rsl_set_stream(rsl_handle h, void* hip_stream); /* NULL = null stream */
int rsl_sync(rsl_handle h);
/* 1 = radix-{2,3,4,5,7,8} LDS FFT, 2 = direct-DFT fallback (any n <= 4096), 0 = unsupported */
int rsl_fft_supported(int n);

/* Per-kernel device time (hipEvents recorded on the handle's stream around every launch). */
int rsl_timing_enable(rsl_handle h, int on);
int rsl_timing_reset(rsl_handle h);
int rsl_timing_read(rsl_handle h, int kernel_id, double* total_ms, long long* launches);
/* The launches of one kernel id since the last rsl_timing_reset: [start, end] of each, in ms after an event that the
 * reset recorded on the handle's stream (one device clock for every stream the handle ran on), in launch order.
 * Writes min(n, max) pairs (nullable arrays) and returns n, the launch count (-1 on a bad argument). */
int rsl_timing_spans(rsl_handle h, int kernel_id, int max, double* start_ms, double* end_ms);

/* a7  SignalPreprocessor.generate_range_doppler_spectrum  (dechirp.py:168-213, incl. process_chirp
 *     :143-166, dechirp_signal :122-141, apply_window :85-108, remove_dc :110-120, chirp_subset :183-187).
 *     cube c64 [F, A, C_total, S]; chirps chirp0 .. chirp0+C-1 are used;
 *     table c64 [S] = conj(reference_chirp) * window, built on the host in fp64 (dechirp.py:74-83);
 *     dc_removal != 0 zeroes range bin 0 (== subtracting the complex mean before the FFT);
 *     work c64 [F, A, C, S] scratch; rds c64 [F, A, S, C], fftshift on both axes. */
int rsl_rds(rsl_handle h, const void* cube, int F, int A, int C_total, int chirp0, int C, int S,
            const void* table, int dc_removal, void* work, void* rds);

/* a8  SignalPreprocessor.extract_range_doppler_peaks  (dechirp.py:215-278).
 *     thr_power = 10^(threshold_db/10) - 1e-12 (a cell passes when (double)|rds|^2 > thr_power);
 *     range gate i_lo <= range_bin <= i_hi (from linspace(0, rr*S, S) on the host);
 *     mask u64 [F, A, S, W], W = ceil(C/64) (bit j%64 of word j/64 = peak at doppler j);
 *     row_count i32 [F, A, S];  db_map f32 [F, A, S, C] (nullable) = 10 log10(|rds|^2 + 1e-12);
 *     peak_pow f32 [F, A, S, C] (nullable): row-compact |rds|^2 of the peaks, slot = rank within the row. */
int rsl_detect(rsl_handle h, const void* rds, int F, int A, int S, int C, double thr_power, int i_lo, int i_hi,
               void* mask, void* row_count, void* db_map, void* peak_pow);

/* a7 + a8 fused: range FFT, then Doppler FFT + fftshift + RDS store + peak detection in one kernel (the RDS is
 *     not re-read for detection).  Arguments as rsl_rds and rsl_detect; falls back to the two calls when the
 *     shape is not covered (C not a power of two <= 1024, or its range-bin tiling does not divide S/2).
 *     peak_pow is written group-compact: the peaks of the G rows r0 .. r0+G-1 of one (frame, antenna)
 *     (row = (f*A + a)*S + i, r0 a multiple of G) are contiguous from slot r0*C, in row order and Doppler order
 *     within a row (full cache lines instead of a short run per row).  *peak_pow_group (host, nullable)
 *     receives G (1 = row-compact, as rsl_detect writes it); pass it to rsl_peak_emit.
 *     work (c64-sized scratch, F A C S 8 bytes): at (S, C) = (256, 64), (512, 128) and (1024, 256) the range
 *     spectra travel packed (6 B per value, chirp-class tiles) in its first F A C S 6 bytes and the rest is not
 *     written; at other shapes it holds the c64 range spectra [F, A, C, S] as in rsl_rds.
 *     The range FFT's tile queue is per stream: the first call on a stream allocates 2 KiB of device memory
 *     (kept for the process) and zeroes it on that stream (likewise rsl_rds). */
int rsl_rds_detect(rsl_handle h, const void* cube, int F, int A, int C_total, int chirp0, int C, int S,
                   const void* table, int dc_removal, void* work, void* rds, double thr_power, int i_lo, int i_hi,
                   void* mask, void* row_count, void* db_map, void* peak_pow, int* peak_pow_group);

/* Offsets for the order-preserving compaction of a8's peak list (antenna -> range -> doppler,
 * dechirp.py:246-271) and of the deduplicated (range, doppler) cells that DoA runs on.
 *     entry_row_off i32 [F*A*S], cell_row_off i32 [F*S], scratch i32 [F*S],
 *     entry_base i64 [F+1], cell_base i64 [F+1] (global exclusive offsets; [F] = totals),
 *     frame_counts i64 [2F] (entries, cells per frame), union_mask u64 [F, S, W] (nullable) = OR over antennas. */
int rsl_peak_offsets(rsl_handle h, const void* mask, const void* row_count, int F, int A, int S, int C,
                     void* entry_row_off, void* cell_row_off, void* scratch, void* entry_base, void* cell_base,
                     void* frame_counts, void* union_mask);

/* Emit the peak entries and the unique cells (c_frame i32, c_rc i32 = range_bin*C + doppler_bin, c_amask u32 =
 * antennas with a peak there).  An entry is e_coord u32 = antenna << 26 | range_bin << 13 | doppler_bin (the
 * RSL_COORD_* macros; S, C <= 8192), e_cell i32 = its cell's list position, e_pdb f32 = power_db (nullable;
 * dechirp.py:235-236, computed in fp32 from the fp32 RDS).  Items beyond *_cap are dropped (compare the totals).
 * With union_mask (from rsl_peak_offsets) and peak_pow (from rsl_detect / rsl_rds_detect, in the row grouping
 * peak_pow_group those report; 1 for rsl_detect) the RDS is not read (rds may be NULL); otherwise power_db is
 * recomputed from rds. */
int rsl_peak_emit(rsl_handle h, const void* rds, const void* mask, const void* union_mask, const void* peak_pow,
                  int peak_pow_group, int F, int A, int S, int C, const void* entry_row_off, const void* cell_row_off, const void* entry_base,
                  const void* cell_base, long long entry_cap, long long cell_cap, void* e_coord, void* e_cell,
                  void* e_pdb, void* c_frame, void* c_rc, void* c_amask);
#define RSL_COORD_ANT(x) ((unsigned)(x) >> 26)
#define RSL_COORD_RANGE(x) (((unsigned)(x) >> 13) & 0x1fffu)
#define RSL_COORD_DOPPLER(x) ((unsigned)(x) & 0x1fffu)

/* Host helper: MFMA operand tables of a steering matrix.  steer_c128 is the host [G][M] complex128
 * matrix of AngleEstimator.generate_steering_vector (angle_estimation.py:92-107) over the azimuth grid
 * (angle_estimation.py:59-60).  rsl_steer_table_floats returns the float count of the table; the build
 * writes (1) the f32 [Re; Im] operand for v_mfma_f32_16x16x4_f32 (*ntiles = its 16-row tiles),
 * (2) the Toeplitz-form f16 hi/lo operand for v_mfma_f32_32x32x16_f16, valid when the steering matrix is a
 * uniform linear array (*flags |= RSL_STEER_TOEPLITZ), and (3) the fp64 matrix itself transposed, [M][G] complex128
 * (the last 4 G M floats), which the exact fp64 re-scan of near-tie cells reads. */
long long rsl_steer_table_floats(int G, int M);
int rsl_steer_table_build(const double* steer_c128, int G, int M, float* host_out, int* ntiles, int* flags);

/* a11-a16  extract_spatial_signature + music_spectrum / estimate_angle_music / estimate_angle_beamforming
 *     (angle_estimation.py:67-176, 227-251; robust_angle_estimation.py:236-245).
 *     Cells (c_frame, c_rc) index rds c64 [*, A, S, C]; n = min(*ncell_dev, ncell) if ncell_dev is non-null
 *     (ncell = the lists' capacity: an overflowed list is processed up to its capacity), else ncell.
 *     steer_tab = device copy of the rsl_steer_table_build output (its fp64 section feeds the exact fp64 re-scan of
 *     the cells whose top-2 gap in the f16 hi/lo or f32 scan is inside that scan's error bound, and of MUSIC's
 *     near-degenerate cells, so out_idx is the fp64 argmax of each cell's own signature; keys within 1e-13 relative
 *     count as ties and the lower index wins, as np.argmax.  The scans' bounds are relative to the cell's best value,
 *     so this exactness is established statistically, not by a worst-case bound); steer_c128 (device fp64 [G][M][2], nullable) is no
 *     longer read by rsl_doa / rsl_doa_extras and is kept for ABI compatibility.
 *     method = RSL_METHOD_* | RSL_DOA_TOEPLITZ (optional; with out_spec it applies to the RSL_DOA_SPEC_BLOCKED layout
 *     without out_gmax, the other spectrum requests take the f32 scan).
 *     out_idx i32 [n] = first-index argmax over the G grid points; out_gmax f32 [n] (nullable) = |a^H s|^2
 *     at the argmax (unit-norm s); out_spec f32 [n, G] (nullable; [G][ncell] with RSL_DOA_SPEC_GMAJOR,
 *     [ceil(ncell / 32)][G][32] with RSL_DOA_SPEC_BLOCKED) = MUSIC
 *     1/(M-|a^H s|^2) with the reference's den > 1e-12 rule, or the beamforming |a^H s|^2. */
int rsl_doa(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
            const void* ncell_dev, long long ncell, const void* steer_tab, const void* steer_c128, int G, int method,
            void* out_idx, void* out_gmax, void* out_spec);

/* a11-a16 + a15 + a26 fused: the Toeplitz argmax of rsl_doa (requires RSL_STEER_TOEPLITZ) plus, from the same
 *     signature load, ESPRIT (f64 deg, nullable; angle_estimation.py:178-225, esprit_scale = lambda/(2 pi d))
 *     and the spatial phase angle(s1 conj(s0)) (f64, nullable; velocity_solver.py:136) of each cell.
 *     Returns RSL_ERR_UNSUPPORTED when the grid does not fit the Toeplitz path. */
int rsl_doa_extras(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
                   const void* ncell_dev, long long ncell, const void* steer_tab, const void* steer_c128, int G,
                   int method, double esprit_scale, void* out_idx, void* out_gmax, void* esprit_deg, void* phase);

/* a11, a15, a26  normalised signature (c64 [n, A], nullable), ESPRIT closed form (f64 deg, nullable;
 *     angle_estimation.py:178-225 with esprit_scale = lambda / (2 pi d)), spatial phase
 *     angle(s1 conj(s0)) (f64, nullable; velocity_solver.py:136), az_out = az_table[gidx] (f64, nullable). */
int rsl_cell_extras(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
                    const void* ncell_dev, long long ncell, double esprit_scale, const void* gidx,
                    const void* az_table, void* sig_out, void* esprit_deg, void* phase, void* az_out);

/* a13-a15 with num_sources != 1  music_spectrum / estimate_angle_music / estimate_angle_esprit
 *     (angle_estimation.py:109-225) for any num_sources (Python slicing semantics for K <= 0 and K >= M), fp64:
 *     sigs c128 [n][M] (device, the signatures as given; MUSIC normalises them), steer_c128 f64 [G][M][2]
 *     (device), spec f64 [n][G] = 1/den or 0 (den <= 1e-12), deg f64 [n] (0.0 where the reference's ESPRIT
 *     raises, NaN where it returns NaN).  The reference's noise / null-space bases for 2 <= K < M come from LAPACK
 *     round-off; these use a fixed Householder completion (rsl_subspace.hip), so only K = 1, K >= M (MUSIC),
 *     K <= 0 (ESPRIT) and zero signatures are reference-determined. */
int rsl_music_subspace(rsl_handle h, const void* sigs, long long n, int M, int num_sources, const void* steer_c128,
                       int G, void* spec);
int rsl_esprit_subspace(rsl_handle h, const void* sigs, long long n, int M, int num_sources, double esprit_scale,
                        void* deg);

/* a19  RobustAngleEstimator.compute_angle_confidence (robust_angle_estimation.py:88-138) for n
 *     (cell, grid index) pairs.  steer_c128 f64 [G][M][2] and steer_phase f64 [G][M] = np.angle(a) are
 *     device copies of the host fp64 tables.  conf f64 [n]. */
int rsl_confidence(rsl_handle h, const void* rds, int A, int S, int C, const void* c_frame, const void* c_rc,
                   long long n, const void* gidx, const void* steer_c128, const void* steer_phase, void* conf);

/* a25-a29  VelocitySolver.two_step_optimization / solve_velocity (velocity_solver.py:65-355): exact
 *     box-constrained LS for (v_x, v_y) per segment (segments = frames).  az f64 [N] radians, or (when gidx
 *     i32 [N] is non-null) az = az_table[gidx] with az_table f64 [G], G <= 2048; y f64 [N]
 *     observed phase, amask u32 [N] (nullable; multiplicity = popcount), seg i64 [F+1] (device; bounds
 *     clamped to n = N, the arrays' length: a capacity-sized list that overflowed ends at its capacity),
 *     k = 4 pi dt / lambda, ridge >= 0, bounds4 (host) = {vx_lo, vx_hi, vy_lo, vy_hi};
 *     out f64 [F, 8] = {vx, vy, cost, rmse, max_residual, n, det, 0}; resid/pred f64 [N] nullable. */
int rsl_velocity(rsl_handle h, const void* az, const void* gidx, const void* az_table, int G, const void* y,
                 const void* amask, const void* seg, long long n, int F, double k, double ridge, const double* bounds4,
                 void* out, void* resid, void* pred);

/* a3-a6  SignalPreprocessor.dechirp_signal / apply_window / remove_dc / process_chirp (dechirp.py:85-166):
 *     out[r, s] = in[r, s] * table[s], then (dc != 0) minus the row's complex mean.  in/out c64 [rows, S]. */
int rsl_preprocess_rows(rsl_handle h, const void* in, long long rows, int S, const void* table, int dc, void* out);

/* a25, a27  compute_phase_difference_model + cost_function (velocity_solver.py:65-176), general 6-DoF:
 *     pred = k (v + w x p).d, d = (cos el cos az, cos el sin az, sin el); pos f64 [n,3], ang f64 [n,2],
 *     x f64 [6] = (v, w) (device); y f64 [n] nullable; wrap != 0 wraps residuals to (-pi, pi]
 *     (velocity_solver_improved.py:255); cost f64 [1] = sum r^2 + ridge |x|^2 (nullable). */
int rsl_phase_model(rsl_handle h, const void* pos, const void* ang, long long n, const void* x, double k,
                    const void* y, int wrap, double ridge, void* pred, void* resid, void* cost);

/* a28  two_step_optimization (velocity_solver.py:178-307) for arbitrary (pos, ang): exact box-constrained
 *     linear least squares over nv = 3 (v, w = 0) or 6 (v, w) unknowns (BVLS active set, fp64).
 *     lo/hi f64 [nv] device bounds; out f64 [nv + 1] = x, cost. */
int rsl_bvls(rsl_handle h, const void* pos, const void* ang, long long n, const void* y, double k, int nv,
             double ridge, const void* lo, const void* hi, void* out);

/* a30  ImprovedVelocitySolver.associate_targets_across_frames (velocity_solver_improved.py:74-129): for each
 *     current target in order, the nearest unused previous target with Euclidean distance < thr (ties to the
 *     lowest index).  cur_xy f64 [nc][2], prev_xy f64 [np][2] (device), scratch u32 [ceil(np/32)],
 *     match i32 [nc] (-1 = none), dist f64 [nc]. */
int rsl_associate(rsl_handle h, const void* cur_xy, int nc, const void* prev_xy, int np, double thr, void* scratch,
                  void* match, void* dist);

/* configs[3] per-frame pattern, peak selection of RobustAngleEstimator.process_targets_robust
 *     (robust_angle_estimation.py:362-369: power_db > thr_db, stable sort by power_db descending, first kmax), for
 *     every cube k of a batch at once.  entry_base i64 [ncube + 1], e_coord u32 / e_pdb f32 [entry_cap] are the
 *     chain's compacted entries (rsl_peak_emit); kmax <= 256.  Outputs (device, slots k * kmax + r): sel_entry i32
 *     (global entry index, -1 past the selection), sel_frame i32 (= k) and sel_rc i32 (range_bin * C + doppler_bin;
 *     a DoA cell list for rsl_doa / rsl_confidence / rsl_cell_extras), sel_n i32 [ncube] = selected count.  The
 *     selection is in the reference's order: power descending, ties in entry (antenna -> range -> Doppler) order. */
int rsl_peak_topk(rsl_handle h, const void* entry_base, long long entry_cap, int ncube, const void* e_coord,
                  const void* e_pdb, double thr_db, int kmax, int C, void* sel_entry, void* sel_frame, void* sel_rc,
                  void* sel_n);

/* configs[3] per-frame pattern: CompleteRadarScenesAnalyzer._create_target_associations
 *     (radarscenes_complete_analysis.py:274-305) for every frame of a batch at once.  Targets of frame f are
 *     [off[f], off[f+1]) of the concatenated f64 arrays range_m, az_rad and s0 (c128: the first component of each
 *     target's spatial signature); off i64 [nframes + 1] on the device.  For target i of frame f > 0: the target j of
 *     frame f-1 with the smallest sqrt((r_i - r_j)^2 + (az_i - az_j)^2), strict '<' against the running minimum and
 *     against thr (first minimum wins; previous targets may be matched many times), in exact float64.  Outputs
 *     [off[nframes]]: match i32 (index within frame f-1, -1 = none; always -1 in frame 0), dist f64, phase f64 =
 *     angle(s0_i * conj(s0_j)) (:296; 0 where unmatched). */
int rsl_associate_nearest(rsl_handle h, const void* range_m, const void* az_rad, const void* s0, const void* off,
                          int nframes, long long ntargets, double thr, void* match, void* dist, void* phase);

/* a30, a31  wrapped-phase ego-motion solve: minimises sum_i wrap(y_i - k J_i.x)^2 + R(x) over the box
 *     [lo6, hi6] (host), J_i = [d_i, p_i x d_i] from pos f64 [n][3] and ang f64 [n][2] (az, el).
 *     mode 0: R = 0.01 |v|^2 + 0.01 |w|^2 (velocity_solver_improved.py:223-266);
 *     mode 1: the piecewise penalties of advanced_velocity_optimization.py:153-223 with weight w, max
 *             velocity vmax, max angular velocity wmax and previous motion prev f64 [6] (device, nullable).
 *     nv = 3 (w fixed at 0; step 1) or 6.  Multi-start projected Gauss-Newton from a grid_n x grid_n grid
 *     over (v_x, v_y) plus nextra extra starts extra f64 [nextra][6] (device), iters iterations each;
 *     out f64 [8] (device) = {x[6], cost, start index}.  scratch >= rsl_wrapped_scratch_bytes(n, grid_n, nextra). */
long long rsl_wrapped_scratch_bytes(long long n, int grid_n, int nextra);

int rsl_wrapped_solve(rsl_handle h, const void* pos, const void* ang, long long n, const void* y, double k, int mode,
                      double w, double vmax, double wmax, const void* prev, const double* lo6, const double* hi6,
                      int nv, int grid_n, const void* extra, int nextra, int iters, void* scratch,
                      long long scratch_bytes, void* out);

/* a30, a31  the same minimisation with a dense multi-start global stage (a heuristic checked by cost <= the reference
 *     DE on recorded runs; it does not guarantee that every basin of the wrapped cost is entered).
 *     Stage 1: projected 2-D Gauss-Newton in (x0, x1) = (v_x, v_y) from every point of a grid with the given spacing
 *     (a fraction of the wrap period 2 pi / k; ceil(width / spacing) points per axis, at most 32768) over
 *     [lo6[0], hi6[0]] x [lo6[1], hi6[1]], with x[2..5] held at base6 (host, clipped to the box; the regulariser's
 *     optimum for them); stage 2: the nv-D Gauss-Newton of rsl_wrapped_solve from the nbest best stage-1 minima
 *     (1..1024) and the extra starts.  out as rsl_wrapped_solve (start index = position among the stage-2 starts).
 *     scratch >= rsl_wrapped_search_scratch_bytes(n, lo6, hi6, spacing, nbest, nextra). */
long long rsl_wrapped_search_scratch_bytes(long long n, const double* lo6, const double* hi6, double spacing,
                                           int nbest, int nextra);
int rsl_wrapped_search(rsl_handle h, const void* pos, const void* ang, long long n, const void* y, double k, int mode,
                       double w, double vmax, double wmax, const void* prev, const double* lo6, const double* hi6,
                       int nv, const double* base6, double spacing, int nbest, const void* extra, int nextra, int iters,
                       void* scratch, long long scratch_bytes, void* out);

/* L4 trajectory  PoseIntegrator.integrate_translational_velocity / integrate_angular_velocity
 *     (pose_integration.py:67-167) as block-wide fp64 prefix scans over one frame block.
 *     vel f64 [F][vstride] (first nv <= 3 components used, missing ones 0), omega f64 [F][ostride] (nullable = 0),
 *     timestamps f64 [F] (nullable: uniform dt); method 0 = trapezoidal, 1 = euler.
 *     pos f64 [F][3] (pos[0] = 0), quat f64 [F][4] (w,x,y,z; quat[0] = identity),
 *     summary f64 [16] (nullable) = {pos[F-1], quat[F-1], v[F-1], v[0], omega[F-1]} for stitching blocks. */
int rsl_traj_scan(rsl_handle h, const void* vel, int vstride, int nv, const void* omega, int ostride,
                  const void* timestamps, double dt, long long F, int method, void* pos, void* quat, void* summary);
/* Stitch: pos[i] += base[0:3], quat[i] = base[3:7] (x) quat[i]; base f64 [7] (device). */
int rsl_traj_apply(rsl_handle h, void* pos, void* quat, long long F, const void* base);
/* Stitch consecutive frame blocks (e.g. one per GPU after an all-gather of the 16-double summaries, rank order):
 *     state f64 [16] (device, in/out) = {pos (3), quat (4), v_last (3), omega_last (3), started, 0, 0}, zero-init
 *     except quat = (1,0,0,0) (plus the initial pose); base f64 [7] (device, out) = offset of block `rank`. */
int rsl_traj_stitch(rsl_handle h, const void* summaries, int R, int rank, double dt, int method, void* state,
                    void* base);
/* uniform_filter1d(x[:, c], size, mode='nearest') per column (pose_integration.py:105-109); x, out f64 [F][ncol]. */
int rsl_traj_smooth(rsl_handle h, const void* x, long long F, int ncol, int size, void* out);

/* SURVEY §8f #3 (evaluation half)  PoseErrorEvaluator (evaluation/compute_pose_error.py:51-361), fp64.
 *     Poses f64 [n][7] = (x, y, z, q0, q1, q2, q3) with q read as scipy quaternions (scalar LAST, normalised), as the
 *     reference's Rotation.from_quat reads them.  scratch >= rsl_pose_error_scratch_bytes(n, nlen) (device).
 *     rsl_pose_align (align_trajectories :51-96 + compute_ape :171-236): align f64 [32] = position rotation R (9,
 *       row-major; Umeyama :98-140), translation t (3), orientation rotation Rq (9; Rotation.mean of gt * est^-1,
 *       :142-169), its quaternion (4, x y z w, w >= 0), scale_factor = cbrt(det R) (1), the two position means (6);
 *       aligned f64 [n][7]; ape_err f64 [3][n] = position, orientation, combined errors; ape_stats f64 [3][5]
 *       (nullable) = {rmse, mean, std, max, n} per series.
 *     rsl_pose_rte (compute_rte :238-306 on rsl_pose_align's aligned poses): lengths f64 [nlen] (device) segment
 *       lengths; err f64 [nlen][n]: the first counts[l] entries of row l are the segment errors (the valid starts of a
 *       positive length are a prefix); counts u64 [nlen]; stats f64 [nlen][5] as above. */
long long rsl_pose_error_scratch_bytes(long long n, int nlen);
int rsl_pose_align(rsl_handle h, const void* est, const void* gt, long long n, void* scratch, void* align,
                   void* aligned, void* ape_err, void* ape_stats);
int rsl_pose_rte(rsl_handle h, const void* aligned, const void* gt, long long n, const void* lengths, int nlen,
                 void* scratch, void* err, void* counts, void* stats);

/* SURVEY §8f #2  FMCWRadarSimulator.synthesize_frame (scripts/simulate_raw.py:147-221) at batch scale.
 *     rsl_synth_pattern: the deterministic part, which does not depend on the chirp index, as fp64 complex
 *       pattern [A][S] (device) from scatterers f64 [n][4] = {range m, azimuth rad, rcs dBsm, radial velocity m/s}
 *       (device); antenna_spacing <= 0 means lambda / 2; S = samples per chirp (int(chirp_duration * fs)).
 *     rsl_synth_cube: cube c64 [F][A][C][S] = pattern + sqrt(noise_power) (n1 + j n2) with standard normal n1, n2
 *       from Philox-4x32-10 (key = seed, counter = global sample index / 2 counted from frame frame0) and
 *       Box-Muller; S must be even.  Frame blocks generated separately (e.g. one per rank) equal one large call. */
int rsl_synth_pattern(rsl_handle h, const void* scatterers, int n, int A, int S, double fc, double bandwidth,
                      double chirp_duration, double antenna_spacing, void* pattern);
int rsl_synth_cube(rsl_handle h, const void* pattern, int F, int A, int C, int S, double noise_power,
                   unsigned long long seed, long long frame0, void* cube);

#ifdef __cplusplus
}
#endif
#endif /* RSL_H */
