// rsl_synth.hip — device synthetic FMCW cube generator.  gfx950 / CDNA4.
//
// Replaces FMCWRadarSimulator.synthesize_frame (reference scripts/simulate_raw.py:147-221) at batch scale.
// The reference signal of a scatterer does not depend on the chirp index (simulate_raw.py:190-209: the chirp
// loop variable enters nothing), so a frame is  sig[a, c, s] = pattern[a, s] + noise[a, c, s]:
//   * k_synth_pattern: the deterministic [A, S] pattern in fp64 with the reference's operations in its order
//     (simulate_raw.py:102-145 and :165-209): t = linspace(0, Tc, S), chirp(t) = exp(j 2 pi (fc t + k t^2 / 2)),
//     per scatterer delay = 2 r / c, amp = sqrt(10^(rcs/10)) / (4 pi r^2), Doppler phase 4 pi vr fc / c,
//     antenna phase 2 pi pos sin(az) / lambda, beat = chirp(t - delay) conj(chirp(t)) where
//     0 <= t - delay <= Tc, accumulated over scatterers in order; invalid scatterers (r <= 0 or non-finite)
//     are skipped (simulate_raw.py:181).
//   * k_synth_cube: cube[f, a, c, s] = pattern[a, s] + sqrt(noise_power) (n1 + j n2), n1, n2 standard normal
//     (simulate_raw.py:216-218), from a counter-based generator: Philox-4x32-10 keyed by the 64-bit seed with
//     counter = (global sample index of the pair) -> 4 uniforms -> Box-Muller -> 2 complex samples.  Any frame
//     range is reproducible from (seed, frame0) alone, so ranks generate their own frame blocks.
// Output c64 [F, A, C, S]; 16-B coalesced stores (two samples per lane).  The noise is statistically, not
// bitwise, the reference's (numpy's legacy Mersenne-Twister stream cannot be split across lanes).
#include "rsl_common.h"
#include "rsl_internal.h"

namespace rsl {

namespace {
constexpr double kC = 3e8;  // simulate_raw.py:24 (scipy.constants are not used by the reference simulator)
constexpr double kPi = 3.14159265358979323846;
}  // namespace

__global__ __launch_bounds__(256) void k_synth_pattern(const double* __restrict__ sc, int n, int A, int S, double fc,
                                                       double bandwidth, double Tc, double d,
                                                       double2* __restrict__ pattern) {
  // numpy's operation order: no fused multiply-adds (the chirp phase reaches 2.5e7 rad, where one rounding step
  // moves the sample by ~1e-9 relative)
#pragma clang fp contract(off)
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)A * S) return;
  const int a = (int)(idx / S), s = (int)(idx - (long)a * S);
  const double lam = kC / fc;
  const double k = bandwidth / Tc;
  const double pos = (double)a * d;
  // numpy.linspace(0, Tc, S): arange(S) * step, the last sample exactly Tc
  const double t = (S > 1) ? (s == S - 1 ? Tc : (double)s * (Tc / (double)(S - 1))) : 0.0;
  double rs, rcs_;
  sincos(2.0 * kPi * (fc * t + 0.5 * k * (t * t)), &rs, &rcs_);  // ref = chirp(t)
  double acc_r = 0.0, acc_i = 0.0;
  for (int q = 0; q < n; ++q) {
    const double r = sc[4 * q], az = sc[4 * q + 1], rcs = sc[4 * q + 2], vr = sc[4 * q + 3];
    if (!(r > 0.0) || !isfinite(r) || !isfinite(az) || !isfinite(rcs) || !isfinite(vr)) continue;
    const double delay = 2.0 * r / kC;
    const double amp = sqrt(pow(10.0, rcs / 10.0)) / (4.0 * kPi * (r * r));
    const double dph = 4.0 * kPi * vr * fc / kC;
    double as, ac;
    sincos(dph + 2.0 * kPi * pos * sin(az) / lam, &as, &ac);
    const double aph_r = amp * ac, aph_i = amp * as;
    const double td = t - delay;
    if (!(td >= 0.0 && td <= Tc)) continue;
    double bs, bc;
    sincos(2.0 * kPi * (fc * td + 0.5 * k * (td * td)), &bs, &bc);  // chirp(td)
    const double bb_r = bc * rcs_ + bs * rs, bb_i = bs * rcs_ - bc * rs;  // chirp(td) * conj(ref)
    acc_r += aph_r * bb_r - aph_i * bb_i;
    acc_i += aph_r * bb_i + aph_i * bb_r;
  }
  pattern[idx] = make_double2(acc_r, acc_i);
}

// Philox-4x32-10 (Salmon et al., SC'11): counter ctr, key (k0, k1).
RSL_DEV uint4 philox4x32_10(uint4 ctr, unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * ctr.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * ctr.z;
    ctr = make_uint4((unsigned)(p1 >> 32) ^ ctr.y ^ k0, (unsigned)p1, (unsigned)(p0 >> 32) ^ ctr.w ^ k1, (unsigned)p0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return ctr;
}

// uint32 -> (0, 1]: (x + 1) 2^-32 (never 0, so log() is finite)
RSL_DEV float u01(unsigned x) { return ((float)x + 1.0f) * 2.3283064365386963e-10f; }

__global__ __launch_bounds__(256) void k_synth_cube(const double2* __restrict__ pattern, long long npair, int A,
                                                    int C, int S, float sigma, unsigned k0, unsigned k1,
                                                    long long g0, float4* __restrict__ cube) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long cs = (long long)C * S;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < npair; p += stride) {
    const long long g = 2 * p;  // first sample of the pair within this launch; S even: same (f, a, c) row
    const long long gg = g0 + g;  // global sample index (counter)
    const uint4 x = philox4x32_10(make_uint4((unsigned)(gg >> 1), (unsigned)(gg >> 33), 0u, 0u), k0, k1);
    const int s = (int)(g % S);
    const int a = (int)((g / cs) % A);
    const double2 q0 = pattern[(size_t)a * S + s], q1 = pattern[(size_t)a * S + s + 1];
    // Box-Muller on the hardware transcendentals: v_log_f32 is log2, v_sin/v_cos_f32 take revolutions
    // (sin(2 pi u) in one instruction); ~1e-6 absolute on unit normals, far below the noise's own scale
    constexpr float kM2Ln2 = -1.38629436111989061883f;  // -2 ln 2
    const float r0 = sigma * __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(x.x)));
    const float r1 = sigma * __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(x.z)));
    const float u1 = u01(x.y), u3 = u01(x.w);
    const float s0 = __builtin_amdgcn_sinf(u1), c0 = __builtin_amdgcn_cosf(u1);
    const float s1 = __builtin_amdgcn_sinf(u3), c1 = __builtin_amdgcn_cosf(u3);
    cube[p] = make_float4((float)q0.x + r0 * c0, (float)q0.y + r0 * s0, (float)q1.x + r1 * c1,
                          (float)q1.y + r1 * s1);
  }
}

hipError_t launch_synth_pattern(hipStream_t st, const double* sc, int n, int A, int S, double fc, double bandwidth,
                                double Tc, double d, double2* pattern) {
  const long tot = (long)A * S;
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_synth_pattern, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, sc, n, A, S, fc,
                     bandwidth, Tc, d, pattern);
  return hipGetLastError();
}

hipError_t launch_synth_cube(hipStream_t st, const double2* pattern, int F, int A, int C, int S, double noise_power,
                             unsigned long long seed, long long frame0, float2* cube) {
  const long long npair = (long long)F * A * C * S / 2;
  if (npair <= 0) return hipSuccess;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  long long nb = (npair + 255) / 256;
  if (nb > (long long)ncu * 16) nb = (long long)ncu * 16;
  const long long g0 = frame0 * (long long)A * C * S;
  hipLaunchKernelGGL(k_synth_cube, dim3((unsigned)nb), dim3(256), 0, st, pattern, npair, A, C, S,
                     (float)sqrt(noise_power), (unsigned)seed, (unsigned)(seed >> 32), g0,
                     reinterpret_cast<float4*>(cube));
  return hipGetLastError();
}

}  // namespace rsl
