// rsl_common.h — shared device helpers for the radar-slam MI355X kernels (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSL_DEV __device__ __forceinline__

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Complex arithmetic on the 2-wide vector inside float2 (an aligned 64-bit register pair): the compiler emits one
// v_pk_add_f32 per complex add and v_pk_mul_f32 + v_pk_fma_f32 (with operand swizzles) per complex multiply, instead of
// scalar ops plus the register-pair shuffles its SLP vectoriser added around the scalar form.  Same roundings:
// re = fma(a.x, b.x, -(a.y b.y)), im = fma(a.x, b.y, a.y b.x).
typedef float rsl_f2v __attribute__((ext_vector_type(2)));
// popcount of the bits of m below this lane, popc(m & ((1 << lane) - 1)), as v_mbcnt_lo + v_mbcnt_hi (2 VALU; the
// compiler emits two ANDs and two v_bcnt for the popcount form)
RSL_DEV int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
RSL_DEV rsl_f2v cv(float2 a) { return __builtin_bit_cast(rsl_f2v, a); }
RSL_DEV float2 cf(rsl_f2v v) { return __builtin_bit_cast(float2, v); }
RSL_DEV float2 cadd(float2 a, float2 b) { return cf(cv(a) + cv(b)); }
RSL_DEV float2 csub(float2 a, float2 b) { return cf(cv(a) - cv(b)); }
RSL_DEV float2 cmul(float2 a, float2 b) {
  const rsl_f2v va = cv(a), vb = cv(b);
  return cf(__builtin_elementwise_fma(va.yy, (rsl_f2v){-vb.y, vb.x}, va.xx * vb));
}
// multiply by -i : (x + iy)(-i) = y - ix
RSL_DEV float2 cmul_mi(float2 a) { return cf(cv(a).yx * (rsl_f2v){1.f, -1.f}); }
RSL_DEV float cabs2(float2 a) { return fmaf(a.x, a.x, a.y * a.y); }

// ------------------------------------------------------------------------------------
// Compile-time FFT plan: N = prod(radices), radices from {8,4,2,5,3,7}.
// ------------------------------------------------------------------------------------
struct FftPlan {
  int n;
  int r[16];
  int ns[16];  // product of radices before stage s (Stockham "Ns")
};

constexpr FftPlan make_plan(int N) {
  FftPlan p{0, {}, {}};
  int m = N;
  int ns = 1;
  // powers of two: radix 8 stages, with one radix-16 stage where it removes a stage (N = 16 * 8^k: 128, 1024)
  // or two where they replace 8 * 8 * 4 (N = 256); every stage is an LDS round trip
  int lg = 0;
  while ((1 << lg) < N) ++lg;
  if ((1 << lg) == N && N >= 128) {
    const int n16 = (lg % 3 == 1) ? 1 : (N == 256 ? 2 : 0);
    for (int q = 0; q < n16; ++q) {
      p.r[p.n] = 16;
      p.ns[p.n] = ns;
      ns *= 16;
      m /= 16;
      p.n++;
    }
  }
  const int order[6] = {8, 4, 2, 5, 3, 7};
  for (int oi = 0; oi < 6; ++oi) {
    int R = order[oi];
    while (m > 1 && m % R == 0) {
      p.r[p.n] = R;
      p.ns[p.n] = ns;
      ns *= R;
      m /= R;
      p.n++;
    }
  }
  if (m != 1) p.n = -1;  // unsupported prime factor
  return p;
}

constexpr bool fft_supported(int N) { return N >= 2 && make_plan(N).n > 0; }

// Forward DFT of R points held in registers (natural order in/out), sign exp(-2 pi i nk/R).
template <int R>
struct Dft;

template <>
struct Dft<2> {
  RSL_DEV static void run(float2* v) {
    float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  }
};

template <>
struct Dft<4> {
  RSL_DEV static void run(float2* v) {
    float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    float2 t2 = cadd(v[1], v[3]), t3 = cmul_mi(csub(v[1], v[3]));
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
  }
};

template <>
struct Dft<8> {
  RSL_DEV static void run(float2* v) {
    const float h = 0.70710678118654752440f;
    // DIF radix-2 split: even outputs from a_n + a_{n+4}, odd from (a_n - a_{n+4}) W8^n
    float2 e[4], o[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      e[n] = cadd(v[n], v[n + 4]);
      o[n] = csub(v[n], v[n + 4]);
    }
    // W8^1 = (h, -h), W8^2 = -i, W8^3 = (-h, -h)
    o[1] = make_float2(h * (o[1].x + o[1].y), h * (o[1].y - o[1].x));
    o[2] = cmul_mi(o[2]);
    o[3] = make_float2(h * (o[3].y - o[3].x), -h * (o[3].x + o[3].y));
    Dft<4>::run(e);
    Dft<4>::run(o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = e[k];
      v[2 * k + 1] = o[k];
    }
  }
};

// 16 points as 4 x 4: n = 4 n1 + n2, k = k1 + 4 k2; DFT4 over n1, twiddle W16^(n2 k1), DFT4 over n2.
template <>
struct Dft<16> {
  RSL_DEV static void run(float2* v) {
    const float h = 0.70710678118654752440f, c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
    float2 y[4][4];  // y[n2][k1]
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
      float2 t[4] = {v[n2], v[4 + n2], v[8 + n2], v[12 + n2]};
      Dft<4>::run(t);
#pragma unroll
      for (int k1 = 0; k1 < 4; ++k1) y[n2][k1] = t[k1];
    }
    // W16^e, e = n2 k1: 1 = (c, -s), 2 = (h, -h), 3 = (s, -c), 4 = -i, 6 = (-h, -h), 9 = (-c, s)
    y[1][1] = cmul(y[1][1], make_float2(c1, -s1));
    y[1][2] = make_float2(h * (y[1][2].x + y[1][2].y), h * (y[1][2].y - y[1][2].x));
    y[1][3] = cmul(y[1][3], make_float2(s1, -c1));
    y[2][1] = make_float2(h * (y[2][1].x + y[2][1].y), h * (y[2][1].y - y[2][1].x));
    y[2][2] = cmul_mi(y[2][2]);
    y[2][3] = make_float2(h * (y[2][3].y - y[2][3].x), -h * (y[2][3].x + y[2][3].y));
    y[3][1] = cmul(y[3][1], make_float2(s1, -c1));
    y[3][2] = make_float2(h * (y[3][2].y - y[3][2].x), -h * (y[3][2].x + y[3][2].y));
    y[3][3] = cmul(y[3][3], make_float2(-c1, s1));
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      float2 t[4] = {y[0][k1], y[1][k1], y[2][k1], y[3][k1]};
      Dft<4>::run(t);
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = t[k2];
    }
  }
};

// Generic small-prime DFT (R = 3, 5, 7) with exact literal roots of unity.
template <int R>
struct Roots;
template <>
struct Roots<3> {
  RSL_DEV static float c(int m) {
    const float t[3] = {1.f, -0.5f, -0.5f};
    return t[m];
  }
  RSL_DEV static float s(int m) {
    const float t[3] = {0.f, -0.86602540378443864676f, 0.86602540378443864676f};
    return t[m];
  }
};
template <>
struct Roots<5> {
  RSL_DEV static float c(int m) {
    const float t[5] = {1.f, 0.30901699437494742410f, -0.80901699437494742410f, -0.80901699437494742410f,
                        0.30901699437494742410f};
    return t[m];
  }
  RSL_DEV static float s(int m) {
    const float t[5] = {0.f, -0.95105651629515357212f, -0.58778525229247312917f, 0.58778525229247312917f,
                        0.95105651629515357212f};
    return t[m];
  }
};
template <>
struct Roots<7> {
  RSL_DEV static float c(int m) {
    const float t[7] = {1.f, 0.62348980185873353053f, -0.22252093395631440429f, -0.90096886790241912624f,
                        -0.90096886790241912624f, -0.22252093395631440429f, 0.62348980185873353053f};
    return t[m];
  }
  RSL_DEV static float s(int m) {
    const float t[7] = {0.f, -0.78183148246802980871f, -0.97492791218182360702f, -0.43388373911755812048f,
                        0.43388373911755812048f, 0.97492791218182360702f, 0.78183148246802980871f};
    return t[m];
  }
};

template <int R>
struct Dft {
  RSL_DEV static void run(float2* v) {
    float2 out[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      float2 acc = v[0];
#pragma unroll
      for (int n = 1; n < R; ++n) {
        const int m = (n * k) % R;
        const float2 w = make_float2(Roots<R>::c(m), Roots<R>::s(m));
        acc = cadd(acc, cmul(v[n], w));
      }
      out[k] = acc;
    }
#pragma unroll
    for (int k = 0; k < R; ++k) v[k] = out[k];
  }
};

// LDS position of FFT point x in a padded row: one pad slot after every 8 points.  Radix-8 Stockham writes
// (stride 8 points = 64 B per lane) and the 8-lane-group pattern of the second stage then land on distinct
// banks; unpadded they are 4- to 8-way bank conflicts.
// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (observed placement, speed only), so
// logical tile L = (b % 8) * (n / 8) + b / 8 gives each XCD a contiguous run of tiles, dispatched back to back:
// tiles sharing halo cache lines then meet in the same 4 MiB L2.  The n % 8 tail keeps the identity order.
// Inclusive scan of an int over the 64 lanes of a wave in DPP: row_shr 1 / 2 / 4 / 8 (bound_ctrl: 0 past the row
// start), then row_bcast:15 into rows 1 and 3 and row_bcast:31 into rows 2 and 3.  Six VALU ops, no LDS round trips
// (the __shfl_up form is six ds_bpermute).  Every lane must be active.
RSL_DEV int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
  return x;
}

RSL_DEV long xcd_tile(long b, long n) {
  const long n8 = n & ~7L;
  return b < n8 ? (b & 7) * (n8 >> 3) + (b >> 3) : b;
}

RSL_DEV constexpr int lp(int x) { return x + (x >> 3); }
// Padded row length for N points.
constexpr int lp_row(int N) { return N + (N + 7) / 8; }
// The same with the padding optional (P = false: plain rows, for kernels whose FFT is not LDS-bound and that
// need the smaller tile for residency)
template <bool P>
RSL_DEV constexpr int lpp(int x) { return P ? x + (x >> 3) : x; }
template <bool P>
constexpr int lp_rowp(int N) { return P ? lp_row(N) : N; }

// One Stockham autosort stage over ROWS independent rows of N points held in LDS
// (row stride LD complex, padded positions).  tw[k] = exp(-2 pi i k / N), k < N (fp64-accurate table).
// In place: every thread reads its butterflies' inputs, the block syncs, then writes.
template <int N, int R, int NS, int ROWS, int NT, int LD, bool PADTW, bool PAD>
RSL_DEV void fft_stage(float2* buf, const float2* tw, int tid) {
  constexpr int NB = N / R;
  constexpr int TOT = ROWS * NB;
  constexpr int PER = (TOT + NT - 1) / NT;
  float2 v[PER][R];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = tid + q * NT;
    if ((TOT % NT) == 0 || idx < TOT) {
      const int row = idx / NB, j = idx - (idx / NB) * NB;
      const float2* src = buf + row * LD;
      if constexpr (NB % 8 == 0 || !PAD) {  // lp(j + r NB) = lp(j) + r (NB + NB/8): immediate LDS offsets
        const float2* s0 = src + lpp<PAD>(j);
#pragma unroll
        for (int r = 0; r < R; ++r) v[q][r] = s0[r * lpp<PAD>(NB)];
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) v[q][r] = src[lp(j + r * NB)];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int idx = tid + q * NT;
    if ((TOT % NT) == 0 || idx < TOT) {
      const int row = idx / NB, j = idx - (idx / NB) * NB;
      const int k = j % NS;
      if (NS > 1) {
        constexpr int STEP = N / (NS * R);
#pragma unroll
        for (int r = 1; r < R; ++r) v[q][r] = cmul(v[q][r], tw[PADTW ? lp(r * k * STEP) : r * k * STEP]);
      }
      Dft<R>::run(v[q]);
      float2* dst = buf + row * LD;
      const int o = (j / NS) * NS * R + k;
      if constexpr (!PAD) {
        float2* d0 = dst + o;
#pragma unroll
        for (int r = 0; r < R; ++r) d0[r * NS] = v[q][r];
      } else if constexpr (NS == 1 && (R & (R - 1)) == 0 && (R <= 8 || R % 8 == 0)) {
        // o = j R (a multiple of 8 or of R): lp(o + r) = lp(o) + r + r / 8
        float2* d0 = dst + lp(o);
#pragma unroll
        for (int r = 0; r < R; ++r) d0[r + (r >> 3)] = v[q][r];
      } else if constexpr (NS % 8 == 0) {
        float2* d0 = dst + lp(o);
#pragma unroll
        for (int r = 0; r < R; ++r) d0[r * (NS + NS / 8)] = v[q][r];
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) dst[lp(o + r * NS)] = v[q][r];
      }
    }
  }
  __syncthreads();
}

template <int N, int S, int ROWS, int NT, int LD, bool PADTW, bool PAD>
RSL_DEV void fft_run(float2* buf, const float2* tw, int tid) {
  constexpr FftPlan P = make_plan(N);
  if constexpr (S < P.n) {
    fft_stage<N, P.r[S], P.ns[S], ROWS, NT, LD, PADTW, PAD>(buf, tw, tid);
    fft_run<N, S + 1, ROWS, NT, LD, PADTW, PAD>(buf, tw, tid);
  }
}

// Forward N-point FFT of ROWS rows in LDS (padded positions, see lp()).  Caller must __syncthreads() before.
// PADTW: the twiddle table is stored at padded positions lp(k) (spreads the strided twiddle reads of the
// later stages over the LDS banks)
// PAD = false: rows hold points at plain positions (row stride LD >= N).
template <int N, int ROWS, int NT, int LD, bool PADTW = false, bool PAD = true>
RSL_DEV void fft_rows(float2* buf, const float2* tw, int tid) {
  static_assert(make_plan(N).n > 0, "unsupported FFT size");
  static_assert(LD >= lp_rowp<PAD>(N), "row stride too small for the row layout");
  fft_run<N, 0, ROWS, NT, LD, PADTW, PAD>(buf, tw, tid);
}

// ESPRIT closed form (reference angle_estimation.py:178-225) on a unit-norm fp64 signature s (A antennas):
// svd of X = [s[:-1], s[1:]] -> U[:,0] = u proportional to X v, v = principal eigenvector of the 2x2 Hermitian
// X^H X; pinv(U1) U2 = u[:-1]^H u[1:] / u[:-1]^H u[:-1] = (nr + i ni) / dd.  The scale/phase of u cancels.
template <int MA, typename T>
RSL_DEV void esprit_phi(const T (&sr)[MA], const T (&si)[MA], int A, T& nr, T& ni, T& dd) {
  T a = 0, cc = 0, br = 0, bi = 0;
#pragma unroll
  for (int m = 0; m + 1 < MA; ++m) {
    if (m + 1 < A) {
      a += sr[m] * sr[m] + si[m] * si[m];
      cc += sr[m + 1] * sr[m + 1] + si[m + 1] * si[m + 1];
      br += sr[m] * sr[m + 1] + si[m] * si[m + 1];  // conj(x0) * x1
      bi += sr[m] * si[m + 1] - si[m] * sr[m + 1];
    }
  }
  const T hd = T(0.5) * (a - cc);
  const T l1 = T(0.5) * (a + cc) + sqrt(hd * hd + br * br + bi * bi);
  T v0r, v0i, v1r, v1i;
  if (a >= cc) {  // v = [l1 - c, conj(b)]
    v0r = l1 - cc; v0i = 0.0; v1r = br; v1i = -bi;
  } else {        // v = [b, l1 - a]
    v0r = br; v0i = bi; v1r = l1 - a; v1i = 0.0;
  }
  // u_m = v0 s_m + v1 s_{m+1}, m < A-1 ; phi = sum conj(u_m) u_{m+1} / sum |u_m|^2, m < A-2
  nr = 0; ni = 0; dd = 0;
  T upr = 0, upi = 0;
#pragma unroll
  for (int m = 0; m + 1 < MA; ++m) {
    if (m + 1 < A) {
      const T ur = v0r * sr[m] - v0i * si[m] + v1r * sr[m + 1] - v1i * si[m + 1];
      const T ui = v0r * si[m] + v0i * sr[m] + v1r * si[m + 1] + v1i * sr[m + 1];
      if (m > 0) {
        nr += upr * ur + upi * ui;
        ni += upr * ui - upi * ur;
        dd += upr * upr + upi * upi;
      }
      upr = ur;
      upi = ui;
    }
  }
}
