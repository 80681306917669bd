/*
 * oracle/silu_ref.c -- TEST INFRASTRUCTURE (never linked into the product).
 *
 * C restatement of what the reference's F.silu (modules/fused.py:133, on CPU tensors)
 * computes on its host: PyTorch 2.10's CPU silu_kernel / silu_backward_kernel
 * (aten/src/ATen/native/cpu/Activation.cpp, under cpu_kernel_vec):
 *
 *   vectorized loop, 2 vectors per step:  x / (1 + Sleef_expf_u10(-x))
 *   scalar remainder of every chunk:      x / (1 + expf(-x))        (glibc libm)
 *   backward (same split):                (g * sig) * fma(x, 1 - sig, 1),
 *                                         sig = 1 / (1 + exp(-x))
 *
 * Third-party algorithms restated here (absent from /root/reference, pinned by the
 * torch build the reference runs on; licenses and attributions in NOTICE -- SLEEF is
 * Boost-1.0, Copyright Naoki Shibata and contributors; glibc is LGPL-2.1-or-later,
 * Copyright Free Software Foundation, Inc.):
 *   - SLEEF 3.x xexpf (sleefsimdsp.c), the FMA build torch links for AVX2 / AVX-512;
 *   - glibc >= 2.27 expf (sysdeps/ieee754/flt-32/e_expf.c + e_exp2f_data.c), the FMA
 *     ifunc variant x86-64 selects on FMA-capable CPUs.
 * Chunking: TensorIterator runs serially below GRAIN_SIZE = 32768 elements or on one
 * thread; otherwise at::parallel_for (ParallelOpenMP.h) splits [0, n) into
 * nt = min(threads, ceil(n / 32768)) chunks of ceil(n / nt), and each chunk runs
 * vectorized_loop (cpu/Loops.h) over len - len % W elements, W = 2 x the vector width.
 *
 * Pinned by tests/test_silu_oracle.py against torch.nn.functional.silu and
 * torch.ops.aten.silu_backward on the reference host (several thread counts and sizes;
 * tests/golden/pin_silu.py runs the exhaustive 2^32 comparison of both exps).
 *
 * Build: gcc -O2 -ffp-contract=off -fno-builtin -shared -fPIC (oracle/build_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static double bits_d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t d_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

/* SLEEF xexpf: Cody-Waite reduction by ln2, degree-6 polynomial, 2-step ldexp */
float oracle_sleef_expf(float d) {
  const float R_LN2f = 1.442695040888963407359924681001892137426645954152985934135449406931f;
  const float L2Uf = 0.693145751953125f, L2Lf = 1.428606765330187045e-06f;
  float fq = rintf(d * R_LN2f);
  if (!(fq > -1000.0f)) fq = -1000.0f;     /* NaN / huge: the result is replaced below */
  if (fq > 1000.0f) fq = 1000.0f;
  const int q = (int)fq;
  float s = fmaf((float)q, -L2Uf, d);
  s = fmaf((float)q, -L2Lf, s);
  float u = 0.000198527617612853646278381f;
  u = fmaf(u, s, 0.00139304355252534151077271f);
  u = fmaf(u, s, 0.00833336077630519866943359f);
  u = fmaf(u, s, 0.0416664853692054748535156f);
  u = fmaf(u, s, 0.166666671633720397949219f);
  u = fmaf(u, s, 0.5f);
  u = 1.0f + fmaf(s * s, u, s);
  const int h = q >> 1;
  if (d >= -104.0f && d <= 100.0f)
    u = (u * bits_f((uint32_t)(h + 0x7f) << 23)) * bits_f((uint32_t)(q - h + 0x7f) << 23);
  if (d < -104.0f) u = 0.0f;
  if (d > 100.0f) u = INFINITY;
  if (isnan(d)) u = d;
  return u;
}

/* glibc expf: x * 32/ln2 = k + r, 2^(k/32) from the table, cubic in r, all in double */
float oracle_glibc_expf(float x) {
  static uint64_t tab[32];
  static int init;
  if (!init) {   /* tab[i] = bits(2^(i/32)) - (i << 47), 2^(i/32) correctly rounded */
    static const uint64_t T[32] = {
        0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL,
        0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL,
        0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL,
        0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL,
        0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL,
        0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL,
        0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL,
        0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL};
    memcpy(tab, T, sizeof T);
    init = 1;
  }
  const uint32_t abstop = (f_bits(x) >> 20) & 0x7ff;
  if (abstop >= (f_bits(88.0f) >> 20)) {
    if (f_bits(x) == f_bits(-INFINITY)) return 0.0f;
    if (abstop >= (f_bits(INFINITY) >> 20)) return x + x;
    if (x > 0x1.62e42ep6f) return INFINITY;
    if (x < -0x1.9fe368p6f) return 0.0f;
  }
  const double N = 32.0;
  const double InvLn2N = 0x1.71547652b82fep+0 * N, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / N / N / N, C1 = 0x1.ebfce50fac4f3p-3 / N / N,
               C2 = 0x1.62e42ff0c52d6p-1 / N;
  const double xd = (double)x;
  double kd = fma(InvLn2N, xd, SHIFT);
  const uint64_t ki = d_bits(kd);
  kd -= SHIFT;
  const double r = fma(InvLn2N, xd, -kd);
  const double s = bits_d(tab[ki % 32] + (ki << 47));
  const double z = fma(C0, r, C1);
  double y = fma(C2, r, 1.0);
  y = fma(z, r * r, y);
  return (float)(y * s);
}

/* scalar[i] = 1 where torch's kernel takes the scalar path for element i */
static void scalar_map(unsigned char *sc, int64_t n, int w, int threads) {
  memset(sc, 0, (size_t)n);
  if (w <= 0 || n <= 0) return;
  int64_t nt = 1;
  if (n >= 32768 && threads > 1) {
    nt = (n + 32767) / 32768;
    if (nt > threads) nt = threads;
  }
  const int64_t ch = (n + nt - 1) / nt;
  for (int64_t b = 0; b < n; b += ch) {
    const int64_t e = b + ch < n ? b + ch : n;
    for (int64_t i = e - (e - b) % w; i < e; ++i) sc[i] = 1;
  }
}

void oracle_silu_scalar_map(unsigned char *sc, int64_t n, int w, int threads) { scalar_map(sc, n, w, threads); }

void oracle_silu_fwd(const float *x, float *y, int64_t n, int w, int threads, unsigned char *sc) {
  scalar_map(sc, n, w, threads);
  for (int64_t i = 0; i < n; ++i) {
    const float e = sc[i] ? oracle_glibc_expf(-x[i]) : oracle_sleef_expf(-x[i]);
    y[i] = x[i] / (1.0f + e);
  }
}

void oracle_silu_bwd(const float *g, const float *x, float *gx, int64_t n, int w, int threads,
                     unsigned char *sc) {
  scalar_map(sc, n, w, threads);
  for (int64_t i = 0; i < n; ++i) {
    const float e = sc[i] ? oracle_glibc_expf(-x[i]) : oracle_sleef_expf(-x[i]);
    const float sig = 1.0f / (1.0f + e);
    gx[i] = (g[i] * sig) * fmaf(x[i], 1.0f - sig, 1.0f);
  }
}

void oracle_exp_both(const float *x, float *ys, float *yg, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    ys[i] = oracle_sleef_expf(x[i]);
    yg[i] = oracle_glibc_expf(x[i]);
  }
}
