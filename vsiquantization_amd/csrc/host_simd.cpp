// host_simd.cpp — AVX-512 loops of the host (CPU-tensor) path (interface and exactness
// contract in host_simd.h).  Host C++ only, compiled by the system C++ compiler with
// -ffp-contract=off; the AVX-512 functions carry their own target attribute, so the file
// runs on any x86-64 host and k_host.hip calls them only when available() says so.
// Reference formulas: quantizers/uniform.py:55,95 (fake quant), :47-56 + the autograd
// of the chain (learnable backward), observers/minmax.py:42-47 + quantization_manager.py
// :66-68 (observer statistics).
#include "host_simd.h"

#include <immintrin.h>

#include <cmath>

#define VSIQ_AVX512 __attribute__((target("avx512f,avx512bw,avx512vl")))

namespace vsiq {
namespace simd {

bool available() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
         __builtin_cpu_supports("avx512vl");
}

namespace {

constexpr int W = 16;

VSIQ_AVX512 inline __m512 act16(__m512 v, int relu) {
  if (!relu) return v;
  const __mmask16 neg = _mm512_cmp_ps_mask(v, _mm512_setzero_ps(), _CMP_LT_OQ);   // NaN, -0.0 kept
  return _mm512_mask_mov_ps(v, neg, _mm512_setzero_ps());
}

VSIQ_AVX512 inline __m512 neg16(__m512 v) {   // exact sign flip (0 - v would turn -(+0) into +0)
  return _mm512_castsi512_ps(_mm512_xor_si512(_mm512_castps_si512(v), _mm512_set1_epi32(INT32_MIN)));
}

VSIQ_AVX512 inline __m512d lo8(__m512 v) { return _mm512_cvtps_pd(_mm512_castps512_ps256(v)); }
VSIQ_AVX512 inline __m512d hi8(__m512 v) {
  return _mm512_cvtps_pd(_mm256_castpd_ps(_mm512_extractf64x4_pd(_mm512_castps_pd(v), 1)));
}

// the scalar twins (chunk tails), k_host.hip's loops term for term
inline float act1(float v, int relu) { return relu && v < 0.0f ? 0.0f : v; }

inline float fq1(float x, float s, float z, float lo, float hi, int discrete, uint8_t *m, uint8_t *code) {
  float u = x / s;
  u = u + z;
  const float r = std::rint(u);
  const float q = r < lo ? lo : (r > hi ? hi : r);
  *m = r >= lo && r <= hi;
  *code = q == q ? (uint8_t)((int)q & 0xff) : 0;
  return discrete ? q : (q - z) * s;
}

// 16 f64 lane accumulators of one sum, folded in lane order
struct Lanes {
  __m512d a, b;   // lanes 0-7, 8-15
};

VSIQ_AVX512 inline double fold(const Lanes &l) {
  alignas(64) double t[W];
  _mm512_store_pd(t, l.a);
  _mm512_store_pd(t + 8, l.b);
  double s = 0.0;
  for (int k = 0; k < W; ++k) s += t[k];
  return s;
}

}  // namespace

VSIQ_AVX512 void observe(const float *x, int64_t n, int relu, double out[6]) {
  __m512 mn = _mm512_set1_ps(INFINITY), mx = _mm512_set1_ps(-INFINITY);
  __m512i nan = _mm512_setzero_si512();
  Lanes sa{_mm512_setzero_pd(), _mm512_setzero_pd()}, s1 = sa, s2 = sa;
  int64_t i = 0;
  for (; i + W <= n; i += W) {
    const __m512 v = act16(_mm512_loadu_ps(x + i), relu);
    nan = _mm512_mask_add_epi32(nan, _mm512_cmp_ps_mask(v, v, _CMP_UNORD_Q), nan, _mm512_set1_epi32(1));
    mn = _mm512_mask_mov_ps(mn, _mm512_cmp_ps_mask(v, mn, _CMP_LT_OQ), v);
    mx = _mm512_mask_mov_ps(mx, _mm512_cmp_ps_mask(v, mx, _CMP_GT_OQ), v);
    const __m512d d0 = lo8(v), d1 = hi8(v);
    sa.a = _mm512_add_pd(sa.a, _mm512_abs_pd(d0));
    sa.b = _mm512_add_pd(sa.b, _mm512_abs_pd(d1));
    s1.a = _mm512_add_pd(s1.a, d0);
    s1.b = _mm512_add_pd(s1.b, d1);
    s2.a = _mm512_add_pd(s2.a, _mm512_mul_pd(d0, d0));
    s2.b = _mm512_add_pd(s2.b, _mm512_mul_pd(d1, d1));
  }
  alignas(64) float tmn[W], tmx[W];
  alignas(64) int32_t tn[W];
  _mm512_store_ps(tmn, mn);
  _mm512_store_ps(tmx, mx);
  _mm512_store_si512((__m512i *)tn, nan);
  float fmn = INFINITY, fmx = -INFINITY;
  double cnt = 0.0;
  for (int k = 0; k < W; ++k) {
    fmn = tmn[k] < fmn ? tmn[k] : fmn;
    fmx = tmx[k] > fmx ? tmx[k] : fmx;
    cnt += (double)tn[k];
  }
  double da = fold(sa), d1 = fold(s1), d2 = fold(s2);
  for (; i < n; ++i) {
    const float v = act1(x[i], relu);
    if (v != v) {
      cnt += 1.0;
    } else {
      fmn = v < fmn ? v : fmn;
      fmx = v > fmx ? v : fmx;
    }
    const double d = (double)v;
    da += std::fabs(d);
    d1 += d;
    d2 += d * d;
  }
  out[0] = fmn; out[1] = fmx; out[2] = cnt; out[3] = da; out[4] = d1; out[5] = d2;
}

VSIQ_AVX512 void fq(const float *x, float *y, uint8_t *codes, uint8_t *mask, int64_t n, int relu, float s, float z,
                    float lo, float hi, int discrete) {
  const __m512 vs = _mm512_set1_ps(s), vz = _mm512_set1_ps(z), vlo = _mm512_set1_ps(lo), vhi = _mm512_set1_ps(hi);
  int64_t i = 0;
  for (; i + W <= n; i += W) {
    const __m512 v = act16(_mm512_loadu_ps(x + i), relu);
    const __m512 u = _mm512_add_ps(_mm512_div_ps(v, vs), vz);
    const __m512 r = _mm512_roundscale_ps(u, _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC);
    __m512 q = _mm512_mask_mov_ps(r, _mm512_cmp_ps_mask(r, vlo, _CMP_LT_OQ), vlo);
    q = _mm512_mask_mov_ps(q, _mm512_cmp_ps_mask(r, vhi, _CMP_GT_OQ), vhi);
    _mm512_storeu_ps(y + i, discrete ? q : _mm512_mul_ps(_mm512_sub_ps(q, vz), vs));
    if (mask) {
      const __mmask16 m = _mm512_cmp_ps_mask(r, vlo, _CMP_GE_OQ) & _mm512_cmp_ps_mask(r, vhi, _CMP_LE_OQ);
      _mm_storeu_si128((__m128i *)(mask + i), _mm_maskz_set1_epi8(m, 1));
    }
    if (codes)   // NaN converts to 0x80000000: low byte 0, like the scalar q == q test
      _mm_storeu_si128((__m128i *)(codes + i), _mm512_cvtepi32_epi8(_mm512_cvttps_epi32(q)));
  }
  for (; i < n; ++i) {
    uint8_t m, c;
    y[i] = fq1(act1(x[i], relu), s, z, lo, hi, discrete, &m, &c);
    if (mask) mask[i] = m;
    if (codes) codes[i] = c;
  }
}

VSIQ_AVX512 void ste(const float *g, const uint8_t *mask, const float *pre, float *gx, int64_t n, int relu, float s) {
  const __m512 vs = _mm512_set1_ps(s), zero = _mm512_setzero_ps();
  int64_t i = 0;
  for (; i + W <= n; i += W) {
    const __m128i mb = _mm_loadu_si128((const __m128i *)(mask + i));
    const __mmask16 m = _mm_test_epi8_mask(mb, mb);
    __m512 o = _mm512_div_ps(_mm512_maskz_mov_ps(m, _mm512_mul_ps(_mm512_loadu_ps(g + i), vs)), vs);
    if (relu) o = _mm512_mask_mov_ps(o, _mm512_cmp_ps_mask(_mm512_loadu_ps(pre + i), zero, _CMP_LE_OQ), zero);
    _mm512_storeu_ps(gx + i, o);
  }
  for (; i < n; ++i) {
    const float o = (mask[i] ? g[i] * s : 0.0f) / s;   // MulBackward0, ClampBackward1, DivBackward0
    gx[i] = relu && pre[i] <= 0.0f ? 0.0f : o;
  }
}

VSIQ_AVX512 void lsq(const float *g, const float *x, float *gx, int64_t n, int relu, float s, float z, float lo,
                     float hi, int zp_learn, double out[2]) {
  const __m512 vs = _mm512_set1_ps(s), vz = _mm512_set1_ps(z), vlo = _mm512_set1_ps(lo), vhi = _mm512_set1_ps(hi);
  const __m512 zero = _mm512_setzero_ps();
  Lanes st{_mm512_setzero_pd(), _mm512_setzero_pd()}, sz = st;
  int64_t i = 0;
  for (; i + W <= n; i += W) {
    const __m512 xr = _mm512_loadu_ps(x + i), gv = _mm512_loadu_ps(g + i);
    const __m512 xa = act16(xr, relu);
    const __m512 u = _mm512_div_ps(xa, vs);
    const __m512 r = _mm512_roundscale_ps(_mm512_add_ps(u, vz), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC);
    __m512 q = _mm512_mask_mov_ps(r, _mm512_cmp_ps_mask(r, vlo, _CMP_LT_OQ), vlo);
    q = _mm512_mask_mov_ps(q, _mm512_cmp_ps_mask(r, vhi, _CMP_GT_OQ), vhi);
    const __mmask16 m = _mm512_cmp_ps_mask(r, vlo, _CMP_GE_OQ) & _mm512_cmp_ps_mask(r, vhi, _CMP_LE_OQ);
    const __m512 gq = _mm512_mul_ps(gv, vs);
    const __m512 gm = _mm512_maskz_mov_ps(m, gq);
    const __m512 t1 = _mm512_mul_ps(gv, _mm512_sub_ps(q, vz));
    const __m512 t2 = _mm512_mul_ps(neg16(gm), _mm512_div_ps(u, vs));
    st.a = _mm512_add_pd(st.a, _mm512_add_pd(lo8(t1), lo8(t2)));
    st.b = _mm512_add_pd(st.b, _mm512_add_pd(hi8(t1), hi8(t2)));
    if (zp_learn) {
      const __m512 ng = neg16(gq);
      sz.a = _mm512_add_pd(sz.a, _mm512_add_pd(lo8(gm), lo8(ng)));
      sz.b = _mm512_add_pd(sz.b, _mm512_add_pd(hi8(gm), hi8(ng)));
    }
    __m512 o = _mm512_div_ps(gm, vs);
    if (relu) o = _mm512_mask_mov_ps(o, _mm512_cmp_ps_mask(xr, zero, _CMP_LE_OQ), zero);
    _mm512_storeu_ps(gx + i, o);
  }
  double t = fold(st), zs = fold(sz);
  for (; i < n; ++i) {   // k_host.hip vsiq_host_lsq_bwd_f32, term by term
    const float xa = act1(x[i], relu);
    const float u = xa / s;
    const float r = std::rint(u + z);
    const float q = r < lo ? lo : (r > hi ? hi : r);
    const bool m = r >= lo && r <= hi;
    const float gq = g[i] * s;
    const float gm = m ? gq : 0.0f;
    const float t1 = g[i] * (q - z);
    const float xs = u / s;
    const float t2 = (-gm) * xs;
    t += (double)t1 + (double)t2;
    if (zp_learn) zs += (double)gm + (double)(-gq);
    const float o = gm / s;
    gx[i] = relu && x[i] <= 0.0f ? 0.0f : o;
  }
  out[0] = t;
  out[1] = zs;
}

}  // namespace simd
}  // namespace vsiq
