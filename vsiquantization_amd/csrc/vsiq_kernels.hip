// vsiq_kernels.hip — MI355X (gfx950 / CDNA4) kernels for VSIQuantization's
// fake-quantize hot path, exported through the C ABI in include/vsiq.h.
//
// Design (DESIGN.md has the full rationale and roofline numbers):
//   * Everything here is HBM-bound elementwise + reduction work: no MFMA.
//     Loads/stores are 16 B per lane (float4) wherever the layout allows, one
//     read and one write of every element per pass, streamed with nontemporal
//     hints (the tensors are touched once per pass).
//   * fp32 arithmetic is IEEE and in the reference's operation order
//     (quantizers/uniform.py:55,95): true division x/s (correctly rounded; the
//     build uses -fhip-fp32-correctly-rounded-divide-sqrt, -ffp-contract=off,
//     denormals kept), rint (half-to-even), NaN-propagating clamp that keeps
//     -0.0.  This is bit-identical to the reference's PyTorch CPU kernels.
//   * qparams (observers/minmax.py:49-74) are computed in float64 on the
//     device from the fp32 min/max, so no `.item()` host round trip is needed.
//   * The straight-through mask travels between forward and backward as ONE BIT
//     per element (ballot words), not a byte: 1/32 of the fp32 traffic.
//   * Reductions are deterministic: fixed per-thread order (grid depends only
//     on n), fixed tree in the workgroup, partials reduced in block order by the
//     last workgroup to arrive (agent-scope release/acquire hand-off,
//     cdna_hip_programming.md G16).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "vsiq.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kWaves = kBlock / kWave;
constexpr int kMaxReduceGrid = 2048;   // partial slots per reducing launch
constexpr int kPartials = 8;           // doubles per partial record

typedef float f4 __attribute__((ext_vector_type(4)));

// tuning knobs (vsiq_set_tuning); -1 / 0 = automatic
struct Tuning {
  int pc_rows_per_block = 0;   // K3 rows per workgroup (0 = auto)
  int nontemporal = 1;         // nt hints on streamed loads/stores
  int flat_grid_cap = 8192;    // max workgroups of the flat streaming kernels
  int lsq_prefetch = 1;        // K4 software prefetch of the next tile
};
Tuning g_tune;

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ----------------------------------------------------------------------------
// Correctly rounded fp32 division by a uniform divisor without v_div_* .
//
// The compiler's IEEE sequence (v_div_scale / v_rcp / v_div_fmas / v_div_fixup)
// funnels every division through VCC, which serialises all divisions of a wave;
// the hot kernels divide 1-3 times per element by the SAME scale.  With
// r = RN(1/b) computed once, two Newton-Markstein corrections give RN(a/b):
//   q0 = RN(a r); q1 = RN(q0 + RN(a - q0 b) r)     (q1 is faithful)
//   q2 = RN(q1 + (a - q1 b) r)                     (Markstein: a - q1 b exact,
//                                                   q2 = RN(a/b))
// valid without underflow/overflow, i.e. for |a|, |b| in [2^-63, 2^63]; a == 0
// returns a*r (signed zero, as IEEE); any other a (NaN, inf, tiny, huge) takes
// the IEEE division.  vsiq_selftest_div() checks this exhaustively against the
// IEEE division for all 2^32 dividends (tests/test_gpu_parity.py).
// ----------------------------------------------------------------------------
struct FastDiv {
  float b, r;
  int fast;   // b in the safe range (uniform)
};

__device__ __forceinline__ FastDiv make_fastdiv(float b) {
  FastDiv d;
  d.b = b;
  d.r = 1.0f / b;   // IEEE, once per thread
  const uint32_t ub = __float_as_uint(b) & 0x7fffffffu;
  d.fast = (ub - 0x20000000u) <= 0x3f000000u;   // |b| in [2^-63, 2^63]
  return d;
}

__device__ __forceinline__ float fdiv(float a, const FastDiv &d) {
  if (!d.fast) return a / d.b;
  const float q0 = a * d.r;
  const float e0 = __builtin_fmaf(-q0, d.b, a);
  const float q1 = __builtin_fmaf(e0, d.r, q0);
  const float e1 = __builtin_fmaf(-q1, d.b, a);
  float q = __builtin_fmaf(e1, d.r, q1);
  const uint32_t ua = __float_as_uint(a) & 0x7fffffffu;
  if (ua == 0u) q = q0;                                  // +-0 / b
  else if ((ua - 0x20000000u) > 0x3f000000u) q = a / d.b;   // rare: IEEE path
  return q;
}

// ----------------------------------------------------------------------------
// element arithmetic (quantizers/uniform.py:95, 55)
// ----------------------------------------------------------------------------
struct QP {
  float s, z, lo, hi;
  int discrete;
  FastDiv d;
};

__device__ __forceinline__ float fq_round(float x, const QP &p) {
  float u = fdiv(x, p.d);   // fp32 true division x / fp32(scale), correctly rounded
  u = u + p.z;              // + fp32(zero_point); -0.0 + 0.0 -> +0.0 like torch.add
  return __builtin_rintf(u);   // torch.round: half to even
}

// torch.clamp(v, lo, hi): NaN propagates, -0.0 survives
__device__ __forceinline__ float fq_clamp(float r, float lo, float hi) {
  return r < lo ? lo : (r > hi ? hi : r);
}

__device__ __forceinline__ uint32_t fq_code_byte(float q) {
  // int8 (sym) / uint8 (asym) share the low byte of the integer; NaN -> 0
  return (q == q) ? (uint32_t)((int)q) & 0xffu : 0u;
}

struct Elem {
  float y;
  uint32_t code;
  bool m;
};

__device__ __forceinline__ Elem fq_elem(float x, const QP &p) {
  const float r = fq_round(x, p);
  const float q = fq_clamp(r, p.lo, p.hi);
  Elem e;
  e.y = p.discrete ? q : (q - p.z) * p.s;
  e.code = fq_code_byte(q);
  e.m = (r >= p.lo && r <= p.hi);   // ClampBackward1: inclusive, on the rounded value
  return e;
}

// where qparams come from (one struct, passed by value -> kernarg / SGPRs)
struct QPSrc {
  const double *qp;     // observer record [scale, zp, ...] or null
  const double *sdev;   // learnable f64 scale or null (then shost)
  const double *zdev;   // f64 zp on the device or null (then zhost)
  double shost, zhost;
  float lo, hi;
  int zround;           // learnable zp: clamp(rint(zp)) (uniform.py:98-102)
  int discrete;         // write clamp(round(x/s+zp)) itself (discreate_tensor) instead of y
};

__device__ __forceinline__ QP load_qp(const QPSrc &a) {
  double s, z;
  if (a.qp) {
    s = a.qp[VSIQ_QP_SCALE];
    z = a.qp[VSIQ_QP_ZP];
  } else {
    s = a.sdev ? *a.sdev : a.shost;
    z = a.zdev ? *a.zdev : a.zhost;
    if (a.zround) {
      // quantizers/uniform.py:98-102: clamp(round(zp), qmin, qmax) in f64, NaN propagates
      const double zr = __builtin_rint(z);
      z = zr < (double)a.lo ? (double)a.lo : (zr > (double)a.hi ? (double)a.hi : zr);
    }
  }
  QP p;
  p.s = (float)s;
  p.z = (float)z;
  p.lo = a.lo;
  p.hi = a.hi;
  p.discrete = a.discrete;
  p.d = make_fastdiv(p.s);
  return p;
}

// ----------------------------------------------------------------------------
// streamed memory access: 16 B per lane, optional nontemporal hint
// ----------------------------------------------------------------------------
template <bool NT>
__device__ __forceinline__ f4 ld4(const float *p) {
  const f4 *q = reinterpret_cast<const f4 *>(p);
  if (NT) return __builtin_nontemporal_load(q);
  return *q;
}
template <bool NT>
__device__ __forceinline__ void st4(float *p, f4 v) {
  f4 *q = reinterpret_cast<f4 *>(p);
  if (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// A group of 4 consecutive elements of a row starting at element 4*i.
// VEC: one 16-B access (row length % 4 == 0, 16-B aligned).  Otherwise 4 scalar
// accesses with per-element bounds ("virtual float4"); invalid lanes replicate
// element 0 so min/max/NaN see no fake values.
template <bool VEC, bool NT>
__device__ __forceinline__ f4 load_group(const float *row, int64_t i, int64_t len) {
  if (VEC) return ld4<NT>(row + 4 * i);
  const int64_t e = 4 * i;
  f4 v;
  v.x = row[e];
  v.y = e + 1 < len ? row[e + 1] : v.x;
  v.z = e + 2 < len ? row[e + 2] : v.x;
  v.w = e + 3 < len ? row[e + 3] : v.x;
  return v;
}

template <bool VEC, bool NT>
__device__ __forceinline__ void store_group(float *row, int64_t i, int64_t len, f4 v) {
  if (VEC) {
    st4<NT>(row + 4 * i, v);
    return;
  }
  const int64_t e = 4 * i;
  row[e] = v.x;
  if (e + 1 < len) row[e + 1] = v.y;
  if (e + 2 < len) row[e + 2] = v.z;
  if (e + 3 < len) row[e + 3] = v.w;
}

__device__ __forceinline__ int valid_in_group(int64_t i, int64_t len) {
  const int64_t r = len - 4 * i;
  return r >= 4 ? 4 : (r > 0 ? (int)r : 0);
}

// ----------------------------------------------------------------------------
// 1-bit straight-through masks (include/vsiq.h: mask layout)
//   row r owns words [r*W, (r+1)*W), W = 4*ceil(rowlen/256); element e of the
//   row -> chunk c = e/256, word 4c + (e%4), bit (e%256)/4.
// Thread with group index i (4 elements 4i..4i+3) in a wave whose 64 lanes hold
// groups 64c..64c+63: lane = i%64, and the four ballots ARE the chunk's words.
// ----------------------------------------------------------------------------
__host__ __device__ inline int64_t mask_words_per_row(int64_t rowlen) { return 4 * cdiv(rowlen, 256); }

__device__ __forceinline__ void store_mask_chunk(uint64_t *words, bool m0, bool m1, bool m2, bool m3) {
  const uint64_t b0 = __ballot(m0), b1 = __ballot(m1), b2 = __ballot(m2), b3 = __ballot(m3);
  const int lane = threadIdx.x % kWave;
  if (lane < 4) words[lane] = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
}

__device__ __forceinline__ uint32_t load_mask_nibble(const uint64_t *words, int lane) {
  const uint64_t w0 = words[0], w1 = words[1], w2 = words[2], w3 = words[3];
  return (uint32_t)((w0 >> lane) & 1u) | ((uint32_t)((w1 >> lane) & 1u) << 1) |
         ((uint32_t)((w2 >> lane) & 1u) << 2) | ((uint32_t)((w3 >> lane) & 1u) << 3);
}

// ----------------------------------------------------------------------------
// wave / block reductions (wave64)
// ----------------------------------------------------------------------------
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off, kWave));
  return v;
}

struct MinOp {
  __device__ float operator()(float a, float b) const { return fminf(a, b); }
};
struct MaxOp {
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
struct AddD {
  __device__ double operator()(double a, double b) const { return a + b; }
};
struct OrU {
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; }
};
struct AddU {
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};

// Last-workgroup-done hand-off.  Every block's thread 0 has stored its partial
// record; returns true (block-uniform) in the block that arrives last, after an
// agent-scope acquire so its plain loads see every other block's partials.
__device__ __forceinline__ bool arrive_last(uint32_t *counter) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == gridDim.x - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

// f64 qparams from the running min/max (observers/minmax.py:49-74).
// min_val <= 0 <= max_val always holds (state starts at 0/0, minmax.py:28-29).
__device__ __forceinline__ void minmax_qparams(double mn, double mx, int sym, double qden,
                                               double eps, double *scale, double *zp) {
  if (sym) {
    const double a = __builtin_fabs(mn), b = __builtin_fabs(mx);
    const double max_abs = b > a ? b : a;   // Python max(): first unless strictly greater
    *scale = max_abs / qden;
    *zp = 0.0;
  } else {
    const double s = (mx - mn) / qden;
    const double v = -mn / (s + eps);
    double z = __builtin_rint(v);           // Python round(): half to even
    if (!__builtin_isfinite(z)) z = __builtin_nan("");   // Python raises here
    if (z == 0.0) z = 0.0;                  // Python int 0 -> +0.0, never -0.0
    *scale = s;
    *zp = z;
  }
}

// Running-state update + qparams (observers/minmax.py:42-47 then :49-74).  A call
// whose tensor holds a NaN changes nothing: `nan < v` is False in Python.
__device__ __forceinline__ void observer_update(float cmn, float cmx, bool has_nan,
                                                float *run_minmax, double *qp_out, int sym,
                                                double qden, double eps) {
  float mn = 0.f, mx = 0.f;
  if (run_minmax) { mn = run_minmax[0]; mx = run_minmax[1]; }
  if (!has_nan) {
    if (cmn < mn) mn = cmn;
    if (cmx > mx) mx = cmx;
  }
  if (run_minmax) { run_minmax[0] = mn; run_minmax[1] = mx; }
  if (qp_out) {
    double s, z;
    minmax_qparams((double)mn, (double)mx, sym, qden, eps, &s, &z);
    qp_out[VSIQ_QP_SCALE] = s;
    qp_out[VSIQ_QP_ZP] = z;
    qp_out[VSIQ_QP_MIN] = mn;
    qp_out[VSIQ_QP_MAX] = mx;
  }
}

// ----------------------------------------------------------------------------
// K1: per-tensor fake-quant forward (flat, grid-stride over 4-element groups)
// ----------------------------------------------------------------------------
template <bool VEC, bool NT, bool CODES, bool MASK>
__global__ __launch_bounds__(kBlock) void k_fq_fwd(const float *__restrict__ x, float *__restrict__ y,
                                                   uint8_t *__restrict__ codes,
                                                   uint64_t *__restrict__ mask, int64_t n,
                                                   QPSrc src) {
  const QP p = load_qp(src);
  const int64_t ng = cdiv(n, 4);
  const int64_t stride = (int64_t)gridDim.x * kBlock;   // multiple of 64: lanes stay chunk-aligned
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i - threadIdx.x % kWave < ng;
       i += stride) {
    const bool in = i < ng;
    Elem e0{}, e1{}, e2{}, e3{};
    if (in) {
      const f4 v = load_group<VEC, NT>(x, i, n);
      e0 = fq_elem(v.x, p);
      e1 = fq_elem(v.y, p);
      e2 = fq_elem(v.z, p);
      e3 = fq_elem(v.w, p);
      f4 o;
      o.x = e0.y; o.y = e1.y; o.z = e2.y; o.w = e3.y;
      store_group<VEC, NT>(y, i, n, o);
      if (CODES) {
        const uint32_t c = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
        if (VEC) reinterpret_cast<uint32_t *>(codes)[i] = c;
        else
          for (int j = 0; j < valid_in_group(i, n); ++j) codes[4 * i + j] = (uint8_t)(c >> (8 * j));
      }
    }
    if (MASK) {
      const int nv = in ? valid_in_group(i, n) : 0;
      store_mask_chunk(mask + 4 * (i / kWave), e0.m && nv > 0, e1.m && nv > 1, e2.m && nv > 2,
                       e3.m && nv > 3);
    }
  }
}

// ----------------------------------------------------------------------------
// K2: per-tensor observer (min, max, NaN count, sum|x|, sum x, sum x^2)
// ----------------------------------------------------------------------------
struct ObsAcc {
  float mn, mx;
  uint32_t nan;
  double sa, s1, s2;
};

__device__ __forceinline__ void obs_init(ObsAcc &a) {
  a.mn = __builtin_inff();
  a.mx = -__builtin_inff();
  a.nan = 0;
  a.sa = a.s1 = a.s2 = 0.0;
}

// fminf/fmaxf skip NaN operands; NaNs are counted separately.  nv valid lanes.
__device__ __forceinline__ void obs_add4(ObsAcc &a, f4 v, int nv) {
  if (nv < 4) {   // tail group: replicate element 0 for min/max, zero for the sums
    const float z0 = v.x;
    v.y = nv > 1 ? v.y : z0;
    v.z = nv > 2 ? v.z : z0;
    v.w = nv > 3 ? v.w : z0;
  }
  a.mn = fminf(fminf(a.mn, v.x), fminf(fminf(v.y, v.z), v.w));
  a.mx = fmaxf(fmaxf(a.mx, v.x), fmaxf(fmaxf(v.y, v.z), v.w));
  const float wy = nv > 1 ? 1.f : 0.f, wz = nv > 2 ? 1.f : 0.f, ww = nv > 3 ? 1.f : 0.f;
  a.nan += (v.x != v.x) + (nv > 1 && v.y != v.y) + (nv > 2 && v.z != v.z) + (nv > 3 && v.w != v.w);
  // fp32 partial over the 4 lanes of the group, float64 across groups
  const float vy = v.y * wy, vz = v.z * wz, vw = v.w * ww;   // NaN*0 stays NaN: sums go NaN, fine
  const float pa = (__builtin_fabsf(v.x) + __builtin_fabsf(vy)) +
                   (__builtin_fabsf(vz) + __builtin_fabsf(vw));
  const float p1 = (v.x + vy) + (vz + vw);
  const double dx = v.x, dy = vy, dz = vz, dw = vw;
  a.sa += (double)pa;
  a.s1 += (double)p1;
  a.s2 += __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, dw * dw)));
}

__device__ __forceinline__ void obs_block_reduce(ObsAcc &a) {
  __shared__ float s_mn[kWaves], s_mx[kWaves];
  __shared__ uint32_t s_nan[kWaves];
  __shared__ double s_sa[kWaves], s_s1[kWaves], s_s2[kWaves];
  a.mn = wave_reduce(a.mn, MinOp());
  a.mx = wave_reduce(a.mx, MaxOp());
  a.nan = wave_reduce(a.nan, AddU());
  a.sa = wave_reduce(a.sa, AddD());
  a.s1 = wave_reduce(a.s1, AddD());
  a.s2 = wave_reduce(a.s2, AddD());
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) {
    s_mn[w] = a.mn; s_mx[w] = a.mx; s_nan[w] = a.nan;
    s_sa[w] = a.sa; s_s1[w] = a.s1; s_s2[w] = a.s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kWaves; ++i) {
      a.mn = fminf(a.mn, s_mn[i]); a.mx = fmaxf(a.mx, s_mx[i]); a.nan += s_nan[i];
      a.sa += s_sa[i]; a.s1 += s_s1[i]; a.s2 += s_s2[i];
    }
  }
  __syncthreads();
}

template <bool VEC, bool NT>
__global__ __launch_bounds__(kBlock) void k_observe(const float *__restrict__ x, int64_t n,
                                                    double *__restrict__ stats_out,
                                                    float *__restrict__ run_minmax,
                                                    double *__restrict__ qp_out, int sym,
                                                    double qden, double eps,
                                                    double *__restrict__ ws,
                                                    uint32_t *__restrict__ counter) {
  ObsAcc a;
  obs_init(a);
  const int64_t ng = cdiv(n, 4);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  constexpr int U = 4;
  for (int64_t base = t0; base < ng; base += stride * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * stride < ng) v[u] = load_group<VEC, NT>(x, base + u * stride, n);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * stride < ng) obs_add4(a, v[u], valid_in_group(base + u * stride, n));
  }
  obs_block_reduce(a);
  if (threadIdx.x == 0) {
    double *r = ws + (int64_t)blockIdx.x * kPartials;
    r[0] = a.mn; r[1] = a.mx; r[2] = (double)a.nan;
    r[3] = a.sa; r[4] = a.s1; r[5] = a.s2;
  }
  if (!arrive_last(counter)) return;

  // ---- epilogue in the last block: fixed-order combine of the partials ----
  obs_init(a);
  double nanc = 0.0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += kBlock) {
    const double *r = ws + (int64_t)b * kPartials;
    a.mn = fminf(a.mn, (float)r[0]);
    a.mx = fmaxf(a.mx, (float)r[1]);
    nanc += r[2];
    a.sa += r[3]; a.s1 += r[4]; a.s2 += r[5];
  }
  {
    __shared__ double s_nanc[kWaves];
    nanc = wave_reduce(nanc, AddD());
    if (threadIdx.x % kWave == 0) s_nanc[threadIdx.x / kWave] = nanc;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 1; i < kWaves; ++i) nanc += s_nanc[i];
  }
  obs_block_reduce(a);
  if (threadIdx.x == 0) {
    const double dn = (double)n;
    const bool has_nan = nanc > 0.0;
    if (stats_out) {
      stats_out[VSIQ_ST_MIN] = (double)a.mn;   // NaN-ignoring; see VSIQ_ST_NAN
      stats_out[VSIQ_ST_MAX] = (double)a.mx;
      stats_out[VSIQ_ST_NAN] = nanc;
      stats_out[VSIQ_ST_SUMABS] = a.sa;
      stats_out[VSIQ_ST_SUM] = a.s1;
      stats_out[VSIQ_ST_SUMSQ] = a.s2;
      stats_out[VSIQ_ST_N] = dn;
      // NaN inputs make torch's fp32 mean/std NaN as well
      const double mean = a.s1 / dn;
      const double var = (a.s2 - a.s1 * mean) / (dn - 1.0);
      stats_out[VSIQ_ST_MEANABS] = has_nan ? __builtin_nan("") : (double)(float)(a.sa / dn);
      stats_out[VSIQ_ST_MEAN] = has_nan ? __builtin_nan("") : (double)(float)mean;
      stats_out[VSIQ_ST_STD] = (has_nan || n < 2)
                                   ? __builtin_nan("")
                                   : (double)(float)__builtin_sqrt(var > 0.0 ? var : 0.0);
    }
    observer_update(a.mn, a.mx, has_nan, run_minmax, qp_out, sym, qden, eps);
    *counter = 0u;   // ready for the next stream-ordered launch
  }
}

// Finalize from an externally reduced stats record (multi-GPU: stats all-reduced
// over RCCL with MAX on [-min, max] and SUM on the counts, then this 1-lane kernel).
__global__ void k_observe_finalize(const double *__restrict__ stats, float *__restrict__ run_minmax,
                                   double *__restrict__ qp_out, int sym, double qden, double eps) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  observer_update((float)stats[VSIQ_ST_MIN], (float)stats[VSIQ_ST_MAX], stats[VSIQ_ST_NAN] > 0.0,
                  run_minmax, qp_out, sym, qden, eps);
}

// ----------------------------------------------------------------------------
// K3: per-channel observe + qparams + fake-quant.  A workgroup owns whole rows
//     (out-channels); a row is held in registers (NV groups of 4 per lane) so
//     it is read once and written once.  With several rows per workgroup the
//     next row's loads are issued before the current row is reduced and
//     stored, so a CU's reads of row k+1 overlap its writes of row k.
// ----------------------------------------------------------------------------
struct PCArgs {
  int64_t rows, rowlen;
  float *run_min, *run_max;
  double *scale_out, *zp_out;
  double *row_stats;   // [rows][3] sum|x|, sum x, sum x^2 (nullable) for qm.py:66-68
  int sym;
  float lo, hi;
  double qden, eps;
};

struct RowSums {
  double sa, s1, s2;
};

__device__ __forceinline__ void rowsums_add4(RowSums &r, f4 v, int nv) {
  const float vy = nv > 1 ? v.y : 0.f, vz = nv > 2 ? v.z : 0.f, vw = nv > 3 ? v.w : 0.f;
  const float pa = (__builtin_fabsf(v.x) + __builtin_fabsf(vy)) +
                   (__builtin_fabsf(vz) + __builtin_fabsf(vw));
  const float p1 = (v.x + vy) + (vz + vw);
  const double dx = v.x, dy = vy, dz = vz, dw = vw;
  r.sa += (double)pa;
  r.s1 += (double)p1;
  r.s2 += __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, dw * dw)));
}

// Row reduction -> running state -> f64 qparams, returned to every lane.
// LDS partials are double-buffered by `par`, so one barrier per row suffices.
template <bool STATS>
__device__ __forceinline__ QP pc_row_qparams(float mn, float mx, uint32_t nan, RowSums rs,
                                             float rmn, float rmx, int64_t row, int par,
                                             const PCArgs &a) {
  __shared__ float s_mn[2][kWaves], s_mx[2][kWaves];
  __shared__ uint32_t s_nan[2][kWaves];
  __shared__ double s_rs[2][3][kWaves];
  mn = wave_reduce(mn, MinOp());
  mx = wave_reduce(mx, MaxOp());
  nan = wave_reduce(nan, OrU());
  if (STATS) {
    rs.sa = wave_reduce(rs.sa, AddD());
    rs.s1 = wave_reduce(rs.s1, AddD());
    rs.s2 = wave_reduce(rs.s2, AddD());
  }
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) {
    s_mn[par][w] = mn; s_mx[par][w] = mx; s_nan[par][w] = nan;
    if (STATS) { s_rs[par][0][w] = rs.sa; s_rs[par][1][w] = rs.s1; s_rs[par][2][w] = rs.s2; }
  }
  __syncthreads();
  mn = s_mn[par][0]; mx = s_mx[par][0]; nan = s_nan[par][0];
#pragma unroll
  for (int i = 1; i < kWaves; ++i) {
    mn = fminf(mn, s_mn[par][i]); mx = fmaxf(mx, s_mx[par][i]); nan |= s_nan[par][i];
  }
  if (!nan) {                         // minmax.py:44-47, strict compares
    if (mn < rmn) rmn = mn;
    if (mx > rmx) rmx = mx;
  }
  double s, z;
  minmax_qparams((double)rmn, (double)rmx, a.sym, a.qden, a.eps, &s, &z);
  if (threadIdx.x == 0) {
    a.run_min[row] = rmn;
    a.run_max[row] = rmx;
    a.scale_out[row] = s;
    a.zp_out[row] = z;
    if (STATS) {
      double sa = s_rs[par][0][0], s1 = s_rs[par][1][0], s2 = s_rs[par][2][0];
      for (int i = 1; i < kWaves; ++i) { sa += s_rs[par][0][i]; s1 += s_rs[par][1][i]; s2 += s_rs[par][2][i]; }
      a.row_stats[row * 3 + 0] = sa;
      a.row_stats[row * 3 + 1] = s1;
      a.row_stats[row * 3 + 2] = s2;
    }
  }
  QP p;
  p.s = (float)s;
  p.z = (float)z;
  p.lo = a.lo;
  p.hi = a.hi;
  p.discrete = 0;
  p.d = make_fastdiv(p.s);
  return p;
}

template <int NV, bool VEC, bool NT>
__device__ __forceinline__ void pc_load_row(f4 (&v)[NV], const float *x, int64_t row, const PCArgs &a) {
  const float *xr = x + row * a.rowlen;
  const int64_t ng = cdiv(a.rowlen, 4);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * kBlock;
    if (i < ng) v[k] = load_group<VEC, NT>(xr, i, a.rowlen);
  }
}

template <int NV, bool VEC, bool NT, bool STATS, bool MASK, bool CODES>
__device__ __forceinline__ void pc_process_row(const f4 (&v)[NV], float rmn, float rmx,
                                               int64_t row, int par, float *__restrict__ y,
                                               uint8_t *__restrict__ codes,
                                               uint64_t *__restrict__ mask, const PCArgs &a) {
  const int64_t ng = cdiv(a.rowlen, 4);
  float mn = __builtin_inff(), mx = -__builtin_inff();
  uint32_t nan = 0;
  RowSums rs{0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * kBlock;
    if (i < ng) {
      const f4 w = v[k];   // invalid tail lanes already replicate element 0
      mn = fminf(mn, fminf(fminf(w.x, w.y), fminf(w.z, w.w)));
      mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
      nan |= (w.x != w.x) | (w.y != w.y) | (w.z != w.z) | (w.w != w.w);
      if (STATS) rowsums_add4(rs, w, VEC ? 4 : valid_in_group(i, a.rowlen));
    }
  }
  const QP p = pc_row_qparams<STATS>(mn, mx, nan, rs, rmn, rmx, row, par, a);
  if (!y) return;
  float *yr = y + row * a.rowlen;
  uint64_t *mr = MASK ? mask + row * mask_words_per_row(a.rowlen) : nullptr;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * kBlock;
    // whole waves past the row end skip; a partially valid wave still ballots
    if (i - threadIdx.x % kWave >= ng) continue;
    const bool in = i < ng;
    Elem e0{}, e1{}, e2{}, e3{};
    if (in) {
      e0 = fq_elem(v[k].x, p); e1 = fq_elem(v[k].y, p);
      e2 = fq_elem(v[k].z, p); e3 = fq_elem(v[k].w, p);
      f4 o;
      o.x = e0.y; o.y = e1.y; o.z = e2.y; o.w = e3.y;
      store_group<VEC, NT>(yr, i, a.rowlen, o);
      if (CODES) {
        const uint32_t c = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
        uint8_t *cr = codes + row * a.rowlen;
        if (VEC) reinterpret_cast<uint32_t *>(cr)[i] = c;
        else
          for (int j = 0; j < valid_in_group(i, a.rowlen); ++j) cr[4 * i + j] = (uint8_t)(c >> (8 * j));
      }
    }
    if (MASK) {
      const int nv = in ? valid_in_group(i, a.rowlen) : 0;
      store_mask_chunk(mr + 4 * (i / kWave), e0.m && nv > 0, e1.m && nv > 1, e2.m && nv > 2,
                       e3.m && nv > 3);
    }
  }
}

// Persistent over rows b, b+G, b+2G, ... with a one-row register prefetch.
template <int NV, bool VEC, bool NT, bool STATS, bool MASK, bool CODES>
__global__ __launch_bounds__(kBlock) void k_pc_observe_fq(const float *__restrict__ x,
                                                          float *__restrict__ y,
                                                          uint8_t *__restrict__ codes,
                                                          uint64_t *__restrict__ mask, PCArgs a) {
  const int64_t G = gridDim.x;
  int64_t row = blockIdx.x;
  f4 A[NV], B[NV];
  pc_load_row<NV, VEC, NT>(A, x, row, a);
  float amn = a.run_min[row], amx = a.run_max[row];
  int par = 0;
  while (true) {
    int64_t nxt = row + G;
    float bmn = 0.f, bmx = 0.f;
    if (nxt < a.rows) {
      pc_load_row<NV, VEC, NT>(B, x, nxt, a);
      bmn = a.run_min[nxt];
      bmx = a.run_max[nxt];
    }
    pc_process_row<NV, VEC, NT, STATS, MASK, CODES>(A, amn, amx, row, par, y, codes, mask, a);
    if (nxt >= a.rows) break;
    row = nxt;
    par ^= 1;
    nxt = row + G;
    if (nxt < a.rows) {
      pc_load_row<NV, VEC, NT>(A, x, nxt, a);
      amn = a.run_min[nxt];
      amx = a.run_max[nxt];
    }
    pc_process_row<NV, VEC, NT, STATS, MASK, CODES>(B, bmn, bmx, row, par, y, codes, mask, a);
    if (nxt >= a.rows) break;
    row = nxt;
    par ^= 1;
  }
}

// Rows too long for registers: two passes over the row (the second from L2).
template <bool VEC, bool NT>
__global__ __launch_bounds__(kBlock) void k_pc_observe_fq_long(const float *__restrict__ x,
                                                               float *__restrict__ y,
                                                               uint8_t *__restrict__ codes,
                                                               uint64_t *__restrict__ mask,
                                                               PCArgs a) {
  const int64_t row = blockIdx.x;
  const float *xr = x + row * a.rowlen;
  const int64_t ng = cdiv(a.rowlen, 4);
  float mn = __builtin_inff(), mx = -__builtin_inff();
  uint32_t nan = 0;
  RowSums rs{0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < ng; i += kBlock) {
    const f4 w = load_group<VEC, false>(xr, i, a.rowlen);
    mn = fminf(mn, fminf(fminf(w.x, w.y), fminf(w.z, w.w)));
    mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
    nan |= (w.x != w.x) | (w.y != w.y) | (w.z != w.z) | (w.w != w.w);
    if (a.row_stats) rowsums_add4(rs, w, valid_in_group(i, a.rowlen));
  }
  const QP p = a.row_stats
                   ? pc_row_qparams<true>(mn, mx, nan, rs, a.run_min[row], a.run_max[row], row, 0, a)
                   : pc_row_qparams<false>(mn, mx, nan, rs, a.run_min[row], a.run_max[row], row, 0, a);
  if (!y) return;
  float *yr = y + row * a.rowlen;
  uint64_t *mr = mask ? mask + row * mask_words_per_row(a.rowlen) : nullptr;
  for (int64_t base = 0; base < ng; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const bool in = i < ng;
    Elem e0{}, e1{}, e2{}, e3{};
    if (in) {
      const f4 w = load_group<VEC, NT>(xr, i, a.rowlen);
      e0 = fq_elem(w.x, p); e1 = fq_elem(w.y, p); e2 = fq_elem(w.z, p); e3 = fq_elem(w.w, p);
      f4 o;
      o.x = e0.y; o.y = e1.y; o.z = e2.y; o.w = e3.y;
      store_group<VEC, NT>(yr, i, a.rowlen, o);
      if (codes) {
        const uint32_t c = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
        for (int j = 0; j < valid_in_group(i, a.rowlen); ++j)
          codes[row * a.rowlen + 4 * i + j] = (uint8_t)(c >> (8 * j));
      }
    }
    if (mr && (i - threadIdx.x % kWave) < ng) {
      const int nv = in ? valid_in_group(i, a.rowlen) : 0;
      store_mask_chunk(mr + 4 * (i / kWave), e0.m && nv > 0, e1.m && nv > 1, e2.m && nv > 2,
                       e3.m && nv > 3);
    }
  }
}

// ----------------------------------------------------------------------------
// per-channel fake-quant with given per-row qparams: grid (rows, chunks)
// ----------------------------------------------------------------------------
struct PCFixed {
  int64_t rowlen;
  const double *scale, *zp;
  int zp_round;
  float lo, hi;
};

__device__ __forceinline__ QP pc_fixed_qp(const PCFixed &a, int64_t row) {
  QPSrc s{nullptr, a.scale + row, a.zp + row, 0.0, 0.0, a.lo, a.hi, a.zp_round, 0};
  return load_qp(s);
}

template <bool VEC, bool NT, bool CODES, bool MASK>
__global__ __launch_bounds__(kBlock) void k_pc_fq_fwd(const float *__restrict__ x, float *__restrict__ y,
                                                      uint8_t *__restrict__ codes,
                                                      uint64_t *__restrict__ mask, PCFixed a) {
  const int64_t row = blockIdx.x;
  const QP p = pc_fixed_qp(a, row);
  const int64_t ng = cdiv(a.rowlen, 4);
  const float *xr = x + row * a.rowlen;
  float *yr = y + row * a.rowlen;
  for (int64_t i = (int64_t)blockIdx.y * kBlock + threadIdx.x; i - threadIdx.x % kWave < ng;
       i += (int64_t)gridDim.y * kBlock) {
    const bool in = i < ng;
    Elem e0{}, e1{}, e2{}, e3{};
    if (in) {
      const f4 v = load_group<VEC, NT>(xr, i, a.rowlen);
      e0 = fq_elem(v.x, p); e1 = fq_elem(v.y, p); e2 = fq_elem(v.z, p); e3 = fq_elem(v.w, p);
      f4 o;
      o.x = e0.y; o.y = e1.y; o.z = e2.y; o.w = e3.y;
      store_group<VEC, NT>(yr, i, a.rowlen, o);
      if (CODES) {
        const uint32_t c = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
        uint8_t *cr = codes + row * a.rowlen;
        if (VEC) reinterpret_cast<uint32_t *>(cr)[i] = c;
        else
          for (int j = 0; j < valid_in_group(i, a.rowlen); ++j) cr[4 * i + j] = (uint8_t)(c >> (8 * j));
      }
    }
    if (MASK) {
      const int nv = in ? valid_in_group(i, a.rowlen) : 0;
      store_mask_chunk(mask + row * mask_words_per_row(a.rowlen) + 4 * (i / kWave), e0.m && nv > 0,
                       e1.m && nv > 1, e2.m && nv > 2, e3.m && nv > 3);
    }
  }
}

// ----------------------------------------------------------------------------
// STE backward with the saved 1-bit mask: gx = (m ? g*s : 0) / s, grid (rows, chunks)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float ste_elem(float g, uint32_t m, const FastDiv &d) {
  const float gq = g * d.b;          // MulBackward0
  const float gm = m ? gq : 0.0f;    // ClampBackward1
  return fdiv(gm, d);                // DivBackward0
}

template <bool VEC, bool NT>
__global__ __launch_bounds__(kBlock) void k_ste_bwd(const float *__restrict__ g,
                                                    const uint64_t *__restrict__ mask,
                                                    float *__restrict__ gx, int64_t rowlen,
                                                    const double *__restrict__ sdev, double shost) {
  const int64_t row = blockIdx.x;
  const FastDiv s = make_fastdiv((float)(sdev ? sdev[row] : shost));
  const int64_t ng = cdiv(rowlen, 4);
  const float *gr = g + row * rowlen;
  float *xr = gx + row * rowlen;
  const uint64_t *mr = mask + row * mask_words_per_row(rowlen);
  const int lane = threadIdx.x % kWave;
  for (int64_t i = (int64_t)blockIdx.y * kBlock + threadIdx.x; i - lane < ng;
       i += (int64_t)gridDim.y * kBlock) {
    const uint32_t m = load_mask_nibble(mr + 4 * (i / kWave), lane);
    if (i < ng) {
      const f4 v = load_group<VEC, NT>(gr, i, rowlen);
      f4 o;
      o.x = ste_elem(v.x, m & 1u, s);
      o.y = ste_elem(v.y, m & 2u, s);
      o.z = ste_elem(v.z, m & 4u, s);
      o.w = ste_elem(v.w, m & 8u, s);
      store_group<VEC, NT>(xr, i, rowlen, o);
    }
  }
}

// ----------------------------------------------------------------------------
// K4: learnable (LSQ) backward, grad_x + f64 scale / zp gradient sums
// ----------------------------------------------------------------------------
struct LsqAcc {
  double t, z;   // sum [g(q-z) + -(gm)(x/s/s)] ; sum [gm + -(g s)]
};

template <bool ZPL>
__device__ __forceinline__ float lsq_elem(float x, float g, const QP &p, LsqAcc &acc, bool valid) {
  const float u = fdiv(x, p.d);
  const float r = __builtin_rintf(u + p.z);
  const float q = fq_clamp(r, p.lo, p.hi);
  const bool m = (r >= p.lo && r <= p.hi);
  const float gq = g * p.s;                 // MulBackward0 (self)
  const float gm = m ? gq : 0.0f;           // ClampBackward1
  const float t1 = g * (q - p.z);           // MulBackward0 (other)
  const float xs = fdiv(u, p.d);            // (self / other) / other
  const float t2 = (-gm) * xs;              // DivBackward0 (other)
  if (valid) {
    acc.t += (double)t1 + (double)t2;
    if (ZPL) acc.z += (double)gm + (double)(-gq);   // AddBackward0 + SubBackward0 (other)
  }
  return fdiv(gm, p.d);                     // DivBackward0 (self)
}

__device__ __forceinline__ void lsq_block_reduce(LsqAcc &c) {
  __shared__ double s[2][kWaves];
  c.t = wave_reduce(c.t, AddD());
  c.z = wave_reduce(c.z, AddD());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) { s[0][w] = c.t; s[1][w] = c.z; }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int i = 1; i < kWaves; ++i) { c.t += s[0][i]; c.z += s[1][i]; }
  __syncthreads();
}

template <bool VEC, bool NT, bool ZPL>
__device__ __forceinline__ void lsq_group(const float *x, const float *g, float *gx, int64_t i,
                                          int64_t n, f4 xv, f4 gv, const QP &p, LsqAcc &c) {
  const int nv = valid_in_group(i, n);
  f4 o;
  o.x = lsq_elem<ZPL>(xv.x, gv.x, p, c, true);
  o.y = lsq_elem<ZPL>(xv.y, gv.y, p, c, nv > 1);
  o.z = lsq_elem<ZPL>(xv.z, gv.z, p, c, nv > 2);
  o.w = lsq_elem<ZPL>(xv.w, gv.w, p, c, nv > 3);
  store_group<VEC, NT>(gx, i, n, o);
}

template <bool VEC, bool NT, bool ZPL>
__global__ __launch_bounds__(kBlock) void k_lsq_bwd(const float *__restrict__ g,
                                                    const float *__restrict__ x,
                                                    float *__restrict__ gx, int64_t n,
                                                    QPSrc src, double gscale, int prefetch,
                                                    double *__restrict__ grad_out,
                                                    double *__restrict__ ws,
                                                    uint32_t *__restrict__ counter) {
  const QP p = load_qp(src);
  LsqAcc c{0.0, 0.0};
  const int64_t ng = cdiv(n, 4);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (prefetch) {
    // software pipeline: the next tile's loads are in flight while this one computes
    f4 xa{}, ga{};
    if (i < ng) { xa = load_group<VEC, NT>(x, i, n); ga = load_group<VEC, NT>(g, i, n); }
    while (i < ng) {
      const int64_t j = i + stride;
      f4 xb{}, gb{};
      if (j < ng) { xb = load_group<VEC, NT>(x, j, n); gb = load_group<VEC, NT>(g, j, n); }
      lsq_group<VEC, NT, ZPL>(x, g, gx, i, n, xa, ga, p, c);
      xa = xb;
      ga = gb;
      i = j;
    }
  } else {
    for (; i < ng; i += stride)
      lsq_group<VEC, NT, ZPL>(x, g, gx, i, n, load_group<VEC, NT>(x, i, n),
                              load_group<VEC, NT>(g, i, n), p, c);
  }
  lsq_block_reduce(c);
  if (threadIdx.x == 0) {
    double *r = ws + (int64_t)blockIdx.x * kPartials;
    r[0] = c.t; r[1] = c.z;
  }
  if (!arrive_last(counter)) return;
  c = LsqAcc{0.0, 0.0};
  for (int b = threadIdx.x; b < (int)gridDim.x; b += kBlock) {
    const double *r = ws + (int64_t)b * kPartials;
    c.t += r[0]; c.z += r[1];
  }
  lsq_block_reduce(c);
  if (threadIdx.x == 0) {
    grad_out[0] = c.t * gscale;
    double gz = 0.0;
    if (ZPL) {
      // ClampBackward of zero_point_rounding (uniform.py:101): in-range test on round(zp)
      const double zr = __builtin_rint(src.zdev ? *src.zdev : src.zhost);   // NaN -> not in range
      const bool zin = zr >= (double)p.lo && zr <= (double)p.hi;
      gz = zin ? c.z * gscale : 0.0;
    }
    grad_out[1] = gz;
    *counter = 0u;
  }
}

// ----------------------------------------------------------------------------
// exhaustive check of fdiv against the IEEE division: every 32-bit pattern a,
// for each divisor b[k]; counts bitwise mismatches (NaNs compare by NaN-ness)
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_selftest_div(const float *__restrict__ bs, int nb,
                                                         unsigned long long *__restrict__ bad) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (int k = 0; k < nb; ++k) {
    const FastDiv d = make_fastdiv(bs[k]);
    uint32_t cnt = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < (1ull << 32); i += stride) {
      const float a = __uint_as_float((uint32_t)i);
      const float q = fdiv(a, d), w = a / d.b;
      const bool same = (__float_as_uint(q) == __float_as_uint(w)) || (q != q && w != w);
      cnt += same ? 0u : 1u;
    }
    cnt = wave_reduce(cnt, AddU());
    if (threadIdx.x % kWave == 0 && cnt) atomicAdd(bad + k, (unsigned long long)cnt);
  }
}

// ----------------------------------------------------------------------------
// host helpers
// ----------------------------------------------------------------------------
inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
inline bool aligned4(const void *p) { return ((uintptr_t)p & 3u) == 0; }
inline bool aligned8(const void *p) { return ((uintptr_t)p & 7u) == 0; }

inline int reduce_grid(int64_t groups, int per_thread) {
  int64_t b = cdiv(groups, (int64_t)kBlock * per_thread);
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, kMaxReduceGrid));
}

inline int flat_grid(int64_t groups) {
  const int64_t b = cdiv(groups, (int64_t)kBlock);
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, std::max(256, g_tune.flat_grid_cap)));
}

// blocks per row for the (row, chunk) kernels: one block per 1024 groups, at most
// ~32 blocks per CU over the whole grid and at most 65535 (chunks are grid-strided)
inline int64_t chunk_grid(int64_t rowlen, int64_t rows) {
  int64_t c = cdiv(cdiv(rowlen, 4), (int64_t)kBlock * 4);
  const int64_t cap = std::max<int64_t>(1, (256 * 32) / std::max<int64_t>(rows, 1));
  return std::max<int64_t>(1, std::min<int64_t>(std::min(c, cap), 65535));
}

inline int launch_rc() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// dispatch helpers: runtime flags -> template instantiations
#define VSIQ_B2(F, A, B, ...)                                 \
  ((A) ? ((B) ? F<true, true>(__VA_ARGS__) : F<true, false>(__VA_ARGS__)) \
       : ((B) ? F<false, true>(__VA_ARGS__) : F<false, false>(__VA_ARGS__)))

template <bool VEC, bool NT>
void launch_fq_fwd(const float *x, float *y, uint8_t *codes, uint64_t *mask, int64_t n,
                   const QPSrc &src, hipStream_t st) {
  const dim3 grid(flat_grid(cdiv(n, 4))), block(kBlock);
  if (codes && mask)
    hipLaunchKernelGGL((k_fq_fwd<VEC, NT, true, true>), grid, block, 0, st, x, y, codes, mask, n, src);
  else if (codes)
    hipLaunchKernelGGL((k_fq_fwd<VEC, NT, true, false>), grid, block, 0, st, x, y, codes, mask, n, src);
  else if (mask)
    hipLaunchKernelGGL((k_fq_fwd<VEC, NT, false, true>), grid, block, 0, st, x, y, codes, mask, n, src);
  else
    hipLaunchKernelGGL((k_fq_fwd<VEC, NT, false, false>), grid, block, 0, st, x, y, codes, mask, n, src);
}

template <int NV, bool VEC, bool NT, bool STATS>
void launch_pc_nv(const float *x, float *y, uint8_t *c, uint64_t *m, const PCArgs &a, int grid,
                  hipStream_t st) {
  const dim3 g(grid), b(kBlock);
  if (c && m)
    hipLaunchKernelGGL((k_pc_observe_fq<NV, VEC, NT, STATS, true, true>), g, b, 0, st, x, y, c, m, a);
  else if (c)
    hipLaunchKernelGGL((k_pc_observe_fq<NV, VEC, NT, STATS, false, true>), g, b, 0, st, x, y, c, m, a);
  else if (m)
    hipLaunchKernelGGL((k_pc_observe_fq<NV, VEC, NT, STATS, true, false>), g, b, 0, st, x, y, c, m, a);
  else
    hipLaunchKernelGGL((k_pc_observe_fq<NV, VEC, NT, STATS, false, false>), g, b, 0, st, x, y, c, m, a);
}

template <bool VEC, bool NT, bool STATS>
int launch_pc(const float *x, float *y, uint8_t *c, uint64_t *m, const PCArgs &a, hipStream_t st) {
  const int64_t ng = cdiv(a.rowlen, 4);
  const int64_t per_lane = cdiv(ng, kBlock);
  // rows per workgroup: >= 2 lets a CU overlap row k's writes with row k+1's reads
  int rpb = g_tune.pc_rows_per_block;
  if (rpb <= 0) rpb = a.rows >= 1024 ? 2 : 1;
  const int grid = (int)std::max<int64_t>(1, cdiv(a.rows, rpb));
  if (per_lane <= 1) launch_pc_nv<1, VEC, NT, STATS>(x, y, c, m, a, grid, st);
  else if (per_lane <= 2) launch_pc_nv<2, VEC, NT, STATS>(x, y, c, m, a, grid, st);
  else if (per_lane <= 4) launch_pc_nv<4, VEC, NT, STATS>(x, y, c, m, a, grid, st);
  else if (per_lane <= 6) launch_pc_nv<6, VEC, NT, STATS>(x, y, c, m, a, grid, st);
  else if (per_lane <= 9) launch_pc_nv<9, VEC, NT, STATS>(x, y, c, m, a, grid, st);
  else if (per_lane <= 12) launch_pc_nv<12, VEC, NT, STATS>(x, y, c, m, a, grid, st);
  else
    hipLaunchKernelGGL((k_pc_observe_fq_long<VEC, NT>), dim3((unsigned)a.rows), dim3(kBlock), 0, st, x,
                       y, c, m, a);
  return launch_rc();
}

template <bool VEC, bool NT>
void launch_pc_fixed(const float *x, float *y, uint8_t *c, uint64_t *m, const PCFixed &a, int64_t rows,
                     hipStream_t st) {
  const dim3 grid((unsigned)rows, (unsigned)chunk_grid(a.rowlen, rows)), block(kBlock);
  if (c && m) hipLaunchKernelGGL((k_pc_fq_fwd<VEC, NT, true, true>), grid, block, 0, st, x, y, c, m, a);
  else if (c) hipLaunchKernelGGL((k_pc_fq_fwd<VEC, NT, true, false>), grid, block, 0, st, x, y, c, m, a);
  else if (m) hipLaunchKernelGGL((k_pc_fq_fwd<VEC, NT, false, true>), grid, block, 0, st, x, y, c, m, a);
  else hipLaunchKernelGGL((k_pc_fq_fwd<VEC, NT, false, false>), grid, block, 0, st, x, y, c, m, a);
}

template <bool VEC, bool NT>
void launch_ste(const float *g, const uint64_t *m, float *gx, int64_t rows, int64_t rowlen,
                const double *sdev, double shost, hipStream_t st) {
  const dim3 grid((unsigned)rows, (unsigned)chunk_grid(rowlen, rows)), block(kBlock);
  hipLaunchKernelGGL((k_ste_bwd<VEC, NT>), grid, block, 0, st, g, m, gx, rowlen, sdev, shost);
}

template <bool VEC, bool NT>
void launch_lsq(const float *g, const float *x, float *gx, int64_t n, const QPSrc &src, int zpl,
                double gscale, double *grad_out, double *ws, uint32_t *counter, int grid,
                hipStream_t st) {
  const int pf = g_tune.lsq_prefetch;
  if (zpl)
    hipLaunchKernelGGL((k_lsq_bwd<VEC, NT, true>), dim3(grid), dim3(kBlock), 0, st, g, x, gx, n, src,
                       gscale, pf, grad_out, ws, counter);
  else
    hipLaunchKernelGGL((k_lsq_bwd<VEC, NT, false>), dim3(grid), dim3(kBlock), 0, st, g, x, gx, n, src,
                       gscale, pf, grad_out, ws, counter);
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int vsiq_abi_version(void) { return VSIQ_ABI_VERSION; }

const char *vsiq_error_string(int code) {
  switch (code) {
    case 0: return "success";
    case VSIQ_E_ARG: return "vsiq: invalid argument";
    case VSIQ_E_ALIGN: return "vsiq: misaligned pointer";
    case VSIQ_E_WS: return "vsiq: workspace too small";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "vsiq: unknown error";
  }
}

int64_t vsiq_workspace_doubles(int64_t n) {
  (void)n;
  return (int64_t)kMaxReduceGrid * kPartials;
}

int64_t vsiq_mask_words(int64_t rows, int64_t rowlen) {
  if (rows < 0 || rowlen < 0) return VSIQ_E_ARG;
  return rows * mask_words_per_row(rowlen);
}

int vsiq_set_tuning(int key, int value) {
  switch (key) {
    case VSIQ_TUNE_PC_ROWS_PER_BLOCK: g_tune.pc_rows_per_block = value; return 0;
    case VSIQ_TUNE_NONTEMPORAL: g_tune.nontemporal = value; return 0;
    case VSIQ_TUNE_FLAT_GRID_CAP: g_tune.flat_grid_cap = value; return 0;
    case VSIQ_TUNE_LSQ_PREFETCH: g_tune.lsq_prefetch = value; return 0;
    default: return VSIQ_E_ARG;
  }
}

int vsiq_selftest_div(const float *divisors, int count, unsigned long long *mismatches,
                      void *stream) {
  if (count < 0 || (count > 0 && (!divisors || !mismatches))) return VSIQ_E_ARG;
  if (count == 0) return 0;
  hipLaunchKernelGGL(k_selftest_div, dim3(256 * 16), dim3(kBlock), 0, (hipStream_t)stream,
                     divisors, count, mismatches);
  return launch_rc();
}

int vsiq_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t n,
                    const double *qp_dev, const double *scale_dev, double scale_host,
                    const double *zp_dev, double zp_host, int zp_round, int discrete, int qmin,
                    int qmax, void *stream) {
  if (n < 0 || qmin > qmax || (n > 0 && (!x || !y))) return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  QPSrc src{qp_dev, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax,
            qp_dev ? 0 : zp_round, discrete ? 1 : 0};
  const bool vec = (n % 4 == 0) && aligned16(x) && aligned16(y) && (!codes || aligned4(codes));
  const bool nt = g_tune.nontemporal != 0;
  uint8_t *c = (uint8_t *)codes;
  VSIQ_B2(launch_fq_fwd, vec, nt, x, y, c, mask, n, src, st);
  return launch_rc();
}

int vsiq_observe_f32(const float *x, int64_t n, double *stats_out, float *run_minmax,
                     double *qp_out, int symmetric, double qden, double eps, double *ws,
                     int64_t ws_len, uint32_t *counter, void *stream) {
  if (n <= 0 || !x || !ws || !counter) return VSIQ_E_ARG;
  const bool vec = aligned16(x) && n % 4 == 0;
  const int grid = reduce_grid(cdiv(n, 4), 4);
  if (ws_len < (int64_t)grid * kPartials) return VSIQ_E_WS;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(grid), b(kBlock);
  if (vec && g_tune.nontemporal)
    hipLaunchKernelGGL((k_observe<true, true>), g, b, 0, st, x, n, stats_out, run_minmax, qp_out,
                       symmetric, qden, eps, ws, counter);
  else if (vec)
    hipLaunchKernelGGL((k_observe<true, false>), g, b, 0, st, x, n, stats_out, run_minmax, qp_out,
                       symmetric, qden, eps, ws, counter);
  else
    hipLaunchKernelGGL((k_observe<false, false>), g, b, 0, st, x, n, stats_out, run_minmax, qp_out,
                       symmetric, qden, eps, ws, counter);
  return launch_rc();
}

int vsiq_observe_finalize(const double *stats, float *run_minmax, double *qp_out, int symmetric,
                          double qden, double eps, void *stream) {
  if (!stats) return VSIQ_E_ARG;
  hipLaunchKernelGGL(k_observe_finalize, dim3(1), dim3(kWave), 0, (hipStream_t)stream, stats,
                     run_minmax, qp_out, symmetric, qden, eps);
  return launch_rc();
}

int vsiq_pc_observe_fq_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t rows,
                           int64_t rowlen, float *run_min, float *run_max, double *scale_out,
                           double *zp_out, double *row_stats, int symmetric, int qmin, int qmax,
                           double qden, double eps, void *stream) {
  if (rows < 0 || rowlen <= 0 || qmin > qmax) return VSIQ_E_ARG;
  if (rows == 0) return 0;
  if (!x || !run_min || !run_max || !scale_out || !zp_out) return VSIQ_E_ARG;
  if (!y && (codes || mask)) return VSIQ_E_ARG;
  if (rows > 0x7fffffffLL) return VSIQ_E_ARG;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  PCArgs a{rows, rowlen, run_min, run_max, scale_out, zp_out, row_stats, symmetric, (float)qmin,
           (float)qmax, qden, eps};
  const bool vec = (rowlen % 4 == 0) && aligned16(x) && (!y || aligned16(y)) && (!codes || aligned4(codes));
  const bool nt = g_tune.nontemporal != 0;
  hipStream_t st = (hipStream_t)stream;
  uint8_t *c = (uint8_t *)codes;
  if (row_stats) {
    if (vec) return nt ? launch_pc<true, true, true>(x, y, c, mask, a, st) : launch_pc<true, false, true>(x, y, c, mask, a, st);
    return launch_pc<false, false, true>(x, y, c, mask, a, st);
  }
  if (vec) return nt ? launch_pc<true, true, false>(x, y, c, mask, a, st) : launch_pc<true, false, false>(x, y, c, mask, a, st);
  return launch_pc<false, false, false>(x, y, c, mask, a, st);
}

int vsiq_pc_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t rows,
                       int64_t rowlen, const double *scale, const double *zp, int zp_round,
                       int qmin, int qmax, void *stream) {
  if (rows < 0 || rowlen <= 0 || qmin > qmax) return VSIQ_E_ARG;
  if (rows == 0) return 0;
  if (!x || !y || !scale || !zp || rows > 0x7fffffffLL) return VSIQ_E_ARG;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  PCFixed a{rowlen, scale, zp, zp_round, (float)qmin, (float)qmax};
  const bool vec = (rowlen % 4 == 0) && aligned16(x) && aligned16(y) && (!codes || aligned4(codes));
  const bool nt = g_tune.nontemporal != 0;
  uint8_t *c = (uint8_t *)codes;
  VSIQ_B2(launch_pc_fixed, vec, nt, x, y, c, mask, a, rows, (hipStream_t)stream);
  return launch_rc();
}

int vsiq_ste_bwd_f32(const float *g, const uint64_t *mask, float *gx, int64_t n,
                     const double *scale_dev, int64_t rowlen, double scale_host, void *stream) {
  if (n < 0) return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (!g || !mask || !gx) return VSIQ_E_ARG;
  if (!aligned8(mask)) return VSIQ_E_ALIGN;
  if (!scale_dev || rowlen <= 0) rowlen = n;
  if (n % rowlen != 0) return VSIQ_E_ARG;
  const int64_t rows = n / rowlen;
  if (rows > 0x7fffffffLL) return VSIQ_E_ARG;
  const bool vec = (rowlen % 4 == 0) && aligned16(g) && aligned16(gx);
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_B2(launch_ste, vec, nt, g, mask, gx, rows, rowlen, scale_dev, scale_host, (hipStream_t)stream);
  return launch_rc();
}

int vsiq_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t n,
                     const double *scale_dev, double scale_host, const double *zp_dev,
                     double zp_host, int zp_learn, int qmin, int qmax, double gscale,
                     double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
                     void *stream) {
  if (n <= 0 || !g || !x || !gx || !grad_out || !ws || !counter || qmin > qmax) return VSIQ_E_ARG;
  const bool vec = (n % 4 == 0) && aligned16(g) && aligned16(x) && aligned16(gx);
  const int grid = reduce_grid(cdiv(n, 4), 4);
  if (ws_len < (int64_t)grid * kPartials) return VSIQ_E_WS;
  // learnable zp: the forward used clamp(rint(zp)); a non-learnable zp is used as given
  QPSrc src{nullptr, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax, zp_learn, 0};
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_B2(launch_lsq, vec, nt, g, x, gx, n, src, zp_learn, gscale, grad_out, ws, counter, grid,
          (hipStream_t)stream);
  return launch_rc();
}

}  // extern "C"
