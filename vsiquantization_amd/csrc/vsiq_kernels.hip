// vsiq_kernels.hip — MI355X (gfx950 / CDNA4) kernels for VSIQuantization's
// fake-quantize hot path, exported through the C ABI in include/vsiq.h.
//
// Design (DESIGN.md has the full rationale and roofline numbers):
//   * Everything here is HBM-bound integer/fp32 elementwise + reduction work:
//     no MFMA.  Loads/stores are 16 B per lane (float4) wherever the layout
//     allows, one read and one write of every element per pass.
//   * fp32 arithmetic is IEEE and in the reference's operation order
//     (quantizers/uniform.py:55,95): true division x/s (correctly rounded; the
//     build uses -fhip-fp32-correctly-rounded-divide-sqrt, -ffp-contract=off,
//     denormals kept), rint (half-to-even), NaN-propagating clamp that keeps
//     -0.0.  This is bit-identical to the reference's PyTorch CPU kernels.
//   * qparams (observers/minmax.py:49-74) are computed in float64 on the
//     device from the fp32 min/max, so no `.item()` host round trip is needed.
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

// ----------------------------------------------------------------------------
// element arithmetic (quantizers/uniform.py:95, 55)
// ----------------------------------------------------------------------------
struct QP {
  float s, z, lo, hi;
  int discrete;
};

__device__ __forceinline__ float fq_round(float x, float s, float z) {
  float u = x / s;   // IEEE fp32 true division (x / fp32(scale))
  u = u + z;         // + fp32(zero_point); -0.0 + 0.0 -> +0.0 like torch.add
  return __builtin_rintf(u);   // torch.round: half to even
}

// torch.clamp(v, lo, hi): NaN propagates, -0.0 survives
__device__ __forceinline__ float fq_clamp(float r, float lo, float hi) {
  return r < lo ? lo : (r > hi ? hi : r);
}

__device__ __forceinline__ float fq_dequant(float q, const QP &p) { return (q - p.z) * p.s; }

__device__ __forceinline__ uint32_t fq_code_byte(float q) {
  // int8 (sym) / uint8 (asym) share the low byte of the integer; NaN -> 0
  return (q == q) ? (uint32_t)((int)q) & 0xffu : 0u;
}

struct Elem {
  float y;
  uint32_t code;
  uint32_t m;
};

__device__ __forceinline__ Elem fq_elem(float x, const QP &p) {
  const float r = fq_round(x, p.s, p.z);
  const float q = fq_clamp(r, p.lo, p.hi);
  Elem e;
  e.y = p.discrete ? q : fq_dequant(q, p);
  e.code = fq_code_byte(q);
  e.m = (r >= p.lo && r <= p.hi) ? 1u : 0u;
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
  return p;
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

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ----------------------------------------------------------------------------
// K1: per-tensor fake-quant forward (flat, grid-stride, float4)
// ----------------------------------------------------------------------------
constexpr int kFqUnroll = 4;

template <bool CODES, bool MASK>
__global__ __launch_bounds__(kBlock) void k_fq_fwd_v4(const float4 *__restrict__ x,
                                                      float4 *__restrict__ y,
                                                      uint32_t *__restrict__ codes,
                                                      uint32_t *__restrict__ mask, int64_t n4,
                                                      QPSrc src) {
  const QP p = load_qp(src);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t base = (int64_t)blockIdx.x * kBlock + threadIdx.x; base < n4;
       base += stride * kFqUnroll) {
    float4 v[kFqUnroll];
#pragma unroll
    for (int u = 0; u < kFqUnroll; ++u) {
      const int64_t i = base + u * stride;
      if (i < n4) v[u] = x[i];
    }
#pragma unroll
    for (int u = 0; u < kFqUnroll; ++u) {
      const int64_t i = base + u * stride;
      if (i < n4) {
        const Elem e0 = fq_elem(v[u].x, p), e1 = fq_elem(v[u].y, p);
        const Elem e2 = fq_elem(v[u].z, p), e3 = fq_elem(v[u].w, p);
        y[i] = make_float4(e0.y, e1.y, e2.y, e3.y);
        if (CODES) codes[i] = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
        if (MASK) mask[i] = e0.m | (e1.m << 8) | (e2.m << 16) | (e3.m << 24);
      }
    }
  }
}

// scalar variant: misaligned pointers / n % 4 tails
__global__ __launch_bounds__(kBlock) void k_fq_fwd_s(const float *__restrict__ x,
                                                     float *__restrict__ y,
                                                     uint8_t *__restrict__ codes,
                                                     uint8_t *__restrict__ mask, int64_t n,
                                                     QPSrc src) {
  const QP p = load_qp(src);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const Elem e = fq_elem(x[i], p);
    y[i] = e.y;
    if (codes) codes[i] = (uint8_t)e.code;
    if (mask) mask[i] = (uint8_t)e.m;
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

// fminf/fmaxf skip NaN operands; NaNs are counted separately.
__device__ __forceinline__ void obs_add4(ObsAcc &a, float4 v) {
  a.mn = fminf(fminf(a.mn, v.x), fminf(fminf(v.y, v.z), v.w));
  a.mx = fmaxf(fmaxf(a.mx, v.x), fmaxf(fmaxf(v.y, v.z), v.w));
  a.nan += (v.x != v.x) + (v.y != v.y) + (v.z != v.z) + (v.w != v.w);
  // fp32 partial over the 4 lanes of the vector, float64 across vectors
  const float pa = (__builtin_fabsf(v.x) + __builtin_fabsf(v.y)) +
                   (__builtin_fabsf(v.z) + __builtin_fabsf(v.w));
  const float p1 = (v.x + v.y) + (v.z + v.w);
  const double dx = v.x, dy = v.y, dz = v.z, dw = v.w;
  a.sa += (double)pa;
  a.s1 += (double)p1;
  a.s2 += __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, dw * dw)));
}

__device__ __forceinline__ void obs_add1(ObsAcc &a, float v) {
  a.mn = fminf(a.mn, v);
  a.mx = fmaxf(a.mx, v);
  a.nan += (v != v);
  const double d = v;
  a.sa += __builtin_fabs(d);
  a.s1 += d;
  a.s2 += d * d;
}

__device__ __forceinline__ void obs_block_reduce(ObsAcc &a) {
  __shared__ float s_mn[kWaves], s_mx[kWaves];
  __shared__ uint32_t s_nan[kWaves];
  __shared__ double s_sa[kWaves], s_s1[kWaves], s_s2[kWaves];
  a.mn = wave_reduce(a.mn, MinOp());
  a.mx = wave_reduce(a.mx, MaxOp());
  a.nan = wave_reduce(a.nan, [](uint32_t u, uint32_t v) { return u + v; });
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

__global__ __launch_bounds__(kBlock) void k_observe(const float *__restrict__ x, int64_t n,
                                                    int vec, double *__restrict__ stats_out,
                                                    float *__restrict__ run_minmax,
                                                    double *__restrict__ qp_out, int sym,
                                                    double qden, double eps,
                                                    double *__restrict__ ws,
                                                    uint32_t *__restrict__ counter) {
  ObsAcc a;
  obs_init(a);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (vec) {
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    const int64_t n4 = n / 4;
    for (int64_t base = t0; base < n4; base += stride * kFqUnroll) {
      float4 v[kFqUnroll];
#pragma unroll
      for (int u = 0; u < kFqUnroll; ++u) {
        const int64_t i = base + u * stride;
        if (i < n4) v[u] = x4[i];
      }
#pragma unroll
      for (int u = 0; u < kFqUnroll; ++u)
        if (base + u * stride < n4) obs_add4(a, v[u]);
    }
    for (int64_t i = 4 * n4 + t0; i < n; i += stride) obs_add1(a, x[i]);
  } else {
    for (int64_t i = t0; i < n; i += stride) obs_add1(a, x[i]);
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
  a.nan = 0;
  // NaN counts fit in f64 exactly; reduce them through the sa slot trick-free path
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
// K3: per-channel observe + qparams + fake-quant, one workgroup per row,
//     the whole row held in registers (NV float4 per lane).
// ----------------------------------------------------------------------------
struct PCArgs {
  int64_t rowlen;
  float *run_min, *run_max;
  double *scale_out, *zp_out;
  double *row_stats;   // [rows][3] sum|x|, sum x, sum x^2 (nullable) for qm.py:66-68
  int sym;
  float lo, hi;
  double qden, eps;
};

// row min / max / NaN -> running state -> f64 qparams; returns fp32 (s, z) to all lanes
__device__ __forceinline__ QP pc_row_qparams(float mn, float mx, uint32_t nan, int64_t row,
                                             const PCArgs &a) {
  __shared__ float s_mn[kWaves], s_mx[kWaves];
  __shared__ uint32_t s_nan[kWaves];
  __shared__ float s_qp[2];
  mn = wave_reduce(mn, MinOp());
  mx = wave_reduce(mx, MaxOp());
  nan = wave_reduce(nan, OrU());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) { s_mn[w] = mn; s_mx[w] = mx; s_nan[w] = nan; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kWaves; ++i) { mn = fminf(mn, s_mn[i]); mx = fmaxf(mx, s_mx[i]); nan |= s_nan[i]; }
    float rmn = a.run_min[row], rmx = a.run_max[row];
    if (!nan) {                         // minmax.py:44-47, strict compares
      if (mn < rmn) rmn = mn;
      if (mx > rmx) rmx = mx;
    }
    a.run_min[row] = rmn;
    a.run_max[row] = rmx;
    double s, z;
    minmax_qparams((double)rmn, (double)rmx, a.sym, a.qden, a.eps, &s, &z);
    a.scale_out[row] = s;
    a.zp_out[row] = z;
    s_qp[0] = (float)s;
    s_qp[1] = (float)z;
  }
  __syncthreads();
  QP p;
  p.s = s_qp[0];
  p.z = s_qp[1];
  p.lo = a.lo;
  p.hi = a.hi;
  p.discrete = 0;
  return p;
}

struct RowSums {
  double sa, s1, s2;
};

__device__ __forceinline__ void rowsums_add4(RowSums &r, float4 v) {
  const float pa = (__builtin_fabsf(v.x) + __builtin_fabsf(v.y)) +
                   (__builtin_fabsf(v.z) + __builtin_fabsf(v.w));
  const float p1 = (v.x + v.y) + (v.z + v.w);
  const double dx = v.x, dy = v.y, dz = v.z, dw = v.w;
  r.sa += (double)pa;
  r.s1 += (double)p1;
  r.s2 += __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, dw * dw)));
}

// block-reduce the row sums; thread 0 stores them
__device__ __forceinline__ void rowsums_store(RowSums r, double *out) {
  __shared__ double s[3][kWaves];
  r.sa = wave_reduce(r.sa, AddD());
  r.s1 = wave_reduce(r.s1, AddD());
  r.s2 = wave_reduce(r.s2, AddD());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) { s[0][w] = r.sa; s[1][w] = r.s1; s[2][w] = r.s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kWaves; ++i) { r.sa += s[0][i]; r.s1 += s[1][i]; r.s2 += s[2][i]; }
    out[0] = r.sa;
    out[1] = r.s1;
    out[2] = r.s2;
  }
}

// y == nullptr: observe only (state + qparams + stats, no stores of the row)
template <int NV, bool STATS>
__global__ __launch_bounds__(kBlock) void k_pc_observe_fq_v4(const float *__restrict__ x,
                                                             float *__restrict__ y,
                                                             uint8_t *__restrict__ codes,
                                                             uint8_t *__restrict__ mask,
                                                             PCArgs a) {
  const int64_t row = blockIdx.x;
  const int n4 = (int)(a.rowlen / 4);
  const float4 *xr = reinterpret_cast<const float4 *>(x + row * a.rowlen);
  float4 v[NV];
  float mn = __builtin_inff(), mx = -__builtin_inff();
  uint32_t nan = 0;
  RowSums rs{0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * kBlock;
    if (i < n4) v[k] = xr[i];
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * kBlock;
    if (i < n4) {
      mn = fminf(mn, fminf(fminf(v[k].x, v[k].y), fminf(v[k].z, v[k].w)));
      mx = fmaxf(mx, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
      nan |= (v[k].x != v[k].x) | (v[k].y != v[k].y) | (v[k].z != v[k].z) | (v[k].w != v[k].w);
      if (STATS) rowsums_add4(rs, v[k]);
    }
  }
  if (STATS) rowsums_store(rs, a.row_stats + row * 3);
  const QP p = pc_row_qparams(mn, mx, nan, row, a);
  if (!y) return;
  float4 *yr = reinterpret_cast<float4 *>(y + row * a.rowlen);
  uint32_t *cr = codes ? reinterpret_cast<uint32_t *>(codes + row * a.rowlen) : nullptr;
  uint32_t *mr = mask ? reinterpret_cast<uint32_t *>(mask + row * a.rowlen) : nullptr;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * kBlock;
    if (i < n4) {
      const Elem e0 = fq_elem(v[k].x, p), e1 = fq_elem(v[k].y, p);
      const Elem e2 = fq_elem(v[k].z, p), e3 = fq_elem(v[k].w, p);
      yr[i] = make_float4(e0.y, e1.y, e2.y, e3.y);
      if (cr) cr[i] = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
      if (mr) mr[i] = e0.m | (e1.m << 8) | (e2.m << 16) | (e3.m << 24);
    }
  }
}

// generic row kernel: any rowlen / alignment; re-reads the row (L2-resident) for pass 2
__global__ __launch_bounds__(kBlock) void k_pc_observe_fq_s(const float *__restrict__ x,
                                                            float *__restrict__ y,
                                                            uint8_t *__restrict__ codes,
                                                            uint8_t *__restrict__ mask,
                                                            PCArgs a) {
  const int64_t row = blockIdx.x;
  const float *xr = x + row * a.rowlen;
  float mn = __builtin_inff(), mx = -__builtin_inff();
  uint32_t nan = 0;
  RowSums rs{0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < a.rowlen; i += kBlock) {
    const float v = xr[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    nan |= (v != v);
    const double d = v;
    rs.sa += __builtin_fabs(d);
    rs.s1 += d;
    rs.s2 += d * d;
  }
  if (a.row_stats) rowsums_store(rs, a.row_stats + row * 3);
  const QP p = pc_row_qparams(mn, mx, nan, row, a);
  if (!y) return;
  for (int64_t i = threadIdx.x; i < a.rowlen; i += kBlock) {
    const Elem e = fq_elem(xr[i], p);
    y[row * a.rowlen + i] = e.y;
    if (codes) codes[row * a.rowlen + i] = (uint8_t)e.code;
    if (mask) mask[row * a.rowlen + i] = (uint8_t)e.m;
  }
}

// per-channel fake-quant with given per-row qparams: grid (rows, chunks)
struct PCFixed {
  int64_t rowlen;
  const double *scale, *zp;
  int zp_round;
  float lo, hi;
};

__device__ __forceinline__ QP pc_fixed_qp(const PCFixed &a, int64_t row) {
  QPSrc s;
  s.qp = nullptr;
  s.sdev = a.scale + row;
  s.zdev = a.zp + row;
  s.shost = 0.0;
  s.zhost = 0.0;
  s.lo = a.lo;
  s.hi = a.hi;
  s.zround = a.zp_round;
  s.discrete = 0;
  return load_qp(s);
}

constexpr int kChunk4 = kBlock * 4;   // float4 per (row, chunk) block

__global__ __launch_bounds__(kBlock) void k_pc_fq_fwd_v4(const float *__restrict__ x,
                                                         float *__restrict__ y,
                                                         uint8_t *__restrict__ codes,
                                                         uint8_t *__restrict__ mask, PCFixed a) {
  const int64_t row = blockIdx.x;
  const QP p = pc_fixed_qp(a, row);
  const int64_t n4 = a.rowlen / 4;
  const float4 *xr = reinterpret_cast<const float4 *>(x + row * a.rowlen);
  float4 *yr = reinterpret_cast<float4 *>(y + row * a.rowlen);
  uint32_t *cr = codes ? reinterpret_cast<uint32_t *>(codes + row * a.rowlen) : nullptr;
  uint32_t *mr = mask ? reinterpret_cast<uint32_t *>(mask + row * a.rowlen) : nullptr;
  for (int64_t c = blockIdx.y; c * kChunk4 < n4; c += gridDim.y) {
    const int64_t i0 = c * kChunk4 + threadIdx.x;
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * kBlock < n4) v[u] = xr[i0 + u * kBlock];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * kBlock;
      if (i < n4) {
        const Elem e0 = fq_elem(v[u].x, p), e1 = fq_elem(v[u].y, p);
        const Elem e2 = fq_elem(v[u].z, p), e3 = fq_elem(v[u].w, p);
        yr[i] = make_float4(e0.y, e1.y, e2.y, e3.y);
        if (cr) cr[i] = e0.code | (e1.code << 8) | (e2.code << 16) | (e3.code << 24);
        if (mr) mr[i] = e0.m | (e1.m << 8) | (e2.m << 16) | (e3.m << 24);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_pc_fq_fwd_s(const float *__restrict__ x,
                                                        float *__restrict__ y,
                                                        uint8_t *__restrict__ codes,
                                                        uint8_t *__restrict__ mask, PCFixed a) {
  const int64_t row = blockIdx.x;
  const QP p = pc_fixed_qp(a, row);
  const int64_t base = row * a.rowlen;
  for (int64_t i = (int64_t)blockIdx.y * kBlock + threadIdx.x; i < a.rowlen;
       i += (int64_t)gridDim.y * kBlock) {
    const Elem e = fq_elem(x[base + i], p);
    y[base + i] = e.y;
    if (codes) codes[base + i] = (uint8_t)e.code;
    if (mask) mask[base + i] = (uint8_t)e.m;
  }
}

// ----------------------------------------------------------------------------
// STE backward with saved mask: gx = (m ? g*s : 0) / s, grid (rows, chunks)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float ste_elem(float g, uint32_t m, float s) {
  const float gq = g * s;            // MulBackward0
  const float gm = m ? gq : 0.0f;    // ClampBackward1
  return gm / s;                     // DivBackward0
}

__global__ __launch_bounds__(kBlock) void k_ste_bwd_v4(const float *__restrict__ g,
                                                       const uint8_t *__restrict__ mask,
                                                       float *__restrict__ gx, int64_t rowlen,
                                                       const double *__restrict__ sdev,
                                                       double shost) {
  const int64_t row = blockIdx.x;
  const float s = (float)(sdev ? sdev[row] : shost);
  const int64_t n4 = rowlen / 4;
  const float4 *gr = reinterpret_cast<const float4 *>(g + row * rowlen);
  const uint32_t *mr = reinterpret_cast<const uint32_t *>(mask + row * rowlen);
  float4 *xr = reinterpret_cast<float4 *>(gx + row * rowlen);
  for (int64_t c = blockIdx.y; c * kChunk4 < n4; c += gridDim.y) {
    const int64_t i0 = c * kChunk4 + threadIdx.x;
    float4 v[4];
    uint32_t m[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * kBlock;
      if (i < n4) { v[u] = gr[i]; m[u] = mr[i]; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * kBlock;
      if (i < n4)
        xr[i] = make_float4(ste_elem(v[u].x, m[u] & 0xffu, s), ste_elem(v[u].y, (m[u] >> 8) & 0xffu, s),
                            ste_elem(v[u].z, (m[u] >> 16) & 0xffu, s), ste_elem(v[u].w, m[u] >> 24, s));
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_ste_bwd_s(const float *__restrict__ g,
                                                      const uint8_t *__restrict__ mask,
                                                      float *__restrict__ gx, int64_t rowlen,
                                                      const double *__restrict__ sdev,
                                                      double shost) {
  const int64_t row = blockIdx.x;
  const float s = (float)(sdev ? sdev[row] : shost);
  const int64_t base = row * rowlen;
  for (int64_t i = (int64_t)blockIdx.y * kBlock + threadIdx.x; i < rowlen;
       i += (int64_t)gridDim.y * kBlock)
    gx[base + i] = ste_elem(g[base + i], mask[base + i], s);
}

// ----------------------------------------------------------------------------
// K4: learnable (LSQ) backward, grad_x + f64 scale / zp gradient sums
// ----------------------------------------------------------------------------
struct LsqAcc {
  double t1, t2, a, b;   // sum g(q-z), sum -(gm)(x/s/s), sum gm, sum -(g s)
};

__device__ __forceinline__ float lsq_elem(float x, float g, const QP &p, LsqAcc &acc) {
  const float u = x / p.s;
  const float r = __builtin_rintf(u + p.z);
  const float q = fq_clamp(r, p.lo, p.hi);
  const bool m = (r >= p.lo && r <= p.hi);
  const float gq = g * p.s;                 // MulBackward0 (self)
  const float gm = m ? gq : 0.0f;           // ClampBackward1
  const float t1 = g * (q - p.z);           // MulBackward0 (other)
  const float xs = u / p.s;                 // (self / other) / other
  const float t2 = (-gm) * xs;              // DivBackward0 (other)
  acc.t1 += (double)t1;
  acc.t2 += (double)t2;
  acc.a += (double)gm;                      // AddBackward0 (other)
  acc.b += (double)(-gq);                   // SubBackward0 (other)
  return gm / p.s;                          // DivBackward0 (self)
}

__device__ __forceinline__ void lsq_block_reduce(LsqAcc &c) {
  __shared__ double s[4][kWaves];
  c.t1 = wave_reduce(c.t1, AddD());
  c.t2 = wave_reduce(c.t2, AddD());
  c.a = wave_reduce(c.a, AddD());
  c.b = wave_reduce(c.b, AddD());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) { s[0][w] = c.t1; s[1][w] = c.t2; s[2][w] = c.a; s[3][w] = c.b; }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int i = 1; i < kWaves; ++i) { c.t1 += s[0][i]; c.t2 += s[1][i]; c.a += s[2][i]; c.b += s[3][i]; }
  __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_lsq_bwd(const float *__restrict__ g,
                                                    const float *__restrict__ x,
                                                    float *__restrict__ gx, int64_t n, int vec,
                                                    QPSrc src, int zp_learn, double gscale,
                                                    double *__restrict__ grad_out,
                                                    double *__restrict__ ws,
                                                    uint32_t *__restrict__ counter) {
  const QP p = load_qp(src);
  LsqAcc c{0.0, 0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (vec) {
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    const float4 *g4 = reinterpret_cast<const float4 *>(g);
    float4 *o4 = reinterpret_cast<float4 *>(gx);
    const int64_t n4 = n / 4;
    for (int64_t base = t0; base < n4; base += stride * 2) {
      float4 xv[2], gv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t i = base + u * stride;
        if (i < n4) { xv[u] = x4[i]; gv[u] = g4[i]; }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t i = base + u * stride;
        if (i < n4) {
          float4 o;
          o.x = lsq_elem(xv[u].x, gv[u].x, p, c);
          o.y = lsq_elem(xv[u].y, gv[u].y, p, c);
          o.z = lsq_elem(xv[u].z, gv[u].z, p, c);
          o.w = lsq_elem(xv[u].w, gv[u].w, p, c);
          o4[i] = o;
        }
      }
    }
    for (int64_t i = 4 * n4 + t0; i < n; i += stride) gx[i] = lsq_elem(x[i], g[i], p, c);
  } else {
    for (int64_t i = t0; i < n; i += stride) gx[i] = lsq_elem(x[i], g[i], p, c);
  }
  lsq_block_reduce(c);
  if (threadIdx.x == 0) {
    double *r = ws + (int64_t)blockIdx.x * kPartials;
    r[0] = c.t1; r[1] = c.t2; r[2] = c.a; r[3] = c.b;
  }
  if (!arrive_last(counter)) return;
  c = LsqAcc{0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < (int)gridDim.x; b += kBlock) {
    const double *r = ws + (int64_t)b * kPartials;
    c.t1 += r[0]; c.t2 += r[1]; c.a += r[2]; c.b += r[3];
  }
  lsq_block_reduce(c);
  if (threadIdx.x == 0) {
    grad_out[0] = (c.t1 + c.t2) * gscale;
    double gz = 0.0;
    if (zp_learn) {
      // ClampBackward of zero_point_rounding (uniform.py:101): in-range test on round(zp)
      const double zr = __builtin_rint(src.zdev ? *src.zdev : src.zhost);   // NaN -> not in range
      const bool zin = zr >= (double)p.lo && zr <= (double)p.hi;
      gz = zin ? (c.a + c.b) * gscale : 0.0;
    }
    grad_out[1] = gz;
    *counter = 0u;
  }
}

// ----------------------------------------------------------------------------
// host helpers
// ----------------------------------------------------------------------------
inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
inline bool aligned4(const void *p) { return ((uintptr_t)p & 3u) == 0; }

inline int flat_grid(int64_t items, int unroll) {
  int64_t b = cdiv(items, (int64_t)kBlock * unroll);
  if (b < 1) b = 1;
  if (b > kMaxReduceGrid) b = kMaxReduceGrid;
  return (int)b;
}

// blocks per row for the (row, chunk) kernels: one block per 4096 elements, at most
// ~16 blocks per CU over the whole grid and at most 65535 (chunks are grid-strided)
inline int64_t chunk_grid(int64_t rowlen, int64_t rows, bool vec) {
  int64_t c = vec ? cdiv(rowlen / 4, kChunk4) : cdiv(rowlen, kBlock);
  const int64_t cap = std::max<int64_t>(1, (256 * 16) / std::max<int64_t>(rows, 1));
  c = std::min(c, std::max<int64_t>(cap, 1));
  return std::max<int64_t>(1, std::min<int64_t>(c, 65535));
}

inline int launch_rc() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

template <bool STATS>
int pc_observe_dispatch(const float *x, float *y, uint8_t *c, uint8_t *mask, int64_t rows,
                        const PCArgs &a, bool vec, hipStream_t st) {
  const int64_t n4 = a.rowlen / 4;
  const dim3 grid((unsigned)rows), block(kBlock);
  if (vec && n4 <= 1 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<1, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else if (vec && n4 <= 2 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<2, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else if (vec && n4 <= 4 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<4, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else if (vec && n4 <= 6 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<6, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else if (vec && n4 <= 9 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<9, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else if (vec && n4 <= 12 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<12, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else if (vec && n4 <= 16 * kBlock)
    hipLaunchKernelGGL((k_pc_observe_fq_v4<16, STATS>), grid, block, 0, st, x, y, c, mask, a);
  else
    hipLaunchKernelGGL(k_pc_observe_fq_s, grid, block, 0, st, x, y, c, mask, a);
  return launch_rc();
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

int vsiq_fq_fwd_f32(const float *x, float *y, void *codes, uint8_t *mask, int64_t n,
                    const double *qp_dev, const double *scale_dev, double scale_host,
                    const double *zp_dev, double zp_host, int zp_round, int discrete, int qmin,
                    int qmax, void *stream) {
  if (n < 0 || qmin > qmax || (n > 0 && (!x || !y))) return VSIQ_E_ARG;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  QPSrc src{qp_dev, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax,
            qp_dev ? 0 : zp_round, discrete ? 1 : 0};
  const bool vec = (n % 4 == 0) && aligned16(x) && aligned16(y) &&
                   (!codes || aligned4(codes)) && (!mask || aligned4(mask));
  if (vec) {
    const int64_t n4 = n / 4;
    const int grid = (int)std::min<int64_t>(cdiv(n4, (int64_t)kBlock * kFqUnroll), 256 * 16);
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    float4 *y4 = reinterpret_cast<float4 *>(y);
    uint32_t *c4 = reinterpret_cast<uint32_t *>(codes);
    uint32_t *m4 = reinterpret_cast<uint32_t *>(mask);
    if (codes && mask)
      hipLaunchKernelGGL((k_fq_fwd_v4<true, true>), dim3(grid), dim3(kBlock), 0, st, x4, y4, c4, m4, n4, src);
    else if (codes)
      hipLaunchKernelGGL((k_fq_fwd_v4<true, false>), dim3(grid), dim3(kBlock), 0, st, x4, y4, c4, m4, n4, src);
    else if (mask)
      hipLaunchKernelGGL((k_fq_fwd_v4<false, true>), dim3(grid), dim3(kBlock), 0, st, x4, y4, c4, m4, n4, src);
    else
      hipLaunchKernelGGL((k_fq_fwd_v4<false, false>), dim3(grid), dim3(kBlock), 0, st, x4, y4, c4, m4, n4, src);
  } else {
    const int grid = (int)std::min<int64_t>(cdiv(n, kBlock), 256 * 16);
    hipLaunchKernelGGL(k_fq_fwd_s, dim3(grid), dim3(kBlock), 0, st, x, y, (uint8_t *)codes, mask, n, src);
  }
  return launch_rc();
}

int vsiq_observe_f32(const float *x, int64_t n, double *stats_out, float *run_minmax,
                     double *qp_out, int symmetric, double qden, double eps, double *ws,
                     int64_t ws_len, uint32_t *counter, void *stream) {
  if (n <= 0 || !x || !ws || !counter) return VSIQ_E_ARG;
  const bool vec = aligned16(x);
  const int grid = flat_grid(vec ? n / 4 + 1 : n, vec ? kFqUnroll : 1);
  if (ws_len < (int64_t)grid * kPartials) return VSIQ_E_WS;
  hipLaunchKernelGGL(k_observe, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, x, n,
                     vec ? 1 : 0, stats_out, run_minmax, qp_out, symmetric, qden, eps, ws, counter);
  return launch_rc();
}

int vsiq_observe_finalize(const double *stats, float *run_minmax, double *qp_out, int symmetric,
                          double qden, double eps, void *stream) {
  if (!stats) return VSIQ_E_ARG;
  hipLaunchKernelGGL(k_observe_finalize, dim3(1), dim3(kWave), 0, (hipStream_t)stream, stats,
                     run_minmax, qp_out, symmetric, qden, eps);
  return launch_rc();
}

int vsiq_pc_observe_fq_f32(const float *x, float *y, void *codes, uint8_t *mask, int64_t rows,
                           int64_t rowlen, float *run_min, float *run_max, double *scale_out,
                           double *zp_out, double *row_stats, int symmetric, int qmin, int qmax,
                           double qden, double eps, void *stream) {
  if (rows < 0 || rowlen <= 0 || qmin > qmax) return VSIQ_E_ARG;
  if (rows == 0) return 0;
  if (!x || !run_min || !run_max || !scale_out || !zp_out) return VSIQ_E_ARG;
  if (!y && (codes || mask)) return VSIQ_E_ARG;
  if (rows > 0x7fffffffLL) return VSIQ_E_ARG;
  PCArgs a{rowlen, run_min, run_max, scale_out, zp_out, row_stats, symmetric, (float)qmin,
           (float)qmax, qden, eps};
  const bool vec = (rowlen % 4 == 0) && aligned16(x) && (!y || aligned16(y)) &&
                   (!codes || aligned4(codes)) && (!mask || aligned4(mask));
  hipStream_t st = (hipStream_t)stream;
  uint8_t *c = (uint8_t *)codes;
  return row_stats ? pc_observe_dispatch<true>(x, y, c, mask, rows, a, vec, st)
                   : pc_observe_dispatch<false>(x, y, c, mask, rows, a, vec, st);
}

int vsiq_pc_fq_fwd_f32(const float *x, float *y, void *codes, uint8_t *mask, int64_t rows,
                       int64_t rowlen, const double *scale, const double *zp, int zp_round,
                       int qmin, int qmax, void *stream) {
  if (rows < 0 || rowlen <= 0 || qmin > qmax) return VSIQ_E_ARG;
  if (rows == 0) return 0;
  if (!x || !y || !scale || !zp || rows > 0x7fffffffLL) return VSIQ_E_ARG;
  PCFixed a{rowlen, scale, zp, zp_round, (float)qmin, (float)qmax};
  const bool vec = (rowlen % 4 == 0) && aligned16(x) && aligned16(y) &&
                   (!codes || aligned4(codes)) && (!mask || aligned4(mask));
  const int64_t chunks = chunk_grid(rowlen, rows, vec);
  const dim3 grid((unsigned)rows, (unsigned)chunks);
  if (vec)
    hipLaunchKernelGGL(k_pc_fq_fwd_v4, grid, dim3(kBlock), 0, (hipStream_t)stream, x, y,
                       (uint8_t *)codes, mask, a);
  else
    hipLaunchKernelGGL(k_pc_fq_fwd_s, grid, dim3(kBlock), 0, (hipStream_t)stream, x, y,
                       (uint8_t *)codes, mask, a);
  return launch_rc();
}

int vsiq_ste_bwd_f32(const float *g, const uint8_t *mask, float *gx, int64_t n,
                     const double *scale_dev, int64_t rowlen, double scale_host, void *stream) {
  if (n < 0) return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (!g || !mask || !gx) return VSIQ_E_ARG;
  if (!scale_dev || rowlen <= 0) rowlen = n;
  if (n % rowlen != 0) return VSIQ_E_ARG;
  const int64_t rows = n / rowlen;
  if (rows > 0x7fffffffLL) return VSIQ_E_ARG;
  const bool vec = (rowlen % 4 == 0) && aligned16(g) && aligned16(gx) && aligned4(mask);
  const int64_t chunks = chunk_grid(rowlen, rows, vec);
  const dim3 grid((unsigned)rows, (unsigned)chunks);
  if (vec)
    hipLaunchKernelGGL(k_ste_bwd_v4, grid, dim3(kBlock), 0, (hipStream_t)stream, g, mask, gx,
                       rowlen, scale_dev, scale_host);
  else
    hipLaunchKernelGGL(k_ste_bwd_s, grid, dim3(kBlock), 0, (hipStream_t)stream, g, mask, gx,
                       rowlen, scale_dev, scale_host);
  return launch_rc();
}

int vsiq_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t n,
                     const double *scale_dev, double scale_host, const double *zp_dev,
                     double zp_host, int zp_learn, int qmin, int qmax, double gscale,
                     double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
                     void *stream) {
  if (n <= 0 || !g || !x || !gx || !grad_out || !ws || !counter || qmin > qmax) return VSIQ_E_ARG;
  const bool vec = aligned16(g) && aligned16(x) && aligned16(gx);
  const int grid = flat_grid(vec ? n / 4 + 1 : n, vec ? 2 : 1);
  if (ws_len < (int64_t)grid * kPartials) return VSIQ_E_WS;
  // learnable zp: the forward used clamp(rint(zp)); a non-learnable zp is used as given
  QPSrc src{nullptr, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax,
            zp_learn, 0};
  hipLaunchKernelGGL(k_lsq_bwd, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, g, x, gx, n,
                     vec ? 1 : 0, src, zp_learn, gscale, grad_out, ws, counter);
  return launch_rc();
}

}  // extern "C"
