#pragma once
// vsiq_common.cuh — MI355X (gfx950 / CDNA4) kernels for VSIQuantization's
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
#include <atomic>

#include "vsiq.h"


namespace vsiq {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kWaves = kBlock / kWave;
constexpr int kMaxReduceGrid = 2048;   // minimum partial-record slots of a workspace
constexpr int kPartials = 8;           // doubles per partial record
constexpr int kArriveFlat = 128;       // grids above this arrive in two levels (arrive_last)
constexpr int kArriveGroups = 32;      // level-1 arrival counters (counter words 1..32)
constexpr int kFoldDirect = 2048;      // two-level arrivals up to this grid: one direct fold
static_assert(1 + kArriveGroups <= VSIQ_COUNTER_WORDS, "counter words");
constexpr int kObsGrid = 512;          // K2 grid-stride: workgroups (fixed: order independent of device)
constexpr int kObsU = 8;               // K2 grid-stride: groups per lane per step
constexpr int kFlatU = 2;              // 4-element groups per lane in the one-shot streaming kernels
constexpr int kLsqGroups = 16;         // max groups per lane in K4 (fewer workgroups -> fewer partials)
constexpr int kLsqPrefetch = 2;        // K4 groups in flight ahead of the one computing

typedef float f4 __attribute__((ext_vector_type(4)));

// tuning knobs (vsiq_set_tuning); -1 / 0 = automatic.  Atomics: vsiq_set_tuning may run
// on one host thread while another (autograd's backward thread) launches.
struct Tuning {
  std::atomic<int> nontemporal{1};         // nt hints on streamed loads/stores
  std::atomic<int> store_defer{-1};        // deferred store phase, units of 512 clocks (-1 = auto, 0 = off)
  std::atomic<int> pc_packed{1};           // per-channel with given qparams / K6: packed short rows (0 = per-row grid)
  std::atomic<int> obs_kernel{0};          // K2: 0 auto (grid-stride), 1 one-shot, 2 grid-stride
  std::atomic<int> lsq_groups{0};          // K4 groups per lane 2 / 4 / 8 / 16 (0 = by size)
  std::atomic<int> store_gate{-1};         // store gate ticks (10 ns) for one-round grids (-1 = auto, 0 = off)
  std::atomic<int> gate_autotune{1};       // store gate tuned online per launch site (0 = fixed estimate)
  std::atomic<int> xcd_order{2};           // XCD block order where neighbours share lines (k_lsq.hip K6 columns)
  std::atomic<int> k2o_form{0};            // K2o: 0 one-shot (one record per workgroup), 1 grid-stride (K2p's records)
  std::atomic<int> k2o_groups{0};          // K2o one-shot groups per lane 1 / 2 / 4 / 8 / 16 (0 = default 2)
  std::atomic<int> k2o_block{0};           // K2o one-shot lanes per workgroup 256 / 512 / 1024 (0 = default 256)
};
extern Tuning g_tune;

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// XCD-contiguous block order.  The dispatcher deals workgroups to the 8 XCDs round
// robin (block b -> XCD b % 8), each XCD with its own L2.  Where neighbouring blocks
// share cache lines (per-channel columns of short rows: a 400-byte row ends mid-line),
// that sends every shared line to two L2s and HBM twice.  xcd_block(b) is the logical
// block physical block b works on: XCD x walks one contiguous range of logical blocks,
// its concurrent blocks neighbours (a bijection on [0, grid)).
constexpr uint32_t kXcds = 8;
__device__ inline uint32_t xcd_block(uint32_t b, uint32_t grid) {
  const uint32_t x = b % kXcds, k = b / kXcds, per = grid / kXcds, rem = grid % kXcds;
  return x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
}

// Grid-stride trip count of a workgroup whose first item is `first` (uniform: it
// depends on blockIdx only, so loops on it are scalar branches and hipcc's
// s_waitcnt insertion stays exact; lanes past the end predicate their stores).
__device__ __forceinline__ int64_t block_iters(int64_t n, int64_t first, int64_t stride) {
  return first < n ? (n - first + stride - 1) / stride : 0;
}

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
  uint32_t fast;   // 0 when b itself is outside the safe range (then every element falls back)
};

__device__ __forceinline__ FastDiv make_fastdiv(float b) {
  FastDiv d;
  d.b = b;
  d.r = 1.0f / b;   // IEEE, once per thread
  const uint32_t ub = __float_as_uint(b) & 0x7fffffffu;
  d.fast = (ub - 0x20000000u) <= 0x3f000000u ? 1u : 0u;   // |b| in [2^-63, 2^63]
  return d;
}

// branch-free: RN(a/b) whenever fdiv_ok(a, d); garbage otherwise
__device__ __forceinline__ float fdiv_fast(float a, const FastDiv &d) {
  const float q0 = a * d.r;
  const float e0 = __builtin_fmaf(-q0, d.b, a);
  const float q1 = __builtin_fmaf(e0, d.r, q0);
  const float e1 = __builtin_fmaf(-q1, d.b, a);
  const float q2 = __builtin_fmaf(e1, d.r, q1);
  return (__float_as_uint(a) & 0x7fffffffu) ? q2 : q0;   // +-0 / b = a * r (signed zero)
}

// 1 when fdiv_fast(a, d) is RN(a/b); bitwise-combinable without branches
__device__ __forceinline__ uint32_t fdiv_ok(float a, const FastDiv &d) {
  const uint32_t ua = __float_as_uint(a) & 0x7fffffffu;
  return d.fast & (((ua - 0x20000000u) <= 0x3f000000u) | (ua == 0u));
}

// IEEE when asked, else the fast path (used by the rare per-group fallback)
template <bool IEEE>
__device__ __forceinline__ float fdiv_t(float a, const FastDiv &d) {
  return IEEE ? a / d.b : fdiv_fast(a, d);
}

__device__ __forceinline__ float fdiv(float a, const FastDiv &d) {
  return fdiv_ok(a, d) ? fdiv_fast(a, d) : a / d.b;
}

// ----------------------------------------------------------------------------
// element arithmetic (quantizers/uniform.py:95, 55)
// ----------------------------------------------------------------------------
struct QP {
  float s, z, lo, hi;
  int discrete;
  FastDiv d;
  uint32_t fast;   // quantizer fast path allowed (fq_fast_qp; K3 also: row finite, no NaN)
};

template <bool IEEE>
__device__ __forceinline__ float fq_round(float x, const QP &p) {
  float u = fdiv_t<IEEE>(x, p.d);   // fp32 true division x / fp32(scale), correctly rounded
  u = u + p.z;                      // + fp32(zero_point); -0.0 + 0.0 -> +0.0 like torch.add
  return __builtin_rintf(u);        // torch.round: half to even
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

template <bool IEEE>
__device__ __forceinline__ Elem fq_elem(float x, const QP &p) {
  const float r = fq_round<IEEE>(x, p);
  const float q = fq_clamp(r, p.lo, p.hi);
  Elem e;
  e.y = p.discrete ? q : (q - p.z) * p.s;
  e.code = fq_code_byte(q);
  e.m = (r >= p.lo && r <= p.hi);   // ClampBackward1: inclusive, on the rounded value
  return e;
}

// the 4 elements of a group; the IEEE division is taken (divergently, rarely) only
// for lanes holding an element outside the fast-division range
__device__ __forceinline__ void fq_group(f4 v, const QP &p, Elem &e0, Elem &e1, Elem &e2, Elem &e3) {
  e0 = fq_elem<false>(v.x, p);
  e1 = fq_elem<false>(v.y, p);
  e2 = fq_elem<false>(v.z, p);
  e3 = fq_elem<false>(v.w, p);
  const uint32_t ok = fdiv_ok(v.x, p.d) & fdiv_ok(v.y, p.d) & fdiv_ok(v.z, p.d) & fdiv_ok(v.w, p.d);
  if (!ok) {
    e0 = fq_elem<true>(v.x, p);
    e1 = fq_elem<true>(v.y, p);
    e2 = fq_elem<true>(v.z, p);
    e3 = fq_elem<true>(v.w, p);
  }
}

// ----------------------------------------------------------------------------
// Quantizer fast path: no per-element division check.
//
// The forward output depends on x/s only through c = clamp(rint(x/s + zp)).
// With s in [2^-20, 2^62] (positive), zp finite and either integer-valued or
// |zp| >= 2^-12, and |x| <= 2^62:
//   * |x| >= 2^-63: the two Markstein steps give RN(x/s) exactly (fdiv proof);
//   * |x| <  2^-63: the true quotient is below 2^-43 and the computed one below
//     2^-38, both under half an ulp of any |zp| >= 2^-12, so RN(q + zp) = zp for
//     both; for zp = 0, rint(q) = +-0 and copysign(q, x) makes the zero's sign
//     that of x/s (s > 0), as IEEE; for integer zp != 0 both give zp.
// So c (value AND sign) is the reference's for every such x; NaN/inf/huge x
// and out-of-range scales take the IEEE path.  vsiq_selftest_fq() checks this
// for all 2^32 inputs on the GPU.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fq_fast_qp(float s, float z) {
  const uint32_t us = __float_as_uint(s);   // sign bit set -> huge -> rejected
  const bool s_ok = (us - 0x35800000u) <= (0x5e800000u - 0x35800000u);   // [2^-20, 2^62]
  const float az = __builtin_fabsf(z);
  const bool z_ok = az <= 0x1p62f && (z == __builtin_rintf(z) || az >= 0x1p-12f);
  return (s_ok && z_ok) ? 1u : 0u;
}

__device__ __forceinline__ float fq_quot(float x, const FastDiv &d) {
  const float q0 = x * d.r;
  const float e0 = __builtin_fmaf(-q0, d.b, x);
  const float q1 = __builtin_fmaf(e0, d.r, q0);
  const float e1 = __builtin_fmaf(-q1, d.b, x);
  const float q2 = __builtin_fmaf(e1, d.r, q1);
  return __builtin_copysignf(q2, x);
}

__device__ __forceinline__ uint32_t fq_x_ok(float x) { return __builtin_fabsf(x) <= 0x1p62f ? 1u : 0u; }   // NaN -> 0

// x not NaN / inf here, so r is finite and the clamp needs no NaN care:
// c = r <= hi ? r : hi, then r >= lo ? c : lo  (== torch.clamp incl. -0.0)
__device__ __forceinline__ Elem fq_elem_fast(float x, const QP &p) {
  const float r = __builtin_rintf(fq_quot(x, p.d) + p.z);
  const bool le = r <= p.hi, ge = r >= p.lo;
  const float c = ge ? (le ? r : p.hi) : p.lo;
  Elem e;
  e.y = p.discrete ? c : (c - p.z) * p.s;
  e.code = (uint32_t)((int)c) & 0xffu;
  e.m = le && ge;
  return e;
}

// group of a row whose fast flag (p.fast) is uniform over the workgroup
__device__ __forceinline__ void fq_group_row(f4 v, const QP &p, Elem &e0, Elem &e1, Elem &e2,
                                             Elem &e3) {
  if (p.fast) {
    e0 = fq_elem_fast(v.x, p);
    e1 = fq_elem_fast(v.y, p);
    e2 = fq_elem_fast(v.z, p);
    e3 = fq_elem_fast(v.w, p);
  } else {
    fq_group(v, p, e0, e1, e2, e3);
  }
}

// group of a flat tensor: one range compare per element, IEEE for the rare group
// holding a NaN / inf / |x| > 2^62 (or for out-of-range qparams)
__device__ __forceinline__ void fq_group_flat(f4 v, const QP &p, Elem &e0, Elem &e1, Elem &e2,
                                              Elem &e3) {
  e0 = fq_elem_fast(v.x, p);
  e1 = fq_elem_fast(v.y, p);
  e2 = fq_elem_fast(v.z, p);
  e3 = fq_elem_fast(v.w, p);
  const uint32_t ok = p.fast & fq_x_ok(v.x) & fq_x_ok(v.y) & fq_x_ok(v.z) & fq_x_ok(v.w);
  if (!ok) {
    e0 = fq_elem<true>(v.x, p);
    e1 = fq_elem<true>(v.y, p);
    e2 = fq_elem<true>(v.z, p);
    e3 = fq_elem<true>(v.w, p);
  }
}

// ----------------------------------------------------------------------------
// STE backward division gx = (m ? RN(g*s) : 0) / s
// p = RN(g*s) is within half an ulp of g*s, so g is a faithful
// quotient of p/s and ONE Markstein step from it is RN(p/s):
//   q = RN(g + RN(p - g*s) * r),   r = RN(1/s),
// the residual p - g*s being exact (it is the product's rounding error).  Valid
// for s in [2^-60, 2^60] and |g| in [2^-40, 2^64) (p and the quotient normal, no
// overflow) or g == +-0 (copysign(q, p): -0/s = -0).  Other groups (NaN, inf,
// tiny g, extreme scales) take the IEEE division.  vsiq_selftest_fq(mode 1)
// checks it for all 2^32 g on the GPU.
// ----------------------------------------------------------------------------
struct SteDiv {
  float s, r;
  uint32_t fast;
};

__device__ __forceinline__ SteDiv make_stediv(float s) {
  SteDiv d;
  d.s = s;
  d.r = 1.0f / s;
  d.fast = (__float_as_uint(s) - 0x21800000u) <= (0x5d800000u - 0x21800000u) ? 1u : 0u;
  return d;
}

__device__ __forceinline__ float ste_quot(float g, const SteDiv &d) {
  const float p = g * d.s;                       // MulBackward0
  const float e = __builtin_fmaf(-g, d.s, p);    // exact residual
  return __builtin_copysignf(__builtin_fmaf(e, d.r, g), p);
}

// branch-free (bitwise-combinable) validity of ste_quot for one element
__device__ __forceinline__ uint32_t ste_ok(float g) {
  const float a = __builtin_fabsf(g);
  return ((uint32_t)(a >= 0x1p-40f) & (uint32_t)(a < 0x1p64f)) | (uint32_t)(g == 0.0f);
}

__device__ __forceinline__ float ste_ieee(float g, bool m, const SteDiv &d) {
  return (m ? g * d.s : 0.0f) / d.s;             // ClampBackward1, DivBackward0 (IEEE)
}

// ----------------------------------------------------------------------------
// Activation fused in front of the activation quantizer (K5): ConvBnReLU's
// F.relu / F.silu (fused.py:124-134) followed by quantize_out (fake_quantize.py:49-50).
// The forward reads the conv output c once; the backward re-derives act(c) and
// applies the activation's backward to the quantizer's grad_x.
//   relu:  c < 0 ? 0 : c          (torch CPU: relu(-0.0) = -0.0, relu(NaN) = NaN)
//          bwd: threshold_backward(g, relu(c), 0) = c <= 0 ? 0 : g  (NaN passes g)
//   silu:  bit for bit what torch's CPU silu_kernel computes (the reference runs F.silu
//          on CPU tensors): see "SiLU as torch's CPU kernel computes it" below.
// ----------------------------------------------------------------------------
enum { kActNone = 0, kActRelu = 1, kActSilu = 2 };

// ----------------------------------------------------------------------------
// SiLU as torch's CPU kernel computes it (aten/src/ATen/native/cpu/Activation.cpp,
// silu_kernel / silu_backward_kernel under cpu_kernel_vec):
//   vectorized loop (2 vectors per step):  c / (1 + Sleef_expf_u10(-c))
//   scalar remainder of each chunk:        c / (1 + expf(-c))          (glibc libm)
//   backward, same split:  (g * sig) * fma(c, 1 - sig, 1),  sig = 1 / (1 + exp(-c))
// The two exps differ in the last bit for ~3.5 % of activation-range inputs, so which
// elements take the scalar path matters: TensorIterator runs serially below
// GRAIN_SIZE = 32768 elements (or on one thread), else at::parallel_for splits [0, n)
// into nt = min(threads, ceil(n / 32768)) chunks of ceil(n / nt); every chunk runs the
// vector loop over its first len - len % W elements (W = 2 x the vector width: 32 on
// AVX-512, 16 on AVX2) and the scalar code over the rest.  SiluRef {W, threads}
// travels in the act argument (VSIQ_ACT_SILU_REF, include/vsiq.h); W = 0 = every
// element on the vector path.  Both exps are ported op for op below and were checked
// against the reference host for all 2^32 inputs (tests/test_silu_oracle.py pins the
// oracle restatement, oracle/silu_ref.c, against torch's CPU kernel).
// ----------------------------------------------------------------------------
struct SiluRef {
  int32_t w, t;   // 2 x vector width (0: vector path only), reference thread count
};
struct SiluLay {          // chunk layout of one tensor of n elements (silu_lay)
  int64_t chunk, last;    // chunk length; start of the last chunk
  int64_t thr, thr_last;  // first scalar offset inside a chunk / inside the last chunk
  double inv;             // RN(1 / chunk)
  int32_t on;             // 0: no element of this tensor takes the scalar path
};

constexpr int64_t kTorchGrain = 32768;   // at::internal::GRAIN_SIZE

__host__ __device__ inline SiluLay silu_lay(int64_t n, SiluRef r) {
  SiluLay L{};
  if (r.w <= 0 || n <= 0) return L;
  int64_t nt = 1;
  if (n >= kTorchGrain && r.t > 1) {
    nt = (n + kTorchGrain - 1) / kTorchGrain;
    if (nt > r.t) nt = r.t;
  }
  L.chunk = (n + nt - 1) / nt;
  L.last = ((n + L.chunk - 1) / L.chunk - 1) * L.chunk;
  L.thr = L.chunk - L.chunk % r.w;
  L.thr_last = (n - L.last) - (n - L.last) % r.w;
  L.inv = 1.0 / (double)L.chunk;
  L.on = (L.thr != L.chunk || L.thr_last != n - L.last) ? 1 : 0;
  return L;
}

// bit j set: element e0 + j takes torch's scalar path (elements past n: don't care)
__host__ __device__ inline uint32_t silu_scalar4(int64_t e0, const SiluLay &L) {
  int64_t cs = L.last;
  if (e0 < L.last) {
    cs = (int64_t)((double)e0 * L.inv) * L.chunk;   // off by at most one chunk
    if (cs > e0) cs -= L.chunk;
    else if (cs + L.chunk <= e0) cs += L.chunk;
  }
  uint32_t m = 0;
  for (int j = 0; j < 4; ++j) {
    const int64_t e = e0 + j;
    const int64_t c = (e - cs >= L.chunk && cs < L.last) ? cs + L.chunk : cs;
    m |= (uint32_t)(e - c >= (c == L.last ? L.thr_last : L.thr)) << j;
  }
  return m;
}

__host__ __device__ __forceinline__ float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ __forceinline__ uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }

// Sleef_expf16_u10 (sleefsimdsp.c xexpf, FMA build), op for op.  A restatement of SLEEF
// (Boost Software License 1.0, Copyright Naoki Shibata and contributors); see NOTICE.
__host__ __device__ __forceinline__ float sleef_expf_u10(float d) {
  const float qf = __builtin_rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  const int q = (int)__builtin_fminf(__builtin_fmaxf(qf, -256.0f), 256.0f);   // |d| > 104: replaced below
  float s = __builtin_fmaf((float)q, -0.693145751953125f, d);
  s = __builtin_fmaf((float)q, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
  u = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
  u = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
  u = __builtin_fmaf(u, s, 0.166666671633720397949219f);
  u = __builtin_fmaf(u, s, 0.5f);
  u = 1.0f + __builtin_fmaf(s * s, u, s);
  const int h = q >> 1;   // vldexp2: two exact power-of-two steps
  u = (u * u2f((uint32_t)(h + 0x7f) << 23)) * u2f((uint32_t)(q - h + 0x7f) << 23);
  if (d < -104.0f) u = 0.0f;
  if (d > 100.0f) u = __builtin_inff();
  return d != d ? d : u;
}

// 2^(i/32) - (i << 47) as doubles' bits (glibc's __exp2f_data.tab).  This table and
// glibc_expf below restate glibc's sysdeps/ieee754/flt-32/e_expf.c + e_exp2f_data.c
// (LGPL-2.1-or-later, Copyright Free Software Foundation, Inc.; see NOTICE).
#define VSIQ_EXP2F_TAB \
  0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL, \
  0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL, \
  0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL, \
  0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL, \
  0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL, \
  0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL, \
  0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL, \
  0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL \

static __constant__ uint64_t kExp2fTabDev[32] = {VSIQ_EXP2F_TAB};
static const uint64_t kExp2fTabHost[32] = {VSIQ_EXP2F_TAB};

// glibc expf (sysdeps/ieee754/flt-32/e_expf.c, the FMA ifunc variant), op for op:
// 2^(k/32) from a 32-entry table times a cubic in r, in double
__host__ __device__ inline float glibc_expf(float x) {
#ifdef __HIP_DEVICE_COMPILE__
  const uint64_t *kT = kExp2fTabDev;
#else
  const uint64_t *kT = kExp2fTabHost;
#endif
  const uint32_t ux = f2u(x), abstop = (ux >> 20) & 0x7ffu;
  if (abstop >= 0x42bu) {   // |x| >= 88 or NaN
    if (ux == 0xff800000u) return 0.0f;
    if (abstop >= 0x7f8u) return x + x;
    if (x > 0x1.62e42ep6f) return __builtin_inff();
    if (x < -0x1.9fe368p6f) return 0.0f;
  }
  const double InvLn2N = 0x1.71547652b82fep+0 * 32.0, Shift = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32768.0, C1 = 0x1.ebfce50fac4f3p-3 / 1024.0,
               C2 = 0x1.62e42ff0c52d6p-1 / 32.0;
  const double xd = (double)x;
  const double kd0 = __builtin_fma(InvLn2N, xd, Shift);
  const uint64_t ki = __builtin_bit_cast(uint64_t, kd0);
  const double kd = kd0 - Shift;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  const double s = __builtin_bit_cast(double, kT[ki % 32] + (ki << 47));
  const double z = __builtin_fma(C0, r, C1);
  double y = __builtin_fma(C2, r, 1.0);
  y = __builtin_fma(z, r * r, y);
  return (float)(y * s);
}

template <bool SCALAR>
__host__ __device__ __forceinline__ float silu_exp(float c) {
  return SCALAR ? glibc_expf(-c) : sleef_expf_u10(-c);
}

template <bool SCALAR>
__host__ __device__ __forceinline__ float silu_fwd(float c) {
  return c / (1.0f + silu_exp<SCALAR>(c));
}

template <bool SCALAR>
__host__ __device__ __forceinline__ float silu_bwd(float g, float c) {
  const float sig = 1.0f / (1.0f + silu_exp<SCALAR>(c));
  return (g * sig) * __builtin_fmaf(c, 1.0f - sig, 1.0f);
}

template <int ACT>
__device__ __forceinline__ float act_fwd(float c) {
  if (ACT == kActRelu) return c < 0.0f ? 0.0f : c;
  if (ACT == kActSilu) return silu_fwd<false>(c);
  return c;
}

template <int ACT>
__device__ __forceinline__ f4 act_fwd4(f4 v) {
  if (ACT == kActNone) return v;
  f4 o;
  o.x = act_fwd<ACT>(v.x); o.y = act_fwd<ACT>(v.y); o.z = act_fwd<ACT>(v.z); o.w = act_fwd<ACT>(v.w);
  return o;
}

// act of the group whose first element is e0: SiLU elements on torch's scalar path
// take glibc's exp (rare: at most W - 1 elements per chunk; divergent)
template <int ACT>
__device__ __forceinline__ f4 act_fwd4_at(f4 v, int64_t e0, const SiluLay &L) {
  f4 o = act_fwd4<ACT>(v);
  if constexpr (ACT == kActSilu) {
    if (L.on) {
      const uint32_t sm = silu_scalar4(e0, L);
      if (sm) {
        if (sm & 1u) o.x = silu_fwd<true>(v.x);
        if (sm & 2u) o.y = silu_fwd<true>(v.y);
        if (sm & 4u) o.z = silu_fwd<true>(v.z);
        if (sm & 8u) o.w = silu_fwd<true>(v.w);
      }
    }
  }
  return o;
}

template <int ACT>
__device__ __forceinline__ float act_bwd(float g, float c) {
  if (ACT == kActRelu) return c <= 0.0f ? 0.0f : g;
  if (ACT == kActSilu) return silu_bwd<false>(g, c);
  return g;
}

template <int ACT>
__device__ __forceinline__ f4 act_bwd4(f4 g, f4 c) {
  if (ACT == kActNone) return g;
  f4 o;
  o.x = act_bwd<ACT>(g.x, c.x); o.y = act_bwd<ACT>(g.y, c.y);
  o.z = act_bwd<ACT>(g.z, c.z); o.w = act_bwd<ACT>(g.w, c.w);
  return o;
}

template <int ACT>
__device__ __forceinline__ f4 act_bwd4_at(f4 g, f4 c, int64_t e0, const SiluLay &L) {
  f4 o = act_bwd4<ACT>(g, c);
  if constexpr (ACT == kActSilu) {
    if (L.on) {
      const uint32_t sm = silu_scalar4(e0, L);
      if (sm) {
        if (sm & 1u) o.x = silu_bwd<true>(g.x, c.x);
        if (sm & 2u) o.y = silu_bwd<true>(g.y, c.y);
        if (sm & 4u) o.z = silu_bwd<true>(g.z, c.z);
        if (sm & 8u) o.w = silu_bwd<true>(g.w, c.w);
      }
    }
  }
  return o;
}

// The act argument of the C ABI: VSIQ_ACT_NONE / _RELU / _SILU in the low byte; for
// SiLU, bits 8-15 = W and bits 16-30 = the reference thread count (VSIQ_ACT_SILU_REF)
__host__ __device__ inline int act_kind(int act) { return act & 0xff; }
inline SiluRef act_ref(int act) { return SiluRef{(act >> 8) & 0xff, (act >> 16) & 0x7fff}; }
inline bool act_ok(int act) {
  const int k = act_kind(act);
  if (act < 0 || k < kActNone || k > kActSilu) return false;
  if (k != kActSilu) return (act >> 8) == 0;
  const int w = (act >> 8) & 0xff;
  return w == 0 || w == 8 || w == 16 || w == 32 || w == 64;
}
inline SiluLay act_lay(int act, int64_t n) {
  return act_kind(act) == kActSilu ? silu_lay(n, act_ref(act)) : SiluLay{};
}

// runtime act -> template dispatch (on the activation kind)
#define VSIQ_ACT(ACTV, F, ...)                                                 \
  (act_kind(ACTV) == kActRelu ? F<kActRelu>(__VA_ARGS__)                       \
                              : act_kind(ACTV) == kActSilu ? F<kActSilu>(__VA_ARGS__) : F<kActNone>(__VA_ARGS__))

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

// A wave-uniform f64 read as a scalar load (s_load_dwordx2).  Scalar loads count on
// lgkmcnt, so a kernel can issue its streaming loads first and then wait for its qparams
// without waiting for those; the same read as a global_load is ordered with them on vmcnt.
// (Round 6, the learnable per-channel forward at C2: the compiler put the scale / zp
// global_loads and their vmcnt(0) waits ahead of the x loads -- the gate sweep's optimum
// sat 0.65 us later than K3's and the kernel at 0.75 against K3's 0.79.)  `p` must be the
// same in every lane; a read-only value of an earlier launch (the scalar cache is
// invalidated at each dispatch).
__device__ __forceinline__ double ld_uniform_f64(const double *p) {
  const uint64_t u = (uint64_t)(uintptr_t)p;
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  return *(const __attribute__((address_space(4))) double *)((hi << 32) | lo);
}

// UNI: every pointer of `a` is wave-uniform -> scalar loads (ld_uniform_f64)
template <bool UNI = false>
__device__ __forceinline__ double ld_qp_f64(const double *p) {
  if constexpr (UNI) return ld_uniform_f64(p);
  else return *p;
}

template <bool UNI = false>
__device__ __forceinline__ QP load_qp(const QPSrc &a) {
  double s, z;
  if (a.qp) {
    s = ld_qp_f64<UNI>(a.qp + VSIQ_QP_SCALE);
    z = ld_qp_f64<UNI>(a.qp + VSIQ_QP_ZP);
  } else {
    s = a.sdev ? ld_qp_f64<UNI>(a.sdev) : a.shost;
    z = a.zdev ? ld_qp_f64<UNI>(a.zdev) : a.zhost;
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
  p.fast = fq_fast_qp(p.s, p.z);
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
// (measured on MI355X, C2 step: write-through sc1 / sc0 sc1 / nt sc1 and plain stores are
// 0.1-4 us slower per launch than nt stores, in K3 and the STE backward alike)
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
  // unconditional (clamped) scalar loads keep the vmcnt bookkeeping exact
  const int64_t e = 4 * i, l = len - 1;
  f4 v;
  v.x = row[e];
  const float y = row[e + 1 < l ? e + 1 : l], z = row[e + 2 < l ? e + 2 : l], w = row[e + 3 < l ? e + 3 : l];
  v.y = e + 1 < len ? y : v.x;
  v.z = e + 2 < len ? z : v.x;
  v.w = e + 3 < len ? w : v.x;
  return v;
}

// group i clamped into [0, ng): loads are issued unconditionally (no branch around a
// load, so hipcc's s_waitcnt counting stays exact); callers predicate the stores
template <bool VEC, bool NT>
__device__ __forceinline__ f4 load_group_c(const float *row, int64_t i, int64_t ng, int64_t len) {
  return load_group<VEC, NT>(row, i < ng ? i : ng - 1, len);
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

// One fake-quantized group i (elements 4i..4i+3 of a row of `len`) ready for its
// stores: y, the 4 code bytes, and the 4 ballot words of the wave's mask chunk
// (wave-uniform, SGPRs).  Each path packs its own result, so the fast/IEEE merge
// is a merge of SGPR words rather than of per-lane booleans.
struct GroupOut {
  f4 o;
  uint32_t c;
  uint64_t b[4];
};

template <bool VEC, bool CODES, bool MASK>
__device__ __forceinline__ GroupOut fq_pack(const Elem (&e)[4], int64_t i, int64_t len) {
  GroupOut g;
  g.o.x = e[0].y; g.o.y = e[1].y; g.o.z = e[2].y; g.o.w = e[3].y;
  g.c = CODES ? (e[0].code | (e[1].code << 8) | (e[2].code << 16) | (e[3].code << 24)) : 0u;
  if (MASK) {
    if (VEC) {   // len % 4 == 0: a group is wholly valid or wholly past the end
      const bool in = 4 * i < len;
      g.b[0] = __ballot(e[0].m && in); g.b[1] = __ballot(e[1].m && in);
      g.b[2] = __ballot(e[2].m && in); g.b[3] = __ballot(e[3].m && in);
    } else {
      const int nv = valid_in_group(i, len);   // 0 past the end
      g.b[0] = __ballot(e[0].m && nv > 0); g.b[1] = __ballot(e[1].m && nv > 1);
      g.b[2] = __ballot(e[2].m && nv > 2); g.b[3] = __ballot(e[3].m && nv > 3);
    }
  } else {
    g.b[0] = g.b[1] = g.b[2] = g.b[3] = 0;
  }
  return g;
}

// Fast path of a group (see fq_elem_fast).  The clamp compares are taken as wave
// lane masks (v_cmp -> SGPR pair): they drive the selects directly and their AND
// IS the STE mask ballot, so no per-lane boolean is ever materialized.
constexpr int kCmpOGE = 3, kCmpOLE = 5;   // llvm FCmp predicates

template <bool VEC, bool CODES, bool MASK>
__device__ __forceinline__ GroupOut fq_out_fast(f4 v, const QP &p, int64_t i, int64_t len) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  float yv[4];
  GroupOut g;
  g.c = 0;
  const int nv = VEC ? 4 : valid_in_group(i, len);
  const uint64_t in_all = (MASK && VEC) ? __ballot(4 * i < len) : 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float r = __builtin_rintf(fq_quot(x[j], p.d) + p.z);
    const uint64_t le = __builtin_amdgcn_fcmpf(r, p.hi, kCmpOLE);
    const uint64_t ge = __builtin_amdgcn_fcmpf(r, p.lo, kCmpOGE);
    float c = __builtin_amdgcn_inverse_ballot_w64(le) ? r : p.hi;
    c = __builtin_amdgcn_inverse_ballot_w64(ge) ? c : p.lo;
    yv[j] = p.discrete ? c : (c - p.z) * p.s;
    if (CODES) g.c |= ((uint32_t)((int)c) & 0xffu) << (8 * j);
    if (MASK) g.b[j] = le & ge & (VEC ? in_all : __ballot(nv > j));
    else g.b[j] = 0;
  }
  g.o.x = yv[0]; g.o.y = yv[1]; g.o.z = yv[2]; g.o.w = yv[3];
  return g;
}

template <bool VEC, bool CODES, bool MASK>
__device__ __forceinline__ GroupOut fq_out_slow(f4 v, const QP &p, int64_t i, int64_t len) {
  Elem e[4];
  fq_group(v, p, e[0], e[1], e[2], e[3]);
  return fq_pack<VEC, CODES, MASK>(e, i, len);
}

// group of a row whose p.fast is uniform over the workgroup
template <bool VEC, bool CODES, bool MASK>
__device__ __forceinline__ GroupOut fq_out_row(f4 v, const QP &p, int64_t i, int64_t len) {
  if (p.fast) return fq_out_fast<VEC, CODES, MASK>(v, p, i, len);
  return fq_out_slow<VEC, CODES, MASK>(v, p, i, len);
}

// group of a flat tensor: one range compare per element; a wave holding any NaN /
// inf / |x| > 2^62 (or out-of-range qparams) takes the checked path as a whole
template <bool VEC, bool CODES, bool MASK>
__device__ __forceinline__ GroupOut fq_out_flat(f4 v, const QP &p, int64_t i, int64_t len) {
  const uint32_t ok = p.fast & fq_x_ok(v.x) & fq_x_ok(v.y) & fq_x_ok(v.z) & fq_x_ok(v.w);
  if (__ballot(!ok) == 0) return fq_out_fast<VEC, CODES, MASK>(v, p, i, len);
  return fq_out_slow<VEC, CODES, MASK>(v, p, i, len);
}

// Mask words of several groups gathered into lanes: lane 4*slot + j receives word
// j of slot `slot` (v_writelane, no select chains); one store per lane later.
__device__ __forceinline__ void mask_put(uint32_t &lo, uint32_t &hi, int slot, const uint64_t (&b)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t l = 4 * slot + j, wl = (uint32_t)b[j], wh = (uint32_t)(b[j] >> 32);
    // lane select in M0 (two SGPR operands would break gfx9's constant-bus limit)
    asm("v_writelane_b32 %0, %1, m0" : "+v"(lo) : "s"(wl), "{m0}"(l));
    asm("v_writelane_b32 %0, %1, m0" : "+v"(hi) : "s"(wh), "{m0}"(l));
  }
}

template <bool VEC, bool NT, bool CODES>
__device__ __forceinline__ void fq_store_out(float *yr, uint8_t *cr, int64_t i, int64_t ng, int64_t len,
                                             const GroupOut &g) {
  if (i < ng) {
    store_group<VEC, NT>(yr, i, len, g.o);
    if (CODES) {
      if (VEC) reinterpret_cast<uint32_t *>(cr)[i] = g.c;
      else
        for (int j = 0; j < valid_in_group(i, len); ++j) cr[4 * i + j] = (uint8_t)(g.c >> (8 * j));
    }
  }
}

// ----------------------------------------------------------------------------
// wave / block reductions (wave64)
// ----------------------------------------------------------------------------
// Wave64 all-reduce on DPP (no LDS traffic): quad swaps, row rotations by 4 and 8
// (every lane then holds its 16-lane row's result), row_bcast:15 / row_bcast:31 to
// fold the four rows into lane 63, read back into an SGPR.  Fixed order, hence
// deterministic.  Requires the whole wave active (all call sites are uniform).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp32(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xF, false);
}

template <int CTRL, int ROW_MASK = 0xF, typename T>
__device__ __forceinline__ T dpp(T v, T old) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit lanes");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp32<CTRL, ROW_MASK>(__builtin_bit_cast(uint32_t, v),
                                                      __builtin_bit_cast(uint32_t, old)));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v), o = __builtin_bit_cast(uint64_t, old);
    const uint32_t lo = dpp32<CTRL, ROW_MASK>((uint32_t)u, (uint32_t)o);
    const uint32_t hi = dpp32<CTRL, ROW_MASK>((uint32_t)(u >> 32), (uint32_t)(o >> 32));
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

template <typename T>
__device__ __forceinline__ T readlane63(T v) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}

template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
  const T id = Op::identity();
  v = op(v, dpp<0xB1>(v, id));         // quad_perm [1,0,3,2]
  v = op(v, dpp<0x4E>(v, id));         // quad_perm [2,3,0,1]
  v = op(v, dpp<0x124>(v, id));        // row_ror:4
  v = op(v, dpp<0x128>(v, id));        // row_ror:8  -> every lane: its row's result
  v = op(v, dpp<0x142, 0xA>(v, id));   // row_bcast:15 into rows 1, 3
  v = op(v, dpp<0x143, 0xC>(v, id));   // row_bcast:31 into rows 2, 3 -> lane 63: the wave's
  return readlane63(v);
}

struct MinOp {
  static __device__ float identity() { return __builtin_inff(); }
  __device__ float operator()(float a, float b) const { return fminf(a, b); }
};
struct MaxOp {
  static __device__ float identity() { return -__builtin_inff(); }
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
struct MinD {
  static __device__ double identity() { return __builtin_inf(); }
  __device__ double operator()(double a, double b) const { return __builtin_fmin(a, b); }
};
struct MaxD {
  static __device__ double identity() { return -__builtin_inf(); }
  __device__ double operator()(double a, double b) const { return __builtin_fmax(a, b); }
};
struct AddD {
  static __device__ double identity() { return 0.0; }
  __device__ double operator()(double a, double b) const { return a + b; }
};
struct OrU {
  static __device__ uint32_t identity() { return 0u; }
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; }
};
struct AddU {
  static __device__ uint32_t identity() { return 0u; }
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};

// Cross-workgroup partials without fences (MI355X_MICROARCH.md "Valid forms",
// row 1): thread 0 of each workgroup stores its partial record write-through
// (sc1), drains it (s_waitcnt vmcnt(0)) and only then bumps the arrival counter;
// the workgroup whose add returns gridDim.x-1 takes an agent acquire and reads
// every record with sc1 loads.  No per-workgroup release fence: a release writes
// back the XCD's whole L2 (buffer_wbl2), which behind streaming stores cost
// microseconds per workgroup.
__device__ __forceinline__ void partial_store(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double partial_load(const double *p) {
  return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Call after thread 0 has partial_store()d its record; returns true (block-uniform)
// in the last workgroup to arrive.  Arrivals on one address serialize at the memory
// side (~10 ns each: +5 us per 512 workgroups, measured on K2), so grids above
// kArriveFlat arrive in two levels: workgroup b bumps group counter 1 + b % G, the
// group's last arrival resets it and bumps counter[0]; the last of the G group-lasts
// is the last workgroup.  counter: VSIQ_COUNTER_WORDS words, counter[0] is reset by
// the caller's epilogue.
__device__ __forceinline__ bool arrive_last(uint32_t *counter) {
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t nb = gridDim.x;
    int last;
    if (nb <= (uint32_t)kArriveFlat) {
      const uint32_t t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (t == nb - 1);
    } else {
      const uint32_t g = blockIdx.x % kArriveGroups;
      const uint32_t members = (nb - g + kArriveGroups - 1) / kArriveGroups;
      const uint32_t t =
          __hip_atomic_fetch_add(counter + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = 0;
      if (t == members - 1) {
        __hip_atomic_store(counter + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t t0 =
            __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (t0 == (uint32_t)kArriveGroups - 1);
      }
    }
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

// Last-workgroup combine of the per-workgroup partial records: thread t folds
// records t, t+B, t+2B, ... in that fixed order (deterministic), but the loads of 4
// consecutive records are issued together -- a serial load->add chain over thousands
// of records was a multi-microsecond tail on large grids.
template <int K, typename F>
__device__ __forceinline__ void fold_partials(const double *ws, int nrec, F &&f) {
  for (int b0 = threadIdx.x; b0 < nrec; b0 += 4 * kBlock) {
    double r[4][K];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = b0 + u * kBlock < nrec ? b0 + u * kBlock : nrec - 1;
#pragma unroll
      for (int k = 0; k < K; ++k) r[u][k] = partial_load(ws + (int64_t)b * kPartials + k);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b0 + u * kBlock < nrec) f(r[u]);
  }
}

// ----------------------------------------------------------------------------
// Two-level fold of per-workgroup partial records (K doubles each, record b at
// ws + b * kPartials, stored by thread 0 with partial_store).  Op supplies
//   static constexpr int K;  init(double (&)[K]);  add(double (&)[K], const double (&)[K]);
//   wave(double (&)[K])  (wave_reduce of every field, any lane holds the result).
// Grids up to kArriveFlat: the last workgroup folds every record.  Larger grids:
// workgroup b belongs to group b % G; the group's last arrival folds the group's
// records (b = g, g + G, ...) into group record nb + g, and the last of the G group
// folds combines those.  Fixed assignment and trees: deterministic for a given grid.
// The workspace needs nb + kArriveGroups records (vsiq_workspace_doubles).
// ----------------------------------------------------------------------------
template <typename Op>
__device__ __forceinline__ void fold_block(const double *ws, uint32_t first, uint32_t count, uint32_t stride,
                                           double (&a)[Op::K]) {
  constexpr int K = Op::K;
  Op::init(a);
  for (uint32_t j0 = threadIdx.x; j0 < count; j0 += 4 * kBlock) {
    double r[4][K];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t j = j0 + u * kBlock < count ? j0 + u * kBlock : count - 1;
#pragma unroll
      for (int k = 0; k < K; ++k) r[u][k] = partial_load(ws + (int64_t)(first + j * stride) * kPartials + k);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (j0 + u * kBlock < count) Op::add(a, r[u]);
  }
  __shared__ double s_w[kWaves][K];
  Op::wave(a);
  if (threadIdx.x % kWave == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) s_w[threadIdx.x / kWave][k] = a[k];
  __syncthreads();
  if (threadIdx.x == 0)
    for (int w = 1; w < kWaves; ++w) {
      double r[K];
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] = s_w[w][k];
      Op::add(a, r);
    }
  __syncthreads();
}

// Returns true (block-uniform) in the workgroup that holds the fold of every record,
// in thread 0's `a`; counter: VSIQ_COUNTER_WORDS words, counter[0] reset by the caller.
template <typename Op>
__device__ __forceinline__ bool fold_arrivals(double *ws, uint32_t *counter, double (&a)[Op::K]) {
  const uint32_t nb = gridDim.x;
  if (nb <= (uint32_t)kArriveFlat) {
    if (!arrive_last(counter)) return false;
    fold_block<Op>(ws, 0, nb, 1, a);
    return true;
  }
  __shared__ int s_role;
  const uint32_t g = blockIdx.x % kArriveGroups;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t members = (nb - g + kArriveGroups - 1) / kArriveGroups;
    const uint32_t t = __hip_atomic_fetch_add(counter + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int role = (t == members - 1);
    if (role) {
      __hip_atomic_store(counter + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_role = role;
  }
  __syncthreads();
  if (!s_role) return false;
  if (nb <= (uint32_t)kFoldDirect) {
    // grids whose records one workgroup folds in <= 2 rounds of loads: the group-last
    // arrives on counter[0] at once and the last of all folds every record in block
    // order -- two memory round trips fewer than folding per group first (no group
    // fold, no group-record store + drain)
    if (threadIdx.x == 0) {
      const uint32_t t0 = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (t0 == (uint32_t)kArriveGroups - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_role = last ? 2 : 0;
    }
    __syncthreads();
    if (s_role != 2) return false;
    fold_block<Op>(ws, 0, nb, 1, a);
    return true;
  }
  fold_block<Op>(ws, g, (nb - g + kArriveGroups - 1) / kArriveGroups, kArriveGroups, a);
  if (threadIdx.x == 0) {
    double *gr = ws + (int64_t)(nb + g) * kPartials;
#pragma unroll
    for (int k = 0; k < Op::K; ++k) partial_store(gr + k, a[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t0 = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t0 == (uint32_t)kArriveGroups - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_role = last ? 2 : 0;
  }
  __syncthreads();
  if (s_role != 2) return false;
  fold_block<Op>(ws + (int64_t)nb * kPartials, 0, kArriveGroups, 1, a);
  return true;
}

// ----------------------------------------------------------------------------
// Wave-0 arrival for kernels that also STORE a streamed output (K4, K7).  A plain
// s_waitcnt vmcnt(0) before the arrival atomic also waits for the workgroup's own
// output stores to be acknowledged (stores and loads share vmcnt on CDNA), which
// keeps every workgroup resident one store round trip longer and stalls the next
// round of workgroups (K4 at 6.5M elements: 23.4 us with the fold vs 17.7 without,
// MI355X).  Instead waves 1..3 store and leave; wave 0 publishes the block record
// with lane 0 (only that store is outstanding when it drains), arrives, THEN stores.
// fold_wave / wave_arrive run in one wave (64 lanes, no __syncthreads).
// ----------------------------------------------------------------------------
// kWaveFold records per lane in flight: one memory round trip folds 64 x kWaveFold
// records (each round is a dependent round trip to the coherence point)
constexpr int kWaveFold = 8;
constexpr uint32_t kWaveFoldDirect = kWave * kWaveFold;   // 512: one round

template <typename Op>
__device__ __forceinline__ void fold_wave(const double *ws, uint32_t first, uint32_t count, uint32_t stride,
                                          double (&a)[Op::K]) {
  constexpr int K = Op::K;
  Op::init(a);
  const uint32_t lane = threadIdx.x % kWave;
  for (uint32_t j0 = lane; j0 < count; j0 += kWaveFold * kWave) {
    double r[kWaveFold][K];
#pragma unroll
    for (int u = 0; u < kWaveFold; ++u) {
      const uint32_t j = j0 + u * kWave < count ? j0 + u * kWave : count - 1;
#pragma unroll
      for (int k = 0; k < K; ++k) r[u][k] = partial_load(ws + (int64_t)(first + j * stride) * kPartials + k);
    }
#pragma unroll
    for (int u = 0; u < kWaveFold; ++u)
      if (j0 + u * kWave < count) Op::add(a, r[u]);
  }
  Op::wave(a);
}

// LDS-only workgroup barrier: LDS writes complete, then s_barrier -- no vmcnt wait,
// so stores issued before it stay in flight.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Called by all lanes of wave 0 with the block record `rec` (lane 0's value used).
// Block `blk` of a grid of nb blocks whose records live at ws[first .. first + nb)
// (+ kArriveGroups group records after them for nb > kFoldDirect); counter words as
// in fold_arrivals.  Returns true (wave-uniform) in the block that holds, in `a`
// (every lane), the fold of every record: flat for nb <= kArriveFlat, else arrivals
// on counter 1 + blk % 32 then counter 0, with one direct fold of all records up to
// kWaveFoldDirect blocks (one round of loads) and per-group folds above (one round per
// group up to 16384 blocks, then one over the 32 group records).  Fixed trees:
// deterministic.
// `after_arrival()` runs in wave 0 right after the block's own arrival, before any
// fold: the caller's stores go there (issued after the record drain; their registers
// are free again before the fold's loads).
template <typename Op, typename F>
__device__ __forceinline__ bool wave_arrive(double *ws, uint32_t first, uint32_t nb, uint32_t blk,
                                            uint32_t *counter, const double (&rec)[Op::K],
                                            double (&a)[Op::K], F &&after_arrival) {
  constexpr int K = Op::K;
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t g = blk % kArriveGroups;
  const uint32_t members = (nb - g + kArriveGroups - 1) / kArriveGroups;
  int role = 0;
  if (lane == 0) {
    double *r = ws + (int64_t)(first + blk) * kPartials;
#pragma unroll
    for (int k = 0; k < K; ++k) partial_store(r + k, rec[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (nb <= (uint32_t)kArriveFlat) {
      const uint32_t t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      role = (t == nb - 1) ? 2 : 0;
    } else {
      const uint32_t t = __hip_atomic_fetch_add(counter + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == members - 1) {
        __hip_atomic_store(counter + 1 + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        role = 1;
      }
    }
    if (role == 1 && nb <= kWaveFoldDirect) {   // straight on to counter 0
      const uint32_t t0 = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      role = (t0 == (uint32_t)kArriveGroups - 1) ? 2 : 0;
    }
    if (role) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  role = __builtin_amdgcn_readfirstlane(role);
  after_arrival();
  if (role == 0) return false;
  if (role == 2) {
    fold_wave<Op>(ws, first, nb, 1, a);
    return true;
  }
  // group-last of a large grid: fold the group, publish the group record, arrive on 0
  fold_wave<Op>(ws, first + g, members, kArriveGroups, a);
  int last = 0;
  if (lane == 0) {
    double *gr = ws + (int64_t)(first + nb + g) * kPartials;
#pragma unroll
    for (int k = 0; k < K; ++k) partial_store(gr + k, a[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t0 = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t0 == (uint32_t)kArriveGroups - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  last = __builtin_amdgcn_readfirstlane(last);
  if (!last) return false;
  fold_wave<Op>(ws + (int64_t)(first + nb) * kPartials, 0, kArriveGroups, 1, a);
  return true;
}

// f64 qparams from the running min/max (observers/minmax.py:49-74).
// min_val <= 0 <= max_val always holds (state starts at 0/0, minmax.py:28-29).
__host__ __device__ __forceinline__ void minmax_qparams(double mn, double mx, int sym, double qden,
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

// The stats record (VSIQ_ST_*) of one call from its folded {min, max, nan count,
// sum|x|, sum x, sum x^2}: quantization_manager.py:66-68's fp32 mean(|x|) / mean /
// unbiased std, NaN when the call held a NaN (torch's fp32 reductions are NaN then).
__host__ __device__ __forceinline__ void write_stats(double *__restrict__ st, const double (&f)[6], int64_t n) {
  const double dn = (double)n;
  const bool has_nan = f[2] > 0.0;
  st[VSIQ_ST_MIN] = (double)(float)f[0];   // NaN-ignoring; see VSIQ_ST_NAN
  st[VSIQ_ST_MAX] = (double)(float)f[1];
  st[VSIQ_ST_NAN] = f[2];
  st[VSIQ_ST_SUMABS] = f[3];
  st[VSIQ_ST_SUM] = f[4];
  st[VSIQ_ST_SUMSQ] = f[5];
  st[VSIQ_ST_N] = dn;
  const double mean = f[4] / dn;
  const double var = (f[5] - f[4] * mean) / (dn - 1.0);
  st[VSIQ_ST_MEANABS] = has_nan ? __builtin_nan("") : (double)(float)(f[3] / dn);
  st[VSIQ_ST_MEAN] = has_nan ? __builtin_nan("") : (double)(float)mean;
  st[VSIQ_ST_STD] = (has_nan || n < 2) ? __builtin_nan("")
                                       : (double)(float)__builtin_sqrt(var > 0.0 ? var : 0.0);
}

// Running-state update + qparams (observers/minmax.py:42-47 then :49-74).  A call
// whose tensor holds a NaN changes nothing: `nan < v` is False in Python.
// Returns the f64 (scale, zp) in *s_out / *z_out when those are given.
__host__ __device__ __forceinline__ void observer_update(float cmn, float cmx, bool has_nan,
                                                         float *run_minmax, double *qp_out, int sym,
                                                         double qden, double eps, double *s_out = nullptr,
                                                         double *z_out = nullptr) {
  float mn = 0.f, mx = 0.f;
  if (run_minmax) { mn = run_minmax[0]; mx = run_minmax[1]; }
  if (!has_nan) {
    if (cmn < mn) mn = cmn;
    if (cmx > mx) mx = cmx;
  }
  if (run_minmax) { run_minmax[0] = mn; run_minmax[1] = mx; }
  if (qp_out || s_out) {
    double s, z;
    minmax_qparams((double)mn, (double)mx, sym, qden, eps, &s, &z);
    if (qp_out) {
      qp_out[VSIQ_QP_SCALE] = s;
      qp_out[VSIQ_QP_ZP] = z;
      qp_out[VSIQ_QP_MIN] = mn;
      qp_out[VSIQ_QP_MAX] = mx;
    }
    if (s_out) { *s_out = s; *z_out = z; }
  }
}


// ----------------------------------------------------------------------------
// host helpers
// ----------------------------------------------------------------------------
inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
inline bool aligned4(const void *p) { return ((uintptr_t)p & 3u) == 0; }
inline bool aligned8(const void *p) { return ((uintptr_t)p & 7u) == 0; }

// Deferred store phase.  A grid that streams its whole input in one round (every
// workgroup resident at once, all loads issued at t = 0) runs faster on MI355X's HBM3E
// when a workgroup holds its stores back for ~2 us after its loads have landed: the
// device then reads, and then writes, instead of interleaving the two from the first
// returned load on (C2 size, 1024 workgroups of 256 lanes x 9 groups: STE 14.0 ->
// 11.9 us, 5.4 -> 6.3 TB/s; measured, tools/exp/phase_*).  Called after a barrier, with
// a wave-uniform unit count (512 clocks each); a pure delay, never a correctness issue.
__device__ __forceinline__ void defer_stores(uint32_t units) {
  for (uint32_t k = 0; k < units; ++k) __builtin_amdgcn_s_sleep(8);
}

// Store gate: hold a one-round grid's stores until `ticks` of the constant wall
// clock (s_memrealtime, 100 MHz on MI355X) have passed since the workgroup started,
// so that the grid's reads run as one phase and its writes as the next (HBM
// read/write turnarounds) without delaying the rows that finish reading after the
// gate (unlike defer_stores).  A pure delay, wave-uniform (scalar clock), never a
// correctness issue.
__device__ __forceinline__ void store_gate_clock(uint64_t t0, uint32_t ticks) {
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

struct GateClk {
  uint64_t t0;   // the workgroup's start on the wall clock (gate != 0)
};

// at the workgroup's start, before its loads are issued
__device__ __forceinline__ GateClk gate_begin(uint32_t gate) {
  return GateClk{gate ? (uint64_t)wall_clock64() : 0ull};
}

// before the workgroup's first store (wave-uniform)
__device__ __forceinline__ void gate_pass(uint32_t gate, const GateClk &c) {
  if (gate) store_gate_clock(c.t0, gate);
}

// Host: the store gate of a one-round grid (gate_tune.hip).  Eligible grids: >= 2
// workgroups per CU and all of them resident at once (`occ` per CU); grids under 2
// workgroups per CU gain nothing and grids of more than one round lose (the next round
// waits behind the gate).  The gate's optimum is sharp and moves with the box's HBM:
// K3 at C2 on one MI355X (tools/exp/gate_timeline.py) 4.52 / 5.00 / 5.28 / 5.60 /
// 6.03 us -> 12.8 / 12.2 / 12.4 / 12.7 / 13.1 us per launch (15.2 without a gate), and
// the fixed 1.05 x (read bytes at 7.5 TB/s) of round 1 sat at the no-gate time on
// another box.  So the gate is tuned online per (kernel, grid, bytes, device): the
// first launches of a site cycle through candidate gates of f x the 7.5 TB/s estimate
// (and no gate), each timed with a pair of HIP events around the launch (no host
// sync: results are harvested by later calls), and the best median is kept.  Capture
// (HIP graphs) uses the current best or the estimate.  Results are identical for every
// gate (a pure delay).  Override: vsiq_set_tuning(VSIQ_TUNE_STORE_GATE, ticks), 0 =
// off; VSIQ_TUNE_GATE_AUTOTUNE 0 = the 1.05 x estimate without tuning.
constexpr uint32_t kGateAuto = 0xffffffffu;   // PCArgs::gate: resolved at launch
int device_cus();
int device_cus(int dev);
int occupancy_blocks(const void *kernel, int block);
int device_wall_clock_khz();
int device_wall_clock_khz(int dev);
struct GateSel {
  uint32_t gate = 0;    // wall-clock ticks for the launch (0 = no gate)
  void *timing = nullptr;   // tuner sample in flight (record its end after the launch)
};
GateSel store_gate_select(const char *label, const void *kernel, int64_t grid, int occ, int64_t read_bytes,
                          hipStream_t st);
void store_gate_launched(GateSel &sel, hipStream_t st);

// host: defer_stores units for a one-round grid of `grid` workgroups of 256 lanes x 9
// groups (override: vsiq_set_tuning(VSIQ_TUNE_STORE_DEFER, units)).  Automatic only
// where it was measured to pay (`auto_ok`: the STE backward, 9216-element rows x 512 /
// 768 / 1024 rows: -8 / -15 / -16 %): 1.5..4 workgroups per CU, ~0.3 x the read phase
// (2.5 units per workgroup per CU).  K3's row reduction already delays its stores
// (deferring further only cost time there), and grids of more than one round lose.
int device_cus();
inline uint32_t store_defer_units(int64_t grid, bool auto_ok) {
  if (g_tune.store_defer >= 0) return (uint32_t)g_tune.store_defer;
  if (!auto_ok) return 0;
  const int64_t cus = device_cus();
  if (2 * grid < 3 * cus || grid > 4 * cus) return 0;
  return (uint32_t)((5 * grid + cus) / (2 * cus));
}

// Packed short rows for per-channel kernels with given qparams (k_pc.hip, K6): one
// workgroup takes R = kPackElems / rowlen whole rows (a contiguous flat range of
// 4-element groups, kPackGroups per lane) when rowlen % 4 == 0 and R >= 2.
constexpr int kPackGroups = 4;                          // groups per lane
constexpr int kPackElems = kBlock * kPackGroups * 4;    // 4096 elements per workgroup
constexpr int kPackMaxRows = kBlock;                    // one row's qparams per thread
constexpr int64_t kPackMaxRowlen = kPackElems / 2;      // >= 2 rows per workgroup

inline bool pc_packed(int64_t rowlen) { return rowlen % 4 == 0 && rowlen <= kPackMaxRowlen; }
// the forward (no reduction) keeps the per-row grid from 1600 up: measured on MI355X at
// 256x64x40x40 axis 1, per-row 36.7 us vs packed 42.5; at 20x20 rows packed 18.3 vs 38.9
inline bool pc_packed_fwd(int64_t rowlen) { return pc_packed(rowlen) && rowlen <= kPackElems / 4; }
inline int64_t pc_pack_rows(int64_t rowlen) { return std::min<int64_t>(kPackMaxRows, kPackElems / rowlen); }

// one-shot streaming grid: every lane owns kFlatU groups, no loop (a loop around
// loads + stores makes hipcc wait for the stores at the loop header: on CDNA the
// stores share vmcnt with the loads)
inline int64_t oneshot_grid(int64_t groups) {
  return std::max<int64_t>(1, cdiv(groups, (int64_t)kBlock * kFlatU));
}

// K4 groups per lane: 4.  Since the two-level fold (fold_arrivals) a workgroup's
// epilogue no longer serializes on one counter, and 4 groups per lane stream better
// than 16 (16-deep straight-line code) at every size measured on MI355X
// (tools/exp/k4_sizes.py, fused ReLU: 105M elements 230 -> 216 us, 3.3M 19.1 -> 15.4,
// 296K 16.4 -> 7.3); 2 per lane pays the epilogue twice as often (105M: 342 us).
// Override: VSIQ_TUNE_LSQ_GROUPS (2 / 4 / 16).
// From 20M elements on, 8 per lane: half the workgroups, half the arrivals
// (C3 77M: 161.5 -> 156.1 us, 26M: 59.8 -> 58.1; at 3.3M 4 stays faster).
inline int lsq_groups_per_lane(int64_t groups) {
  if (g_tune.lsq_groups > 0) return g_tune.lsq_groups;
  return groups >= (int64_t)5 << 20 ? 8 : 4;
}

inline int64_t lsq_grid(int64_t groups, int per_lane) {
  return std::max<int64_t>(1, cdiv(groups, (int64_t)kBlock * per_lane));
}

inline int64_t lsq_grid(int64_t groups) { return lsq_grid(groups, lsq_groups_per_lane(groups));
}

// partial records a reducing grid writes (its own + the group records of fold_arrivals)
inline int64_t fold_records(int64_t grid) { return grid + (grid > kArriveFlat ? kArriveGroups : 0); }


// every exported entry point ends with launch_rc(): the count of library calls that
// launched (gate_tune.hip), so a store-gate burst sample never spans another kernel of
// this library between two launches of its site
extern std::atomic<uint64_t> g_lib_launches;

inline int launch_rc() {
  g_lib_launches.fetch_add(1, std::memory_order_relaxed);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// dispatch helpers: runtime flags -> template instantiations
#define VSIQ_B2(F, A, B, ...)                                 \
  ((A) ? ((B) ? F<true, true>(__VA_ARGS__) : F<true, false>(__VA_ARGS__)) \
       : ((B) ? F<false, true>(__VA_ARGS__) : F<false, false>(__VA_ARGS__)))

}  // namespace vsiq
