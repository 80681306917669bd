// k_body.cuh — block bodies shared by the single-tensor kernels (K1 k_fq.hip, K4
// k_lsq.hip) and the multi-tensor launches (k_multi.hip).  A body processes block
// `blk` of its tensor's grid, so a multi-tensor launch maps blockIdx.x -> (tensor,
// blk) and runs exactly the per-element code of the single-tensor kernel.
#pragma once
#include "vsiq_common.cuh"

namespace vsiq {

// A body's qparams: a QP computed by the caller, or a callable that loads them (round 6:
// called once the body's first loads are issued, so a kernel's qparam reads -- scalar
// loads, load_qp<true> -- overlap its streaming loads instead of preceding them)
__device__ __forceinline__ const QP &qp_of(const QP &p) { return p; }
template <class F>
__device__ __forceinline__ QP qp_of(const F &f) { return f(); }

// ----------------------------------------------------------------------------
// K1: y = fq(act(x)), one-shot (kFlatU groups per lane, no loop: exact vmcnt)
// ----------------------------------------------------------------------------
// U groups per lane: kFlatU, or 9 for a one-round grid whose stores wait behind the
// store gate (gc: gate_begin at the workgroup start; gate 0 = no gate).
template <bool VEC, bool NT, bool CODES, bool MASK, int ACT, int U = kFlatU, class QF = QP>
__device__ __forceinline__ void fq_fwd_block(const float *__restrict__ x, float *__restrict__ y,
                                             uint8_t *__restrict__ codes, uint64_t *__restrict__ mask,
                                             int64_t n, const QF &qf, int64_t blk, GateClk gc = GateClk{0},
                                             uint32_t gate = 0, const SiluLay &L = SiluLay{}) {
  const int64_t ng = cdiv(n, 4);
  const int64_t base = blk * kBlock * U + threadIdx.x;   // lanes chunk-aligned
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = load_group_c<VEC, NT>(x, base + u * kBlock, ng, n);
  const QP &p = qp_of(qf);
  GroupOut go[U];
  uint32_t mlo = 0, mhi = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    go[u] = fq_out_flat<VEC, CODES, MASK>(act_fwd4_at<ACT>(v[u], 4 * (base + u * kBlock), L), p,
                                          base + u * kBlock, n);
    if (MASK) mask_put(mlo, mhi, u, go[u].b);
  }
  gate_pass(gate, gc);
  const int lane = threadIdx.x % kWave;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kBlock;
    if (i - lane >= ng) break;   // whole wave past the end (uniform)
    fq_store_out<VEC, NT, CODES>(y, codes, i, ng, n, go[u]);
  }
  if (MASK && lane < 4 * U) {   // lane 4u+j: word j of slot u's chunk
    const int64_t first = base - lane + (lane >> 2) * kBlock;
    if (first < ng) mask[4 * (first / kWave) + (lane & 3)] = ((uint64_t)mhi << 32) | mlo;
  }
}

// ----------------------------------------------------------------------------
// K4: learnable (LSQ) backward, grad_x + f64 scale / zp gradient sums
// ----------------------------------------------------------------------------
struct LsqAcc {
  double t, z;   // sum [g(q-z) + -(gm)(x/s/s)] ; sum [gm + -(g s)]
};

// grad_x's division RN(RN(g*s)/s) in one Markstein step from g (the STE backward's
// quotient, vsiq_common.cuh ste_quot: g is a faithful quotient of RN(g*s)/s) -- for s in
// [2^-60, 2^60] (both ends included), positive (ste_fast_s, uniform), and g inside
// ste_ok; 4 instead of ~8 instructions per element.  Bitwise RN(gm/s) there
// (vsiq_selftest_fq mode 1 proves the quotient over all 2^32 gradients).
__device__ __forceinline__ uint32_t ste_fast_s(const FastDiv &d) {
  return (__float_as_uint(d.b) - 0x21800000u) <= (0x5d800000u - 0x21800000u) ? 1u : 0u;
}

// RN(a/b) up to the sign of a zero quotient (fdiv_fast without its signed-zero select),
// for quotients whose zero sign cannot matter: the STEQ element's x/s (it only enters
// rint(u + z), where +-0 + z gives the same r, and u/s) and u/s (it only multiplies into
// a gradient term whose zero sign the f64 sum absorbs: the accumulator is never -0).
// Same conditions as fdiv_fast (fdiv_ok; a == +-0 gives a zero).
__device__ __forceinline__ float fdiv_fast_nz(float a, const FastDiv &d) {
  const float q0 = a * d.r;
  const float e0 = __builtin_fmaf(-q0, d.b, a);
  const float q1 = __builtin_fmaf(e0, d.r, q0);
  const float e1 = __builtin_fmaf(-q1, d.b, a);
  return __builtin_fmaf(e1, d.r, q1);
}

// r = rint(u + z) and its clamp q = clamp(r, lo, hi) as one med3, m = (q == r): the same
// m as r in [lo, hi] for every r (NaN: false either way), the same q for finite r (the
// only r the fast paths use; a zero's sign in q - z is absorbed like fdiv_fast_nz's)
struct RQM {
  float r, q;
  bool m;
};
__device__ __forceinline__ RQM lsq_rqm(float u, const QP &p) {
  RQM o;
  o.r = __builtin_rintf(u + p.z);
  o.q = __builtin_amdgcn_fmed3f(o.r, p.lo, p.hi);
  o.m = o.q == o.r;
  return o;
}

// one element of the learnable backward; returns grad_x, adds the f64 gradient terms
// (STEQ: grad_x by the one-step STE quotient -- the caller checked ste_fast_s and the
// group test lsq_fast_ok4x)
template <bool ZPL, bool IEEE, bool STEQ = false>
__device__ __forceinline__ float lsq_elem(float x, float g, const QP &p, LsqAcc &acc, bool valid) {
  if (STEQ) {   // the fast path's element (every quotient in range, x finite)
    // a lane past the tensor's end takes g = 0: its terms are +-0, which the accumulator
    // absorbs (it starts at +0 and never becomes -0), and its grad_x is not stored
    g = valid ? g : 0.0f;
    const float u = fdiv_fast_nz(x, p.d);
    const RQM e = lsq_rqm(u, p);
    const float gq = g * p.d.b;               // MulBackward0 (self); d.b is s
    const float gm = e.m ? gq : 0.0f;         // ClampBackward1
    const float t1 = g * (e.q - p.z);         // MulBackward0 (other)
    const float t2 = (-gm) * fdiv_fast_nz(u, p.d);   // DivBackward0 (other): -(gm) * ((x/s)/s)
    acc.t += (double)t1 + (double)t2;
    // AddBackward0 + SubBackward0 (other): gm + (-gq) is +0 when in range (acc starts at
    // +0 and never becomes -0, so adding +0 is a no-op) and -gq when clamped -- the same
    // bits with one conversion and one f64 add fewer
    if (ZPL) acc.z += e.m ? 0.0 : -(double)gq;
    // DivBackward0 (self): ste_quot_d from the product already formed; 0/s signed like IEEE
    const float qd = __builtin_copysignf(__builtin_fmaf(__builtin_fmaf(-g, p.d.b, gq), p.d.r, g), gq);
    return e.m ? qd : 0.0f * p.d.r;
  }
  const float u = fdiv_t<IEEE>(x, p.d);
  const float r = __builtin_rintf(u + p.z);
  const float q = fq_clamp(r, p.lo, p.hi);
  const bool m = (r >= p.lo && r <= p.hi);
  const float gq = g * p.s;                 // MulBackward0 (self)
  const float gm = m ? gq : 0.0f;           // ClampBackward1
  const float t1 = g * (q - p.z);           // MulBackward0 (other)
  const float xs = fdiv_t<IEEE>(u, p.d);    // (self / other) / other
  const float t2 = (-gm) * xs;              // DivBackward0 (other)
  // lanes past the tensor's end (valid false) add +0 terms: selects, not exec branches
  // (acc starts at +0.0, so adding +0.0 never changes its bits)
  acc.t += valid ? (double)t1 + (double)t2 : 0.0;
  if (ZPL) acc.z += (valid && !m) ? -(double)gq : 0.0;   // AddBackward0 + SubBackward0 (other), as above
  return fdiv_t<IEEE>(gm, p.d);             // DivBackward0 (self)
}

// all three divisions of an element inside the fast-division range?
__device__ __forceinline__ uint32_t lsq_fast_ok(float x, float g, const QP &p) {
  const float u = fdiv_fast(x, p.d);
  const float r = __builtin_rintf(u + p.z);
  const bool m = (r >= p.lo && r <= p.hi);
  const float gm = m ? g * p.s : 0.0f;
  return fdiv_ok(x, p.d) & fdiv_ok(u, p.d) & fdiv_ok(gm, p.d);
}

// The STEQ element's conditions for a whole group, as two integer range trees instead
// of per-element compares: every x/s and u/s inside fdiv_ok's [2^-63, 2^63] and every
// in-range g inside ste_ok's [2^-40, 2^64).  u's range is implied by x's instead of
// tested: with s in [2^-60, 2^60] (ste_fast_s), |x| in [s * 2^-61, s * 2^61] (both
// products exact: s * 2^-61 >= 2^-121 is normal) gives |x/s| in [2^-61, 2^61], so RN(x/s)
// is inside [2^-63, 2^63]; x = +-0 gives u = +-0.  One tree over x and the in-range g
// with the bounds [max(2^-40, s * 2^-61), min(2^63, s * 2^61)] -- inside fdiv_ok (x) and
// ste_ok (g).  NaN / inf fail (their bits are above 2^63); zeros wrap to 0xffffffff in
// the "- 1" tree.  The caller checked ste_fast_s (which implies d.fast).
__device__ __forceinline__ uint32_t lsq_fast_ok4x(f4 xv, f4 gv, const QP &p) {
  const uint32_t lo = max(0x2b800000u, __float_as_uint(p.d.b * 0x1p-61f));
  const uint32_t hi = min(0x5f000000u, __float_as_uint(p.d.b * 0x1p61f));
  const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
  uint32_t mx = 0u, mn = 0xffffffffu;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float u = fdiv_fast_nz(xs[k], p.d);
    const bool m = lsq_rqm(u, p).m;
    const uint32_t a = __float_as_uint(xs[k]) & 0x7fffffffu;
    const uint32_t c = m ? (__float_as_uint(gs[k]) & 0x7fffffffu) : 0x3f800000u;   // 1.0: g unused
    mx = max(mx, max(a, c));
    mn = min(mn, min(a - 1u, c - 1u));
  }
  return (mx <= hi && mn >= lo - 1u) ? 1u : 0u;
}

struct LsqFold {   // partial record {sum t, sum z}
  static constexpr int K = 2;
  __device__ static void init(double (&a)[2]) { a[0] = a[1] = 0.0; }
  __device__ static void add(double (&a)[2], const double (&r)[2]) { a[0] += r[0]; a[1] += r[1]; }
  __device__ static void wave(double (&a)[2]) {
    a[0] = wave_reduce(a[0], AddD());
    a[1] = wave_reduce(a[1], AddD());
  }
};

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

// xc: the loaded input -- the quantizer input itself, or (ACT) the pre-activation c
// whose act(c) the forward quantized; grad_x then goes through the act's backward.
// Returns the group's grad_x (not stored).
template <bool ZPL, int ACT>
__device__ __forceinline__ f4 lsq_group_out(int64_t i, int64_t ng, int64_t n, f4 xc, f4 gv, const QP &p,
                                            LsqAcc &c, const SiluLay &L = SiluLay{}) {
  const f4 xv = act_fwd4_at<ACT>(xc, 4 * i, L);
  const int nv = i < ng ? valid_in_group(i, n) : 0;
  f4 o;
  if (ste_fast_s(p.d) && lsq_fast_ok4x(xv, gv, p)) {
    o.x = lsq_elem<ZPL, false, true>(xv.x, gv.x, p, c, nv > 0);
    o.y = lsq_elem<ZPL, false, true>(xv.y, gv.y, p, c, nv > 1);
    o.z = lsq_elem<ZPL, false, true>(xv.z, gv.z, p, c, nv > 2);
    o.w = lsq_elem<ZPL, false, true>(xv.w, gv.w, p, c, nv > 3);
    return act_bwd4_at<ACT>(o, xc, 4 * i, L);
  }
  const uint32_t ok = lsq_fast_ok(xv.x, gv.x, p) & lsq_fast_ok(xv.y, gv.y, p) & lsq_fast_ok(xv.z, gv.z, p) &
                      lsq_fast_ok(xv.w, gv.w, p);
  if (ok) {
    o.x = lsq_elem<ZPL, false>(xv.x, gv.x, p, c, nv > 0);
    o.y = lsq_elem<ZPL, false>(xv.y, gv.y, p, c, nv > 1);
    o.z = lsq_elem<ZPL, false>(xv.z, gv.z, p, c, nv > 2);
    o.w = lsq_elem<ZPL, false>(xv.w, gv.w, p, c, nv > 3);
  } else {   // rare (divergent): an element outside the fast-division range
    o.x = lsq_elem<ZPL, true>(xv.x, gv.x, p, c, nv > 0);
    o.y = lsq_elem<ZPL, true>(xv.y, gv.y, p, c, nv > 1);
    o.z = lsq_elem<ZPL, true>(xv.z, gv.z, p, c, nv > 2);
    o.w = lsq_elem<ZPL, true>(xv.w, gv.w, p, c, nv > 3);
  }
  return act_bwd4_at<ACT>(o, xc, 4 * i, L);
}

template <bool VEC, bool NT, bool ZPL, int ACT>
__device__ __forceinline__ void lsq_group(float *gx, int64_t i, int64_t ng, int64_t n, f4 xc, f4 gv,
                                          const QP &p, LsqAcc &c) {
  const f4 o = lsq_group_out<ZPL, ACT>(i, ng, n, xc, gv, p, c);
  if (i < ng) store_group<VEC, NT>(gx, i, n, o);
}

// Block `blk` of the K4 grid: G groups per lane, straight-line (fully unrolled):
// group k+kLsqPrefetch is loaded while group k computes, so x/g loads stay in flight
// and s_waitcnt counts are exact.  Adds this thread's terms to c (not reduced) and
// leaves grad_x in o[] (stored by lsq_store_block once the block has arrived).
template <bool VEC, bool NT, bool ZPL, int ACT, int G, class QF = QP>
__device__ __forceinline__ QP lsq_bwd_block(const float *__restrict__ g, const float *__restrict__ x,
                                            int64_t n, const QF &qf, int64_t blk, LsqAcc &c, f4 (&o)[G],
                                            const SiluLay &L = SiluLay{}) {
  const int64_t ng = cdiv(n, 4);
  const int64_t base = blk * kBlock * G + threadIdx.x;
  f4 xv[G], gv[G];
#pragma unroll
  for (int k = 0; k < kLsqPrefetch && k < G; ++k) {
    xv[k] = load_group_c<VEC, NT>(x, base + k * kBlock, ng, n);
    gv[k] = load_group_c<VEC, NT>(g, base + k * kBlock, ng, n);
  }
  const QP &p = qp_of(qf);
#pragma unroll
  for (int k = 0; k < G; ++k) {
    if (k + kLsqPrefetch < G) {
      xv[k + kLsqPrefetch] = load_group_c<VEC, NT>(x, base + (k + kLsqPrefetch) * kBlock, ng, n);
      gv[k + kLsqPrefetch] = load_group_c<VEC, NT>(g, base + (k + kLsqPrefetch) * kBlock, ng, n);
    }
    o[k] = lsq_group_out<ZPL, ACT>(base + k * kBlock, ng, n, xv[k], gv[k], p, c, L);
  }
  return p;
}

template <bool VEC, bool NT, int G>
__device__ __forceinline__ void lsq_store_block(float *__restrict__ gx, int64_t n, int64_t blk, const f4 (&o)[G]) {
  const int64_t ng = cdiv(n, 4);
  const int64_t base = blk * kBlock * G + threadIdx.x;
#pragma unroll
  for (int k = 0; k < G; ++k)
    if (base + k * kBlock < ng) store_group<VEC, NT>(gx, base + k * kBlock, n, o[k]);
}

// Block sum of the K4 terms with the waves split (wave_arrive): DPP wave sums -> LDS;
// waves 1..3 store their grad_x and return false; wave 0 passes an LDS-only barrier
// and gets the block record {sum t, sum z} (fixed order) in every lane.  STORE false:
// the caller stored every wave's grad_x already (records-only K4d).
template <bool VEC, bool NT, int G, bool STORE = true>
__device__ __forceinline__ bool lsq_block_record(LsqAcc c, float *__restrict__ gx, int64_t n, int64_t blk,
                                                 const f4 (&o)[G], double (&rec)[2]) {
  __shared__ double s[kWaves][2];
  c.t = wave_reduce(c.t, AddD());
  c.z = wave_reduce(c.z, AddD());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) { s[w][0] = c.t; s[w][1] = c.z; }
  if (STORE && w != 0) lsq_store_block<VEC, NT, G>(gx, n, blk, o);
  lds_barrier();
  if (w != 0) return false;
  rec[0] = s[0][0]; rec[1] = s[0][1];
#pragma unroll
  for (int i = 1; i < kWaves; ++i) { rec[0] += s[i][0]; rec[1] += s[i][1]; }
  return true;
}

// gradient of the zero point after the fold: ClampBackward of zero_point_rounding
// (uniform.py:101) -- the in-range test on round(zp); NaN -> not in range
__device__ __forceinline__ double lsq_grad_zp(double zsum, const QPSrc &src, const QP &p, double gscale) {
  // zp_learn 2 (a symmetric quantizer given a gradient-requiring zero point,
  // uniform.py:47-56 with `not self.symmetric` False): zp enters x/s + zp and (x_int - zp)
  // as given -- no rounding, no clamp, no ScaleGradient
  if (!src.zround) return zsum;
  const double zr = __builtin_rint(src.zdev ? *src.zdev : src.zhost);
  const bool zin = zr >= (double)p.lo && zr <= (double)p.hi;
  return zin ? zsum * gscale : 0.0;
}

}  // namespace vsiq
