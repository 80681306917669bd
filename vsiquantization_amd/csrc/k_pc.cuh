// k_pc.cuh — K3 per-channel observe + qparams + fake-quant (templates; the
// register-resident instantiations are compiled in k_pc_bs{256,512,1024}.hip).
#pragma once
#include "vsiq_common.cuh"

namespace vsiq {

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
  uint32_t defer;      // deferred store phase (defer_stores units), 0 = off
  uint32_t gate;       // store gate: no stores before workgroup start + gate ticks (10 ns), 0 = off
};

struct RowSums {
  double sa, s1, s2;
};

__device__ __forceinline__ void rowsums_add4(RowSums &r, f4 v, int nv) {
  const float vy = nv > 1 ? v.y : 0.f, vz = nv > 2 ? v.z : 0.f, vw = nv > 3 ? v.w : 0.f;
  const float pa = (__builtin_fabsf(v.x) + __builtin_fabsf(vy)) +
                   (__builtin_fabsf(vz) + __builtin_fabsf(vw));
  const float p1 = (v.x + vy) + (vz + vw);
  const float p2 = (v.x * v.x + vy * vy) + (vz * vz + vw * vw);   // fp32 over 4, f64 across groups
  r.sa += (double)pa;
  r.s1 += (double)p1;
  r.s2 += (double)p2;
}

// Row reduction -> running state -> f64 qparams, returned to every lane (one barrier:
// a workgroup reduces one row).
template <bool STATS, int BS = kBlock>
__device__ __forceinline__ QP pc_row_qparams(float mn, float mx, uint32_t nan, RowSums rs,
                                             float rmn, float rmx, int64_t row, const PCArgs &a) {
  constexpr int NW = BS / kWave;
  __shared__ float s_mn[NW], s_mx[NW];
  __shared__ uint32_t s_nan[NW];
  __shared__ double s_rs[3][NW];
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
    s_mn[w] = mn; s_mx[w] = mx; s_nan[w] = nan;
    if (STATS) { s_rs[0][w] = rs.sa; s_rs[1][w] = rs.s1; s_rs[2][w] = rs.s2; }
  }
  __syncthreads();
  mn = s_mn[0]; mx = s_mx[0]; nan = s_nan[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) {
    mn = fminf(mn, s_mn[i]); mx = fmaxf(mx, s_mx[i]); nan |= s_nan[i];
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
      double sa = s_rs[0][0], s1 = s_rs[1][0], s2 = s_rs[2][0];
      for (int i = 1; i < NW; ++i) { sa += s_rs[0][i]; s1 += s_rs[1][i]; s2 += s_rs[2][i]; }
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
  p.fast = (fq_fast_qp(p.s, p.z) && !nan &&
            __builtin_fmaxf(__builtin_fabsf(mn), __builtin_fabsf(mx)) <= 0x1p62f) ? 1u : 0u;
  return p;
}

template <int NV, bool VEC, bool NT, int BS>
__device__ __forceinline__ void pc_load_row(f4 (&v)[NV], const float *x, int64_t row, const PCArgs &a) {
  const float *xr = x + row * a.rowlen;
  const int64_t ng = cdiv(a.rowlen, 4);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * BS;
    v[k] = load_group_c<VEC, NT>(xr, i, ng, a.rowlen);
  }
}

template <int NV, bool VEC, bool NT, bool STATS, bool MASK, bool CODES, int BS>
__device__ __forceinline__ void pc_process_row(const f4 (&v)[NV], float rmn, float rmx,
                                               int64_t row, float *__restrict__ y,
                                               uint8_t *__restrict__ codes,
                                               uint64_t *__restrict__ mask, const PCArgs &a,
                                               GateClk gc = GateClk{0}) {
  const int64_t ng = cdiv(a.rowlen, 4);
  float mn = __builtin_inff(), mx = -__builtin_inff();
  uint32_t nan = 0;
  RowSums rs{0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * BS;
    if (i < ng) {
      const f4 w = v[k];   // invalid tail lanes already replicate element 0
      mn = fminf(mn, fminf(fminf(w.x, w.y), fminf(w.z, w.w)));
      mx = fmaxf(mx, fmaxf(fmaxf(w.x, w.y), fmaxf(w.z, w.w)));
      nan |= (w.x != w.x) | (w.y != w.y) | (w.z != w.z) | (w.w != w.w);
      if (STATS) rowsums_add4(rs, w, VEC ? 4 : valid_in_group(i, a.rowlen));
    }
  }
  const QP p = pc_row_qparams<STATS, BS>(mn, mx, nan, rs, rmn, rmx, row, a);
  if (!y) return;
  float *yr = y + row * a.rowlen;
  uint8_t *cr = CODES ? codes + row * a.rowlen : nullptr;
  GroupOut go[NV];
  uint32_t mlo = 0, mhi = 0;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    go[k] = fq_out_row<VEC, CODES, MASK>(v[k], p, threadIdx.x + k * BS, a.rowlen);
    if (MASK) mask_put(mlo, mhi, k, go[k].b);
  }
  if (a.defer) defer_stores(a.defer);   // after pc_row_qparams' barrier
  gate_pass(a.gate, gc);
  const int lane = threadIdx.x % kWave;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * BS;
    if (i - lane >= ng) continue;   // whole wave past the row end (uniform)
    fq_store_out<VEC, NT, CODES>(yr, cr, i, ng, a.rowlen, go[k]);
  }
  if (MASK && lane < 4 * NV) {   // lane 4k+j: word j of group slot k's chunk
    const int64_t first = threadIdx.x - lane + (lane >> 2) * BS;
    if (first < ng)
      mask[row * mask_words_per_row(a.rowlen) + 4 * (first / kWave) + (lane & 3)] =
          ((uint64_t)mhi << 32) | mlo;
  }
}

// One row per workgroup, straight-line code: the row's loads are all issued up front and
// hipcc's s_waitcnt counts stay exact (no loop).  RPB (rows per workgroup) is 1: the
// two-row form measured no faster (its parameter stays in the kernel's name, which the
// profiles and tools/pmc_to_traffic.py match).
template <int NV, bool VEC, bool NT, bool STATS, bool MASK, bool CODES, int BS, int RPB>
__global__ __launch_bounds__(BS) void k_pc_observe_fq(const float *__restrict__ x,
                                                      float *__restrict__ y,
                                                      uint8_t *__restrict__ codes,
                                                      uint64_t *__restrict__ mask, PCArgs a) {
  static_assert(RPB == 1, "rows per block");
  const GateClk gc = gate_begin(a.gate);
  const int64_t row = blockIdx.x;
  f4 v[NV];
  pc_load_row<NV, VEC, NT, BS>(v, x, row, a);
  const float rmn = a.run_min[row], rmx = a.run_max[row];
  pc_process_row<NV, VEC, NT, STATS, MASK, CODES, BS>(v, rmn, rmx, row, y, codes, mask, a, gc);
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
                   ? pc_row_qparams<true>(mn, mx, nan, rs, a.run_min[row], a.run_max[row], row, a)
                   : pc_row_qparams<false>(mn, mx, nan, rs, a.run_min[row], a.run_max[row], row, a);
  if (!y) return;
  float *yr = y + row * a.rowlen;
  uint64_t *mr = mask ? mask + row * mask_words_per_row(a.rowlen) : nullptr;
  for (int64_t base = 0; base < ng; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const bool in = i < ng;
    Elem e0, e1, e2, e3;
    fq_group_row(load_group_c<VEC, NT>(xr, i, ng, a.rowlen), p, e0, e1, e2, e3);
    if (in) {
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


template <int NV, bool VEC, bool NT, bool STATS, bool MASK, bool CODES, int BS>
void launch_pc_k(const float *x, float *y, uint8_t *c, uint64_t *m, const PCArgs &a, hipStream_t st) {
  const auto kern = k_pc_observe_fq<NV, VEC, NT, STATS, MASK, CODES, BS, 1>;
  PCArgs b = a;
  GateSel gs;
  if (a.gate == kGateAuto) {
    // one-round grids of >= 2 rows per CU: stores wait for the grid's read phase
    static const int occ = occupancy_blocks(reinterpret_cast<const void *>(kern), BS);
    gs = store_gate_select("k3_pc_observe_fq", reinterpret_cast<const void *>(kern), a.rows, occ,
                           a.rows * a.rowlen * (int64_t)sizeof(float), st);
    b.gate = gs.gate;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)a.rows), dim3(BS), 0, st, x, y, c, m, b);
  store_gate_launched(gs, st);
}

template <int NV, bool VEC, bool NT, bool STATS, int BS>
void launch_pc_nv(const float *x, float *y, uint8_t *c, uint64_t *m, const PCArgs &a, hipStream_t st) {
  if (c && m) launch_pc_k<NV, VEC, NT, STATS, true, true, BS>(x, y, c, m, a, st);
  else if (c) launch_pc_k<NV, VEC, NT, STATS, false, true, BS>(x, y, c, m, a, st);
  else if (m) launch_pc_k<NV, VEC, NT, STATS, true, false, BS>(x, y, c, m, a, st);
  else launch_pc_k<NV, VEC, NT, STATS, false, false, BS>(x, y, c, m, a, st);
}

// groups per lane -> register-resident instantiation; false if the row is too long
template <bool VEC, bool NT, bool STATS, int BS>
bool launch_pc_bs(const float *x, float *y, uint8_t *c, uint64_t *m, const PCArgs &a, hipStream_t st) {
  const int64_t per_lane = cdiv(cdiv(a.rowlen, 4), BS);
  if (per_lane <= 1) launch_pc_nv<1, VEC, NT, STATS, BS>(x, y, c, m, a, st);
  else if (per_lane <= 2) launch_pc_nv<2, VEC, NT, STATS, BS>(x, y, c, m, a, st);
  else if (per_lane <= 3) launch_pc_nv<3, VEC, NT, STATS, BS>(x, y, c, m, a, st);
  else if (per_lane <= 5) launch_pc_nv<5, VEC, NT, STATS, BS>(x, y, c, m, a, st);
  else if (per_lane <= 9) launch_pc_nv<9, VEC, NT, STATS, BS>(x, y, c, m, a, st);
  else if (per_lane <= 12) launch_pc_nv<12, VEC, NT, STATS, BS>(x, y, c, m, a, st);
  else return false;
  return true;
}

}  // namespace vsiq
