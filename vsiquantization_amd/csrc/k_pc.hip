// k_pc.hip — K3 dispatch + per-channel fake-quant with given qparams, and their C ABI.
#include "k_pc.cuh"

namespace vsiq {

extern template bool launch_pc_bs<true, true, true, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, true, false, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, false, true, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, false, false, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<false, false, true, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<false, false, false, 256>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, true, true, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, true, false, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, false, true, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, false, false, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<false, false, true, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<false, false, false, 512>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, true, true, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, true, false, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, false, true, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<true, false, false, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<false, false, true, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);
extern template bool launch_pc_bs<false, false, false, 1024>(const float *, float *, uint8_t *, uint64_t *, const PCArgs &, hipStream_t);

template <bool VEC, bool NT, bool STATS>
int launch_pc(const float *x, float *y, uint8_t *c, uint64_t *m, const PCArgs &a, hipStream_t st) {
  const int64_t ng = cdiv(a.rowlen, 4);
  // workgroup size: the smallest that holds the row in <= 9 groups per lane
  // (measured on MI355X at 1024 x 9216: 256 lanes x 9 groups 13.0 us, 512 x 5 15.9,
  //  1024 x 3 17.4 -- more rows in flight per CU beats fewer groups per lane)
  const int bs = ng <= 9 * 256 ? 256 : (ng <= 9 * 512 ? 512 : 1024);
  PCArgs b = a;
  b.defer = bs == 256 ? store_defer_units(a.rows, false) : 0;
  b.gate = kGateAuto;   // resolved per instantiation (launch_pc_k)
  bool ok = false;
  if (bs == 1024) ok = launch_pc_bs<VEC, NT, STATS, 1024>(x, y, c, m, b, st);
  else if (bs == 512) ok = launch_pc_bs<VEC, NT, STATS, 512>(x, y, c, m, b, st);
  else ok = launch_pc_bs<VEC, NT, STATS, 256>(x, y, c, m, b, st);
  if (!ok)
    hipLaunchKernelGGL((k_pc_observe_fq_long<VEC, NT>), dim3((unsigned)a.rows), dim3(kBlock), 0, st, x,
                       y, c, m, a);
  return launch_rc();
}


// ----------------------------------------------------------------------------
// per-channel fake-quant with given per-row qparams: grid (rows, chunks)
// ----------------------------------------------------------------------------
// row r uses qparams [r % channels]: channels == rows for axis 0 of a [C, ...]
// tensor; channels == C for axis 1 of an [N, C, ...] tensor viewed as [N*C, HW...]
struct PCFixed {
  int64_t rowlen;
  const double *scale, *zp;   // zp nullable: 0
  int zp_round;
  float lo, hi;
  int64_t channels;
};

// UNI: `row` is wave-uniform (scalar qparam loads, ld_uniform_f64); rows < 2^31 (host check)
template <bool UNI = false>
__device__ __forceinline__ QP pc_fixed_qp(const PCFixed &a, int64_t row) {
  const int64_t c = (uint32_t)row % (uint32_t)a.channels;
  QPSrc s{nullptr, a.scale + c, a.zp ? a.zp + c : nullptr, 0.0, 0.0, a.lo, a.hi, a.zp_round, 0};
  return load_qp<UNI>(s);
}

// U groups per lane: kFlatU, or 9 for a one-round grid behind the store gate
// (gate 0 = none; gc = gate_begin at the workgroup start)
template <bool VEC, bool NT, bool CODES, bool MASK, int U>
__global__ __launch_bounds__(kBlock) void k_pc_fq_fwd(const float *__restrict__ x, float *__restrict__ y,
                                                      uint8_t *__restrict__ codes,
                                                      uint64_t *__restrict__ mask, uint32_t chunks,
                                                      PCFixed a, uint32_t gate) {
  const GateClk gc = gate_begin(gate);
  const int64_t row = blockIdx.x / chunks;
  const int64_t chunk = blockIdx.x % chunks;
  const int64_t ng = cdiv(a.rowlen, 4);
  const float *xr = x + row * a.rowlen;
  float *yr = y + row * a.rowlen;
  const int64_t base = chunk * kBlock * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = load_group_c<VEC, NT>(xr, base + u * kBlock, ng, a.rowlen);
  const QP p = pc_fixed_qp<true>(a, row);   // after the x loads are issued, on lgkmcnt
  GroupOut go[U];
  uint32_t mlo = 0, mhi = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    go[u] = fq_out_flat<VEC, CODES, MASK>(v[u], p, base + u * kBlock, a.rowlen);
    if (MASK) mask_put(mlo, mhi, u, go[u].b);
  }
  gate_pass(gate, gc);
  uint8_t *cr = CODES ? codes + row * a.rowlen : nullptr;
  const int lane = threadIdx.x % kWave;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kBlock;
    if (i - lane >= ng) break;
    fq_store_out<VEC, NT, CODES>(yr, cr, i, ng, a.rowlen, go[u]);
  }
  if (MASK && lane < 4 * U) {
    const int64_t first = base - lane + (lane >> 2) * kBlock;
    if (first < ng)
      mask[row * mask_words_per_row(a.rowlen) + 4 * (first / kWave) + (lane & 3)] =
          ((uint64_t)mhi << 32) | mlo;
  }
}

// one-round grids of 9 groups per lane behind the store gate where that applies (as K1,
// k_fq.hip), else (rows, kFlatU chunks)
template <bool VEC, bool NT, bool CODES, bool MASK>
void launch_pc_fixed_k(const float *x, float *y, uint8_t *c, uint64_t *m, const PCFixed &a, int64_t rows,
                       hipStream_t st) {
  const int64_t ng = cdiv(a.rowlen, 4);
  const int64_t chunks9 = cdiv(ng, (int64_t)kBlock * 9);
  GateSel gs;
  if (g_tune.store_gate != 0 && chunks9 * kBlock * 9 - ng <= ng / 8) {
    const void *kern = reinterpret_cast<const void *>(k_pc_fq_fwd<VEC, NT, CODES, MASK, 9>);
    static const int occ = occupancy_blocks(kern, kBlock);
    gs = store_gate_select("pc_fq_fwd", kern, rows * chunks9, occ, 4 * rows * a.rowlen, st);
  }
  if (gs.gate) {
    hipLaunchKernelGGL((k_pc_fq_fwd<VEC, NT, CODES, MASK, 9>), dim3((unsigned)(rows * chunks9)), dim3(kBlock),
                       0, st, x, y, c, m, (uint32_t)chunks9, a, gs.gate);
  } else {
    const int64_t chunks = oneshot_grid(ng);
    hipLaunchKernelGGL((k_pc_fq_fwd<VEC, NT, CODES, MASK, kFlatU>), dim3((unsigned)(rows * chunks)),
                       dim3(kBlock), 0, st, x, y, c, m, (uint32_t)chunks, a, 0u);
  }
  store_gate_launched(gs, st);   // a tuning sample of "no gate" times the kFlatU grid
}

template <bool VEC, bool NT>
void launch_pc_fixed(const float *x, float *y, uint8_t *c, uint64_t *m, const PCFixed &a, int64_t rows,
                     hipStream_t st) {
  if (c && m) launch_pc_fixed_k<VEC, NT, true, true>(x, y, c, m, a, rows, st);
  else if (c) launch_pc_fixed_k<VEC, NT, true, false>(x, y, c, m, a, rows, st);
  else if (m) launch_pc_fixed_k<VEC, NT, false, true>(x, y, c, m, a, rows, st);
  else launch_pc_fixed_k<VEC, NT, false, false>(x, y, c, m, a, rows, st);
}

// ----------------------------------------------------------------------------
// Packed short rows (rowlen % 4 == 0, rowlen <= kPackMaxRowlen): one workgroup takes
// R = kPackElems / rowlen WHOLE rows (up to 256), i.e. a contiguous flat range of
// groups, 4 per lane.  The one-workgroup-per-row grid above leaves most lanes idle
// on LSQFakeQuantize's axis-1 activations (rows of H*W = 100..1600 elements: 686 GB/s
// at 256x256x10x10 on MI355X).  Per-row qparams are built once per workgroup into
// LDS; each group reads its row's.  No mask output (its word layout assumes one row
// per wave): a mask request takes the per-row kernel.
// ----------------------------------------------------------------------------
template <bool VEC, bool NT, bool CODES>
__global__ __launch_bounds__(kBlock) void k_pcp_fq_fwd(const float *__restrict__ x, float *__restrict__ y,
                                                       uint8_t *__restrict__ codes, int64_t rows,
                                                       uint32_t rpb, PCFixed a) {
  __shared__ QP s_qp[kPackMaxRows];
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const uint32_t nr = (uint32_t)std::min<int64_t>(rpb, rows - r0);
  const uint32_t gpr = (uint32_t)(a.rowlen / 4);
  const int64_t n = rows * a.rowlen, ng = rows * gpr;
  const int64_t j0 = r0 * gpr;
  const uint32_t nj = nr * gpr;
  f4 v[kPackGroups];
#pragma unroll
  for (int k = 0; k < kPackGroups; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    v[k] = load_group_c<VEC, NT>(x, j0 + (j < nj ? j : nj - 1), ng, n);
  }
  if (threadIdx.x < nr) s_qp[threadIdx.x] = pc_fixed_qp(a, r0 + threadIdx.x);
  lds_barrier();   // the loads stay in flight
  GroupOut go[kPackGroups];
#pragma unroll
  for (int k = 0; k < kPackGroups; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    const QP p = s_qp[(j < nj ? j : nj - 1) / gpr];
    go[k] = fq_out_flat<VEC, CODES, false>(v[k], p, j0 + j, n);
  }
#pragma unroll
  for (int k = 0; k < kPackGroups; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    if (j < nj) fq_store_out<VEC, NT, CODES>(y, codes, j0 + j, ng, n, go[k]);
  }
}

template <bool VEC, bool NT>
void launch_pcp_fixed(const float *x, float *y, uint8_t *c, const PCFixed &a, int64_t rows, hipStream_t st) {
  const int64_t rpb = pc_pack_rows(a.rowlen);
  const dim3 grid((unsigned)cdiv(rows, rpb)), block(kBlock);
  if (c) hipLaunchKernelGGL((k_pcp_fq_fwd<VEC, NT, true>), grid, block, 0, st, x, y, c, rows, (uint32_t)rpb, a);
  else hipLaunchKernelGGL((k_pcp_fq_fwd<VEC, NT, false>), grid, block, 0, st, x, y, c, rows, (uint32_t)rpb, a);
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

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
           (float)qmax, qden, eps, 0u};
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

int vsiq_pcm_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t rows,
                        int64_t rowlen, int64_t channels, const double *scale, const double *zp,
                        int zp_round, int qmin, int qmax, void *stream) {
  if (rows < 0 || rowlen <= 0 || qmin > qmax || channels <= 0) return VSIQ_E_ARG;
  if (rows == 0) return 0;
  if (!x || !y || !scale || rows % channels || rows * oneshot_grid(cdiv(rowlen, 4)) > 0x7fffffffLL)
    return VSIQ_E_ARG;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  PCFixed a{rowlen, scale, zp, zp_round, (float)qmin, (float)qmax, channels};
  const bool vec = (rowlen % 4 == 0) && aligned16(x) && aligned16(y) && (!codes || aligned4(codes));
  const bool nt = g_tune.nontemporal != 0;
  uint8_t *c = (uint8_t *)codes;
  if (!mask && pc_packed_fwd(rowlen) && g_tune.pc_packed != 0)
    VSIQ_B2(launch_pcp_fixed, vec, nt, x, y, c, a, rows, (hipStream_t)stream);
  else
    VSIQ_B2(launch_pc_fixed, vec, nt, x, y, c, mask, a, rows, (hipStream_t)stream);
  return launch_rc();
}

int vsiq_pc_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t rows,
                       int64_t rowlen, const double *scale, const double *zp, int zp_round,
                       int qmin, int qmax, void *stream) {
  if (rows > 0 && !zp) return VSIQ_E_ARG;
  return vsiq_pcm_fq_fwd_f32(x, y, codes, mask, rows, rowlen, rows > 0 ? rows : 1, scale, zp, zp_round,
                             qmin, qmax, stream);
}

}  // extern "C"
