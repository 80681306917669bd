// k_lsq.hip — K4 learnable (LSQ) backward: grad_x + f64 scale / zero-point gradient
// sums (optionally through a fused ReLU/SiLU, K5), and its C ABI entry points.
#include "k_body.cuh"

namespace vsiq {

// PART: the block record {sum t, sum z} goes to ws[2 * block] with a plain store and
// the block leaves -- no drain, no arrival, no fold (vsiq_act_lsq_bwd_part_f32: the
// fold of every layer's records runs later in one launch, k_lsq_fold_multi).  `gate`:
// the one-round PART grids' store gate (round 5, launch_lsq_g; 0 = none).
template <bool VEC, bool NT, bool ZPL, int ACT, int G, bool PART = false>
__global__ __launch_bounds__(kBlock) void k_lsq_bwd(const float *__restrict__ g,
                                                    const float *__restrict__ x,
                                                    float *__restrict__ gx, int64_t n,
                                                    QPSrc src, double gscale, SiluLay L,
                                                    double *__restrict__ grad_out,
                                                    double *__restrict__ ws,
                                                    uint32_t *__restrict__ counter, uint32_t gate) {
  const GateClk gc = gate_begin(gate);
  LsqAcc c{0.0, 0.0};
  f4 o[G];
  // G <= 2 (C4's small one-round layers): the kernel-uniform qparams as scalar loads after
  // the first x / g loads are issued (round 6).  Deeper grids keep them first: the late
  // loads cost 2 VGPRs there, one wave per SIMD at G = 4 / 8 (C3's K4: 98 VGPRs, 4 waves),
  // and measured equal at C3 (profiles/r06/r06x_k4_late_qparams.txt).
  QP p;
  if constexpr (G <= 2) {
    p = lsq_bwd_block<VEC, NT, ZPL, ACT, G>(g, x, n, [&] { return load_qp<true>(src); }, blockIdx.x, c, o, L);
  } else {
    p = load_qp(src);
    (void)lsq_bwd_block<VEC, NT, ZPL, ACT, G>(g, x, n, p, blockIdx.x, c, o, L);
  }
  if (PART) {
    // no arrival to order against: every wave issues its grad_x stores first, so the
    // block reduction runs while they drain (the one-round grids of small layers end
    // with it otherwise on the critical path)
    gate_pass(gate, gc);
    lsq_store_block<VEC, NT, G>(gx, n, blockIdx.x, o);
    double rec[2];
    if (!lsq_block_record<VEC, NT, G, false>(c, gx, n, blockIdx.x, o, rec)) return;
    if (threadIdx.x == 0) {
      ws[2 * (int64_t)blockIdx.x] = rec[0];
      ws[2 * (int64_t)blockIdx.x + 1] = rec[1];
    }
    return;
  }
  double rec[2], f[2];
  if (!lsq_block_record<VEC, NT, G>(c, gx, n, blockIdx.x, o, rec)) return;   // waves 1..3 done
  const bool last = wave_arrive<LsqFold>(ws, 0, gridDim.x, blockIdx.x, counter, rec, f, [&]() {
    lsq_store_block<VEC, NT, G>(gx, n, blockIdx.x, o);   // wave 0's grad_x, after its arrival
  });
  if (!last) return;
  if (threadIdx.x == 0) {
    grad_out[0] = f[0] * gscale;
    grad_out[1] = ZPL ? lsq_grad_zp(f[1], src, p, gscale) : 0.0;
    *counter = 0u;
  }
}


template <int ACT, bool VEC, bool NT, int G>
void launch_lsq_g(const float *g, const float *x, float *gx, int64_t n, const QPSrc &src, int zpl,
                  double gscale, double *grad_out, double *ws, uint32_t *counter, int64_t grid,
                  const SiluLay &L, hipStream_t st) {
  if (!counter) {   // records only (PART)
    // a one-round grid (store_gate_select takes grids of 2..occ workgroups per CU only):
    // the tuned store gate between the read and the write phase
    GateSel gs;
    {
      const void *kern = zpl ? reinterpret_cast<const void *>(k_lsq_bwd<VEC, NT, true, ACT, G, true>)
                             : reinterpret_cast<const void *>(k_lsq_bwd<VEC, NT, false, ACT, G, true>);
      static const int occ_t = occupancy_blocks(reinterpret_cast<const void *>(k_lsq_bwd<VEC, NT, true, ACT, G, true>),
                                                kBlock);
      static const int occ_f = occupancy_blocks(
          reinterpret_cast<const void *>(k_lsq_bwd<VEC, NT, false, ACT, G, true>), kBlock);
      gs = store_gate_select("k4d_lsq_bwd_part", kern, grid, zpl ? occ_t : occ_f, 8 * n, st);
    }
    if (zpl)
      hipLaunchKernelGGL((k_lsq_bwd<VEC, NT, true, ACT, G, true>), dim3((unsigned)grid), dim3(kBlock), 0, st, g,
                         x, gx, n, src, gscale, L, grad_out, ws, counter, gs.gate);
    else
      hipLaunchKernelGGL((k_lsq_bwd<VEC, NT, false, ACT, G, true>), dim3((unsigned)grid), dim3(kBlock), 0, st, g,
                         x, gx, n, src, gscale, L, grad_out, ws, counter, gs.gate);
    store_gate_launched(gs, st);
    return;
  }
  if (zpl)
    hipLaunchKernelGGL((k_lsq_bwd<VEC, NT, true, ACT, G>), dim3((unsigned)grid), dim3(kBlock), 0, st, g, x,
                       gx, n, src, gscale, L, grad_out, ws, counter, 0u);
  else
    hipLaunchKernelGGL((k_lsq_bwd<VEC, NT, false, ACT, G>), dim3((unsigned)grid), dim3(kBlock), 0, st, g, x,
                       gx, n, src, gscale, L, grad_out, ws, counter, 0u);
}

// Records-only K4 (K4d): groups per lane 2.  Without an arrival chain more, smaller
// workgroups cost nothing and stream better at every C4 size (MI355X kernel trace, 3.3M
// -> 105M elements: 9.9 / 16.2 / 28.0 / 51.7 / 101.0 / 205.3 us at 2 per lane against
// 11.1 / 16.6 / 28.4 / 54.2 / 103.2 / 207.9 us at K4's 4 / 8, profiles/r03g_c4_groups.txt);
// the 4x larger record count is folded by the two-stage k_lsq_fold_chunks.
// (1 group per lane for the small layers measured slower still: 10.4 against 9.8 us at
// 3.3M elements, 214 against 201 us at 105M, profiles/r04h_c4_k4d.txt.)
// Round 5 (per-dispatch kernel trace of the C4 leg at 2 / 4 / 8 / 16 groups per lane,
// every one-round grid gated -- launch_lsq_g --, profiles/r05/r05p_k4d_groups.txt): 2 per
// lane is best or level up to 26M elements (3.3M 8.7 us gated against 9.6-10.6 for 4-16;
// 6.6M / 13M / 26M within 1 % of 4 per lane; the one-round 8 / 16 grids of 13M / 26M are
// slower even gated), 4 per lane from ~50M (52M 98.5 against 100.0 us, 105M 195.9
// against 204.8).
inline int lsq_part_groups_per_lane(int64_t n) {
  const int g = g_tune.lsq_groups;
  return g > 0 ? g : (n >= ((int64_t)48 << 20) ? 4 : 2);
}

template <int ACT, bool VEC, bool NT>
void launch_lsq_act(const float *g, const float *x, float *gx, int64_t n, const QPSrc &src, int zpl,
                    double gscale, double *grad_out, double *ws, uint32_t *counter, int64_t grid,
                    const SiluLay &L, hipStream_t st) {
  const int per_lane = counter ? lsq_groups_per_lane(cdiv(n, 4)) : lsq_part_groups_per_lane(n);
  if (per_lane == kLsqGroups)
    launch_lsq_g<ACT, VEC, NT, kLsqGroups>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
  else if (per_lane == 8)
    launch_lsq_g<ACT, VEC, NT, 8>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
  else if (per_lane == 4)
    launch_lsq_g<ACT, VEC, NT, 4>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
  else
    launch_lsq_g<ACT, VEC, NT, 2>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
}

template <int ACT>
void launch_lsq(bool vec, bool nt, const float *g, const float *x, float *gx, int64_t n,
                const QPSrc &src, int zpl, double gscale, double *grad_out, double *ws,
                uint32_t *counter, int64_t grid, const SiluLay &L, hipStream_t st) {
  if (vec && nt) launch_lsq_act<ACT, true, true>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
  else if (vec) launch_lsq_act<ACT, true, false>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
  else if (nt) launch_lsq_act<ACT, false, true>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
  else launch_lsq_act<ACT, false, false>(g, x, gx, n, src, zpl, gscale, grad_out, ws, counter, grid, L, st);
}

int lsq_bwd(const float *g, const float *x, float *gx, int64_t n, int act, const double *scale_dev,
            double scale_host, const double *zp_dev, double zp_host, int zp_learn, int qmin, int qmax,
            double gscale, double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
            void *stream) {
  if (n <= 0 || !g || !x || !gx || !grad_out || !ws || !counter || qmin > qmax || !act_ok(act))
    return VSIQ_E_ARG;
  const bool vec = (n % 4 == 0) && aligned16(g) && aligned16(x) && aligned16(gx);
  const int64_t grid = lsq_grid(cdiv(n, 4));
  if (grid > 0x7fffffffLL) return VSIQ_E_ARG;
  if (ws_len < fold_records(grid) * kPartials) return VSIQ_E_WS;
  // learnable zp (1): the forward used clamp(rint(zp)); 0 / 2: zp as given (2: with its gradient)
  if (zp_learn < 0 || zp_learn > 2) return VSIQ_E_ARG;
  QPSrc src{nullptr, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax, zp_learn == 1, 0};
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_ACT(act, launch_lsq, vec, nt, g, x, gx, n, src, zp_learn != 0, gscale, grad_out, ws, counter, grid,
           act_lay(act, n), (hipStream_t)stream);
  return launch_rc();
}

// Records-only K4 (PART): same grid, per-element code and block records as lsq_bwd.
int lsq_bwd_part(const float *g, const float *x, float *gx, int64_t n, int act, const double *scale_dev,
                 double scale_host, const double *zp_dev, double zp_host, int zp_learn, int qmin, int qmax,
                 double *records, int64_t records_len, void *stream) {
  if (n <= 0 || !g || !x || !gx || !records || qmin > qmax || !act_ok(act))
    return VSIQ_E_ARG;
  const bool vec = (n % 4 == 0) && aligned16(g) && aligned16(x) && aligned16(gx);
  const int64_t grid = lsq_grid(cdiv(n, 4), lsq_part_groups_per_lane(n));
  if (grid > 0x7fffffffLL) return VSIQ_E_ARG;
  if (records_len < 2 * grid) return VSIQ_E_WS;
  if (zp_learn < 0 || zp_learn > 1) return VSIQ_E_ARG;   // the deferred fold knows modes 0 / 1 only
  QPSrc src{nullptr, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax, zp_learn, 0};
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_ACT(act, launch_lsq, vec, nt, g, x, gx, n, src, zp_learn, 0.0, nullptr, records, nullptr, grid,
           act_lay(act, n), (hipStream_t)stream);
  return launch_rc();
}

// ----------------------------------------------------------------------------
// Fold of records-only K4 calls, two launches (quantizers/uniform.py:47-56 + ScaleGradient
// :242-255, zero_point_rounding :98-102):
//   k_lsq_fold_chunks  one workgroup per chunk of kFoldChunk records of a call: every
//                      thread issues its 4 record loads at once, adds them in order, the
//                      fixed block tree sums the workgroup; the chunk's {sum t, sum z}
//                      replaces the chunk's first record (the records are scratch);
//   k_lsq_fold_multi   workgroup t folds call t's chunk sums in chunk order -> grad_out[t]
//                      = {sum t * gscale, ClampBackward of round(zp) ? sum z * gscale : 0}.
// Deterministic (fixed chunks, fixed trees).  Round 2's single launch walked a call's
// records with one dependent load round trip per 256 records (14.6 us at C4, 54.6 us
// with the 4x record count of 2 groups per lane, profiles/r03g_c4_groups.txt).
// ----------------------------------------------------------------------------
constexpr int kFoldMulti = 64;    // calls per launch pair (descriptor table in the kernel arguments)
constexpr int kFoldPer = 4;       // records per thread of a chunk workgroup
constexpr int64_t kFoldChunk = (int64_t)kBlock * kFoldPer;

struct FCall {
  double *rec;
  const double *zdev;
  double *out;
  int64_t nrec;
  double zhost, gscale;
  float lo, hi;
  int zpl;
};

struct FBatch {
  FCall t[kFoldMulti];
  uint32_t c0[kFoldMulti + 1];   // first chunk workgroup of each call
  int count;
};

__global__ __launch_bounds__(kBlock) void k_lsq_fold_chunks(const FBatch b) {
  int t = 0;
  const uint32_t blk = blockIdx.x;
  while (t + 1 < b.count && blk >= b.c0[t + 1]) ++t;   // scalar: c0 is a kernel argument
  const FCall &T = b.t[t];
  const int64_t r0 = (int64_t)(blk - b.c0[t]) * kFoldChunk;
  double2 v[kFoldPer];
#pragma unroll
  for (int k = 0; k < kFoldPer; ++k) {
    const int64_t i = r0 + threadIdx.x + (int64_t)k * kBlock;
    v[k] = i < T.nrec ? *reinterpret_cast<const double2 *>(T.rec + 2 * i) : double2{0.0, 0.0};
  }
  LsqAcc acc{0.0, 0.0};
#pragma unroll
  for (int k = 0; k < kFoldPer; ++k) {
    if (r0 + threadIdx.x + (int64_t)k * kBlock < T.nrec) {
      acc.t += v[k].x;
      acc.z += v[k].y;
    }
  }
  lsq_block_reduce(acc);   // every thread's loads were consumed before its first barrier
  if (threadIdx.x == 0) {
    T.rec[2 * r0] = acc.t;
    T.rec[2 * r0 + 1] = acc.z;
  }
}

__global__ __launch_bounds__(kBlock) void k_lsq_fold_multi(const FBatch b) {
  const FCall &T = b.t[blockIdx.x];
  const int64_t nch = cdiv(T.nrec, kFoldChunk);
  LsqAcc acc{0.0, 0.0};
  for (int64_t c = threadIdx.x; c < nch; c += kBlock) {
    acc.t += T.rec[2 * c * kFoldChunk];
    acc.z += T.rec[2 * c * kFoldChunk + 1];
  }
  lsq_block_reduce(acc);
  if (threadIdx.x == 0) {
    T.out[0] = acc.t * T.gscale;
    double gz = 0.0;
    if (T.zpl) {
      const double zr = __builtin_rint(T.zdev ? *T.zdev : T.zhost);
      gz = (zr >= (double)T.lo && zr <= (double)T.hi) ? acc.z * T.gscale : 0.0;
    }
    T.out[1] = gz;
  }
}

// ----------------------------------------------------------------------------
// K6: per-channel learnable (LSQ) backward -- LSQFakeQuantize's per-channel path
// (quantizers/lsq_module.py:134-166) and a learnable PerChannelUniformQuantizer.
// A [rows, rowlen] view; row r uses the qparams of channel r % channels.
// Stage 1: workgroup (row, chunk) of kPcmGroups groups per lane -> grad_x and one
//          {sum t, sum z} record.  Stage 2: one workgroup per channel folds its
//          records (rows c, c+C, ...; chunks in order) -> grad_scale[c], grad_zp[c].
// ----------------------------------------------------------------------------
constexpr int kPcmGroups = 4;

inline int64_t pcm_chunks(int64_t rowlen) { return cdiv(cdiv(rowlen, 4), (int64_t)kBlock * kPcmGroups); }

template <bool VEC, bool NT, bool ZPL>
__global__ __launch_bounds__(kBlock) void k_pcm_lsq_bwd(const float *__restrict__ g,
                                                        const float *__restrict__ x,
                                                        float *__restrict__ gx, int64_t rowlen,
                                                        uint32_t chunks, int64_t channels,
                                                        const double *__restrict__ scale,
                                                        const double *__restrict__ zp, float lo,
                                                        float hi, double *__restrict__ ws) {
  const int64_t row = blockIdx.x / chunks;
  const int64_t chunk = blockIdx.x % chunks;
  const int64_t c = row % channels;
  const QPSrc src{nullptr, scale + c, zp ? zp + c : nullptr, 0.0, 0.0, lo, hi, ZPL ? 1 : 0, 0};
  const QP p = load_qp(src);
  LsqAcc acc{0.0, 0.0};
  const int64_t ng = cdiv(rowlen, 4);
  const float *xr = x + row * rowlen, *gr = g + row * rowlen;
  float *gxr = gx + row * rowlen;
  const int64_t base = chunk * kBlock * kPcmGroups + threadIdx.x;
  f4 xv[kPcmGroups], gv[kPcmGroups];
#pragma unroll
  for (int k = 0; k < kPcmGroups; ++k) {
    xv[k] = load_group_c<VEC, NT>(xr, base + k * kBlock, ng, rowlen);
    gv[k] = load_group_c<VEC, NT>(gr, base + k * kBlock, ng, rowlen);
  }
#pragma unroll
  for (int k = 0; k < kPcmGroups; ++k)
    lsq_group<VEC, NT, ZPL, kActNone>(gxr, base + k * kBlock, ng, rowlen, xv[k], gv[k], p, acc);
  lsq_block_reduce(acc);
  if (threadIdx.x == 0) {
    ws[2 * (int64_t)blockIdx.x] = acc.t;
    ws[2 * (int64_t)blockIdx.x + 1] = acc.z;
  }
}

__global__ __launch_bounds__(kBlock) void k_pcm_lsq_fold(const double *__restrict__ ws, int64_t rows,
                                                         uint32_t chunks, int64_t channels,
                                                         const double *__restrict__ zp, int zp_learn,
                                                         float lo, float hi, double gscale,
                                                         double *__restrict__ gs_out,
                                                         double *__restrict__ gz_out) {
  const int64_t c = blockIdx.x;
  const int64_t per = rows / channels * chunks;   // records of channel c, in (row, chunk) order
  LsqAcc acc{0.0, 0.0};
  for (int64_t k = threadIdx.x; k < per; k += kBlock) {
    const int64_t rec = ((k / chunks) * channels + c) * chunks + k % chunks;
    acc.t += ws[2 * rec];
    acc.z += ws[2 * rec + 1];
  }
  lsq_block_reduce(acc);
  if (threadIdx.x == 0) {
    gs_out[c] = acc.t * gscale;
    if (gz_out) {
      double gz = 0.0;
      if (zp_learn) {   // ClampBackward of the rounded zero point (lsq_module.py:339-343)
        const double zr = __builtin_rint(zp ? zp[c] : 0.0);
        gz = (zr >= (double)lo && zr <= (double)hi) ? acc.z * gscale : 0.0;
      }
      gz_out[c] = gz;
    }
  }
}

// K6 stage 1 on packed short rows (pc_packed): R whole rows per workgroup (see
// k_pcp_fq_fwd); each group's {t, z} terms go to LDS, then wave w sums rows w, w+4,
// ... (lanes over the row's groups in order, DPP tree) into the row's record -- the
// same ws layout as k_pcm_lsq_bwd with one chunk per row, folded by k_pcm_lsq_fold.
template <bool VEC, bool NT, bool ZPL>
__global__ __launch_bounds__(kBlock) void k_pcp_lsq_bwd(const float *__restrict__ g,
                                                        const float *__restrict__ x,
                                                        float *__restrict__ gx, int64_t rows,
                                                        int64_t rowlen, uint32_t rpb, int64_t channels,
                                                        const double *__restrict__ scale,
                                                        const double *__restrict__ zp, float lo,
                                                        float hi, double *__restrict__ ws) {
  __shared__ QP s_qp[kPackMaxRows];
  __shared__ double s_t[kPackGroups * kBlock], s_z[kPackGroups * kBlock];
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const uint32_t nr = (uint32_t)std::min<int64_t>(rpb, rows - r0);
  const uint32_t gpr = (uint32_t)(rowlen / 4);
  const int64_t n = rows * rowlen, ng = rows * gpr;
  const int64_t j0 = r0 * gpr;
  const uint32_t nj = nr * gpr;
  f4 xv[kPackGroups], gv[kPackGroups];
#pragma unroll
  for (int k = 0; k < kPackGroups; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    const int64_t i = j0 + (j < nj ? j : nj - 1);
    xv[k] = load_group_c<VEC, NT>(x, i, ng, n);
    gv[k] = load_group_c<VEC, NT>(g, i, ng, n);
  }
  if (threadIdx.x < nr) {
    const int64_t c = (r0 + threadIdx.x) % channels;
    s_qp[threadIdx.x] = load_qp(QPSrc{nullptr, scale + c, zp ? zp + c : nullptr, 0.0, 0.0, lo, hi,
                                      ZPL ? 1 : 0, 0});
  }
  lds_barrier();
  f4 o[kPackGroups];
#pragma unroll
  for (int k = 0; k < kPackGroups; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    const uint32_t jj = j < nj ? j : nj - 1;
    LsqAcc acc{0.0, 0.0};
    o[k] = lsq_group_out<ZPL, kActNone>(j0 + jj, ng, n, xv[k], gv[k], s_qp[jj / gpr], acc);
    if (j < nj) { s_t[j] = acc.t; s_z[j] = acc.z; }
  }
#pragma unroll
  for (int k = 0; k < kPackGroups; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    if (j < nj) store_group<VEC, NT>(gx, j0 + j, n, o[k]);
  }
  lds_barrier();   // the grad_x stores stay in flight
  const uint32_t w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  for (uint32_t r = w; r < nr; r += kWaves) {   // wave-uniform
    double t = 0.0, z = 0.0;
    for (uint32_t q = lane; q < gpr; q += kWave) { t += s_t[r * gpr + q]; z += s_z[r * gpr + q]; }
    t = wave_reduce(t, AddD());
    z = wave_reduce(z, AddD());
    if (lane == 0) {
      ws[2 * (r0 + r)] = t;
      ws[2 * (r0 + r) + 1] = z;
    }
  }
}

// K6 for axis 0 with whole rows in registers (rows == channels, 256 <= groups per row
// <= 9 x 256): workgroup c holds row c, so the row's {sum t, sum z} is the channel's
// total -- grad_scale[c] / grad_zp[c] are written directly (no records, no fold
// launch), and one-round grids store behind the store gate.  Same per-element code
// (lsq_group_out) as the two-stage form; the f64 sums differ only in order.
// At least 4 waves per SIMD (<= 128 VGPRs): 4 workgroups per CU, so the 1024 rows of a
// C2-shaped weight are ONE round on 256 CUs (round 5's learnable-zero-point variant at 9
// groups per lane took 134 VGPRs = 3 workgroups per CU = a second, quarter-occupied
// round: 24.2 us for 113 MB).  SPLIT (9 groups per lane): grad_x waits for the store gate
// in LDS (NV x 256 x 16 B) instead of registers, and the second half of the x / g loads
// is issued once ISSUE groups of the first half are computed (a scheduling barrier keeps
// the compiler from hoisting them) -- 111 VGPRs at ISSUE 3 (95 at 5, 119 at 2), no spills,
// where holding everything took 128 + 8-17 spilled (round 6, C2 bench leg
// pc_learn_bwd_k6: 0.67 against 0.56-0.66 for the other forms on the same boxes,
// profiles/r06/r06f_k6_stages.txt; issue point 5 / 3 / 2 twice each on one box: 0.683 /
// 0.703 / 0.701, then 0.687 / 0.702 / 0.700, profiles/r06/r06i_k6_issue.txt).  g by LDS-DMA
// (global_load_lds, all 18 loads at once) measured no better (profiles/r06/r06q_k6_glds.txt).
template <bool VEC, bool NT, bool ZPL, int NV, bool SPLIT, int ISSUE = 3>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_pcr_lsq_bwd(
    const float *__restrict__ g, const float *__restrict__ x, float *__restrict__ gx, int64_t rowlen,
    const double *__restrict__ scale, const double *__restrict__ zp, float lo, float hi, double gscale,
    double *__restrict__ gs_out, double *__restrict__ gz_out, uint32_t gate) {
  extern __shared__ f4 s_o[];   // SPLIT: [NV][kBlock]
  const GateClk gc = gate_begin(gate);
  const int64_t row = blockIdx.x;
  const int64_t ng = cdiv(rowlen, 4);
  const float *xr = x + row * rowlen, *gr = g + row * rowlen;
  float *gxr = gx + row * rowlen;
  f4 xv[NV], gv[NV], o[SPLIT ? 1 : NV];
  constexpr int H1 = SPLIT ? (NV + 1) / 2 : NV;
  LsqAcc acc{0.0, 0.0};
#pragma unroll
  for (int k = 0; k < H1; ++k) {
    xv[k] = load_group_c<VEC, NT>(xr, threadIdx.x + k * kBlock, ng, rowlen);
    gv[k] = load_group_c<VEC, NT>(gr, threadIdx.x + k * kBlock, ng, rowlen);
  }
  // the row's qparams after its loads are issued, as scalar loads (ld_uniform_f64)
  const QP p = load_qp<true>(QPSrc{nullptr, scale + row, zp ? zp + row : nullptr, 0.0, 0.0, lo, hi, ZPL ? 1 : 0, 0});
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (SPLIT && k == ISSUE) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = H1; j < NV; ++j) {
        xv[j] = load_group_c<VEC, NT>(xr, threadIdx.x + j * kBlock, ng, rowlen);
        gv[j] = load_group_c<VEC, NT>(gr, threadIdx.x + j * kBlock, ng, rowlen);
      }
    }
    const f4 r = lsq_group_out<ZPL, kActNone>(threadIdx.x + k * kBlock, ng, rowlen, xv[k], gv[k], p, acc);
    if constexpr (SPLIT) s_o[k * kBlock + threadIdx.x] = r;
    else o[k] = r;
  }
  lsq_block_reduce(acc);
  if (threadIdx.x == 0) {
    gs_out[row] = acc.t * gscale;
    if (gz_out) {   // ClampBackward of the rounded zero point (lsq_module.py:339-343)
      double gz = 0.0;
      if (ZPL) {
        const double zr = __builtin_rint(zp ? zp[row] : 0.0);
        gz = (zr >= (double)lo && zr <= (double)hi) ? acc.z * gscale : 0.0;
      }
      gz_out[row] = gz;
    }
  }
  gate_pass(gate, gc);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * kBlock;
    if (i < ng) store_group<VEC, NT>(gxr, i, rowlen, SPLIT ? s_o[k * kBlock + threadIdx.x] : o[k]);
  }
}

template <bool VEC, bool NT, bool ZPL, int NV>
void launch_pcr_nv(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                   const double *scale, const double *zp, float lo, float hi, double gscale,
                   double *gs, double *gz, hipStream_t st) {
  constexpr bool SPLIT = NV == 9;
  GateSel sel;
  const void *kern = reinterpret_cast<const void *>(k_pcr_lsq_bwd<VEC, NT, ZPL, NV, SPLIT>);
  if (g_tune.store_gate != 0) {
    static const int occ = occupancy_blocks(kern, kBlock);
    sel = store_gate_select("k6_pcr_lsq_bwd", kern, rows, occ, 8 * rows * rowlen, st);
  }
  const size_t lds = SPLIT ? (size_t)NV * kBlock * sizeof(f4) : 0;
  hipLaunchKernelGGL((k_pcr_lsq_bwd<VEC, NT, ZPL, NV, SPLIT>), dim3((unsigned)rows), dim3(kBlock), lds, st, g, x,
                     gx, rowlen, scale, zp, lo, hi, gscale, gs, gz, sel.gate);
  store_gate_launched(sel, st);
}

// rows == channels and whole rows fit 9 groups per lane with >= 1 per lane
inline bool pcr_fits(int64_t rows, int64_t rowlen, int64_t channels) {
  const int64_t ng = cdiv(rowlen, 4);
  return rows == channels && ng >= kBlock && ng <= 9 * kBlock;
}

template <bool VEC, bool NT>
void launch_pcr_lsq(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                    const double *scale, const double *zp, int zp_learn, float lo, float hi,
                    double gscale, double *gs, double *gz, hipStream_t st) {
  const int64_t per_lane = cdiv(cdiv(rowlen, 4), (int64_t)kBlock);
#define VSIQ_PCR(ZPL)                                                                               \
  (per_lane <= 1   ? launch_pcr_nv<VEC, NT, ZPL, 1>(g, x, gx, rows, rowlen, scale, zp, lo, hi, gscale, gs, gz, st) \
   : per_lane <= 2 ? launch_pcr_nv<VEC, NT, ZPL, 2>(g, x, gx, rows, rowlen, scale, zp, lo, hi, gscale, gs, gz, st) \
   : per_lane <= 3 ? launch_pcr_nv<VEC, NT, ZPL, 3>(g, x, gx, rows, rowlen, scale, zp, lo, hi, gscale, gs, gz, st) \
   : per_lane <= 5 ? launch_pcr_nv<VEC, NT, ZPL, 5>(g, x, gx, rows, rowlen, scale, zp, lo, hi, gscale, gs, gz, st) \
                   : launch_pcr_nv<VEC, NT, ZPL, 9>(g, x, gx, rows, rowlen, scale, zp, lo, hi, gscale, gs, gz, st))
  if (zp_learn) VSIQ_PCR(true);
  else VSIQ_PCR(false);
#undef VSIQ_PCR
}

template <bool VEC, bool NT>
void launch_pcp_lsq(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                    int64_t channels, const double *scale, const double *zp, int zp_learn, float lo,
                    float hi, double *ws, hipStream_t st) {
  const int64_t rpb = pc_pack_rows(rowlen);
  const dim3 grid((unsigned)cdiv(rows, rpb)), block(kBlock);
  if (zp_learn)
    hipLaunchKernelGGL((k_pcp_lsq_bwd<VEC, NT, true>), grid, block, 0, st, g, x, gx, rows, rowlen,
                       (uint32_t)rpb, channels, scale, zp, lo, hi, ws);
  else
    hipLaunchKernelGGL((k_pcp_lsq_bwd<VEC, NT, false>), grid, block, 0, st, g, x, gx, rows, rowlen,
                       (uint32_t)rpb, channels, scale, zp, lo, hi, ws);
}

// K6 stage 1 on channel columns (axis 1, short rows): workgroup (i, c) takes the rows
// (n, c) of NB consecutive images n = i*NB .. (the same channel, hence one qparam pair
// and one running {t, z} per thread), ~kPackElems elements; the workgroup's sums go to
// record i*C + c -- k_pcm_lsq_fold's layout for rows' = cdiv(N, NB) * C, one chunk.  No
// per-group LDS arrays or per-row reductions (the packed-rows form's tail), one block
// reduction; rows are rowlen floats contiguous (rowlen % 4 == 0, vector path only).
// 8 groups per lane (round 6; 4 before): 81 images of 10x10 per workgroup, 4 waves / SIMD,
// ONE round at 256x256x10x10 (1024 workgroups) where 4 groups took 1.17 rounds at 6 / SIMD.
// Kernel-trace medians, two passes on one box (profiles/r06/r06n_k6_column_groups.txt):
// 10x10 19.08 / 19.00 us against 20.20 / 19.40; 40x40 57.3 / 57.4 against 59.4 / 60.5;
// 20x20 32.4 / 32.6 against 32.1 / 32.0.  Channel tiles (a workgroup = adjacent channels'
// contiguous rows of a few images, every load coalesced over the run) measured slower:
// 24-26 us at 10x10, 38-39 at 20x20 (profiles/r06/r06o_k6_channel_tiles.txt).
constexpr int kColGroups = 8;
inline int64_t pcc_images(int64_t rowlen) {
  return std::max<int64_t>(1, (int64_t)kBlock * kColGroups * 4 / rowlen);
}

// ARRIVE (vsiq_pcm_lsq_bwd_arrive_f32): instead of a second launch, the channel's last
// workgroup folds it -- each workgroup stores its record write-through, drains it and
// bumps counters[c] (agent-scope relaxed add, the arrive_last pattern of K2 / K4); the
// one whose add returns nib - 1 takes an agent acquire, folds records i*C + c in the
// fixed order of k_pcm_lsq_fold (same bits), writes grad_scale[c] / grad_zp[c] and
// resets counters[c].  grad_x is stored after the arrival, so the drain waits only for
// the record.  No workgroup waits for another.
// Round 6 at 256x256x10x10: the channel's qparams as scalar loads after the x / g loads
// 22.2 -> 21.3 us; grad_x staged in LDS at 7 waves / SIMD (11 spilled VGPRs) 25.4 us, not
// taken (profiles/r06/r06k_k6_column.txt).
template <bool NT, bool ZPL, bool ARRIVE, int CG = kColGroups>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_pcc_lsq_bwd(const float *__restrict__ g,
                                                        const float *__restrict__ x,
                                                        float *__restrict__ gx, int64_t images,
                                                        int64_t rowlen, uint32_t nb_img, int64_t channels,
                                                        const double *__restrict__ scale,
                                                        const double *__restrict__ zp, float lo, float hi,
                                                        double *__restrict__ ws, uint32_t xo,
                                                        uint32_t *__restrict__ counters, uint32_t nib,
                                                        double gscale, double *__restrict__ gs_out,
                                                        double *__restrict__ gz_out) {
  // logical block i*C + c.  xo 1: XCD-contiguous (xcd_block); xo 2 (channels % 8 == 0): XCD x
  // takes channels [x C/8, (x+1) C/8) of every image block, image blocks outermost, so the
  // neighbours sharing lines stay on one XCD and the short last image block runs last
  uint32_t b = blockIdx.x;
  if (xo == 1) {
    b = xcd_block(blockIdx.x, gridDim.x);
  } else if (xo == 2) {
    const uint32_t cpx = (uint32_t)channels / kXcds, k = blockIdx.x / kXcds;
    b = (k / cpx) * (uint32_t)channels + (blockIdx.x % kXcds) * cpx + k % cpx;
  }
  const int64_t c = b % channels;
  const int64_t n0 = (int64_t)(b / channels) * nb_img;
  const uint32_t nr = (uint32_t)std::min<int64_t>(nb_img, images - n0);
  const uint32_t gpr = (uint32_t)(rowlen / 4);
  const uint32_t nj = nr * gpr;
  const int64_t rstride = channels * rowlen;               // floats between (n, c) and (n+1, c)
  const int64_t base = (n0 * channels + c) * rowlen;
  const float *xb = x + base, *gb = g + base;
  float *gxb = gx + base;
  f4 xv[CG], gv[CG];
  uint32_t off[CG];   // floats from base: < nb_img * channels * rowlen < 2^31 (host check)
#pragma unroll
  for (int k = 0; k < CG; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    const uint32_t jj = j < nj ? j : nj - 1;
    off[k] = (jj / gpr) * (uint32_t)rstride + 4 * (jj % gpr);
    xv[k] = load_group<true, NT>(xb + off[k], 0, 4);
    gv[k] = load_group<true, NT>(gb + off[k], 0, 4);
  }
  // the channel's qparams after the loads are issued, as scalar loads (ld_uniform_f64)
  const QP p = load_qp<true>(QPSrc{nullptr, scale + c, zp ? zp + c : nullptr, 0.0, 0.0, lo, hi, ZPL ? 1 : 0, 0});
  LsqAcc acc{0.0, 0.0};
  f4 o[CG];
#pragma unroll
  for (int k = 0; k < CG; ++k) {
    const uint32_t j = threadIdx.x + k * kBlock;
    o[k] = lsq_group_out<ZPL, kActNone>(j < nj ? 0 : 1, 1, 4, xv[k], gv[k], p, acc);   // i=1: no terms
  }
  if (!ARRIVE) {
#pragma unroll
    for (int k = 0; k < CG; ++k)
      if (threadIdx.x + k * kBlock < nj) store_group<true, NT>(gxb + off[k], 0, 4, o[k]);
    lsq_block_reduce(acc);
    if (threadIdx.x == 0) {
      ws[2 * (int64_t)b] = acc.t;
      ws[2 * (int64_t)b + 1] = acc.z;
    }
    return;
  }
  lsq_block_reduce(acc);
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    partial_store(ws + 2 * (int64_t)b, acc.t);
    partial_store(ws + 2 * (int64_t)b + 1, acc.z);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(counters + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == nib - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CG; ++k)
    if (threadIdx.x + k * kBlock < nj) store_group<true, NT>(gxb + off[k], 0, 4, o[k]);
  if (!s_last) return;
  LsqAcc f{0.0, 0.0};   // k_pcm_lsq_fold's order: thread j sums records j, j + 256, ... then the tree
  for (uint32_t i = threadIdx.x; i < nib; i += kBlock) {
    const int64_t rec = (int64_t)i * channels + c;
    f.t += partial_load(ws + 2 * rec);
    f.z += partial_load(ws + 2 * rec + 1);
  }
  lsq_block_reduce(f);
  if (threadIdx.x == 0) {
    gs_out[c] = f.t * gscale;
    if (gz_out) {
      double gz = 0.0;
      if (ZPL) {   // ClampBackward of the rounded zero point (lsq_module.py:339-343)
        const double zr = __builtin_rint(zp ? zp[c] : 0.0);
        gz = (zr >= (double)lo && zr <= (double)hi) ? f.z * gscale : 0.0;
      }
      gz_out[c] = gz;
    }
    __hip_atomic_store(counters + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


template <bool NT, bool ZPL, bool ARRIVE>
void launch_pcc_k(const float *g, const float *x, float *gx, int64_t images, int64_t rowlen, int64_t nb,
                  int64_t channels, int64_t grid, const double *scale, const double *zp, float lo, float hi,
                  double *ws, uint32_t *counters, double gscale, double *gs, double *gz, hipStream_t st) {
  // XCD-contiguous order where a row ends mid-line: at 10x10 rows ~half of the lines
  // are shared with the neighbouring channel's workgroup (PMC fetch 1.30x -> 1.04x the
  // algorithmic bytes, 24.2 -> 21.7 us at 256x256x10x10); 20x20 and up measured slower.
  // Order 2 (round 6, the default where channels % 8 == 0) keeps that sharing and runs the
  // short last image block last: 18.78 / 18.36 us against order 1's 18.84 / 18.96 and the
  // hardware order's 21.60 / 20.74 on one box (profiles/r06/r06l_k6_xcd_order.txt)
  uint32_t xo = g_tune.xcd_order != 0 && (rowlen * 4) % 128 != 0 && rowlen * 4 <= 512 ? 1u : 0u;
  if (xo && g_tune.xcd_order == 2 && channels % kXcds == 0) xo = 2;
  hipLaunchKernelGGL((k_pcc_lsq_bwd<NT, ZPL, ARRIVE>), dim3((unsigned)grid), dim3(kBlock), 0, st, g, x, gx, images,
                     rowlen, (uint32_t)nb, channels, scale, zp, lo, hi, ws, xo, counters,
                     (uint32_t)cdiv(images, nb), gscale, gs, gz);
}

// counters != nullptr: the channel's last workgroup folds (no second launch)
template <bool NT>
int64_t launch_pcc_lsq(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                       int64_t channels, const double *scale, const double *zp, int zp_learn, float lo,
                       float hi, double *ws, uint32_t *counters, double gscale, double *gs, double *gz,
                       hipStream_t st) {
  const int64_t images = rows / channels, nb = pcc_images(rowlen);
  const int64_t iblocks = cdiv(images, nb), grid = iblocks * channels;
#define VSIQ_PCC(ZPL, AR) \
  launch_pcc_k<NT, ZPL, AR>(g, x, gx, images, rowlen, nb, channels, grid, scale, zp, lo, hi, ws, counters, gscale, gs, gz, st)
  if (counters) {
    if (zp_learn) VSIQ_PCC(true, true);
    else VSIQ_PCC(false, true);
  } else {
    if (zp_learn) VSIQ_PCC(true, false);
    else VSIQ_PCC(false, false);
  }
#undef VSIQ_PCC
  return iblocks * channels;   // record rows for k_pcm_lsq_fold (one chunk each)
}

template <bool VEC, bool NT>
void launch_pcm_lsq(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                    int64_t channels, const double *scale, const double *zp, int zp_learn, float lo,
                    float hi, double *ws, hipStream_t st) {
  const int64_t chunks = pcm_chunks(rowlen);
  const dim3 grid((unsigned)(rows * chunks)), block(kBlock);
  if (zp_learn)
    hipLaunchKernelGGL((k_pcm_lsq_bwd<VEC, NT, true>), grid, block, 0, st, g, x, gx, rowlen,
                       (uint32_t)chunks, channels, scale, zp, lo, hi, ws);
  else
    hipLaunchKernelGGL((k_pcm_lsq_bwd<VEC, NT, false>), grid, block, 0, st, g, x, gx, rowlen,
                       (uint32_t)chunks, channels, scale, zp, lo, hi, ws);
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t n,
                     const double *scale_dev, double scale_host, const double *zp_dev,
                     double zp_host, int zp_learn, int qmin, int qmax, double gscale,
                     double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
                     void *stream) {
  return lsq_bwd(g, x, gx, n, kActNone, scale_dev, scale_host, zp_dev, zp_host, zp_learn, qmin, qmax,
                 gscale, grad_out, ws, ws_len, counter, stream);
}

int vsiq_act_lsq_bwd_f32(const float *g, const float *c, float *gc, int64_t n, int act,
                         const double *scale_dev, double scale_host, const double *zp_dev,
                         double zp_host, int zp_learn, int qmin, int qmax, double gscale,
                         double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
                         void *stream) {
  return lsq_bwd(g, c, gc, n, act, scale_dev, scale_host, zp_dev, zp_host, zp_learn, qmin, qmax,
                 gscale, grad_out, ws, ws_len, counter, stream);
}

int64_t vsiq_lsq_part_records(int64_t n) {
  if (n <= 0) return VSIQ_E_ARG;
  return lsq_grid(cdiv(n, 4), lsq_part_groups_per_lane(n));
}

int vsiq_act_lsq_bwd_part_f32(const float *g, const float *c, float *gc, int64_t n, int act,
                              const double *scale_dev, double scale_host, const double *zp_dev, double zp_host,
                              int zp_learn, int qmin, int qmax, double *records, int64_t records_len,
                              void *stream) {
  return lsq_bwd_part(g, c, gc, n, act, scale_dev, scale_host, zp_dev, zp_host, zp_learn, qmin, qmax, records,
                      records_len, stream);
}

int vsiq_lsq_fold_multi(const vsiq_lsq_fold *folds, int count, void *stream) {
  if (count < 0 || (count > 0 && !folds)) return VSIQ_E_ARG;
  for (int i = 0; i < count; ++i)
    if (!folds[i].records || folds[i].nrec <= 0 || !folds[i].grad_out || folds[i].qmin > folds[i].qmax)
      return VSIQ_E_ARG;
  for (int i0 = 0; i0 < count; i0 += kFoldMulti) {
    FBatch b{};
    b.count = std::min(kFoldMulti, count - i0);
    uint32_t chunks = 0;
    for (int k = 0; k < b.count; ++k) {
      const vsiq_lsq_fold &F = folds[i0 + k];
      b.t[k] = FCall{F.records, F.zp_dev, F.grad_out, F.nrec, F.zp_host, F.gscale, (float)F.qmin, (float)F.qmax,
                     F.zp_learn};
      b.c0[k] = chunks;
      chunks += (uint32_t)cdiv(F.nrec, kFoldChunk);
    }
    b.c0[b.count] = chunks;
    hipLaunchKernelGGL(k_lsq_fold_chunks, dim3(chunks), dim3(kBlock), 0, (hipStream_t)stream, b);
    int rc = launch_rc();
    if (rc) return rc;
    hipLaunchKernelGGL(k_lsq_fold_multi, dim3((unsigned)b.count), dim3(kBlock), 0, (hipStream_t)stream, b);
    rc = launch_rc();
    if (rc) return rc;
  }
  return 0;
}

int64_t vsiq_pcm_workspace_doubles(int64_t rows, int64_t rowlen) {
  if (rows < 0 || rowlen <= 0) return VSIQ_E_ARG;
  return 2 * rows * pcm_chunks(rowlen);
}

int vsiq_pcm_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                         int64_t channels, const double *scale, const double *zp, int zp_learn,
                         int qmin, int qmax, double gscale, double *grad_scale_out,
                         double *grad_zp_out, double *ws, int64_t ws_len, void *stream) {
  return vsiq_pcm_lsq_bwd_arrive_f32(g, x, gx, rows, rowlen, channels, scale, zp, zp_learn, qmin, qmax, gscale,
                                     grad_scale_out, grad_zp_out, ws, ws_len, nullptr, 0, stream);
}

int vsiq_pcm_lsq_bwd_arrive_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                                int64_t channels, const double *scale, const double *zp, int zp_learn, int qmin,
                                int qmax, double gscale, double *grad_scale_out, double *grad_zp_out, double *ws,
                                int64_t ws_len, uint32_t *counters, int64_t counters_len, void *stream) {
  if (rows <= 0 || rowlen <= 0 || channels <= 0 || rows % channels || qmin > qmax || !g || !x ||
      !gx || !scale || !grad_scale_out || !ws || (zp_learn && !zp))
    return VSIQ_E_ARG;
  if (counters && counters_len < channels) return VSIQ_E_WS;
  const int64_t chunks = pcm_chunks(rowlen);
  if (rows * chunks > 0x7fffffffLL || channels > 0x7fffffffLL) return VSIQ_E_ARG;
  if (ws_len < 2 * rows * chunks) return VSIQ_E_WS;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (rowlen % 4 == 0) && aligned16(g) && aligned16(x) && aligned16(gx);
  const bool nt = g_tune.nontemporal != 0;
  if (pcr_fits(rows, rowlen, channels) && g_tune.pc_packed != 0) {   // axis 0, rows in registers
    VSIQ_B2(launch_pcr_lsq, vec, nt, g, x, gx, rows, rowlen, scale, zp, zp_learn, (float)qmin, (float)qmax,
            gscale, grad_scale_out, grad_zp_out, st);
    return launch_rc();
  }
  int64_t frows = rows, fchunks = chunks;   // record layout the fold reads
  const int packed = g_tune.pc_packed;
  if (vec && pc_packed(rowlen) && rows > channels && packed == 1 &&
      pcc_images(rowlen) * channels * rowlen < ((int64_t)1 << 31)) {   // axis 1, short rows: columns
    frows = nt ? launch_pcc_lsq<true>(g, x, gx, rows, rowlen, channels, scale, zp, zp_learn, (float)qmin,
                                      (float)qmax, ws, counters, gscale, grad_scale_out, grad_zp_out, st)
               : launch_pcc_lsq<false>(g, x, gx, rows, rowlen, channels, scale, zp, zp_learn, (float)qmin,
                                       (float)qmax, ws, counters, gscale, grad_scale_out, grad_zp_out, st);
    fchunks = 1;
    if (counters) return launch_rc();   // folded in the launch
  } else if (pc_packed(rowlen) && packed != 0) {   // one chunk per row: same record layout
    VSIQ_B2(launch_pcp_lsq, vec, nt, g, x, gx, rows, rowlen, channels, scale, zp, zp_learn, (float)qmin,
            (float)qmax, ws, st);
  } else {
    VSIQ_B2(launch_pcm_lsq, vec, nt, g, x, gx, rows, rowlen, channels, scale, zp, zp_learn, (float)qmin,
            (float)qmax, ws, st);
  }
  hipLaunchKernelGGL(k_pcm_lsq_fold, dim3((unsigned)channels), dim3(kBlock), 0, st, ws, frows,
                     (uint32_t)fchunks, channels, zp, zp_learn, (float)qmin, (float)qmax, gscale,
                     grad_scale_out, grad_zp_out);
  return launch_rc();
}

}  // extern "C"
