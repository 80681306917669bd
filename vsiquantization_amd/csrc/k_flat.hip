// k_flat.hip — K2 per-tensor observer (optionally over a fused ReLU/SiLU), the
// division / fast-path self-tests, and the library-level C ABI entry points
// (K1 lives in k_fq.hip, K4 in k_lsq.hip, the STE backward in k_ste.hip).
#include "k_body.cuh"   // K1 block body (K9); includes vsiq_common.cuh

namespace vsiq {

Tuning g_tune;

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
  const float p2 = (v.x * v.x + vy * vy) + (vz * vz + vw * vw);   // fp32 over 4, f64 across groups
  a.sa += (double)pa;
  a.s1 += (double)p1;
  a.s2 += (double)p2;
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

struct ObsFold {   // partial record {min, max, nan count, sum|x|, sum x, sum x^2}
  static constexpr int K = 6;
  __device__ static void init(double (&a)[6]) {
    a[0] = __builtin_inf(); a[1] = -__builtin_inf();
    a[2] = a[3] = a[4] = a[5] = 0.0;
  }
  __device__ static void add(double (&a)[6], const double (&r)[6]) {
    a[0] = __builtin_fmin(a[0], r[0]); a[1] = __builtin_fmax(a[1], r[1]);
    a[2] += r[2]; a[3] += r[3]; a[4] += r[4]; a[5] += r[5];
  }
  __device__ static void wave(double (&a)[6]) {
    a[0] = wave_reduce(a[0], MinD()); a[1] = wave_reduce(a[1], MaxD());
#pragma unroll
    for (int k = 2; k < 6; ++k) a[k] = wave_reduce(a[k], AddD());
  }
};

// Block partial -> workspace record; the workgroup holding the fold of every record
// writes the stats record and applies the running update.
__device__ __forceinline__ void observe_epilogue(ObsAcc &a, int64_t n, double *__restrict__ stats_out,
                                                 float *__restrict__ run_minmax,
                                                 double *__restrict__ qp_out, int sym, double qden,
                                                 double eps, double *__restrict__ ws,
                                                 uint32_t *__restrict__ counter) {
  obs_block_reduce(a);
  double f[6];
  if (gridDim.x == 1) {   // one workgroup (small tensors): no records, no arrival
    f[0] = a.mn; f[1] = a.mx; f[2] = (double)a.nan; f[3] = a.sa; f[4] = a.s1; f[5] = a.s2;
    if (threadIdx.x == 0) {
      if (stats_out) write_stats(stats_out, f, n);
      observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax, qp_out, sym, qden, eps);
    }
    return;
  }
  if (threadIdx.x == 0) {
    double *r = ws + (int64_t)blockIdx.x * kPartials;
    partial_store(r + 0, a.mn); partial_store(r + 1, a.mx); partial_store(r + 2, (double)a.nan);
    partial_store(r + 3, a.sa); partial_store(r + 4, a.s1); partial_store(r + 5, a.s2);
  }
  if (!fold_arrivals<ObsFold>(ws, counter, f)) return;
  if (threadIdx.x == 0) {
    if (stats_out) write_stats(stats_out, f, n);
    observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax, qp_out, sym, qden, eps);
    *counter = 0u;   // ready for the next stream-ordered launch
  }
}

// Grid-stride accumulation of a fixed grid over x (U groups per lane per step): the
// body shared by k_observe_loop and k_observe_part.
// Block `blk` of an `nblk`-block grid over x (the multi-tensor K2m runs the same body
// on its tensors' block ranges).
template <bool VEC, bool NT, int ACT, int U>
__device__ __forceinline__ void observe_stride_b(const float *__restrict__ x, int64_t n, ObsAcc &a,
                                                 int64_t blk, int64_t nblk, const SiluLay &L) {
  obs_init(a);
  const int64_t ng = cdiv(n, 4);
  const int64_t nfull = n / 4;
  const int64_t step = nblk * kBlock * U;
  for (int64_t b = blk * kBlock * U; b < ng; b += step) {
    f4 v[U];
    if (VEC && b + (int64_t)kBlock * U <= nfull) {
      // every group of this step is whole (block-uniform): one uniform base pointer and
      // 32-bit lane offsets (no per-group 64-bit clamp / address arithmetic: -16 VGPRs,
      // -40 instructions per step at U = 8), straight-line, no per-group exec-mask
      // branches (they were ~1/3 of the K2p instruction stream)
      const float *xb = x + 4 * b;
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ld4<NT>(xb + 4 * (threadIdx.x + k * kBlock));
#pragma unroll
      for (int k = 0; k < U; ++k) obs_add4(a, act_fwd4_at<ACT>(v[k], 4 * (b + threadIdx.x + k * kBlock), L), 4);
      continue;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = load_group_c<VEC, NT>(x, b + threadIdx.x + k * kBlock, ng, n);
    if (b + (int64_t)kBlock * U <= nfull) {
#pragma unroll
      for (int k = 0; k < U; ++k) obs_add4(a, act_fwd4_at<ACT>(v[k], 4 * (b + threadIdx.x + k * kBlock), L), 4);
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int64_t i = b + threadIdx.x + k * kBlock;
        if (i < nfull) obs_add4(a, act_fwd4_at<ACT>(v[k], 4 * i, L), 4);
        else if (i < ng) obs_add4(a, act_fwd4_at<ACT>(v[k], 4 * i, L), valid_in_group(i, n));
      }
    }
  }
}

template <bool VEC, bool NT, int ACT, int U>
__device__ __forceinline__ void observe_stride(const float *__restrict__ x, int64_t n, ObsAcc &a,
                                               const SiluLay &L) {
  observe_stride_b<VEC, NT, ACT, U>(x, n, a, blockIdx.x, gridDim.x, L);
}

// One-shot: G groups per lane (grid = ng / (256 G)), all G loads issued up front
// (no loop: the loads of a wave stay in flight together and s_waitcnt is exact).
template <bool VEC, bool NT, int ACT, int G>
__global__ __launch_bounds__(kBlock) void k_observe(const float *__restrict__ x, int64_t n,
                                                    double *__restrict__ stats_out,
                                                    float *__restrict__ run_minmax,
                                                    double *__restrict__ qp_out, int sym,
                                                    double qden, double eps,
                                                    double *__restrict__ ws,
                                                    uint32_t *__restrict__ counter, SiluLay L) {
  ObsAcc a;
  obs_init(a);
  const int64_t ng = cdiv(n, 4);
  const int64_t base = (int64_t)blockIdx.x * kBlock * G + threadIdx.x;
  f4 v[G];
#pragma unroll
  for (int k = 0; k < G; ++k) v[k] = load_group_c<VEC, NT>(x, base + k * kBlock, ng, n);
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int64_t i = base + k * kBlock;
    if (i < ng) obs_add4(a, act_fwd4_at<ACT>(v[k], 4 * i, L), valid_in_group(i, n));
  }
  observe_epilogue(a, n, stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter);
}

// Grid-stride: a fixed grid (at most kObsGrid workgroups, independent of the device, so
// the accumulation order is fixed per n) walks the tensor U groups per lane per step.
// A pure read (no stores share vmcnt with the loads), latency hidden by the other
// waves of the CU.  Fewer, longer-lived workgroups than the one-shot form: fewer
// partial records to fold and arrivals to serialize (MI355X, C5 layer sizes:
// 52M elements 53.2 -> 38.6 us, 1.6M 10.1 -> 9.4 us; tools/exp/obs_bench.py).
template <bool VEC, bool NT, int ACT, int U>
__global__ __launch_bounds__(kBlock) void k_observe_loop(const float *__restrict__ x, int64_t n,
                                                          double *__restrict__ stats_out,
                                                          float *__restrict__ run_minmax,
                                                          double *__restrict__ qp_out, int sym,
                                                          double qden, double eps,
                                                          double *__restrict__ ws,
                                                          uint32_t *__restrict__ counter, SiluLay L) {
  ObsAcc a;
  observe_stride<VEC, NT, ACT, U>(x, n, a, L);
  observe_epilogue(a, n, stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter);
}

// One K2p record per WAVE (DPP reductions only): no LDS round trip and no barrier in
// the tail of the grid (C5 observe phase 263 -> 253-258 us on MI355X,
// tools/exp/floor_bench.py).  Record {min, max, nan count, sum|x|, sum x, sum x^2, n,
// records} of wave w of block blk.
__device__ __forceinline__ void store_part_record(ObsAcc &a, double *__restrict__ parts, int64_t blk,
                                                  int64_t nblk, int64_t n) {
  a.mn = wave_reduce(a.mn, MinOp());
  a.mx = wave_reduce(a.mx, MaxOp());
  a.nan = wave_reduce(a.nan, AddU());
  a.sa = wave_reduce(a.sa, AddD());
  a.s1 = wave_reduce(a.s1, AddD());
  a.s2 = wave_reduce(a.s2, AddD());
  if (threadIdx.x % kWave == 0) {
    double *r = parts + (blk * kWaves + threadIdx.x / kWave) * VSIQ_PART_LEN;
    r[0] = a.mn; r[1] = a.mx; r[2] = (double)a.nan; r[3] = a.sa;
    r[4] = a.s1; r[5] = a.s2; r[6] = (double)n; r[7] = (double)nblk * kWaves;
  }
}

// K2p: the grid-stride pass of k_observe_loop WITHOUT the cross-workgroup fold.  Each
// wave stores its record {min, max, nan count, sum|x|, sum x, sum x^2, n, records}
// (VSIQ_PART_LEN doubles, plain stores) and exits: no arrival atomics, no
// last-block fold, no running update.  For calibration, where nothing consumes an
// observer's result before the calibration ends: k_observe_fold_parts folds every
// call's records at once (deferred sync), and the running min/max is replayed there.
template <bool VEC, bool NT, int ACT, int U>
__global__ __launch_bounds__(kBlock) void k_observe_part(const float *__restrict__ x, int64_t n,
                                                          double *__restrict__ parts, SiluLay L) {
  ObsAcc a;
  observe_stride<VEC, NT, ACT, U>(x, n, a, L);
  store_part_record(a, parts, blockIdx.x, gridDim.x, n);
}

// ----------------------------------------------------------------------------
// K2o: a calibration forward of a fused layer in ONE pass -- y = act(c), the tensor the
// next layer consumes (modules/fused.py:133), and the deferred observer's K2p records of
// act(c) (minmax.py:42-43 + qm.py:66-68) -- instead of an activation pass that writes y
// and an observer pass that reads it again (8 instead of 12 B per element) and with
// nothing queued that user code could modify before it is observed.  Same grid, groups
// per lane and accumulation order as k_observe_part, so the records are the same bits.
// ----------------------------------------------------------------------------
template <bool VEC, bool NT, int ACT, int U>
__global__ __launch_bounds__(kBlock) void k_observe_part_out(const float *__restrict__ x, float *__restrict__ y,
                                                              int64_t n, double *__restrict__ parts, SiluLay L) {
  ObsAcc a;
  obs_init(a);
  const int64_t ng = cdiv(n, 4);
  const int64_t nfull = n / 4;
  const int64_t step = (int64_t)gridDim.x * kBlock * U;
  for (int64_t b = (int64_t)blockIdx.x * kBlock * U; b < ng; b += step) {
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = load_group_c<VEC, NT>(x, b + threadIdx.x + k * kBlock, ng, n);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = b + threadIdx.x + k * kBlock;
      v[k] = act_fwd4_at<ACT>(v[k], 4 * i, L);
      if (i < nfull) obs_add4(a, v[k], 4);
      else if (i < ng) obs_add4(a, v[k], valid_in_group(i, n));
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = b + threadIdx.x + k * kBlock;
      if (i < ng) store_group<VEC, NT>(y, i, n, v[k]);
    }
  }
  store_part_record(a, parts, blockIdx.x, gridDim.x, n);
}

// K2o one-shot form (the default): workgroup b (BS lanes) takes groups
// [b*BS*G, (b+1)*BS*G) -- G loads per lane issued at once, act + observer terms in
// registers, the workgroup's record through LDS, then the G stores: no loop, so no store
// shares a vmcnt wait with a later load (a grid-stride step waits for its own stores
// before the next step's loads can be consumed: hipcc's s_waitcnt treats mixed load /
// store counts as out of order).  One record per WORKGROUP (k2o_records(n)); the block
// reduction runs before the stores (no fence between the y stores and the barrier).
// Measured on MI355X (profiles/r04b_k2o_*): G = 2 streams best at every C5 size (52M
// elements: 68.1 us = 0.77 of 8 TB/s, vs 76.8 us at G = 16 and 96 % of the activation
// alone); BS trades the record count (the sync's fold) against the tail.  `gate`: the
// one-round G = 9 form's store gate (round 5, launch_k2o_gated; 0 = none), like K1's.
template <bool VEC, bool NT, int ACT, int G, int BS>
__global__ __launch_bounds__(BS) void k_observe_part_out1(const float *__restrict__ x, float *__restrict__ y,
                                                           int64_t n, double *__restrict__ parts, SiluLay L,
                                                           uint32_t gate) {
  const GateClk gc = gate_begin(gate);
  constexpr int NW = BS / kWave;
  __shared__ float s_mn[NW], s_mx[NW];
  __shared__ uint32_t s_nan[NW];
  __shared__ double s_sa[NW], s_s1[NW], s_s2[NW];
  const int64_t ng = cdiv(n, 4);
  const int64_t nfull = n / 4;
  const int64_t base = (int64_t)blockIdx.x * BS * G;
  ObsAcc a;
  obs_init(a);
  f4 v[G];
  const bool whole = VEC && base + (int64_t)BS * G <= nfull;   // block-uniform
  if (whole) {
    const float *xb = x + 4 * base;
#pragma unroll
    for (int k = 0; k < G; ++k) v[k] = ld4<NT>(xb + 4 * (threadIdx.x + k * BS));
#pragma unroll
    for (int k = 0; k < G; ++k) {
      v[k] = act_fwd4_at<ACT>(v[k], 4 * (base + threadIdx.x + k * BS), L);
      obs_add4(a, v[k], 4);
    }
  } else {
#pragma unroll
    for (int k = 0; k < G; ++k) v[k] = load_group_c<VEC, NT>(x, base + threadIdx.x + k * BS, ng, n);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int64_t i = base + threadIdx.x + k * BS;
      v[k] = act_fwd4_at<ACT>(v[k], 4 * i, L);
      if (i < nfull) obs_add4(a, v[k], 4);
      else if (i < ng) obs_add4(a, v[k], valid_in_group(i, n));
    }
  }
  a.mn = wave_reduce(a.mn, MinOp());
  a.mx = wave_reduce(a.mx, MaxOp());
  a.nan = wave_reduce(a.nan, AddU());
  a.sa = wave_reduce(a.sa, AddD());
  a.s1 = wave_reduce(a.s1, AddD());
  a.s2 = wave_reduce(a.s2, AddD());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) {
    s_mn[w] = a.mn; s_mx[w] = a.mx; s_nan[w] = a.nan;
    s_sa[w] = a.sa; s_s1[w] = a.s1; s_s2[w] = a.s2;
  }
  __syncthreads();
  gate_pass(gate, gc);
  if (whole) {
    float *yb = y + 4 * base;
#pragma unroll
    for (int k = 0; k < G; ++k) st4<NT>(yb + 4 * (threadIdx.x + k * BS), v[k]);
  } else {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int64_t i = base + threadIdx.x + k * BS;
      if (i < ng) store_group<VEC, NT>(y, i, n, v[k]);
    }
  }
  if (threadIdx.x == 0) {   // waves in order: fixed per n
    double f[6] = {s_mn[0], s_mx[0], (double)s_nan[0], s_sa[0], s_s1[0], s_s2[0]};
    for (int i = 1; i < NW; ++i) {
      f[0] = fminf((float)f[0], s_mn[i]); f[1] = fmaxf((float)f[1], s_mx[i]); f[2] += s_nan[i];
      f[3] += s_sa[i]; f[4] += s_s1[i]; f[5] += s_s2[i];
    }
    double *r = parts + (int64_t)blockIdx.x * VSIQ_PART_LEN;
    r[0] = f[0]; r[1] = f[1]; r[2] = f[2]; r[3] = f[3];
    r[4] = f[4]; r[5] = f[5]; r[6] = (double)n; r[7] = (double)gridDim.x;
  }
}

// ----------------------------------------------------------------------------
// K8: per-tensor observe + qparams + fake quant of a SMALL tensor in one launch.  One
// 1024-lane workgroup holds the whole tensor in registers (<= 16 groups per lane,
// 65536 elements): it reduces min / max / NaN / sums (the K2 stats record), applies the
// running update and the f64 qparams (minmax.py:42-74, qm.py:66-68) and fake-quantizes
// from registers (uniform.py:55,95) -- K2 + K1 (two launches, the qparams through
// memory) in one.  The reference's per-call observe+quantize of a small tensor
// (quantization_manager.py:73-90; a calibration call on a weight, BASELINE C1).
// ----------------------------------------------------------------------------
constexpr int kSmallBlock = 1024;
constexpr int kSmallGroups = 16;
constexpr int64_t kSmallMax = (int64_t)kSmallBlock * kSmallGroups * 4;

template <bool VEC, bool NT, int ACT, bool MASK, bool CODES, int U>
__global__ __launch_bounds__(kSmallBlock) void k_observe_fq_small(
    const float *__restrict__ x, float *__restrict__ y, uint8_t *__restrict__ codes,
    uint64_t *__restrict__ mask, int64_t n, double *__restrict__ stats_out, float *__restrict__ run_minmax,
    double *__restrict__ qp_out, int sym, double qden, double eps, float lo, float hi, SiluLay L) {
  constexpr int NW = kSmallBlock / kWave;
  __shared__ float s_mn[NW], s_mx[NW];
  __shared__ uint32_t s_nan[NW];
  __shared__ double s_sa[NW], s_s1[NW], s_s2[NW];
  __shared__ double s_qp[2];
  const int64_t ng = cdiv(n, 4);
  f4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k)
    v[k] = act_fwd4_at<ACT>(load_group_c<VEC, NT>(x, threadIdx.x + k * kSmallBlock, ng, n),
                            4 * (int64_t)(threadIdx.x + k * kSmallBlock), L);
  ObsAcc a;
  obs_init(a);
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int64_t i = threadIdx.x + k * kSmallBlock;
    if (i < ng) obs_add4(a, v[k], valid_in_group(i, n));
  }
  a.mn = wave_reduce(a.mn, MinOp());
  a.mx = wave_reduce(a.mx, MaxOp());
  a.nan = wave_reduce(a.nan, AddU());
  a.sa = wave_reduce(a.sa, AddD());
  a.s1 = wave_reduce(a.s1, AddD());
  a.s2 = wave_reduce(a.s2, AddD());
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) {
    s_mn[w] = a.mn; s_mx[w] = a.mx; s_nan[w] = a.nan;
    s_sa[w] = a.sa; s_s1[w] = a.s1; s_s2[w] = a.s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double f[6] = {s_mn[0], s_mx[0], (double)s_nan[0], s_sa[0], s_s1[0], s_s2[0]};
    for (int i = 1; i < NW; ++i) {   // fixed order
      f[0] = fminf((float)f[0], s_mn[i]); f[1] = fmaxf((float)f[1], s_mx[i]); f[2] += s_nan[i];
      f[3] += s_sa[i]; f[4] += s_s1[i]; f[5] += s_s2[i];
    }
    if (stats_out) write_stats(stats_out, f, n);
    observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax, qp_out, sym, qden, eps, &s_qp[0],
                    &s_qp[1]);
  }
  __syncthreads();
  QP p;
  p.s = (float)s_qp[0];
  p.z = (float)s_qp[1];
  p.lo = lo;
  p.hi = hi;
  p.discrete = 0;
  p.d = make_fastdiv(p.s);
  p.fast = fq_fast_qp(p.s, p.z);
  // every load was consumed before the barrier: each group is stored as soon as it is
  // quantized (no output array held in registers, no vmcnt hazard)
  uint32_t mlo = 0, mhi = 0;
  const int lane = threadIdx.x % kWave;
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int64_t i = threadIdx.x + k * kSmallBlock;
    const GroupOut go = fq_out_flat<VEC, CODES, MASK>(v[k], p, i, n);
    if (MASK) mask_put(mlo, mhi, k, go.b);
    if (i - lane < ng) fq_store_out<VEC, NT, CODES>(y, codes, i, ng, n, go);   // wave-uniform test
  }
  if (MASK && lane < 4 * U) {   // lane 4k+j: word j of slot k's chunk
    const int64_t first = (int64_t)threadIdx.x - lane + (lane >> 2) * kSmallBlock;
    if (first < ng) mask[4 * (first / kWave) + (lane & 3)] = ((uint64_t)mhi << 32) | mlo;
  }
}

template <bool VEC, bool NT, int ACT>
void launch_observe_fq_small(const float *x, float *y, uint8_t *c, uint64_t *m, int64_t n, double *st,
                             float *run, double *qp, int sym, double qden, double eps, float lo, float hi,
                             const SiluLay &L, hipStream_t s) {
  // groups per lane: 2 up to 8192 elements (no clamped duplicate loads), else 16
#define K8(MASK, CODES)                                                                                    \
  if (n <= (int64_t)kSmallBlock * 2 * 4)                                                                   \
    hipLaunchKernelGGL((k_observe_fq_small<VEC, NT, ACT, MASK, CODES, 2>), dim3(1), dim3(kSmallBlock), 0, s, x, \
                       y, c, m, n, st, run, qp, sym, qden, eps, lo, hi, L);                                    \
  else                                                                                                     \
    hipLaunchKernelGGL((k_observe_fq_small<VEC, NT, ACT, MASK, CODES, kSmallGroups>), dim3(1), dim3(kSmallBlock), \
                       0, s, x, y, c, m, n, st, run, qp, sym, qden, eps, lo, hi, L)
  if (m && c) { K8(true, true); }
  else if (m) { K8(true, false); }
  else if (c) { K8(false, true); }
  else { K8(false, false); }
#undef K8
}

// ----------------------------------------------------------------------------
// K9: per-call observe + fake quant of a mid-size tensor (K8's limit .. kFoldFqMax) in
// two launches and WITHOUT K2's cross-workgroup arrival chain (~3 us of atomics, fence
// and last-block fold at C1's 65536 elements, profiles/r02p_c1_sweep.txt).  K2p writes
// one record per wave (plain stores); then every workgroup of the fake-quant launch
// folds all of them in the same fixed order (the same bits in every workgroup), derives
// the running update and the f64 qparams itself (minmax.py:42-74) and quantizes its
// share with K1's block body (uniform.py:55,95).  Workgroup 0 alone writes the running
// state, the qparams record and the stats record.  The running update is idempotent
// (min / max; a NaN call changes nothing, minmax.py:42-47), so a workgroup that reads
// the state after workgroup 0 has written it computes the same qparams.
// ----------------------------------------------------------------------------
constexpr int kK2oGroups = 2;                  // K2o one-shot: groups per lane (default)
constexpr int kK2oBlock = 256;                 // K2o one-shot: lanes per workgroup (default)
constexpr int kFoldFqGrid = 32;                 // K2p workgroups: <= 128 records per fold
constexpr int kFoldFqU = 4;                     // K2p groups per lane per step
constexpr int64_t kFoldFqMax = (int64_t)1 << 18;   // largest n (fq grid <= 128 workgroups)

template <int ACT, int U>
void launch_observe_part_u(bool vec, bool nt, const float *x, int64_t n, double *parts, int64_t grid,
                           const SiluLay &L, hipStream_t st);   // K2p launch, below

inline int64_t fold_fq_part_grid(int64_t n) {
  const int64_t units = cdiv(cdiv(n, 4), (int64_t)kBlock);
  return std::min<int64_t>(kFoldFqGrid, std::max<int64_t>(1, cdiv(units, kFoldFqU)));
}

template <bool VEC, bool NT, bool CODES, bool MASK, int ACT>
__global__ __launch_bounds__(kBlock) void k_fold_fq_fwd(
    const float *__restrict__ x, float *__restrict__ y, uint8_t *__restrict__ codes,
    uint64_t *__restrict__ mask, int64_t n, const double *__restrict__ parts, int nrec,
    double *__restrict__ stats_out, float *__restrict__ run_minmax, double *__restrict__ qp_out, int sym,
    double qden, double eps, float lo, float hi, SiluLay L) {
  __shared__ double s_f[kWaves][6];
  __shared__ double s_qp[2];
  double f[6];
  ObsFold::init(f);
  for (int i = threadIdx.x; i < nrec; i += kBlock) {   // k_observe_fold_parts' order
    const double *r = parts + (int64_t)i * VSIQ_PART_LEN;
    const double rr[6] = {r[0], r[1], r[2], r[3], r[4], r[5]};
    ObsFold::add(f, rr);
  }
  ObsFold::wave(f);
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) s_f[w][k] = f[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kWaves; ++i) {
      const double rr[6] = {s_f[i][0], s_f[i][1], s_f[i][2], s_f[i][3], s_f[i][4], s_f[i][5]};
      ObsFold::add(f, rr);
    }
    float state[2] = {0.f, 0.f};
    if (run_minmax) { state[0] = run_minmax[0]; state[1] = run_minmax[1]; }
    const bool lead = blockIdx.x == 0;
    observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax ? state : nullptr, lead ? qp_out : nullptr,
                    sym, qden, eps, &s_qp[0], &s_qp[1]);
    if (lead) {
      if (run_minmax) { run_minmax[0] = state[0]; run_minmax[1] = state[1]; }
      if (stats_out) write_stats(stats_out, f, n);
    }
  }
  __syncthreads();
  QP p;
  p.s = (float)s_qp[0];
  p.z = (float)s_qp[1];
  p.lo = lo;
  p.hi = hi;
  p.discrete = 0;
  p.d = make_fastdiv(p.s);
  p.fast = fq_fast_qp(p.s, p.z);
  fq_fwd_block<VEC, NT, CODES, MASK, ACT, kFlatU>(x, y, codes, mask, n, p, blockIdx.x, GateClk{0}, 0u, L);
}

template <int ACT>
void launch_fold_fq_act(bool vec, bool nt, const float *x, float *y, uint8_t *c, uint64_t *m, int64_t n,
                        double *parts, double *st, float *run, double *qp, int sym, double qden, double eps,
                        float lo, float hi, const SiluLay &L, hipStream_t s) {
  const int64_t pgrid = fold_fq_part_grid(n);
  launch_observe_part_u<ACT, kFoldFqU>(vec, nt, x, n, parts, pgrid, L, s);
  const int nrec = (int)(pgrid * kWaves);
  const dim3 grid((unsigned)oneshot_grid(cdiv(n, 4)));
#define K9(V, T, C, M)                                                                                       \
  hipLaunchKernelGGL((k_fold_fq_fwd<V, T, C, M, ACT>), grid, dim3(kBlock), 0, s, x, y, c, m, n, parts, nrec, st, \
                     run, qp, sym, qden, eps, lo, hi, L)
#define K9CM(V, T)                  \
  if (c && m) { K9(V, T, true, true); }        \
  else if (c) { K9(V, T, true, false); }       \
  else if (m) { K9(V, T, false, true); }       \
  else { K9(V, T, false, false); }
  if (vec && nt) { K9CM(true, true) }
  else if (vec) { K9CM(true, false) }
  else { K9CM(false, false) }
#undef K9CM
#undef K9
}

// ----------------------------------------------------------------------------
// K10: K9 in ONE launch.  The grid is K2p's (fold_fq_part_grid(n) <= 32 workgroups,
// kFoldFqU groups per lane per step, <= 2 steps up to kFoldFqMax), so every workgroup
// holds its share of act(x) in registers (<= 8 groups per lane), accumulates it in
// k_observe_part's order and stores its per-wave records write-through -- the same bits
// as K9's K2p launch.  A grid barrier on two counter words replaces the kernel
// boundary: arrive, spin (s_sleep) until every workgroup has arrived, fold all records
// in K9's fixed order, derive the running update + f64 qparams (minmax.py:42-74) and
// quantize from registers (uniform.py:55,95).  The running state is read BEFORE the
// arrival, so workgroup 0's write after the barrier cannot race a reader; the last
// workgroup to leave resets both words (stream-ordered reuse).  The grid is tiny
// (<= 32 workgroups of 256 lanes on 256 CUs): co-resident with room to spare; a
// workgroup that waits longer than kGridBarTimeout (42 ms) stops waiting, counts the
// event in counter word kGridBarErrors and writes NaN, so no wave can spin forever.
// ----------------------------------------------------------------------------
constexpr int kGridBarArrive = 1 + kArriveGroups;   // counter words (after arrive_last's 0..32)
constexpr int kGridBarDepart = 2 + kArriveGroups;
constexpr int kGridBarErrors = 3 + kArriveGroups;
static_assert(kGridBarErrors < VSIQ_COUNTER_WORDS, "counter words");
static_assert(kGridBarErrors == VSIQ_COUNTER_GRID_ERRORS, "include/vsiq.h names this word");
constexpr uint64_t kGridBarTimeout = 1ull << 22;    // wall-clock ticks (100 MHz)

template <bool VEC, bool NT, bool CODES, bool MASK, int ACT, int S>
__global__ __launch_bounds__(kBlock) void k_observe_fq_grid(
    const float *__restrict__ x, float *__restrict__ y, uint8_t *__restrict__ codes,
    uint64_t *__restrict__ mask, int64_t n, double *__restrict__ parts, uint32_t *__restrict__ counter,
    double *__restrict__ stats_out, float *__restrict__ run_minmax, double *__restrict__ qp_out, int sym,
    double qden, double eps, float lo, float hi, SiluLay L) {
  constexpr int U = kFoldFqU;
  __shared__ double s_f[kWaves][6];
  __shared__ double s_qp[2];
  __shared__ int s_ok;
  const int64_t ng = cdiv(n, 4);
  const int64_t nfull = n / 4;
  const int64_t step = (int64_t)gridDim.x * kBlock * U;
  const int64_t b0 = (int64_t)blockIdx.x * kBlock * U;
  const int64_t base = b0 + threadIdx.x;
  const int lane = threadIdx.x % kWave, w = threadIdx.x / kWave;
  float state[2] = {0.f, 0.f};
  if (run_minmax && threadIdx.x == 0) { state[0] = run_minmax[0]; state[1] = run_minmax[1]; }
  f4 v[S * U];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int k = 0; k < U; ++k) v[s * U + k] = load_group_c<VEC, NT>(x, base + s * step + k * kBlock, ng, n);
  ObsAcc a;
  obs_init(a);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (b0 + s * step >= ng) break;   // block-uniform: observe_stride_b's loop condition
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = base + s * step + k * kBlock;
      v[s * U + k] = act_fwd4_at<ACT>(v[s * U + k], 4 * i, L);
      if (i < nfull) obs_add4(a, v[s * U + k], 4);
      else if (i < ng) obs_add4(a, v[s * U + k], valid_in_group(i, n));
    }
  }
  // store_part_record's reductions, the record stored write-through and drained
  a.mn = wave_reduce(a.mn, MinOp());
  a.mx = wave_reduce(a.mx, MaxOp());
  a.nan = wave_reduce(a.nan, AddU());
  a.sa = wave_reduce(a.sa, AddD());
  a.s1 = wave_reduce(a.s1, AddD());
  a.s2 = wave_reduce(a.s2, AddD());
  if (lane < 6) {   // the reduced fields are wave-uniform: lane k stores field k (one 48-B write)
    double *r = parts + ((int64_t)blockIdx.x * kWaves + w) * VSIQ_PART_LEN;
    const double fv = lane == 0 ? (double)a.mn : lane == 1 ? (double)a.mx : lane == 2 ? (double)a.nan
                    : lane == 3 ? a.sa : lane == 4 ? a.s1 : a.s2;
    partial_store(r + lane, fv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // grid barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(counter + kGridBarArrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    int ok = 1;
    while (__hip_atomic_load(counter + kGridBarArrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
      if (wall_clock64() - t0 > kGridBarTimeout) {
        ok = 0;
        __hip_atomic_fetch_add(counter + kGridBarErrors, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_ok = ok;
  }
  __syncthreads();
  // k_fold_fq_fwd's fold (k_observe_fold_parts' order): the same bits in every workgroup
  const int nrec = (int)gridDim.x * kWaves;
  double f[6];
  ObsFold::init(f);
  for (int i = threadIdx.x; i < nrec; i += kBlock) {
    const double *r = parts + (int64_t)i * VSIQ_PART_LEN;
    const double rr[6] = {partial_load(r + 0), partial_load(r + 1), partial_load(r + 2),
                          partial_load(r + 3), partial_load(r + 4), partial_load(r + 5)};
    ObsFold::add(f, rr);
  }
  ObsFold::wave(f);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) s_f[w][k] = f[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kWaves; ++i) {
      const double rr[6] = {s_f[i][0], s_f[i][1], s_f[i][2], s_f[i][3], s_f[i][4], s_f[i][5]};
      ObsFold::add(f, rr);
    }
    const bool lead = blockIdx.x == 0;
    observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax ? state : nullptr, lead ? qp_out : nullptr,
                    sym, qden, eps, &s_qp[0], &s_qp[1]);
    if (lead) {
      if (run_minmax) { run_minmax[0] = state[0]; run_minmax[1] = state[1]; }
      if (stats_out) write_stats(stats_out, f, n);
    }
    // leave the barrier; the last workgroup out resets it for the next launch
    if (__hip_atomic_fetch_add(counter + kGridBarDepart, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        gridDim.x - 1) {
      __hip_atomic_store(counter + kGridBarArrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(counter + kGridBarDepart, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  QP p;
  p.s = s_ok ? (float)s_qp[0] : __builtin_nanf("");
  p.z = (float)s_qp[1];
  p.lo = lo;
  p.hi = hi;
  p.discrete = 0;
  p.d = make_fastdiv(p.s);
  p.fast = fq_fast_qp(p.s, p.z);
  GroupOut go[S * U];
  uint32_t mlo = 0, mhi = 0;
#pragma unroll
  for (int sl = 0; sl < S * U; ++sl) {
    go[sl] = fq_out_flat<VEC, CODES, MASK>(v[sl], p, base + (sl / U) * step + (sl % U) * kBlock, n);
    if (MASK) mask_put(mlo, mhi, sl, go[sl].b);
  }
#pragma unroll
  for (int sl = 0; sl < S * U; ++sl) {   // group indices increase with sl
    const int64_t i = base + (sl / U) * step + (sl % U) * kBlock;
    if (i - lane >= ng) break;   // whole wave past the end (uniform)
    fq_store_out<VEC, NT, CODES>(y, codes, i, ng, n, go[sl]);
  }
  if (MASK && lane < 4 * S * U) {   // lane 4 sl + j: word j of slot sl's chunk
    const int sl = lane >> 2;
    const int64_t first = base - lane + (sl / U) * step + (sl % U) * kBlock;
    if (first < ng) mask[4 * (first / kWave) + (lane & 3)] = ((uint64_t)mhi << 32) | mlo;
  }
}

inline int observe_fq_grid_steps(int64_t n) {
  return cdiv(cdiv(n, 4), fold_fq_part_grid(n) * kBlock * kFoldFqU) <= 1 ? 1 : 2;
}

template <int ACT>
void launch_observe_fq_grid_act(bool vec, bool nt, const float *x, float *y, uint8_t *c, uint64_t *m, int64_t n,
                                double *parts, uint32_t *counter, double *st, float *run, double *qp, int sym,
                                double qden, double eps, float lo, float hi, const SiluLay &L, hipStream_t s) {
  const dim3 grid((unsigned)fold_fq_part_grid(n));
  const int steps = observe_fq_grid_steps(n);
#define K10(V, T, C, M, S_)                                                                                      \
  hipLaunchKernelGGL((k_observe_fq_grid<V, T, C, M, ACT, S_>), grid, dim3(kBlock), 0, s, x, y, c, m, n, parts, \
                     counter, st, run, qp, sym, qden, eps, lo, hi, L)
#define K10S(V, T, C, M)                \
  if (steps == 1) { K10(V, T, C, M, 1); } \
  else { K10(V, T, C, M, 2); }
#define K10CM(V, T)                             \
  if (c && m) { K10S(V, T, true, true) }        \
  else if (c) { K10S(V, T, true, false) }       \
  else if (m) { K10S(V, T, false, true) }       \
  else { K10S(V, T, false, false) }
  if (vec && nt) { K10CM(true, true) }
  else if (vec) { K10CM(true, false) }
  else { K10CM(false, false) }
#undef K10CM
#undef K10S
#undef K10
}

// ----------------------------------------------------------------------------
// K1r: the per-call multi-GPU observer exchange's fold + fake quant in ONE launch.  The
// ranks' stats records (one K2 pass over each rank's shard, then one all_gather, rank
// order) are folded by EVERY workgroup in rank order -- min / max exact, counts and sums
// in float64, the same bits on every rank and in every workgroup -- into the running
// update and the f64 qparams (minmax.py:42-74), and the workgroup quantizes its share
// (uniform.py:55,95).  K9's idempotent-update trick: workgroup 0 alone writes the
// running state, the qparams record and the batch's stats record; a workgroup that reads
// the state after that recomputes the same qparams.  Replaces k_observe_finalize_ranks
// + K1 (two launches, the qparams through memory) of the round-2 exchange.
// ----------------------------------------------------------------------------
template <bool VEC, bool NT, bool CODES, bool MASK, int ACT>
__global__ __launch_bounds__(kBlock) void k_ranks_fq_fwd(
    const float *__restrict__ x, float *__restrict__ y, uint8_t *__restrict__ codes,
    uint64_t *__restrict__ mask, int64_t n, const double *__restrict__ gathered, int world,
    double *__restrict__ stats_out, float *__restrict__ run_minmax, double *__restrict__ qp_out, int sym,
    double qden, double eps, float lo, float hi, SiluLay L) {
  __shared__ double s_qp[2];
  if (threadIdx.x == 0) {
    double f[6] = {__builtin_inf(), -__builtin_inf(), 0.0, 0.0, 0.0, 0.0};
    double nn = 0.0;
    for (int r = 0; r < world; ++r) {   // rank order (k_observe_finalize_ranks' fold)
      const double *g = gathered + (int64_t)r * VSIQ_ST_LEN;
      f[0] = __builtin_fmin(f[0], g[VSIQ_ST_MIN]);
      f[1] = __builtin_fmax(f[1], g[VSIQ_ST_MAX]);
      f[2] += g[VSIQ_ST_NAN];
      f[3] += g[VSIQ_ST_SUMABS];
      f[4] += g[VSIQ_ST_SUM];
      f[5] += g[VSIQ_ST_SUMSQ];
      nn += g[VSIQ_ST_N];
    }
    float state[2] = {0.f, 0.f};
    if (run_minmax) { state[0] = run_minmax[0]; state[1] = run_minmax[1]; }
    const bool lead = blockIdx.x == 0;
    observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax ? state : nullptr, lead ? qp_out : nullptr,
                    sym, qden, eps, &s_qp[0], &s_qp[1]);
    if (lead) {
      if (run_minmax) { run_minmax[0] = state[0]; run_minmax[1] = state[1]; }
      if (stats_out) write_stats(stats_out, f, (int64_t)nn);
    }
  }
  __syncthreads();
  QP p;
  p.s = (float)s_qp[0];
  p.z = (float)s_qp[1];
  p.lo = lo;
  p.hi = hi;
  p.discrete = 0;
  p.d = make_fastdiv(p.s);
  p.fast = fq_fast_qp(p.s, p.z);
  fq_fwd_block<VEC, NT, CODES, MASK, ACT, kFlatU>(x, y, codes, mask, n, p, blockIdx.x, GateClk{0}, 0u, L);
}

template <int ACT>
void launch_ranks_fq_act(bool vec, bool nt, const float *x, float *y, uint8_t *c, uint64_t *m, int64_t n,
                         const double *gathered, int world, double *st, float *run, double *qp, int sym,
                         double qden, double eps, float lo, float hi, const SiluLay &L, hipStream_t s) {
  const dim3 grid((unsigned)oneshot_grid(cdiv(n, 4)));
#define K1R(V, T, C, M)                                                                                    \
  hipLaunchKernelGGL((k_ranks_fq_fwd<V, T, C, M, ACT>), grid, dim3(kBlock), 0, s, x, y, c, m, n, gathered, \
                     world, st, run, qp, sym, qden, eps, lo, hi, L)
#define K1RCM(V, T)                             \
  if (c && m) { K1R(V, T, true, true); }        \
  else if (c) { K1R(V, T, true, false); }       \
  else if (m) { K1R(V, T, false, true); }       \
  else { K1R(V, T, false, false); }
  if (vec && nt) { K1RCM(true, true) }
  else if (vec) { K1RCM(true, false) }
  else { K1RCM(false, false) }
#undef K1RCM
#undef K1R
}

template <int ACT>
void launch_observe_fq_small_act(bool vec, bool nt, const float *x, float *y, uint8_t *c, uint64_t *m, int64_t n,
                                 double *st, float *run, double *qp, int sym, double qden, double eps, float lo,
                                 float hi, const SiluLay &L, hipStream_t s) {
  if (vec && nt) launch_observe_fq_small<true, true, ACT>(x, y, c, m, n, st, run, qp, sym, qden, eps, lo, hi, L, s);
  else if (vec) launch_observe_fq_small<true, false, ACT>(x, y, c, m, n, st, run, qp, sym, qden, eps, lo, hi, L, s);
  else launch_observe_fq_small<false, false, ACT>(x, y, c, m, n, st, run, qp, sym, qden, eps, lo, hi, L, s);
}

// ----------------------------------------------------------------------------
// K2m: many deferred observer calls (K2p) in ONE launch.  Block b of the launch runs
// block b - blk0[t] of tensor t's own K2p grid (same grid, groups per lane and body as
// vsiq_act_observe_part_f32 for that n), so every tensor's records are bit-identical
// to its single-tensor K2p launch; only the ~3 us launch floor and the grid tail are
// paid once per batch instead of once per layer (C5: 27 layers per calibration batch).
// ----------------------------------------------------------------------------
constexpr int kPartMulti = 32;   // tensors per launch (descriptor table in the kernel arguments)

struct PTensor {
  const float *x;
  double *parts;
  int64_t n;
  uint32_t grid;
  int u;      // groups per lane per step (observe_part_u)
  int vec;
};

struct PBatch {
  PTensor t[kPartMulti];
  uint32_t blk0[kPartMulti + 1];
  int count;
  SiluRef sref;   // SiLU: the reference CPU layout (each tensor's chunks from its own n)
};

// ALLVEC: every tensor of the batch takes the 16-byte path (the usual case: activation
// tensors of n % 4 == 0), so the scalar-path variants, which set the register budget
// of the generic kernel (152 VGPRs: 3 waves per SIMD), are not compiled in.
template <bool NT, int ACT, bool ALLVEC>
__global__ __launch_bounds__(kBlock) void k_observe_part_multi(const PBatch b) {
  int t = 0;
  const uint32_t blk = blockIdx.x;
  while (t + 1 < b.count && blk >= b.blk0[t + 1]) ++t;   // scalar: blk0 is a kernel argument
  const PTensor &T = b.t[t];
  const int64_t lb = (int64_t)blk - b.blk0[t], nb = T.grid;
  SiluLay L{};
  if constexpr (ACT == kActSilu) L = silu_lay(T.n, b.sref);
  ObsAcc a;
  if (ALLVEC || T.vec) {
    if (T.u == 8) observe_stride_b<true, NT, ACT, 8>(T.x, T.n, a, lb, nb, L);
    else if (T.u == 4) observe_stride_b<true, NT, ACT, 4>(T.x, T.n, a, lb, nb, L);
    else observe_stride_b<true, NT, ACT, 2>(T.x, T.n, a, lb, nb, L);
  } else {
    if (T.u == 8) observe_stride_b<false, false, ACT, 8>(T.x, T.n, a, lb, nb, L);
    else if (T.u == 4) observe_stride_b<false, false, ACT, 4>(T.x, T.n, a, lb, nb, L);
    else observe_stride_b<false, false, ACT, 2>(T.x, T.n, a, lb, nb, L);
  }
  store_part_record(a, T.parts, lb, nb, T.n);
}

// Fold of deferred K2p records: workgroup c folds call c's records (call_stride doubles
// apart; the count is the grid stored in every record) in a fixed order -> its stats
// record (VSIQ_ST_LEN).  Deterministic; min/max exact, sums in float64.
__global__ __launch_bounds__(kBlock) void k_observe_fold_parts(const double *__restrict__ parts,
                                                               int64_t call_stride,
                                                               double *__restrict__ stats_out) {
  const double *P = parts + (int64_t)blockIdx.x * call_stride;
  const int64_t maxrec = call_stride / VSIQ_PART_LEN;
  const double dg = P[7], dn = P[6];
  // a slot that was never written (or garbage) folds nothing instead of reading out of range
  const int64_t nrec = (dg >= 1.0 && dg <= (double)maxrec) ? (int64_t)dg : 0;
  double f[6];
  ObsFold::init(f);
  // thread t folds records t, t + 256, t + 512, ... in that order; kFoldU of them are loaded
  // at once (a one-shot K2o call has up to n / 2048 records: one load round trip per
  // record would make the sync latency-bound)
  constexpr int kFoldU = 8;
  for (int64_t i0 = threadIdx.x; i0 < nrec; i0 += (int64_t)kBlock * kFoldU) {
    double rr[kFoldU][6];
#pragma unroll
    for (int u = 0; u < kFoldU; ++u) {
      const int64_t i = i0 + (int64_t)u * kBlock;
      const double *r = P + (i < nrec ? i : nrec - 1) * VSIQ_PART_LEN;
#pragma unroll
      for (int k = 0; k < 6; ++k) rr[u][k] = r[k];
    }
#pragma unroll
    for (int u = 0; u < kFoldU; ++u)
      if (i0 + (int64_t)u * kBlock < nrec) ObsFold::add(f, rr[u]);
  }
  ObsFold::wave(f);
  __shared__ double s[kWaves][6];
  const int w = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) s[w][k] = f[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kWaves; ++i) {
      const double rr[6] = {s[i][0], s[i][1], s[i][2], s[i][3], s[i][4], s[i][5]};
      ObsFold::add(f, rr);
    }
    write_stats(stats_out + (int64_t)blockIdx.x * VSIQ_ST_LEN, f, nrec ? (int64_t)dn : 0);
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

// Per-call multi-GPU observer exchange, the fold side: `world` stats records gathered
// from the ranks (all_gather, rank order) -> the whole batch's record (min / max exact,
// counts and sums in float64 in rank order: the same bits on every rank) -> fp32 means /
// std (qm.py:66-68) -> running update + f64 qparams (minmax.py:42-74).  One launch
// instead of two all-reduces plus the host-side finish of round 1.
__global__ void k_observe_finalize_ranks(const double *__restrict__ gathered, int world,
                                         double *__restrict__ stats_out, float *__restrict__ run_minmax,
                                         double *__restrict__ qp_out, int sym, double qden, double eps) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double f[6] = {__builtin_inf(), -__builtin_inf(), 0.0, 0.0, 0.0, 0.0};
  double n = 0.0;
  for (int r = 0; r < world; ++r) {
    const double *g = gathered + (int64_t)r * VSIQ_ST_LEN;
    f[0] = __builtin_fmin(f[0], g[VSIQ_ST_MIN]);
    f[1] = __builtin_fmax(f[1], g[VSIQ_ST_MAX]);
    f[2] += g[VSIQ_ST_NAN];
    f[3] += g[VSIQ_ST_SUMABS];
    f[4] += g[VSIQ_ST_SUM];
    f[5] += g[VSIQ_ST_SUMSQ];
    n += g[VSIQ_ST_N];
  }
  if (stats_out) write_stats(stats_out, f, (int64_t)n);
  observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax, qp_out, sym, qden, eps);
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


// exhaustive check of the no-check fast paths, every 32-bit input pattern:
//   mode 0: quantizer code c = clamp(rint(x/s + zp)) (value, sign, STE mask bit)
//           of fq_elem_fast vs the IEEE element, for x with fq_x_ok(x), per
//           (scales[k], zps[k]) inside fq_fast_qp;
//   mode 1: STE quotient ste_quot(g) vs RN(RN(g*s)/s), for g with ste_ok(g).
// counts[2k] = mismatches, counts[2k+1] = inputs checked (0 if the qparams are
// outside the fast domain).
__global__ __launch_bounds__(kBlock) void k_selftest_fq(int mode, const float *__restrict__ ss,
                                                        const float *__restrict__ zs, int nk, float lo,
                                                        float hi, unsigned long long *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (int k = 0; k < nk; ++k) {
    QP p;
    p.s = ss[k];
    p.z = mode == 0 ? zs[k] : 0.f;
    p.lo = lo;
    p.hi = hi;
    p.discrete = 1;
    p.d = make_fastdiv(p.s);
    p.fast = fq_fast_qp(p.s, p.z);
    const SteDiv sd = make_stediv(p.s);
    const bool dom = mode == 0 ? p.fast != 0 : sd.fast != 0;
    uint32_t bad = 0, seen = 0;
    if (dom) {
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x = __uint_as_float((uint32_t)i);
        if (mode == 0) {
          if (!fq_x_ok(x)) continue;
          const Elem f = fq_elem_fast(x, p), w = fq_elem<true>(x, p);
          bad += (__float_as_uint(f.y) != __float_as_uint(w.y) || f.m != w.m) ? 1u : 0u;
        } else {
          if (!ste_ok(x)) continue;
          const float f = ste_quot(x, sd), w = ste_ieee(x, true, sd);
          bad += (__float_as_uint(f) != __float_as_uint(w) && !(f != f && w != w)) ? 1u : 0u;
        }
        ++seen;
      }
    }
    bad = wave_reduce(bad, AddU());
    seen = wave_reduce(seen, AddU());
    if (threadIdx.x % kWave == 0) {
      if (bad) atomicAdd(out + 2 * k, (unsigned long long)bad);
      if (seen) atomicAdd(out + 2 * k + 1, (unsigned long long)seen);
    }
  }
}

template <int ACT, bool VEC, bool NT, int G>
void launch_observe_g(const float *x, int64_t n, double *stats_out, float *run_minmax, double *qp_out,
                      int sym, double qden, double eps, double *ws, uint32_t *counter, int64_t grid,
                      const SiluLay &L, hipStream_t st) {
  hipLaunchKernelGGL((k_observe<VEC, NT, ACT, G>), dim3((unsigned)grid), dim3(kBlock), 0, st, x, n,
                     stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter, L);
}

template <int ACT, bool VEC, bool NT>
void launch_observe_loop(const float *x, int64_t n, double *stats_out, float *run_minmax, double *qp_out,
                         int sym, double qden, double eps, double *ws, uint32_t *counter, int64_t grid,
                         const SiluLay &L, hipStream_t st) {
  hipLaunchKernelGGL((k_observe_loop<VEC, NT, ACT, kObsU>), dim3((unsigned)grid), dim3(kBlock), 0, st, x,
                     n, stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter, L);
}

// K2 grid: grid-stride kernel (default) or the one-shot kernel (VSIQ_TUNE_OBS_KERNEL 1)
// Tensors of at most kObsSingle groups (8K elements: one load round per lane) take ONE
// workgroup and skip the record / arrival / fold chain.  (At 64K elements a single
// workgroup's 8 serial load rounds cost more than the chain: 12.5 vs 6.8 us, MI355X.)
constexpr int64_t kObsSingle = (int64_t)kBlock * kObsU;
// K2 (per-call observer) reads tensors under this many MB with cached loads: the fake
// quant re-reading it right after may hit the 256 MB Infinity Cache
constexpr int64_t kObsTemporalMB = 256;

// one-shot K2 has 2 / 4 / 16 groups-per-lane instances: K4's 8 runs as 4
inline int obs_groups_per_lane(int64_t ng) {
  const int p = lsq_groups_per_lane(ng);
  return p == 8 ? 4 : p;
}

inline int64_t observe_grid(int64_t ng) {
  if (g_tune.obs_kernel == 1) return lsq_grid(ng, obs_groups_per_lane(ng));
  if (ng <= kObsSingle) return 1;
  return std::min<int64_t>(kObsGrid, std::max<int64_t>(1, cdiv(ng, (int64_t)kBlock * kObsU)));
}

template <int ACT>
void launch_observe(bool vec, bool nt, const float *x, int64_t n, double *stats_out, float *run_minmax,
                    double *qp_out, int sym, double qden, double eps, double *ws, uint32_t *counter,
                    const SiluLay &L, hipStream_t st) {
  const int64_t ng = cdiv(n, 4);
  const int64_t grid = observe_grid(ng);
  if (g_tune.obs_kernel != 1) {
    if (vec && nt) launch_observe_loop<ACT, true, true>(x, n, stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter, grid, L, st);
    else if (vec) launch_observe_loop<ACT, true, false>(x, n, stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter, grid, L, st);
    else launch_observe_loop<ACT, false, false>(x, n, stats_out, run_minmax, qp_out, sym, qden, eps, ws, counter, grid, L, st);
    return;
  }
  // one-shot: K4's groups-per-lane rule (8 -> 4) and grid
  const int per_lane = obs_groups_per_lane(ng);
#define VSIQ_OBS(V, N)                                                                              \
  (per_lane == kLsqGroups                                                                           \
       ? launch_observe_g<ACT, V, N, kLsqGroups>(x, n, stats_out, run_minmax, qp_out, sym, qden, eps, \
                                                 ws, counter, grid, L, st)                          \
   : per_lane == 4 ? launch_observe_g<ACT, V, N, 4>(x, n, stats_out, run_minmax, qp_out, sym, qden,  \
                                                    eps, ws, counter, grid, L, st)                  \
                   : launch_observe_g<ACT, V, N, 2>(x, n, stats_out, run_minmax, qp_out, sym, qden,  \
                                                    eps, ws, counter, grid, L, st))
  if (vec && nt) VSIQ_OBS(true, true);
  else if (vec) VSIQ_OBS(true, false);
  else VSIQ_OBS(false, false);
#undef VSIQ_OBS
}

int observe(const float *x, int64_t n, int act, double *stats_out, float *run_minmax, double *qp_out,
            int symmetric, double qden, double eps, double *ws, int64_t ws_len, uint32_t *counter,
            void *stream) {
  if (n <= 0 || !x || !ws || !counter || !act_ok(act)) return VSIQ_E_ARG;
  const bool vec = aligned16(x) && n % 4 == 0;
  const int64_t grid = observe_grid(cdiv(n, 4));
  if (grid > 0x7fffffffLL) return VSIQ_E_ARG;
  if (ws_len < fold_records(grid) * kPartials) return VSIQ_E_WS;
  // kObsTemporalMB: observe + quantize (K2 -> K1) may re-read x from the Infinity Cache
  const bool nt = g_tune.nontemporal != 0 && !((n * 4) >> 20 < kObsTemporalMB);
  VSIQ_ACT(act, launch_observe, vec, nt, x, n, stats_out, run_minmax, qp_out,
           symmetric, qden, eps, ws, counter, act_lay(act, n), (hipStream_t)stream);
  return launch_rc();
}

// K2p groups per lane per step: 8 while the grid reaches 512 workgroups, else fewer so
// that small layers still spread over >= ~512 workgroups (all CUs issuing; a 1.6M-
// element layer at 8 per lane was 200 workgroups).  Fixed per n: deterministic.
inline int observe_part_u(int64_t n) {
  const int64_t units = cdiv(cdiv(n, 4), (int64_t)kBlock);   // lanes' worth of groups
  return units >= 512 * 8 ? 8 : (units >= 512 * 4 ? 4 : 2);
}

// K2p grid (fixed per n), at most VSIQ_PART_MAX_RECORDS / kWaves workgroups (a record per wave)
inline int64_t observe_part_grid(int64_t n) {
  const int64_t units = cdiv(cdiv(n, 4), (int64_t)kBlock);
  const int u = observe_part_u(n);
  // large tensors: kObsGrid workgroups striding over the tensor; small: one step each
  static_assert(kObsGrid <= VSIQ_PART_MAX_RECORDS / kWaves, "K2p records");
  const int64_t cap = u == 8 ? kObsGrid : VSIQ_PART_MAX_RECORDS / kWaves;
  return std::min<int64_t>(cap, std::max<int64_t>(1, cdiv(units, u)));
}

template <int ACT, int U>
void launch_observe_part_u(bool vec, bool nt, const float *x, int64_t n, double *parts, int64_t grid,
                           const SiluLay &L, hipStream_t st) {
  if (vec && nt)
    hipLaunchKernelGGL((k_observe_part<true, true, ACT, U>), dim3((unsigned)grid), dim3(kBlock), 0, st, x, n, parts, L);
  else if (vec)
    hipLaunchKernelGGL((k_observe_part<true, false, ACT, U>), dim3((unsigned)grid), dim3(kBlock), 0, st, x, n, parts, L);
  else
    hipLaunchKernelGGL((k_observe_part<false, false, ACT, U>), dim3((unsigned)grid), dim3(kBlock), 0, st, x, n, parts, L);
}

template <int ACT>
void launch_observe_part(bool vec, bool nt, const float *x, int64_t n, double *parts, int64_t grid,
                         const SiluLay &L, hipStream_t st) {
  const int u = observe_part_u(n);
  if (u == 8) launch_observe_part_u<ACT, 8>(vec, nt, x, n, parts, grid, L, st);
  else if (u == 4) launch_observe_part_u<ACT, 4>(vec, nt, x, n, parts, grid, L, st);
  else launch_observe_part_u<ACT, 2>(vec, nt, x, n, parts, grid, L, st);
}

// CU count of the current device (cached; 256 on MI355X)
int occupancy_blocks(const void *kernel, int block) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, block, 0) != hipSuccess) return 0;
  return n;
}

// per-device attribute caches: relaxed atomics (any thread may fill them; the value
// is the same whoever wins)
int device_wall_clock_khz() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 100000;
  return device_wall_clock_khz(dev);
}

int device_wall_clock_khz(int dev) {
  static std::atomic<int> khz[64];
  if (dev < 0 || dev >= 64) return 100000;
  if (!khz[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) != hipSuccess || v <= 0) v = 100000;
    khz[dev] = v;
  }
  return khz[dev];
}

int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  return device_cus(dev);
}

int device_cus(int dev) {
  static std::atomic<int> cus[64];
  if (dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cus[dev] = v;
  }
  return cus[dev];
}

}  // namespace vsiq

using namespace vsiq;

// K2o one-shot shape: G groups per lane (k2o_groups knob, default 2) and BS lanes per
// workgroup (k2o_block knob, default kK2oBlock); fixed per n and knobs: deterministic
inline int k2o_groups() {
  const int t = g_tune.k2o_groups;
  return t ? t : kK2oGroups;
}

inline int k2o_block() {
  const int t = g_tune.k2o_block;
  return t ? t : kK2oBlock;
}

inline int64_t k2o_records(int64_t n) {
  if (g_tune.k2o_form == 1) return observe_part_grid(n) * kWaves;
  return cdiv(cdiv(n, 4), (int64_t)k2o_block() * k2o_groups());
}

template <bool VEC, bool NT, int ACT, int BS>
void launch_k2o1_bs(int g, int64_t grid, const float *c, float *y, int64_t n, double *parts, const SiluLay &L,
                    hipStream_t st) {
#define K2O1(G_) hipLaunchKernelGGL((k_observe_part_out1<VEC, NT, ACT, G_, BS>), dim3((unsigned)grid), dim3(BS), 0, \
                                    st, c, y, n, parts, L, 0u)
  switch (g) {
    case 1: K2O1(1); break;
    case 2: K2O1(2); break;
    case 4: K2O1(4); break;
    case 8: K2O1(8); break;
    default: K2O1(16); break;
  }
#undef K2O1
}

template <bool VEC, bool NT, int ACT>
void launch_k2o1(int g, int bs, int64_t grid, const float *c, float *y, int64_t n, double *parts, const SiluLay &L,
                 hipStream_t st) {
  if (bs == 1024) launch_k2o1_bs<VEC, NT, ACT, 1024>(g, grid, c, y, n, parts, L, st);
  else if (bs == 512) launch_k2o1_bs<VEC, NT, ACT, 512>(g, grid, c, y, n, parts, L, st);
  else launch_k2o1_bs<VEC, NT, ACT, 256>(g, grid, c, y, n, parts, L, st);
}

template <int ACT>
void launch_k2o1_act(bool vec, bool nt, int g, int bs, int64_t grid, const float *c, float *y, int64_t n,
                     double *parts, const SiluLay &L, hipStream_t st) {
  if (vec && nt) launch_k2o1<true, true, ACT>(g, bs, grid, c, y, n, parts, L, st);
  else if (vec) launch_k2o1<true, false, ACT>(g, bs, grid, c, y, n, parts, L, st);
  else launch_k2o1<false, false, ACT>(g, bs, grid, c, y, n, parts, L, st);
}

// K2o's one-round forms (round 5): where 9 groups per lane of 256 lanes make a grid of
// 2..occ workgroups per CU (every workgroup resident at once; on MI355X 4.7M..18.9M
// elements -- C5's 6.6M / 13M layers), one pass of loads, the record, the store gate
// (tuned online per site like K1's, gate_tune.hip), then the stores: reads and writes as
// two phases instead of interleaved.  Smaller calls whose default 2-groups-per-lane grid
// is one round (C5's 1.6M / 3.3M layers) get the gate on that grid.  The form is chosen
// by the shape alone (not by the gate), so a call's records are fixed per n; the gate
// is only a delay.  Records: one per workgroup, never more than the G = 2 form's that
// size the slot (k2o_records).
template <int ACT, bool VEC, bool NT, int G>
bool launch_k2o_gated_g(const float *c, float *y, int64_t n, double *parts, const SiluLay &L, hipStream_t st) {
  constexpr int kBS = 256;
  const int64_t ng = cdiv(n, 4);
  const int64_t grid = cdiv(ng, (int64_t)kBS * G);
  const void *kern = reinterpret_cast<const void *>(k_observe_part_out1<VEC, NT, ACT, G, kBS>);
  static const int occ = occupancy_blocks(kern, kBS);
  const int64_t cus = device_cus();
  if (grid < 2 * cus || grid > (int64_t)occ * cus || grid * kBS * G - ng > ng / 8) return false;
  GateSel gs = store_gate_select("k2o_observe_out", kern, grid, occ, 4 * n, st);
  hipLaunchKernelGGL((k_observe_part_out1<VEC, NT, ACT, G, kBS>), dim3((unsigned)grid), dim3(kBS), 0, st, c, y, n,
                     parts, L, gs.gate);
  store_gate_launched(gs, st);
  return true;
}

template <int ACT, bool VEC, bool NT>
bool launch_k2o_gated_vn(const float *c, float *y, int64_t n, double *parts, const SiluLay &L, hipStream_t st) {
  static_assert(kK2oGroups == 2 && kK2oBlock == 256, "the G = 2 gated form is the default grid");
  // (a 16-groups form is not one round at 26M: 5 workgroups per CU by its registers)
  return launch_k2o_gated_g<ACT, VEC, NT, 2>(c, y, n, parts, L, st) ||
         launch_k2o_gated_g<ACT, VEC, NT, 9>(c, y, n, parts, L, st);
}

template <int ACT>
bool launch_k2o_gated(bool vec, bool nt, const float *c, float *y, int64_t n, double *parts, const SiluLay &L,
                      hipStream_t st) {
  if (vec && nt) return launch_k2o_gated_vn<ACT, true, true>(c, y, n, parts, L, st);
  if (vec) return launch_k2o_gated_vn<ACT, true, false>(c, y, n, parts, L, st);
  return launch_k2o_gated_vn<ACT, false, false>(c, y, n, parts, L, st);
}

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
  // the largest reducing grid any kernel / tuning can use for n: 2 groups per lane (K4
  // and the one-shot K2 at VSIQ_TUNE_LSQ_GROUPS 2; the one-shot K2 runs K4's 8 as 4)
  const int64_t g = std::max<int64_t>(kMaxReduceGrid, lsq_grid(cdiv(std::max<int64_t>(n, 0), 4), 2));
  return (g + kArriveGroups) * kPartials;
}

int64_t vsiq_mask_words(int64_t rows, int64_t rowlen) {
  if (rows < 0 || rowlen < 0) return VSIQ_E_ARG;
  return rows * mask_words_per_row(rowlen);
}

int vsiq_set_tuning(int key, int value) {
  switch (key) {
    case VSIQ_TUNE_NONTEMPORAL: g_tune.nontemporal = value; return 0;
    case VSIQ_TUNE_OBS_KERNEL:
      if (value < 0 || value > 2) return VSIQ_E_ARG;
      g_tune.obs_kernel = value;
      return 0;
    case VSIQ_TUNE_LSQ_GROUPS:
      if (value != 0 && value != 2 && value != 4 && value != 8 && value != 16) return VSIQ_E_ARG;
      g_tune.lsq_groups = value;
      return 0;
    case VSIQ_TUNE_STORE_DEFER:
      if (value < -1 || value > 64) return VSIQ_E_ARG;
      g_tune.store_defer = value;
      return 0;
    case VSIQ_TUNE_PC_PACKED:
      if (value < 0 || value > 2) return VSIQ_E_ARG;
      g_tune.pc_packed = value;
      return 0;
    case VSIQ_TUNE_STORE_GATE:
      if (value < -1 || value > 4000) return VSIQ_E_ARG;
      g_tune.store_gate = value;
      return 0;
    case VSIQ_TUNE_GATE_AUTOTUNE:
      if (value != 0 && value != 1) return VSIQ_E_ARG;
      g_tune.gate_autotune = value;
      return 0;
    case VSIQ_TUNE_XCD_ORDER:
      if (value < 0 || value > 2) return VSIQ_E_ARG;
      g_tune.xcd_order = value;
      return 0;
    case VSIQ_TUNE_K2O_FORM:
      if (value != 0 && value != 1) return VSIQ_E_ARG;
      g_tune.k2o_form = value;
      return 0;
    case VSIQ_TUNE_K2O_GROUPS:
      if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16) return VSIQ_E_ARG;
      g_tune.k2o_groups = value;
      return 0;
    case VSIQ_TUNE_K2O_BLOCK:
      if (value != 0 && value != 256 && value != 512 && value != 1024) return VSIQ_E_ARG;
      g_tune.k2o_block = value;
      return 0;
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

int vsiq_selftest_fq(int mode, const float *scales, const float *zero_points, int count,
                     float qmin, float qmax, unsigned long long *counts, void *stream) {
  if (mode != 0 && mode != 1) return VSIQ_E_ARG;
  if (count < 0 || (count > 0 && (!scales || !counts || (mode == 0 && !zero_points))))
    return VSIQ_E_ARG;
  if (count == 0) return 0;
  hipLaunchKernelGGL(k_selftest_fq, dim3(256 * 16), dim3(kBlock), 0, (hipStream_t)stream, mode,
                     scales, zero_points, count, qmin, qmax, counts);
  return launch_rc();
}

int vsiq_observe_f32(const float *x, int64_t n, double *stats_out, float *run_minmax,
                     double *qp_out, int symmetric, double qden, double eps, double *ws,
                     int64_t ws_len, uint32_t *counter, void *stream) {
  return observe(x, n, kActNone, stats_out, run_minmax, qp_out, symmetric, qden, eps, ws, ws_len,
                 counter, stream);
}

int vsiq_act_observe_f32(const float *c, int64_t n, int act, double *stats_out, float *run_minmax,
                         double *qp_out, int symmetric, double qden, double eps, double *ws,
                         int64_t ws_len, uint32_t *counter, void *stream) {
  if (!act_ok(act)) return VSIQ_E_ARG;
  return observe(c, n, act, stats_out, run_minmax, qp_out, symmetric, qden, eps, ws, ws_len, counter,
                 stream);
}

int64_t vsiq_observe_part_records(int64_t n) {
  if (n <= 0) return VSIQ_E_ARG;
  return observe_part_grid(n) * kWaves;
}

int vsiq_act_observe_part_f32(const float *c, int64_t n, int act, double *parts, int64_t parts_len,
                              void *stream) {
  if (n <= 0 || !c || !parts || !act_ok(act)) return VSIQ_E_ARG;
  const int64_t grid = observe_part_grid(n);
  if (parts_len < grid * kWaves * VSIQ_PART_LEN) return VSIQ_E_WS;
  const bool vec = aligned16(c) && n % 4 == 0;
  VSIQ_ACT(act, launch_observe_part, vec, g_tune.nontemporal != 0, c, n, parts, grid, act_lay(act, n),
           (hipStream_t)stream);
  return launch_rc();
}

int64_t vsiq_observe_part_out_records(int64_t n) {
  if (n <= 0) return VSIQ_E_ARG;
  return k2o_records(n);
}

int vsiq_act_observe_part_out_f32(const float *c, float *y, int64_t n, int act, double *parts, int64_t parts_len,
                                  void *stream) {
  if (n <= 0 || !c || !y || !parts || !act_ok(act)) return VSIQ_E_ARG;
  const bool vec = aligned16(c) && aligned16(y) && n % 4 == 0;
  const bool nt = g_tune.nontemporal != 0;
  const SiluLay L = act_lay(act, n);
  const hipStream_t st = (hipStream_t)stream;
  if (g_tune.k2o_form != 1) {
    const int64_t grid = k2o_records(n);
    if (grid > 0x7fffffffLL) return VSIQ_E_ARG;
    if (parts_len < grid * VSIQ_PART_LEN) return VSIQ_E_WS;
    // default shape knobs: the one-round gated form where the size allows it
    if (g_tune.k2o_groups == 0 && g_tune.k2o_block == 0 &&
        VSIQ_ACT(act, launch_k2o_gated, vec, nt, c, y, n, parts, L, st))
      return launch_rc();
    VSIQ_ACT(act, launch_k2o1_act, vec, nt, k2o_groups(), k2o_block(), grid, c, y, n, parts, L, st);
    return launch_rc();
  }
  const int64_t grid = observe_part_grid(n);
  if (parts_len < grid * kWaves * VSIQ_PART_LEN) return VSIQ_E_WS;
  const int u = observe_part_u(n);
#define K2O(A, U_)                                                                                              \
  if (vec && nt) hipLaunchKernelGGL((k_observe_part_out<true, true, A, U_>), dim3((unsigned)grid), dim3(kBlock), 0, \
                                    st, c, y, n, parts, L);                                                     \
  else if (vec) hipLaunchKernelGGL((k_observe_part_out<true, false, A, U_>), dim3((unsigned)grid), dim3(kBlock), 0, \
                                   st, c, y, n, parts, L);                                                      \
  else hipLaunchKernelGGL((k_observe_part_out<false, false, A, U_>), dim3((unsigned)grid), dim3(kBlock), 0, st, c,  \
                          y, n, parts, L);
#define K2OU(A)                     \
  if (u == 8) { K2O(A, 8) }         \
  else if (u == 4) { K2O(A, 4) }    \
  else { K2O(A, 2) }
  if (act_kind(act) == kActRelu) { K2OU(kActRelu) }
  else if (act_kind(act) == kActSilu) { K2OU(kActSilu) }
  else { K2OU(kActNone) }
#undef K2OU
#undef K2O
  return launch_rc();
}

int vsiq_act_observe_part_multi_f32(const vsiq_part_tensor *tensors, int count, int act, void *stream) {
  if (count < 0 || (count > 0 && !tensors) || !act_ok(act)) return VSIQ_E_ARG;
  for (int i = 0; i < count; ++i) {
    const vsiq_part_tensor &T = tensors[i];
    if (T.n <= 0 || !T.c || !T.parts) return VSIQ_E_ARG;
    if (T.parts_len < observe_part_grid(T.n) * kWaves * VSIQ_PART_LEN) return VSIQ_E_WS;
  }
  const bool nt = g_tune.nontemporal != 0;
  for (int i0 = 0; i0 < count; i0 += kPartMulti) {
    PBatch b{};
    b.count = std::min(kPartMulti, count - i0);
    b.sref = act_ref(act);
    uint32_t blk = 0;
    for (int k = 0; k < b.count; ++k) {
      const vsiq_part_tensor &T = tensors[i0 + k];
      PTensor &P = b.t[k];
      P.x = T.c;
      P.parts = T.parts;
      P.n = T.n;
      P.grid = (uint32_t)observe_part_grid(T.n);
      P.u = observe_part_u(T.n);
      P.vec = aligned16(T.c) && T.n % 4 == 0;
      b.blk0[k] = blk;
      blk += P.grid;
    }
    b.blk0[b.count] = blk;
    const hipStream_t st = (hipStream_t)stream;
    bool allvec = true;
    for (int k = 0; k < b.count; ++k) allvec = allvec && b.t[k].vec;
#define K2M(A)                                                                                                 \
  if (nt && allvec) hipLaunchKernelGGL((k_observe_part_multi<true, A, true>), dim3(blk), dim3(kBlock), 0, st, b); \
  else if (nt) hipLaunchKernelGGL((k_observe_part_multi<true, A, false>), dim3(blk), dim3(kBlock), 0, st, b);    \
  else if (allvec) hipLaunchKernelGGL((k_observe_part_multi<false, A, true>), dim3(blk), dim3(kBlock), 0, st, b); \
  else hipLaunchKernelGGL((k_observe_part_multi<false, A, false>), dim3(blk), dim3(kBlock), 0, st, b);
    if (act_kind(act) == kActRelu) { K2M(kActRelu) }
    else if (act_kind(act) == kActSilu) { K2M(kActSilu) }
    else { K2M(kActNone) }
#undef K2M
    const int rc = launch_rc();
    if (rc) return rc;
  }
  return 0;
}

int64_t vsiq_observe_fq_max_elems(void) { return kSmallMax; }

int64_t vsiq_observe_fq_parts_max_elems(void) { return kFoldFqMax; }

int vsiq_act_observe_fq_parts_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                                  double *stats_out, float *run_minmax, double *qp_out, int symmetric,
                                  double qden, double eps, int qmin, int qmax, double *ws, int64_t ws_len,
                                  void *stream) {
  if (n <= 0 || n > kFoldFqMax || !c || !y || !ws || qmin > qmax || !act_ok(act))
    return VSIQ_E_ARG;
  if (ws_len < fold_fq_part_grid(n) * kWaves * VSIQ_PART_LEN) return VSIQ_E_WS;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  const bool vec = n % 4 == 0 && aligned16(c) && aligned16(y) && (!codes || aligned4(codes));
  VSIQ_ACT(act, launch_fold_fq_act, vec, g_tune.nontemporal != 0, c, y, (uint8_t *)codes, mask, n, ws,
           stats_out, run_minmax, qp_out, symmetric, qden, eps, (float)qmin, (float)qmax, act_lay(act, n),
           (hipStream_t)stream);
  return launch_rc();
}

int vsiq_act_observe_fq_grid_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                                 double *stats_out, float *run_minmax, double *qp_out, int symmetric,
                                 double qden, double eps, int qmin, int qmax, double *ws, int64_t ws_len,
                                 uint32_t *counter, void *stream) {
  if (n <= 0 || n > kFoldFqMax || !c || !y || !ws || !counter || qmin > qmax || !act_ok(act))
    return VSIQ_E_ARG;
  if (ws_len < fold_fq_part_grid(n) * kWaves * VSIQ_PART_LEN) return VSIQ_E_WS;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  if (!aligned4(counter)) return VSIQ_E_ALIGN;
  const bool vec = n % 4 == 0 && aligned16(c) && aligned16(y) && (!codes || aligned4(codes));
  VSIQ_ACT(act, launch_observe_fq_grid_act, vec, g_tune.nontemporal != 0, c, y, (uint8_t *)codes, mask, n, ws,
           counter, stats_out, run_minmax, qp_out, symmetric, qden, eps, (float)qmin, (float)qmax,
           act_lay(act, n), (hipStream_t)stream);
  return launch_rc();
}

int vsiq_act_fq_fwd_ranks_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                              const double *gathered, int world, double *stats_out, float *run_minmax,
                              double *qp_out, int symmetric, double qden, double eps, int qmin, int qmax,
                              void *stream) {
  if (n <= 0 || !c || !y || !gathered || world <= 0 || qmin > qmax || !act_ok(act)) return VSIQ_E_ARG;
  if (oneshot_grid(cdiv(n, 4)) > 0x7fffffffLL) return VSIQ_E_ARG;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  const bool vec = n % 4 == 0 && aligned16(c) && aligned16(y) && (!codes || aligned4(codes));
  VSIQ_ACT(act, launch_ranks_fq_act, vec, g_tune.nontemporal != 0, c, y, (uint8_t *)codes, mask, n, gathered,
           world, stats_out, run_minmax, qp_out, symmetric, qden, eps, (float)qmin, (float)qmax, act_lay(act, n),
           (hipStream_t)stream);
  return launch_rc();
}

int vsiq_act_observe_fq_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                            double *stats_out, float *run_minmax, double *qp_out, int symmetric, double qden,
                            double eps, int qmin, int qmax, void *stream) {
  if (n <= 0 || n > kSmallMax || !c || !y || qmin > qmax || !act_ok(act))
    return VSIQ_E_ARG;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  const bool vec = n % 4 == 0 && aligned16(c) && aligned16(y) && (!codes || aligned4(codes));
  VSIQ_ACT(act, launch_observe_fq_small_act, vec, g_tune.nontemporal != 0, c, y, (uint8_t *)codes, mask, n,
           stats_out, run_minmax, qp_out, symmetric, qden, eps, (float)qmin, (float)qmax, act_lay(act, n),
           (hipStream_t)stream);
  return launch_rc();
}

int vsiq_observe_fold_parts(const double *parts, int64_t ncalls, int64_t call_stride, double *stats_out,
                            void *stream) {
  if (ncalls < 0 || ncalls > 0x7fffffffLL) return VSIQ_E_ARG;
  if (ncalls == 0) return 0;
  if (!parts || !stats_out || call_stride < VSIQ_PART_LEN) return VSIQ_E_ARG;
  hipLaunchKernelGGL(k_observe_fold_parts, dim3((unsigned)ncalls), dim3(kBlock), 0, (hipStream_t)stream,
                     parts, call_stride, stats_out);
  return launch_rc();
}

int vsiq_observe_finalize(const double *stats, float *run_minmax, double *qp_out, int symmetric,
                          double qden, double eps, void *stream) {
  if (!stats) return VSIQ_E_ARG;
  hipLaunchKernelGGL(k_observe_finalize, dim3(1), dim3(kWave), 0, (hipStream_t)stream, stats,
                     run_minmax, qp_out, symmetric, qden, eps);
  return launch_rc();
}

int vsiq_observe_finalize_ranks(const double *gathered, int world, double *stats_out, float *run_minmax,
                                double *qp_out, int symmetric, double qden, double eps, void *stream) {
  if (!gathered || world <= 0) return VSIQ_E_ARG;
  hipLaunchKernelGGL(k_observe_finalize_ranks, dim3(1), dim3(kWave), 0, (hipStream_t)stream, gathered, world,
                     stats_out, run_minmax, qp_out, symmetric, qden, eps);
  return launch_rc();
}

}  // extern "C"
