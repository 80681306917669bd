// k_multi.hip — multi-tensor ("foreach") learnable fake quant: many per-tensor
// LSQ quantizers (the weight quantizers of every fused layer of a model) in ONE
// forward launch (K1 bodies) and ONE backward launch (K4 bodies with a per-tensor
// fold), instead of one launch per layer.  A small weight's launch is all fixed
// cost (dispatch ramp, load latency, the K4 arrival/fold chain: 4.6 us forward and
// 6-7 us backward per YOLOv8n weight on MI355X, rocprof r01e); in one launch those
// costs are paid once and the tensors' blocks share the machine.
//
// Per element, per block and per tensor reduction order this is exactly the
// single-tensor path (same bodies, same grid per tensor, same flat fold), so the
// outputs are bit-identical to vsiq_fq_fwd_f32 / vsiq_lsq_bwd_f32 per tensor.
#include "k_body.cuh"

namespace vsiq {

constexpr int kMulti = 32;    // tensors per launch: the descriptor table travels as kernel arguments (3.5 KB)
constexpr int kMultiG = 4;    // K4 groups per lane (the single-tensor default)
// backward: a tensor's grid must arrive flat (one counter word per tensor)
constexpr int64_t kMultiMaxGroups = (int64_t)kArriveFlat * kBlock * kMultiG;

struct MTensor {
  const float *x;
  float *y;          // forward output
  const float *g;    // backward input
  float *gx;         // backward output
  const double *sdev, *zdev;
  double *gout;
  int64_t n;
  double shost, zhost, gscale;
  float lo, hi;
  int zpl, vec;
};

struct MBatch {
  MTensor t[kMulti];
  uint32_t blk0[kMulti + 1];   // first block of tensor i; blk0[count] = grid
  int count;
};

// tensor owning this block (scalar: blk0 lives in the kernel arguments)
__device__ __forceinline__ int mtensor_of(const MBatch &b) {
  int t = 0;
  const uint32_t blk = blockIdx.x;
  while (t + 1 < b.count && blk >= b.blk0[t + 1]) ++t;
  return t;
}

__device__ __forceinline__ QPSrc mtensor_qp(const MTensor &T) {
  return QPSrc{nullptr, T.sdev, T.zdev, T.shost, T.zhost, T.lo, T.hi, T.zpl, 0};
}

template <bool NT>
__global__ __launch_bounds__(kBlock) void k_lsq_fwd_multi(const MBatch b) {
  const int t = mtensor_of(b);
  const MTensor &T = b.t[t];
  const int64_t blk = (int64_t)blockIdx.x - b.blk0[t];
  // the tensor's qparams (workgroup-uniform) as scalar loads, after the x loads are issued
  const auto qf = [&] { return load_qp<true>(mtensor_qp(T)); };
  if (T.vec) fq_fwd_block<true, NT, false, false, kActNone>(T.x, T.y, nullptr, nullptr, T.n, qf, blk);
  else fq_fwd_block<false, NT, false, false, kActNone>(T.x, T.y, nullptr, nullptr, T.n, qf, blk);
}

// Backward: block partial -> ws record (global block index), flat arrival on the
// tensor's own counter word, the tensor's last block folds its records in block order.
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_lsq_bwd_multi(const MBatch b, double *__restrict__ ws,
                                                          uint32_t *__restrict__ counter) {
  const int t = mtensor_of(b);
  const MTensor &T = b.t[t];
  const QPSrc src = mtensor_qp(T);
  const auto qf = [&] { return load_qp<true>(src); };   // scalar loads, after the first loads
  const uint32_t first = b.blk0[t], nb = b.blk0[t + 1] - first;
  const int64_t blk = (int64_t)blockIdx.x - first;
  LsqAcc c{0.0, 0.0};
  // the zero-point sum is always accumulated (only read when T.zpl): the scale sum and
  // grad_x do not depend on it
  f4 o[kMultiG];
  double rec[2], f[2];
  bool w0;
  QP p;
  if (T.vec) {
    p = lsq_bwd_block<true, NT, true, kActNone, kMultiG>(T.g, T.x, T.n, qf, blk, c, o);
    w0 = lsq_block_record<true, NT, kMultiG>(c, T.gx, T.n, blk, o, rec);
  } else {
    p = lsq_bwd_block<false, NT, true, kActNone, kMultiG>(T.g, T.x, T.n, qf, blk, c, o);
    w0 = lsq_block_record<false, NT, kMultiG>(c, T.gx, T.n, blk, o, rec);
  }
  if (!w0) return;   // waves 1..3 have stored their grad_x
  // flat arrival on the tensor's own counter word, records in block order: the
  // single-tensor kernel's fold for grids <= kArriveFlat, bit for bit
  const bool last = wave_arrive<LsqFold>(ws, first, nb, (uint32_t)blk, counter + t, rec, f, [&]() {
    if (T.vec) lsq_store_block<true, NT, kMultiG>(T.gx, T.n, blk, o);
    else lsq_store_block<false, NT, kMultiG>(T.gx, T.n, blk, o);
  });
  if (!last) return;
  if (threadIdx.x == 0) {
    T.gout[0] = f[0] * T.gscale;
    T.gout[1] = T.zpl ? lsq_grad_zp(f[1], src, p, T.gscale) : 0.0;
    counter[t] = 0u;   // ready for the next stream-ordered launch
  }
}

inline int64_t multi_grid(bool bwd, int64_t n) {
  const int64_t ng = cdiv(n, 4);
  return bwd ? cdiv(ng, (int64_t)kBlock * kMultiG) : oneshot_grid(ng);
}

// a descriptor the multi-tensor launch accepts (else: invalid, or routed to the
// single-tensor kernel when only its size is the problem)
inline int check_desc(const vsiq_lsq_tensor &d, bool bwd) {
  if (d.n <= 0 || !d.x || d.qmin > d.qmax) return VSIQ_E_ARG;
  if (bwd ? (!d.g || !d.gx || !d.grad_out) : !d.y) return VSIQ_E_ARG;
  return 0;
}

inline bool multi_fits(const vsiq_lsq_tensor &d, bool bwd) {
  return !bwd || cdiv(d.n, (int64_t)4) <= kMultiMaxGroups;
}

inline MTensor to_mtensor(const vsiq_lsq_tensor &d, bool bwd) {
  MTensor m;
  m.x = d.x; m.y = d.y; m.g = d.g; m.gx = d.gx;
  m.sdev = d.scale_dev; m.zdev = d.zp_dev; m.gout = d.grad_out;
  m.n = d.n; m.shost = d.scale_host; m.zhost = d.zp_host; m.gscale = d.gscale;
  m.lo = (float)d.qmin; m.hi = (float)d.qmax; m.zpl = d.zp_learn ? 1 : 0;
  m.vec = (d.n % 4 == 0) && aligned16(d.x) &&
          (bwd ? aligned16(d.g) && aligned16(d.gx) : aligned16(d.y));
  return m;
}

// records a batch of the given tensors needs (max over the launches of one call)
int64_t multi_ws_records(const vsiq_lsq_tensor *ts, int count) {
  int64_t best = 0, cur = 0;
  int in_batch = 0;
  for (int i = 0; i < count; ++i) {
    if (!multi_fits(ts[i], true)) {   // single-tensor K4 with the same workspace
      best = std::max<int64_t>(best, fold_records(lsq_grid(cdiv(ts[i].n, (int64_t)4))));
      continue;
    }
    if (in_batch == kMulti) { best = std::max(best, cur); cur = 0; in_batch = 0; }
    cur += multi_grid(true, ts[i].n);
    ++in_batch;
  }
  return std::max(best, cur);
}

int lsq_bwd(const float *g, const float *x, float *gx, int64_t n, int act, const double *scale_dev,
            double scale_host, const double *zp_dev, double zp_host, int zp_learn, int qmin, int qmax,
            double gscale, double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
            void *stream);   // k_lsq.hip

int lsq_multi(bool bwd, const vsiq_lsq_tensor *ts, int count, double *ws, int64_t ws_len,
              uint32_t *counter, void *stream) {
  if (count < 0 || (count > 0 && !ts)) return VSIQ_E_ARG;
  if (count == 0) return 0;
  if (bwd && (!ws || !counter)) return VSIQ_E_ARG;
  for (int i = 0; i < count; ++i)
    if (int rc = check_desc(ts[i], bwd)) return rc;
  if (bwd && ws_len < multi_ws_records(ts, count) * kPartials) return VSIQ_E_WS;
  hipStream_t st = (hipStream_t)stream;
  const bool nt = g_tune.nontemporal != 0;
  MBatch b;
  auto flush = [&]() {
    if (b.count == 0) return;
    const dim3 grid(b.blk0[b.count]), block(kBlock);
    if (bwd) {
      if (nt) hipLaunchKernelGGL(k_lsq_bwd_multi<true>, grid, block, 0, st, b, ws, counter);
      else hipLaunchKernelGGL(k_lsq_bwd_multi<false>, grid, block, 0, st, b, ws, counter);
    } else {
      if (nt) hipLaunchKernelGGL(k_lsq_fwd_multi<true>, grid, block, 0, st, b);
      else hipLaunchKernelGGL(k_lsq_fwd_multi<false>, grid, block, 0, st, b);
    }
    b.count = 0;
    b.blk0[0] = 0;
  };
  b.count = 0;
  b.blk0[0] = 0;
  for (int i = 0; i < count; ++i) {
    const vsiq_lsq_tensor &d = ts[i];
    if (!multi_fits(d, bwd)) {   // too large for one flat arrival: the single-tensor kernel
      flush();
      const int rc = lsq_bwd(d.g, d.x, d.gx, d.n, kActNone, d.scale_dev, d.scale_host, d.zp_dev, d.zp_host,
                             d.zp_learn, d.qmin, d.qmax, d.gscale, d.grad_out, ws, ws_len, counter, stream);
      if (rc) return rc;
      continue;
    }
    const int64_t grid = multi_grid(bwd, d.n);
    if (b.count == kMulti || (int64_t)b.blk0[b.count] + grid > 0x7fffffffLL) flush();
    b.t[b.count] = to_mtensor(d, bwd);
    b.blk0[b.count + 1] = b.blk0[b.count] + (uint32_t)grid;
    ++b.count;
  }
  flush();
  return launch_rc();
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int64_t vsiq_lsq_multi_workspace_doubles(const vsiq_lsq_tensor *tensors, int count) {
  if (count < 0 || (count > 0 && !tensors)) return VSIQ_E_ARG;
  return multi_ws_records(tensors, count) * kPartials;
}

int vsiq_lsq_fwd_multi_f32(const vsiq_lsq_tensor *tensors, int count, void *stream) {
  return lsq_multi(false, tensors, count, nullptr, 0, nullptr, stream);
}

int vsiq_lsq_bwd_multi_f32(const vsiq_lsq_tensor *tensors, int count, double *ws, int64_t ws_len,
                           uint32_t *counter, void *stream) {
  return lsq_multi(true, tensors, count, ws, ws_len, counter, stream);
}

}  // extern "C"
