// k_fq.hip — K1 per-tensor fake-quant forward (optionally behind a fused ReLU/SiLU,
// K5), and its C ABI entry points.
#include "k_body.cuh"

namespace vsiq {

// K1 kernel: one tensor, block body in k_body.cuh
template <bool VEC, bool NT, bool CODES, bool MASK, int ACT, int U>
__global__ __launch_bounds__(kBlock) void k_fq_fwd(const float *__restrict__ x, float *__restrict__ y,
                                                   uint8_t *__restrict__ codes,
                                                   uint64_t *__restrict__ mask, int64_t n,
                                                   QPSrc src, uint32_t gate, SiluLay L) {
  const GateClk gc = gate_begin(gate);
  // the kernel-uniform qparams as scalar loads, after the x loads are issued
  fq_fwd_block<VEC, NT, CODES, MASK, ACT, U>(x, y, codes, mask, n, [&] { return load_qp<true>(src); }, blockIdx.x,
                                             gc, gate, L);
}

// One-round grids get the store gate (store_gate_select: >= 2 workgroups per CU, all
// resident): the kFlatU grid where it is one round (round 5: C4's 3.3M / 6.6M-element
// layers), else 9 groups per lane where that is (13M), else kFlatU ungated.
template <bool VEC, bool NT, bool CODES, bool MASK, int ACT>
void launch_fq_k(const float *x, float *y, uint8_t *codes, uint64_t *mask, int64_t n,
                 const QPSrc &src, const SiluLay &L, hipStream_t st) {
  const int64_t ng = cdiv(n, 4);
  const int64_t grid9 = cdiv(ng, (int64_t)kBlock * 9), gridu = oneshot_grid(ng);
  const void *kern9 = reinterpret_cast<const void *>(k_fq_fwd<VEC, NT, CODES, MASK, ACT, 9>);
  const void *kernu = reinterpret_cast<const void *>(k_fq_fwd<VEC, NT, CODES, MASK, ACT, kFlatU>);
  static const int occ9 = occupancy_blocks(kern9, kBlock);
  static const int occu = occupancy_blocks(kernu, kBlock);
  const int64_t cus = device_cus();
  GateSel gs;
  if (g_tune.store_gate != 0 && gridu >= 2 * cus && gridu <= (int64_t)occu * cus) {
    gs = store_gate_select("k1_fq_fwd_flat", kernu, gridu, occu, 4 * n, st);
  } else if (g_tune.store_gate != 0 && grid9 * kBlock * 9 - ng <= ng / 8 && grid9 >= 2 * cus &&
             grid9 <= (int64_t)occ9 * cus) {
    gs = store_gate_select("k1_fq_fwd", kern9, grid9, occ9, 4 * n, st);
    if (gs.gate) {
      hipLaunchKernelGGL((k_fq_fwd<VEC, NT, CODES, MASK, ACT, 9>), dim3((unsigned)grid9), dim3(kBlock), 0, st,
                         x, y, codes, mask, n, src, gs.gate, L);
      store_gate_launched(gs, st);
      return;
    }
  }
  hipLaunchKernelGGL((k_fq_fwd<VEC, NT, CODES, MASK, ACT, kFlatU>), dim3((unsigned)gridu), dim3(kBlock), 0, st, x,
                     y, codes, mask, n, src, gs.gate, L);
  store_gate_launched(gs, st);   // for the 9-group site: a tuning sample of "no gate" times the kFlatU grid
}

template <int ACT, bool VEC, bool NT>
void launch_fq_act(const float *x, float *y, uint8_t *codes, uint64_t *mask, int64_t n,
                   const QPSrc &src, const SiluLay &L, hipStream_t st) {
  if (codes && mask) launch_fq_k<VEC, NT, true, true, ACT>(x, y, codes, mask, n, src, L, st);
  else if (codes) launch_fq_k<VEC, NT, true, false, ACT>(x, y, codes, mask, n, src, L, st);
  else if (mask) launch_fq_k<VEC, NT, false, true, ACT>(x, y, codes, mask, n, src, L, st);
  else launch_fq_k<VEC, NT, false, false, ACT>(x, y, codes, mask, n, src, L, st);
}

template <int ACT>
void launch_fq(bool vec, bool nt, const float *x, float *y, uint8_t *codes, uint64_t *mask, int64_t n,
               const QPSrc &src, const SiluLay &L, hipStream_t st) {
  if (vec && nt) launch_fq_act<ACT, true, true>(x, y, codes, mask, n, src, L, st);
  else if (vec) launch_fq_act<ACT, true, false>(x, y, codes, mask, n, src, L, st);
  else if (nt) launch_fq_act<ACT, false, true>(x, y, codes, mask, n, src, L, st);
  else launch_fq_act<ACT, false, false>(x, y, codes, mask, n, src, L, st);
}

int fq_fwd(const float *x, float *y, void *codes, uint64_t *mask, int64_t n, int act,
           const double *qp_dev, const double *scale_dev, double scale_host, const double *zp_dev,
           double zp_host, int zp_round, int discrete, int qmin, int qmax, void *stream) {
  if (n < 0 || qmin > qmax || (n > 0 && (!x || !y)) || !act_ok(act))
    return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (mask && !aligned8(mask)) return VSIQ_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  QPSrc src{qp_dev, scale_dev, zp_dev, scale_host, zp_host, (float)qmin, (float)qmax,
            qp_dev ? 0 : zp_round, discrete ? 1 : 0};
  const bool vec = (n % 4 == 0) && aligned16(x) && aligned16(y) && (!codes || aligned4(codes));
  const bool nt = g_tune.nontemporal != 0;
  uint8_t *c = (uint8_t *)codes;
  VSIQ_ACT(act, launch_fq, vec, nt, x, y, c, mask, n, src, act_lay(act, n), st);
  return launch_rc();
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t n,
                    const double *qp_dev, const double *scale_dev, double scale_host,
                    const double *zp_dev, double zp_host, int zp_round, int discrete, int qmin,
                    int qmax, void *stream) {
  return fq_fwd(x, y, codes, mask, n, kActNone, qp_dev, scale_dev, scale_host, zp_dev, zp_host,
                zp_round, discrete, qmin, qmax, stream);
}

int vsiq_act_fq_fwd_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                        const double *qp_dev, const double *scale_dev, double scale_host,
                        const double *zp_dev, double zp_host, int zp_round, int discrete, int qmin,
                        int qmax, void *stream) {
  return fq_fwd(c, y, codes, mask, n, act, qp_dev, scale_dev, scale_host, zp_dev, zp_host,
                zp_round, discrete, qmin, qmax, stream);
}

}  // extern "C"
