// k_act.hip — the fused layers' activation on its own: F.relu / F.silu of
// modules/fused.py:133 where its output is not fake-quantized in the same pass
// (calibration forwards, whose output feeds the next layer; quantize_out off), and its
// backward.  Same element code as K5 (vsiq_common.cuh): SiLU bit for bit as torch's CPU
// kernel on the reference host, so a calibration forward hands the next layer the
// reference's activations, not torch's HIP silu (a different exp).
#include "vsiq_common.cuh"

namespace vsiq {

// one-shot, kFlatU groups per lane: loads first, then compute, then stores
template <bool VEC, bool NT, int ACT, bool BWD>
__global__ __launch_bounds__(kBlock) void k_act(const float *__restrict__ g, const float *__restrict__ c,
                                                float *__restrict__ y, int64_t n, SiluLay L) {
  const int64_t ng = cdiv(n, 4);
  const int64_t base = (int64_t)blockIdx.x * kBlock * kFlatU + threadIdx.x;
  f4 cv[kFlatU], gv[kFlatU];
#pragma unroll
  for (int u = 0; u < kFlatU; ++u) {
    cv[u] = load_group_c<VEC, NT>(c, base + u * kBlock, ng, n);
    if (BWD) gv[u] = load_group_c<VEC, NT>(g, base + u * kBlock, ng, n);
  }
  f4 o[kFlatU];
#pragma unroll
  for (int u = 0; u < kFlatU; ++u) {
    const int64_t e0 = 4 * (base + u * kBlock);
    o[u] = BWD ? act_bwd4_at<ACT>(gv[u], cv[u], e0, L) : act_fwd4_at<ACT>(cv[u], e0, L);
  }
#pragma unroll
  for (int u = 0; u < kFlatU; ++u)
    if (base + u * kBlock < ng) store_group<VEC, NT>(y, base + u * kBlock, n, o[u]);
}

template <int ACT>
void launch_act(bool vec, bool nt, bool bwd, const float *g, const float *c, float *y, int64_t n,
                const SiluLay &L, hipStream_t st) {
  const dim3 grid((unsigned)oneshot_grid(cdiv(n, 4)));
#define KA(V, T, B) hipLaunchKernelGGL((k_act<V, T, ACT, B>), grid, dim3(kBlock), 0, st, g, c, y, n, L)
  if (bwd) {
    if (vec && nt) KA(true, true, true);
    else if (vec) KA(true, false, true);
    else KA(false, false, true);
  } else {
    if (vec && nt) KA(true, true, false);
    else if (vec) KA(true, false, false);
    else KA(false, false, false);
  }
#undef KA
}

// exp self-test: both exps of the SiLU element code (Sleef's vectorized expf, glibc's
// scalar expf) for arbitrary inputs, checked bitwise against the oracle's restatement
__global__ __launch_bounds__(kBlock) void k_selftest_exp(const float *__restrict__ x, float *__restrict__ ys,
                                                         float *__restrict__ yg, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const float v = x[i];
    ys[i] = sleef_expf_u10(v);
    yg[i] = glibc_expf(v);
  }
}

int act_run(const float *g, const float *c, float *y, int64_t n, int act, bool bwd, void *stream) {
  if (n < 0 || !act_ok(act) || act_kind(act) == kActNone) return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (!c || !y || (bwd && !g)) return VSIQ_E_ARG;
  if (oneshot_grid(cdiv(n, 4)) > 0x7fffffffLL) return VSIQ_E_ARG;
  const bool vec = n % 4 == 0 && aligned16(c) && aligned16(y) && (!bwd || aligned16(g));
  VSIQ_ACT(act, launch_act, vec, g_tune.nontemporal != 0, bwd, g, c, y, n, act_lay(act, n),
           (hipStream_t)stream);
  return launch_rc();
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_act_fwd_f32(const float *c, float *y, int64_t n, int act, void *stream) {
  return act_run(nullptr, c, y, n, act, false, stream);
}

int vsiq_act_bwd_f32(const float *g, const float *c, float *gc, int64_t n, int act, void *stream) {
  return act_run(g, c, gc, n, act, true, stream);
}

int vsiq_selftest_exp_f32(const float *x, float *sleef_out, float *glibc_out, int64_t n, void *stream) {
  if (n < 0 || (n > 0 && (!x || !sleef_out || !glibc_out))) return VSIQ_E_ARG;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_selftest_exp, dim3((unsigned)std::min<int64_t>(cdiv(n, kBlock), 4096)), dim3(kBlock), 0,
                     (hipStream_t)stream, x, sleef_out, glibc_out, n);
  return launch_rc();
}

}  // extern "C"
