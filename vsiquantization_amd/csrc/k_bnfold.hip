// k_bnfold.hip — BatchNorm folding into the preceding conv / linear weight and bias
// (modules/fused.py:100-108 ConvBnReLU, :294-300 LinearBnReLU), one launch:
//   std = sqrt(running_var + eps);  f = gamma / std
//   W'[r, :] = W[r, :] * f[r];      b'[r] = beta[r] + (b[r] - running_mean[r]) * f[r]
// fp32, the reference's operation order (bit-exact with torch's CPU ops).
#include "vsiq_common.cuh"

namespace vsiq {

// grid (rows, chunks): every workgroup recomputes its row's factor (cheap, no sync)
__global__ __launch_bounds__(kBlock) void k_bn_fold(const float *w, const float *__restrict__ b,
                                                    const float *__restrict__ gamma,
                                                    const float *__restrict__ beta,
                                                    const float *__restrict__ mean,
                                                    const float *__restrict__ var, float eps,
                                                    float *w_out, float *__restrict__ b_out,
                                                    int64_t rowlen, uint32_t chunks) {
  const int64_t row = blockIdx.x / chunks;
  const int64_t chunk = blockIdx.x % chunks;
  const float sd = __builtin_sqrtf(var[row] + eps);
  const float f = gamma[row] / sd;
  for (int64_t i = chunk * kBlock + threadIdx.x; i < rowlen; i += (int64_t)chunks * kBlock)
    w_out[row * rowlen + i] = w[row * rowlen + i] * f;
  if (chunk == 0 && threadIdx.x == 0 && b_out) {
    const float bb = b ? b[row] : 0.0f;
    b_out[row] = beta[row] + (bb - mean[row]) * f;
  }
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_bn_fold_f32(const float *w, const float *b, const float *gamma, const float *beta,
                     const float *running_mean, const float *running_var, float eps, float *w_out,
                     float *b_out, int64_t rows, int64_t rowlen, void *stream) {
  if (rows < 0 || rowlen < 0) return VSIQ_E_ARG;
  if (rows == 0) return 0;
  if (!w || !gamma || !beta || !running_mean || !running_var || !w_out) return VSIQ_E_ARG;
  const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(cdiv(rowlen, kBlock), 64));
  if (rows * chunks > 0x7fffffffLL) return VSIQ_E_ARG;
  hipLaunchKernelGGL(k_bn_fold, dim3((unsigned)(rows * chunks)), dim3(kBlock), 0, (hipStream_t)stream, w, b,
                     gamma, beta, running_mean, running_var, eps, w_out, b_out, rowlen, (uint32_t)chunks);
  return launch_rc();
}

}  // extern "C"
