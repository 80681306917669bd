// k_ste.hip — straight-through backward from the saved 1-bit mask, and its C ABI.
#include "vsiq_common.cuh"

namespace vsiq {

// ----------------------------------------------------------------------------
// STE backward with the saved 1-bit mask: gx = (m ? g*s : 0) / s, grid (rows, chunks)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float ste_gm(float g, uint32_t m, const FastDiv &d) {
  const float gq = g * d.b;          // MulBackward0
  return m ? gq : 0.0f;              // ClampBackward1
}

// one-shot: workgroup b covers chunk b % chunks of row b / chunks (kFlatU groups per lane)
template <bool VEC, bool NT>
__global__ __launch_bounds__(kBlock) void k_ste_bwd(const float *__restrict__ g,
                                                    const uint64_t *__restrict__ mask,
                                                    float *__restrict__ gx, int64_t rowlen,
                                                    uint32_t chunks, const double *__restrict__ sdev,
                                                    double shost) {
  const int64_t row = blockIdx.x / chunks;
  const int64_t chunk = blockIdx.x % chunks;
  const FastDiv s = make_fastdiv((float)(sdev ? sdev[row] : shost));
  const int64_t ng = cdiv(rowlen, 4);
  const float *gr = g + row * rowlen;
  float *xr = gx + row * rowlen;
  const uint64_t *mr = mask + row * mask_words_per_row(rowlen);
  const int lane = threadIdx.x % kWave;
  const int64_t base = chunk * kBlock * kFlatU + threadIdx.x;
  f4 v[kFlatU];
  uint32_t m[kFlatU];
#pragma unroll
  for (int u = 0; u < kFlatU; ++u) {
    const int64_t i = base + u * kBlock;
    const int64_t ic = i < ng ? i : ng - 1;
    v[u] = load_group<VEC, NT>(gr, ic, rowlen);
    m[u] = load_mask_nibble(mr + 4 * (ic / kWave), (int)(ic % kWave));
  }
#pragma unroll
  for (int u = 0; u < kFlatU; ++u) {
    const int64_t i = base + u * kBlock;
    const float a0 = ste_gm(v[u].x, m[u] & 1u, s), a1 = ste_gm(v[u].y, m[u] & 2u, s);
    const float a2 = ste_gm(v[u].z, m[u] & 4u, s), a3 = ste_gm(v[u].w, m[u] & 8u, s);
    f4 o;   // DivBackward0: gm / s
    o.x = fdiv_fast(a0, s); o.y = fdiv_fast(a1, s); o.z = fdiv_fast(a2, s); o.w = fdiv_fast(a3, s);
    if (!(fdiv_ok(a0, s) & fdiv_ok(a1, s) & fdiv_ok(a2, s) & fdiv_ok(a3, s))) {
      o.x = a0 / s.b; o.y = a1 / s.b; o.z = a2 / s.b; o.w = a3 / s.b;   // rare: IEEE
    }
    if (i < ng) store_group<VEC, NT>(xr, i, rowlen, o);
  }
  (void)lane;
}


template <bool VEC, bool NT>
void launch_ste(const float *g, const uint64_t *m, float *gx, int64_t rows, int64_t rowlen,
                const double *sdev, double shost, hipStream_t st) {
  const int64_t chunks = oneshot_grid(cdiv(rowlen, 4));
  hipLaunchKernelGGL((k_ste_bwd<VEC, NT>), dim3((unsigned)(rows * chunks)), dim3(kBlock), 0, st, g, m,
                     gx, rowlen, (uint32_t)chunks, sdev, shost);
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_ste_bwd_f32(const float *g, const uint64_t *mask, float *gx, int64_t n,
                     const double *scale_dev, int64_t rowlen, double scale_host, void *stream) {
  if (n < 0) return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (!g || !mask || !gx) return VSIQ_E_ARG;
  if (!aligned8(mask)) return VSIQ_E_ALIGN;
  if (!scale_dev || rowlen <= 0) rowlen = n;
  if (n % rowlen != 0) return VSIQ_E_ARG;
  const int64_t rows = n / rowlen;
  if (rows * oneshot_grid(cdiv(rowlen, 4)) > 0x7fffffffLL) return VSIQ_E_ARG;
  const bool vec = (rowlen % 4 == 0) && aligned16(g) && aligned16(gx);
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_B2(launch_ste, vec, nt, g, mask, gx, rows, rowlen, scale_dev, scale_host, (hipStream_t)stream);
  return launch_rc();
}

}  // extern "C"
