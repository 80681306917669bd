// k_ste.hip — straight-through backward from the saved 1-bit mask, and its C ABI.
#include "vsiq_common.cuh"

namespace vsiq {

// ----------------------------------------------------------------------------
// STE backward with the saved 1-bit mask: gx = (m ? g*s : 0) / s, grid (rows, chunks)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float ste_elem(float g, uint32_t m, const FastDiv &d) {
  const float gq = g * d.b;          // MulBackward0
  const float gm = m ? gq : 0.0f;    // ClampBackward1
  return fdiv(gm, d);                // DivBackward0
}

template <bool VEC, bool NT>
__global__ __launch_bounds__(kBlock) void k_ste_bwd(const float *__restrict__ g,
                                                    const uint64_t *__restrict__ mask,
                                                    float *__restrict__ gx, int64_t rowlen,
                                                    const double *__restrict__ sdev, double shost) {
  const int64_t row = blockIdx.x;
  const FastDiv s = make_fastdiv((float)(sdev ? sdev[row] : shost));
  const int64_t ng = cdiv(rowlen, 4);
  const float *gr = g + row * rowlen;
  float *xr = gx + row * rowlen;
  const uint64_t *mr = mask + row * mask_words_per_row(rowlen);
  const int lane = threadIdx.x % kWave;
  for (int64_t i = (int64_t)blockIdx.y * kBlock + threadIdx.x; i - lane < ng;
       i += (int64_t)gridDim.y * kBlock) {
    const uint32_t m = load_mask_nibble(mr + 4 * (i / kWave), lane);
    if (i < ng) {
      const f4 v = load_group<VEC, NT>(gr, i, rowlen);
      f4 o;
      o.x = ste_elem(v.x, m & 1u, s);
      o.y = ste_elem(v.y, m & 2u, s);
      o.z = ste_elem(v.z, m & 4u, s);
      o.w = ste_elem(v.w, m & 8u, s);
      store_group<VEC, NT>(xr, i, rowlen, o);
    }
  }
}


template <bool VEC, bool NT>
void launch_ste(const float *g, const uint64_t *m, float *gx, int64_t rows, int64_t rowlen,
                const double *sdev, double shost, hipStream_t st) {
  const dim3 grid((unsigned)rows, (unsigned)chunk_grid(rowlen, rows)), block(kBlock);
  hipLaunchKernelGGL((k_ste_bwd<VEC, NT>), grid, block, 0, st, g, m, gx, rowlen, sdev, shost);
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
  if (rows > 0x7fffffffLL) return VSIQ_E_ARG;
  const bool vec = (rowlen % 4 == 0) && aligned16(g) && aligned16(gx);
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_B2(launch_ste, vec, nt, g, mask, gx, rows, rowlen, scale_dev, scale_host, (hipStream_t)stream);
  return launch_rc();
}

}  // extern "C"
