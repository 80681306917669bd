// STE-backward shape experiments at the C2 size (experiment only, not product):
// groups per lane SU, mask source (scalar words / none), row-per-workgroup form.
#include "vsiq_common.cuh"

using namespace vsiq;

// MM: 0 = scalar mask words (product), 1 = no mask (all pass)
template <int SU, int MM>
__global__ __launch_bounds__(kBlock) void k_ste_x(const float *__restrict__ g,
                                                  const uint64_t *__restrict__ mask,
                                                  float *__restrict__ gx, int64_t n, float s) {
  const SteDiv d = make_stediv(s);
  const int64_t ng = n / 4;
  const int64_t base = (int64_t)blockIdx.x * kBlock * SU + threadIdx.x;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  f4 v[SU];
  uint64_t w[SU][4];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    v[u] = ld4<true>(g + 4 * (i < ng ? i : ng - 1));
    const int64_t c = (int64_t)blockIdx.x * (kBlock / kWave) * SU + u * (kBlock / kWave) + wave0;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[u][j] = MM == 0 ? mask[4 * c + j] : ~0ull;
  }
  f4 o[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const bool m0 = __builtin_amdgcn_inverse_ballot_w64(w[u][0]);
    const bool m1 = __builtin_amdgcn_inverse_ballot_w64(w[u][1]);
    const bool m2 = __builtin_amdgcn_inverse_ballot_w64(w[u][2]);
    const bool m3 = __builtin_amdgcn_inverse_ballot_w64(w[u][3]);
    o[u].x = m0 ? ste_quot(v[u].x, d) : 0.0f;
    o[u].y = m1 ? ste_quot(v[u].y, d) : 0.0f;
    o[u].z = m2 ? ste_quot(v[u].z, d) : 0.0f;
    o[u].w = m3 ? ste_quot(v[u].w, d) : 0.0f;
    if (!(d.fast & ste_ok(v[u].x) & ste_ok(v[u].y) & ste_ok(v[u].z) & ste_ok(v[u].w))) {
      o[u].x = ste_ieee(v[u].x, m0, d);
      o[u].y = ste_ieee(v[u].y, m1, d);
      o[u].z = ste_ieee(v[u].z, m2, d);
      o[u].w = ste_ieee(v[u].w, m3, d);
    }
  }
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    if (i < ng) st4<true>(gx + 4 * i, o[u]);
  }
}

// pure scaled copy with the same grid shape (no mask, no division)
template <int SU>
__global__ __launch_bounds__(kBlock) void k_scale_x(const float *__restrict__ g, float *__restrict__ gx,
                                                    int64_t n, float s) {
  const int64_t ng = n / 4;
  const int64_t base = (int64_t)blockIdx.x * kBlock * SU + threadIdx.x;
  f4 v[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    v[u] = ld4<true>(g + 4 * (i < ng ? i : ng - 1));
  }
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    if (i < ng) st4<true>(gx + 4 * i, v[u] * s);
  }
}

extern "C" int exp_ste(const float *g, const uint64_t *m, float *gx, int64_t n, float s, int su, int mm,
                       void *st) {
  const int64_t ng = n / 4;
  auto S = (hipStream_t)st;
#define L(SU, MM)                                                                              \
  hipLaunchKernelGGL((k_ste_x<SU, MM>), dim3((unsigned)cdiv(ng, kBlock * SU)), dim3(kBlock), 0, S, g, \
                     m, gx, n, s)
#define LS(SU) \
  hipLaunchKernelGGL((k_scale_x<SU>), dim3((unsigned)cdiv(ng, kBlock * SU)), dim3(kBlock), 0, S, g, gx, n, s)
  if (mm == 2) {
    if (su == 1) LS(1); else if (su == 2) LS(2); else if (su == 4) LS(4); else if (su == 8) LS(8); else return -1;
  } else if (mm == 0) {
    if (su == 1) L(1, 0); else if (su == 2) L(2, 0); else if (su == 4) L(4, 0); else if (su == 8) L(8, 0); else return -1;
  } else {
    if (su == 1) L(1, 1); else if (su == 2) L(2, 1); else if (su == 4) L(4, 1); else if (su == 8) L(8, 1); else return -1;
  }
  return (int)hipGetLastError();
}
