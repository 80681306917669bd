// STE-backward shape experiments at the C2 size (experiment only, not product):
// groups per lane SU, mask source (scalar words / none), row-per-workgroup form.
#include "vsiq_common.cuh"

using namespace vsiq;

// MM: 0 = scalar mask words (product), 1 = no mask (all pass)
template <int SU, int MM, int BAR = 0>
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
  if (BAR) __syncthreads();   // the workgroup's stores go out as one burst
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    if (i < ng) st4<true>(gx + 4 * i, o[u]);
  }
}

// two halves: all 2H groups' loads issued up front; half 0 is computed and stored
// (unconditional stores: the workgroup is wholly in range) while half 1's loads
// are still in flight -- the row experiment's "2 rows per workgroup" overlap.
template <int H>
__device__ __forceinline__ void ste_half(const f4 (&v)[H], const uint64_t (&w)[H][4], f4 (&o)[H],
                                         const SteDiv &d) {
#pragma unroll
  for (int u = 0; u < H; ++u) {
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
}

template <int H>
__global__ __launch_bounds__(kBlock) void k_ste_h(const float *__restrict__ g,
                                                  const uint64_t *__restrict__ mask,
                                                  float *__restrict__ gx, int64_t n, float s) {
  const SteDiv d = make_stediv(s);
  const int64_t ng = n / 4;
  const int64_t base = (int64_t)blockIdx.x * kBlock * 2 * H + threadIdx.x;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  f4 a[H], b[H];
  uint64_t wa[H][4], wb[H][4];
#pragma unroll
  for (int u = 0; u < 2 * H; ++u) {
    const int64_t i = base + u * kBlock;
    const f4 t = ld4<true>(g + 4 * (i < ng ? i : ng - 1));
    const int64_t c = (int64_t)blockIdx.x * (kBlock / kWave) * 2 * H + u * (kBlock / kWave) + wave0;
    if (u < H) a[u] = t; else b[u - H] = t;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (u < H) wa[u][j] = mask[4 * c + j]; else wb[u - H][j] = mask[4 * c + j];
    }
  }
  f4 o[H];
  ste_half<H>(a, wa, o, d);
#pragma unroll
  for (int u = 0; u < H; ++u) st4<true>(gx + 4 * (base + u * kBlock), o[u]);   // C2: no tail
  ste_half<H>(b, wb, o, d);
#pragma unroll
  for (int u = 0; u < H; ++u) st4<true>(gx + 4 * (base + (H + u) * kBlock), o[u]);
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
                       void *st, int lds) {
  const int64_t ng = n / 4;
  auto S = (hipStream_t)st;
#define L(SU, MM)                                                                              \
  hipLaunchKernelGGL((k_ste_x<SU, MM>), dim3((unsigned)cdiv(ng, kBlock * SU)), dim3(kBlock), lds, S, g, \
                     m, gx, n, s)
#define LS(SU) \
  hipLaunchKernelGGL((k_scale_x<SU>), dim3((unsigned)cdiv(ng, kBlock * SU)), dim3(kBlock), lds, S, g, gx, n, s)
#define LB(SU)                                                                                   \
  hipLaunchKernelGGL((k_ste_x<SU, 0, 1>), dim3((unsigned)cdiv(ng, kBlock * SU)), dim3(kBlock), lds, S, g, \
                     m, gx, n, s)
#define LH(H) \
  hipLaunchKernelGGL((k_ste_h<H>), dim3((unsigned)cdiv(ng, kBlock * 2 * H)), dim3(kBlock), lds, S, g, m, gx, n, s)
  if (mm == 4) {
    if (ng % (kBlock * 2 * su)) return -2;
    if (su == 1) LH(1); else if (su == 2) LH(2); else if (su == 3) LH(3); else if (su == 4) LH(4); else if (su == 8) LH(8); else return -1;
  } else if (mm == 3) {
    if (su == 1) LB(1); else if (su == 2) LB(2); else if (su == 4) LB(4); else if (su == 8) LB(8); else if (su == 9) LB(9); else return -1;
  } else if (mm == 2) {
    if (su == 1) LS(1); else if (su == 2) LS(2); else if (su == 4) LS(4); else if (su == 8) LS(8); else return -1;
  } else if (mm == 0) {
    if (su == 1) L(1, 0); else if (su == 2) L(2, 0); else if (su == 4) L(4, 0); else if (su == 8) L(8, 0); else if (su == 9) L(9, 0); else return -1;
  } else {
    if (su == 1) L(1, 1); else if (su == 2) L(2, 1); else if (su == 4) L(4, 1); else if (su == 8) L(8, 1); else return -1;
  }
  return (int)hipGetLastError();
}
