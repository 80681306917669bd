// Why does K3 (row reduce between its loads and its stores) beat a plain copy of the
// same bytes?  Copy-shaped kernels with SU float4 per lane, optional barrier, optional
// s_sleep and optional LDS min/max reduction between the load and the store phase.
// Experiment only (not product).
#include "vsiq_common.cuh"

using namespace vsiq;

template <int SU, int MODE, int SLEEP>
__global__ __launch_bounds__(kBlock) void k_phase(const float *__restrict__ x, float *__restrict__ y,
                                                  int64_t n) {
  __shared__ float red[kBlock / kWave];
  const int64_t ng = n / 4;
  const int64_t base = (int64_t)blockIdx.x * kBlock * SU + threadIdx.x;
  f4 v[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    v[u] = ld4<true>(x + 4 * (i < ng ? i : ng - 1));
  }
  float k = 1.0f;
  if (MODE >= 1) {
    float m = 0.0f;
#pragma unroll
    for (int u = 0; u < SU; ++u) m = fmaxf(m, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
    if (MODE == 2) {
      m = wave_reduce(m, MaxOp());
      if (threadIdx.x % kWave == 0) red[threadIdx.x / kWave] = m;
    }
    __syncthreads();
    if (MODE == 2) {
      m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      k = m > 1e30f ? 0.5f : 1.0f;
    }
  }
  if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = base + u * kBlock;
    if (i < ng) st4<true>(y + 4 * i, v[u] * k);
  }
}

template <int SU, int MODE>
static void go_sleep(const float *x, float *y, int64_t n, int sleep, hipStream_t s) {
  const unsigned grid = (unsigned)cdiv(n / 4, (int64_t)kBlock * SU);
  switch (sleep) {
#define PH(S) case S: hipLaunchKernelGGL((k_phase<SU, MODE, S>), dim3(grid), dim3(kBlock), 0, s, x, y, n); break;
    PH(0) PH(4) PH(16) PH(32) PH(48) PH(64) PH(80) PH(96) PH(127)
#undef PH
    default: break;
  }
}

template <int SU>
static void go_mode(const float *x, float *y, int64_t n, int mode, int sleep, hipStream_t s) {
  if (mode == 0) go_sleep<SU, 0>(x, y, n, sleep, s);
  else if (mode == 1) go_sleep<SU, 1>(x, y, n, sleep, s);
  else go_sleep<SU, 2>(x, y, n, sleep, s);
}

extern "C" int exp_phase(const float *x, float *y, int64_t n, int su, int mode, int sleep, void *st) {
  auto s = (hipStream_t)st;
  if (su == 2) go_mode<2>(x, y, n, mode, sleep, s);
  else if (su == 4) go_mode<4>(x, y, n, mode, sleep, s);
  else go_mode<9>(x, y, n, mode, sleep, s);
  return (int)hipGetLastError();
}

// the product STE body (per-row scale from sdev), one row per workgroup (SU groups per
// lane), optional barrier + s_sleep between the load and the store phase
template <int SU, int BAR, int SLEEP>
__global__ __launch_bounds__(kBlock) void k_ste_phase(const float *__restrict__ g,
                                                      const uint64_t *__restrict__ mask,
                                                      float *__restrict__ gx, int64_t rowlen,
                                                      const double *__restrict__ sdev) {
  const int64_t row = blockIdx.x;
  const SteDiv d = make_stediv((float)sdev[row]);
  const int64_t ng = cdiv(rowlen, 4);
  const int64_t nchunk = cdiv(ng, kWave);
  const float *gr = g + row * rowlen;
  float *xr = gx + row * rowlen;
  const uint64_t *mr = mask + row * mask_words_per_row(rowlen);
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  f4 v[SU];
  uint64_t w[SU][4];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = threadIdx.x + u * kBlock;
    v[u] = load_group<true, true>(gr, i < ng ? i : ng - 1, rowlen);
    int64_t c = u * (kBlock / kWave) + wave0;
    c = c < nchunk ? c : nchunk - 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[u][j] = mr[4 * c + j];
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
  if (BAR) __syncthreads();
  if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = threadIdx.x + u * kBlock;
    if (i < ng) store_group<true, true>(xr, i, rowlen, o[u]);
  }
}

#define STE_CASE(B, S)                                                                           \
  if (bar == B && sleep == S) {                                                                  \
    hipLaunchKernelGGL((k_ste_phase<9, B, S>), dim3((unsigned)rows), dim3(kBlock), 0, s, g, m, gx, \
                       rowlen, sdev);                                                            \
    return (int)hipGetLastError();                                                               \
  }

extern "C" int exp_ste_phase(const float *g, const uint64_t *m, float *gx, int64_t rows, int64_t rowlen,
                             const double *sdev, int bar, int sleep, void *st) {
  auto s = (hipStream_t)st;
  if (cdiv(rowlen, 4) > 9 * kBlock) return 1;
  STE_CASE(0, 0) STE_CASE(1, 0) STE_CASE(1, 16) STE_CASE(1, 48) STE_CASE(1, 80) STE_CASE(1, 127)
  STE_CASE(0, 48) STE_CASE(0, 127) STE_CASE(1, 64) STE_CASE(1, 96)
  return 2;
}

// ---- gated store phase: stores start once the device's read phase is (about) over
// GATE 1: realtime clock, wait until t0 + ticks (t0 = this workgroup's start)
// GATE 2: arrival counter (all workgroups' loads done) + generation word, bounded polls
__device__ uint32_t g_arrive[2];   // [0] arrivals, [1] generation

__device__ __forceinline__ void gate_wait(int gate, uint64_t t0, uint32_t ticks, uint32_t nblk) {
  if (gate == 1) {
    if (threadIdx.x == 0) {
      const uint64_t until = t0 + ticks;
      while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
  } else if (gate == 2) {
    __syncthreads();   // every wave's loads consumed
    if (threadIdx.x == 0) {
      const uint32_t gen0 = __hip_atomic_load(&g_arrive[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t old = __hip_atomic_fetch_add(&g_arrive[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == nblk) {
        __hip_atomic_store(&g_arrive[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&g_arrive[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (int k = 0; k < 4000; ++k) {
          if (__hip_atomic_load(&g_arrive[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen0) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
  }
}

template <int SU, int GATE>
__global__ __launch_bounds__(kBlock) void k_ste_gate(const float *__restrict__ g,
                                                     const uint64_t *__restrict__ mask,
                                                     float *__restrict__ gx, int64_t rowlen,
                                                     const double *__restrict__ sdev, uint32_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t row = blockIdx.x;
  const SteDiv d = make_stediv((float)sdev[row]);
  const int64_t ng = cdiv(rowlen, 4);
  const int64_t nchunk = cdiv(ng, kWave);
  const float *gr = g + row * rowlen;
  float *xr = gx + row * rowlen;
  const uint64_t *mr = mask + row * mask_words_per_row(rowlen);
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  f4 v[SU];
  uint64_t w[SU][4];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = threadIdx.x + u * kBlock;
    v[u] = load_group<true, true>(gr, i < ng ? i : ng - 1, rowlen);
    int64_t c = u * (kBlock / kWave) + wave0;
    c = c < nchunk ? c : nchunk - 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[u][j] = mr[4 * c + j];
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
  gate_wait(GATE, t0, ticks, gridDim.x);
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int64_t i = threadIdx.x + u * kBlock;
    if (i < ng) store_group<true, true>(xr, i, rowlen, o[u]);
  }
}

extern "C" int exp_ste_gate(const float *g, const uint64_t *m, float *gx, int64_t rows, int64_t rowlen,
                            const double *sdev, int gate, uint32_t ticks, void *st) {
  auto s = (hipStream_t)st;
  if (cdiv(rowlen, 4) > 9 * kBlock) return 1;
  if (gate == 1)
    hipLaunchKernelGGL((k_ste_gate<9, 1>), dim3((unsigned)rows), dim3(kBlock), 0, s, g, m, gx, rowlen, sdev, ticks);
  else
    hipLaunchKernelGGL((k_ste_gate<9, 2>), dim3((unsigned)rows), dim3(kBlock), 0, s, g, m, gx, rowlen, sdev, ticks);
  return (int)hipGetLastError();
}

extern "C" int exp_wallclock_khz() {
  int v = 0;
  hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, 0);
  return v;
}

// ---- 2-read / 1-write streaming ceiling (x, g -> x*g), one-shot U groups per lane
template <int U>
__global__ __launch_bounds__(kBlock) void k_tri(const float *__restrict__ x, const float *__restrict__ g,
                                                float *__restrict__ y, int64_t n) {
  const int64_t ng = n / 4;
  const int64_t base = (int64_t)blockIdx.x * kBlock * U + threadIdx.x;
  f4 a[U], b[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kBlock;
    a[u] = ld4<true>(x + 4 * (i < ng ? i : ng - 1));
    b[u] = ld4<true>(g + 4 * (i < ng ? i : ng - 1));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kBlock;
    if (i < ng) st4<true>(y + 4 * i, a[u] * b[u]);
  }
}

extern "C" int exp_tri(const float *x, const float *g, float *y, int64_t n, int u, void *st) {
  auto s = (hipStream_t)st;
  const int64_t ng = n / 4;
#define TRI(U) if (u == U) { hipLaunchKernelGGL((k_tri<U>), dim3((unsigned)cdiv(ng, (int64_t)kBlock * U)), dim3(kBlock), 0, s, x, g, y, n); return (int)hipGetLastError(); }
  TRI(1) TRI(2) TRI(4) TRI(8) TRI(16)
#undef TRI
  return 1;
}
