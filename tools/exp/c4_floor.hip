// c4_floor.hip -- experiment (not product): the plain 2:1 streaming floor at the C4
// activation sizes.  exp_add2: y = a + b over n/4 float4 groups, 16-byte nontemporal loads
// and stores, 256 lanes, G groups per lane, one-shot grid (no loop: all G loads of a lane
// issued, then the G stores) -- the access pattern of K4d records-only (read g, read x,
// write grad_x) without its element math and records.  exp_relu1: y = max(a, 0), the
// 1:1 floor of the C4 forward (K1 with the fused ReLU: read c, write y).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o c4_floor.so c4_floor.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int G>
__global__ __launch_bounds__(256) void k_add2(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                              f4 *__restrict__ y, int64_t ng) {
  const int64_t base = (int64_t)blockIdx.x * 256 * G + threadIdx.x;
  f4 u[G], v[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int64_t i = base + k * 256, j = i < ng ? i : ng - 1;
    u[k] = __builtin_nontemporal_load(a + j);
    v[k] = __builtin_nontemporal_load(b + j);
  }
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int64_t i = base + k * 256;
    if (i < ng) __builtin_nontemporal_store(u[k] + v[k], y + i);
  }
}

extern "C" int exp_add2(const void *a, const void *b, void *y, int64_t ng, int g, void *stream) {
  const hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((ng + 256 * g - 1) / (256 * g));
  switch (g) {
    case 1: hipLaunchKernelGGL(k_add2<1>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (const f4 *)b, (f4 *)y, ng); break;
    case 2: hipLaunchKernelGGL(k_add2<2>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (const f4 *)b, (f4 *)y, ng); break;
    case 4: hipLaunchKernelGGL(k_add2<4>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (const f4 *)b, (f4 *)y, ng); break;
    case 8: hipLaunchKernelGGL(k_add2<8>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (const f4 *)b, (f4 *)y, ng); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}

template <int G>
__global__ __launch_bounds__(256) void k_relu1(const f4 *__restrict__ a, f4 *__restrict__ y, int64_t ng) {
  const int64_t base = (int64_t)blockIdx.x * 256 * G + threadIdx.x;
  f4 u[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int64_t i = base + k * 256, j = i < ng ? i : ng - 1;
    u[k] = __builtin_nontemporal_load(a + j);
  }
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int64_t i = base + k * 256;
    const f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
    if (i < ng) __builtin_nontemporal_store(__builtin_elementwise_max(u[k], z), y + i);
  }
}

extern "C" int exp_relu1(const void *a, void *y, int64_t ng, int g, void *stream) {
  const hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((ng + 256 * g - 1) / (256 * g));
  switch (g) {
    case 1: hipLaunchKernelGGL(k_relu1<1>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (f4 *)y, ng); break;
    case 2: hipLaunchKernelGGL(k_relu1<2>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (f4 *)y, ng); break;
    case 4: hipLaunchKernelGGL(k_relu1<4>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (f4 *)y, ng); break;
    case 8: hipLaunchKernelGGL(k_relu1<8>, dim3(grid), dim3(256), 0, st, (const f4 *)a, (f4 *)y, ng); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}
