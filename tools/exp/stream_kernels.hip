// Streaming ceilings at the C2 size on MI355X: float4 copy / read / write kernels,
// plain and nontemporal, grid-stride or one-pass.  Experiment only (not product).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ x, f4* __restrict__ y, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n4; b += stride * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (b + u * stride < n4) v[u] = NT ? __builtin_nontemporal_load(&x[b + u * stride]) : x[b + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) if (b + u * stride < n4) { if (NT) __builtin_nontemporal_store(v[u], &y[b + u * stride]); else y[b + u * stride] = v[u]; }
  }
}

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ x, float* out, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  float acc = 0.f;
  for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n4; b += stride * 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (b + u * stride < n4) v[u] = x[b + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (b + u * stride < n4) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(float4* __restrict__ y, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n4; b += stride) y[b] = make_float4(1.f, 2.f, 3.f, 4.f);
}

extern "C" int exp_copy(const void* x, void* y, int64_t n4, int grid, int nt, int unroll, void* st) {
  auto s = (hipStream_t)st;
  auto X = (const f4*)x; auto Y = (f4*)y;
  if (nt) { if (unroll == 1) hipLaunchKernelGGL((k_copy<true, 1>), dim3(grid), dim3(256), 0, s, X, Y, n4); else hipLaunchKernelGGL((k_copy<true, 4>), dim3(grid), dim3(256), 0, s, X, Y, n4); }
  else { if (unroll == 1) hipLaunchKernelGGL((k_copy<false, 1>), dim3(grid), dim3(256), 0, s, X, Y, n4); else hipLaunchKernelGGL((k_copy<false, 4>), dim3(grid), dim3(256), 0, s, X, Y, n4); }
  return (int)hipGetLastError();
}
extern "C" int exp_read(const void* x, void* out, int64_t n4, int grid, void* st) {
  hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, (hipStream_t)st, (const float4*)x, (float*)out, n4);
  return (int)hipGetLastError();
}
extern "C" int exp_write(void* y, int64_t n4, int grid, void* st) {
  hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, (hipStream_t)st, (float4*)y, n4);
  return (int)hipGetLastError();
}
