// stream_mix.hip — experiment: the HBM rate plain streaming kernels reach on MI355X for
// the read:write mixes of the fake-quant kernels (1:1 = K1 / K3 / STE, 2:1 = K4,
// 1:0 = K2 observer), with the same access pattern as the product kernels (16-byte
// nontemporal loads / stores, 256 lanes, G groups per lane, one-shot grids).  Buffers
// rotate past the 256 MB MALL.  Prints GB/s per mix and size.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o stream_mix stream_mix.hip && ./stream_mix
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int G>
__global__ __launch_bounds__(256) void k_copy(const f4 *__restrict__ a, f4 *__restrict__ y, long ng) {
  const long base = (long)blockIdx.x * 256 * G + threadIdx.x;
  f4 v[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const long i = base + k * 256;
    v[k] = __builtin_nontemporal_load(a + (i < ng ? i : ng - 1));
  }
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const long i = base + k * 256;
    if (i < ng) __builtin_nontemporal_store(v[k] * 1.5f, y + i);
  }
}

template <int G>
__global__ __launch_bounds__(256) void k_add(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                             f4 *__restrict__ y, long ng) {
  const long base = (long)blockIdx.x * 256 * G + threadIdx.x;
  f4 u[G], v[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const long i = base + k * 256, j = i < ng ? i : ng - 1;
    u[k] = __builtin_nontemporal_load(a + j);
    v[k] = __builtin_nontemporal_load(b + j);
  }
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const long i = base + k * 256;
    if (i < ng) __builtin_nontemporal_store(u[k] + v[k], y + i);
  }
}

template <int G>
__global__ __launch_bounds__(256) void k_read(const f4 *__restrict__ a, float *__restrict__ out, long ng) {
  const long base = (long)blockIdx.x * 256 * G + threadIdx.x;
  f4 s = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const long i = base + k * 256;
    s += __builtin_nontemporal_load(a + (i < ng ? i : ng - 1));
  }
  const float t = s.x + s.y + s.z + s.w;
  if (t == 123.456f) out[blockIdx.x] = t;   // keeps the loads; never true for the fill
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const long sizes[] = {9437184L, 77070336L, 104857600L};   // C2 weight, C3 tensor, C4 largest layer
  for (long n : sizes) {
    const long ng = n / 4;
    const int sets = (int)std::max(2L, (3L << 30) / (12 * n) + 1);
    std::vector<f4 *> A(sets), B(sets), Y(sets);
    for (int s = 0; s < sets; ++s) {
      CK(hipMalloc(&A[s], n * 4));
      CK(hipMalloc(&B[s], n * 4));
      CK(hipMalloc(&Y[s], n * 4));
      CK(hipMemset(A[s], 0, n * 4));
      CK(hipMemset(B[s], 0, n * 4));
    }
    float *out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 200;
    auto time_it = [&](auto launch, double bytes, const char *name) {
      for (int r = 0; r < 20; ++r) launch(r % sets);
      hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) launch(r % sets);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      std::printf("n=%10ld %-22s %8.2f us  %7.0f GB/s\n", n, name, us, bytes / us / 1e3);
    };
    const unsigned g2 = (unsigned)((ng + 512 - 1) / 512), g8 = (unsigned)((ng + 2048 - 1) / 2048);
    time_it([&](int s) { hipLaunchKernelGGL(k_copy<2>, dim3(g2), dim3(256), 0, 0, A[s], Y[s], ng); }, 8.0 * n,
            "1:1 copy  G=2");
    time_it([&](int s) { hipLaunchKernelGGL(k_copy<8>, dim3(g8), dim3(256), 0, 0, A[s], Y[s], ng); }, 8.0 * n,
            "1:1 copy  G=8");
    time_it([&](int s) { hipLaunchKernelGGL(k_add<2>, dim3(g2), dim3(256), 0, 0, A[s], B[s], Y[s], ng); },
            12.0 * n, "2:1 add   G=2");
    time_it([&](int s) { hipLaunchKernelGGL(k_add<8>, dim3(g8), dim3(256), 0, 0, A[s], B[s], Y[s], ng); },
            12.0 * n, "2:1 add   G=8");
    time_it([&](int s) { hipLaunchKernelGGL(k_read<8>, dim3(g8), dim3(256), 0, 0, A[s], out, ng); }, 4.0 * n,
            "1:0 read  G=8");
    for (int s = 0; s < sets; ++s) {
      hipFree(A[s]);
      hipFree(B[s]);
      hipFree(Y[s]);
    }
    hipFree(out);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
  return 0;
}
