// Structure experiments for the per-channel kernel (K3) at the C2 shape: what do
// "whole row in registers, reduce, then store" and its pipelined forms cost compared
// with a plain copy?  Experiment only (not product).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int BS, int NV>
__device__ __forceinline__ void load_row(f4 (&v)[NV], const f4 *__restrict__ x, int64_t row, int ng) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int i = threadIdx.x + k * BS;
    i = i < ng ? i : ng - 1;
    v[k] = __builtin_nontemporal_load(&x[row * ng + i]);
  }
}

__device__ __forceinline__ float wmin(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

template <int BS, int NV, int RED>
__device__ __forceinline__ void proc_row(f4 (&v)[NV], f4 *__restrict__ y, int64_t row, int ng,
                                         int par, float (*lds)[2][BS / 64]) {
  float s = 2.f, o = 0.f;
  if (RED) {
    float mn = __builtin_inff(), mx = -__builtin_inff();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      mn = fminf(mn, fminf(fminf(v[k].x, v[k].y), fminf(v[k].z, v[k].w)));
      mx = fmaxf(mx, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
    }
    mn = wmin(mn);
    mx = wmax(mx);
    if (threadIdx.x % 64 == 0) {
      lds[par][0][threadIdx.x / 64] = mn;
      lds[par][1][threadIdx.x / 64] = mx;
    }
    __syncthreads();
    mn = lds[par][0][0];
    mx = lds[par][1][0];
#pragma unroll
    for (int w = 1; w < BS / 64; ++w) {
      mn = fminf(mn, lds[par][0][w]);
      mx = fmaxf(mx, lds[par][1][w]);
    }
    s = 1.f / (mx - mn + 1.f);
    o = -mn * s;
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * BS;
    f4 r = v[k] * s + o;
    if (i < ng) __builtin_nontemporal_store(r, &y[row * ng + i]);
  }
}

// one row per workgroup
template <int BS, int NV, int RED>
__global__ __launch_bounds__(BS) void k_row1(const f4 *__restrict__ x, f4 *__restrict__ y, int ng) {
  __shared__ float lds[2][2][BS / 64];
  f4 v[NV];
  load_row<BS, NV>(v, x, blockIdx.x, ng);
  proc_row<BS, NV, RED>(v, y, blockIdx.x, ng, 0, lds);
}

// RPB rows per workgroup (row = blockIdx + r*grid), fully unrolled, 2-deep prefetch:
// loads of row r+1 are in flight while row r is reduced and stored.
template <int BS, int NV, int RPB, int RED>
__global__ __launch_bounds__(BS) void k_rowpipe(const f4 *__restrict__ x, f4 *__restrict__ y, int ng) {
  __shared__ float lds[2][2][BS / 64];
  f4 a[NV], b[NV];
  const int64_t g = gridDim.x;
  load_row<BS, NV>(a, x, blockIdx.x, ng);
  if (RPB > 1) load_row<BS, NV>(b, x, blockIdx.x + g, ng);
#pragma unroll
  for (int r = 0; r < RPB; ++r) {
    const int64_t row = blockIdx.x + r * g;
    if (r % 2 == 0) {
      proc_row<BS, NV, RED>(a, y, row, ng, 0, lds);
      if (r + 2 < RPB) load_row<BS, NV>(a, x, row + 2 * g, ng);
    } else {
      proc_row<BS, NV, RED>(b, y, row, ng, 1, lds);
      if (r + 2 < RPB) load_row<BS, NV>(b, x, row + 2 * g, ng);
    }
  }
}

#define L1(BS, NV, RED) hipLaunchKernelGGL((k_row1<BS, NV, RED>), dim3(rows), dim3(BS), lds, s, X, Y, ng)
#define LP(BS, NV, RPB, RED) hipLaunchKernelGGL((k_rowpipe<BS, NV, RPB, RED>), dim3(rows / RPB), dim3(BS), lds, s, X, Y, ng)

extern "C" int exp_row(const void *x, void *y, int rows, int rowlen, int bs, int rpb, int red,
                       int lds, void *st) {
  auto s = (hipStream_t)st;
  auto X = (const f4 *)x;
  auto Y = (f4 *)y;
  const int ng = rowlen / 4;
  if (ng > 512 * 5 || ng <= 256 * 8 || rowlen % 4) return -1;   // C2-shaped rows only
  if (bs == 512) {
    if (rpb == 1) { if (red) L1(512, 5, 1); else L1(512, 5, 0); }
    else if (rpb == 2) { if (red) LP(512, 5, 2, 1); else LP(512, 5, 2, 0); }
    else if (rpb == 4) { if (red) LP(512, 5, 4, 1); else LP(512, 5, 4, 0); }
    else return -1;
  } else if (bs == 256) {
    if (rpb == 1) { if (red) L1(256, 9, 1); else L1(256, 9, 0); }
    else if (rpb == 2) { if (red) LP(256, 9, 2, 1); else LP(256, 9, 2, 0); }
    else if (rpb == 4) { if (red) LP(256, 9, 4, 1); else LP(256, 9, 4, 0); }
    else if (rpb == 8) { if (red) LP(256, 9, 8, 1); else LP(256, 9, 8, 0); }
    else return -1;
  } else if (bs == 1024) {
    if (rpb == 1) { if (red) L1(1024, 3, 1); else L1(1024, 3, 0); }
    else if (rpb == 2) { if (red) LP(1024, 3, 2, 1); else LP(1024, 3, 2, 0); }
    else if (rpb == 4) { if (red) LP(1024, 3, 4, 1); else LP(1024, 3, 4, 0); }
    else return -1;
  } else return -1;
  return (int)hipGetLastError();
}
