// Per-workgroup timeline of a K3-shaped one-round grid (one 9216-element row per
// workgroup, row min/max reduce, store gate): wall-clock ticks of start, loads landed,
// gate release and stores complete, written to rec[grid][4].  Experiment only.
#include "vsiq_common.cuh"

using namespace vsiq;

template <int NV>
__global__ __launch_bounds__(kBlock) void k_tl(const float *__restrict__ x, float *__restrict__ y,
                                               int64_t rowlen, uint32_t gate, uint64_t *rec) {
  const uint64_t t0 = wall_clock64();
  __shared__ float red[kBlock / kWave];
  const int64_t ng = rowlen / 4;
  const float *xr = x + blockIdx.x * rowlen;
  float *yr = y + blockIdx.x * rowlen;
  f4 v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t i = threadIdx.x + k * kBlock;
    v[k] = load_group_c<true, true>(xr, i, ng, rowlen);
  }
  float m = 0.0f;
#pragma unroll
  for (int k = 0; k < NV; ++k) m = fmaxf(m, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
  m = wave_reduce(m, MaxOp());
  if (threadIdx.x % kWave == 0) red[threadIdx.x / kWave] = m;
  __syncthreads();
  const uint64_t t1 = wall_clock64();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float k = m > 1e30f ? 0.5f : 1.0f;
  if (gate) store_gate_clock(t0, gate);
  const uint64_t t2 = wall_clock64();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int64_t i = threadIdx.x + j * kBlock;
    if (i < ng) store_group<true, true>(yr, i, rowlen, v[j] * k);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t3 = wall_clock64();
    rec[4 * blockIdx.x + 0] = t0;
    rec[4 * blockIdx.x + 1] = t1;
    rec[4 * blockIdx.x + 2] = t2;
    rec[4 * blockIdx.x + 3] = t3;
  }
}

extern "C" int exp_tl(const float *x, float *y, int64_t rows, int64_t rowlen, int gate, uint64_t *rec,
                      void *st) {
  if (rowlen != 9216) return -1;
  hipLaunchKernelGGL((k_tl<9>), dim3((unsigned)rows), dim3(kBlock), 0, (hipStream_t)st, x, y, rowlen,
                     (uint32_t)gate, rec);
  return (int)hipGetLastError();
}
