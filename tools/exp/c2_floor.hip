// c2_floor.hip -- experiment (not product): the plain 1:1 floor of C2's forward at the
// K3 grid shape.  k_copy_gated: y = x over a [rows, 9216] fp32 tensor, one row per
// workgroup of 256 lanes, 9 float4 nontemporal loads per lane (K3's pc_load_row order),
// then -- after the same wall-clock store gate as the product (vsiq_common.cuh
// store_gate_clock: `gate` ticks of the 100 MHz clock since the workgroup started; 0 = no
// gate) -- 9 nontemporal stores.  No reduction, no qparams, no mask: what the traffic
// mix costs at this shape with and without phase separation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o c2_floor.so c2_floor.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(256) void k_copy_gated(const f4 *__restrict__ x, f4 *__restrict__ y, int64_t row4,
                                                     uint32_t gate) {
  const uint64_t t0 = gate ? clk() : 0;
  const f4 *xr = x + (int64_t)blockIdx.x * row4;
  f4 *yr = y + (int64_t)blockIdx.x * row4;
  f4 v[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int64_t i = threadIdx.x + k * 256;
    v[k] = __builtin_nontemporal_load(xr + (i < row4 ? i : row4 - 1));
  }
  if (gate)
    while (clk() - t0 < gate) __builtin_amdgcn_s_sleep(2);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int64_t i = threadIdx.x + k * 256;
    if (i < row4) __builtin_nontemporal_store(v[k], yr + i);
  }
}

extern "C" int exp_copy_gated(const void *x, void *y, int64_t rows, int64_t rowlen, uint32_t gate, void *stream) {
  if (rowlen % 4 || rowlen / 4 > 9 * 256) return 1;
  hipLaunchKernelGGL(k_copy_gated, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, (const f4 *)x, (f4 *)y,
                     rowlen / 4, gate);
  return (int)hipGetLastError();
}
