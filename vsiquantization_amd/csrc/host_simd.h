// host_simd.h — AVX-512 loops of the host (CPU-tensor) path, host_simd.cpp.  Plain C++
// interface (no HIP): k_host.hip calls them per fixed chunk when the CPU has AVX-512
// F/BW/VL and the activation is none or ReLU; otherwise it runs its scalar loops.
// Elementwise results are bit-identical to the scalar loops (IEEE division, rint by
// vrndscaleps round-to-nearest-even, the same compare/blend clamp that keeps NaN and
// -0.0, no FMA); f64 sums use 16 lane accumulators folded in lane order (deterministic
// for a given chunk; the statistics are compared to tolerances, not bits).
#pragma once
#include <cstdint>

namespace vsiq {
namespace simd {

bool available();

// {min, max, nan count, sum|v|, sum v, sum v^2} of v = act(x[0..n)); min / max over the
// non-NaN elements with strict compares (+inf / -inf when there is none)
void observe(const float *x, int64_t n, int relu, double out[6]);

// y = fq(act(x)); codes / mask nullable (1 byte per element)
void fq(const float *x, float *y, uint8_t *codes, uint8_t *mask, int64_t n, int relu, float s, float z, float lo,
        float hi, int discrete);

// gx = act'((mask ? g*s : 0) / s); pre: the pre-activation (relu only)
void ste(const float *g, const uint8_t *mask, const float *pre, float *gx, int64_t n, int relu, float s);

// learnable backward: gx, and out = {sum t, sum z} (k_host.hip's term order)
void lsq(const float *g, const float *x, float *gx, int64_t n, int relu, float s, float z, float lo, float hi,
         int zp_learn, double out[2]);

}  // namespace simd
}  // namespace vsiq
