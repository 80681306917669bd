// mean_cascade.cuh — the order in which torch's CPU kernel sums an fp32 tensor, so that
// mean|x| / mean x of an observer call are the reference's bits, not only its value
// (quantization_manager.py:66-67 records torch.mean(torch.abs(x)).cpu().item() and
// torch.mean(x); init_scaling_factor_for_learning (qm.py:112) turns the mean|x| list
// into the learnable scale).  PyTorch 2.10 CPU (aten/src/ATen/native/cpu/SumKernel.cpp
// cascade_sum, accumulating in float; ReduceOps.cpp mean_out = sum / float(numel)):
//
//   chunks   below GRAIN_SIZE = 32768 elements or on one thread: one serial pass.
//            Otherwise two_pass_reduction: at::parallel_for cuts [0, n) into
//            nt = min(threads, ceil(n / 32768)) chunks of ceil(n / nt) (exactly 32768
//            elements: one chunk, thread 0), chunk t's sum lands in slot t of a zeroed
//            buffer of `threads` floats, and the buffer is summed by the same loop.
//   a chunk  L / V vectors (V = 8: Vectorized<float> of the AVX2 kernel, which this
//            torch build also dispatches on AVX-512 hosts -- pinned, tests/test_mean_oracle.py)
//            in rows of 4 vectors: 4V interleaved fp32 accumulator streams, stream
//            (k, l) holding element (4 r + k) V + l of row r.  Each stream is a 4-level
//            cascade (multi_row_sum): level 0 sums B = 2^max(4, ceil(log2 rows) / 4)
//            rows, level 1 sums B level-0 blocks, level 2 B level-1 nodes, level 3 the
//            level-2 nodes; the partial levels fold as ((tail + l1) + l2) + l3.  Then the
//            <= 3 tail vectors into stream k = 0, the 4 k-streams lane by lane, the
//            scalar tail in order from 0, then the V lanes in order.  A chunk shorter
//            than V runs the same row_sum on scalars (4 streams of 1 lane).
//
// The sequential restatement below serves the host path and the small pieces of the
// GPU kernel K11 (k_mean.hip), which computes the level-0 / level-1 nodes in parallel
// (each node is still a sequential fp32 sum in torch's order).  Every add starts from
// +0.0f like torch's accumulators.  Checked against oracle/mean_ref.c, itself pinned
// against torch.mean on the reference host.
#pragma once
#include "vsiq_common.cuh"

namespace vsiq {

constexpr int kMeanMaxLanes = 16;   // V <= 16 (AVX-512's Vectorized<float>)
constexpr int kMeanMaxLevelPow = 6; // level steps up to 64 rows (chunks below 2^30 elements)

struct MAcc {   // the two sums of one accumulator: |act(x)| and act(x)
  float a, s;
};

__host__ __device__ __forceinline__ void acc_add(MAcc &x, const MAcc &y) {
  x.a += y.a;
  x.s += y.s;
}

__host__ __device__ inline int64_t ceil_log2_i(int64_t x) {
  if (x <= 2) return 1;
  return 64 - __builtin_clzll((uint64_t)(x - 1));
}

// multi_row_sum's level power for a pass over `rows` rows
__host__ __device__ inline int mean_level_power(int64_t rows) {
  const int64_t lp = ceil_log2_i(rows) / 4;
  return lp < 4 ? 4 : (int)lp;
}

// torch's chunking of one reduction over n elements on `threads` threads
struct MeanLay {
  int64_t nchunks;   // chunks that hold elements
  int64_t cs;        // chunk length (the last one may be shorter)
  int twopass;       // the chunk sums go through the `threads`-slot buffer
};

__host__ __device__ inline MeanLay mean_lay(int64_t n, int threads) {
  MeanLay m{n > 0 ? 1 : 0, n, 0};
  if (n < kTorchGrain || threads <= 1) return m;
  m.twopass = 1;
  if (n == kTorchGrain) return m;
  int64_t nt = cdiv(n, kTorchGrain);
  if (nt > threads) nt = threads;
  m.cs = cdiv(n, nt);
  m.nchunks = cdiv(n, m.cs);
  return m;
}

// Every sequential helper works in `buf`: kMeanScratch accumulators the caller provides
// (a local array on the host, LDS in the GPU's one-lane stages, where a dynamically
// indexed local array would live in scratch memory).
constexpr int kMeanScratch = 16 * kMeanMaxLanes + 4 * kMeanMaxLanes + kMeanMaxLanes;

// multi_row_sum<acc, 4> over `size` rows of 4 * lanes items; item c of row i = ld(i * 4 * lanes + c)
template <class LD>
__host__ __device__ void mean_multi_row_seq(const LD &ld, int64_t size, int lanes, MAcc *out, MAcc *buf) {
  const int w = 4 * lanes;
  if (size <= 0) {   // no rows: every accumulator stays +0 (the same bits, ~300 LDS ops fewer
                     // for the one-lane final stage, where rows = threads / (4 V) is 0)
    for (int c = 0; c < w; ++c) out[c] = MAcc{0.0f, 0.0f};
    return;
  }
  const int lp = mean_level_power(size);
  const int64_t step = (int64_t)1 << lp, mask = step - 1;
  MAcc *acc[4] = {buf, buf + 4 * kMeanMaxLanes, buf + 8 * kMeanMaxLanes, buf + 12 * kMeanMaxLanes};
  for (int j = 0; j < 4; ++j)
    for (int c = 0; c < w; ++c) acc[j][c] = MAcc{0.0f, 0.0f};
  int64_t i = 0;
  while (i + step <= size) {
    for (int64_t r = 0; r < step; ++r, ++i)
      for (int c = 0; c < w; ++c) acc_add(acc[0][c], ld(i * w + c));
    for (int j = 1; j < 4; ++j) {
      for (int c = 0; c < w; ++c) {
        acc_add(acc[j][c], acc[j - 1][c]);
        acc[j - 1][c] = MAcc{0.0f, 0.0f};
      }
      if ((i & (mask << (j * lp))) != 0) break;
    }
  }
  for (; i < size; ++i)
    for (int c = 0; c < w; ++c) acc_add(acc[0][c], ld(i * w + c));
  for (int j = 1; j < 4; ++j)
    for (int c = 0; c < w; ++c) acc_add(acc[0][c], acc[j][c]);
  for (int c = 0; c < w; ++c) out[c] = acc[0][c];
}

// row_sum<acc, 4>: `size` items of `lanes` values; the lanes' sums in out[0..lanes)
template <class LD>
__host__ __device__ void mean_row_seq(const LD &ld, int64_t size, int lanes, MAcc *out, MAcc *buf) {
  MAcc *p = buf + 16 * kMeanMaxLanes;
  const int64_t ilp = size / 4;
  mean_multi_row_seq(ld, ilp, lanes, p, buf);
  for (int64_t i = ilp * 4; i < size; ++i)
    for (int l = 0; l < lanes; ++l) acc_add(p[l], ld(i * lanes + l));
  for (int k = 1; k < 4; ++k)
    for (int l = 0; l < lanes; ++l) acc_add(p[l], p[k * lanes + l]);
  for (int l = 0; l < lanes; ++l) out[l] = p[l];
}

// the reduce loop over one chunk of len items (vectorized_inner_sum / its scalar form)
template <class LD>
__host__ __device__ MAcc mean_chunk_seq(const LD &ld, int64_t len, int V, MAcc *buf) {
  MAcc *lanes = buf + 20 * kMeanMaxLanes;
  if (len < V) {
    mean_row_seq(ld, len, 1, lanes, buf);
    return lanes[0];
  }
  const int64_t nv = len / V;
  mean_row_seq(ld, nv, V, lanes, buf);
  MAcc acc{0.0f, 0.0f};
  for (int64_t k = nv * V; k < len; ++k) acc_add(acc, ld(k));
  for (int l = 0; l < V; ++l) acc_add(acc, lanes[l]);
  return acc;
}

// the second pass: `threads` slots, chunk sums in the first nchunks (0 + sum), zeros after
template <class CS>
__host__ __device__ MAcc mean_final_seq(const CS &csum, const MeanLay &m, int V, int threads, MAcc *buf) {
  MAcc out{0.0f, 0.0f};
  if (!m.twopass) {
    if (m.nchunks > 0) acc_add(out, csum(0));
    return out;
  }
  auto slot = [&](int64_t t) {
    MAcc v{0.0f, 0.0f};
    if (t < m.nchunks) acc_add(v, csum(t));
    return v;
  };
  acc_add(out, mean_chunk_seq(slot, threads, V, buf));
  return out;
}

// element loader: {|act(x[e])|, act(x[e])} with the activation's reference layout
template <int ACT>
__host__ __device__ __forceinline__ MAcc mean_elem(float v, int64_t e, const SiluLay &L) {
  float t = v;
  if (ACT == kActRelu) t = v < 0.0f ? 0.0f : v;
  if (ACT == kActSilu) t = (L.on && (silu_scalar4(e, L) & 1u)) ? silu_fwd<true>(v) : silu_fwd<false>(v);
  return MAcc{__builtin_fabsf(t), t};
}

}  // namespace vsiq
