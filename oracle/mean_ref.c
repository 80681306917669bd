/*
 * oracle/mean_ref.c -- TEST INFRASTRUCTURE (never linked into the product).
 *
 * C restatement of what the reference records as mean|x| / mean x per observer call,
 * `torch.mean(torch.abs(x)).cpu().item()` / `torch.mean(x)` on fp32 CPU tensors
 * (/root/reference/quantizers/quantization_manager.py:66-67), i.e. PyTorch 2.10's CPU
 * mean = sum, then an fp32 division by float(numel) (aten ReduceOps.cpp mean_out), and
 * its fp32 sum (aten/src/ATen/native/cpu/SumKernel.cpp, cascade_sum, acc type float):
 *
 *   chunking   TensorIterator::parallel_reduce: serial below GRAIN_SIZE = 32768 elements
 *              or on one thread; otherwise two_pass_reduction: at::parallel_for splits
 *              [0, n) into nt = min(threads, ceil(n / 32768)) chunks of ceil(n / nt)
 *              (exactly GRAIN_SIZE elements: one chunk, thread 0), each chunk's sum goes
 *              to its thread's slot of a zeroed buffer of `threads` floats, and the
 *              buffer is summed by the same loop;
 *   one chunk  vectorized_inner_sum: L / V vectors of V floats (V = 16 AVX-512, 8 AVX2)
 *              summed by row_sum (4 interleaved vector accumulators, multi_row_sum's
 *              4-level cascade with 2^max(4, ceil(log2 rows) / 4) rows per level step),
 *              then the scalar tail, then the V lanes, in that order; a chunk shorter
 *              than V runs row_sum on scalars.
 *
 * Pinned by tests/test_mean_oracle.py against torch.mean itself on this host (sizes
 * around every boundary, 1..16 threads, AVX-512 and -- in a subprocess with
 * ATEN_CPU_CAPABILITY=avx2 -- AVX2).  The GPU kernel K11 (csrc/k_mean.hip) and the host
 * loop (csrc/host_mean.cpp) are checked against this file.
 *
 * Build: gcc -O2 -ffp-contract=off -fno-builtin -shared -fPIC (oracle/build_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define GRAIN 32768
#define MAXLANES 16

typedef struct {
  const float *x;
  int absf;
} Src;

static float ld(const Src *s, int64_t e) {
  const float v = s->x[e];
  return s->absf ? fabsf(v) : v;
}

static int64_t ceil_log2(int64_t x) {
  if (x <= 2) return 1;
  return 64 - __builtin_clzll((uint64_t)(x - 1));
}

/* multi_row_sum<acc, 4>: row i, column c (= k * lanes + l) at base + i * 4 * lanes + c */
static void multi_row_sum(const Src *s, int64_t base, int64_t size, int lanes, float *out) {
  const int levels = 4, w = 4 * lanes;
  int64_t lp = ceil_log2(size) / levels;
  if (lp < 4) lp = 4;
  const int64_t step = (int64_t)1 << lp, mask = step - 1;
  float acc[4][4 * MAXLANES];
  memset(acc, 0, sizeof acc);
  int64_t i = 0;
  while (i + step <= size) {
    for (int64_t j = 0; j < step; ++j, ++i)
      for (int c = 0; c < w; ++c) acc[0][c] += ld(s, base + i * w + c);
    for (int j = 1; j < levels; ++j) {
      for (int c = 0; c < w; ++c) {
        acc[j][c] += acc[j - 1][c];
        acc[j - 1][c] = 0.0f;
      }
      if ((i & (mask << (j * lp))) != 0) break;
    }
  }
  for (; i < size; ++i)
    for (int c = 0; c < w; ++c) acc[0][c] += ld(s, base + i * w + c);
  for (int j = 1; j < levels; ++j)
    for (int c = 0; c < w; ++c) acc[0][c] += acc[j][c];
  memcpy(out, acc[0], sizeof(float) * w);
}

/* row_sum<acc, 4>: `size` items of `lanes` floats at base; returns the lanes in out */
static void row_sum(const Src *s, int64_t base, int64_t size, int lanes, float *out) {
  float p[4 * MAXLANES];
  const int64_t ilp = size / 4;
  multi_row_sum(s, base, ilp, lanes, p);
  for (int64_t i = ilp * 4; i < size; ++i)
    for (int l = 0; l < lanes; ++l) p[l] += ld(s, base + i * lanes + l);
  for (int k = 1; k < 4; ++k)
    for (int l = 0; l < lanes; ++l) p[l] += p[k * lanes + l];
  memcpy(out, p, sizeof(float) * lanes);
}

/* the reduce loop over [o, o + len) */
static float chunk_sum(const Src *s, int64_t o, int64_t len, int V) {
  float lanes[MAXLANES];
  if (len < V) {
    row_sum(s, o, len, 1, lanes);
    return lanes[0];
  }
  const int64_t nv = len / V;
  row_sum(s, o, nv, V, lanes);
  float acc = 0.0f;
  for (int64_t k = nv * V; k < len; ++k) acc += ld(s, o + k);
  for (int l = 0; l < V; ++l) acc += lanes[l];
  return acc;
}

float oracle_torch_sum_f32(const float *x, int64_t n, int absf, int V, int threads) {
  Src s = {x, absf};
  if (V < 1 || V > MAXLANES || threads < 1) return NAN;
  if (n < GRAIN || threads == 1) return 0.0f + chunk_sum(&s, 0, n, V);
  float buf[1024];
  if (threads > 1024) return NAN;
  for (int t = 0; t < threads; ++t) buf[t] = 0.0f;
  if (n == GRAIN) {
    buf[0] += chunk_sum(&s, 0, n, V);
  } else {
    int64_t nt = (n + GRAIN - 1) / GRAIN;
    if (nt > threads) nt = threads;
    const int64_t cs = (n + nt - 1) / nt;
    for (int64_t t = 0; t < nt; ++t) {
      const int64_t b = t * cs;
      if (b >= n) break;
      const int64_t e = b + cs < n ? b + cs : n;
      buf[t] += chunk_sum(&s, b, e - b, V);
    }
  }
  Src sb = {buf, 0};
  return 0.0f + chunk_sum(&sb, 0, threads, V);
}

/* torch.mean: the sum divided (fp32) by float(n) */
float oracle_torch_mean_f32(const float *x, int64_t n, int absf, int V, int threads) {
  const float sum = oracle_torch_sum_f32(x, n, absf, V, threads);
  return sum / (float)n;
}
