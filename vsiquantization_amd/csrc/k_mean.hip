// k_mean.hip — K11: the reference's mean|x| and mean x of an observer call, bit for bit
// as torch's CPU kernel sums them on the reference host (mean_cascade.cuh; reference
// quantization_manager.py:66-67).  Opt-in (the manager's mean reference, _hip.py
// set_mean_reference): one extra read of the tensor per call (4 B / element), because
// torch's order cuts the tensor by its CPU threads, which no observer grid follows.
//
//   tiles  (grid: super-tiles x chunks, 256 lanes) every complete level-1 node of every
//          chunk: B x B rows of 4V streams (V = 8: 8192 elements at B = 16).  A lane holds
//          one stream of B / slots level-0 blocks, each a sequential fp32 sum of B rows
//          (loads issued 16 at a time, adds in row order); the B level-0 sums of a stream
//          meet in LDS and one lane sums them in block order -> ws.
//   l2     (grid: level-2 nodes x chunks, 64 lanes) every complete level-2 node: a
//          stream's B level-1 nodes in order.
//   chunks (one 256-lane workgroup per chunk) per stream, in parallel: the trailing
//          complete level-0 blocks, then the four open levels (level 3 = the level-2
//          nodes), ((tail + l1) + l2) + l3; lane 0 then folds the tail vectors, the 4
//          k-streams, the scalar tail and the V lanes -> the chunk's sum.  Every
//          sequential chain loads 16 values at a time (round 6's first form chained up
//          to 1600 dependent loads per lane at one thread: 290 us at 52M elements).
//   final  (one lane) the `threads`-slot second pass, then sum / float(n).
//   std    (with a stats record) torch.std(act(x)) as torch's CPU kernel computes it
//          (ATen std_var_all_cpu, quantization_manager.py:68): the fp32 mean above taken
//          as a double, the sum of (double(v) - mean)^2 in f64, / (n - 1), sqrt, rounded
//          to fp32 once.  The f64 sum's order differs from torch's parallel_reduce, which
//          moves the result ~1e-16 relative: the fp32 rounding absorbs it except when the
//          value straddles a rounding boundary.  kStdParts fixed-order partials (16-B
//          loads, kStdU groups in flight per lane), one fold.
// Both sums (|act(x)| and act(x)) ride the same pass.  HBM: 4 B / element read; the
// level-1 nodes (8 B per 256 elements at V = 8) are written once and read once.
#include "mean_cascade.cuh"

namespace vsiq {
namespace {

struct MeanArgs {
  const float *x;
  int64_t n, cs, nchunks, tiles_max, l2_max;
  MAcc *l1;     // [nchunks][tiles_max][4V]: level-1 nodes
  MAcc *l2;     // [nchunks][l2_max][4V]: complete level-2 nodes
  MAcc *csum;   // [nchunks]
  SiluLay L;
};

// rows / level power / B / tiles of the chunk starting at o
struct ChunkGeo {
  int64_t o, len, nv, rows, B, B2, tiles, l2;   // l2: complete level-2 nodes (B tiles each)
  int lp;
};

__host__ __device__ inline ChunkGeo chunk_geo(int64_t n, int64_t cs, int64_t c, int V) {
  ChunkGeo g;
  g.o = c * cs;
  g.len = n - g.o < cs ? n - g.o : cs;
  g.nv = g.len / V;
  g.rows = g.nv / 4;
  g.lp = mean_level_power(g.rows);
  g.B = (int64_t)1 << g.lp;
  g.B2 = g.B << g.lp;
  g.tiles = g.len < V ? 0 : g.rows / g.B2;
  g.l2 = g.tiles / g.B;
  return g;
}

template <int V, int ACT>
__global__ __launch_bounds__(256) void k_mean_tiles(MeanArgs a) {
  constexpr int S = 4 * V, SLOTS = 256 / S;
  extern __shared__ MAcc l0[];   // [B][S]
  const int64_t c = blockIdx.y, tile = blockIdx.x;
  const ChunkGeo g = chunk_geo(a.n, a.cs, c, V);
  if (tile >= g.tiles) return;   // workgroup-uniform
  const int s = threadIdx.x % S, q = threadIdx.x / S;
  const int64_t e0 = g.o + tile * g.B2 * S + s;   // stream s of the tile's first row
  for (int64_t b = q; b < g.B; b += SLOTS) {
    MAcc acc{0.0f, 0.0f};
    const int64_t eb = e0 + b * g.B * S;
    for (int64_t r = 0; r < g.B; r += 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = a.x[eb + (r + j) * S];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc_add(acc, mean_elem<ACT>(v[j], eb + (r + j) * S, a.L));
    }
    l0[b * S + s] = acc;
  }
  __syncthreads();
  if (q == 0) {
    MAcc l1{0.0f, 0.0f};
    for (int64_t b = 0; b < g.B; ++b) acc_add(l1, l0[b * S + s]);
    a.l1[(c * a.tiles_max + tile) * S + s] = l1;
  }
}

// level-2 nodes: workgroup (d, chunk), lane s: the sequential sum of level-1 nodes
// d*B .. d*B + B - 1 of stream s (loads 16 at a time, adds in node order)
template <int V>
__global__ __launch_bounds__(64) void k_mean_l2(MeanArgs a) {
  constexpr int S = 4 * V;
  const int64_t c = blockIdx.y, d = blockIdx.x;
  const ChunkGeo g = chunk_geo(a.n, a.cs, c, V);
  const int s = threadIdx.x;
  if (d >= g.l2 || s >= S) return;
  const MAcc *l1 = a.l1 + (c * a.tiles_max + d * g.B) * S + s;
  MAcc acc{0.0f, 0.0f};
  for (int64_t k = 0; k < g.B; k += 16) {
    MAcc v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = l1[(k + j) * S];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc_add(acc, v[j]);
  }
  a.l2[(c * a.l2_max + d) * S + s] = acc;
}

// sequential sum (from +0) of m values v(i), loaded 16 at a time
template <class LD>
__device__ __forceinline__ MAcc seq_batched(const LD &v, int64_t m) {
  MAcc acc{0.0f, 0.0f};
  int64_t i = 0;
  for (; i + 16 <= m; i += 16) {
    MAcc t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = v(i + j);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc_add(acc, t[j]);
  }
  for (; i < m; ++i) acc_add(acc, v(i));
  return acc;
}

// one workgroup per chunk: the open levels of every stream in parallel -- slots compute
// the trailing complete level-0 blocks (LDS), then slot 0 / 1 / 2 / 3 of each stream the
// open level 1 (those blocks), open level 2 (level-1 nodes after the last level-2 node),
// level 3 (the level-2 nodes) and the open level 0 (tail rows); ((l0 + l1) + l2) + l3;
// lane 0 then folds the tail vectors, the 4 k-streams, the scalar tail and the V lanes
template <int V, int ACT>
__global__ __launch_bounds__(256) void k_mean_chunks(MeanArgs a) {
  constexpr int S = 4 * V, SLOTS = 256 / S;
  __shared__ MAcc l0r[64 * S];   // trailing complete level-0 blocks (< B <= 64) x streams
  __shared__ MAcc part[4][S];
  const int64_t c = blockIdx.x;
  const ChunkGeo g = chunk_geo(a.n, a.cs, c, V);
  const int s = threadIdx.x % S, q = threadIdx.x / S;
  auto ld = [&](int64_t i) { return mean_elem<ACT>(a.x[g.o + i], g.o + i, a.L); };
  if (g.len < V) {   // a chunk shorter than a vector: row_sum on scalars
    if (threadIdx.x == 0) a.csum[c] = mean_chunk_seq(ld, g.len, V, &l0r[0]);
    return;
  }
  const int64_t r0 = g.tiles * g.B2;              // first row after the complete tiles
  const int64_t rb = (g.rows - r0) / g.B;          // complete level-0 blocks after them
  const int64_t rt = r0 + rb * g.B;                // first tail row
  for (int64_t b = q; b < rb; b += SLOTS)
    l0r[b * S + s] = seq_batched([&](int64_t j) { return ld((r0 + b * g.B + j) * S + s); }, g.B);
  __syncthreads();
  if (q < 4) {
    MAcc v{0.0f, 0.0f};
    if (q == 0) {
      v = seq_batched([&](int64_t b) { return l0r[b * S + s]; }, rb);
    } else if (q == 1) {
      const MAcc *l1 = a.l1 + (c * a.tiles_max + g.l2 * g.B) * S + s;
      v = seq_batched([&](int64_t t) { return l1[t * S]; }, g.tiles - g.l2 * g.B);
    } else if (q == 2) {
      const MAcc *l2 = a.l2 + c * a.l2_max * S + s;
      v = seq_batched([&](int64_t d) { return l2[d * S]; }, g.l2);
    } else {
      v = seq_batched([&](int64_t r) { return ld((rt + r) * S + s); }, g.rows - rt);
    }
    part[q][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < S) {   // ((tail + l1) + l2) + l3 per stream, in LDS for lane 0
    MAcc t = part[3][threadIdx.x];
    acc_add(t, part[0][threadIdx.x]);
    acc_add(t, part[1][threadIdx.x]);
    acc_add(t, part[2][threadIdx.x]);
    l0r[threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MAcc *p = l0r;
    for (int64_t vi = g.rows * 4; vi < g.nv; ++vi)   // tail vectors -> stream k = 0
      for (int l = 0; l < V; ++l) acc_add(p[l], ld(vi * V + l));
    for (int k = 1; k < 4; ++k)
      for (int l = 0; l < V; ++l) acc_add(p[l], p[k * V + l]);
    MAcc fin{0.0f, 0.0f};
    for (int64_t e = g.nv * V; e < g.len; ++e) acc_add(fin, ld(e));
    for (int l = 0; l < V; ++l) acc_add(fin, p[l]);
    a.csum[c] = fin;
  }
}

__global__ __launch_bounds__(64) void k_mean_final(const MAcc *csum, MeanLay m, int V, int threads, int64_t n,
                                                   float *out4, double *stats) {
  __shared__ MAcc buf[kMeanScratch];   // the one lane's accumulators: LDS, not scratch
  if (threadIdx.x != 0) return;
  const MAcc t = mean_final_seq([&](int64_t i) { return csum[i]; }, m, V, threads, buf);
  const float fn = (float)n;
  const float ma = t.a / fn, ms = t.s / fn;
  if (out4) {
    out4[0] = t.a;
    out4[1] = t.s;
    out4[2] = ma;
    out4[3] = ms;
  }
  if (stats) {
    stats[VSIQ_ST_MEANABS] = (double)ma;
    stats[VSIQ_ST_MEAN] = (double)ms;
  }
}

constexpr int kStdParts = 1024;
constexpr int kStdU = 4;   // groups of 4 elements in flight per lane per iteration

// one element's squared deviation in f64 (0 for lanes past the end)
template <int ACT>
__device__ __forceinline__ double std_term(float v, int64_t e, bool valid, double m, const SiluLay &L) {
  const double d = (double)mean_elem<ACT>(v, e, L).s - m;
  return valid ? d * d : 0.0;
}

// kStdParts workgroups stride over the tensor's 4-element groups, kStdU groups per lane
// per iteration (all loads issued before the arithmetic); VEC: 16-B aligned x
template <int ACT, bool VEC>
__global__ __launch_bounds__(256) void k_std_part(const float *__restrict__ x, int64_t n,
                                                  const double *__restrict__ stats, SiluLay L,
                                                  double *__restrict__ part) {
  __shared__ double s_w[256 / kWave];
  const double m = stats[VSIQ_ST_MEAN];   // torch: self.mean().item<double>()
  const int64_t ng = cdiv(n, 4);
  const int64_t stride = (int64_t)gridDim.x * 256;
  double acc = 0.0;
  for (int64_t g0 = (int64_t)blockIdx.x * 256 + threadIdx.x; g0 < ng; g0 += kStdU * stride) {
    f4 v[kStdU];
#pragma unroll
    for (int u = 0; u < kStdU; ++u) v[u] = load_group_c<VEC, true>(x, g0 + u * stride, ng, n);
#pragma unroll
    for (int u = 0; u < kStdU; ++u) {
      const int64_t gi = g0 + u * stride;
      const int nv = gi < ng ? valid_in_group(gi, n) : 0;
      acc += std_term<ACT>(v[u].x, 4 * gi, nv > 0, m, L);
      acc += std_term<ACT>(v[u].y, 4 * gi + 1, nv > 1, m, L);
      acc += std_term<ACT>(v[u].z, 4 * gi + 2, nv > 2, m, L);
      acc += std_term<ACT>(v[u].w, 4 * gi + 3, nv > 3, m, L);
    }
  }
  acc = wave_reduce(acc, AddD());
  if (threadIdx.x % kWave == 0) s_w[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 256 / kWave; ++w) t += s_w[w];
    part[blockIdx.x] = t;
  }
}

// kStdParts / 256 independent loads per lane (issued together), then the block's tree
__global__ __launch_bounds__(256) void k_std_final(const double *__restrict__ part, int64_t n,
                                                   double *__restrict__ stats) {
  static_assert(kStdParts % 256 == 0, "k_std_final: whole rows of partials");
  __shared__ double s_w[256 / kWave];
  double v[kStdParts / 256];
#pragma unroll
  for (int k = 0; k < kStdParts / 256; ++k) v[k] = part[threadIdx.x + 256 * k];
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < kStdParts / 256; ++k) t += v[k];
  t = wave_reduce(t, AddD());
  if (threadIdx.x % kWave == 0) s_w[threadIdx.x / kWave] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 256 / kWave; ++w) t += s_w[w];
    const double dn = (double)n - 1.0;
    const double var = t / (dn > 0.0 ? dn : 0.0);   // n <= 1: 0 / 0 = NaN, as torch
    stats[VSIQ_ST_STD] = (double)(float)__builtin_sqrt(var);
  }
}

template <int ACT>
void launch_std(const float *x, int64_t n, double *stats, const SiluLay &L, double *part, hipStream_t st) {
  if (n % 4 == 0 && aligned16(x))
    hipLaunchKernelGGL((k_std_part<ACT, true>), dim3(kStdParts), dim3(256), 0, st, x, n, stats, L, part);
  else
    hipLaunchKernelGGL((k_std_part<ACT, false>), dim3(kStdParts), dim3(256), 0, st, x, n, stats, L, part);
}

int64_t tiles_max_of(const MeanLay &m, int64_t n, int V) {
  int64_t t = 0;
  if (m.nchunks > 0) {
    t = chunk_geo(n, m.cs, 0, V).tiles;
    const int64_t tl = chunk_geo(n, m.cs, m.nchunks - 1, V).tiles;
    if (tl > t) t = tl;
  }
  return t;
}

int64_t l2_max_of(const MeanLay &m, int64_t n, int V) {
  int64_t t = 0;
  if (m.nchunks > 0) {
    t = chunk_geo(n, m.cs, 0, V).l2;
    const int64_t tl = chunk_geo(n, m.cs, m.nchunks - 1, V).l2;
    if (tl > t) t = tl;
  }
  return t;
}

bool mean_args_ok(int64_t n, int vec, int threads) {
  if (n < 0 || (vec != 8 && vec != 16) || threads < 1 || threads > 4096) return false;
  const MeanLay m = mean_lay(n, threads);
  return m.nchunks == 0 || chunk_geo(n, m.cs, 0, vec).lp <= kMeanMaxLevelPow;
}

template <int V, int ACT>
void launch_mean(const MeanArgs &a, const MeanLay &m, hipStream_t st) {
  constexpr int S = 4 * V;
  if (a.tiles_max > 0) {
    const int64_t B = chunk_geo(a.n, a.cs, 0, V).B;
    const int64_t Bl = chunk_geo(a.n, a.cs, a.nchunks - 1, V).B;
    const size_t lds = (size_t)(B > Bl ? B : Bl) * S * sizeof(MAcc);
    hipLaunchKernelGGL((k_mean_tiles<V, ACT>), dim3((unsigned)a.tiles_max, (unsigned)m.nchunks), dim3(256), lds, st,
                       a);
  }
  if (a.l2_max > 0)
    hipLaunchKernelGGL((k_mean_l2<V>), dim3((unsigned)a.l2_max, (unsigned)m.nchunks), dim3(64), 0, st, a);
  hipLaunchKernelGGL((k_mean_chunks<V, ACT>), dim3((unsigned)m.nchunks), dim3(256), 0, st, a);
}

template <int ACT>
void launch_mean8(const MeanArgs &a, const MeanLay &m, hipStream_t st) {
  launch_mean<8, ACT>(a, m, st);
}

template <int ACT>
void launch_mean16(const MeanArgs &a, const MeanLay &m, hipStream_t st) {
  launch_mean<16, ACT>(a, m, st);
}

}  // namespace

int64_t mean_ws_bytes(int64_t n, int vec, int threads) {
  const MeanLay m = mean_lay(n, threads);
  const int64_t tm = tiles_max_of(m, n, vec), l2 = l2_max_of(m, n, vec);
  return (int64_t)sizeof(MAcc) * (m.nchunks * (tm + l2) * 4 * vec + (m.nchunks > 0 ? m.nchunks : 1)) +
         (int64_t)sizeof(double) * kStdParts;   // the std pass's partials (8-B aligned: MAcc is 8 B)
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int64_t vsiq_torch_mean_ws_bytes(int64_t n, int vec, int threads) {
  if (!mean_args_ok(n, vec, threads)) return -1;
  return mean_ws_bytes(n, vec, threads);
}

int vsiq_torch_mean_f32(const float *x, int64_t n, int act, int vec, int threads, float *out4, double *stats,
                        void *ws, int64_t ws_bytes, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!mean_args_ok(n, vec, threads) || !act_ok(act) || (n > 0 && !x) || !ws || (!out4 && !stats))
    return VSIQ_E_ARG;
  if (ws_bytes < mean_ws_bytes(n, vec, threads)) return VSIQ_E_WS;
  const MeanLay m = mean_lay(n, threads);
  MeanArgs a;
  a.x = x;
  a.n = n;
  a.cs = m.cs;
  a.nchunks = m.nchunks;
  a.tiles_max = tiles_max_of(m, n, vec);
  a.l2_max = l2_max_of(m, n, vec);
  a.l1 = static_cast<MAcc *>(ws);
  a.l2 = a.l1 + m.nchunks * a.tiles_max * 4 * vec;
  a.csum = a.l2 + m.nchunks * a.l2_max * 4 * vec;
  a.L = act_lay(act, n);
  if (m.nchunks > 0) {
    if (vec == 8) VSIQ_ACT(act, launch_mean8, a, m, st);
    else VSIQ_ACT(act, launch_mean16, a, m, st);
  }
  hipLaunchKernelGGL(k_mean_final, dim3(1), dim3(64), 0, st, a.csum, m, vec, threads, n, out4, stats);
  if (stats) {
    double *part = reinterpret_cast<double *>(a.csum + (m.nchunks > 0 ? m.nchunks : 1));
    VSIQ_ACT(act, launch_std, x, n, stats, a.L, part, st);
    hipLaunchKernelGGL(k_std_final, dim3(1), dim3(256), 0, st, part, n, stats);
  }
  return launch_rc();
}

}  // extern "C"
