// k_host.hip — the fake-quant path on the HOST, for CPU tensors: the reference's own
// environment (it runs UniformQuantizer / MinMaxObserver on CPU tensors, BASELINE C1).
// Native C++ loops with the kernels' element arithmetic (vsiq_common.cuh): IEEE fp32
// division, rint (half to even), the NaN-propagating clamp that keeps -0.0, f64 qparams
// with Python round()'s NaN-for-raise convention, and the SiLU exp split of torch's CPU
// kernel.  Work is cut into fixed 64K-element chunks folded in chunk order, so every
// result is independent of the number of host threads (VSIQ_HOST_THREADS, default the
// CPUs this process may run on; a persistent pool).  No activation / ReLU run the
// AVX-512 loops of host_simd.cpp where the CPU has them (elementwise bit-identical to
// the scalar loops; VSIQ_HOST_SIMD=0 forces the scalar ones).  No device memory, no HIP
// calls.
#include <sched.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "host_simd.h"
#include "mean_cascade.cuh"
#include "vsiq_common.cuh"

namespace vsiq {
namespace host {

constexpr int64_t kChunk = 1 << 16;
constexpr int64_t kPoolMinChunks = 4;   // below this the pool's wake-up costs more than it saves
constexpr int kLanes = 16;               // host_simd.cpp's accumulator lanes (one __m512 of fp32)

// VSIQ_HOST_THREADS, else the CPUs this process may run on: the affinity mask capped by
// the cgroup v2 CPU quota (a shared GPU box can grant 16 CPUs' worth of time on a
// 256-CPU affinity mask, and threads beyond the quota only queue behind each other).
inline int usable_cpus() {
  static const int n = [] {
    if (const char *e = std::getenv("VSIQ_HOST_THREADS")) {
      const int v = std::atoi(e);
      if (v > 0) return v;
    }
    int c = (int)std::thread::hardware_concurrency();
    cpu_set_t s;
    if (sched_getaffinity(0, sizeof s, &s) == 0) c = CPU_COUNT(&s);
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long per = 0;
      if (std::fscanf(f, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
        const long long quota = std::atoll(q) / per;
        c = (int)std::min<long long>(c, std::max<long long>(1, quota));
      }
      std::fclose(f);
    }
    return c > 0 ? c : 1;
  }();
  return n;
}

// Persistent workers (created on first use, usable_cpus() - 1 of them; the caller is the
// last): run(nc, f) calls f(0..nc-1), each chunk exactly once, and returns when all are
// done.  A call made while the pool is busy (another thread's host op), in a forked
// child (the workers do not exist there; DataLoader workers fork) or from inside a chunk
// of a running job (a per-channel row's own chunk loop, on a worker or on the caller)
// runs serially; the last case is known from a thread-local flag, without the mutex.
// A job of fewer than kPoolMinChunks chunks runs serially WITHOUT holding the pool, so
// the calls inside its chunks can still use it (2 rows of 50M elements: both rows'
// chunk loops on every worker).
// Every job has its own counters (Job, held by shared_ptr): a worker still inside work()
// for an earlier job only ever touches that job's counters, whose next >= nc, so it can
// neither take a chunk of the new job nor miscount its completion.
class Pool {
 public:
  static Pool &get() {
    static Pool p;
    return p;
  }

  template <class F>
  void run(int64_t nc, F &&f) {
    if (inside_ || nc < kPoolMinChunks || getpid() != pid_ || workers_.empty()) {
      for (int64_t c = 0; c < nc; ++c) f(c);
      return;
    }
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) {
      for (int64_t c = 0; c < nc; ++c) f(c);
      return;
    }
    auto job = std::make_shared<Job>();
    job->fn = [&f](int64_t c) { f(c); };
    job->nc = nc;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    inside_ = true;
    work(*job);
    inside_ = false;
    {
      std::unique_lock<std::mutex> lk(job->mu);
      job->cv.wait(lk, [&] { return job->done.load() == nc; });
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (job_ == job) job_.reset();
  }

  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto &t : workers_)
      if (t.joinable()) t.join();
  }

 private:
  struct Job {
    std::function<void(int64_t)> fn;   // refers to the caller's frame: called only while next < nc
    int64_t nc = 0;
    std::atomic<int64_t> next{0}, done{0};
    std::mutex mu;
    std::condition_variable cv;
  };

  Pool() : pid_(getpid()) {
    const int n = usable_cpus() - 1;
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }

  static void work(Job &j) {   // take chunks of j until none is left
    for (int64_t c; (c = j.next.fetch_add(1)) < j.nc;) {
      j.fn(c);
      if (j.done.fetch_add(1) + 1 == j.nc) {
        std::lock_guard<std::mutex> lk(j.mu);
        j.cv.notify_all();
      }
    }
  }

  void loop() {
    inside_ = true;   // a worker only ever runs chunks of a job
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        j = job_;
      }
      if (j) work(*j);
    }
  }

  static thread_local bool inside_;   // this thread is running a chunk of a job
  const pid_t pid_;
  std::vector<std::thread> workers_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

thread_local bool Pool::inside_ = false;

// f(chunk, begin, end) over the fixed chunks of [0, n)
template <class F>
void for_chunks(int64_t n, F &&f) {
  const int64_t nc = cdiv(n, kChunk);
  Pool::get().run(nc, [&](int64_t c) { f(c, c * kChunk, std::min<int64_t>(n, (c + 1) * kChunk)); });
}

// the AVX-512 loops (host_simd.cpp) for no activation / ReLU on hosts that have them
inline bool use_simd(int kind) {
  static const bool ok = [] {
    const char *e = std::getenv("VSIQ_HOST_SIMD");   // "0" forces the scalar loops
    return simd::available() && !(e && std::strcmp(e, "0") == 0);
  }();
  return ok && kind != kActSilu;
}

inline float act_at(float c, int kind, int64_t e, const SiluLay &L) {
  if (kind == kActRelu) return c < 0.0f ? 0.0f : c;
  if (kind == kActSilu) return (L.on && (silu_scalar4(e, L) & 1u)) ? silu_fwd<true>(c) : silu_fwd<false>(c);
  return c;
}

inline float act_bwd_at(float g, float c, int kind, int64_t e, const SiluLay &L) {
  if (kind == kActRelu) return c <= 0.0f ? 0.0f : g;
  if (kind == kActSilu) return (L.on && (silu_scalar4(e, L) & 1u)) ? silu_bwd<true>(g, c) : silu_bwd<false>(g, c);
  return g;
}

struct HQP {
  float s, z, lo, hi;
};

// uniform.py:98-102 for a learned zero point: clamp(round(zp), qmin, qmax) in f64
inline HQP make_hqp(double s, double z, int zround, int qmin, int qmax) {
  if (zround) {
    const double zr = __builtin_rint(z);
    z = zr < (double)qmin ? (double)qmin : (zr > (double)qmax ? (double)qmax : zr);
  }
  return HQP{(float)s, (float)z, (float)qmin, (float)qmax};
}

// uniform.py:55,95: r = rint(x / s + zp); q = clamp(r); y = (q - zp) * s
inline float fq(float x, const HQP &p, int discrete, bool *m, uint8_t *code) {
  float u = x / p.s;
  u = u + p.z;
  const float r = __builtin_rintf(u);
  const float q = r < p.lo ? p.lo : (r > p.hi ? p.hi : r);
  *m = r >= p.lo && r <= p.hi;
  *code = q == q ? (uint8_t)((int)q & 0xff) : 0;
  return discrete ? q : (q - p.z) * p.s;
}

// One segment of at most kChunk elements, no activation: exactly what the per-tensor
// entry points below do on one chunk (the AVX-512 loop where the CPU has it, else the
// scalar loop in its 16-lane order), so a short row processed here gives the bits of a
// per-tensor call on that row -- without that call's allocation and per-call setup.
// (segments shorter than kSegSimd run the scalar loop: the same bits, without the AVX-512
// call's setup -- an [N, C] activation's rows are one element each)
constexpr int64_t kSegSimd = 64;

inline void fq_seg(const float *x, float *y, uint8_t *mask, int64_t len, const HQP &p) {
  if (len >= kSegSimd && use_simd(kActNone)) {
    simd::fq(x, y, nullptr, mask, len, 0, p.s, p.z, p.lo, p.hi, 0);
    return;
  }
  for (int64_t i = 0; i < len; ++i) {
    bool m;
    uint8_t c;
    y[i] = fq(x[i], p, 0, &m, &c);
    if (mask) mask[i] = m;
  }
}

inline void ste_seg(const float *g, const uint8_t *mask, float *gx, int64_t len, float s) {
  if (len >= kSegSimd && use_simd(kActNone)) {
    simd::ste(g, mask, nullptr, gx, len, 0, s);
    return;
  }
  for (int64_t i = 0; i < len; ++i) gx[i] = (mask[i] ? g[i] * s : 0.0f) / s;
}

// autograd of uniform.py:47-56 term by term (k_body.cuh lsq_elem): gx and {sum t, sum z}
inline void lsq_seg(const float *g, const float *x, float *gx, int64_t len, const HQP &p, int zp_learn,
                    double out[2]) {
  if (len >= kSegSimd && use_simd(kActNone)) {
    simd::lsq(g, x, gx, len, 0, p.s, p.z, p.lo, p.hi, zp_learn, out);
    return;
  }
  double lt[kLanes] = {}, lz[kLanes] = {};
  auto elem = [&](int64_t i, double *st, double *sz) {
    const float u = x[i] / p.s;
    const float r = __builtin_rintf(u + p.z);
    const float q = r < p.lo ? p.lo : (r > p.hi ? p.hi : r);
    const bool m = r >= p.lo && r <= p.hi;
    const float gq = g[i] * p.s;
    const float gm = m ? gq : 0.0f;
    const float t1 = g[i] * (q - p.z);
    const float xs = u / p.s;
    const float t2 = (-gm) * xs;
    *st += (double)t1 + (double)t2;
    if (zp_learn) *sz += (double)gm + (double)(-gq);
    gx[i] = gm / p.s;
  };
  int64_t i = 0;
  for (; i + kLanes <= len; i += kLanes)
    for (int k = 0; k < kLanes; ++k) elem(i + k, &lt[k], &lz[k]);
  double st = 0.0, sz = 0.0;
  for (int k = 0; k < kLanes; ++k) st += lt[k], sz += lz[k];
  for (; i < len; ++i) elem(i, &st, &sz);
  out[0] = st;
  out[1] = sz;
}

// rows of at most kChunk elements: blocks of whole rows (~kChunk elements each) on the
// pool, each row one segment call with its channel's qparams
template <class F>
void short_rows(int64_t rows, int64_t rowlen, F &&row) {
  const int64_t per = std::max<int64_t>(1, kChunk / std::max<int64_t>(1, rowlen));
  Pool::get().run(cdiv(rows, per), [&](int64_t b) {
    const int64_t r1 = std::min(rows, (b + 1) * per);
    for (int64_t r = b * per; r < r1; ++r) row(r);
  });
}

}  // namespace host
}  // namespace vsiq

using namespace vsiq;
using namespace vsiq::host;

extern "C" {

int vsiq_host_observe_f32(const float *x, int64_t n, int act, double *stats_out, float *run_minmax, double *qp_out,
                          int symmetric, double qden, double eps) {
  if (n <= 0 || !x || !act_ok(act)) return VSIQ_E_ARG;
  const int kind = act_kind(act);
  const SiluLay L = act_lay(act, n);
  const int64_t nc = cdiv(n, kChunk);
  std::vector<double> part((size_t)nc * 6);
  const bool vec = use_simd(kind);
  for_chunks(n, [&](int64_t c, int64_t b, int64_t e) {
    if (vec) {
      simd::observe(x + b, e - b, kind == kActRelu, &part[(size_t)c * 6]);
      return;
    }
    // host_simd.cpp's order: 16 lanes (element i + k into lane k) over the whole 16-blocks,
    // folded in lane order, then the tail in sequence -- so the scalar and AVX-512 loops
    // give the same sums and the same signed-zero min/max
    float lmn[kLanes], lmx[kLanes];
    double lsa[kLanes] = {}, ls1[kLanes] = {}, ls2[kLanes] = {}, lnan[kLanes] = {};
    for (int k = 0; k < kLanes; ++k) lmn[k] = __builtin_inff(), lmx[k] = -__builtin_inff();
    int64_t i = b;
    for (; i + kLanes <= e; i += kLanes)
      for (int k = 0; k < kLanes; ++k) {
        const float v = act_at(x[i + k], kind, i + k, L);
        if (v != v) lnan[k] += 1.0;
        lmn[k] = v < lmn[k] ? v : lmn[k];
        lmx[k] = v > lmx[k] ? v : lmx[k];
        const double d = (double)v;
        lsa[k] += __builtin_fabs(d);
        ls1[k] += d;
        ls2[k] += d * d;
      }
    float mn = __builtin_inff(), mx = -__builtin_inff();
    double nan = 0.0, sa = 0.0, s1 = 0.0, s2 = 0.0;
    for (int k = 0; k < kLanes; ++k) {
      mn = lmn[k] < mn ? lmn[k] : mn;
      mx = lmx[k] > mx ? lmx[k] : mx;
      nan += lnan[k];
      sa += lsa[k];
      s1 += ls1[k];
      s2 += ls2[k];
    }
    for (; i < e; ++i) {
      const float v = act_at(x[i], kind, i, L);
      if (v != v) {
        nan += 1.0;
      } else {
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
      }
      const double d = (double)v;
      sa += __builtin_fabs(d);
      s1 += d;
      s2 += d * d;
    }
    double *p = &part[(size_t)c * 6];
    p[0] = mn; p[1] = mx; p[2] = nan; p[3] = sa; p[4] = s1; p[5] = s2;
  });
  double f[6] = {__builtin_inf(), -__builtin_inf(), 0.0, 0.0, 0.0, 0.0};
  for (int64_t c = 0; c < nc; ++c) {   // chunk order: independent of the thread count
    const double *p = &part[(size_t)c * 6];
    f[0] = p[0] < f[0] ? p[0] : f[0];
    f[1] = p[1] > f[1] ? p[1] : f[1];
    f[2] += p[2]; f[3] += p[3]; f[4] += p[4]; f[5] += p[5];
  }
  if (stats_out) write_stats(stats_out, f, n);
  observer_update((float)f[0], (float)f[1], f[2] > 0.0, run_minmax, qp_out, symmetric, qden, eps);
  return 0;
}

int vsiq_host_fq_fwd_f32(const float *x, float *y, uint8_t *codes, uint8_t *mask, int64_t n, int act,
                         const double *qp, double scale, double zp, int zp_round, int discrete, int qmin,
                         int qmax) {
  if (n < 0 || qmin > qmax || (n > 0 && (!x || !y)) || !act_ok(act)) return VSIQ_E_ARG;
  const HQP p = qp ? make_hqp(qp[VSIQ_QP_SCALE], qp[VSIQ_QP_ZP], 0, qmin, qmax)
                   : make_hqp(scale, zp, zp_round, qmin, qmax);
  const int kind = act_kind(act);
  const SiluLay L = act_lay(act, n);
  const bool vec = use_simd(kind);
  for_chunks(n, [&](int64_t, int64_t b, int64_t e) {
    if (vec) {
      simd::fq(x + b, y + b, codes ? codes + b : nullptr, mask ? mask + b : nullptr, e - b, kind == kActRelu, p.s,
               p.z, p.lo, p.hi, discrete);
      return;
    }
    for (int64_t i = b; i < e; ++i) {
      bool m;
      uint8_t c;
      y[i] = fq(act_at(x[i], kind, i, L), p, discrete, &m, &c);
      if (mask) mask[i] = m;
      if (codes) codes[i] = c;
    }
  });
  return 0;
}

int vsiq_host_ste_bwd_f32(const float *g, const uint8_t *mask, const float *pre, float *gx, int64_t n, int act,
                          double scale) {
  if (n < 0 || (n > 0 && (!g || !mask || !gx)) || !act_ok(act) || (act_kind(act) != kActNone && !pre))
    return VSIQ_E_ARG;
  const float s = (float)scale;
  const int kind = act_kind(act);
  const SiluLay L = act_lay(act, n);
  const bool vec = use_simd(kind);
  for_chunks(n, [&](int64_t, int64_t b, int64_t e) {
    if (vec) {
      simd::ste(g + b, mask + b, pre ? pre + b : nullptr, gx + b, e - b, kind == kActRelu, s);
      return;
    }
    for (int64_t i = b; i < e; ++i) {
      const float o = (mask[i] ? g[i] * s : 0.0f) / s;   // MulBackward0, ClampBackward1, DivBackward0
      gx[i] = kind == kActNone ? o : act_bwd_at(o, pre[i], kind, i, L);
    }
  });
  return 0;
}

int vsiq_host_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t n, int act, double scale, double zp,
                          int zp_learn, int qmin, int qmax, double gscale, double *grad_out) {
  if (n <= 0 || !g || !x || !gx || !grad_out || qmin > qmax || !act_ok(act) || zp_learn < 0 || zp_learn > 2)
    return VSIQ_E_ARG;
  const HQP p = make_hqp(scale, zp, zp_learn == 1, qmin, qmax);
  const int kind = act_kind(act);
  const SiluLay L = act_lay(act, n);
  const int64_t nc = cdiv(n, kChunk);
  std::vector<double> part((size_t)nc * 2);
  const bool vec = use_simd(kind);
  for_chunks(n, [&](int64_t c, int64_t b, int64_t e) {
    if (vec) {
      simd::lsq(g + b, x + b, gx + b, e - b, kind == kActRelu, p.s, p.z, p.lo, p.hi, zp_learn, &part[(size_t)c * 2]);
      return;
    }
    // autograd of uniform.py:47-56, term by term (k_body.cuh lsq_elem); the sums in
    // host_simd.cpp's 16-lane order (see the observer above)
    double lt[kLanes] = {}, lz[kLanes] = {};
    auto elem = [&](int64_t i, double *st, double *sz) {
      const float xa = act_at(x[i], kind, i, L);
      const float u = xa / p.s;
      const float r = __builtin_rintf(u + p.z);
      const float q = r < p.lo ? p.lo : (r > p.hi ? p.hi : r);
      const bool m = r >= p.lo && r <= p.hi;
      const float gq = g[i] * p.s;
      const float gm = m ? gq : 0.0f;
      const float t1 = g[i] * (q - p.z);
      const float xs = u / p.s;
      const float t2 = (-gm) * xs;
      *st += (double)t1 + (double)t2;
      if (zp_learn) *sz += (double)gm + (double)(-gq);
      const float o = gm / p.s;
      gx[i] = kind == kActNone ? o : act_bwd_at(o, x[i], kind, i, L);
    };
    int64_t i = b;
    for (; i + kLanes <= e; i += kLanes)
      for (int k = 0; k < kLanes; ++k) elem(i + k, &lt[k], &lz[k]);
    double st = 0.0, sz = 0.0;
    for (int k = 0; k < kLanes; ++k) st += lt[k], sz += lz[k];
    for (; i < e; ++i) elem(i, &st, &sz);
    part[(size_t)c * 2] = st;
    part[(size_t)c * 2 + 1] = sz;
  });
  double t = 0.0, z = 0.0;
  for (int64_t c = 0; c < nc; ++c) {
    t += part[(size_t)c * 2];
    z += part[(size_t)c * 2 + 1];
  }
  grad_out[0] = t * gscale;
  if (zp_learn == 2) {   // zp as given, no ScaleGradient (symmetric quantizer, k_body.cuh lsq_grad_zp)
    grad_out[1] = z;
  } else if (zp_learn) {   // ClampBackward of zero_point_rounding: the in-range test on round(zp)
    const double zr = __builtin_rint(zp);
    grad_out[1] = (zr >= (double)qmin && zr <= (double)qmax) ? z * gscale : 0.0;
  } else {
    grad_out[1] = 0.0;
  }
  return 0;
}

// Per-channel (axis 0, rows = out-channels) host loops: PerChannelMinMaxObserver /
// PerChannelUniformQuantizer on CPU tensors.  SURVEY §0.2 defines per channel as the
// reference classes applied to each row W[c] (observers/minmax.py:42-74 with a running
// state per row, quantizers/uniform.py:34-56 / 95 with the row's qparams), so every row
// runs exactly the per-tensor host code above (the same bits as vsiq_host_observe_f32 /
// _fq_fwd_f32 / _ste_bwd_f32 / _lsq_bwd_f32 on that row alone).  Rows go to the pool
// (a row's own chunk loop then runs serially inside it), or, for fewer than
// kPoolMinChunks rows, one after the other with the pool inside each row.
int vsiq_host_pc_observe_fq_f32(const float *x, float *y, uint8_t *mask, int64_t rows, int64_t rowlen,
                                float *run_min, float *run_max, double *scale_out, double *zp_out,
                                double *row_stats, int symmetric, double qden, double eps, int qmin, int qmax) {
  if (rows <= 0 || rowlen <= 0 || !x || !run_min || !run_max || !scale_out || !zp_out || qmin > qmax)
    return VSIQ_E_ARG;
  std::atomic<int> rc{0};
  Pool::get().run(rows, [&](int64_t r) {
    const float *xr = x + r * rowlen;
    float st[2] = {run_min[r], run_max[r]};
    double qp[VSIQ_QP_LEN], stats[VSIQ_ST_LEN];
    int e = vsiq_host_observe_f32(xr, rowlen, kActNone, stats, st, qp, symmetric, qden, eps);
    run_min[r] = st[0];
    run_max[r] = st[1];
    scale_out[r] = qp[VSIQ_QP_SCALE];
    zp_out[r] = qp[VSIQ_QP_ZP];
    if (row_stats) {
      row_stats[3 * r] = stats[VSIQ_ST_SUMABS];
      row_stats[3 * r + 1] = stats[VSIQ_ST_SUM];
      row_stats[3 * r + 2] = stats[VSIQ_ST_SUMSQ];
    }
    if (!e && y)
      e = vsiq_host_fq_fwd_f32(xr, y + r * rowlen, nullptr, mask ? mask + r * rowlen : nullptr, rowlen, kActNone,
                               qp, 0.0, 0.0, 0, 0, qmin, qmax);
    if (e) rc.store(e);
  });
  return rc.load();
}

int vsiq_host_pc_fq_fwd_f32(const float *x, float *y, uint8_t *mask, int64_t rows, int64_t rowlen,
                            const double *scale, const double *zp, int zp_round, int qmin, int qmax) {
  return vsiq_host_pcm_fq_fwd_f32(x, y, mask, rows, rowlen, rows > 0 ? rows : 1, scale, zp, zp_round, qmin, qmax);
}

int vsiq_host_pc_ste_bwd_f32(const float *g, const uint8_t *mask, float *gx, int64_t rows, int64_t rowlen,
                             const double *scale) {
  return vsiq_host_pcm_ste_bwd_f32(g, mask, gx, rows, rowlen, rows > 0 ? rows : 1, scale);
}

int vsiq_host_pc_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                             const double *scale, const double *zp, int zp_learn, int qmin, int qmax, double gscale,
                             double *grad_scale_out, double *grad_zp_out) {
  return vsiq_host_pcm_lsq_bwd_f32(g, x, gx, rows, rowlen, rows, scale, zp, zp_learn, qmin, qmax, gscale,
                                   grad_scale_out, grad_zp_out);
}

// Axis 1 ([N, C, ...]): row r = n * channels + c in channel c, each row the per-tensor host
// call with its channel's qparams; the learnable gradients summed per channel over its
// rows in row order (f64), then times gscale once -- for channels == rows exactly the
// per-row t * gscale of vsiq_host_lsq_bwd_f32.
int vsiq_host_pcm_fq_fwd_f32(const float *x, float *y, uint8_t *mask, int64_t rows, int64_t rowlen, int64_t channels,
                             const double *scale, const double *zp, int zp_round, int qmin, int qmax) {
  if (rows < 0 || rowlen < 0 || channels <= 0 || rows % channels || (rows > 0 && (!x || !y || !scale)) ||
      qmin > qmax)
    return VSIQ_E_ARG;
  if (rowlen <= kChunk) {   // short rows (an [N, C] activation: one element each): no per-row call
    std::vector<HQP> hq((size_t)channels);
    for (int64_t c = 0; c < channels; ++c) hq[(size_t)c] = make_hqp(scale[c], zp ? zp[c] : 0.0, zp_round, qmin, qmax);
    short_rows(rows, rowlen, [&](int64_t r) {
      const int64_t o = r * rowlen;
      fq_seg(x + o, y + o, mask ? mask + o : nullptr, rowlen, hq[(size_t)(r % channels)]);
    });
    return 0;
  }
  std::atomic<int> rc{0};
  Pool::get().run(rows, [&](int64_t r) {
    const int64_t c = r % channels;
    const int e = vsiq_host_fq_fwd_f32(x + r * rowlen, y + r * rowlen, nullptr, mask ? mask + r * rowlen : nullptr,
                                       rowlen, kActNone, nullptr, scale[c], zp ? zp[c] : 0.0, zp_round, 0, qmin,
                                       qmax);
    if (e) rc.store(e);
  });
  return rc.load();
}

int vsiq_host_pcm_ste_bwd_f32(const float *g, const uint8_t *mask, float *gx, int64_t rows, int64_t rowlen,
                              int64_t channels, const double *scale) {
  if (rows < 0 || rowlen < 0 || channels <= 0 || rows % channels || (rows > 0 && (!g || !mask || !gx || !scale)))
    return VSIQ_E_ARG;
  if (rowlen <= kChunk) {
    short_rows(rows, rowlen, [&](int64_t r) {
      const int64_t o = r * rowlen;
      ste_seg(g + o, mask + o, gx + o, rowlen, (float)scale[r % channels]);
    });
    return 0;
  }
  std::atomic<int> rc{0};
  Pool::get().run(rows, [&](int64_t r) {
    const int64_t o = r * rowlen;
    const int e = vsiq_host_ste_bwd_f32(g + o, mask + o, nullptr, gx + o, rowlen, kActNone, scale[r % channels]);
    if (e) rc.store(e);
  });
  return rc.load();
}

int vsiq_host_pcm_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                              int64_t channels, const double *scale, const double *zp, int zp_learn, int qmin, int qmax,
                              double gscale, double *grad_scale_out, double *grad_zp_out) {
  if (rows <= 0 || rowlen <= 0 || channels <= 0 || rows % channels || !g || !x || !gx || !scale || !grad_scale_out ||
      qmin > qmax || (zp_learn && !zp) || zp_learn < 0 || zp_learn > 1)
    return VSIQ_E_ARG;
  std::atomic<int> rc{0};
  const int64_t per = std::max<int64_t>(1, kChunk / rowlen), nb = cdiv(rows, per);
  if (rowlen < kSegSimd && nb * channels <= ((int64_t)1 << 24)) {
    // short rows (an [N, C] activation: one element each): blocks of ~kChunk elements of
    // whole rows on the pool; each block sums its rows per channel in row order, the
    // blocks fold in block order (fixed blocks: independent of the thread count)
    std::vector<HQP> hq((size_t)channels);
    std::vector<char> zok((size_t)channels, 0);
    for (int64_t c = 0; c < channels; ++c) {
      hq[(size_t)c] = make_hqp(scale[c], zp ? zp[c] : 0.0, zp_learn, qmin, qmax);
      if (zp_learn) {   // ClampBackward of the rounded zero point (lsq_module.py:339-343)
        const double zr = __builtin_rint(zp[c]);
        zok[(size_t)c] = zr >= (double)qmin && zr <= (double)qmax;
      }
    }
    std::vector<double> blk((size_t)(nb * channels * 2), 0.0);
    Pool::get().run(nb, [&](int64_t b) {
      double *acc = &blk[(size_t)(b * channels * 2)];
      const int64_t r1 = std::min(rows, (b + 1) * per);
      for (int64_t r = b * per; r < r1; ++r) {
        const int64_t o = r * rowlen, c = r % channels;
        double t[2];
        lsq_seg(g + o, x + o, gx + o, rowlen, hq[(size_t)c], zp_learn, t);
        acc[c * 2] += t[0];
        if (zok[(size_t)c]) acc[c * 2 + 1] += t[1];
      }
    });
    for (int64_t c = 0; c < channels; ++c) {
      double ts = 0.0, zs = 0.0;
      for (int64_t b = 0; b < nb; ++b) {
        ts += blk[(size_t)((b * channels + c) * 2)];
        zs += blk[(size_t)((b * channels + c) * 2 + 1)];
      }
      grad_scale_out[c] = ts * gscale;
      if (grad_zp_out) grad_zp_out[c] = zs * gscale;
    }
    return 0;
  }
  std::vector<double> part((size_t)rows * 2);
  Pool::get().run(rows, [&](int64_t r) {
    const int64_t o = r * rowlen, c = r % channels;
    const int e = vsiq_host_lsq_bwd_f32(g + o, x + o, gx + o, rowlen, kActNone, scale[c], zp ? zp[c] : 0.0,
                                        zp_learn, qmin, qmax, 1.0, &part[(size_t)r * 2]);
    if (e) rc.store(e);
  });
  // row order per channel (independent of the thread count), one sequential pass
  std::vector<double> acc((size_t)channels * 2, 0.0);
  for (int64_t r = 0; r < rows; ++r) {
    const size_t c = (size_t)(r % channels);
    acc[c * 2] += part[(size_t)r * 2];
    acc[c * 2 + 1] += part[(size_t)r * 2 + 1];
  }
  for (int64_t c = 0; c < channels; ++c) {
    grad_scale_out[c] = acc[(size_t)c * 2] * gscale;
    if (grad_zp_out) grad_zp_out[c] = acc[(size_t)c * 2 + 1] * gscale;
  }
  return rc.load();
}

// K11 on the host: torch CPU's mean|act(x)| / mean act(x) bits (mean_cascade.cuh), the
// chunks of torch's layout on the pool, the second pass in slot order
int vsiq_host_torch_mean_f32(const float *x, int64_t n, int act, int vec, int threads, float *out4) {
  if (n < 0 || (n > 0 && !x) || !out4 || (vec != 8 && vec != 16) || threads < 1 || threads > 4096 ||
      !act_ok(act))
    return VSIQ_E_ARG;
  const MeanLay m = mean_lay(n, threads);
  const SiluLay L = act_lay(act, n);
  std::vector<MAcc> cs((size_t)(m.nchunks > 0 ? m.nchunks : 1));
  auto chunk = [&](int64_t c) {
    MAcc buf[kMeanScratch];
    const int64_t o = c * m.cs, len = std::min(m.cs, n - o);
    switch (act_kind(act)) {
      case kActRelu:
        cs[c] = mean_chunk_seq([&](int64_t i) { return mean_elem<kActRelu>(x[o + i], o + i, L); }, len, vec, buf);
        break;
      case kActSilu:
        cs[c] = mean_chunk_seq([&](int64_t i) { return mean_elem<kActSilu>(x[o + i], o + i, L); }, len, vec, buf);
        break;
      default:
        cs[c] = mean_chunk_seq([&](int64_t i) { return mean_elem<kActNone>(x[o + i], o + i, L); }, len, vec, buf);
    }
  };
  Pool::get().run(m.nchunks, chunk);
  MAcc buf[kMeanScratch];
  const MAcc t = mean_final_seq([&](int64_t i) { return cs[(size_t)i]; }, m, vec, threads, buf);
  out4[0] = t.a;
  out4[1] = t.s;
  out4[2] = t.a / (float)n;
  out4[3] = t.s / (float)n;
  return 0;
}

int vsiq_host_threads(void) { return usable_cpus(); }

int vsiq_host_simd(void) { return use_simd(kActNone) ? 1 : 0; }

}  // extern "C"
