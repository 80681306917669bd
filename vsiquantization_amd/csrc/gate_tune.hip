// gate_tune.hip — online tuner of the one-round store gate (store_gate_select in
// vsiq_common.cuh).  Host code only.
//
// A launch site is (kernel, grid, read bytes, device).  Its first launches cycle
// through candidate gates f x (read bytes at 7.5 TB/s), and no gate, each bracketed by
// a pair of HIP events on the launch stream; later calls harvest finished pairs
// (hipEventQuery, never a host sync; the events skip the system-scope fence, so timing a
// launch neither writes back / invalidates the caches nor slows the launches after it),
// and once every candidate has kSamples times, the kFinal candidates with the smallest
// medians are timed kSamples more each (round 5: neighbouring gates differ by less than
// the spread of 8 samples on some boxes) and the smallest median over all of a
// finalist's samples wins and is used from then on.  The candidates are issued in a
// fresh pseudo-random order every pass (round 5): sites launched alternately (K3 then the
// STE backward in a training step) would otherwise always time candidate i of one site
// right after candidate i of the other, and a gate's median would carry its partner's
// tail.
//
// Bursts (round 5): where a site is launched back to back -- the next launch of the same
// site is the next launch of this library (g_lib_launches: an untuned kernel in between,
// e.g. a larger layer's, ends the burst), on the same stream, within kBurstGapUs of host
// time -- a sample spans up to kBurst consecutive launches with the same gate and counts
// the mean of their durations.  Each launch of a burst has its own pair of events (round
// 6): kernels of other libraries (torch, MIOpen) queued on the stream between two
// launches of the burst are outside every pair, so they never enter a sample.  A lone launch's timing
// includes how the GPU comes out of the previous, different kernel; launches that stream
// back to back (a bench's group of one kernel, several layers of one shape in a row)
// have a different, sharper optimum (tools/exp/c2_floor.py: K3 at C2 12.0 us at 518
// ticks, 12.95 at 557, where lone-launch medians were flat within their noise).  A
// training step's launches of one site are a step apart: their samples stay single.  All state is behind one mutex
// (autograd's backward thread launches too); launches under HIP-graph capture take the
// current choice and are never timed.
//
// Drift (round 3): a tuned site keeps timing one launch in kWatchEvery; when the median of
// kWatch such samples moves more than kDrift from the winner's tuned median (the load
// around the launches changed: RCCL or conv kernels overlapping the quantizers in a real
// step, a different clock state), the site tunes again.  vsiq_gate_retune() re-tunes
// every site on demand (e.g. once a training loop is warm).  A re-tune needs two drifting
// checks in a row, and one that lands on the gate the site had already doubles that
// site's watch interval (up to kWatchMax): a site whose launches simply vary with the
// caller's pace (isolated per-call launches vs back-to-back ones) stops paying for timing
// and re-tuning.  The gate is a delay only: results are bit-identical whatever it is.
#include "vsiq_common.cuh"

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace vsiq {
namespace {

constexpr double kFactors[] = {0.0, 0.90, 0.95, 0.975, 1.0, 1.025, 1.05, 1.075, 1.10, 1.15, 1.20, 1.30};
constexpr int kCand = sizeof(kFactors) / sizeof(kFactors[0]);
constexpr int kSamples = 8;        // timed launches per candidate
constexpr int kFinal = 3;          // finalists of the refinement round, kSamples more each
constexpr double kDefault = 1.05;  // before (or without) tuning
constexpr double kCapUs = 40.0;
constexpr int kWatchEvery = 128;   // a tuned site times one launch in this many
constexpr int kWatchMax = 128 * 64;
constexpr int kWatch = 8;          // samples per drift check
constexpr double kDrift = 0.15;    // relative change of the median that triggers re-tuning
constexpr int kBurst = 4;          // launches per burst sample
constexpr double kBurstGapUs = 25.0;   // host time between the launches of a burst, at most

struct Site {
  std::string label;
  std::string table_key;            // "<kernel symbol> <grid> <bytes>": the saved-table key
  bool preset = false;              // gate taken from a loaded table (never timed)
  int64_t grid = 0, bytes = 0;
  int dev = 0;
  double est = 0.0;                 // ticks of read bytes at 7.5 TB/s
  uint32_t ticks[kCand] = {};
  std::vector<float> ms[kCand];
  int issued[kCand] = {};
  int perm[kCand] = {};             // this pass's issue order
  int pos = kCand;                  // next index into perm (kCand: reshuffle)
  uint64_t rng = 0;                 // xorshift state, seeded per site
  bool refine = false;              // the finalists' round
  int target[kCand] = {};           // samples wanted per candidate in this round
  bool done = false;
  uint32_t best = 0;
  float best_ms = 0.0f;             // the winner's median when tuned
  std::vector<float> watch;         // drift samples of the chosen gate
  int since_watch = 0;
  int watch_every = kWatchEvery;
  int drifting = 0;                 // consecutive drifting checks
  uint32_t prev_best = 0;           // the gate before the running re-tune
  int retunes = 0;
  int gen = 0;                      // tuning round: retune() starts a new one
  uint64_t last_sel = 0;            // g_sel when this site was last launched
  struct Sample *open = nullptr;    // burst in progress (not in g_pending yet)
  uint64_t open_sel = 0;            // g_sel at the burst's last launch
  uint64_t open_lib = 0;            // g_lib_launches at the burst's last launch
  std::chrono::steady_clock::time_point open_t;   // host time of the burst's last launch
};

struct Sample {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;   // start / end per launch; ev[0..n) recorded
  Site *site = nullptr;
  int cand = 0;   // -1: a drift sample of the tuned gate
  int dev = 0;
  int gen = 0;    // the site's tuning round when issued: samples of an earlier round are dropped
  int n = 0;      // launches recorded (a select in flight has pushed ev[n] already)
  hipStream_t st = nullptr;
};

double us_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
}

using Key = std::tuple<const void *, int64_t, int64_t, int>;

std::mutex g_mu;
std::map<Key, Site> g_sites;
std::vector<Sample *> g_pending;
std::map<int, std::vector<std::pair<hipEvent_t, hipEvent_t>>> g_pool;
uint64_t g_sel = 0;    // launches through the tuner (a clock for "launched since")
uint64_t g_mark = 0;   // g_sel at the previous vsiq_gate_tuning_pending()
uint32_t clamp_ticks(double t, int khz) {
  const double cap = kCapUs * khz / 1e3;
  return (uint32_t)std::max(0.0, std::min(cap, t));
}

float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n % 2 ? v[n / 2] : 0.5f * (v[n / 2 - 1] + v[n / 2]);
}

// Gate table (round 6): gates loaded with vsiq_gate_import, by table key; frozen: no
// launch is ever timed (a loaded site keeps its gate, a site missing from the table runs
// the fixed default), so a process's timing does not depend on tuner state.
std::map<std::string, uint32_t> g_preset;
bool g_frozen = false;

// "<kernel host-stub symbol> <grid> <read bytes>": stable across processes of the same
// build (the stubs are exported; dladdr names them), unlike the stub's address
std::string table_key(const char *label, const void *kernel, int64_t grid, int64_t bytes) {
  Dl_info info;
  const char *name = (dladdr(kernel, &info) != 0 && info.dli_sname) ? info.dli_sname : label;
  char tail[64];
  std::snprintf(tail, sizeof tail, " %lld %lld", (long long)grid, (long long)bytes);
  return std::string(name) + tail;
}

// caller holds g_mu: a site with a loaded gate is tuned; in a frozen table a site
// without one keeps the default and is never timed
void apply_preset(Site &s, int khz) {
  auto it = g_preset.find(s.table_key);
  if (it != g_preset.end()) {
    s.best = it->second;
    s.preset = true;
  } else if (g_frozen) {
    s.best = clamp_ticks(kDefault * s.est, khz);
  } else {
    return;
  }
  s.done = true;
  s.best_ms = 0.0f;
  s.watch.clear();
  s.since_watch = 0;
  s.drifting = 0;
}

void start_round(Site &s) {
  for (int c = 0; c < kCand; ++c) s.target[c] = kSamples;
  s.refine = false;
}

void finish_if_complete(Site &s) {
  if (s.done) return;
  for (int c = 0; c < kCand; ++c)
    if ((int)s.ms[c].size() < s.target[c]) return;
  if (!s.refine) {   // coarse round complete: the kFinal best medians get kSamples more
    int order[kCand];
    float med[kCand];
    for (int c = 0; c < kCand; ++c) order[c] = c, med[c] = median(s.ms[c]);
    std::stable_sort(order, order + kCand, [&](int a, int b) { return med[a] < med[b]; });
    for (int k = 0; k < kFinal; ++k) s.target[order[k]] = 2 * kSamples;
    s.refine = true;
    return;
  }
  int bc = -1;
  float bm = 0.0f;
  for (int c = 0; c < kCand; ++c) {
    if (s.target[c] <= kSamples) continue;   // not a finalist
    const float m = median(s.ms[c]);
    if (bc < 0 || m < bm) { bm = m; bc = c; }
  }
  s.best = s.ticks[bc];
  s.best_ms = bm;
  s.done = true;
  s.watch.clear();
  s.since_watch = 0;
  s.drifting = 0;
  if (s.retunes > 0 && s.best == s.prev_best) s.watch_every = std::min(2 * s.watch_every, kWatchMax);
}

void retune(Site &s) {
  for (int c = 0; c < kCand; ++c) {
    s.ms[c].clear();
    s.issued[c] = 0;
  }
  start_round(s);
  s.pos = kCand;
  s.prev_best = s.best;
  s.done = false;
  s.watch.clear();
  s.since_watch = 0;
  s.drifting = 0;
  ++s.retunes;
  ++s.gen;   // timings still in flight belong to the old round (taken under the old load)
}

void watch_sample(Site &s, float ms) {
  if (!s.done) return;   // re-tuning already
  s.watch.push_back(ms);
  if ((int)s.watch.size() < kWatch) return;
  const float m = median(s.watch);
  s.watch.clear();
  const bool drift = s.best_ms > 0.0f && (m > (1.0 + kDrift) * s.best_ms || m < (1.0 - kDrift) * s.best_ms);
  s.drifting = drift ? s.drifting + 1 : 0;
  if (s.drifting >= 2) retune(s);
}

// caller holds g_mu: a start / end event pair for one timed launch (pooled per device)
bool take_pair(int dev, std::pair<hipEvent_t, hipEvent_t> &ev) {
  auto &pool = g_pool[dev];
  if (!pool.empty()) {
    ev = pool.back();
    pool.pop_back();
    return true;
  }
  ev = {nullptr, nullptr};
  if (hipEventCreateWithFlags(&ev.first, hipEventDisableSystemFence) != hipSuccess ||
      hipEventCreateWithFlags(&ev.second, hipEventDisableSystemFence) != hipSuccess) {
    (void)hipGetLastError();
    if (ev.first) (void)hipEventDestroy(ev.first);
    return false;
  }
  return true;
}

// caller holds g_mu: an open burst becomes a sample to harvest
void close_burst_locked(Site &s) {
  if (!s.open) return;
  g_pending.push_back(s.open);
  s.open = nullptr;
}

// caller holds g_mu; all: every open burst, else those whose last launch is past the gap
void close_bursts_locked(bool all) {
  for (auto &kv : g_sites)
    if (kv.second.open && (all || us_since(kv.second.open_t) >= kBurstGapUs)) close_burst_locked(kv.second);
}

// caller holds g_mu
void harvest_locked() {
  size_t keep = 0;
  for (size_t i = 0; i < g_pending.size(); ++i) {
    Sample *p = g_pending[i];
    const hipError_t q = p->n > 0 ? hipEventQuery(p->ev[p->n - 1].second) : hipErrorInvalidValue;
    if (q == hipErrorNotReady) {
      g_pending[keep++] = p;
      continue;
    }
    float ms = 0.0f;
    bool ok = q == hipSuccess;
    for (int k = 0; ok && k < p->n; ++k) {   // one stream: the last end done -> every pair done
      float d = 0.0f;
      ok = hipEventElapsedTime(&d, p->ev[k].first, p->ev[k].second) == hipSuccess && d > 0.0f;
      ms += d;
    }
    const bool current = p->gen == p->site->gen;
    if (ok) {
      ms /= (float)p->n;
      if (!current) {
        // a sample of the round before a re-tune: not counted in the new round's issued[]
      } else if (p->cand < 0) {
        watch_sample(*p->site, ms);
      } else if (!p->site->done) {
        p->site->ms[p->cand].push_back(ms);
        finish_if_complete(*p->site);
      }
      for (auto &e : p->ev) g_pool[p->dev].push_back(e);
    } else {
      if (current && p->cand >= 0 && !p->site->done) p->site->issued[p->cand]--;   // lost sample: issue again
      (void)hipGetLastError();
    }
    delete p;
  }
  g_pending.resize(keep);
}

}  // namespace

std::atomic<uint64_t> g_lib_launches{0};

GateSel store_gate_select(const char *label, const void *kernel, int64_t grid, int occ, int64_t read_bytes,
                          hipStream_t st) {
  GateSel sel;
  const int forced = g_tune.store_gate;
  if (forced >= 0) {
    sel.gate = (uint32_t)forced;
    return sel;
  }
  int dev = 0;   // one device query per launch (the attribute caches are per device)
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    dev = -1;
  }
  const int64_t cus = device_cus(dev);
  if (grid < 2 * cus || occ <= 0 || grid > (int64_t)occ * cus) return sel;
  const int khz = device_wall_clock_khz(dev);
  const double est = (double)read_bytes / 7.5e12 * 1e3 * (double)khz;
  if (!g_tune.gate_autotune || dev < 0) {
    sel.gate = clamp_ticks(kDefault * est, khz);
    return sel;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  Site &s = g_sites[Key{kernel, grid, read_bytes, dev}];
  // no other tuned launch since the burst's last, and no other library call that launched
  // (the burst's own launch_rc() counts once)
  const bool adjacent = s.open && s.open_sel == g_sel &&
                        g_lib_launches.load(std::memory_order_relaxed) <= s.open_lib + 1;
  s.last_sel = ++g_sel;
  if (s.grid == 0) {
    s.label = label;
    s.grid = grid;
    s.bytes = read_bytes;
    s.dev = dev;
    s.est = est;
    for (int c = 0; c < kCand; ++c) s.ticks[c] = clamp_ticks(kFactors[c] * est, khz);
    s.rng = 0x9e3779b97f4a7c15ull ^ (uint64_t)(uintptr_t)kernel ^ ((uint64_t)grid << 20) ^ (uint64_t)read_bytes;
    start_round(s);
    s.table_key = table_key(label, kernel, grid, read_bytes);
    apply_preset(s, khz);
  }
  if (s.open) {
    Sample *o = s.open;
    hipStreamCaptureStatus ocs = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(st, &ocs) != hipSuccess || ocs != hipStreamCaptureStatusNone;
    if (capturing) (void)hipGetLastError();
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (adjacent && !capturing && o->st == st && o->n < kBurst && o->gen == s.gen &&
        us_since(s.open_t) < kBurstGapUs && take_pair(dev, ev)) {   // the burst goes on, same gate
      if (hipEventRecord(ev.first, st) == hipSuccess) {
        o->ev.push_back(ev);
        sel.gate = o->cand >= 0 ? s.ticks[o->cand] : s.best;
        sel.timing = o;
        // the caller owns the sample until store_gate_launched re-opens it: a select of
        // this site from another thread meanwhile finds no open burst, so the sample can
        // never be published to g_pending while the caller still records into it
        s.open = nullptr;
        return sel;
      }
      (void)hipGetLastError();
      g_pool[dev].push_back(ev);
    }
    close_burst_locked(s);
  }
  int cand = -2;
  if (s.done) {
    sel.gate = s.best;
    if (s.preset || g_frozen) return sel;   // a loaded / frozen gate is never timed
    if (++s.since_watch < s.watch_every) return sel;
    s.since_watch = 0;
    cand = -1;   // time this launch: a drift sample
  } else {
    sel.gate = clamp_ticks(kDefault * est, khz);
  }
  // under capture: no event work at all (queries are not allowed in global capture mode)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return sel;
  }
  close_bursts_locked(false);   // other sites' bursts whose last launch is past the gap
  if (!g_pending.empty()) harvest_locked();
  int c = cand;
  if (c == -2) {
    if (s.done) {
      sel.gate = s.best;
      return sel;
    }
    for (int k = 0; k < 2 * kCand && c < 0; ++k) {
      if (s.pos == kCand) {   // a new pass: Fisher-Yates over the candidates
        for (int i = 0; i < kCand; ++i) s.perm[i] = i;
        for (int i = kCand - 1; i > 0; --i) {
          s.rng ^= s.rng << 13;
          s.rng ^= s.rng >> 7;
          s.rng ^= s.rng << 17;
          std::swap(s.perm[i], s.perm[s.rng % (uint64_t)(i + 1)]);
        }
        s.pos = 0;
      }
      const int j = s.perm[s.pos++];
      if (s.issued[j] < s.target[j]) c = j;
    }
    if (c < 0) return sel;   // every sample issued, results still in flight
  } else if (!s.done) {
    return sel;   // the harvest above started a re-tune: plain launch this time
  }
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  if (!take_pair(dev, ev)) return sel;
  if (hipEventRecord(ev.first, st) != hipSuccess) {
    (void)hipGetLastError();
    g_pool[dev].push_back(ev);
    return sel;
  }
  Sample *p = new Sample;
  p->ev.push_back(ev);
  p->site = &s;
  p->cand = c;
  p->dev = dev;
  p->gen = s.gen;
  p->st = st;
  if (c >= 0) {
    s.issued[c]++;
    sel.gate = s.ticks[c];
  }
  sel.timing = p;
  return sel;
}

void store_gate_launched(GateSel &sel, hipStream_t st) {
  if (!sel.timing) return;
  Sample *p = static_cast<Sample *>(sel.timing);
  sel.timing = nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  Site &s = *p->site;
  if (hipEventRecord(p->ev.back().second, st) != hipSuccess) {
    (void)hipGetLastError();
    g_pool[p->dev].push_back(p->ev.back());   // this launch's pair: never completed
    p->ev.pop_back();
    if (s.open == p) s.open = nullptr;
    if (p->n > 0) {   // the burst's earlier launches stand on their own
      g_pending.push_back(p);
      return;
    }
    if (p->cand >= 0 && p->gen == s.gen) s.issued[p->cand]--;
    delete p;
    return;
  }
  ++p->n;
  // another thread may have opened a burst of this site while p was out: that one is
  // complete as far as it goes, so it is published before p takes its place
  if (s.open && s.open != p) close_burst_locked(s);
  s.open = p;   // open until kBurst launches, another tuned launch, a gap or a read-out
  s.open_sel = g_sel;
  s.open_lib = g_lib_launches.load(std::memory_order_relaxed);
  s.open_t = std::chrono::steady_clock::now();
  if (p->n >= kBurst) close_burst_locked(s);
}

int gate_sites_tuning() {
  std::lock_guard<std::mutex> lk(g_mu);
  close_bursts_locked(true);
  harvest_locked();
  int n = 0;
  for (auto &kv : g_sites)
    if (!kv.second.done && kv.second.last_sel > g_mark) ++n;
  g_mark = g_sel;
  return n;
}

int64_t gate_report(char *buf, int64_t len) {
  std::lock_guard<std::mutex> lk(g_mu);
  close_bursts_locked(true);
  harvest_locked();
  std::string out;
  char line[512];
  for (auto &kv : g_sites) {
    const Site &s = kv.second;
    std::snprintf(line, sizeof line,
                  "%s dev=%d grid=%lld bytes=%lld est=%.0f done=%d best=%u retunes=%d watch=%d preset=%d",
                  s.label.c_str(), s.dev, (long long)s.grid, (long long)s.bytes, s.est, s.done ? 1 : 0,
                  s.best, s.retunes, s.watch_every, s.preset ? 1 : 0);
    out += line;
    for (int c = 0; c < kCand; ++c) {
      if (s.ms[c].empty()) continue;
      std::snprintf(line, sizeof line, " %u:%.2f", s.ticks[c], 1e3 * median(s.ms[c]));
      out += line;
    }
    out += "\n";
  }
  if (buf && len > 0) {
    const int64_t n = std::min<int64_t>(len - 1, (int64_t)out.size());
    std::copy(out.begin(), out.begin() + n, buf);
    buf[n] = '\0';
  }
  return (int64_t)out.size();
}

int gate_retune() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_frozen) return 0;   // a frozen table stays as loaded
  close_bursts_locked(true);
  harvest_locked();
  int n = 0;
  for (auto &kv : g_sites) {
    kv.second.preset = false;
    retune(kv.second);
    ++n;
  }
  return n;
}

// "<symbol> <grid> <bytes> <ticks>" per tuned site (loaded ones included)
int64_t gate_export(char *buf, int64_t len) {
  std::lock_guard<std::mutex> lk(g_mu);
  close_bursts_locked(true);
  harvest_locked();
  std::map<std::string, uint32_t> table = g_preset;   // loaded entries this process never launched stay
  for (auto &kv : g_sites)
    if (kv.second.done && (kv.second.preset || !g_frozen || g_preset.count(kv.second.table_key)))
      table[kv.second.table_key] = kv.second.best;
  std::string out;
  for (auto &kv : table) out += kv.first + " " + std::to_string(kv.second) + "\n";
  if (buf && len > 0) {
    const int64_t n = std::min<int64_t>(len - 1, (int64_t)out.size());
    std::copy(out.begin(), out.begin() + n, buf);
    buf[n] = '\0';
  }
  return (int64_t)out.size();
}

// parse gate_export's text; every existing site whose key is listed takes its gate
int gate_import(const char *text) {
  if (!text) return -1;
  std::map<std::string, uint32_t> add;
  const char *p = text;
  while (*p) {
    const char *e = p;
    while (*e && *e != '\n') ++e;
    std::string line(p, e);
    p = *e ? e + 1 : e;
    if (line.empty() || line[0] == '#') continue;
    const size_t k = line.find_last_of(' ');
    if (k == std::string::npos || k == 0) return -1;
    char *end = nullptr;
    const unsigned long v = std::strtoul(line.c_str() + k + 1, &end, 10);
    if (end == line.c_str() + k + 1 || *end != '\0' || v > 0xffffffffull) return -1;
    // the key is "<symbol> <grid> <bytes>": two numeric fields before the gate
    const size_t k2 = line.find_last_of(' ', k - 1);
    const size_t k1 = k2 == std::string::npos || k2 == 0 ? std::string::npos : line.find_last_of(' ', k2 - 1);
    if (k1 == std::string::npos) return -1;
    add[line.substr(0, k)] = (uint32_t)v;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  close_bursts_locked(true);
  harvest_locked();
  for (auto &kv : add) g_preset[kv.first] = kv.second;
  for (auto &kv : g_sites) {
    Site &s = kv.second;
    if (s.grid == 0) continue;
    auto it = add.find(s.table_key);
    if (it == add.end()) continue;
    s.preset = true;
    s.best = it->second;
    s.done = true;
    s.best_ms = 0.0f;
    ++s.gen;   // timings in flight belong to the tuning this replaces
  }
  return (int)add.size();
}

// on: no launch is timed from now on; sites still tuning take the default gate
int gate_freeze(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int was = g_frozen ? 1 : 0;
  g_frozen = on != 0;
  if (g_frozen) {
    close_bursts_locked(true);
    for (auto &kv : g_sites) {
      Site &s = kv.second;
      if (s.grid == 0 || s.done) continue;
      const int khz = device_wall_clock_khz(s.dev);
      s.best = clamp_ticks(kDefault * s.est, khz);
      s.done = true;
      s.best_ms = 0.0f;
      ++s.gen;
    }
  }
  return was;
}

int gate_reset() {
  std::lock_guard<std::mutex> lk(g_mu);
  close_bursts_locked(true);
  harvest_locked();
  if (!g_pending.empty()) return 1;   // samples in flight keep their sites alive
  g_sites.clear();
  g_preset.clear();   // and every loaded gate (the frozen flag stays as set)
  return 0;
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_gate_tuning_pending(void) { return gate_sites_tuning(); }

int64_t vsiq_gate_report(char *buf, int64_t len) { return gate_report(buf, len); }

int vsiq_gate_reset(void) { return gate_reset(); }

int vsiq_gate_retune(void) { return gate_retune(); }

int64_t vsiq_gate_export(char *buf, int64_t len) { return gate_export(buf, len); }

int vsiq_gate_import(const char *text) { return gate_import(text); }

int vsiq_gate_freeze(int on) { return gate_freeze(on); }

}  // extern "C"
