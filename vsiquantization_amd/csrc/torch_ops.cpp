// torch_ops.cpp — C++ autograd nodes over the C ABI (include/vsiq.h) for the public
// Python API's per-call paths: `_vsiq_torch.so`, a pybind11 module built against
// torch's headers and linked to `_vsiq_hip.so`.
//
// Why: the same kernels behind a Python torch.autograd.Function cost ~130 us of host
// time per C2 fwd+bwd step (Function.apply bookkeeping, ctypes marshalling, and the
// autograd engine waking a Python backward on its device thread under the GIL) for
// ~26 us of GPU time.  Here the forward is one pybind call and the backward a C++ node
// the engine runs without the GIL.  Numerics are the kernels' own: every result is
// bit-identical to the ctypes path (tests/test_gpu_torch_ext.py).
//
// Round 3: the nodes are plain torch::autograd::Node subclasses wired by hand (the way
// torch's generated ops are), not torch::autograd::Function<>: no IValue-keyed
// saved_data dictionary, no output wrapping of the non-differentiable qparam outputs
// (they are ordinary tensors without history), one SavedVariable where a version check
// is needed.  The learnable node also takes its reduction workspace from a per-(device,
// stream | capture) cache here instead of from Python.
//
// Each node mirrors one Python autograd.Function of vsiquantization_amd/fakequant.py:
//   PcObserveFqBackward  PerChannelObserveFQFn  (K3 forward, STE backward from the 1-bit mask)
//   FqFixedBackward      FakeQuantFixedFn       (K1 / K5 forward, STE backward)
//   FqLearnBackward      FakeQuantLearnFn       (K1 / K5 forward, K4 backward: grad_x, d scale, d zp)
//   LsqMultiBackward     FakeQuantLearnMultiFn  (K7: every weight quantizer in one launch each way)
//   FqLearnDeferredBackward  quantizers/deferred.py DeferredLearnFn  (K1 / K5 forward, records-only
//                        K4d backward; the pending calls are folded by deferred_fold)
// Inputs are validated on the Python side (CUDA, float32, contiguous); the library
// never allocates: every buffer here comes from torch's caching allocator, every
// launch goes to torch's current HIP stream of the tensor's device.
#include <torch/extension.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/functions/utils.h>
#include <torch/csrc/autograd/saved_variable.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/EmptyTensor.h>

#include <list>
#include <map>
#include <mutex>
#include <unordered_map>
#include <optional>
#include <tuple>

#include "vsiq.h"

namespace {

using torch::autograd::Node;
using torch::autograd::SavedVariable;
using torch::autograd::variable_list;
using at::Tensor;

hipStream_t stream_of(const Tensor &t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check(int rc, const char *what) {
  TORCH_CHECK(rc == 0, what, " failed (", rc, "): ", vsiq_error_string(rc));
}

template <typename T>
T *ptr(const Tensor &t) {
  return t.defined() ? static_cast<T *>(t.data_ptr()) : nullptr;
}

// (device f64 tensor or undefined, host value) of a scale / zero-point argument:
// a CUDA tensor is read by the kernel through its pointer (converted to a contiguous
// f64 copy on x's device when it is not one already), anything else is the host value.
Tensor f64_on(const std::optional<Tensor> &v, const Tensor &x) {
  if (!v.has_value() || !v->defined()) return Tensor();
  Tensor t = v->detach();
  TORCH_CHECK(t.numel() == 1, "expected a scalar (1-element) qparam tensor, got ", t.sizes());
  if (t.device() != x.device() || t.scalar_type() != at::kDouble || !t.is_contiguous())
    t = t.to(x.device(), at::kDouble).contiguous();
  return t;
}

Tensor mask_buffer(int64_t rows, int64_t rowlen, const Tensor &like) {
  const int64_t words = vsiq_mask_words(rows, rowlen);
  return at::empty({std::max<int64_t>(words, 1)}, like.options().dtype(at::kLong));
}

bool needs_grad(const Tensor &t) { return t.defined() && t.requires_grad(); }

// Reduction workspace + self-resetting arrival counter per (device, stream), or per HIP
// graph capture (every graph its own, from that graph's pool: graphs replayed
// concurrently on two streams never share a counter) -- _hip.workspace's C++ twin.
struct Ws {
  Tensor ws, counter;
};
std::mutex g_ws_mu;
std::map<std::tuple<int, void *, unsigned long long>, Ws> g_ws;

Ws &workspace_doubles(const Tensor &like, int64_t need) {
  const int dev = like.device().index();
  const hipStream_t st = stream_of(like);
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  if (hipStreamGetCaptureInfo(st, &status, &cid) != hipSuccess || status != hipStreamCaptureStatusActive) cid = 0;
  const auto key = std::make_tuple(dev, cid ? nullptr : (void *)st, cid);
  std::lock_guard<std::mutex> lock(g_ws_mu);
  Ws &w = g_ws[key];
  if (!w.counter.defined()) w.counter = at::zeros({VSIQ_COUNTER_WORDS}, like.options().dtype(at::kInt));
  if (!w.ws.defined() || w.ws.numel() < need) w.ws = at::empty({need}, like.options().dtype(at::kDouble));
  return w;
}

Ws &workspace(const Tensor &like, int64_t n) { return workspace_doubles(like, vsiq_workspace_doubles(n)); }

// drop the workspaces of finished captures (utils.graph.GraphedStep.release)
void release_captures(const std::vector<int64_t> &ids) {
  std::lock_guard<std::mutex> lock(g_ws_mu);
  for (auto it = g_ws.begin(); it != g_ws.end();) {
    bool drop = false;
    for (int64_t id : ids) drop = drop || std::get<2>(it->first) == (unsigned long long)id;
    it = drop ? g_ws.erase(it) : std::next(it);
  }
}

int64_t capture_workspaces() {
  std::lock_guard<std::mutex> lock(g_ws_mu);
  int64_t n = 0;
  for (auto &kv : g_ws) n += std::get<2>(kv.first) != 0;
  return n;
}

// --------------------------------------------------------------------------- K3 + STE
struct PcObserveFqBackward : public Node {
  Tensor mask, scale;   // internal buffers: no version check needed
  std::string name() const override { return "PcObserveFqBackward"; }
  void release_variables() override {
    mask.reset();
    scale.reset();
  }
  variable_list apply(variable_list &&grads) override {
    TORCH_CHECK(mask.defined(), "PcObserveFqBackward: backward through the graph a second time");
    if (!grads[0].defined()) return {Tensor()};
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::detail::empty_cuda(g.sizes(), at::kFloat, g.device(), std::nullopt);
    const int64_t C = scale.numel();   // one scale per row
    const int64_t rowlen = C > 0 ? g.numel() / C : 0;
    check(vsiq_ste_bwd_f32(ptr<float>(g), ptr<uint64_t>(mask), ptr<float>(gx), g.numel(), ptr<double>(scale), rowlen,
                           0.0, stream_of(g)),
          "vsiq_ste_bwd_f32");
    return {gx};
  }
};

std::vector<Tensor> pc_observe_fq(Tensor x, Tensor run_min, Tensor run_max, bool sym, int64_t qmin, int64_t qmax,
                                  double qden, double eps, bool want_row_stats) {
  const int64_t C = x.dim() > 0 ? x.size(0) : 1;
  const int64_t rowlen = C > 0 ? x.numel() / C : 0;
  Tensor y = at::empty_like(x);
  // scale and zp (and the row stats) in ONE allocation: host time per call of the public
  // API step (views of a no-history buffer; nothing differentiates through them)
  Tensor q64 = at::empty({(want_row_stats ? 5 : 2) * C}, x.options().dtype(at::kDouble));
  Tensor scale = q64.narrow(0, 0, C);
  Tensor zp = q64.narrow(0, C, C);
  const bool grad = torch::autograd::compute_requires_grad(x);
  Tensor mask = grad ? mask_buffer(C, rowlen, x) : Tensor();
  Tensor rs = want_row_stats ? q64.narrow(0, 2 * C, 3 * C).view({C, 3}) : Tensor();   // None
  check(vsiq_pc_observe_fq_f32(ptr<float>(x), ptr<float>(y), nullptr, ptr<uint64_t>(mask), C, rowlen,
                               ptr<float>(run_min), ptr<float>(run_max), ptr<double>(scale), ptr<double>(zp),
                               want_row_stats ? ptr<double>(rs) : nullptr, sym ? 1 : 0, (int)qmin, (int)qmax, qden,
                               eps, stream_of(x)),
        "vsiq_pc_observe_fq_f32");
  if (grad) {
    auto node = std::shared_ptr<PcObserveFqBackward>(new PcObserveFqBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(x));
    node->mask = mask;
    node->scale = scale;
    torch::autograd::set_history(y, node);
  }
  return {y, scale, zp, rs};
}

// A 1-D typed alias of part of `buf`'s storage, built without the dispatcher (the way
// at::alias makes its TensorImpl): for internal buffers with no autograd history.
Tensor part_of(const Tensor &buf, at::ScalarType dt, int64_t offset, int64_t n) {
  auto impl = c10::make_intrusive<c10::TensorImpl>(c10::TensorImpl::VIEW, c10::Storage(buf.storage()), buf.key_set(),
                                                   c10::scalarTypeToTypeMeta(dt));
  impl->set_sizes_contiguous({n});
  impl->set_storage_offset(offset);
  return Tensor(std::move(impl));
}

// The per-channel observe + fake quant bound to one observer state and quantizer range:
// the public-API C2 step calls it with the tensor alone.  Host time per call is the
// point (the step's kernels are ~13 us each way, torch's own trivial step is the bar):
// the eligibility checks run here instead of in Python (None back when x is not a
// contiguous grad-requiring CUDA f32 tensor of this state's rows under grad mode, and the
// caller takes the general path), y comes from the allocator without the dispatcher, and
// scale, zp and the STE mask share ONE allocation (aliases made without the dispatcher).
// The mask's bytes then live as long as the returned scale / zp (~1/32 of x).
struct PcObserveFqOp {
  Tensor run_min, run_max;
  bool sym;
  int64_t qmin, qmax;
  double qden, eps;
  pybind11::object call(pybind11::handle h) const {
    if (!THPVariable_Check(h.ptr())) return pybind11::none();
    const Tensor &x = THPVariable_Unpack(h.ptr());
    if (!x.is_cuda() || x.scalar_type() != at::kFloat || !x.requires_grad() || !at::GradMode::is_enabled() ||
        x.dim() == 0 || !x.is_contiguous() || x.size(0) != run_min.numel() || x.device() != run_min.device())
      return pybind11::none();
    const int64_t C = x.size(0);
    const int64_t rowlen = x.numel() / std::max<int64_t>(C, 1);
    const int64_t words = std::max<int64_t>(vsiq_mask_words(C, rowlen), 1);
    Tensor y = at::detail::empty_cuda(x.sizes(), at::kFloat, x.device(), std::nullopt);
    Tensor buf = at::detail::empty_cuda({2 * C + words}, at::kDouble, x.device(), std::nullopt);
    Tensor scale = part_of(buf, at::kDouble, 0, C), zp = part_of(buf, at::kDouble, C, C);
    Tensor mask = part_of(buf, at::kLong, 2 * C, words);
    check(vsiq_pc_observe_fq_f32(ptr<float>(x), ptr<float>(y), nullptr, ptr<uint64_t>(mask), C, rowlen,
                                 ptr<float>(run_min), ptr<float>(run_max), ptr<double>(scale), ptr<double>(zp),
                                 nullptr, sym ? 1 : 0, (int)qmin, (int)qmax, qden, eps, stream_of(x)),
          "vsiq_pc_observe_fq_f32");
    auto node = std::shared_ptr<PcObserveFqBackward>(new PcObserveFqBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(x));
    node->mask = mask;
    node->scale = scale;
    torch::autograd::set_history(y, node);
    return pybind11::make_tuple(std::move(y), std::move(scale), std::move(zp));
  }
};

// --------------------------------------------------------------------------- K1/K5 + STE
struct FqFixedBackward : public Node {
  Tensor mask, sb;      // internal mask; scale for the backward (record entry / device copy)
  SavedVariable pre;    // the pre-activation (act != NONE): version-checked like an input
  double scale_host = 0.0;
  int act = VSIQ_ACT_NONE;
  std::string name() const override { return "FqFixedBackward"; }
  void release_variables() override {
    mask.reset();
    sb.reset();
    pre.reset_data();
  }
  variable_list apply(variable_list &&grads) override {
    TORCH_CHECK(mask.defined(), "FqFixedBackward: backward through the graph a second time");
    if (!grads[0].defined()) return {Tensor()};
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::empty_like(g);
    const Tensor c = act != VSIQ_ACT_NONE ? pre.unpack() : Tensor();
    check(vsiq_act_ste_bwd_f32(ptr<float>(g), ptr<uint64_t>(mask), ptr<float>(c), ptr<float>(gx), g.numel(), act,
                               ptr<double>(sb), 0, scale_host, stream_of(g)),
          "vsiq_act_ste_bwd_f32");
    return {gx};
  }
};

Tensor fq_fixed(Tensor x, std::optional<Tensor> scale, double scale_host, std::optional<Tensor> zp, double zp_host,
                int64_t qmin, int64_t qmax, std::optional<Tensor> qp, int64_t act) {
  Tensor y = at::empty_like(x);
  const bool grad = torch::autograd::compute_requires_grad(x);
  Tensor mask = grad ? mask_buffer(1, x.numel(), x) : Tensor();
  Tensor qpt = qp.has_value() ? *qp : Tensor();
  Tensor sd = qpt.defined() ? Tensor() : f64_on(scale, x);
  Tensor zd = qpt.defined() ? Tensor() : f64_on(zp, x);
  check(vsiq_act_fq_fwd_f32(ptr<float>(x), ptr<float>(y), nullptr, ptr<uint64_t>(mask), x.numel(), (int)act,
                            ptr<double>(qpt), ptr<double>(sd), scale_host, ptr<double>(zd), zp_host, 0, 0, (int)qmin,
                            (int)qmax, stream_of(x)),
        "vsiq_act_fq_fwd_f32");
  if (grad) {
    auto node = std::shared_ptr<FqFixedBackward>(new FqFixedBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(x));
    node->mask = mask;
    // backward scale: the qparams record's scale entry, the device scale, or the host value
    // (not version-checked, like the Python Function's ctx.scale: an in-place update of a
    // scale tensor between forward and backward is not an error)
    node->sb = qpt.defined() ? qpt.narrow(0, VSIQ_QP_SCALE, 1) : sd;
    node->scale_host = scale_host;
    node->act = (int)act;
    if (act != VSIQ_ACT_NONE) node->pre = SavedVariable(x, false);
    torch::autograd::set_history(y, node);
  }
  return y;
}

// --------------------------------------------------------------------------- K1/K5 + K4
// a 0-dim f64 gradient value as the gradient of a parameter of the given shape / options
Tensor as_param(Tensor v, const std::vector<int64_t> &sizes, const at::TensorOptions &o) {
  if (v.device() != o.device() || v.scalar_type() != o.dtype().toScalarType()) v = v.to(o.device(), o.dtype().toScalarType());
  return sizes.empty() ? v : v.reshape(sizes);
}

struct FqLearnBackward : public Node {
  SavedVariable x;
  Tensor sd, zd;                 // the qparams the forward read (device f64 copies) or undefined
  std::vector<int64_t> s_sizes, z_sizes;   // the learnable tensors as given: gradient shape,
  at::TensorOptions s_opts, z_opts;        // dtype and device
  double scale_host = 0.0, zp_host = 0.0, gscale = 0.0;
  int qmin = 0, qmax = 0, act = VSIQ_ACT_NONE;
  bool learn_zp = false, grad_s = false, grad_z = false;
  std::string name() const override { return "FqLearnBackward"; }
  void release_variables() override {
    x.reset_data();
    sd.reset();
    zd.reset();
  }
  variable_list apply(variable_list &&grads) override {
    if (!grads[0].defined()) return {Tensor(), Tensor(), Tensor()};
    const Tensor xv = x.unpack();
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::empty_like(g);
    Tensor go = at::empty({2}, g.options().dtype(at::kDouble));
    Ws &w = workspace(g, g.numel());
    check(vsiq_act_lsq_bwd_f32(ptr<float>(g), ptr<float>(xv), ptr<float>(gx), g.numel(), act, ptr<double>(sd),
                               scale_host, ptr<double>(zd), zp_host, learn_zp ? 1 : 0, qmin, qmax, gscale,
                               ptr<double>(go), ptr<double>(w.ws), w.ws.numel(), ptr<uint32_t>(w.counter),
                               stream_of(g)),
          "vsiq_act_lsq_bwd_f32");
    Tensor gs, gz;
    if (grad_s) gs = as_param(go.select(0, 0), s_sizes, s_opts);
    if (learn_zp && grad_z) gz = as_param(go.select(0, 1), z_sizes, z_opts);
    return {gx, gs, gz};
  }
};

// ws / counter: accepted for signature compatibility (the node takes its workspace from
// the C++ cache above when its backward runs)
Tensor fq_learn(Tensor x, std::optional<Tensor> scale, double scale_host, std::optional<Tensor> zp, double zp_host,
                int64_t qmin, int64_t qmax, double gscale, bool learn_zp, int64_t act, std::optional<Tensor> /*ws*/,
                std::optional<Tensor> /*counter*/) {
  Tensor y = at::empty_like(x);
  Tensor sd = f64_on(scale, x), zd = f64_on(zp, x);
  check(vsiq_act_fq_fwd_f32(ptr<float>(x), ptr<float>(y), nullptr, nullptr, x.numel(), (int)act, nullptr,
                            ptr<double>(sd), scale_host, ptr<double>(zd), zp_host, learn_zp ? 1 : 0, 0, (int)qmin,
                            (int)qmax, stream_of(x)),
        "vsiq_act_fq_fwd_f32");
  const Tensor st = scale.has_value() ? *scale : Tensor();
  const Tensor zt = zp.has_value() ? *zp : Tensor();
  if (torch::autograd::compute_requires_grad(x, st, zt)) {
    auto node = std::shared_ptr<FqLearnBackward>(new FqLearnBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(x, st, zt));
    node->x = SavedVariable(x, false);
    node->sd = sd;
    node->zd = zd;
    node->scale_host = scale_host;
    node->zp_host = zp_host;
    node->gscale = gscale;
    node->qmin = (int)qmin;
    node->qmax = (int)qmax;
    node->act = (int)act;
    node->learn_zp = learn_zp;
    node->grad_s = needs_grad(st);
    node->grad_z = needs_grad(zt);
    if (node->grad_s) {
      node->s_sizes = st.sizes().vec();
      node->s_opts = st.options();
    }
    if (node->grad_z) {
      node->z_sizes = zt.sizes().vec();
      node->z_opts = zt.options();
    }
    torch::autograd::set_history(y, node);
  }
  return y;
}

// --------------------------------------------------------------------------- K1/K5 + K4d (deferred fold)
// quantizers/deferred.py's DeferredLearnFn as a C++ node: the records-only backward
// (vsiq_act_lsq_bwd_part_f32) returns placeholder qparam gradients -- views of a pending
// f64[2] -- and registers the call here; the model's bundle node (QParamBundleFn) folds
// every pending call in one vsiq_lsq_fold_multi launch (deferred_fold) before AccumulateGrad
// sees the values.  Same kernels and arguments as the Python Function: the same bits.
struct PendingFold {
  Tensor records, out, zd;
  int64_t nrec = 0, gen = 0;
  double zh = 0.0, gscale = 0.0;
  int qmin = 0, qmax = 0;
  bool learn_zp = false;
};
std::mutex g_pend_mu;
std::list<std::pair<uintptr_t, PendingFold>> g_pend;   // oldest first
std::unordered_map<uintptr_t, std::list<std::pair<uintptr_t, PendingFold>>::iterator> g_pend_at;
int64_t g_pend_gen = 0;
constexpr size_t kPendMax = size_t(1) << 14;   // a backward that never reaches the bundle leaves entries

struct FqLearnDeferredBackward : public Node {
  SavedVariable x;
  Tensor sd, zd;
  std::vector<int64_t> s_sizes, z_sizes;
  double scale_host = 0.0, zp_host = 0.0, gscale = 0.0;
  int qmin = 0, qmax = 0, act = VSIQ_ACT_NONE;
  bool learn_zp = false, grad_s = false, grad_z = false;
  std::string name() const override { return "FqLearnDeferredBackward"; }
  void release_variables() override {
    x.reset_data();
    sd.reset();
    zd.reset();
  }
  variable_list apply(variable_list &&grads) override {
    if (!grads[0].defined()) return {Tensor(), Tensor(), Tensor()};
    const Tensor xv = x.unpack();
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::empty_like(g);
    PendingFold e;
    e.nrec = vsiq_lsq_part_records(g.numel());
    TORCH_CHECK(e.nrec > 0, "vsiq_lsq_part_records failed (", e.nrec, ")");
    e.records = at::empty({2 * e.nrec}, g.options().dtype(at::kDouble));
    e.out = at::empty({2}, g.options().dtype(at::kDouble));
    check(vsiq_act_lsq_bwd_part_f32(ptr<float>(g), ptr<float>(xv), ptr<float>(gx), g.numel(), act, ptr<double>(sd),
                                    scale_host, ptr<double>(zd), zp_host, learn_zp ? 1 : 0, qmin, qmax,
                                    ptr<double>(e.records), 2 * e.nrec, stream_of(g)),
          "vsiq_act_lsq_bwd_part_f32");
    e.zd = zd;
    e.zh = zp_host;
    e.gscale = gscale;
    e.qmin = qmin;
    e.qmax = qmax;
    e.learn_zp = learn_zp;
    Tensor gs, gz;
    if (grad_s) gs = e.out.select(0, 0).view(s_sizes);
    if (learn_zp && grad_z) gz = e.out.select(0, 1).view(z_sizes);
    const uintptr_t key = reinterpret_cast<uintptr_t>(e.out.data_ptr());
    {
      std::lock_guard<std::mutex> lock(g_pend_mu);
      e.gen = g_pend_gen;
      g_pend.emplace_back(key, std::move(e));
      g_pend_at[key] = std::prev(g_pend.end());
      while (g_pend.size() > kPendMax) {
        g_pend_at.erase(g_pend.front().first);
        g_pend.pop_front();
      }
    }
    return {gx, gs, gz};
  }
};

Tensor fq_learn_deferred(Tensor x, Tensor scale, std::optional<Tensor> zp, double zp_host, int64_t qmin,
                         int64_t qmax, double gscale, bool learn_zp, int64_t act) {
  Tensor y = at::empty_like(x);
  Tensor sd = f64_on(scale, x), zd = f64_on(zp, x);
  check(vsiq_act_fq_fwd_f32(ptr<float>(x), ptr<float>(y), nullptr, nullptr, x.numel(), (int)act, nullptr,
                            ptr<double>(sd), 0.0, ptr<double>(zd), zp_host, learn_zp ? 1 : 0, 0, (int)qmin,
                            (int)qmax, stream_of(x)),
        "vsiq_act_fq_fwd_f32");
  const Tensor zt = zp.has_value() ? *zp : Tensor();
  if (torch::autograd::compute_requires_grad(x, scale, zt)) {
    auto node = std::shared_ptr<FqLearnDeferredBackward>(new FqLearnDeferredBackward(), torch::autograd::deleteNode);
    node->set_next_edges(torch::autograd::collect_next_edges(x, scale, zt));
    node->x = SavedVariable(x, false);
    node->sd = sd;
    node->zd = zd;
    node->zp_host = zp_host;
    node->gscale = gscale;
    node->qmin = (int)qmin;
    node->qmax = (int)qmax;
    node->act = (int)act;
    node->learn_zp = learn_zp;
    node->grad_s = needs_grad(scale);
    node->grad_z = needs_grad(zt);
    if (node->grad_s) node->s_sizes = scale.sizes().vec();
    if (node->grad_z) node->z_sizes = zt.sizes().vec();
    torch::autograd::set_history(y, node);
  }
  return y;
}

// Fold the pending calls whose placeholder gradients have these data pointers (a
// grad_scale view points at out[0], a grad_zp view at out[1]) in ONE vsiq_lsq_fold_multi
// launch on the current stream; returns how many pointers matched no pending call here.
int64_t deferred_fold(const std::vector<int64_t> &ptrs) {
  std::vector<PendingFold> taken;
  int64_t missing = 0;
  {
    std::lock_guard<std::mutex> lock(g_pend_mu);
    for (int64_t p : ptrs) {
      auto it = g_pend_at.find((uintptr_t)p);
      if (it == g_pend_at.end()) it = g_pend_at.find((uintptr_t)p - sizeof(double));
      if (it == g_pend_at.end()) {
        bool done = false;   // the other view of a call already taken
        for (const auto &t : taken) {
          const uintptr_t k = reinterpret_cast<uintptr_t>(t.out.data_ptr());
          done = done || k == (uintptr_t)p || k + sizeof(double) == (uintptr_t)p;
        }
        missing += done ? 0 : 1;
        continue;
      }
      taken.push_back(std::move(it->second->second));
      g_pend.erase(it->second);
      g_pend_at.erase(it);
    }
  }
  if (taken.empty()) return missing;
  std::vector<vsiq_lsq_fold> folds(taken.size());
  for (size_t i = 0; i < taken.size(); ++i) {
    const PendingFold &e = taken[i];
    folds[i] = vsiq_lsq_fold{ptr<double>(e.records), e.nrec, ptr<double>(e.zd), e.zh, e.gscale,
                             ptr<double>(e.out), e.qmin, e.qmax, e.learn_zp ? 1 : 0, 0};
  }
  check(vsiq_lsq_fold_multi(folds.data(), (int)folds.size(), stream_of(taken[0].out)), "vsiq_lsq_fold_multi");
  return missing;
}

// --------------------------------------------------------------------------- K7 (multi-tensor learnable)
// fakequant.py's FakeQuantLearnMultiFn as a C++ node: every learnable weight quantizer of
// a model in ONE forward launch (vsiq_lsq_fwd_multi_f32) and ONE backward launch
// (vsiq_lsq_bwd_multi_f32); per tensor bit-identical to the single-tensor K1 / K4.
// Inputs: the k tensors, then per tensor its scale / zero point (a device f64 tensor or
// undefined = the host value); edges to the xs and to the scale / zp tensors that need
// a gradient, in that order (the Python Function's input order).
struct LsqMultiBackward : public Node {
  std::vector<SavedVariable> xs;
  std::vector<Tensor> sd, zd;
  std::vector<double> sh, zh, gscale;
  std::vector<int> qmin, qmax, learn_zp;
  // per tensor: output slot of its scale / zp gradient (-1: none), the parameter's shape / options
  std::vector<int64_t> s_slot, z_slot;
  std::vector<std::vector<int64_t>> s_sizes, z_sizes;
  std::vector<at::TensorOptions> s_opts, z_opts;
  std::string name() const override { return "LsqMultiBackward"; }
  void release_variables() override {
    for (auto &x : xs) x.reset_data();
    sd.clear();
    zd.clear();
  }
  variable_list apply(variable_list &&grads) override {
    const size_t k = xs.size();
    std::vector<Tensor> x(k), g(k), gx(k);
    for (size_t i = 0; i < k; ++i) {
      x[i] = xs[i].unpack();
      g[i] = grads[i].defined() ? grads[i].contiguous() : at::zeros_like(x[i]);
      gx[i] = at::empty_like(x[i]);
    }
    Tensor go = at::empty({(int64_t)k, 2}, x[0].options().dtype(at::kDouble));
    std::vector<vsiq_lsq_tensor> d(k);
    for (size_t i = 0; i < k; ++i)
      d[i] = vsiq_lsq_tensor{ptr<float>(x[i]), nullptr, ptr<float>(g[i]), ptr<float>(gx[i]), ptr<double>(sd[i]),
                             ptr<double>(zd[i]), ptr<double>(go) + 2 * i, x[i].numel(), sh[i], zh[i], gscale[i],
                             qmin[i], qmax[i], learn_zp[i], 0};
    const int64_t need = vsiq_lsq_multi_workspace_doubles(d.data(), (int)k);
    check(need < 0 ? (int)need : 0, "vsiq_lsq_multi_workspace_doubles");
    Ws &w = workspace_doubles(x[0], need);
    check(vsiq_lsq_bwd_multi_f32(d.data(), (int)k, ptr<double>(w.ws), w.ws.numel(), ptr<uint32_t>(w.counter),
                                 stream_of(x[0])),
          "vsiq_lsq_bwd_multi_f32");
    variable_list out(num_outputs());
    for (size_t i = 0; i < k; ++i) out[i] = gx[i];
    for (size_t i = 0; i < k; ++i) {
      if (s_slot[i] >= 0 && should_compute_output(s_slot[i]))
        out[s_slot[i]] = as_param(go.select(0, i).select(0, 0), s_sizes[i], s_opts[i]);
      if (z_slot[i] >= 0 && learn_zp[i] && should_compute_output(z_slot[i]))
        out[z_slot[i]] = as_param(go.select(0, i).select(0, 1), z_sizes[i], z_opts[i]);
    }
    return out;
  }
};

std::vector<Tensor> lsq_multi(const std::vector<Tensor> &xs, const std::vector<std::optional<Tensor>> &scales,
                              const std::vector<double> &scale_hosts, const std::vector<std::optional<Tensor>> &zps,
                              const std::vector<double> &zp_hosts, const std::vector<int64_t> &qmins,
                              const std::vector<int64_t> &qmaxs, const std::vector<double> &gscales,
                              const std::vector<bool> &learn_zps) {
  const size_t k = xs.size();
  TORCH_CHECK(scales.size() == k && scale_hosts.size() == k && zps.size() == k && zp_hosts.size() == k &&
                  qmins.size() == k && qmaxs.size() == k && gscales.size() == k && learn_zps.size() == k,
              "lsq_multi: argument lists of different lengths");
  if (k == 0) return {};
  std::vector<Tensor> ys(k), sd(k), zd(k), st(k), zt(k);
  std::vector<vsiq_lsq_tensor> d(k);
  for (size_t i = 0; i < k; ++i) {
    TORCH_CHECK(xs[i].device() == xs[0].device(), "multi-tensor fake quant: all tensors must be on one device");
    ys[i] = at::empty_like(xs[i]);
    sd[i] = f64_on(scales[i], xs[i]);
    zd[i] = f64_on(zps[i], xs[i]);
    st[i] = scales[i].has_value() ? *scales[i] : Tensor();
    zt[i] = zps[i].has_value() ? *zps[i] : Tensor();
    d[i] = vsiq_lsq_tensor{ptr<float>(xs[i]), ptr<float>(ys[i]), nullptr, nullptr, ptr<double>(sd[i]),
                           ptr<double>(zd[i]), nullptr, xs[i].numel(), scale_hosts[i], zp_hosts[i], gscales[i],
                           (int32_t)qmins[i], (int32_t)qmaxs[i], learn_zps[i] ? 1 : 0, 0};
  }
  check(vsiq_lsq_fwd_multi_f32(d.data(), (int)k, stream_of(xs[0])), "vsiq_lsq_fwd_multi_f32");
  bool any = false;
  for (size_t i = 0; i < k; ++i) any = any || needs_grad(xs[i]) || needs_grad(st[i]) || needs_grad(zt[i]);
  if (!any || !at::GradMode::is_enabled()) return ys;
  auto node = std::shared_ptr<LsqMultiBackward>(new LsqMultiBackward(), torch::autograd::deleteNode);
  torch::autograd::edge_list edges;
  for (size_t i = 0; i < k; ++i) edges.push_back(torch::autograd::impl::gradient_edge(xs[i]));
  node->s_slot.assign(k, -1);
  node->z_slot.assign(k, -1);
  node->s_sizes.resize(k);
  node->z_sizes.resize(k);
  node->s_opts.resize(k);
  node->z_opts.resize(k);
  int64_t slot = (int64_t)k;
  for (size_t i = 0; i < k; ++i) {   // the Python Function's parameter order: scale, then zero point
    if (needs_grad(st[i])) {
      node->s_slot[i] = slot++;
      node->s_sizes[i] = st[i].sizes().vec();
      node->s_opts[i] = st[i].options();
      edges.push_back(torch::autograd::impl::gradient_edge(st[i]));
    }
    if (needs_grad(zt[i])) {
      node->z_slot[i] = slot++;
      node->z_sizes[i] = zt[i].sizes().vec();
      node->z_opts[i] = zt[i].options();
      edges.push_back(torch::autograd::impl::gradient_edge(zt[i]));
    }
  }
  node->set_next_edges(std::move(edges));
  for (size_t i = 0; i < k; ++i) {
    node->xs.emplace_back(xs[i], false);
    node->sh.push_back(scale_hosts[i]);
    node->zh.push_back(zp_hosts[i]);
    node->gscale.push_back(gscales[i]);
    node->qmin.push_back((int)qmins[i]);
    node->qmax.push_back((int)qmaxs[i]);
    node->learn_zp.push_back(learn_zps[i] ? 1 : 0);
  }
  node->sd = sd;
  node->zd = zd;
  torch::autograd::set_history(ys, node);
  return ys;
}

// A new forward generation: drop the entries of backwards older than the previous one
// (orphans of a backward that never reached the bundle; one generation of slack for a
// checkpointed layer whose forward re-runs inside the backward).
void deferred_generation() {
  std::lock_guard<std::mutex> lock(g_pend_mu);
  ++g_pend_gen;
  for (auto it = g_pend.begin(); it != g_pend.end();) {
    if (it->second.gen < g_pend_gen - 1) {
      g_pend_at.erase(it->first);
      it = g_pend.erase(it);
    } else {
      ++it;
    }
  }
}

int64_t deferred_pending() {
  std::lock_guard<std::mutex> lock(g_pend_mu);
  return (int64_t)g_pend.size();
}

}  // namespace

PYBIND11_MODULE(_vsiq_torch, m) {
  m.doc() = "C++ autograd nodes over the vsiq C ABI (K3/K1/K5 forwards, STE/K4 backwards)";
  m.def("abi_version", []() { return vsiq_abi_version(); });
  m.def("pc_observe_fq", &pc_observe_fq, "K3 per-channel observe + fake quant; STE backward");
  pybind11::class_<PcObserveFqOp>(m, "PcObserveFqOp")
      .def(pybind11::init([](Tensor run_min, Tensor run_max, bool sym, int64_t qmin, int64_t qmax, double qden,
                             double eps) { return PcObserveFqOp{run_min, run_max, sym, qmin, qmax, qden, eps}; }))
      .def("__call__", &PcObserveFqOp::call,
           "(y, scale, zp) of pc_observe_fq(x) with the bound state / range, or None when x is not a "
           "contiguous grad-requiring CUDA float32 tensor of the state's rows under grad mode");
  m.def("fq_fixed", &fq_fixed, "K1/K5 fake quant with fixed qparams; STE backward");
  m.def("fq_learn", &fq_learn, "K1/K5 learnable fake quant; K4 backward", pybind11::arg("x"), pybind11::arg("scale"),
        pybind11::arg("scale_host"), pybind11::arg("zp"), pybind11::arg("zp_host"), pybind11::arg("qmin"),
        pybind11::arg("qmax"), pybind11::arg("gscale"), pybind11::arg("learn_zp"), pybind11::arg("act"),
        pybind11::arg("ws") = pybind11::none(), pybind11::arg("counter") = pybind11::none());
  m.def("fq_learn_deferred", &fq_learn_deferred, "K1/K5 learnable fake quant; records-only K4d backward",
        pybind11::arg("x"), pybind11::arg("scale"), pybind11::arg("zp"), pybind11::arg("zp_host"),
        pybind11::arg("qmin"), pybind11::arg("qmax"), pybind11::arg("gscale"), pybind11::arg("learn_zp"),
        pybind11::arg("act"));
  m.def("lsq_multi", &lsq_multi, "K7 multi-tensor learnable fake quant (one launch each way)");
  m.def("deferred_fold", &deferred_fold, "fold the pending K4d calls of these placeholder gradients in one launch");
  m.def("deferred_generation", &deferred_generation, "new forward generation: drop orphaned pending K4d calls");
  m.def("deferred_pending", &deferred_pending, "pending K4d calls held by the C++ nodes");
  m.def("release_captures", &release_captures, "drop the C++ workspaces of the given HIP graph capture ids");
  m.def("capture_workspaces", &capture_workspaces, "number of capture-owned C++ workspaces held");
}
