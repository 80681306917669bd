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
// Each node mirrors one Python autograd.Function of vsiquantization_amd/fakequant.py:
//   PcObserveFq   PerChannelObserveFQFn  (K3 forward, STE backward from the 1-bit mask)
//   FqFixed       FakeQuantFixedFn       (K1 / K5 forward, STE backward)
//   FqLearn       FakeQuantLearnFn       (K1 / K5 forward, K4 backward: grad_x, d scale, d zp)
// Inputs are validated on the Python side (CUDA, float32, contiguous); the library
// never allocates: every buffer here comes from torch's caching allocator, every
// launch goes to torch's current HIP stream of the tensor's device.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <optional>

#include "vsiq.h"

namespace {

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;
using at::Tensor;

void *stream_of(const Tensor &t) {
  return (void *)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

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

// --------------------------------------------------------------------------- K3 + STE
struct PcObserveFq : public torch::autograd::Function<PcObserveFq> {
  static variable_list forward(AutogradContext *ctx, Tensor x, Tensor run_min, Tensor run_max,
                               bool sym, int64_t qmin, int64_t qmax, double qden, double eps,
                               bool want_row_stats) {
    const int64_t C = x.dim() > 0 ? x.size(0) : 1;
    const int64_t rowlen = C > 0 ? x.numel() / C : 0;
    Tensor y = at::empty_like(x);
    // separate buffers, not rows of one: view outputs cost the engine extra bookkeeping
    Tensor scale = at::empty({C}, x.options().dtype(at::kDouble));
    Tensor zp = at::empty({C}, x.options().dtype(at::kDouble));
    Tensor mask = mask_buffer(C, rowlen, x);
    Tensor rs = want_row_stats ? at::empty({C, 3}, x.options().dtype(at::kDouble))
                               : at::empty({0}, x.options().dtype(at::kDouble));
    check(vsiq_pc_observe_fq_f32(ptr<float>(x), ptr<float>(y), nullptr, ptr<uint64_t>(mask), C, rowlen,
                                 ptr<float>(run_min), ptr<float>(run_max), ptr<double>(scale),
                                 ptr<double>(zp), want_row_stats ? ptr<double>(rs) : nullptr, sym ? 1 : 0,
                                 (int)qmin, (int)qmax, qden, eps, stream_of(x)),
          "vsiq_pc_observe_fq_f32");
    ctx->save_for_backward({mask, scale});
    ctx->mark_non_differentiable({scale, zp, rs});
    // the engine would otherwise materialize zero gradients for the three
    // non-differentiable outputs (two allocations + fill launches per backward)
    ctx->set_materialize_grads(false);
    return {y, scale, zp, rs};
  }

  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    if (!grads[0].defined())
      return {Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
    const auto saved = ctx->get_saved_variables();
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::empty_like(g);
    const int64_t C = saved[1].numel();   // one scale per row
    const int64_t rowlen = C > 0 ? g.numel() / C : 0;
    check(vsiq_ste_bwd_f32(ptr<float>(g), ptr<uint64_t>(saved[0]), ptr<float>(gx), g.numel(),
                           ptr<double>(saved[1]), rowlen, 0.0, stream_of(g)),
          "vsiq_ste_bwd_f32");
    return {gx, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

std::vector<Tensor> pc_observe_fq(Tensor x, Tensor run_min, Tensor run_max, bool sym, int64_t qmin,
                                  int64_t qmax, double qden, double eps, bool want_row_stats) {
  return PcObserveFq::apply(x, run_min, run_max, sym, qmin, qmax, qden, eps, want_row_stats);
}

// --------------------------------------------------------------------------- K1/K5 + STE
struct FqFixed : public torch::autograd::Function<FqFixed> {
  static Tensor forward(AutogradContext *ctx, Tensor x, std::optional<Tensor> scale, double scale_host,
                        std::optional<Tensor> zp, double zp_host, int64_t qmin, int64_t qmax,
                        std::optional<Tensor> qp, int64_t act) {
    Tensor y = at::empty_like(x);
    Tensor mask = mask_buffer(1, x.numel(), x);
    Tensor qpt = qp.has_value() ? *qp : Tensor();
    Tensor sd = qpt.defined() ? Tensor() : f64_on(scale, x);
    Tensor zd = qpt.defined() ? Tensor() : f64_on(zp, x);
    check(vsiq_act_fq_fwd_f32(ptr<float>(x), ptr<float>(y), nullptr, ptr<uint64_t>(mask), x.numel(), (int)act,
                              ptr<double>(qpt), ptr<double>(sd), scale_host, ptr<double>(zd), zp_host, 0, 0,
                              (int)qmin, (int)qmax, stream_of(x)),
          "vsiq_act_fq_fwd_f32");
    // backward scale: the qparams record's scale entry, the device scale, or the host value
    // (held outside save_for_backward, like the Python Function's ctx.scale: an in-place
    // update of a scale tensor between forward and backward is not a version error)
    Tensor sb = qpt.defined() ? qpt.narrow(0, VSIQ_QP_SCALE, 1) : sd;
    ctx->save_for_backward({mask, act != VSIQ_ACT_NONE ? x : Tensor()});
    ctx->saved_data["has_sb"] = sb.defined();
    if (sb.defined()) ctx->saved_data["sb"] = sb;
    ctx->saved_data["scale_host"] = scale_host;
    ctx->saved_data["act"] = act;
    return y;
  }

  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::empty_like(g);
    const int act = (int)ctx->saved_data["act"].toInt();
    const Tensor sb = ctx->saved_data["has_sb"].toBool() ? ctx->saved_data["sb"].toTensor() : Tensor();
    check(vsiq_act_ste_bwd_f32(ptr<float>(g), ptr<uint64_t>(saved[0]), act ? ptr<float>(saved[1]) : nullptr,
                               ptr<float>(gx), g.numel(), act, ptr<double>(sb), 0,
                               ctx->saved_data["scale_host"].toDouble(), stream_of(g)),
          "vsiq_act_ste_bwd_f32");
    return {gx, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

Tensor fq_fixed(Tensor x, std::optional<Tensor> scale, double scale_host, std::optional<Tensor> zp,
                double zp_host, int64_t qmin, int64_t qmax, std::optional<Tensor> qp, int64_t act) {
  return FqFixed::apply(x, scale, scale_host, zp, zp_host, qmin, qmax, qp, act);
}

// --------------------------------------------------------------------------- K1/K5 + K4
struct FqLearn : public torch::autograd::Function<FqLearn> {
  static Tensor forward(AutogradContext *ctx, Tensor x, std::optional<Tensor> scale, double scale_host,
                        std::optional<Tensor> zp, double zp_host, int64_t qmin, int64_t qmax, double gscale,
                        bool learn_zp, int64_t act, Tensor ws, Tensor counter) {
    Tensor y = at::empty_like(x);
    Tensor sd = f64_on(scale, x), zd = f64_on(zp, x);
    check(vsiq_act_fq_fwd_f32(ptr<float>(x), ptr<float>(y), nullptr, nullptr, x.numel(), (int)act, nullptr,
                              ptr<double>(sd), scale_host, ptr<double>(zd), zp_host, learn_zp ? 1 : 0, 0,
                              (int)qmin, (int)qmax, stream_of(x)),
          "vsiq_act_fq_fwd_f32");
    ctx->save_for_backward({x, ws, counter});
    ctx->saved_data["has_sd"] = sd.defined();
    ctx->saved_data["has_zd"] = zd.defined();
    if (sd.defined()) ctx->saved_data["sd"] = sd;
    if (zd.defined()) ctx->saved_data["zd"] = zd;
    ctx->saved_data["scale_host"] = scale_host;
    ctx->saved_data["zp_host"] = zp_host;
    ctx->saved_data["qmin"] = qmin;
    ctx->saved_data["qmax"] = qmax;
    ctx->saved_data["gscale"] = gscale;
    ctx->saved_data["learn_zp"] = learn_zp;
    ctx->saved_data["act"] = act;
    // gradient targets: the learnable tensors as given (shape / dtype / device of each)
    // (needs_input_grad counts Variable inputs only, whose positions move with the optional
    // tensors, so requires_grad is recorded here instead)
    ctx->saved_data["has_scale_t"] = scale.has_value() && scale->defined() && scale->requires_grad();
    ctx->saved_data["has_zp_t"] = zp.has_value() && zp->defined() && zp->requires_grad();
    if (scale.has_value() && scale->defined()) ctx->saved_data["scale_t"] = scale->detach();
    if (zp.has_value() && zp->defined()) ctx->saved_data["zp_t"] = zp->detach();
    return y;
  }

  static variable_list backward(AutogradContext *ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const Tensor &x = saved[0], &ws = saved[1], &counter = saved[2];
    const Tensor g = grads[0].contiguous();
    Tensor gx = at::empty_like(g);
    Tensor go = at::empty({2}, g.options().dtype(at::kDouble));
    auto &d = ctx->saved_data;
    const Tensor sd = d["has_sd"].toBool() ? d["sd"].toTensor() : Tensor();
    const Tensor zd = d["has_zd"].toBool() ? d["zd"].toTensor() : Tensor();
    const bool learn_zp = d["learn_zp"].toBool();
    check(vsiq_act_lsq_bwd_f32(ptr<float>(g), ptr<float>(x), ptr<float>(gx), g.numel(), (int)d["act"].toInt(),
                               ptr<double>(sd), d["scale_host"].toDouble(), ptr<double>(zd),
                               d["zp_host"].toDouble(), learn_zp ? 1 : 0, (int)d["qmin"].toInt(),
                               (int)d["qmax"].toInt(), d["gscale"].toDouble(), ptr<double>(go),
                               ptr<double>(ws), ws.numel(), ptr<uint32_t>(counter), stream_of(g)),
          "vsiq_act_lsq_bwd_f32");
    Tensor gs, gz;
    if (d["has_scale_t"].toBool()) {
      const Tensor p = d["scale_t"].toTensor();
      gs = go.narrow(0, 0, 1).to(p.device(), p.scalar_type()).reshape(p.sizes());
    }
    if (learn_zp && d["has_zp_t"].toBool()) {
      const Tensor p = d["zp_t"].toTensor();
      gz = go.narrow(0, 1, 1).to(p.device(), p.scalar_type()).reshape(p.sizes());
    }
    return {gx, gs, Tensor(), gz, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

Tensor fq_learn(Tensor x, std::optional<Tensor> scale, double scale_host, std::optional<Tensor> zp,
                double zp_host, int64_t qmin, int64_t qmax, double gscale, bool learn_zp, int64_t act,
                Tensor ws, Tensor counter) {
  return FqLearn::apply(x, scale, scale_host, zp, zp_host, qmin, qmax, gscale, learn_zp, act, ws, counter);
}

}  // namespace

PYBIND11_MODULE(_vsiq_torch, m) {
  m.doc() = "C++ autograd nodes over the vsiq C ABI (K3/K1/K5 forwards, STE/K4 backwards)";
  m.def("abi_version", []() { return vsiq_abi_version(); });
  m.def("pc_observe_fq", &pc_observe_fq, "K3 per-channel observe + fake quant; STE backward");
  m.def("fq_fixed", &fq_fixed, "K1/K5 fake quant with fixed qparams; STE backward");
  m.def("fq_learn", &fq_learn, "K1/K5 learnable fake quant; K4 backward");
}
