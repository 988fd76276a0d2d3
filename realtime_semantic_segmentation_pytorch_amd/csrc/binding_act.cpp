// torch.library registration of the point-wise activation family (kernel: act.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

// dense, 16-byte aligned, in x's own memory order
static at::Tensor dense_aligned(const at::Tensor& t, at::MemoryFormat fmt) {
  at::Tensor c = t.contiguous(fmt);
  if (reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 != 0) c = c.clone(fmt);
  return c;
}

static at::MemoryFormat fmt_of(const at::Tensor& x) {
  return x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && !x.is_contiguous()
             ? at::MemoryFormat::ChannelsLast
             : at::MemoryFormat::Contiguous;
}

static ActArgs act_args(const at::Tensor& x, int64_t kind, const std::optional<at::Tensor>& w, double a, double b) {
  TORCH_CHECK(x.is_cuda(), "rtseg.act: expected a GPU tensor");
  TORCH_CHECK(kind >= kActPReLU && kind <= kActGELUTanh, "rtseg.act: bad activation kind ", kind);
  TORCH_CHECK(x.numel() < (int64_t{1} << 32), "rtseg.act: tensor too large");
  ActArgs r{};
  r.dtype = dtype_code(x);
  r.kind = static_cast<int>(kind);
  r.n = x.numel();
  r.a = static_cast<float>(a);
  r.b = static_cast<float>(b);
  r.C = 1;
  r.inner = 1;
  if (w.has_value()) {
    TORCH_CHECK(kind == kActPReLU, "rtseg.act: a weight tensor is PReLU-only");
    TORCH_CHECK(w->is_cuda() && w->scalar_type() == at::kFloat && w->is_contiguous(),
                "rtseg.act: PReLU weight must be a contiguous fp32 GPU tensor");
    const int64_t C = w->numel();
    if (C > 1) {
      TORCH_CHECK(x.dim() >= 2 && x.size(1) == C, "rtseg.act: PReLU weight size ", C, " != channels ",
                  x.dim() >= 2 ? x.size(1) : 0);
      TORCH_CHECK(C <= 4096, "rtseg.act: PReLU with more than 4096 channels");
      r.C = static_cast<int>(C);
      r.inner = fmt_of(x) == at::MemoryFormat::ChannelsLast ? 1 : x.numel() / (x.size(0) * C);
    }
    r.w = w->data_ptr<float>();
  }
  return r;
}

static at::Tensor act_fwd(const at::Tensor& x, int64_t kind, const std::optional<at::Tensor>& w, double a,
                          double b) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const auto fmt = fmt_of(x);
  at::Tensor xx = dense_aligned(x, fmt);
  ActArgs r = act_args(xx, kind, w, a, b);
  at::Tensor y = at::empty_like(xx, xx.options().memory_format(fmt));
  r.x = xx.data_ptr();
  r.out = y.data_ptr();
  launch_act(r, cur_stream());
  return y;
}

// inference: prelu(x * scale + shift) with an eval BN's fp32 [2C] scale | shift and a per-channel
// PReLU weight [C]: BN + PReLU in one pass (ops/bn.py bn_act)
static at::Tensor bn_prelu_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& ss) {
  TORCH_CHECK(x.dim() == 4 && w.numel() == x.size(1) && w.scalar_type() == at::kFloat && ss.scalar_type() == at::kFloat &&
                  ss.numel() == 2 * x.size(1) && ss.is_contiguous() && w.is_contiguous(),
              "rtseg.bn_prelu_fwd: per-channel PReLU weight [C] and fp32 scale_shift [2C]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const auto fmt = fmt_of(x);
  at::Tensor xx = dense_aligned(x, fmt);
  ActArgs r = act_args(xx, 0, w, 0.0, 0.0);
  at::Tensor y = at::empty_like(xx, xx.options().memory_format(fmt));
  r.x = xx.data_ptr();
  r.out = y.data_ptr();
  r.ss = ss.data_ptr<float>();
  launch_act(r, cur_stream());
  return y;
}

// -> (dx, dw); dw is empty unless a PReLU weight is given
static std::tuple<at::Tensor, at::Tensor> act_bwd(const at::Tensor& dy, const at::Tensor& x, int64_t kind,
                                                  const std::optional<at::Tensor>& w, double a, double b) {
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "rtseg.act_bwd: dy / x mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const auto fmt = fmt_of(x);
  at::Tensor xx = dense_aligned(x, fmt), gg = dense_aligned(dy, fmt);
  ActArgs r = act_args(xx, kind, w, a, b);
  at::Tensor dx = at::empty_like(xx, xx.options().memory_format(fmt));
  r.x = xx.data_ptr();
  r.dy = gg.data_ptr();
  r.out = dx.data_ptr();
  r.bwd = true;
  at::Tensor dw, part;
  if (w.has_value()) {
    const ActPreluPlan p = act_prelu_plan(r);
    part = at::empty({p.planes ? static_cast<int64_t>(p.blocks) : static_cast<int64_t>(p.blocks) * r.C},
                     xx.options().dtype(at::kFloat));
    dw = at::empty({r.C}, xx.options().dtype(at::kFloat));
    r.part = part.data_ptr<float>();
    r.dw = dw.data_ptr<float>();
  }
  launch_act(r, cur_stream());
  if (dw.defined()) dw = dw.view(w->sizes());
  return {dx, dw.defined() ? dw : at::empty({0}, xx.options().dtype(at::kFloat))};
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("act_fwd(Tensor x, int kind, Tensor? w, float a, float b) -> Tensor");
  m.def("bn_prelu_fwd(Tensor x, Tensor w, Tensor scale_shift) -> Tensor");
  m.def("act_bwd(Tensor dy, Tensor x, int kind, Tensor? w, float a, float b) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("act_fwd", &rtseg::act_fwd);
  m.impl("bn_prelu_fwd", &rtseg::bn_prelu_fwd);
  m.impl("act_bwd", &rtseg::act_bwd);
}
