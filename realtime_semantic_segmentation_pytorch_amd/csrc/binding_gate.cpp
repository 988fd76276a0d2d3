// torch.library registration of the attention-gating kernels (gate.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {
namespace {

void check_cl4(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  (t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf),
              "rtseg.gate: ", what, " must be a channels-last fp32/bf16/fp16 GPU tensor");
}

GateArgs make_args(const at::Tensor& x, const at::Tensor& att, const std::optional<at::Tensor>& y, int64_t mode,
                   bool sigmoid) {
  check_cl4(x, "x");
  TORCH_CHECK(mode >= kGateMul && mode <= kGateBlend, "rtseg.gate: bad mode");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  GateArgs g{};
  g.x = x.data_ptr();
  g.dtype = dtype_code(x);
  g.mode = static_cast<int>(mode);
  g.sigmoid = sigmoid;
  g.M = N * H * W;
  g.HW = static_cast<int>(H * W);
  g.C = static_cast<int>(C);
  TORCH_CHECK(gate_vec_width(g.dtype, g.C) > 0, "rtseg.gate: unsupported channel count");
  TORCH_CHECK(att.is_cuda() && att.dim() == 4 && att.size(0) == N, "rtseg.gate: gate must be 4-D on the GPU");
  if (att.size(1) == C && att.size(2) == 1 && att.size(3) == 1 && H * W > 1) {
    g.bc = kGateChannel;
  } else if (att.size(1) == 1 && att.size(2) == H && att.size(3) == W && C > 1) {
    g.bc = kGateSpatial;
  } else {
    TORCH_CHECK(att.sizes() == x.sizes(), "rtseg.gate: gate must be [N,C,1,1], [N,1,H,W] or x's shape");
    g.bc = kGateFull;
  }
  if (g.bc == kGateFull) {
    check_cl4(att, "gate");
    TORCH_CHECK(att.scalar_type() == x.scalar_type(), "rtseg.gate: full-size gate must have x's dtype");
  } else {
    TORCH_CHECK(att.scalar_type() == at::kFloat && att.is_contiguous(), "rtseg.gate: broadcast gate must be contiguous fp32");
  }
  g.att = att.data_ptr();
  g.y = nullptr;
  if (mode == kGateBlend) {
    TORCH_CHECK(y.has_value() && y->defined(), "rtseg.gate: blend needs the second input");
    check_cl4(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes() && y->scalar_type() == x.scalar_type(), "rtseg.gate: y must match x");
    g.y = y->data_ptr();
  }
  return g;
}

at::Tensor gate_fwd(const at::Tensor& x, const at::Tensor& att, const std::optional<at::Tensor>& y, int64_t mode,
                    bool sigmoid) {
  GateArgs g = make_args(x, att, y, mode, sigmoid);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor out = at::empty_like(x);
  g.out = out.data_ptr();
  if (g.M > 0) launch_gate_fwd(g, cur_stream());
  return out;
}

// -> (grad x, grad y (blend) or empty, grad gate (fp32 for broadcast gates))
std::tuple<at::Tensor, at::Tensor, at::Tensor> gate_bwd(const at::Tensor& go, const at::Tensor& x, const at::Tensor& att,
                                                        const std::optional<at::Tensor>& y, int64_t mode, bool sigmoid) {
  GateArgs g = make_args(x, att, y, mode, sigmoid);
  check_cl4(go, "grad");
  TORCH_CHECK(go.sizes() == x.sizes() && go.scalar_type() == x.scalar_type(), "rtseg.gate_bwd: grad must match x");
  TORCH_CHECK(gate_bwd_supported(g.dtype, g.C, g.bc), "rtseg.gate_bwd: unsupported channel count for this gate");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor gx = at::empty_like(x);
  at::Tensor gy = mode == kGateBlend ? at::empty_like(x) : at::Tensor();
  at::Tensor gatt = g.bc == kGateFull ? at::empty_like(att) : at::empty(att.sizes(), att.options());
  at::Tensor part;
  if (g.bc == kGateChannel) {
    const int N = static_cast<int>(x.size(0));
    part = at::empty({N, gate_channel_blocks(g.HW, N), g.C}, x.options().dtype(at::kFloat));
  }
  if (g.M > 0)
    launch_gate_bwd(g, go.data_ptr(), gx.data_ptr(), gy.defined() ? gy.data_ptr() : nullptr, gatt.data_ptr(),
                    part.defined() ? part.data_ptr<float>() : nullptr, cur_stream());
  return {gx, gy, gatt};
}

bool gate_supported(int64_t dtype, int64_t C, int64_t bc) {
  return gate_vec_width(static_cast<int>(dtype), static_cast<int>(C)) > 0 &&
         gate_bwd_supported(static_cast<int>(dtype), static_cast<int>(C), static_cast<int>(bc));
}

}  // namespace
}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("gate_fwd(Tensor x, Tensor att, Tensor? y, int mode, bool sigmoid) -> Tensor");
  m.def("gate_bwd(Tensor grad, Tensor x, Tensor att, Tensor? y, int mode, bool sigmoid) -> (Tensor, Tensor, Tensor)");
  m.def("gate_supported(int dtype, int C, int bcast) -> bool", &rtseg::gate_supported);
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("gate_fwd", &rtseg::gate_fwd);
  m.impl("gate_bwd", &rtseg::gate_bwd);
}
