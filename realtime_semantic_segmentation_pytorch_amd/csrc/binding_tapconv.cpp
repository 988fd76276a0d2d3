// torch.library registration of the narrow dilated 1-D convolution (kernel: tapconv.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

static bool narrow_ok(int64_t c) { return c == 4 || c == 8 || c == 16; }

// x [N, ci, H, W] channels-last (fp32 / bf16); w fp32 [K, ci, co] contiguous; bias fp32 [co] or empty
static at::Tensor tapconv_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias, int64_t dil,
                              int64_t axis) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, "rtseg.tapconv: expected a 4-D GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "rtseg.tapconv: fp32 / bf16 only");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "rtseg.tapconv: x must be channels-last");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 3,
              "rtseg.tapconv: w must be a contiguous fp32 [K, ci, co] GPU tensor");
  const int64_t k = w.size(0), ci = w.size(1), co = w.size(2);
  TORCH_CHECK(ci == x.size(1) && narrow_ok(ci) && narrow_ok(co), "rtseg.tapconv: channels must be 4, 8 or 16");
  TORCH_CHECK(k >= 1 && k <= kTapConvMaxTaps && k % 2 == 1, "rtseg.tapconv: odd tap count <= 7 required");
  TORCH_CHECK(dil >= 1 && (axis == 0 || axis == 1), "rtseg.tapconv: bad dilation / axis");
  TORCH_CHECK(x.numel() < (int64_t{1} << 31) && x.size(0) * x.size(2) * x.size(3) * 16 < (int64_t{1} << 31),
              "rtseg.tapconv: tensor too large for 32-bit indexing");
  const bool has_b = bias.numel() > 0;
  if (has_b)
    TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.numel() == co && bias.is_contiguous(),
                "rtseg.tapconv: bias must be fp32 [co]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor y = at::empty({x.size(0), co, x.size(2), x.size(3)}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (y.numel() == 0) return y;
  TapConvGeo geo{static_cast<int>(x.size(0)), static_cast<int>(x.size(2)), static_cast<int>(x.size(3)),
                 static_cast<int>(k), static_cast<int>(dil), static_cast<int>(axis), axis == 0 ? x.size(3) : 1};
  launch_tapconv(x.data_ptr(), w.data_ptr<float>(), has_b ? bias.data_ptr<float>() : nullptr, y.data_ptr(), geo,
                 static_cast<int>(ci), static_cast<int>(co), dtype_code(x),
                 cur_stream());
  return y;
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("tapconv_fwd(Tensor x, Tensor w, Tensor bias, int dil, int axis) -> Tensor");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) { m.impl("tapconv_fwd", &rtseg::tapconv_fwd); }
