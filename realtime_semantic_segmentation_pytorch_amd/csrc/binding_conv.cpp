// torch.library registration of the MFMA implicit-GEMM convolution (conv_mfma.hip) and
// of the BatchNorm finalize entry points that consume its statistics slab.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {
namespace {

const float* fptr(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}
float* fptr_mut(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? const_cast<float*>(t->data_ptr<float>()) : nullptr;
}
int64_t* nbt_ptr(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<int64_t>() : nullptr;
}

// x [N,Cin,H,W] bf16 channels-last; wk [Cout,KH,KW,Cin] bf16 contiguous -> (y, part)
std::tuple<at::Tensor, at::Tensor> conv_mfma(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                             at::IntArrayRef padding, at::IntArrayRef dilation, bool stats,
                                             const std::optional<at::Tensor>& scale_shift,
                                             const std::optional<at::Tensor>& residual, int64_t act) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "rtseg.conv_mfma: input must be a channels-last bf16 GPU tensor");
  TORCH_CHECK(wk.is_cuda() && wk.dim() == 4 && wk.scalar_type() == at::kBFloat16 && wk.is_contiguous(),
              "rtseg.conv_mfma: weights must be contiguous bf16 [Cout, KH, KW, Cin]");
  TORCH_CHECK(stride.size() == 2 && padding.size() == 2 && dilation.size() == 2, "rtseg.conv_mfma: 2-D geometry");
  TORCH_CHECK(act >= 0 && act <= 2, "rtseg.conv_mfma: bad activation");
  const int64_t N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = wk.size(0), KH = wk.size(1), KW = wk.size(2);
  TORCH_CHECK(wk.size(3) == Cin, "rtseg.conv_mfma: weight/input channel mismatch");
  TORCH_CHECK(Cin % 32 == 0 && Cout % 8 == 0, "rtseg.conv_mfma: needs Cin % 32 == 0 and Cout % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(wk.data_ptr()) % 16 == 0,
              "rtseg.conv_mfma: operands must be 16-byte aligned");
  const int64_t Ho = (H + 2 * padding[0] - dilation[0] * (KH - 1) - 1) / stride[0] + 1;
  const int64_t Wo = (W + 2 * padding[1] - dilation[1] * (KW - 1) - 1) / stride[1] + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "rtseg.conv_mfma: empty output");
  TORCH_CHECK(N * Ho * Wo < (int64_t{1} << 31) && N * H * W * Cin < (int64_t{1} << 40),
              "rtseg.conv_mfma: problem too large for 32-bit pixel indexing");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({N, Cout, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  ConvGeom g;
  g.x = x.data_ptr(); g.w = wk.data_ptr(); g.y = y.data_ptr();
  g.part = nullptr; g.scale_shift = nullptr; g.res = nullptr; g.act = static_cast<int>(act);
  g.n = static_cast<int>(N); g.h = static_cast<int>(H); g.w_in = static_cast<int>(W); g.cin = static_cast<int>(Cin);
  g.ho = static_cast<int>(Ho); g.wo = static_cast<int>(Wo); g.cout = static_cast<int>(Cout);
  g.kh = static_cast<int>(KH); g.kw = static_cast<int>(KW);
  g.sh = static_cast<int>(stride[0]); g.sw = static_cast<int>(stride[1]);
  g.ph = static_cast<int>(padding[0]); g.pw = static_cast<int>(padding[1]);
  g.dh = static_cast<int>(dilation[0]); g.dw = static_cast<int>(dilation[1]);
  at::Tensor part;
  if (stats) {
    part = at::empty({conv_mfma_slabs(g), 2 * Cout}, x.options().dtype(at::kFloat));
    g.part = part.data_ptr<float>();
  }
  if (scale_shift.has_value() && scale_shift->defined()) {
    TORCH_CHECK(scale_shift->scalar_type() == at::kFloat && scale_shift->is_contiguous() &&
                    scale_shift->numel() == 2 * Cout,
                "rtseg.conv_mfma: scale_shift must be fp32 [2*Cout]");
    g.scale_shift = scale_shift->data_ptr<float>();
    if (residual.has_value() && residual->defined()) {
      TORCH_CHECK(residual->sizes() == y.sizes() && residual->scalar_type() == at::kBFloat16 &&
                      residual->is_contiguous(at::MemoryFormat::ChannelsLast),
                  "rtseg.conv_mfma: residual must match the output (bf16, channels-last)");
      g.res = residual->data_ptr();
    }
  } else {
    TORCH_CHECK(!(residual.has_value() && residual->defined()) && act == 0,
                "rtseg.conv_mfma: residual / activation need the BN epilogue (scale_shift)");
  }
  launch_conv_mfma(g, cur_stream());
  return {y, part};
}

// BN forward from a statistics slab [G, 2C] -> (mean_invstd, scale_shift, sums[2C+1])
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_finalize_slab(
    const at::Tensor& part, const std::optional<at::Tensor>& w, const std::optional<at::Tensor>& b,
    const std::optional<at::Tensor>& rmean, const std::optional<at::Tensor>& rvar,
    const std::optional<at::Tensor>& nbt, double momentum, double eps, double count) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 && part.is_contiguous() &&
                  part.size(1) % 2 == 0,
              "rtseg.bn_finalize_slab: slab must be contiguous fp32 [G, 2C]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(part.device());
  const int C = static_cast<int>(part.size(1) / 2);
  auto f32 = part.options();
  at::Tensor mi = at::empty({2 * C}, f32), ss = at::empty({2 * C}, f32);
  at::Tensor sums = at::empty({2 * C + 1}, part.options().dtype(at::kDouble));
  launch_bn_finalize_partials(part.data_ptr<float>(), static_cast<int>(part.size(0)), C, count, fptr(w), fptr(b),
                              fptr_mut(rmean), fptr_mut(rvar), nbt_ptr(nbt), static_cast<float>(momentum),
                              static_cast<float>(eps), mi.data_ptr<float>(), ss.data_ptr<float>(),
                              sums.data_ptr<double>(), cur_stream(), nullptr,
                              SlabScratch(static_cast<int>(part.size(0)), C, part).ptr());
  return {mi, ss, sums};
}

// SyncBN: slab -> fp64 sums[2C+1] (sum, second moment, count) to be all-reduced
at::Tensor bn_slab_sums(const at::Tensor& part, double count) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 && part.is_contiguous(),
              "rtseg.bn_slab_sums: slab must be contiguous fp32 [G, 2C]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(part.device());
  const int C = static_cast<int>(part.size(1) / 2);
  at::Tensor sums = at::empty({2 * C + 1}, part.options().dtype(at::kDouble));
  launch_bn_slab_to_sums(part.data_ptr<float>(), static_cast<int>(part.size(0)), C, count, sums.data_ptr<double>(),
                         cur_stream(), nullptr, SlabScratch(static_cast<int>(part.size(0)), C, part).ptr());
  return sums;
}

}  // namespace
}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("conv_mfma(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, bool stats, "
        "Tensor? scale_shift, Tensor? residual, int act) -> (Tensor, Tensor)");
  m.def("bn_finalize_slab(Tensor part, Tensor? weight, Tensor? bias, Tensor(a!)? running_mean, "
        "Tensor(b!)? running_var, Tensor(c!)? num_batches_tracked, float momentum, float eps, float count) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("bn_slab_sums(Tensor part, float count) -> Tensor");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("conv_mfma", &rtseg::conv_mfma);
  m.impl("bn_finalize_slab", &rtseg::bn_finalize_slab);
  m.impl("bn_slab_sums", &rtseg::bn_slab_sums);
}
