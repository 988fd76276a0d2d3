// torch.library registration of the GPU-side training augmentation (kernel: augment.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

// img uint8 [N, H, W, 3]; msk uint8 [N, H, W] or None; params fp32 [N, kAugParams]; lut uint8 [256];
// norm fp32 [6]; out [N, 3, ch, cw] (fp32 / bf16 / fp16, any strides) and mout [N, ch, cw] (int64 /
// uint8, contiguous) are written in place.  contrast: some sample's jitter includes a contrast op.
static void augment(const at::Tensor& img, const std::optional<at::Tensor>& msk, const at::Tensor& params,
                    const at::Tensor& lut, const at::Tensor& norm, const at::Tensor& out,
                    const std::optional<at::Tensor>& mout, double pad_value, int64_t mask_pad, bool contrast) {
  TORCH_CHECK(img.is_cuda() && img.scalar_type() == at::kByte && img.dim() == 4 && img.size(3) == 3 &&
                  img.is_contiguous(),
              "rtseg.augment: image must be a contiguous uint8 [N, H, W, 3] GPU tensor");
  const int64_t n = img.size(0), h = img.size(1), w = img.size(2);
  TORCH_CHECK(n > 0 && n < 65536 && h > 0 && w > 0, "rtseg.augment: bad batch geometry");
  TORCH_CHECK(params.is_cuda() && params.scalar_type() == at::kFloat && params.is_contiguous() && params.dim() == 2 &&
                  params.size(0) == n && params.size(1) == kAugParams,
              "rtseg.augment: params must be contiguous fp32 [N, ", static_cast<int>(kAugParams), "]");
  TORCH_CHECK(lut.is_cuda() && lut.scalar_type() == at::kByte && lut.is_contiguous() && lut.numel() == 256,
              "rtseg.augment: lut must be contiguous uint8 [256]");
  TORCH_CHECK(norm.is_cuda() && norm.scalar_type() == at::kFloat && norm.is_contiguous() && norm.numel() == 6,
              "rtseg.augment: norm must be contiguous fp32 [6] (mean, std)");
  TORCH_CHECK(out.is_cuda() && out.dim() == 4 && out.size(0) == n && out.size(1) == 3,
              "rtseg.augment: out must be a [N, 3, ch, cw] GPU tensor");
  const int64_t ch = out.size(2), cw = out.size(3);
  TORCH_CHECK(ch > 0 && cw > 0 && ch * cw < (int64_t{1} << 31), "rtseg.augment: bad crop size");
  const uint8_t* mp = nullptr;
  if (msk.has_value()) {
    TORCH_CHECK(msk->is_cuda() && msk->scalar_type() == at::kByte && msk->is_contiguous() && msk->dim() == 3 &&
                    msk->size(0) == n && msk->size(1) == h && msk->size(2) == w,
                "rtseg.augment: mask must be a contiguous uint8 [N, H, W] matching the image");
    mp = msk->data_ptr<uint8_t>();
  }
  void* mo = nullptr;
  int mbytes = 8;
  if (mout.has_value()) {
    TORCH_CHECK(mp != nullptr, "rtseg.augment: mask output without a mask input");
    TORCH_CHECK(mout->is_cuda() && mout->is_contiguous() && mout->dim() == 3 && mout->size(0) == n &&
                    mout->size(1) == ch && mout->size(2) == cw &&
                    (mout->scalar_type() == at::kLong || mout->scalar_type() == at::kByte),
                "rtseg.augment: mask output must be contiguous int64 / uint8 [N, ch, cw]");
    mo = mout->data_ptr();
    mbytes = mout->scalar_type() == at::kLong ? 8 : 1;
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(img.device());
  at::Tensor part;
  if (contrast) part = at::empty({n * augment_stat_blocks(static_cast<int>(ch), static_cast<int>(cw))},
                                 params.options());
  AugArgs a{};
  a.img = img.data_ptr<uint8_t>();
  a.msk = mp;
  a.params = params.data_ptr<float>();
  a.lut = lut.data_ptr<uint8_t>();
  a.norm = norm.data_ptr<float>();
  a.part = contrast ? part.data_ptr<float>() : nullptr;
  a.out = view4(out);
  a.mout = mo;
  a.mask_bytes = mbytes;
  a.n = static_cast<int>(n); a.h = static_cast<int>(h); a.w = static_cast<int>(w);
  a.ch = static_cast<int>(ch); a.cw = static_cast<int>(cw);
  a.pad_value = static_cast<float>(pad_value);
  a.mask_pad = static_cast<int>(mask_pad);
  launch_augment(a, cur_stream());
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("augment(Tensor img, Tensor? msk, Tensor params, Tensor lut, Tensor norm, Tensor(a!) out, Tensor(b!)? mout, "
        "float pad_value, int mask_pad, bool contrast) -> ()");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) { m.impl("augment", &rtseg::augment); }
