// torch.library registration of PixelShuffle / PixelUnshuffle / channel shuffle (kernel: shuffle.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

// mode: kShufPixel / kShufPixelInv / kShufChannel; r: upscale factor or group count.
// The output keeps the input's memory format (channels-last in -> channels-last out).
static at::Tensor shuffle(const at::Tensor& x, int64_t mode, int64_t r) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, "rtseg.shuffle: expected a 4-D GPU tensor");
  TORCH_CHECK(r >= 1 && mode >= kShufPixel && mode <= kShufChannel, "rtseg.shuffle: bad mode / factor");
  const int64_t n = x.size(0), c = x.size(1), h = x.size(2), w = x.size(3);
  int64_t oc = c, oh = h, ow = w;
  if (mode == kShufPixel) {
    TORCH_CHECK(c % (r * r) == 0, "rtseg.shuffle: channels not divisible by r^2");
    oc = c / (r * r); oh = h * r; ow = w * r;
  } else if (mode == kShufPixelInv) {
    TORCH_CHECK(h % r == 0 && w % r == 0, "rtseg.shuffle: spatial size not divisible by r");
    oc = c * r * r; oh = h / r; ow = w / r;
  } else {
    TORCH_CHECK(c % r == 0, "rtseg.shuffle: channels not divisible by the group count");
  }
  TORCH_CHECK(x.numel() < (int64_t{1} << 32), "rtseg.shuffle: tensor too large");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const bool cl = x.is_contiguous(at::MemoryFormat::ChannelsLast) && !x.is_contiguous();
  at::Tensor y = at::empty({n, oc, oh, ow},
                           x.options().memory_format(cl ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous));
  launch_shuffle(view4(x), view4(y), static_cast<int>(mode), static_cast<int>(r), cl, cur_stream());
  return y;
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) { m.def("shuffle(Tensor x, int mode, int r) -> Tensor"); }

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) { m.impl("shuffle", &rtseg::shuffle); }
