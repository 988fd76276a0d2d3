// Prediction post-processing for CDNA4 (gfx950): per-pixel argmax over the class logits,
// colour lookup and the optional alpha blend with the raw image, in one pass.
//
// Reference: core/seg_trainer.py:172-191 (argmax -> colormap LUT gather -> PIL Image.blend)
// and the ONNX-export head of models/ddrnet.py:55-58 / models/stdc.py:90-93 (argmax as a
// compact class map).  Stock PyTorch materialises an int64 [N, H, W] argmax and a
// [N, H, W, 3] int64 gather before the copy to the host; here a thread owns one pixel, scans
// its C logits (any strides; channels-last reads are one contiguous row), and writes the
// uint8 class id, the uint8 RGB colour and, given the raw image, the uint8 blend
// raw + alpha * (colour - raw), computed and truncated exactly like PIL's Image.blend.
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

namespace {

constexpr int kColBlock = 256;

template <typename T>
__global__ void __launch_bounds__(kColBlock) colorize_kernel(Tensor4 x, const uint8_t* __restrict__ lut,
                                                             const uint8_t* __restrict__ img, float alpha,
                                                             uint8_t* __restrict__ cls, uint8_t* __restrict__ rgb,
                                                             uint8_t* __restrict__ blend, FastDiv fw, FastDiv fh,
                                                             uint32_t total) {
  const T* xp = static_cast<const T*>(x.data);
  for (uint32_t i = blockIdx.x * kColBlock + threadIdx.x; i < total; i += gridDim.x * kColBlock) {
    uint32_t c_, r_;
    const uint32_t t = fw.divmod(i, c_);
    const uint32_t n = fh.divmod(t, r_);
    const T* p = xp + static_cast<int64_t>(n) * x.sn + static_cast<int64_t>(r_) * x.sh + static_cast<int64_t>(c_) * x.sw;
    float best = Io<T>::ld(p);
    int arg = 0;
    for (int k = 1; k < x.c; ++k) {
      const float v = Io<T>::ld(p + static_cast<int64_t>(k) * x.sc);
      const bool take = v > best || (v != v && best == best);  // first maximum; NaN wins (torch.argmax)
      best = take ? v : best;
      arg = take ? k : arg;
    }
    if (cls != nullptr) cls[i] = static_cast<uint8_t>(arg);
    const uint8_t r = lut[3 * arg], g = lut[3 * arg + 1], b = lut[3 * arg + 2];
    if (rgb != nullptr) {
      rgb[3 * static_cast<int64_t>(i)] = r;
      rgb[3 * static_cast<int64_t>(i) + 1] = g;
      rgb[3 * static_cast<int64_t>(i) + 2] = b;
    }
    if (img != nullptr) {
      const uint8_t col[3] = {r, g, b};
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        // fp32 multiply then add, no contraction, truncated: bit-identical to PIL's blend
        const float a = static_cast<float>(img[3 * static_cast<int64_t>(i) + ch]);
        const float v = __fadd_rn(a, __fmul_rn(alpha, static_cast<float>(col[ch]) - a));
        blend[3 * static_cast<int64_t>(i) + ch] = static_cast<uint8_t>(fminf(fmaxf(v, 0.f), 255.f));
      }
    }
  }
}

}  // namespace

void launch_colorize(const Tensor4& x, const uint8_t* lut, const uint8_t* img, float alpha, uint8_t* cls,
                     uint8_t* rgb, uint8_t* blend, hipStream_t st) {
  const uint32_t total = static_cast<uint32_t>(static_cast<int64_t>(x.n) * x.h * x.w);
  const int g = stream_grid(total, kColBlock);
  const FastDiv fw = FastDiv::make(x.w), fh = FastDiv::make(x.h);
  switch (x.dtype) {
    case kF32:
      colorize_kernel<float><<<g, kColBlock, 0, st>>>(x, lut, img, alpha, cls, rgb, blend, fw, fh, total);
      break;
    case kBF16:
      colorize_kernel<uint16_t><<<g, kColBlock, 0, st>>>(x, lut, img, alpha, cls, rgb, blend, fw, fh, total);
      break;
    default:
      colorize_kernel<_Float16><<<g, kColBlock, 0, st>>>(x, lut, img, alpha, cls, rgb, blend, fw, fh, total);
      break;
  }
}

}  // namespace rtseg
