// Data-movement remaps for CDNA4 (gfx950): PixelShuffle / PixelUnshuffle (sub-pixel
// convolution) and the ShuffleNet channel shuffle, as one gather pass in any input layout ->
// contiguous or channels-last output, instead of PyTorch's reshape + permute + copy (which, on a
// channels-last tensor, first materialises an NCHW copy).
//
// Reference sites: models/farseenet.py:59,82 (nn.PixelShuffle(2) / (4) sub-pixel fusion),
// models/modules.py:18-32 (channel_shuffle, used by LEDNet's SS-nbt and Lite-HRNet's shuffle
// blocks).  Backward passes are the inverse remaps (unshuffle / shuffle with C / g groups).
//
// A thread owns one OUTPUT element in the output's memory order (coalesced writes); the source
// element is found by integer index maps with FastDiv (no 64-bit division per element).
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

namespace {

constexpr int kShufBlock = 256;

struct ShufMap {
  FastDiv fc, fh, fw;  // output C, H, W
  FastDiv fr, frr;     // r, r * r (pixel modes) / groups (channel mode: fr = g, frr = C / g)
};

template <typename T>
__global__ void __launch_bounds__(kShufBlock) shuffle_kernel(Tensor4 in, Tensor4 out, int mode, bool out_cl,
                                                             ShufMap m, uint32_t total) {
  const T* ip = static_cast<const T*>(in.data);
  T* op = static_cast<T*>(out.data);
  for (uint32_t i = blockIdx.x * kShufBlock + threadIdx.x; i < total; i += gridDim.x * kShufBlock) {
    uint32_t n, c, h, w, t;
    if (out_cl) {  // i = ((n * H + h) * W + w) * C + c
      t = m.fc.divmod(i, c);
      t = m.fw.divmod(t, w);
      n = m.fh.divmod(t, h);
    } else {       // i = ((n * C + c) * H + h) * W + w
      t = m.fw.divmod(i, w);
      t = m.fh.divmod(t, h);
      n = m.fc.divmod(t, c);
    }
    uint32_t ci, hi, wi;
    if (mode == kShufPixel) {  // out [N, C, H*r, W*r] <- in [N, C*r*r, H, W]
      uint32_t i0, j0;
      hi = m.fr.divmod(h, i0);
      wi = m.fr.divmod(w, j0);
      ci = c * m.frr.d + i0 * m.fr.d + j0;
    } else if (mode == kShufPixelInv) {  // out [N, C*r*r, H, W] <- in [N, C, H*r, W*r]
      uint32_t rem, j0;
      ci = m.frr.divmod(c, rem);
      const uint32_t i0 = m.fr.divmod(rem, j0);
      hi = h * m.fr.d + i0;
      wi = w * m.fr.d + j0;
    } else {  // channel shuffle with g groups of k = C / g: out channel c = kk * g + gi <- gi * k + kk
      uint32_t gi;
      const uint32_t kk = m.fr.divmod(c, gi);
      ci = gi * m.frr.d + kk;
      hi = h;
      wi = w;
    }
    const int64_t src = static_cast<int64_t>(n) * in.sn + static_cast<int64_t>(ci) * in.sc +
                        static_cast<int64_t>(hi) * in.sh + static_cast<int64_t>(wi) * in.sw;
    op[i] = ip[src];
  }
}

}  // namespace

void launch_shuffle(const Tensor4& in, const Tensor4& out, int mode, int r, bool out_cl, hipStream_t st) {
  const uint32_t total = static_cast<uint32_t>(static_cast<int64_t>(out.n) * out.c * out.h * out.w);
  if (total == 0) return;
  ShufMap m;
  m.fc = FastDiv::make(static_cast<uint32_t>(out.c));
  m.fh = FastDiv::make(static_cast<uint32_t>(out.h));
  m.fw = FastDiv::make(static_cast<uint32_t>(out.w));
  if (mode == kShufChannel) {
    m.fr = FastDiv::make(static_cast<uint32_t>(r));
    m.frr = FastDiv::make(static_cast<uint32_t>(out.c / r));
  } else {
    m.fr = FastDiv::make(static_cast<uint32_t>(r));
    m.frr = FastDiv::make(static_cast<uint32_t>(r * r));
  }
  const int g = stream_grid(total, kShufBlock);
  // element size is all that matters for a copy
  if (in.dtype == kF32) shuffle_kernel<uint32_t><<<g, kShufBlock, 0, st>>>(in, out, mode, out_cl, m, total);
  else shuffle_kernel<uint16_t><<<g, kShufBlock, 0, st>>>(in, out, mode, out_cl, m, total);
}

}  // namespace rtseg
