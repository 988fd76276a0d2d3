// Narrow dilated 1-D convolution (K taps along H or W, C_in, C_out in {4, 8, 16}),
// channels-last.  Reference: CFPNet's FeaturePyramidChannel (3,1)/(1,3) ConvBNActs,
// reference models/cfpnet.py:108-138, whose MIOpen solver search faulted on MI355X.
//
// One thread per output pixel: the K x CI input taps are 16-byte-vector loads of a
// contiguous channel run, the CI x CO x K weights sit in LDS (<= 3 KiB), CO fp32
// accumulators live in registers.  The op is HBM-bound (CI, CO <= 16 -> <= 2*CO FMAs per
// loaded byte pair), so the design point is one read of x and one write of y.  The
// data gradient is the same kernel with the taps flipped and W_t transposed (host side).
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {
namespace {

constexpr int kTapBlock = 256;

template <typename T, int CI, int CO>
__global__ __launch_bounds__(kTapBlock) void tapconv_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, T* __restrict__ y,
                                                            TapConvGeo g, FastDiv divw, FastDiv divh) {
  __shared__ float ws[kTapConvMaxTaps * CI * CO];
  for (int i = threadIdx.x; i < g.k * CI * CO; i += kTapBlock) ws[i] = w[i];
  __syncthreads();
  const uint32_t total = static_cast<uint32_t>(g.n) * g.h * g.w;
  const int half = (g.k - 1) / 2;
  for (uint32_t p = blockIdx.x * kTapBlock + threadIdx.x; p < total; p += gridDim.x * kTapBlock) {
    uint32_t wi, hi;
    const uint32_t nh = divw.divmod(p, wi);
    divh.divmod(nh, hi);
    float acc[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[o] = bias ? bias[o] : 0.f;
    const int pos = g.axis == 0 ? static_cast<int>(hi) : static_cast<int>(wi);
    const int lim = g.axis == 0 ? g.h : g.w;
    for (int t = 0; t < g.k; ++t) {
      const int q = pos + (t - half) * g.dil;
      if (q < 0 || q >= lim) continue;
      const int64_t src = static_cast<int64_t>(p) + static_cast<int64_t>(q - pos) * g.tap_stride;
      const T* xp = x + src * CI;
      float xv[CI];
#pragma unroll
      for (int c = 0; c < CI; ++c) xv[c] = Io<T>::ld(xp + c);
      const float* wt = ws + t * CI * CO;
#pragma unroll
      for (int c = 0; c < CI; ++c) {
#pragma unroll
        for (int o = 0; o < CO; ++o) acc[o] = fmaf(xv[c], wt[c * CO + o], acc[o]);
      }
    }
    T* yp = y + static_cast<int64_t>(p) * CO;
#pragma unroll
    for (int o = 0; o < CO; ++o) Io<T>::st(yp + o, acc[o]);
  }
}

template <typename T, int CI>
void launch_ci(const void* x, const float* w, const float* b, void* y, const TapConvGeo& g, int co, hipStream_t st) {
  const uint32_t total = static_cast<uint32_t>(g.n) * g.h * g.w;
  const int grid = stream_grid(total, kTapBlock);
  const FastDiv dw = FastDiv::make(g.w), dh = FastDiv::make(g.h);
  const T* xp = static_cast<const T*>(x);
  T* yp = static_cast<T*>(y);
  if (co == 4) tapconv_kernel<T, CI, 4><<<grid, kTapBlock, 0, st>>>(xp, w, b, yp, g, dw, dh);
  else if (co == 8) tapconv_kernel<T, CI, 8><<<grid, kTapBlock, 0, st>>>(xp, w, b, yp, g, dw, dh);
  else tapconv_kernel<T, CI, 16><<<grid, kTapBlock, 0, st>>>(xp, w, b, yp, g, dw, dh);
}

template <typename T>
void launch_t(const void* x, const float* w, const float* b, void* y, const TapConvGeo& g, int ci, int co,
              hipStream_t st) {
  if (ci == 4) launch_ci<T, 4>(x, w, b, y, g, co, st);
  else if (ci == 8) launch_ci<T, 8>(x, w, b, y, g, co, st);
  else launch_ci<T, 16>(x, w, b, y, g, co, st);
}

}  // namespace

void launch_tapconv(const void* x, const float* w, const float* bias, void* y, const TapConvGeo& g, int ci, int co,
                    int dtype, hipStream_t st) {
  if (dtype == kF32) launch_t<float>(x, w, bias, y, g, ci, co, st);
  else launch_t<uint16_t>(x, w, bias, y, g, ci, co, st);
}

}  // namespace rtseg
