// STDC detail loss, fused (gfx950).
//
// Reference: core/seg_trainer.py:68-82 + core/loss.py:23-52 + models/stdc.py:131-147.
//   gt   = [lap_1(L), up_nearest(lap_2(L)), up_nearest(lap_4(L))]    (3x3 Laplacian of the
//          float label map at stride 1/2/4, padding 1, nearest-resized back to H x W)
//   gt   = (detail_conv(gt) > thrs)                                  (1x1, 3 -> 1, + bias)
//   p    = bilinear_align_corners(detail_logits [N,1,H/8,W/8] -> H x W)
//   loss = dice_coef * mean_n(1 - (2 sum p*gt + 1) / (sum p + sum gt + 1))   (RAW logits)
//        + bce_coef * mean(BCEWithLogits(p, gt))
// Stock PyTorch runs this as three 1-channel convolutions, two nearest resizes, a concat,
// a 1x1 conv, a threshold, a x8 bilinear resize and ~10 full-resolution elementwise /
// reduction kernels, each over N x H x W fp32.  Here:
//   * forward: one pass per full-resolution pixel -- the three Laplacian responses straight
//     from the label map (27 label loads that hit L1/L2), the 1x1 fuse + threshold, the
//     bilinear sample of the low-resolution logits, and the four per-sample sums (block
//     partials in fp64, one finalize block); the binary target is kept as uint8 for the
//     backward;
//   * backward: dL/dp per full-resolution pixel into an fp32 map, which the separable
//     bilinear backward (interp.hip) folds onto the low-resolution logits.
// The threshold makes the target piecewise constant in the detail_conv parameters, so (as
// in the reference) they receive no gradient.
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

namespace {

constexpr int kDlBlock = 256;

template <typename L>
struct LabelMap {
  const L* p;
  int h, w;
  __device__ __forceinline__ float at(int n, int r, int c) const {
    const bool ok = r >= 0 && r < h && c >= 0 && c < w;
    const int rr = ok ? r : 0, cc = ok ? c : 0;
    const float v = static_cast<float>(p[(static_cast<int64_t>(n) * h + rr) * w + cc]);
    return ok ? v : 0.f;
  }
  // 3x3 Laplacian [-1 ... 8 ... -1] centred at (r, c), zero padding
  __device__ __forceinline__ float lap(int n, int r, int c) const {
    float s = 0.f;
#pragma unroll
    for (int i = -1; i <= 1; ++i)
#pragma unroll
      for (int j = -1; j <= 1; ++j) s += at(n, r + i, c + j);
    return 9.f * at(n, r, c) - s;
  }
};

// ATen "nearest" source index: floor(dst * (in / out)) clamped to in - 1, in fp32 like ATen
__device__ __forceinline__ int nearest_src(int dst, int in, float scale) {
  const int s = static_cast<int>(floorf(static_cast<float>(dst) * scale));
  return s < in - 1 ? s : in - 1;
}

struct DetailGeo {
  int n, h, w;       // full-resolution label / target size
  int h2, w2, h4, w4;  // stride-2 / stride-4 Laplacian output sizes
  float s2h, s2w, s4h, s4w;
  float thrs;
  FastDiv fw;
};

template <typename L>
__device__ __forceinline__ float detail_target(const LabelMap<L>& lm, const DetailGeo& g, const float* wb, int n,
                                               int r, int c) {
  const float l1 = lm.lap(n, r, c);
  const int r2 = nearest_src(r, g.h2, g.s2h), c2 = nearest_src(c, g.w2, g.s2w);
  const float l2 = lm.lap(n, 2 * r2, 2 * c2);
  const int r4 = nearest_src(r, g.h4, g.s4h), c4 = nearest_src(c, g.w4, g.s4w);
  const float l4 = lm.lap(n, 4 * r4, 4 * c4);
  const float t = fmaf(wb[0], l1, fmaf(wb[1], l2, fmaf(wb[2], l4, wb[3])));
  return t > g.thrs ? 1.f : 0.f;
}

template <typename T>
__device__ __forceinline__ float sample_bilinear(const T* d, const Tensor4& ds, int n, int r, int c, const LinMap& mh,
                                                 const LinMap& mw) {
  int h0, h1, w0, w1;
  float lh, lw;
  mh.map(r, h0, h1, lh);
  mw.map(c, w0, w1, lw);
  const T* b = d + static_cast<int64_t>(n) * ds.sn;
  const float v00 = Io<T>::ld(b + h0 * ds.sh + w0 * ds.sw), v01 = Io<T>::ld(b + h0 * ds.sh + w1 * ds.sw);
  const float v10 = Io<T>::ld(b + h1 * ds.sh + w0 * ds.sw), v11 = Io<T>::ld(b + h1 * ds.sh + w1 * ds.sw);
  const float top = fmaf(lw, v01 - v00, v00), bot = fmaf(lw, v11 - v10, v10);
  return fmaf(lh, bot - top, top);
}

__device__ __forceinline__ float bce_logits(float p, float y) {
  return fmaxf(p, 0.f) - p * y + log1pf(__expf(-fabsf(p)));
}

// grid (G, N): block partial sums [N][G][4] = (sum p*y, sum p, sum y, sum bce)
template <typename T, typename L>
__global__ void __launch_bounds__(kDlBlock) detail_fwd_kernel(Tensor4 ds, LabelMap<L> lm, DetailGeo g, const float* wb,
                                                              LinMap mh, LinMap mw, uint8_t* __restrict__ yout,
                                                              double* __restrict__ part) {
  const T* d = static_cast<const T*>(ds.data);
  const int n = blockIdx.y;
  const uint32_t hw = static_cast<uint32_t>(g.h) * g.w;
  const float w4[4] = {wb[0], wb[1], wb[2], wb[3]};
  float s_py = 0.f, s_p = 0.f, s_y = 0.f, s_b = 0.f;
  for (uint32_t q = blockIdx.x * kDlBlock + threadIdx.x; q < hw; q += gridDim.x * kDlBlock) {
    uint32_t c;
    const int r = static_cast<int>(g.fw.divmod(q, c));
    const float y = detail_target(lm, g, w4, n, r, static_cast<int>(c));
    const float p = sample_bilinear(d, ds, n, r, static_cast<int>(c), mh, mw);
    yout[static_cast<int64_t>(n) * hw + q] = static_cast<uint8_t>(y);
    s_py = fmaf(p, y, s_py);
    s_p += p;
    s_y += y;
    s_b += bce_logits(p, y);
  }
  __shared__ double red[kDlBlock / kWave];
  const double v0 = block_sum(static_cast<double>(s_py), red);
  const double v1 = block_sum(static_cast<double>(s_p), red);
  const double v2 = block_sum(static_cast<double>(s_y), red);
  const double v3 = block_sum(static_cast<double>(s_b), red);
  if (threadIdx.x == 0) {
    double* o = part + (static_cast<int64_t>(n) * gridDim.x + blockIdx.x) * 4;
    o[0] = v0; o[1] = v1; o[2] = v2; o[3] = v3;
  }
}

// one block: per-sample totals -> sums [N][4] (kept for the backward) and the loss
__global__ void __launch_bounds__(kDlBlock) detail_finalize_kernel(const double* __restrict__ part, int N, int G,
                                                                   double numel, float dice_coef, float bce_coef,
                                                                   double* __restrict__ sums, float* __restrict__ out) {
  __shared__ double red[kDlBlock / kWave];
  double dice = 0.0, bce = 0.0;
  for (int n = 0; n < N; ++n) {
    double t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double v = 0.0;
      for (int i = threadIdx.x; i < G; i += kDlBlock) v += part[(static_cast<int64_t>(n) * G + i) * 4 + k];
      t[k] = block_sum(v, red);
    }
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) sums[n * 4 + k] = t[k];
    }
    dice += 1.0 - (2.0 * t[0] + 1.0) / (t[1] + t[2] + 1.0);
    bce += t[3];
  }
  if (threadIdx.x == 0) *out = static_cast<float>(dice_coef * dice / N + bce_coef * bce / numel);
}

// dL/dp per full-resolution pixel (fp32 [N, H, W])
template <typename T>
__global__ void __launch_bounds__(kDlBlock) detail_bwd_kernel(Tensor4 ds, DetailGeo g, LinMap mh, LinMap mw,
                                                              const uint8_t* __restrict__ yin,
                                                              const double* __restrict__ sums, const float* gout,
                                                              float dice_coef, float bce_coef, float* __restrict__ gp) {
  const T* d = static_cast<const T*>(ds.data);
  const int n = blockIdx.y;
  const uint32_t hw = static_cast<uint32_t>(g.h) * g.w;
  const double z = sums[n * 4 + 1] + sums[n * 4 + 2] + 1.0;
  const float num = static_cast<float>(2.0 * sums[n * 4 + 0] + 1.0);
  const float kd = static_cast<float>(-dice_coef / (static_cast<double>(g.n) * z * z)) * *gout;
  const float zf = static_cast<float>(z);
  const float kb = static_cast<float>(bce_coef / (static_cast<double>(g.n) * hw)) * *gout;
  for (uint32_t q = blockIdx.x * kDlBlock + threadIdx.x; q < hw; q += gridDim.x * kDlBlock) {
    uint32_t c;
    const int r = static_cast<int>(g.fw.divmod(q, c));
    const float y = static_cast<float>(yin[static_cast<int64_t>(n) * hw + q]);
    const float p = sample_bilinear(d, ds, n, r, static_cast<int>(c), mh, mw);
    const float sig = 1.f / (1.f + __expf(-p));
    gp[static_cast<int64_t>(n) * hw + q] = kd * (2.f * y * zf - num) + kb * (sig - y);
  }
}

DetailGeo make_geo(int n, int h, int w, float thrs) {
  DetailGeo g;
  g.n = n; g.h = h; g.w = w;
  g.h2 = (h - 1) / 2 + 1; g.w2 = (w - 1) / 2 + 1;
  g.h4 = (h - 1) / 4 + 1; g.w4 = (w - 1) / 4 + 1;
  g.s2h = static_cast<float>(g.h2) / static_cast<float>(h);
  g.s2w = static_cast<float>(g.w2) / static_cast<float>(w);
  g.s4h = static_cast<float>(g.h4) / static_cast<float>(h);
  g.s4w = static_cast<float>(g.w4) / static_cast<float>(w);
  g.thrs = thrs;
  g.fw = FastDiv::make(static_cast<uint32_t>(w));
  return g;
}

template <typename F>
void by_dtype(int dt, F&& f) {
  switch (dt) {
    case kF32: f(float{}); break;
    case kBF16: f(uint16_t{}); break;
    default: f(_Float16{}); break;
  }
}

}  // namespace

int detail_loss_blocks(int n, int h, int w) {
  const int64_t hw = static_cast<int64_t>(h) * w;
  int64_t g = (1024 + n - 1) / n;
  const int64_t need = (hw + kDlBlock - 1) / kDlBlock;
  if (g > need) g = need;
  return static_cast<int>(g < 1 ? 1 : g);
}

void launch_detail_fwd(const Tensor4& d, const void* labels, bool labels_u8, int n, int h, int w, const float* wb,
                       float thrs, float dice_coef, float bce_coef, uint8_t* yout, double* part, double* sums,
                       float* out, hipStream_t st) {
  const DetailGeo g = make_geo(n, h, w, thrs);
  const LinMap mh = LinMap::make(d.h, h, true), mw = LinMap::make(d.w, w, true);
  const int G = detail_loss_blocks(n, h, w);
  dim3 grid(G, n);
  by_dtype(d.dtype, [&](auto tag) {
    using T = decltype(tag);
    if (labels_u8)
      detail_fwd_kernel<T, uint8_t><<<grid, kDlBlock, 0, st>>>(d, LabelMap<uint8_t>{static_cast<const uint8_t*>(labels), h, w},
                                                              g, wb, mh, mw, yout, part);
    else
      detail_fwd_kernel<T, int64_t><<<grid, kDlBlock, 0, st>>>(d, LabelMap<int64_t>{static_cast<const int64_t*>(labels), h, w},
                                                              g, wb, mh, mw, yout, part);
  });
  detail_finalize_kernel<<<1, kDlBlock, 0, st>>>(part, n, G, static_cast<double>(n) * h * w, dice_coef, bce_coef, sums,
                                                 out);
}

void launch_detail_bwd(const Tensor4& d, int n, int h, int w, const uint8_t* yin, const double* sums,
                       const float* gout, float dice_coef, float bce_coef, float* gp, hipStream_t st) {
  const DetailGeo g = make_geo(n, h, w, 0.f);
  const LinMap mh = LinMap::make(d.h, h, true), mw = LinMap::make(d.w, w, true);
  dim3 grid(detail_loss_blocks(n, h, w), n);
  by_dtype(d.dtype, [&](auto tag) {
    using T = decltype(tag);
    detail_bwd_kernel<T><<<grid, kDlBlock, 0, st>>>(d, g, mh, mw, yin, sums, gout, dice_coef, bce_coef, gp);
  });
}

}  // namespace rtseg
