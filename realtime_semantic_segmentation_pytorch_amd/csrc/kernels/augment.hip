// GPU-side training augmentation for CDNA4 (gfx950): random scale + centred pad + random crop +
// colour jitter + horizontal flip + normalisation of a batch of raw uint8 images (and the
// nearest-resampled, label-remapped masks) in one pass over the OUTPUT crop.
//
// Reference: the albumentations pipeline of datasets/cityscapes.py:115-124 (Scale, RandomScale,
// PadIfNeeded(114 / mask 0), RandomCrop, ColorJitter, HorizontalFlip, Normalize) and the label-id
// -> train-id remap of datasets/cityscapes.py:150-156.  At 1024 x 2048 that pipeline costs tens
// of CPU-milliseconds per image; here the host only decodes and draws the per-sample random
// parameters (same draw order as datasets/transforms.py, so both paths see the same stream)
// and the GPU does the pixel work: a thread owns one output pixel, walks back through
// flip -> crop -> pad -> resize to the source pixel, samples it (bilinear, half-pixel centres,
// rounded to uint8 like cv2.INTER_LINEAR; masks nearest with floor(y * scale) like
// cv2.INTER_NEAREST), applies the jitter ops in the drawn order on [0, 1] floats, re-quantises
// to uint8 exactly as the CPU path does, normalises and writes every output channel.
//
// Contrast needs the mean grey level of the whole crop in its pre-contrast state: aug_stats
// computes it (per-image, per-block partial sums, deterministic) with the same per-pixel code.
#include "rtseg_common.h"
#include "rtseg_launch.h"

#include <algorithm>

namespace rtseg {

namespace {

constexpr int kAugBlock = 256;

struct AugP {
  int nh, nw, top, left, cy, cx, flip, nops, code;
  float f[4];  // brightness, contrast, saturation factors; hue shift
};

__device__ __forceinline__ AugP load_params(const float* __restrict__ p) {
  AugP a;
  a.nh = static_cast<int>(p[kAugNh]);
  a.nw = static_cast<int>(p[kAugNw]);
  a.top = static_cast<int>(p[kAugTop]);
  a.left = static_cast<int>(p[kAugLeft]);
  a.cy = static_cast<int>(p[kAugCy]);
  a.cx = static_cast<int>(p[kAugCx]);
  a.flip = static_cast<int>(p[kAugFlip]);
  a.nops = static_cast<int>(p[kAugNops]);
  a.code = static_cast<int>(p[kAugCode]);
  a.f[0] = p[kAugBright];
  a.f[1] = p[kAugContrast];
  a.f[2] = p[kAugSat];
  a.f[3] = p[kAugHue];
  return a;
}

// scaled-image coordinate -> source coordinate (ATen / cv2 bilinear, align_corners = False)
__device__ __forceinline__ void lin(int o, float scale, int in, int& i0, int& i1, float& l) {
  const float s = fmaxf(scale * (static_cast<float>(o) + 0.5f) - 0.5f, 0.f);
  int f = static_cast<int>(s);
  if (f > in - 1) f = in - 1;
  i0 = f;
  i1 = f + (f < in - 1 ? 1 : 0);
  l = s - static_cast<float>(f);
}

__device__ __forceinline__ float grey(const float* x) { return 0.299f * x[0] + 0.587f * x[1] + 0.114f * x[2]; }

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }

__device__ __forceinline__ void hue_shift(float* x, float dh) {
  const float r = x[0], g = x[1], b = x[2];
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b)), d = mx - mn;
  float h = 0.f;
  if (d > 1e-12f) {
    const float rc = (mx - r) / d, gc = (mx - g) / d, bc = (mx - b) / d;
    h = r == mx ? bc - gc : (g == mx ? 2.f + rc - bc : 4.f + gc - rc);
    h = h / 6.f;
    h = h - floorf(h);
  }
  const float s = mx > 1e-12f ? d / mx : 0.f, v = mx;
  h = h + dh;
  h = h - floorf(h);
  const float i = floorf(h * 6.f), f = h * 6.f - i;
  const float p = v * (1.f - s), q = v * (1.f - s * f), t = v * (1.f - s * (1.f - f));
  switch (static_cast<int>(i) % 6) {
    case 0: x[0] = v; x[1] = t; x[2] = p; break;
    case 1: x[0] = q; x[1] = v; x[2] = p; break;
    case 2: x[0] = p; x[1] = v; x[2] = t; break;
    case 3: x[0] = p; x[1] = q; x[2] = v; break;
    case 4: x[0] = t; x[1] = p; x[2] = v; break;
    default: x[0] = v; x[1] = p; x[2] = q; break;
  }
}

// one jitter op (0 brightness, 1 contrast, 2 saturation, 3 hue) on [0, 1] RGB
__device__ __forceinline__ void jitter_op(int op, const AugP& a, float cmean, float* x) {
  if (op == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = clamp01(x[c] * a.f[0]);
  } else if (op == 1) {
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = clamp01((x[c] - cmean) * a.f[1] + cmean);
  } else if (op == 2) {
    const float gr = grey(x);
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = clamp01(gr + (x[c] - gr) * a.f[2]);
  } else {
    hue_shift(x, a.f[3]);
  }
}

struct AugGeo {
  const uint8_t* img;  // [N, H, W, 3]
  const uint8_t* msk;  // [N, H, W] or null
  const float* params; // [N, kAugParams]
  int H, W, ch, cw;
  float pad_value;     // image pad (0..255)
  int mask_pad;
};

// geometric stage: uint8-valued RGB of output pixel (oy, ox) of image n (and its raw label)
__device__ __forceinline__ void sample(const AugGeo& g, const AugP& a, int n, int oy, int ox, float* rgb,
                                       int* label) {
  const int xx = a.flip ? g.cw - 1 - ox : ox;
  const int py = oy + a.cy - a.top, px = xx + a.cx - a.left;
  if (py < 0 || px < 0 || py >= a.nh || px >= a.nw) {
    rgb[0] = rgb[1] = rgb[2] = g.pad_value;
    if (label) *label = g.mask_pad;
    return;
  }
  const float sy = static_cast<float>(g.H) / static_cast<float>(a.nh);
  const float sx = static_cast<float>(g.W) / static_cast<float>(a.nw);
  int y0, y1, x0, x1;
  float ly, lx;
  lin(py, sy, g.H, y0, y1, ly);
  lin(px, sx, g.W, x0, x1, lx);
  const uint8_t* base = g.img + static_cast<int64_t>(n) * g.H * g.W * 3;
  const uint8_t* p00 = base + (static_cast<int64_t>(y0) * g.W + x0) * 3;
  const uint8_t* p01 = base + (static_cast<int64_t>(y0) * g.W + x1) * 3;
  const uint8_t* p10 = base + (static_cast<int64_t>(y1) * g.W + x0) * 3;
  const uint8_t* p11 = base + (static_cast<int64_t>(y1) * g.W + x1) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float top = static_cast<float>(p00[c]) + lx * (static_cast<float>(p01[c]) - static_cast<float>(p00[c]));
    const float bot = static_cast<float>(p10[c]) + lx * (static_cast<float>(p11[c]) - static_cast<float>(p10[c]));
    rgb[c] = fminf(fmaxf(rintf(top + ly * (bot - top)), 0.f), 255.f);
  }
  if (label) {
    int my = static_cast<int>(floorf(static_cast<float>(py) * sy));
    int mx = static_cast<int>(floorf(static_cast<float>(px) * sx));
    my = my < g.H - 1 ? my : g.H - 1;
    mx = mx < g.W - 1 ? mx : g.W - 1;
    *label = g.msk[static_cast<int64_t>(n) * g.H * g.W + static_cast<int64_t>(my) * g.W + mx];
  }
}

// per-image partial sums of the crop's grey level just before the contrast op
__global__ void __launch_bounds__(kAugBlock) aug_stats_kernel(AugGeo g, float* __restrict__ part) {
  __shared__ float red[kAugBlock / kWave];
  const int n = blockIdx.y;
  const AugP a = load_params(g.params + static_cast<int64_t>(n) * kAugParams);
  const int npix = g.ch * g.cw;
  float s = 0.f;
  for (int i = blockIdx.x * kAugBlock + threadIdx.x; i < npix; i += gridDim.x * kAugBlock) {
    const int oy = i / g.cw, ox = i - oy * g.cw;
    float x[3];
    sample(g, a, n, oy, ox, x, nullptr);
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = __fdiv_rn(x[c], 255.f);
    for (int k = 0; k < a.nops; ++k) {
      const int op = (a.code >> (2 * k)) & 3;
      if (op == 1) break;
      jitter_op(op, a, 0.f, x);
    }
    s += grey(x);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[static_cast<int64_t>(n) * gridDim.x + blockIdx.x] = s;
}

template <typename TO, typename TM>
__global__ void __launch_bounds__(kAugBlock) aug_apply_kernel(AugGeo g, const uint8_t* __restrict__ lut,
                                                              const float* __restrict__ part, int nparts,
                                                              const float* __restrict__ norm, Tensor4 out,
                                                              TM* __restrict__ mout) {
  const int n = blockIdx.y;
  const AugP a = load_params(g.params + static_cast<int64_t>(n) * kAugParams);
  const int npix = g.ch * g.cw;
  float cmean = 0.f;
  if (a.nops > 0 && part != nullptr) {  // same fixed-order sum in every thread: deterministic
    float s = 0.f;
    for (int j = 0; j < nparts; ++j) s += part[static_cast<int64_t>(n) * nparts + j];
    cmean = s / static_cast<float>(npix);
  }
  float mean[3], istd[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    mean[c] = norm[c];
    istd[c] = 1.f / norm[3 + c];
  }
  TO* op = static_cast<TO*>(out.data);
  for (int i = blockIdx.x * kAugBlock + threadIdx.x; i < npix; i += gridDim.x * kAugBlock) {
    const int oy = i / g.cw, ox = i - oy * g.cw;
    float x[3];
    int label = 0;
    sample(g, a, n, oy, ox, x, mout != nullptr ? &label : nullptr);
    if (a.nops > 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c) x[c] = __fdiv_rn(x[c], 255.f);
      for (int k = 0; k < a.nops; ++k) jitter_op((a.code >> (2 * k)) & 3, a, cmean, x);
#pragma unroll
      for (int c = 0; c < 3; ++c) x[c] = fminf(fmaxf(floorf(x[c] * 255.f + 0.5f), 0.f), 255.f);
    }
    TO* po = op + static_cast<int64_t>(n) * out.sn + static_cast<int64_t>(oy) * out.sh + static_cast<int64_t>(ox) * out.sw;
#pragma unroll
    for (int c = 0; c < 3; ++c) Io<TO>::st(po + c * out.sc, (x[c] * (1.f / 255.f) - mean[c]) * istd[c]);
    if (mout != nullptr) mout[static_cast<int64_t>(n) * npix + i] = static_cast<TM>(lut[label]);
  }
}

template <typename TO>
void launch_apply(const AugGeo& g, const uint8_t* lut, const float* part, int nparts, const float* norm,
                  const Tensor4& out, void* mout, int mask_bytes, dim3 grid, hipStream_t st) {
  if (mask_bytes == 8)
    aug_apply_kernel<TO, int64_t><<<grid, kAugBlock, 0, st>>>(g, lut, part, nparts, norm, out,
                                                             static_cast<int64_t*>(mout));
  else
    aug_apply_kernel<TO, uint8_t><<<grid, kAugBlock, 0, st>>>(g, lut, part, nparts, norm, out,
                                                             static_cast<uint8_t*>(mout));
}

}  // namespace

int augment_stat_blocks(int ch, int cw) {
  const int64_t npix = static_cast<int64_t>(ch) * cw;
  return static_cast<int>(std::min<int64_t>(64, std::max<int64_t>(1, (npix + kAugBlock * 16 - 1) / (kAugBlock * 16))));
}

void launch_augment(const AugArgs& a, hipStream_t st) {
  AugGeo g{a.img, a.msk, a.params, a.h, a.w, a.ch, a.cw, a.pad_value, a.mask_pad};
  const int nb = augment_stat_blocks(a.ch, a.cw);
  if (a.part != nullptr) aug_stats_kernel<<<dim3(nb, a.n), kAugBlock, 0, st>>>(g, a.part);
  const int64_t npix = static_cast<int64_t>(a.ch) * a.cw;
  const int gx = static_cast<int>(std::min<int64_t>((npix + kAugBlock - 1) / kAugBlock, 4096 / std::max(1, a.n) + 1));
  const dim3 grid(std::max(gx, 1), a.n);
  switch (a.out.dtype) {
    case kF32: launch_apply<float>(g, a.lut, a.part, nb, a.norm, a.out, a.mout, a.mask_bytes, grid, st); break;
    case kBF16: launch_apply<uint16_t>(g, a.lut, a.part, nb, a.norm, a.out, a.mout, a.mask_bytes, grid, st); break;
    default: launch_apply<_Float16>(g, a.lut, a.part, nb, a.norm, a.out, a.mout, a.mask_bytes, grid, st); break;
  }
}

}  // namespace rtseg
