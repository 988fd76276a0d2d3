// 2-D pooling family for CDNA4 (gfx950): average / max pooling with fixed windows,
// adaptive average pooling (incl. the global 1x1 case) and their backward passes.
//
// Reference sites: DDRNet DAPPM AvgPool2d(5/9/17, s 2/4/8) + global pool
// (models/ddrnet.py:248-264), STDC AvgPool2d(3,2,1) on every stride-2 module
// (models/stdc.py:116), BiSeNetV2 stem MaxPool2d(3,2,1) / GE AvgPool / CE global pool
// (models/bisenetv2.py:117,131,144), PPM AdaptiveAvgPool(1,2,4,6) (models/modules.py:147),
// and every AdaptiveAvgPool2d(1) of the zoo and SMP decoders.
//
// Layout: NHWC (channels-last) activations; a work item is VEC contiguous channels
// of one output (forward) or input (backward) pixel, so every access is a 16-byte
// load/store for bf16 with C % 8 == 0.  Other layouts take the VEC = 1 strided path.
//
// * Forward: one item per output vector, loop over its window (semantics of ATen:
//   count_include_pad divisor clipped to the padded extent; max keeps the first
//   maximum in scan order and propagates the first NaN).  Max pooling also writes the
//   window-relative argmax as one uint8 per output element.
// * Backward: gather form (one item per INPUT vector, loop over the few windows that
//   cover it), so there are no atomics and the result is deterministic.  Max backward
//   compares the stored uint8 offsets -- no re-scan of the window.
// * Global average pooling (output 1x1) is a reduction: a block owns a channel slab
//   of one image and a slice of its pixels, rows of threads stride the pixels and
//   reduce through LDS; slices write fp32 partials that a second kernel sums, scales
//   and casts, so small batches still fill 256 CUs.
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_vec.h"

#include <algorithm>
#include <type_traits>

namespace rtseg {

namespace {

constexpr int kPoolBlock = 256;

struct PoolDivs {
  FastDiv c, w, h;  // channel vectors, width, height of the indexed space
};

__device__ __forceinline__ void adaptive_range(int o, int in, int out, int& s, int& e) {
  s = (o * in) / out;
  e = ((o + 1) * in + out - 1) / out;
}

template <typename T, int VEC, int MODE, bool ADAPT>
__global__ void __launch_bounds__(kPoolBlock) pool_fwd_kernel(Tensor4 x, Tensor4 y, PoolParams p, PoolDivs d,
                                                              uint8_t* __restrict__ idx, uint32_t total) {
  const T* xp = static_cast<const T*>(x.data);
  T* yp = static_cast<T*>(y.data);
  for (uint32_t i = blockIdx.x * kPoolBlock + threadIdx.x; i < total; i += gridDim.x * kPoolBlock) {
    uint32_t cv, ow, oh;
    const uint32_t r0 = d.c.divmod(i, cv);
    const uint32_t r1 = d.w.divmod(r0, ow);
    const uint32_t n = d.h.divmod(r1, oh);
    int hs, he, ws, we, hs0, ws0;
    float div = 1.f;
    if constexpr (ADAPT) {
      adaptive_range(static_cast<int>(oh), x.h, y.h, hs, he);
      adaptive_range(static_cast<int>(ow), x.w, y.w, ws, we);
      hs0 = hs;
      ws0 = ws;
      div = static_cast<float>((he - hs) * (we - ws));
    } else {
      hs0 = static_cast<int>(oh) * p.sh - p.ph;
      ws0 = static_cast<int>(ow) * p.sw - p.pw;
      he = min(hs0 + p.kh, x.h + p.ph);
      we = min(ws0 + p.kw, x.w + p.pw);
      const int padded = (he - hs0) * (we - ws0);
      hs = max(hs0, 0);
      ws = max(ws0, 0);
      he = min(he, x.h);
      we = min(we, x.w);
      div = static_cast<float>(p.count_include_pad ? padded : (he - hs) * (we - ws));
    }
    const int c0 = static_cast<int>(cv) * VEC;
    const T* xb = xp + static_cast<int64_t>(n) * x.sn + static_cast<int64_t>(c0) * x.sc;
    float acc[VEC];
    int arg[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      acc[v] = MODE == kPoolMax ? -INFINITY : 0.f;
      arg[v] = 0;
    }
    for (int ih = hs; ih < he; ++ih) {
      for (int iw = ws; iw < we; ++iw) {
        float v_[VEC];
        Vec<T, VEC>::load(xb + static_cast<int64_t>(ih) * x.sh + static_cast<int64_t>(iw) * x.sw, v_);
        if constexpr (MODE == kPoolMax) {
          const int o = (ih - hs0) * p.kw + (iw - ws0);
#pragma unroll
          for (int v = 0; v < VEC; ++v) {
            const bool take = v_[v] > acc[v] || (v_[v] != v_[v] && acc[v] == acc[v]);
            acc[v] = take ? v_[v] : acc[v];
            arg[v] = take ? o : arg[v];
          }
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[v] += v_[v];
        }
      }
    }
    if constexpr (MODE == kPoolAvg) {
      const float inv = 1.f / div;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] *= inv;
    }
    const int64_t yo = static_cast<int64_t>(n) * y.sn + static_cast<int64_t>(c0) * y.sc +
                       static_cast<int64_t>(oh) * y.sh + static_cast<int64_t>(ow) * y.sw;
    Vec<T, VEC>::store(yp + yo, acc);
    if constexpr (MODE == kPoolMax) {
      // idx is dense NHWC [n, oh, ow, c] whatever y's layout
      uint8_t* ib = idx + ((static_cast<int64_t>(n) * y.h + oh) * y.w + ow) * y.c + c0;
#pragma unroll
      for (int v = 0; v < VEC; ++v) ib[v] = static_cast<uint8_t>(arg[v]);
    }
  }
}

// Average pooling with large windows over few outputs (DDRNet's DAPPM: 5/9/17-tap windows
// on a 1/64-resolution map -> a few thousand output vectors, each a serial loop of up to 289
// loads): 16 lanes share one output vector, stride its window taps and reduce by shuffles.
template <typename T, int VEC, bool ADAPT>
__global__ void __launch_bounds__(kPoolBlock) pool_avg_split_kernel(Tensor4 x, Tensor4 y, PoolParams p, PoolDivs d,
                                                                    uint32_t total) {
  constexpr uint32_t G = 16;
  const T* xp = static_cast<const T*>(x.data);
  T* yp = static_cast<T*>(y.data);
  const int lane = threadIdx.x & (G - 1);
  for (uint32_t i = (blockIdx.x * kPoolBlock + threadIdx.x) / G; i < total; i += gridDim.x * (kPoolBlock / G)) {
    uint32_t cv, ow, oh;
    const uint32_t r0 = d.c.divmod(i, cv);
    const uint32_t r1 = d.w.divmod(r0, ow);
    const uint32_t n = d.h.divmod(r1, oh);
    int hs, he, ws, we;
    float div;
    if constexpr (ADAPT) {
      adaptive_range(static_cast<int>(oh), x.h, y.h, hs, he);
      adaptive_range(static_cast<int>(ow), x.w, y.w, ws, we);
      div = static_cast<float>((he - hs) * (we - ws));
    } else {
      const int hs0 = static_cast<int>(oh) * p.sh - p.ph, ws0 = static_cast<int>(ow) * p.sw - p.pw;
      he = min(hs0 + p.kh, x.h + p.ph);
      we = min(ws0 + p.kw, x.w + p.pw);
      const int padded = (he - hs0) * (we - ws0);
      hs = max(hs0, 0);
      ws = max(ws0, 0);
      he = min(he, x.h);
      we = min(we, x.w);
      div = static_cast<float>(p.count_include_pad ? padded : (he - hs) * (we - ws));
    }
    const int c0 = static_cast<int>(cv) * VEC;
    const T* xb = xp + static_cast<int64_t>(n) * x.sn + static_cast<int64_t>(c0) * x.sc;
    const int ww = we - ws, cnt = (he - hs) * ww;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    for (int t = lane; t < cnt; t += G) {
      const int dh = t / ww;
      const int ih = hs + dh, iw = ws + (t - dh * ww);
      float v_[VEC];
      Vec<T, VEC>::load(xb + static_cast<int64_t>(ih) * x.sh + static_cast<int64_t>(iw) * x.sw, v_);
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] += v_[v];
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] += __shfl_xor(acc[v], o, kWave);
    if (lane == 0) {
      const float inv = 1.f / div;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] *= inv;
      const int64_t yo = static_cast<int64_t>(n) * y.sn + static_cast<int64_t>(c0) * y.sc +
                         static_cast<int64_t>(oh) * y.sh + static_cast<int64_t>(ow) * y.sw;
      Vec<T, VEC>::store(yp + yo, acc);
    }
  }
}

template <typename T, int VEC, int MODE, bool ADAPT>
__global__ void __launch_bounds__(kPoolBlock) pool_bwd_kernel(Tensor4 gy, Tensor4 gx, PoolParams p, PoolDivs d,
                                                              const uint8_t* __restrict__ idx, uint32_t total) {
  const T* gp = static_cast<const T*>(gy.data);
  T* xp = static_cast<T*>(gx.data);
  for (uint32_t i = blockIdx.x * kPoolBlock + threadIdx.x; i < total; i += gridDim.x * kPoolBlock) {
    uint32_t cv, iw_, ih_;
    const uint32_t r0 = d.c.divmod(i, cv);
    const uint32_t r1 = d.w.divmod(r0, iw_);
    const uint32_t n = d.h.divmod(r1, ih_);
    const int ih = static_cast<int>(ih_), iw = static_cast<int>(iw_);
    int oh_lo, oh_hi, ow_lo, ow_hi;
    if constexpr (ADAPT) {
      oh_lo = max((ih * gy.h) / gx.h - 1, 0);
      oh_hi = min(((ih + 1) * gy.h) / gx.h + 1, gy.h - 1);
      ow_lo = max((iw * gy.w) / gx.w - 1, 0);
      ow_hi = min(((iw + 1) * gy.w) / gx.w + 1, gy.w - 1);
    } else {
      const int ah = ih + p.ph - p.kh + 1, aw = iw + p.pw - p.kw + 1;
      oh_lo = ah > 0 ? (ah + p.sh - 1) / p.sh : 0;
      ow_lo = aw > 0 ? (aw + p.sw - 1) / p.sw : 0;
      oh_hi = min((ih + p.ph) / p.sh, gy.h - 1);
      ow_hi = min((iw + p.pw) / p.sw, gy.w - 1);
    }
    const int c0 = static_cast<int>(cv) * VEC;
    const T* gb = gp + static_cast<int64_t>(n) * gy.sn + static_cast<int64_t>(c0) * gy.sc;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        float w = 1.f;
        int rel = 0;
        if constexpr (ADAPT) {
          int hs, he, ws, we;
          adaptive_range(oh, gx.h, gy.h, hs, he);
          adaptive_range(ow, gx.w, gy.w, ws, we);
          if (ih < hs || ih >= he || iw < ws || iw >= we) continue;
          w = 1.f / static_cast<float>((he - hs) * (we - ws));
        } else {
          const int hs0 = oh * p.sh - p.ph, ws0 = ow * p.sw - p.pw;
          if constexpr (MODE == kPoolAvg) {
            int he = min(hs0 + p.kh, gx.h + p.ph), we = min(ws0 + p.kw, gx.w + p.pw);
            int cnt = (he - hs0) * (we - ws0);
            if (!p.count_include_pad)
              cnt = (min(he, gx.h) - max(hs0, 0)) * (min(we, gx.w) - max(ws0, 0));
            w = 1.f / static_cast<float>(cnt);
          } else {
            rel = (ih - hs0) * p.kw + (iw - ws0);
          }
        }
        float g_[VEC];
        Vec<T, VEC>::load(gb + static_cast<int64_t>(oh) * gy.sh + static_cast<int64_t>(ow) * gy.sw, g_);
        if constexpr (MODE == kPoolMax) {
          const uint8_t* ib = idx + ((static_cast<int64_t>(n) * gy.h + oh) * gy.w + ow) * gy.c + c0;
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[v] += (static_cast<int>(ib[v]) == rel) ? g_[v] : 0.f;
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[v] = fmaf(w, g_[v], acc[v]);
        }
      }
    }
    const int64_t xo = static_cast<int64_t>(n) * gx.sn + static_cast<int64_t>(c0) * gx.sc +
                       static_cast<int64_t>(ih) * gx.sh + static_cast<int64_t>(iw) * gx.sw;
    Vec<T, VEC>::store(xp + xo, acc);
  }
}

// Global average pool, stage 1: block (cb, n, slice) sums pixels [slice*per, ...) of
// image n for channel vectors cb*cpb .. +cpb.  rows = 256 / cpb thread rows stride
// the pixels; LDS reduce over rows; fp32 partial [slice, n, C].
template <typename T, int VEC>
__global__ void __launch_bounds__(kPoolBlock) gap_partial_kernel(Tensor4 x, int cpb, int per_slice,
                                                                 float* __restrict__ part) {
  __shared__ float red[kPoolBlock * VEC];
  const T* xp = static_cast<const T*>(x.data);
  const int rows = kPoolBlock / cpb;
  const int r = threadIdx.x / cpb, cl = threadIdx.x - r * cpb;
  const int n = blockIdx.y;
  const int cv = blockIdx.x * cpb + cl;
  const int c0 = cv * VEC;
  const int hw = x.h * x.w;
  const int p_beg = blockIdx.z * per_slice;
  const int p_end = min(p_beg + per_slice, hw);
  float acc[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
  if (r < rows && c0 < x.c) {
    const T* xb = xp + static_cast<int64_t>(n) * x.sn + static_cast<int64_t>(c0) * x.sc;
    int ph = (p_beg + r) / x.w, pw = (p_beg + r) - ph * x.w;  // row/col of the first pixel
    const int dh = rows / x.w, dw = rows - dh * x.w;
    for (int q = p_beg + r; q < p_end; q += rows) {
      float v_[VEC];
      Vec<T, VEC>::load(xb + static_cast<int64_t>(ph) * x.sh + static_cast<int64_t>(pw) * x.sw, v_);
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] += v_[v];
      ph += dh;
      pw += dw;
      if (pw >= x.w) {
        pw -= x.w;
        ++ph;
      }
    }
  }
#pragma unroll
  for (int v = 0; v < VEC; ++v) red[(r * cpb + cl) * VEC + v] = acc[v];
  __syncthreads();
  if (r == 0 && c0 < x.c) {
    for (int rr = 1; rr < rows; ++rr) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] += red[(rr * cpb + cl) * VEC + v];
    }
    float* pb = part + (static_cast<int64_t>(blockIdx.z) * gridDim.y + n) * x.c + c0;
#pragma unroll
    for (int v = 0; v < VEC; ++v) pb[v] = acc[v];
  }
}

// stage 2: y[n, c] = sum_slices part / (H*W), cast to T (y is [N, C, 1, 1], any strides)
template <typename T>
__global__ void __launch_bounds__(kPoolBlock) gap_final_kernel(const float* __restrict__ part, int slices, int N,
                                                               int C, float inv, Tensor4 y) {
  T* yp = static_cast<T*>(y.data);
  for (int i = blockIdx.x * kPoolBlock + threadIdx.x; i < N * C; i += gridDim.x * kPoolBlock) {
    const int n = i / C, c = i - n * C;
    float s = 0.f;
    for (int k = 0; k < slices; ++k) s += part[(static_cast<int64_t>(k) * N + n) * C + c];
    Io<T>::st(yp + static_cast<int64_t>(n) * y.sn + static_cast<int64_t>(c) * y.sc, s * inv);
  }
}

template <typename F>
void by_dtype(int dt, F&& f) {
  switch (dt) {
    case kF32: f(float{}); break;
    case kBF16: f(uint16_t{}); break;
    default: f(_Float16{}); break;
  }
}

// VEC usable for a tensor: channel stride 1, C and the pixel strides multiples of VEC,
// base aligned to VEC elements.
int vec_of(const Tensor4& t, int want) {
  const int esz = t.dtype == kF32 ? 4 : 2;
  for (int v = want; v > 1; v >>= 1) {
    if (t.sc == 1 && t.c % v == 0 && t.sw % v == 0 && t.sh % v == 0 && t.sn % v == 0 &&
        reinterpret_cast<uintptr_t>(t.data) % (static_cast<uintptr_t>(v) * esz) == 0)
      return v;
  }
  return 1;
}

template <typename T, int VEC, typename F>
void with_vec(int vec, F&& f) {
  if constexpr (VEC == 1) {
    f(std::integral_constant<int, 1>{});
  } else {
    if (vec >= VEC) f(std::integral_constant<int, VEC>{});
    else with_vec<T, VEC / 2>(vec, f);
  }
}

int want_vec(int dt) { return dt == kF32 ? 4 : 8; }

}  // namespace

void launch_pool_fwd(const Tensor4& x, const Tensor4& y, const PoolParams& p, uint8_t* idx, hipStream_t st) {
  const int vec = std::min(vec_of(x, want_vec(x.dtype)), vec_of(y, want_vec(y.dtype)));
  by_dtype(x.dtype, [&](auto tag) {
    using T = decltype(tag);
    with_vec<T, 8>(vec, [&](auto vc) {
      constexpr int V = decltype(vc)::value;
      if constexpr (!(std::is_same_v<T, float> && V == 8)) {
        const uint32_t cvs = static_cast<uint32_t>(y.c / V);
        const uint32_t total = static_cast<uint32_t>(static_cast<int64_t>(y.n) * y.h * y.w * cvs);
        PoolDivs d{FastDiv::make(cvs), FastDiv::make(y.w), FastDiv::make(y.h)};
        const int g = stream_grid(total, kPoolBlock);
        // mean window size: taps per output (adaptive: input / output area)
        const int64_t taps = p.adaptive ? (static_cast<int64_t>(x.h) * x.w) / (static_cast<int64_t>(y.h) * y.w)
                                        : static_cast<int64_t>(p.kh) * p.kw;
        if (p.mode == kPoolAvg && taps >= 16 && total < 256u * 256u) {
          const int gs = stream_grid(static_cast<int64_t>(total) * 16, kPoolBlock);
          if (p.adaptive) pool_avg_split_kernel<T, V, true><<<gs, kPoolBlock, 0, st>>>(x, y, p, d, total);
          else pool_avg_split_kernel<T, V, false><<<gs, kPoolBlock, 0, st>>>(x, y, p, d, total);
        } else if (p.mode == kPoolMax)
          pool_fwd_kernel<T, V, kPoolMax, false><<<g, kPoolBlock, 0, st>>>(x, y, p, d, idx, total);
        else if (p.adaptive)
          pool_fwd_kernel<T, V, kPoolAvg, true><<<g, kPoolBlock, 0, st>>>(x, y, p, d, nullptr, total);
        else
          pool_fwd_kernel<T, V, kPoolAvg, false><<<g, kPoolBlock, 0, st>>>(x, y, p, d, nullptr, total);
      }
    });
  });
}

void launch_pool_bwd(const Tensor4& gy, const Tensor4& gx, const PoolParams& p, const uint8_t* idx, hipStream_t st) {
  const int vec = std::min(vec_of(gy, want_vec(gy.dtype)), vec_of(gx, want_vec(gx.dtype)));
  by_dtype(gy.dtype, [&](auto tag) {
    using T = decltype(tag);
    with_vec<T, 8>(vec, [&](auto vc) {
      constexpr int V = decltype(vc)::value;
      if constexpr (!(std::is_same_v<T, float> && V == 8)) {
        const uint32_t cvs = static_cast<uint32_t>(gx.c / V);
        const uint32_t total = static_cast<uint32_t>(static_cast<int64_t>(gx.n) * gx.h * gx.w * cvs);
        PoolDivs d{FastDiv::make(cvs), FastDiv::make(gx.w), FastDiv::make(gx.h)};
        const int g = stream_grid(total, kPoolBlock);
        if (p.mode == kPoolMax)
          pool_bwd_kernel<T, V, kPoolMax, false><<<g, kPoolBlock, 0, st>>>(gy, gx, p, d, idx, total);
        else if (p.adaptive)
          pool_bwd_kernel<T, V, kPoolAvg, true><<<g, kPoolBlock, 0, st>>>(gy, gx, p, d, nullptr, total);
        else
          pool_bwd_kernel<T, V, kPoolAvg, false><<<g, kPoolBlock, 0, st>>>(gy, gx, p, d, nullptr, total);
      }
    });
  });
}

GapPlan gap_plan(const Tensor4& x) {
  GapPlan pl;
  pl.vec = vec_of(x, want_vec(x.dtype));
  const int cvs = x.c / pl.vec;
  pl.cpb = cvs < kPoolBlock ? cvs : kPoolBlock;
  pl.cblocks = (cvs + pl.cpb - 1) / pl.cpb;
  const int hw = x.h * x.w;
  const int rows = kPoolBlock / pl.cpb;
  int slices = (512 + x.n * pl.cblocks - 1) / (x.n * pl.cblocks);
  const int max_slices = (hw + 16 * rows - 1) / (16 * rows);  // >= 16 pixels per thread row
  if (slices > max_slices) slices = max_slices;
  if (slices < 1) slices = 1;
  if (slices > 65535) slices = 65535;
  pl.per_slice = (hw + slices - 1) / slices;
  pl.slices = (hw + pl.per_slice - 1) / pl.per_slice;
  return pl;
}

void launch_gap_fwd(const Tensor4& x, const Tensor4& y, const GapPlan& pl, float* part, hipStream_t st) {
  by_dtype(x.dtype, [&](auto tag) {
    using T = decltype(tag);
    with_vec<T, 8>(pl.vec, [&](auto vc) {
      constexpr int V = decltype(vc)::value;
      if constexpr (!(std::is_same_v<T, float> && V == 8)) {
        dim3 grid(pl.cblocks, x.n, pl.slices);
        gap_partial_kernel<T, V><<<grid, kPoolBlock, 0, st>>>(x, pl.cpb, pl.per_slice, part);
      }
    });
    const int nc = x.n * x.c;
    gap_final_kernel<T><<<stream_grid(nc, kPoolBlock), kPoolBlock, 0, st>>>(
        part, pl.slices, x.n, x.c, 1.f / static_cast<float>(x.h * x.w), y);
  });
}

}  // namespace rtseg

// ---------------------------------------------------------------------------------------------
// MaxPool2d(return_indices=True) / MaxUnpool2d (reference enet.py:131,139, segnet.py:54,65).
// Indices follow PyTorch: int64 flat offsets h * W + w into each input plane.  Unpooling with
// kernel == stride and no padding (the paired pool's windows tile the plane) is a GATHER: output
// pixel (h, w) belongs to exactly one window (h / kh, w / kw) and takes that window's value iff
// the window's index names it -- every output is written once, no zero-fill, no scatter.  The
// same kernel is the backward of the indexed max pool.
namespace rtseg {
namespace {

template <typename T>
__global__ void __launch_bounds__(256) unpool_gather_kernel(Tensor4 x, Tensor4 idx, Tensor4 y, int kh, int kw) {
  const int64_t total = static_cast<int64_t>(y.n) * y.c * y.h * y.w;
  const T* xs = static_cast<const T*>(x.data);
  const int64_t* is = static_cast<const int64_t*>(idx.data);
  T* ys = static_cast<T*>(y.data);
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    // e enumerates y in (n, h, w, c) order: channel-fastest, coalesced for channels-last y
    const int c = static_cast<int>(e % y.c);
    int64_t r = e / y.c;
    const int w = static_cast<int>(r % y.w);
    r /= y.w;
    const int h = static_cast<int>(r % y.h);
    const int n = static_cast<int>(r / y.h);
    const int i = h / kh, j = w / kw;
    float v = 0.f;
    if (i < x.h && j < x.w) {
      const int64_t want = static_cast<int64_t>(h) * y.w + w;
      if (is[n * idx.sn + c * idx.sc + i * idx.sh + j * idx.sw] == want)
        v = Io<T>::ld(xs + n * x.sn + c * x.sc + i * x.sh + j * x.sw);
    }
    Io<T>::st(ys + n * y.sn + c * y.sc + h * y.sh + w * y.sw, v);
  }
}

// gx[n, c, i, j] = gy[n, c, idx / W, idx % W]   (backward of the unpool)
template <typename T>
__global__ void __launch_bounds__(256) unpool_bwd_kernel(Tensor4 gy, Tensor4 idx, Tensor4 gx) {
  const int64_t total = static_cast<int64_t>(gx.n) * gx.c * gx.h * gx.w;
  const T* gs = static_cast<const T*>(gy.data);
  const int64_t* is = static_cast<const int64_t*>(idx.data);
  T* xs = static_cast<T*>(gx.data);
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(e % gx.c);
    int64_t r = e / gx.c;
    const int j = static_cast<int>(r % gx.w);
    r /= gx.w;
    const int i = static_cast<int>(r % gx.h);
    const int n = static_cast<int>(r / gx.h);
    const int64_t f = is[n * idx.sn + c * idx.sc + i * idx.sh + j * idx.sw];
    float v = 0.f;
    if (f >= 0 && f < static_cast<int64_t>(gy.h) * gy.w) {
      const int64_t hh = f / gy.w, ww = f - hh * gy.w;
      v = Io<T>::ld(gs + n * gy.sn + c * gy.sc + hh * gy.sh + ww * gy.sw);
    }
    Io<T>::st(xs + n * gx.sn + c * gx.sc + i * gx.sh + j * gx.sw, v);
  }
}

// uint8 window offsets [N, OH, OW, C] (pool2d_fwd's argmax map) -> int64 flat plane indices
__global__ void __launch_bounds__(256) maxpool_flat_index_kernel(const uint8_t* __restrict__ win, Tensor4 out,
                                                                 int in_w, PoolParams p) {
  const int64_t total = static_cast<int64_t>(out.n) * out.c * out.h * out.w;
  int64_t* os = static_cast<int64_t*>(out.data);
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(e % out.c);
    int64_t r = e / out.c;
    const int ow = static_cast<int>(r % out.w);
    r /= out.w;
    const int oh = static_cast<int>(r % out.h);
    const int n = static_cast<int>(r / out.h);
    const int k = win[e];
    const int hh = oh * p.sh - p.ph + k / p.kw, ww = ow * p.sw - p.pw + k % p.kw;
    os[n * out.sn + c * out.sc + oh * out.sh + ow * out.sw] = static_cast<int64_t>(hh) * in_w + ww;
  }
}

}  // namespace

void launch_unpool_gather(const Tensor4& x, const Tensor4& idx, const Tensor4& y, int kh, int kw, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(y.n) * y.c * y.h * y.w;
  by_dtype(y.dtype, [&](auto tag) {
    using T = decltype(tag);
    unpool_gather_kernel<T><<<stream_grid(total, 256), 256, 0, st>>>(x, idx, y, kh, kw);
  });
}

void launch_unpool_bwd(const Tensor4& gy, const Tensor4& idx, const Tensor4& gx, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(gx.n) * gx.c * gx.h * gx.w;
  by_dtype(gx.dtype, [&](auto tag) {
    using T = decltype(tag);
    unpool_bwd_kernel<T><<<stream_grid(total, 256), 256, 0, st>>>(gy, idx, gx);
  });
}

void launch_maxpool_flat_index(const uint8_t* win, const Tensor4& out, int in_w, const PoolParams& p,
                               hipStream_t st) {
  const int64_t total = static_cast<int64_t>(out.n) * out.c * out.h * out.w;
  maxpool_flat_index_kernel<<<stream_grid(total, 256), 256, 0, st>>>(win, out, in_w, p);
}

}  // namespace rtseg

// ---------------------------------------------------------------------------------------------
// Global max pool with argmax (AdaptiveMaxPool2d(1): canet.py:103, dfanet.py:149,
// pp_liteseg.py:190).  Block = (image, 64-channel group); 4 rows of 64 lanes scan the plane
// (channel-fastest lanes: coalesced for channels-last), LDS merge.  Ties keep the first pixel
// and NaN wins, as ATen's adaptive max pool.  idx: int64 flat plane index [N, C].
namespace rtseg {
namespace {

__device__ __forceinline__ bool gmax_better(float v, int i, float m, int mi) {
  if (v != v) return !(m != m) || i < mi;  // NaN propagates (first NaN)
  if (m != m) return false;
  return v > m || (v == m && i < mi);
}

template <typename T>
__global__ void __launch_bounds__(256) global_max_kernel(Tensor4 x, T* __restrict__ y, int64_t* __restrict__ idx) {
  __shared__ float sm[256];
  __shared__ int si[256];
  const int n = blockIdx.y, c = blockIdx.x * 64 + (threadIdx.x & 63), row = threadIdx.x >> 6;
  const T* xp = static_cast<const T*>(x.data);
  const int hw = x.h * x.w;
  float m = -INFINITY;
  int mi = 0x7fffffff;
  if (c < x.c) {
    const T* xb = xp + static_cast<int64_t>(n) * x.sn + static_cast<int64_t>(c) * x.sc;
    for (int p = row; p < hw; p += 4) {
      const int hh = p / x.w, ww = p - hh * x.w;
      const float v = Io<T>::ld(xb + static_cast<int64_t>(hh) * x.sh + static_cast<int64_t>(ww) * x.sw);
      if (gmax_better(v, p, m, mi)) { m = v; mi = p; }
    }
  }
  sm[threadIdx.x] = m;
  si[threadIdx.x] = mi;
  __syncthreads();
  if (row == 0 && c < x.c) {
    for (int r = 1; r < 4; ++r) {
      const float v = sm[threadIdx.x + 64 * r];
      const int i = si[threadIdx.x + 64 * r];
      if (gmax_better(v, i, m, mi)) { m = v; mi = i; }
    }
    Io<T>::st(y + static_cast<int64_t>(n) * x.c + c, m);
    idx[static_cast<int64_t>(n) * x.c + c] = mi == 0x7fffffff ? 0 : mi;
  }
}

}  // namespace

// y: dense [N, C] of x's dtype, idx: int64 [N, C]
void launch_global_max(const Tensor4& x, void* y, int64_t* idx, hipStream_t st) {
  by_dtype(x.dtype, [&](auto tag) {
    using T = decltype(tag);
    global_max_kernel<T><<<dim3((x.c + 63) / 64, x.n), 256, 0, st>>>(x, static_cast<T*>(y), idx);
  });
}

}  // namespace rtseg
