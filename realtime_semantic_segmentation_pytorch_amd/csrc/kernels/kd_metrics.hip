// Knowledge-distillation KL loss and the mIoU confusion matrix for CDNA4 (gfx950).
//
// KD (reference core/loss.py:80-88):
//   loss = T^2 / (N*C*H*W) * sum_{n,h,w} KL( softmax(t/T) || softmax(s/T) )
// Per pixel  KL = sum_c p_t,c (b_c - a_c) - lse(b) + lse(a),   a = s/T, b = t/T,
// so the forward needs one max pass and one exp pass over the C logits of both
// tensors (the second pass hits L1/L2).  The forward stores lse(a), lse(b) per
// pixel, which makes the backward a single streaming pass:
//   dL/ds_c = g * T / numel * (exp(a_c - lse_a) - exp(b_c - lse_b)).
// Partial sums are per block (fp64) and reduced by one finalize block, so the
// loss is deterministic and never touches the host.
//
// Confusion matrix (reference utils/metrics.py:4-7 via torchmetrics
// JaccardIndex): argmax over C fused with an LDS-private C x C histogram, one
// global 64-bit atomic per non-empty bin per block.
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

namespace {

struct PixIdx {
  int hw, w;
  __device__ __forceinline__ void split(int64_t p, int& n, int& h, int& x) const {
    n = static_cast<int>(p / hw);
    const int r = static_cast<int>(p - static_cast<int64_t>(n) * hw);
    h = r / w;
    x = r - h * w;
  }
};

constexpr int kKdBlock = 256;

template <typename T>
__global__ void __launch_bounds__(kKdBlock) kd_fwd_kernel(Tensor4 s, Tensor4 t, float inv_t,
                                                          float* lse, double* part) {
  const T* sp = static_cast<const T*>(s.data);
  const T* tp = static_cast<const T*>(t.data);
  const int64_t npix = static_cast<int64_t>(s.n) * s.h * s.w;
  const PixIdx pi{s.h * s.w, s.w};
  double acc = 0.0;
  for (int64_t p = blockIdx.x * static_cast<int64_t>(kKdBlock) + threadIdx.x; p < npix;
       p += static_cast<int64_t>(gridDim.x) * kKdBlock) {
    int n, h, x;
    pi.split(p, n, h, x);
    const int64_t so = n * s.sn + h * s.sh + x * s.sw;
    const int64_t to = n * t.sn + h * t.sh + x * t.sw;
    float ma = -INFINITY, mb = -INFINITY;
    for (int c = 0; c < s.c; ++c) {
      ma = fmaxf(ma, Io<T>::ld(sp + so + c * s.sc) * inv_t);
      mb = fmaxf(mb, Io<T>::ld(tp + to + c * t.sc) * inv_t);
    }
    float za = 0.f, zb = 0.f, cross = 0.f;
    for (int c = 0; c < s.c; ++c) {
      const float a = Io<T>::ld(sp + so + c * s.sc) * inv_t;
      const float b = Io<T>::ld(tp + to + c * t.sc) * inv_t;
      za += __expf(a - ma);
      const float eb = __expf(b - mb);
      zb += eb;
      cross += eb * (b - a);
    }
    const float la = ma + __logf(za), lb = mb + __logf(zb);
    lse[p] = la;
    lse[npix + p] = lb;
    acc += static_cast<double>(cross / zb - lb + la);
  }
  __shared__ double red[kKdBlock / kWave];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(kKdBlock) kd_finalize_kernel(const double* part, int nparts, double scale,
                                                               float* out) {
  double v = 0.0;
  for (int i = threadIdx.x; i < nparts; i += kKdBlock) v += part[i];
  __shared__ double red[kKdBlock / kWave];
  v = block_sum(v, red);
  if (threadIdx.x == 0) *out = static_cast<float>(v * scale);
}

template <typename T>
__global__ void __launch_bounds__(kKdBlock) kd_bwd_kernel(Tensor4 s, Tensor4 t, Tensor4 gs, float inv_t,
                                                          const float* lse, const float* gout,
                                                          float coef) {
  const T* sp = static_cast<const T*>(s.data);
  const T* tp = static_cast<const T*>(t.data);
  T* gp = static_cast<T*>(gs.data);
  const int64_t npix = static_cast<int64_t>(s.n) * s.h * s.w;
  const PixIdx pi{s.h * s.w, s.w};
  const float k = *gout * coef;
  for (int64_t p = blockIdx.x * static_cast<int64_t>(kKdBlock) + threadIdx.x; p < npix;
       p += static_cast<int64_t>(gridDim.x) * kKdBlock) {
    int n, h, x;
    pi.split(p, n, h, x);
    const int64_t so = n * s.sn + h * s.sh + x * s.sw;
    const int64_t to = n * t.sn + h * t.sh + x * t.sw;
    const int64_t go = n * gs.sn + h * gs.sh + x * gs.sw;
    const float la = lse[p], lb = lse[npix + p];
    for (int c = 0; c < s.c; ++c) {
      const float a = Io<T>::ld(sp + so + c * s.sc) * inv_t;
      const float b = Io<T>::ld(tp + to + c * t.sc) * inv_t;
      Io<T>::st(gp + go + c * gs.sc, k * (__expf(a - la) - __expf(b - lb)));
    }
  }
}

// ---- channels-last, LDS-staged variants ----------------------------------------
// With NHWC logits a pixel's C (e.g. 19) channels are 38 contiguous bytes, so a
// per-pixel thread's scalar loads make every wave-instruction touch ~38 cache lines
// (the texture path, not HBM, was the limit: 6x off roofline).  Here a block stages
// its 256 pixels x C channels of both tensors with coalesced 16-byte loads into LDS,
// computes per pixel from LDS, and (backward) stages the gradient the same way out.
constexpr int kKdPix = 256;

template <typename T>
__device__ __forceinline__ void stage_in(const T* __restrict__ g, int64_t first, int64_t nelem, T* lds) {
  // g + first is 16-byte aligned (host check); nelem elements, tail handled per element
  const int64_t nvec = nelem * static_cast<int64_t>(sizeof(T)) / 16;
  const uint4* src = reinterpret_cast<const uint4*>(g + first);
  uint4* dst = reinterpret_cast<uint4*>(lds);
  for (int64_t v = threadIdx.x; v < nvec; v += kKdPix) dst[v] = src[v];
  for (int64_t e = nvec * 16 / static_cast<int64_t>(sizeof(T)) + threadIdx.x; e < nelem; e += kKdPix)
    lds[e] = g[first + e];
}

// Student logits at the head's resolution with the model's final bilinear upsample folded in
// (ops/kd.py: the trainer's DeferredLogits): the staged student values of a full-resolution pixel
// are interpolated from the low-resolution channels-last tensor -- the same arithmetic and bf16
// rounding as interp.hip's interp_fwd_cl_pix_lds -- instead of read from a materialised full-
// resolution copy (0.64 GB written and read twice per KD step at batch 16, 1024 x 2048).
struct KdFold {
  const void* lo;          // [N][Hl][Wl][C] dense channels-last
  int hl, wl;
  LinMap mh, mw;
  FastDiv fw, fh;          // full-resolution W, H
};

template <typename T>
__device__ __forceinline__ void stage_fold(const KdFold& f, int C, int64_t p0, int np, T* lds) {
  const int i = threadIdx.x;
  if (i >= np) return;
  uint32_t ox, oy;
  const uint32_t r1 = f.fw.divmod(static_cast<uint32_t>(p0 + i), ox);
  const int n = static_cast<int>(f.fh.divmod(r1, oy));
  int y0, y1, x0, x1;
  float ly, lx;
  f.mh.map(static_cast<int>(oy), y0, y1, ly);
  f.mw.map(static_cast<int>(ox), x0, x1, lx);
  const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx), w11 = ly * lx;
  const T* b = static_cast<const T*>(f.lo) + static_cast<int64_t>(n) * f.hl * f.wl * C;
  const T* p00 = b + (static_cast<int64_t>(y0) * f.wl + x0) * C;
  const T* p01 = b + (static_cast<int64_t>(y0) * f.wl + x1) * C;
  const T* p10 = b + (static_cast<int64_t>(y1) * f.wl + x0) * C;
  const T* p11 = b + (static_cast<int64_t>(y1) * f.wl + x1) * C;
  T* q = lds + i * C;
  for (int c = 0; c < C; ++c) {
    const float v = w00 * Io<T>::ld(p00 + c) + w01 * Io<T>::ld(p01 + c) + w10 * Io<T>::ld(p10 + c) +
                    w11 * Io<T>::ld(p11 + c);
    Io<T>::st(q + c, v);
  }
}

template <typename T, bool FOLD = false>
__global__ void __launch_bounds__(kKdPix) kd_fwd_cl_kernel(const T* __restrict__ s, const T* __restrict__ t, int C,
                                                           int64_t npix, float inv_t, float* lse, double* part,
                                                           KdFold fold = {}) {
  extern __shared__ __attribute__((aligned(16))) unsigned char kd_lds[];
  T* ls = reinterpret_cast<T*>(kd_lds);
  T* lt = ls + kKdPix * C;
  double acc = 0.0;
  for (int64_t p0 = static_cast<int64_t>(blockIdx.x) * kKdPix; p0 < npix; p0 += static_cast<int64_t>(gridDim.x) * kKdPix) {
    const int np = static_cast<int>(npix - p0 < kKdPix ? npix - p0 : kKdPix);
    __syncthreads();
    if constexpr (FOLD) stage_fold(fold, C, p0, np, ls);
    else stage_in(s, p0 * C, static_cast<int64_t>(np) * C, ls);
    stage_in(t, p0 * C, static_cast<int64_t>(np) * C, lt);
    __syncthreads();
    if (static_cast<int>(threadIdx.x) < np) {
      const T* a_ = ls + threadIdx.x * C;
      const T* b_ = lt + threadIdx.x * C;
      float ma = -INFINITY, mb = -INFINITY;
      for (int c = 0; c < C; ++c) {
        ma = fmaxf(ma, Io<T>::ld(a_ + c) * inv_t);
        mb = fmaxf(mb, Io<T>::ld(b_ + c) * inv_t);
      }
      float za = 0.f, zb = 0.f, cross = 0.f;
      for (int c = 0; c < C; ++c) {
        const float a = Io<T>::ld(a_ + c) * inv_t, b = Io<T>::ld(b_ + c) * inv_t;
        za += __expf(a - ma);
        const float eb = __expf(b - mb);
        zb += eb;
        cross += eb * (b - a);
      }
      const float la = ma + __logf(za), lb = mb + __logf(zb);
      const int64_t p = p0 + threadIdx.x;
      lse[p] = la;
      lse[npix + p] = lb;
      acc += static_cast<double>(cross / zb - lb + la);
    }
  }
  __shared__ double red[kKdPix / kWave];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

template <typename T, bool FOLD = false>
__global__ void __launch_bounds__(kKdPix) kd_bwd_cl_kernel(const T* __restrict__ s, const T* __restrict__ t,
                                                           T* __restrict__ gs, int C, int64_t npix, float inv_t,
                                                           const float* lse, const float* gout, float coef,
                                                           KdFold fold = {}) {
  extern __shared__ __attribute__((aligned(16))) unsigned char kd_lds[];
  T* ls = reinterpret_cast<T*>(kd_lds);
  T* lt = ls + kKdPix * C;
  const float k = *gout * coef;
  for (int64_t p0 = static_cast<int64_t>(blockIdx.x) * kKdPix; p0 < npix; p0 += static_cast<int64_t>(gridDim.x) * kKdPix) {
    const int np = static_cast<int>(npix - p0 < kKdPix ? npix - p0 : kKdPix);
    __syncthreads();
    if constexpr (FOLD) stage_fold(fold, C, p0, np, ls);
    else stage_in(s, p0 * C, static_cast<int64_t>(np) * C, ls);
    stage_in(t, p0 * C, static_cast<int64_t>(np) * C, lt);
    __syncthreads();
    if (static_cast<int>(threadIdx.x) < np) {
      const int64_t p = p0 + threadIdx.x;
      const float la = lse[p], lb = lse[npix + p];
      T* a_ = ls + threadIdx.x * C;
      const T* b_ = lt + threadIdx.x * C;
      for (int c = 0; c < C; ++c) {  // gradient overwrites the staged student logits in place
        const float a = Io<T>::ld(a_ + c) * inv_t, b = Io<T>::ld(b_ + c) * inv_t;
        Io<T>::st(a_ + c, k * (__expf(a - la) - __expf(b - lb)));
      }
    }
    __syncthreads();
    const int64_t nelem = static_cast<int64_t>(np) * C;
    const int64_t nvec = nelem * static_cast<int64_t>(sizeof(T)) / 16;
    uint4* dst = reinterpret_cast<uint4*>(gs + p0 * C);
    const uint4* src = reinterpret_cast<const uint4*>(ls);
    for (int64_t v = threadIdx.x; v < nvec; v += kKdPix) dst[v] = src[v];
    for (int64_t e = nvec * 16 / static_cast<int64_t>(sizeof(T)) + threadIdx.x; e < nelem; e += kKdPix)
      gs[p0 * C + e] = ls[e];
  }
}

// ---- confusion matrix ---------------------------------------------------------
constexpr int kCmBlock = 256;

template <typename T, bool LDS>
__global__ void __launch_bounds__(kCmBlock) confmat_kernel(Tensor4 x, const int64_t* target, int ignore,
                                                           unsigned long long* cm) {
  extern __shared__ unsigned hist[];
  const int C = x.c;
  if constexpr (LDS) {
    for (int i = threadIdx.x; i < C * C; i += kCmBlock) hist[i] = 0u;
    __syncthreads();
  }
  const T* xp = static_cast<const T*>(x.data);
  const int64_t npix = static_cast<int64_t>(x.n) * x.h * x.w;
  const PixIdx pi{x.h * x.w, x.w};
  for (int64_t p = blockIdx.x * static_cast<int64_t>(kCmBlock) + threadIdx.x; p < npix;
       p += static_cast<int64_t>(gridDim.x) * kCmBlock) {
    const int64_t lbl = target[p];
    if (lbl == ignore || lbl < 0 || lbl >= C) continue;
    int n, h, w;
    pi.split(p, n, h, w);
    const T* q = xp + n * x.sn + h * x.sh + w * x.sw;
    float best = Io<T>::ld(q);
    int arg = 0;
    for (int c = 1; c < C; ++c) {
      const float v = Io<T>::ld(q + c * x.sc);
      if (v > best || (v != v && best == best)) { best = v; arg = c; }  // NaN wins, like torch.argmax
    }
    const int bin = static_cast<int>(lbl) * C + arg;
    if constexpr (LDS) atomicAdd(&hist[bin], 1u);
    else atomicAdd(&cm[bin], 1ull);
  }
  if constexpr (LDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < C * C; i += kCmBlock) {
      const unsigned v = hist[i];
      if (v) atomicAdd(&cm[i], static_cast<unsigned long long>(v));
    }
  }
}

template <typename F>
void by_dtype(int dtype, F&& f) {
  if (dtype == kF32) f(float{});
  else if (dtype == kBF16) f(uint16_t{});
  else f(_Float16{});
}

}  // namespace

int kd_partial_blocks(int64_t npix) { return stream_grid(npix, kKdBlock); }

// dense channels-last (NHWC-contiguous), 16-byte aligned, LDS-sized channel count
static bool kd_cl_ok(const Tensor4& a) {
  const int64_t esz = a.dtype == kF32 ? 4 : 2;
  return a.sc == 1 && a.sw == a.c && a.sh == static_cast<int64_t>(a.w) * a.c &&
         a.sn == static_cast<int64_t>(a.h) * a.w * a.c && (reinterpret_cast<uintptr_t>(a.data) % 16) == 0 &&
         2 * kKdPix * a.c * esz <= 64 * 1024;
}

static size_t kd_lds_bytes(const Tensor4& a) { return 2 * kKdPix * static_cast<size_t>(a.c) * (a.dtype == kF32 ? 4 : 2); }

void launch_kd_fwd(const Tensor4& s, const Tensor4& t, float temperature, float* lse, double* part,
                   float* out, hipStream_t st) {
  const int64_t npix = static_cast<int64_t>(s.n) * s.h * s.w;
  const int g = kd_partial_blocks(npix);
  const float inv_t = 1.f / temperature;
  const bool cl = kd_cl_ok(s) && kd_cl_ok(t);
  by_dtype(s.dtype, [&](auto tag) {
    using T = decltype(tag);
    if (cl)
      kd_fwd_cl_kernel<T><<<g, kKdPix, kd_lds_bytes(s), st>>>(static_cast<const T*>(s.data),
                                                              static_cast<const T*>(t.data), s.c, npix, inv_t, lse, part);
    else
      kd_fwd_kernel<T><<<g, kKdBlock, 0, st>>>(s, t, inv_t, lse, part);
  });
  const double numel = static_cast<double>(npix) * s.c;
  const double scale = static_cast<double>(temperature) * temperature / numel;
  kd_finalize_kernel<<<1, kKdBlock, 0, st>>>(part, g, scale, out);
}

// student logits s_lo at head resolution, the model's final bilinear upsample to t's size folded
// in (KdFold); t and gs dense channels-last at full resolution
static KdFold make_fold(const Tensor4& s_lo, const Tensor4& t, bool align) {
  KdFold f;
  f.lo = s_lo.data;
  f.hl = s_lo.h;
  f.wl = s_lo.w;
  f.mh = LinMap::make(s_lo.h, t.h, align);
  f.mw = LinMap::make(s_lo.w, t.w, align);
  f.fw = FastDiv::make(t.w);
  f.fh = FastDiv::make(t.h);
  return f;
}

bool kd_fold_ok(const Tensor4& s_lo, const Tensor4& t) {
  return kd_cl_ok(s_lo) && kd_cl_ok(t) && s_lo.dtype == t.dtype && s_lo.c == t.c && s_lo.n == t.n &&
         static_cast<int64_t>(t.n) * t.h * t.w < (int64_t{1} << 31);
}

void launch_kd_fwd_fold(const Tensor4& s_lo, const Tensor4& t, bool align, float temperature, float* lse, double* part,
                        float* out, hipStream_t st) {
  const int64_t npix = static_cast<int64_t>(t.n) * t.h * t.w;
  const int g = kd_partial_blocks(npix);
  const float inv_t = 1.f / temperature;
  const KdFold f = make_fold(s_lo, t, align);
  by_dtype(t.dtype, [&](auto tag) {
    using T = decltype(tag);
    kd_fwd_cl_kernel<T, true><<<g, kKdPix, kd_lds_bytes(t), st>>>(nullptr, static_cast<const T*>(t.data), t.c, npix,
                                                                   inv_t, lse, part, f);
  });
  const double numel = static_cast<double>(npix) * t.c;
  const double scale = static_cast<double>(temperature) * temperature / numel;
  kd_finalize_kernel<<<1, kKdBlock, 0, st>>>(part, g, scale, out);
}

void launch_kd_bwd_fold(const Tensor4& s_lo, const Tensor4& t, const Tensor4& gs, bool align, float temperature,
                        const float* lse, const float* gout, hipStream_t st) {
  const int64_t npix = static_cast<int64_t>(t.n) * t.h * t.w;
  const int g = kd_partial_blocks(npix);
  const double numel = static_cast<double>(npix) * t.c;
  const float coef = static_cast<float>(static_cast<double>(temperature) / numel);
  const KdFold f = make_fold(s_lo, t, align);
  by_dtype(t.dtype, [&](auto tag) {
    using T = decltype(tag);
    kd_bwd_cl_kernel<T, true><<<g, kKdPix, kd_lds_bytes(t), st>>>(nullptr, static_cast<const T*>(t.data),
                                                                   static_cast<T*>(gs.data), t.c, npix, 1.f / temperature,
                                                                   lse, gout, coef, f);
  });
}

void launch_kd_bwd(const Tensor4& s, const Tensor4& t, const Tensor4& gs, float temperature,
                   const float* lse, const float* gout, hipStream_t st) {
  const int64_t npix = static_cast<int64_t>(s.n) * s.h * s.w;
  const int g = kd_partial_blocks(npix);
  const double numel = static_cast<double>(npix) * s.c;
  const float coef = static_cast<float>(static_cast<double>(temperature) / numel);
  const bool cl = kd_cl_ok(s) && kd_cl_ok(t) && kd_cl_ok(gs);
  by_dtype(s.dtype, [&](auto tag) {
    using T = decltype(tag);
    if (cl)
      kd_bwd_cl_kernel<T><<<g, kKdPix, kd_lds_bytes(s), st>>>(static_cast<const T*>(s.data), static_cast<const T*>(t.data),
                                                              static_cast<T*>(gs.data), s.c, npix, 1.f / temperature, lse,
                                                              gout, coef);
    else
      kd_bwd_kernel<T><<<g, kKdBlock, 0, st>>>(s, t, gs, 1.f / temperature, lse, gout, coef);
  });
}

void launch_confmat(const Tensor4& x, const int64_t* target, int ignore, unsigned long long* cm,
                    hipStream_t st) {
  const int64_t npix = static_cast<int64_t>(x.n) * x.h * x.w;
  const int g = stream_grid(npix, kCmBlock);
  const size_t lds = static_cast<size_t>(x.c) * x.c * sizeof(unsigned);
  const bool use_lds = lds <= 64 * 1024;
  by_dtype(x.dtype, [&](auto tag) {
    using T = decltype(tag);
    if (use_lds) confmat_kernel<T, true><<<g, kCmBlock, lds, st>>>(x, target, ignore, cm);
    else confmat_kernel<T, false><<<g, kCmBlock, 0, st>>>(x, target, ignore, cm);
  });
}

}  // namespace rtseg
