// Bilinear resize (align_corners True/False) with a fused "+ skip, activation"
// epilogue, and an atomic-free gather backward.
//
// Replaces the reference's F.interpolate(..., mode='bilinear') call sites
// (78 of them, e.g. reference models/ddrnet.py:233-236 BilateralFusion,
// ddrnet.py:275-289 DAPPM, modules.py:150-153 PPM) and the
// "upsample + add (+relu)" feature-fusion pattern that follows most of them.
//
// Layouts: any strided 4-D tensor. Channels-last bf16 tensors whose channel
// count is a multiple of 8 take a 16-byte vector path (one thread = 8
// channels of one pixel), everything else a scalar path walking the output in
// memory order. Backward is a gather (each input pixel sums the output pixels
// that read it) so no float atomics are issued.
#include "rtseg_common.h"
#include "rtseg_launch.h"

#include <cstdlib>

namespace rtseg {

struct Shape4 { int n, c, h, w; int64_t sn, sc, sh, sw; };

__device__ __forceinline__ int64_t off4(const Shape4& s, int n, int c, int h, int w) {
  return n * s.sn + c * s.sc + h * s.sh + w * s.sw;
}

// ------------------------------- forward -----------------------------------
template <typename T, int ACT, bool SKIP>
__global__ void __launch_bounds__(256) interp_fwd_scalar(
    const T* __restrict__ x, Shape4 xs, const T* __restrict__ skip, Shape4 ks,
    T* __restrict__ y, Shape4 ys, LinMap mh, LinMap mw) {
  const int64_t total = static_cast<int64_t>(ys.n) * ys.c * ys.h * ys.w;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int ox = static_cast<int>(i % ys.w);
    int64_t t = i / ys.w;
    int oy = static_cast<int>(t % ys.h);
    t /= ys.h;
    int c = static_cast<int>(t % ys.c);
    int n = static_cast<int>(t / ys.c);
    int y0, y1, x0, x1; float ly, lx;
    mh.map(oy, y0, y1, ly);
    mw.map(ox, x0, x1, lx);
    const T* b = x + n * xs.sn + c * xs.sc;
    float v00 = Io<T>::ld(b + y0 * xs.sh + x0 * xs.sw);
    float v01 = Io<T>::ld(b + y0 * xs.sh + x1 * xs.sw);
    float v10 = Io<T>::ld(b + y1 * xs.sh + x0 * xs.sw);
    float v11 = Io<T>::ld(b + y1 * xs.sh + x1 * xs.sw);
    float v = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
    if constexpr (SKIP) v += Io<T>::ld(skip + off4(ks, n, c, oy, ox));
    Io<T>::st(y + off4(ys, n, c, oy, ox), act_fwd<ACT>(v));
  }
}

// Channels-last output with a channel count that is not a multiple of 8 (e.g.
// 19-class logits): walk the output in NHWC order so stores stay coalesced.
template <typename T, int ACT, bool SKIP>
__global__ void __launch_bounds__(256) interp_fwd_cl_scalar(
    const T* __restrict__ x, Shape4 xs, const T* __restrict__ skip, Shape4 ks,
    T* __restrict__ y, Shape4 ys, LinMap mh, LinMap mw, FastDiv fc, FastDiv fw, FastDiv fh, uint32_t total) {
  // 32-bit index split by invariant-divisor multiplies: a 64-bit `/` and `%` per element
  // cost more than the interpolation itself (the x8 logits upsample ran 14x off roofline).
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t c, ox, oy;
    const uint32_t r0 = fc.divmod(i, c);
    const uint32_t r1 = fw.divmod(r0, ox);
    const int n = static_cast<int>(fh.divmod(r1, oy));
    int y0, y1, x0, x1; float ly, lx;
    mh.map(static_cast<int>(oy), y0, y1, ly);
    mw.map(static_cast<int>(ox), x0, x1, lx);
    const T* b = x + n * xs.sn + static_cast<int64_t>(c) * xs.sc;
    float v00 = Io<T>::ld(b + y0 * xs.sh + x0 * xs.sw);
    float v01 = Io<T>::ld(b + y0 * xs.sh + x1 * xs.sw);
    float v10 = Io<T>::ld(b + y1 * xs.sh + x0 * xs.sw);
    float v11 = Io<T>::ld(b + y1 * xs.sh + x1 * xs.sw);
    float v = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
    if constexpr (SKIP) v += Io<T>::ld(skip + off4(ks, n, static_cast<int>(c), static_cast<int>(oy), static_cast<int>(ox)));
    Io<T>::st(y + off4(ys, n, static_cast<int>(c), static_cast<int>(oy), static_cast<int>(ox)), act_fwd<ACT>(v));
  }
}

// Same, one thread per output PIXEL looping over the (few, e.g. 19) channels: the two
// source-coordinate maps are computed once per pixel instead of once per element (the
// per-element form is instruction-bound: ~80 VALU ops for 4 loads and 1 store).
template <typename T, int ACT, bool SKIP>
__global__ void __launch_bounds__(256) interp_fwd_cl_pix(
    const T* __restrict__ x, Shape4 xs, const T* __restrict__ skip, Shape4 ks,
    T* __restrict__ y, Shape4 ys, LinMap mh, LinMap mw, FastDiv fw, FastDiv fh, uint32_t npix) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < npix; i += gridDim.x * 256u) {
    uint32_t ox, oy;
    const uint32_t r1 = fw.divmod(i, ox);
    const int n = static_cast<int>(fh.divmod(r1, oy));
    int y0, y1, x0, x1; float ly, lx;
    mh.map(static_cast<int>(oy), y0, y1, ly);
    mw.map(static_cast<int>(ox), x0, x1, lx);
    const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx), w11 = ly * lx;
    const T* b = x + n * xs.sn;
    const T* p00 = b + y0 * xs.sh + x0 * xs.sw;
    const T* p01 = b + y0 * xs.sh + x1 * xs.sw;
    const T* p10 = b + y1 * xs.sh + x0 * xs.sw;
    const T* p11 = b + y1 * xs.sh + x1 * xs.sw;
    T* q = y + off4(ys, n, 0, static_cast<int>(oy), static_cast<int>(ox));
    const T* k = SKIP ? skip + off4(ks, n, 0, static_cast<int>(oy), static_cast<int>(ox)) : nullptr;
    for (int c = 0; c < ys.c; ++c) {
      float v = w00 * Io<T>::ld(p00 + c) + w01 * Io<T>::ld(p01 + c) + w10 * Io<T>::ld(p10 + c) +
                w11 * Io<T>::ld(p11 + c);
      if constexpr (SKIP) v += Io<T>::ld(k + c * ks.sc);
      Io<T>::st(q + c, act_fwd<ACT>(v));
    }
  }
}

// Same, for a dense channels-last output whose pixel is not a whole number of 16-byte
// vectors (e.g. 19-class logits: 38 bytes): a block computes 256 consecutive output pixels
// into LDS and writes them back as one contiguous run of 16-byte stores -- the per-pixel
// scalar stores above touch ~19 partial lines per wave instruction (TA-bound, ~5x off HBM).
template <typename T, int ACT, bool SKIP>
__global__ void __launch_bounds__(256) interp_fwd_cl_pix_lds(
    const T* __restrict__ x, Shape4 xs, const T* __restrict__ skip, Shape4 ks,
    T* __restrict__ y, Shape4 ys, LinMap mh, LinMap mw, FastDiv fw, FastDiv fh, uint32_t npix) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ip_lds[];
  T* st = reinterpret_cast<T*>(ip_lds);
  const int C = ys.c;
  for (uint32_t p0 = blockIdx.x * 256u; p0 < npix; p0 += gridDim.x * 256u) {
    const uint32_t i = p0 + threadIdx.x;
    if (i < npix) {
      uint32_t ox, oy;
      const uint32_t r1 = fw.divmod(i, ox);
      const int n = static_cast<int>(fh.divmod(r1, oy));
      int y0, y1, x0, x1; float ly, lx;
      mh.map(static_cast<int>(oy), y0, y1, ly);
      mw.map(static_cast<int>(ox), x0, x1, lx);
      const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx), w11 = ly * lx;
      const T* b = x + n * xs.sn;
      const T* p00 = b + y0 * xs.sh + x0 * xs.sw;
      const T* p01 = b + y0 * xs.sh + x1 * xs.sw;
      const T* p10 = b + y1 * xs.sh + x0 * xs.sw;
      const T* p11 = b + y1 * xs.sh + x1 * xs.sw;
      const T* k = SKIP ? skip + off4(ks, n, 0, static_cast<int>(oy), static_cast<int>(ox)) : nullptr;
      T* q = st + threadIdx.x * C;
      for (int c = 0; c < C; ++c) {
        float v = w00 * Io<T>::ld(p00 + c) + w01 * Io<T>::ld(p01 + c) + w10 * Io<T>::ld(p10 + c) +
                  w11 * Io<T>::ld(p11 + c);
        if constexpr (SKIP) v += Io<T>::ld(k + c * ks.sc);
        Io<T>::st(q + c, act_fwd<ACT>(v));
      }
    }
    __syncthreads();
    const uint32_t np = npix - p0 < 256u ? npix - p0 : 256u;
    const int64_t nelem = static_cast<int64_t>(np) * C;
    const int64_t nvec = nelem * static_cast<int64_t>(sizeof(T)) / 16;
    uint4* dst = reinterpret_cast<uint4*>(y + static_cast<int64_t>(p0) * C);
    const uint4* src = reinterpret_cast<const uint4*>(st);
    for (int64_t v = threadIdx.x; v < nvec; v += 256) dst[v] = src[v];
    for (int64_t e = nvec * 16 / static_cast<int64_t>(sizeof(T)) + threadIdx.x; e < nelem; e += 256)
      y[static_cast<int64_t>(p0) * C + e] = st[e];
    __syncthreads();
  }
}

// Large up-scaling of a few-channel map into a dense channels-last output (the models' final
// x8 logits upsample in inference: 19 channels, 38-byte pixels): one block per output ROW.  The
// row's two source rows are staged in LDS as fp32 and blended vertically once; the column map
// (x0, lambda) of every output column is tabulated once; then every thread writes 16-byte runs of
// the flat output row (8 consecutive elements, crossing pixel boundaries), each element two LDS
// reads and one lerp.  The per-pixel kernel above spends ~76 scalar loads per 19-channel pixel.
template <typename T, int ACT>
__global__ void __launch_bounds__(256) interp_fwd_cl_rows(const T* __restrict__ x, Shape4 xs, T* __restrict__ y,
                                                          Shape4 ys, LinMap mh, LinMap mw) {
  extern __shared__ __attribute__((aligned(16))) float rl[];
  const int C = ys.c, Wi = xs.w, Wo = ys.w;
  float* row = rl;                                          // [Wi][C] blended source row
  float* lam = rl + Wi * C;                                 // [Wo] horizontal weights
  int* col = reinterpret_cast<int*>(lam + Wo);              // [Wo] left source column
  const int oy = blockIdx.x % ys.h, n = blockIdx.x / ys.h;
  int y0, y1; float ly;
  mh.map(oy, y0, y1, ly);
  const T* r0 = x + n * xs.sn + y0 * xs.sh;
  const T* r1 = x + n * xs.sn + y1 * xs.sh;
  for (int e = threadIdx.x; e < Wi * C; e += 256) {
    const int ix = e / C, c = e - ix * C;
    const float a = Io<T>::ld(r0 + ix * xs.sw + c), b = Io<T>::ld(r1 + ix * xs.sw + c);
    row[e] = a + ly * (b - a);
  }
  for (int ox = threadIdx.x; ox < Wo; ox += 256) {
    int x0, x1; float lx;
    mw.map(ox, x0, x1, lx);
    col[ox] = x0;
    lam[ox] = x1 == x0 ? 0.f : lx;  // clamped last column: no right tap
  }
  __syncthreads();
  constexpr int E = 16 / static_cast<int>(sizeof(T));
  const int nvec = Wo * C / E;
  T* out = y + n * ys.sn + oy * ys.sh;
  for (int v = threadIdx.x; v < nvec; v += 256) {
    int e = v * E;
    int ox = e / C, c = e - ox * C;
    alignas(16) T o[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float* p = row + col[ox] * C + c;
      const float l = lam[ox];
      const float a = p[0];
      const float val = l == 0.f ? a : a + l * (p[C] - a);
      Io<T>::st(o + j, act_fwd<ACT>(val));
      if (++c == C) { c = 0; ++ox; }
    }
    *reinterpret_cast<uint4*>(out + static_cast<int64_t>(v) * E) = *reinterpret_cast<const uint4*>(o);
  }
}

typedef short short8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void unpack8(const short8& v, float* f) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf16_to_f32(static_cast<uint16_t>(v[j]));
}

// Channels-last bf16, C % 8 == 0: one thread = 8 channels of one output pixel.
template <int ACT, bool SKIP>
__global__ void __launch_bounds__(256) interp_fwd_cl_bf16(
    const uint16_t* __restrict__ x, Shape4 xs, const uint16_t* __restrict__ skip, Shape4 ks,
    uint16_t* __restrict__ y, Shape4 ys, LinMap mh, LinMap mw) {
  const int cv = ys.c >> 3;
  const int64_t total = static_cast<int64_t>(ys.n) * ys.h * ys.w * cv;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int c8 = static_cast<int>(i % cv);
    int64_t t = i / cv;
    int ox = static_cast<int>(t % ys.w);
    t /= ys.w;
    int oy = static_cast<int>(t % ys.h);
    int n = static_cast<int>(t / ys.h);
    int y0, y1, x0, x1; float ly, lx;
    mh.map(oy, y0, y1, ly);
    mw.map(ox, x0, x1, lx);
    const uint16_t* b = x + n * xs.sn + (c8 << 3);
    short8 a00 = *reinterpret_cast<const short8*>(b + y0 * xs.sh + x0 * xs.sw);
    short8 a01 = *reinterpret_cast<const short8*>(b + y0 * xs.sh + x1 * xs.sw);
    short8 a10 = *reinterpret_cast<const short8*>(b + y1 * xs.sh + x0 * xs.sw);
    short8 a11 = *reinterpret_cast<const short8*>(b + y1 * xs.sh + x1 * xs.sw);
    float f00[8], f01[8], f10[8], f11[8], fk[8];
    unpack8(a00, f00); unpack8(a01, f01); unpack8(a10, f10); unpack8(a11, f11);
    if constexpr (SKIP) {
      short8 k = *reinterpret_cast<const short8*>(skip + n * ks.sn + oy * ks.sh + ox * ks.sw + (c8 << 3));
      unpack8(k, fk);
    }
    const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx;
    const float w10 = ly * (1.f - lx), w11 = ly * lx;
    short8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = w00 * f00[j] + w01 * f01[j] + w10 * f10[j] + w11 * f11[j];
      if constexpr (SKIP) v += fk[j];
      o[j] = static_cast<short>(f32_to_bf16(act_fwd<ACT>(v)));
    }
    *reinterpret_cast<short8*>(y + n * ys.sn + oy * ys.sh + ox * ys.sw + (c8 << 3)) = o;
  }
}

// ------------------------------- backward ----------------------------------
// grad_x[n,c,iy,ix] = sum_{oy,ox} wy(oy,iy) * wx(ox,ix) * g[n,c,oy,ox]
template <typename T>
__global__ void __launch_bounds__(256) interp_bwd_scalar(
    const T* __restrict__ g, Shape4 gs, T* __restrict__ gx, Shape4 xs, LinMap mh, LinMap mw) {
  const int64_t total = static_cast<int64_t>(xs.n) * xs.c * xs.h * xs.w;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int ix = static_cast<int>(i % xs.w);
    int64_t t = i / xs.w;
    int iy = static_cast<int>(t % xs.h);
    t /= xs.h;
    int c = static_cast<int>(t % xs.c);
    int n = static_cast<int>(t / xs.c);
    int ylo, yhi, xlo, xhi;
    mh.out_range(iy, gs.h, ylo, yhi);
    mw.out_range(ix, gs.w, xlo, xhi);
    const T* gb = g + n * gs.sn + c * gs.sc;
    float acc = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      float wy = mh.weight(oy, iy);
      if (wy == 0.f) continue;
      float row = 0.f;
      for (int ox = xlo; ox <= xhi; ++ox) {
        float wx = mw.weight(ox, ix);
        if (wx != 0.f) row += wx * Io<T>::ld(gb + oy * gs.sh + ox * gs.sw);
      }
      acc += wy * row;
    }
    Io<T>::st(gx + off4(xs, n, c, iy, ix), acc);
  }
}

__global__ void __launch_bounds__(256) interp_bwd_cl_bf16(
    const uint16_t* __restrict__ g, Shape4 gs, uint16_t* __restrict__ gx, Shape4 xs, LinMap mh,
    LinMap mw) {
  const int cv = xs.c >> 3;
  const int64_t total = static_cast<int64_t>(xs.n) * xs.h * xs.w * cv;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int c8 = static_cast<int>(i % cv);
    int64_t t = i / cv;
    int ix = static_cast<int>(t % xs.w);
    t /= xs.w;
    int iy = static_cast<int>(t % xs.h);
    int n = static_cast<int>(t / xs.h);
    int ylo, yhi, xlo, xhi;
    mh.out_range(iy, gs.h, ylo, yhi);
    mw.out_range(ix, gs.w, xlo, xhi);
    const uint16_t* gb = g + n * gs.sn + (c8 << 3);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      float wy = mh.weight(oy, iy);
      if (wy == 0.f) continue;
      for (int ox = xlo; ox <= xhi; ++ox) {
        float w = wy * mw.weight(ox, ix);
        if (w == 0.f) continue;
        float f[8];
        unpack8(*reinterpret_cast<const short8*>(gb + oy * gs.sh + ox * gs.sw), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += w * f[j];
      }
    }
    short8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = static_cast<short>(f32_to_bf16(acc[j]));
    *reinterpret_cast<short8*>(gx + n * xs.sn + iy * xs.sh + ix * xs.sw + (c8 << 3)) = o;
  }
}

// Separable backward for large up-scaling (e.g. the x8 logits upsample a KD loss or a
// non-deferred loss materialises): gx = Rh^T . g . Rw as two gathers through an fp32
// [N, OH, IW, C] workspace -- W-pass then H-pass, ~(2s+1) taps each -- instead of one
// gather over a (2s+1)^2 window per input element.  Index order is channel-fastest so
// channels-last gradients are read coalesced; loads are never behind a weight test.
template <typename T>
__global__ void __launch_bounds__(256) interp_bwd_sep_w(const T* __restrict__ g, Shape4 gs, float* __restrict__ t,
                                                        int iw, LinMap mw, FastDiv fc, FastDiv fiw, FastDiv foh,
                                                        uint32_t total) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t c, ix, oy;
    const uint32_t r0 = fc.divmod(i, c);
    const uint32_t r1 = fiw.divmod(r0, ix);
    const uint32_t n = foh.divmod(r1, oy);
    int lo, hi;
    mw.out_range(static_cast<int>(ix), gs.w, lo, hi);
    const T* gb = g + static_cast<int64_t>(n) * gs.sn + static_cast<int64_t>(c) * gs.sc +
                  static_cast<int64_t>(oy) * gs.sh;
    float acc = 0.f;
    for (int ox = lo; ox <= hi; ++ox) acc = fmaf(mw.weight(ox, static_cast<int>(ix)), Io<T>::ld(gb + ox * gs.sw), acc);
    t[i] = acc;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) interp_bwd_sep_h(const float* __restrict__ t, int oh, T* __restrict__ gx,
                                                        Shape4 xs, LinMap mh, FastDiv fc, FastDiv fiw, FastDiv fih,
                                                        uint32_t total) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t c, ix, iy;
    const uint32_t r0 = fc.divmod(i, c);
    const uint32_t r1 = fiw.divmod(r0, ix);
    const uint32_t n = fih.divmod(r1, iy);
    int lo, hi;
    mh.out_range(static_cast<int>(iy), oh, lo, hi);
    const int64_t row = static_cast<int64_t>(xs.w) * xs.c;  // t row stride (IW * C)
    const float* tb = t + static_cast<int64_t>(n) * oh * row + static_cast<int64_t>(ix) * xs.c + c;
    float acc = 0.f;
    for (int oy = lo; oy <= hi; ++oy) acc = fmaf(mh.weight(oy, static_cast<int>(iy)), tb[oy * row], acc);
    Io<T>::st(gx + off4(xs, static_cast<int>(n), static_cast<int>(c), static_cast<int>(iy), static_cast<int>(ix)), acc);
  }
}

// g_masked = act'(y) * g (also the gradient of the fused skip input).
template <typename T, int ACT>
__global__ void __launch_bounds__(256) act_mask_kernel(const T* __restrict__ g,
                                                       const T* __restrict__ y,
                                                       T* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    Io<T>::st(out + i, act_bwd_from_out<ACT>(Io<T>::ld(g + i), Io<T>::ld(y + i)));
  }
}

// ------------------------------- launchers ---------------------------------
static Shape4 mk(const Tensor4& t) {
  Shape4 s;
  s.n = t.n; s.c = t.c; s.h = t.h; s.w = t.w;
  s.sn = t.sn; s.sc = t.sc; s.sh = t.sh; s.sw = t.sw;
  return s;
}

static bool cl_vec_ok(const Tensor4& t) {
  return t.sc == 1 && (t.c % 8) == 0 && (t.sw % 8) == 0 && (t.sh % 8) == 0 && (t.sn % 8) == 0 &&
         (reinterpret_cast<uintptr_t>(t.data) % 16) == 0;
}

template <typename T, int ACT, bool SKIP>
static void fwd_dispatch(const Tensor4& x, const Tensor4* skip, const Tensor4& y, LinMap mh,
                         LinMap mw, hipStream_t st) {
  Shape4 xs = mk(x), ys = mk(y), ks = skip ? mk(*skip) : ys;
  const T* kp = skip ? static_cast<const T*>(skip->data) : nullptr;
  if constexpr (sizeof(T) == 2 && !std::is_same<T, _Float16>::value) {
    if (cl_vec_ok(x) && cl_vec_ok(y) && (!skip || cl_vec_ok(*skip))) {
      int64_t work = static_cast<int64_t>(y.n) * y.h * y.w * (y.c / 8);
      interp_fwd_cl_bf16<ACT, SKIP><<<stream_grid(work, 256), 256, 0, st>>>(
          static_cast<const uint16_t*>(x.data), xs, kp, ks, static_cast<uint16_t*>(y.data), ys, mh, mw);
      return;
    }
  }
  int64_t work = static_cast<int64_t>(y.n) * y.c * y.h * y.w;
  const int64_t npix = static_cast<int64_t>(y.n) * y.h * y.w;
  const bool dense_cl = y.sc == 1 && y.sw == y.c && y.sh == static_cast<int64_t>(y.w) * y.c &&
                        y.sn == static_cast<int64_t>(y.h) * y.w * y.c &&
                        reinterpret_cast<uintptr_t>(y.data) % 16 == 0;
  const size_t lds = static_cast<size_t>(256) * y.c * sizeof(T);
  // the row kernel: no skip, >= x4 horizontally, a 16-byte multiple per output row, LDS for two
  // fp32 source rows and the column table (RTSEG_INTERP_ROWS=0: off)
  static const bool rows_on = [] { const char* e = std::getenv("RTSEG_INTERP_ROWS"); return !(e && e[0] == '0'); }();
  const size_t rlds = (static_cast<size_t>(x.w) * y.c + 2 * static_cast<size_t>(y.w)) * 4;
  if (rows_on && !SKIP && dense_cl && x.sc == 1 && y.c > 1 && y.c < 64 && y.w >= 4 * x.w && rlds <= 65536 &&
      (static_cast<int64_t>(y.w) * y.c * static_cast<int64_t>(sizeof(T))) % 16 == 0 &&
      static_cast<int64_t>(y.n) * y.h < (int64_t{1} << 31)) {
    interp_fwd_cl_rows<T, ACT><<<static_cast<int>(y.n * y.h), 256, rlds, st>>>(
        static_cast<const T*>(x.data), xs, static_cast<T*>(y.data), ys, mh, mw);
    return;
  }
  if (dense_cl && x.sc == 1 && y.c > 1 && lds <= 32768 && npix < (int64_t{1} << 31)) {
    interp_fwd_cl_pix_lds<T, ACT, SKIP><<<stream_grid(npix, 256), 256, lds, st>>>(
        static_cast<const T*>(x.data), xs, kp, ks, static_cast<T*>(y.data), ys, mh, mw, FastDiv::make(y.w),
        FastDiv::make(y.h), static_cast<uint32_t>(npix));
    return;
  }
  if (y.sc == 1 && x.sc == 1 && y.c > 1 && y.c <= 64 && npix < (int64_t{1} << 31)) {
    interp_fwd_cl_pix<T, ACT, SKIP><<<stream_grid(npix, 256), 256, 0, st>>>(
        static_cast<const T*>(x.data), xs, kp, ks, static_cast<T*>(y.data), ys, mh, mw, FastDiv::make(y.w),
        FastDiv::make(y.h), static_cast<uint32_t>(npix));
    return;
  }
  if (y.sc == 1 && y.c > 1 && work < (int64_t{1} << 31)) {
    interp_fwd_cl_scalar<T, ACT, SKIP><<<stream_grid(work, 256), 256, 0, st>>>(
        static_cast<const T*>(x.data), xs, kp, ks, static_cast<T*>(y.data), ys, mh, mw, FastDiv::make(y.c),
        FastDiv::make(y.w), FastDiv::make(y.h), static_cast<uint32_t>(work));
    return;
  }
  interp_fwd_scalar<T, ACT, SKIP><<<stream_grid(work, 256), 256, 0, st>>>(
      static_cast<const T*>(x.data), xs, kp, ks, static_cast<T*>(y.data), ys, mh, mw);
}

template <typename T>
static void fwd_act(const Tensor4& x, const Tensor4* skip, const Tensor4& y, int act, LinMap mh,
                    LinMap mw, hipStream_t st) {
  if (skip) {
    if (act == kActReLU) fwd_dispatch<T, kActReLU, true>(x, skip, y, mh, mw, st);
    else if (act == kActReLU6) fwd_dispatch<T, kActReLU6, true>(x, skip, y, mh, mw, st);
    else fwd_dispatch<T, kActNone, true>(x, skip, y, mh, mw, st);
  } else {
    if (act == kActReLU) fwd_dispatch<T, kActReLU, false>(x, skip, y, mh, mw, st);
    else if (act == kActReLU6) fwd_dispatch<T, kActReLU6, false>(x, skip, y, mh, mw, st);
    else fwd_dispatch<T, kActNone, false>(x, skip, y, mh, mw, st);
  }
}

void launch_interp_fwd(const Tensor4& x, const Tensor4* skip, const Tensor4& y, int act,
                       bool align_corners, hipStream_t st) {
  LinMap mh = LinMap::make(x.h, y.h, align_corners);
  LinMap mw = LinMap::make(x.w, y.w, align_corners);
  switch (x.dtype) {
    case kF32: fwd_act<float>(x, skip, y, act, mh, mw, st); break;
    case kBF16: fwd_act<uint16_t>(x, skip, y, act, mh, mw, st); break;
    default: fwd_act<_Float16>(x, skip, y, act, mh, mw, st); break;
  }
}

int64_t interp_bwd_ws_elems(const Tensor4& g, const Tensor4& gx) {
  // the vectorised channels-last bf16 gather stays faster up to x8 (DDRNet's x2..x8 fusions);
  // the separable path takes the scalar cases (odd C, e.g. 19-class logits) and larger scales
  const bool vec = g.dtype == kBF16 && cl_vec_ok(g) && cl_vec_ok(gx);
  const bool big = vec ? (g.h > 8 * gx.h || g.w > 8 * gx.w) : (g.h > 2 * gx.h || g.w > 2 * gx.w);
  const int64_t ws = static_cast<int64_t>(g.n) * g.h * gx.w * gx.c;
  const int64_t out = static_cast<int64_t>(gx.n) * gx.h * gx.w * gx.c;
  return (big && ws < (int64_t{1} << 31) && out < (int64_t{1} << 31)) ? ws : 0;
}

template <typename T>
static void bwd_t(const Tensor4& g, const Tensor4& gx, LinMap mh, LinMap mw, float* ws, hipStream_t st) {
  Shape4 gs = mk(g), xs = mk(gx);
  if (ws != nullptr) {
    const uint32_t tw = static_cast<uint32_t>(static_cast<int64_t>(g.n) * g.h * gx.w * gx.c);
    interp_bwd_sep_w<T><<<stream_grid(tw, 256), 256, 0, st>>>(static_cast<const T*>(g.data), gs, ws, gx.w, mw,
                                                              FastDiv::make(gx.c), FastDiv::make(gx.w),
                                                              FastDiv::make(g.h), tw);
    const uint32_t th = static_cast<uint32_t>(static_cast<int64_t>(gx.n) * gx.h * gx.w * gx.c);
    interp_bwd_sep_h<T><<<stream_grid(th, 256), 256, 0, st>>>(ws, g.h, static_cast<T*>(gx.data), xs, mh,
                                                              FastDiv::make(gx.c), FastDiv::make(gx.w),
                                                              FastDiv::make(gx.h), th);
    return;
  }
  if constexpr (std::is_same<T, uint16_t>::value) {
    if (cl_vec_ok(g) && cl_vec_ok(gx)) {
      int64_t work = static_cast<int64_t>(gx.n) * gx.h * gx.w * (gx.c / 8);
      interp_bwd_cl_bf16<<<stream_grid(work, 256), 256, 0, st>>>(
          static_cast<const uint16_t*>(g.data), gs, static_cast<uint16_t*>(gx.data), xs, mh, mw);
      return;
    }
  }
  int64_t work = static_cast<int64_t>(gx.n) * gx.c * gx.h * gx.w;
  interp_bwd_scalar<T><<<stream_grid(work, 256), 256, 0, st>>>(
      static_cast<const T*>(g.data), gs, static_cast<T*>(gx.data), xs, mh, mw);
}

void launch_interp_bwd(const Tensor4& g, const Tensor4& gx, bool align_corners, float* ws, hipStream_t st) {
  LinMap mh = LinMap::make(gx.h, g.h, align_corners);
  LinMap mw = LinMap::make(gx.w, g.w, align_corners);
  switch (g.dtype) {
    case kF32: bwd_t<float>(g, gx, mh, mw, ws, st); break;
    case kBF16: bwd_t<uint16_t>(g, gx, mh, mw, ws, st); break;
    default: bwd_t<_Float16>(g, gx, mh, mw, ws, st); break;
  }
}

void launch_act_mask(const void* g, const void* y, void* out, int64_t n, int dtype, int act,
                     hipStream_t st) {
  int grid = stream_grid(n, 256);
#define RT_MASK(T)                                                                              \
  if (act == kActReLU6)                                                                         \
    act_mask_kernel<T, kActReLU6><<<grid, 256, 0, st>>>(static_cast<const T*>(g),               \
                                                        static_cast<const T*>(y), static_cast<T*>(out), n); \
  else                                                                                          \
    act_mask_kernel<T, kActReLU><<<grid, 256, 0, st>>>(static_cast<const T*>(g),                \
                                                       static_cast<const T*>(y), static_cast<T*>(out), n);
  if (dtype == kF32) { RT_MASK(float) }
  else if (dtype == kBF16) { RT_MASK(uint16_t) }
  else { RT_MASK(_Float16) }
#undef RT_MASK
}

}  // namespace rtseg
