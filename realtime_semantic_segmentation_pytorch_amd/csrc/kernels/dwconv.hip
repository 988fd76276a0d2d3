// Depth-wise 2-D convolution (groups == C_in, channel multiplier M = C_out / C_in)
// for channels-last activations on CDNA4 (gfx950).
//
// Reference sites: models/modules.py:46-59 (DWConvBNAct, incl. the BiSeNetV2
// x6 multiplier, bisenetv2.py:140-148), raw depth-wise convs in cgnet.py:79-82,
// mininet.py:79-91, and the asymmetric / dilated variants (3,1)/(1,3)/(5,1),
// dilation 2..17 used across the zoo.
//
// Layout: x [N, H, W, Cin], y/dy [N, Ho, Wo, Cout] (NHWC physical), weights are
// passed TAP-MAJOR in fp32: wt[KH*KW][Cout] (the binding transposes the tiny
// [Cout,1,KH,KW] tensor), so one vector load fetches the VEC channels a thread
// owns.  Work item = (pixel, vector of VEC contiguous channels); consecutive
// threads own consecutive channel vectors of the same pixel, so every global
// access of a wave is contiguous 16-byte chunks.  The KH*KW re-reads of an input
// pixel by neighbouring outputs hit L1/L2; HBM sees each tensor once.
//
//  fwd  : y[p, co]   = sum_t x[p*s - pad + t*d, co / M] * w[t][co] (+ b[co])
//  dgrad: dx[q, ci]  = sum_m sum_t dy[(q + pad - t*d) / s, ci*M + m] * w[t][ci*M+m]
//         (gather form -- no atomics; taps whose source is not on the stride grid skip)
//  wgrad: dw[t][co]  = sum_p dy[p, co] * x[p*s - pad + t*d, co / M]
//         per-block partials [G][taps][Cout] fp32 + a deterministic column reduce.
#include "rtseg_common.h"
#include "rtseg_launch.h"

#include <type_traits>

namespace rtseg {

namespace {

constexpr int kDwBlock = 256;
constexpr int kMaxTaps = 9;  // taps accumulated per wgrad thread (tap groups cover larger kernels)

template <typename T, int VEC> struct Vec;
template <typename T> struct Vec<T, 1> {
  __device__ __forceinline__ static void load(const T* p, float* v) { v[0] = Io<T>::ld(p); }
  __device__ __forceinline__ static void store(T* p, const float* v) { Io<T>::st(p, v[0]); }
};
template <> struct Vec<uint16_t, 8> {
  __device__ __forceinline__ static void load(const uint16_t* p, float* v) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float* v) {
    uint4 r;
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = static_cast<unsigned>(f32_to_bf16(v[2 * i])) | (static_cast<unsigned>(f32_to_bf16(v[2 * i + 1])) << 16);
    r.x = w[0]; r.y = w[1]; r.z = w[2]; r.w = w[3];
    *reinterpret_cast<uint4*>(p) = r;
  }
};
template <> struct Vec<uint16_t, 4> {
  __device__ __forceinline__ static void load(const uint16_t* p, float* v) {
    const uint2 r = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(r.x << 16); v[1] = __uint_as_float(r.x & 0xffff0000u);
    v[2] = __uint_as_float(r.y << 16); v[3] = __uint_as_float(r.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float* v) {
    uint2 r;
    r.x = static_cast<unsigned>(f32_to_bf16(v[0])) | (static_cast<unsigned>(f32_to_bf16(v[1])) << 16);
    r.y = static_cast<unsigned>(f32_to_bf16(v[2])) | (static_cast<unsigned>(f32_to_bf16(v[3])) << 16);
    *reinterpret_cast<uint2*>(p) = r;
  }
};
template <> struct Vec<uint16_t, 2> {
  __device__ __forceinline__ static void load(const uint16_t* p, float* v) {
    const unsigned r = *reinterpret_cast<const unsigned*>(p);
    v[0] = __uint_as_float(r << 16); v[1] = __uint_as_float(r & 0xffff0000u);
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float* v) {
    *reinterpret_cast<unsigned*>(p) =
        static_cast<unsigned>(f32_to_bf16(v[0])) | (static_cast<unsigned>(f32_to_bf16(v[1])) << 16);
  }
};
template <int VEC> struct VecF {  // fp32 and fp16 via element loops the compiler merges
  template <typename T> __device__ __forceinline__ static void load(const T* p, float* v) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[i] = Io<T>::ld(p + i);
  }
  template <typename T> __device__ __forceinline__ static void store(T* p, const float* v) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) Io<T>::st(p + i, v[i]);
  }
};
template <int VEC> struct Vec<float, VEC> {
  __device__ __forceinline__ static void load(const float* p, float* v) { VecF<VEC>::load(p, v); }
  __device__ __forceinline__ static void store(float* p, const float* v) { VecF<VEC>::store(p, v); }
};
template <int VEC> struct Vec<_Float16, VEC> {
  __device__ __forceinline__ static void load(const _Float16* p, float* v) { VecF<VEC>::load(p, v); }
  __device__ __forceinline__ static void store(_Float16* p, const float* v) { VecF<VEC>::store(p, v); }
};
template <> struct Vec<float, 1> {
  __device__ __forceinline__ static void load(const float* p, float* v) { v[0] = *p; }
  __device__ __forceinline__ static void store(float* p, const float* v) { *p = v[0]; }
};
template <> struct Vec<_Float16, 1> {
  __device__ __forceinline__ static void load(const _Float16* p, float* v) { v[0] = static_cast<float>(*p); }
  __device__ __forceinline__ static void store(_Float16* p, const float* v) { *p = static_cast<_Float16>(v[0]); }
};

// ---------------------------------------------------------------- forward
template <typename T, int VEC, bool MULT>
__global__ void __launch_bounds__(kDwBlock) dw_fwd_kernel(DwGeom g, const T* __restrict__ x,
                                                          const float* __restrict__ wt,
                                                          const float* __restrict__ bias, T* __restrict__ y) {
  const int cv_n = g.cout / VEC;
  const int64_t total = static_cast<int64_t>(g.n) * g.ho * g.wo * cv_n;
  for (int64_t it = blockIdx.x * static_cast<int64_t>(kDwBlock) + threadIdx.x; it < total;
       it += static_cast<int64_t>(gridDim.x) * kDwBlock) {
    const int cv = static_cast<int>(it % cv_n);
    int64_t pix = it / cv_n;
    const int wo = static_cast<int>(pix % g.wo);
    pix /= g.wo;
    const int ho = static_cast<int>(pix % g.ho);
    const int n = static_cast<int>(pix / g.ho);
    const int co = cv * VEC;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = bias ? bias[co + v] : 0.f;
    const int hb = ho * g.sh - g.ph, wb = wo * g.sw - g.pw;
    for (int i = 0; i < g.kh; ++i) {
      const int hi = hb + i * g.dh;
      if (hi < 0 || hi >= g.h) continue;
      const T* xrow = x + (static_cast<int64_t>(n) * g.h + hi) * g.w * g.cin;
      for (int j = 0; j < g.kw; ++j) {
        const int wi = wb + j * g.dw;
        if (wi < 0 || wi >= g.w) continue;
        float xv[VEC], wv[VEC];
        const float* wp = wt + (i * g.kw + j) * g.cout + co;
#pragma unroll
        for (int v = 0; v < VEC; ++v) wv[v] = wp[v];
        if constexpr (!MULT) {
          Vec<T, VEC>::load(xrow + static_cast<int64_t>(wi) * g.cin + co, xv);
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) xv[v] = Io<T>::ld(xrow + static_cast<int64_t>(wi) * g.cin + (co + v) / g.mult);
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = fmaf(xv[v], wv[v], acc[v]);
      }
    }
    Vec<T, VEC>::store(y + ((static_cast<int64_t>(n) * g.ho + ho) * g.wo + wo) * g.cout + co, acc);
  }
}

// ---------------------------------------------------------------- data grad
template <typename T, int VEC, bool MULT>
__global__ void __launch_bounds__(kDwBlock) dw_dgrad_kernel(DwGeom g, const T* __restrict__ dy,
                                                            const float* __restrict__ wt, T* __restrict__ dx) {
  const int cv_n = g.cin / VEC;
  const int64_t total = static_cast<int64_t>(g.n) * g.h * g.w * cv_n;
  for (int64_t it = blockIdx.x * static_cast<int64_t>(kDwBlock) + threadIdx.x; it < total;
       it += static_cast<int64_t>(gridDim.x) * kDwBlock) {
    const int cv = static_cast<int>(it % cv_n);
    int64_t pix = it / cv_n;
    const int wi = static_cast<int>(pix % g.w);
    pix /= g.w;
    const int hi = static_cast<int>(pix % g.h);
    const int n = static_cast<int>(pix / g.h);
    const int ci = cv * VEC;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    for (int i = 0; i < g.kh; ++i) {
      const int hn = hi + g.ph - i * g.dh;
      if (hn < 0) continue;
      const int ho = hn / g.sh;
      if (ho * g.sh != hn || ho >= g.ho) continue;
      const T* dyrow = dy + (static_cast<int64_t>(n) * g.ho + ho) * g.wo * g.cout;
      for (int j = 0; j < g.kw; ++j) {
        const int wn = wi + g.pw - j * g.dw;
        if (wn < 0) continue;
        const int wo = wn / g.sw;
        if (wo * g.sw != wn || wo >= g.wo) continue;
        const T* dp = dyrow + static_cast<int64_t>(wo) * g.cout;
        const float* wp = wt + (i * g.kw + j) * g.cout;
        if constexpr (!MULT) {
          float dv[VEC];
          Vec<T, VEC>::load(dp + ci, dv);
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[v] = fmaf(dv[v], wp[ci + v], acc[v]);
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) {
            const int c0 = (ci + v) * g.mult;
            for (int m = 0; m < g.mult; ++m) acc[v] = fmaf(Io<T>::ld(dp + c0 + m), wp[c0 + m], acc[v]);
          }
        }
      }
    }
    Vec<T, VEC>::store(dx + ((static_cast<int64_t>(n) * g.h + hi) * g.w + wi) * g.cin + ci, acc);
  }
}

// ---------------------------------------------------------------- weight grad
// grid: x = pixel slices (G), y = channel chunks, z = tap groups.  Block = LANES
// channel-vector lanes x ROWS pixel rows; each thread accumulates <= kMaxTaps
// taps x VEC channels over its pixel stride, then the ROWS partials are reduced
// through LDS and one [taps x VEC] partial per (slice, channel vector) is stored.
template <typename T, int VEC, bool MULT>
__global__ void __launch_bounds__(kDwBlock) dw_wgrad_kernel(DwGeom g, const T* __restrict__ dy,
                                                            const T* __restrict__ x, float* __restrict__ part,
                                                            int lanes) {
  const int rows = kDwBlock / lanes;
  const int lane = threadIdx.x % lanes;
  const int row = threadIdx.x / lanes;
  const int cv = blockIdx.y * lanes + lane;
  const int cv_n = g.cout / VEC;
  const int taps = g.kh * g.kw;
  const int t0 = blockIdx.z * kMaxTaps;
  const int nt = min(kMaxTaps, taps - t0);
  const bool active = cv < cv_n;
  const int co = cv * VEC;
  float acc[kMaxTaps][VEC];
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t)
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[t][v] = 0.f;
  const int64_t npix = static_cast<int64_t>(g.n) * g.ho * g.wo;
  if (active) {
    for (int64_t p = static_cast<int64_t>(blockIdx.x) * rows + row; p < npix;
         p += static_cast<int64_t>(gridDim.x) * rows) {
      const int wo = static_cast<int>(p % g.wo);
      const int64_t r = p / g.wo;
      const int ho = static_cast<int>(r % g.ho);
      const int n = static_cast<int>(r / g.ho);
      float dv[VEC];
      Vec<T, VEC>::load(dy + p * g.cout + co, dv);
      const int hb = ho * g.sh - g.ph, wb = wo * g.sw - g.pw;
#pragma unroll
      for (int t = 0; t < kMaxTaps; ++t) {
        if (t < nt) {  // fully unrolled with a block-uniform guard: acc stays in registers
          const int tap = t0 + t;
          const int i = tap / g.kw, j = tap - (tap / g.kw) * g.kw;
          const int hi = hb + i * g.dh, wi = wb + j * g.dw;
          if (hi >= 0 && hi < g.h && wi >= 0 && wi < g.w) {
            const T* xp = x + ((static_cast<int64_t>(n) * g.h + hi) * g.w + wi) * g.cin;
            float xv[VEC];
            if constexpr (!MULT) {
              Vec<T, VEC>::load(xp + co, xv);
            } else {
#pragma unroll
              for (int v = 0; v < VEC; ++v) xv[v] = Io<T>::ld(xp + (co + v) / g.mult);
            }
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[t][v] = fmaf(dv[v], xv[v], acc[t][v]);
          }
        }
      }
    }
  }
  // reduce the `rows` pixel rows of each lane through LDS, one tap at a time
  __shared__ float red[kDwBlock * 8];
  const int64_t slab = static_cast<int64_t>(blockIdx.x) * taps * g.cout;
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t) {
    if (t < nt) {  // nt is block-uniform, so the barriers below are reached by every thread
      __syncthreads();
#pragma unroll
      for (int v = 0; v < VEC; ++v) red[(row * lanes + lane) * VEC + v] = acc[t][v];
      __syncthreads();
      for (int k = threadIdx.x; k < lanes * VEC; k += kDwBlock) {
        float s = 0.f;
        for (int rr = 0; rr < rows; ++rr) s += red[rr * lanes * VEC + k];
        const int c = blockIdx.y * lanes * VEC + k;
        if (c < g.cout) part[slab + static_cast<int64_t>(t0 + t) * g.cout + c] = s;
      }
    }
  }
}

// dw[co][tap] = sum_G part[G][tap][co]   (output in the [Cout, 1, KH, KW] layout)
__global__ void __launch_bounds__(kDwBlock) dw_wgrad_reduce_kernel(const float* __restrict__ part, int G,
                                                                   int taps, int cout, float* __restrict__ dw) {
  const int k = blockIdx.x * kDwBlock + threadIdx.x;  // k = tap * cout + co
  if (k >= taps * cout) return;
  float s = 0.f;
  for (int gi = 0; gi < G; ++gi) s += part[static_cast<int64_t>(gi) * taps * cout + k];
  const int tap = k / cout, co = k - (k / cout) * cout;
  dw[static_cast<int64_t>(co) * taps + tap] = s;
}

template <typename F>
void dw_dispatch(int dtype, int vec, bool mult, F&& f) {
  auto by_vec = [&](auto tag) {
    using T = decltype(tag);
    if (mult) {
      if (vec == 8) f(T{}, std::integral_constant<int, 8>{}, std::true_type{});
      else if (vec == 4) f(T{}, std::integral_constant<int, 4>{}, std::true_type{});
      else if (vec == 2) f(T{}, std::integral_constant<int, 2>{}, std::true_type{});
      else f(T{}, std::integral_constant<int, 1>{}, std::true_type{});
    } else {
      if (vec == 8) f(T{}, std::integral_constant<int, 8>{}, std::false_type{});
      else if (vec == 4) f(T{}, std::integral_constant<int, 4>{}, std::false_type{});
      else if (vec == 2) f(T{}, std::integral_constant<int, 2>{}, std::false_type{});
      else f(T{}, std::integral_constant<int, 1>{}, std::false_type{});
    }
  };
  if (dtype == kF32) by_vec(float{});
  else if (dtype == kBF16) by_vec(uint16_t{});
  else by_vec(_Float16{});
}

}  // namespace

int dw_vec(int dtype, int c) {
  const int maxv = dtype == kF32 ? 4 : 8;  // 16-byte vectors
  for (int v = maxv; v > 1; v >>= 1)
    if (c % v == 0) return v;
  return 1;
}

void launch_dw_fwd(const DwGeom& g, int dtype, const void* x, const float* wt, const float* bias, void* y,
                   hipStream_t st) {
  const int vec = dw_vec(dtype, g.cout);
  const bool mult = g.mult != 1;
  const int64_t items = static_cast<int64_t>(g.n) * g.ho * g.wo * (g.cout / vec);
  const int grid = stream_grid(items, kDwBlock);
  dw_dispatch(dtype, vec, mult, [&](auto t, auto v, auto m) {
    using T = decltype(t);
    dw_fwd_kernel<T, decltype(v)::value, decltype(m)::value><<<grid, kDwBlock, 0, st>>>(
        g, static_cast<const T*>(x), wt, bias, static_cast<T*>(y));
  });
}

void launch_dw_dgrad(const DwGeom& g, int dtype, const void* dy, const float* wt, void* dx, hipStream_t st) {
  const int vec = dw_vec(dtype, g.cin);
  const bool mult = g.mult != 1;
  const int64_t items = static_cast<int64_t>(g.n) * g.h * g.w * (g.cin / vec);
  const int grid = stream_grid(items, kDwBlock);
  dw_dispatch(dtype, vec, mult, [&](auto t, auto v, auto m) {
    using T = decltype(t);
    dw_dgrad_kernel<T, decltype(v)::value, decltype(m)::value><<<grid, kDwBlock, 0, st>>>(
        g, static_cast<const T*>(dy), wt, static_cast<T*>(dx));
  });
}

DwWgradPlan dw_wgrad_plan(const DwGeom& g, int dtype) {
  DwWgradPlan p;
  p.vec = dw_vec(dtype, g.cout);
  const int cv_n = g.cout / p.vec;
  p.lanes = 64;
  while (p.lanes > 1 && p.lanes / 2 >= cv_n) p.lanes /= 2;
  p.chunks = (cv_n + p.lanes - 1) / p.lanes;
  p.tap_groups = (g.kh * g.kw + kMaxTaps - 1) / kMaxTaps;
  const int64_t npix = static_cast<int64_t>(g.n) * g.ho * g.wo;
  const int rows = kDwBlock / p.lanes;
  // ~4 waves of blocks over 256 CUs, but every block keeps >= 16 pixels per row
  int64_t G = 2048 / (static_cast<int64_t>(p.chunks) * p.tap_groups);
  const int64_t gmax = (npix + static_cast<int64_t>(rows) * 16 - 1) / (static_cast<int64_t>(rows) * 16);
  if (G > gmax) G = gmax;
  if (G < 1) G = 1;
  p.slices = static_cast<int>(G);
  return p;
}

void launch_dw_wgrad(const DwGeom& g, int dtype, const void* dy, const void* x, float* part, float* dw,
                     hipStream_t st) {
  const DwWgradPlan p = dw_wgrad_plan(g, dtype);
  const bool mult = g.mult != 1;
  dim3 grid(p.slices, p.chunks, p.tap_groups);
  dw_dispatch(dtype, p.vec, mult, [&](auto t, auto v, auto m) {
    using T = decltype(t);
    dw_wgrad_kernel<T, decltype(v)::value, decltype(m)::value><<<grid, kDwBlock, 0, st>>>(
        g, static_cast<const T*>(dy), static_cast<const T*>(x), part, p.lanes);
  });
  const int taps = g.kh * g.kw;
  const int rb = (taps * g.cout + kDwBlock - 1) / kDwBlock;
  dw_wgrad_reduce_kernel<<<rb, kDwBlock, 0, st>>>(part, p.slices, taps, g.cout, dw);
}

}  // namespace rtseg
