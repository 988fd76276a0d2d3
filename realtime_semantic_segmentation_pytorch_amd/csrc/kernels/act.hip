// Point-wise activation family for CDNA4 (gfx950): forward and backward of PReLU (scalar or
// per-channel weight, with its weight gradient), LeakyReLU, ELU, CELU, SELU, Hardswish,
// Hardtanh, SiLU, Sigmoid, Tanh and GELU (erf / tanh), fp32 / bf16 / fp16, any dense layout.
//
// Reference sites: models/modules.py:111-131 (Activation: the act hub every ConvBNAct /
// DSConvBNAct / DeConvBNAct of the zoo instantiates), PReLU throughout ENet / ESPNet(v2) /
// CGNet / DABNet / CFPNet / FSSNet, ELU in ERFNet's relatives, SELU / Hardswish in the hub.
//
// * elementwise kernels run 16-byte vectors (8 x bf16 / fp16, 4 x fp32) per lane, grid-stride,
//   with a scalar tail; the backward recomputes f'(x) from the saved input (no extra tensor);
// * PReLU backward produces dx AND the weight gradient in the same pass: a [M, C]
//   (channels-last) or [N, C, HW] (contiguous) view; each block owns a row range, every thread
//   a fixed set of channel columns, per-thread partials sit in LDS slots only their owner
//   touches, the block folds them in fixed order into one slab row, and act_prelu_wfinal sums
//   the slab rows in fixed order -> deterministic, no atomics.
#include "rtseg_common.h"
#include "rtseg_launch.h"

#include <algorithm>

namespace rtseg {

namespace {

constexpr int kActBlock = 256;

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + __expf(-v)); }

template <int K>
__device__ __forceinline__ float f_fwd(float x, float a, float b) {
  if constexpr (K == kActLeaky) return x > 0.f ? x : a * x;
  else if constexpr (K == kActELU) return x > 0.f ? x : a * (__expf(x) - 1.f);
  else if constexpr (K == kActCELU) return x > 0.f ? x : a * (__expf(x / a) - 1.f);
  else if constexpr (K == kActSELU) {
    constexpr float al = 1.6732632423543772f, sc = 1.0507009873554805f;
    return x > 0.f ? sc * x : sc * al * (__expf(x) - 1.f);
  } else if constexpr (K == kActHardswish) return x * fminf(fmaxf(x + 3.f, 0.f), 6.f) * (1.f / 6.f);
  else if constexpr (K == kActHardtanh) return fminf(fmaxf(x, a), b);
  else if constexpr (K == kActSiLU) return x * sigm(x);
  else if constexpr (K == kActSigmoid) return sigm(x);
  else if constexpr (K == kActTanh) return tanhf(x);
  else if constexpr (K == kActGELU) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  else if constexpr (K == kActGELUTanh) {
    const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + tanhf(u));
  } else return x > 0.f ? x : a * x;  // PReLU with a scalar slope
}

// d f / d x at x (a, b: the activation's parameters)
template <int K>
__device__ __forceinline__ float f_grad(float x, float a, float b) {
  if constexpr (K == kActLeaky) return x > 0.f ? 1.f : a;
  else if constexpr (K == kActELU) return x > 0.f ? 1.f : a * __expf(x);
  else if constexpr (K == kActCELU) return x > 0.f ? 1.f : __expf(x / a);
  else if constexpr (K == kActSELU) {
    constexpr float al = 1.6732632423543772f, sc = 1.0507009873554805f;
    return x > 0.f ? sc : sc * al * __expf(x);
  } else if constexpr (K == kActHardswish) {  // ATen: 0 at x <= -3, 1 at x >= 3
    return x <= -3.f ? 0.f : (x < 3.f ? (2.f * x + 3.f) * (1.f / 6.f) : 1.f);
  }
  else if constexpr (K == kActHardtanh) return (x > a && x < b) ? 1.f : 0.f;
  else if constexpr (K == kActSiLU) {
    const float s = sigm(x);
    return s * (1.f + x * (1.f - s));
  } else if constexpr (K == kActSigmoid) {
    const float s = sigm(x);
    return s * (1.f - s);
  } else if constexpr (K == kActTanh) {
    const float t = tanhf(x);
    return 1.f - t * t;
  } else if constexpr (K == kActGELU) {
    const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
    const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
    return cdf + x * pdf;
  } else if constexpr (K == kActGELUTanh) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (x + k1 * x * x * x), t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  } else return x > 0.f ? 1.f : a;
}

template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int N = 4; typedef float4 type; };
template <> struct Vec<uint16_t> { static constexpr int N = 8; typedef uint4 type; };
template <> struct Vec<_Float16> { static constexpr int N = 8; typedef uint4 type; };

template <typename T, int N>
__device__ __forceinline__ void unpack(const typename Vec<T>::type& v, float* f) {
  const T* p = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int i = 0; i < N; ++i) f[i] = Io<T>::ld(p + i);
}
template <typename T, int N>
__device__ __forceinline__ typename Vec<T>::type pack(const float* f) {
  typename Vec<T>::type v;
  T* p = reinterpret_cast<T*>(&v);
#pragma unroll
  for (int i = 0; i < N; ++i) Io<T>::st(p + i, f[i]);
  return v;
}

// y = f(x) (BWD = false) or dx = dy * f'(x) (BWD = true) over n elements; 16-byte aligned bases
template <typename T, int K, bool BWD>
__global__ void __launch_bounds__(kActBlock) act_ew_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                           T* __restrict__ out, int64_t n, float a, float b) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::type VT;
  const int64_t nv = n / V;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kActBlock;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kActBlock) + threadIdx.x; i < nv; i += stride) {
    float xv[V], r[V];
    unpack<T, V>(reinterpret_cast<const VT*>(x)[i], xv);
    if constexpr (BWD) {
      float g[V];
      unpack<T, V>(reinterpret_cast<const VT*>(dy)[i], g);
#pragma unroll
      for (int e = 0; e < V; ++e) r[e] = g[e] * f_grad<K>(xv[e], a, b);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) r[e] = f_fwd<K>(xv[e], a, b);
    }
    reinterpret_cast<VT*>(out)[i] = pack<T, V>(r);
  }
  for (int64_t i = nv * V + blockIdx.x * static_cast<int64_t>(kActBlock) + threadIdx.x; i < n; i += stride) {
    const float xv = Io<T>::ld(x + i);
    Io<T>::st(out + i, BWD ? Io<T>::ld(dy + i) * f_grad<K>(xv, a, b) : f_fwd<K>(xv, a, b));
  }
}

// per-channel PReLU forward: channel of element i = (i / inner) % C (n < 2^32, host-checked)
template <typename T>
__global__ void __launch_bounds__(kActBlock) prelu_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                              T* __restrict__ y, uint32_t n, FastDiv fin, FastDiv fc,
                                                              const float* __restrict__ ss, int C) {
  for (uint32_t i = blockIdx.x * kActBlock + threadIdx.x; i < n; i += gridDim.x * kActBlock) {
    uint32_t c;
    fc.divmod(fin.div(i), c);
    float v = Io<T>::ld(x + i);
    if (ss != nullptr) v = fmaf(v, ss[c], ss[C + c]);  // eval BN first (per-channel weight: c = channel)
    Io<T>::st(y + i, v > 0.f ? v : w[c] * v);
  }
}

// PReLU backward, channels-last / flat view [M, C] (C = 1 for a scalar weight over any layout):
// thread (tx, ty) of a TX x TY block owns channels tx, tx + TX, ... and rows ty, ty + TY, ...
// of the block's row range; its dw partials live in LDS slots acc[ty][c] only it touches.
template <typename T>
__global__ void __launch_bounds__(kActBlock) prelu_bwd_rows_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                                   const float* __restrict__ w, T* __restrict__ dx,
                                                                   float* __restrict__ part, int64_t M, int C,
                                                                   int64_t rows_per_block, int TX) {
  extern __shared__ float acc[];  // [TY][C]
  const int TY = kActBlock / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const bool live = ty < TY;  // TX need not divide the block: the spare threads only join the fold
  if (live)
    for (int c = tx; c < C; c += TX) acc[ty * C + c] = 0.f;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = live ? min(r0 + rows_per_block, M) : r0;
  for (int64_t r = r0 + ty; r < r1; r += TY) {
    for (int c = tx; c < C; c += TX) {
      const int64_t i = r * C + c;
      const float v = Io<T>::ld(x + i), g = Io<T>::ld(dy + i);
      const bool pos = v > 0.f;
      Io<T>::st(dx + i, pos ? g : w[c] * g);
      if (!pos) acc[ty * C + c] += g * v;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kActBlock) {
    float s = 0.f;
    for (int k = 0; k < TY; ++k) s += acc[k * C + c];
    part[static_cast<int64_t>(blockIdx.x) * C + c] = s;
  }
}

// 16-byte-vector forms for channels-last with C % V == 0: a lane owns V consecutive channels
template <typename T>
__global__ void __launch_bounds__(kActBlock) prelu_fwd_vec_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                                  T* __restrict__ y, uint32_t nv, FastDiv fcv,
                                                                  const float* __restrict__ ss, int C) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::type VT;
  for (uint32_t i = blockIdx.x * kActBlock + threadIdx.x; i < nv; i += gridDim.x * kActBlock) {
    uint32_t cg;
    fcv.divmod(i, cg);  // channel group of vector i
    float v[V];
    unpack<T, V>(reinterpret_cast<const VT*>(x)[i], v);
    if (ss != nullptr) {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = fmaf(v[e], ss[cg * V + e], ss[C + cg * V + e]);
    }
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = v[e] > 0.f ? v[e] : w[cg * V + e] * v[e];
    reinterpret_cast<VT*>(y)[i] = pack<T, V>(v);
  }
}

template <typename T>
__global__ void __launch_bounds__(kActBlock) prelu_bwd_rows_vec_kernel(const T* __restrict__ x,
                                                                       const T* __restrict__ dy,
                                                                       const float* __restrict__ w, T* __restrict__ dx,
                                                                       float* __restrict__ part, int64_t M, int C,
                                                                       int64_t rows_per_block, int TX) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::type VT;
  extern __shared__ float acc[];  // [TY][C]
  const int CG = C / V, TY = kActBlock / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const bool live = ty < TY;
  if (live)
    for (int g = tx; g < CG; g += TX)
#pragma unroll
      for (int e = 0; e < V; ++e) acc[ty * C + g * V + e] = 0.f;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = live ? min(r0 + rows_per_block, M) : r0;
  for (int64_t r = r0 + ty; r < r1; r += TY) {
    for (int g = tx; g < CG; g += TX) {
      const int64_t i = r * CG + g;  // vector index
      float v[V], d[V], o[V];
      unpack<T, V>(reinterpret_cast<const VT*>(x)[i], v);
      unpack<T, V>(reinterpret_cast<const VT*>(dy)[i], d);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const bool pos = v[e] > 0.f;
        o[e] = pos ? d[e] : w[g * V + e] * d[e];
        if (!pos) acc[ty * C + g * V + e] += d[e] * v[e];
      }
      reinterpret_cast<VT*>(dx)[i] = pack<T, V>(o);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kActBlock) {
    float s = 0.f;
    for (int k = 0; k < TY; ++k) s += acc[k * C + c];
    part[static_cast<int64_t>(blockIdx.x) * C + c] = s;
  }
}

// PReLU backward, contiguous [N, C, HW]: one block per (n, c) plane slice
template <typename T>
__global__ void __launch_bounds__(kActBlock) prelu_bwd_planes_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                                     const float* __restrict__ w, T* __restrict__ dx,
                                                                     float* __restrict__ part, int C, int64_t HW,
                                                                     int slices) {
  __shared__ float red[kActBlock / kWave];
  const int plane = blockIdx.x / slices, sl = blockIdx.x % slices;
  const int c = plane % C;
  const float wc = w[c];
  const int64_t per = (HW + slices - 1) / slices;
  const int64_t p0 = static_cast<int64_t>(sl) * per, p1 = min(p0 + per, HW);
  const int64_t base = static_cast<int64_t>(plane) * HW;
  float s = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += kActBlock) {
    const float v = Io<T>::ld(x + base + p), g = Io<T>::ld(dy + base + p);
    const bool pos = v > 0.f;
    Io<T>::st(dx + base + p, pos ? g : wc * g);
    if (!pos) s += g * v;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;  // [N][C][slices]
}

// dw[c] = sum over the slab rows in fixed order.  rows layout: part[r * C + c] (rows mode) or
// part[(n * C + c) * slices + s] (planes mode: rows = N * slices).  One block per 64 channels;
// 16 waves take interleaved rows (independent loads in flight), then the 16 wave partials are
// summed in wave order (deterministic).  A single thread per channel walking up to 2048 rows
// serially took ~140 us per call (33 ms per CFPNet step, profiles/r3_models).
constexpr int kWfWaves = 16;
__global__ void __launch_bounds__(kWfWaves * 64) act_prelu_wfinal(const float* __restrict__ part,
                                                                  float* __restrict__ dw, int C, int rows,
                                                                  int planes_slices) {
  __shared__ float red[kWfWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < C) {
    if (planes_slices == 0) {
#pragma unroll 4
      for (int r = w; r < rows; r += kWfWaves) s += part[static_cast<int64_t>(r) * C + c];
    } else {
      const int n_items = rows / C;  // (batch entry, slice) pairs
#pragma unroll 4
      for (int it = w; it < n_items; it += kWfWaves) {
        const int i = it / planes_slices, k = it - (it / planes_slices) * planes_slices;
        s += part[(static_cast<int64_t>(i) * C + c) * planes_slices + k];
      }
    }
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int u = 0; u < kWfWaves; ++u) t += red[u][lane];
    dw[c] = t;
  }
}

template <typename T, bool BWD>
void ew_dispatch(const ActArgs& a, int grid, hipStream_t st) {
  const T* x = static_cast<const T*>(a.x);
  const T* dy = static_cast<const T*>(a.dy);
  T* out = static_cast<T*>(a.out);
#define RTSEG_ACT_CASE(K)                                                                          \
  case K: act_ew_kernel<T, K, BWD><<<grid, kActBlock, 0, st>>>(x, dy, out, a.n, a.a, a.b); break;
  switch (a.kind) {
    RTSEG_ACT_CASE(kActPReLU)
    RTSEG_ACT_CASE(kActLeaky)
    RTSEG_ACT_CASE(kActELU)
    RTSEG_ACT_CASE(kActCELU)
    RTSEG_ACT_CASE(kActSELU)
    RTSEG_ACT_CASE(kActHardswish)
    RTSEG_ACT_CASE(kActHardtanh)
    RTSEG_ACT_CASE(kActSiLU)
    RTSEG_ACT_CASE(kActSigmoid)
    RTSEG_ACT_CASE(kActTanh)
    RTSEG_ACT_CASE(kActGELU)
    RTSEG_ACT_CASE(kActGELUTanh)
    default: break;
  }
#undef RTSEG_ACT_CASE
}

template <typename T>
void launch_typed(const ActArgs& a, hipStream_t st) {
  const int grid = stream_grid((a.n + 7) / 8, kActBlock);
  const bool channel_w = a.kind == kActPReLU && a.w != nullptr;
  const ActPreluPlan p = act_prelu_plan(a);
  if (!a.bwd) {
    if (channel_w && p.vec > 1) {
      const uint32_t nv = static_cast<uint32_t>(a.n / p.vec);
      prelu_fwd_vec_kernel<T><<<stream_grid(nv, kActBlock), kActBlock, 0, st>>>(
          static_cast<const T*>(a.x), a.w, static_cast<T*>(a.out), nv, FastDiv::make(static_cast<uint32_t>(a.C / p.vec)),
          a.ss, a.C);
    } else if (channel_w) {
      prelu_fwd_kernel<T><<<stream_grid(a.n, kActBlock), kActBlock, 0, st>>>(
          static_cast<const T*>(a.x), a.w, static_cast<T*>(a.out), static_cast<uint32_t>(a.n),
          FastDiv::make(static_cast<uint32_t>(a.inner)), FastDiv::make(static_cast<uint32_t>(a.C)), a.ss, a.C);
    } else {
      ew_dispatch<T, false>(a, grid, st);
    }
    return;
  }
  if (!channel_w) {
    ew_dispatch<T, true>(a, grid, st);
    return;
  }
  const T* x = static_cast<const T*>(a.x);
  const T* dy = static_cast<const T*>(a.dy);
  T* dx = static_cast<T*>(a.out);
  if (p.planes) {
    prelu_bwd_planes_kernel<T><<<p.blocks, kActBlock, 0, st>>>(x, dy, a.w, dx, a.part, a.C, a.inner, p.slices);
    act_prelu_wfinal<<<(a.C + 63) / 64, kWfWaves * 64, 0, st>>>(a.part, a.dw, a.C, p.blocks, p.slices);
  } else {
    const int TY = kActBlock / p.tx;
    const size_t lds = static_cast<size_t>(TY) * a.C * sizeof(float);
    if (p.vec > 1)
      prelu_bwd_rows_vec_kernel<T><<<p.blocks, kActBlock, lds, st>>>(x, dy, a.w, dx, a.part, a.n / a.C, a.C,
                                                                       p.rows_per_block, p.tx);
    else
      prelu_bwd_rows_kernel<T><<<p.blocks, kActBlock, lds, st>>>(x, dy, a.w, dx, a.part, a.n / a.C, a.C,
                                                                   p.rows_per_block, p.tx);
    act_prelu_wfinal<<<(a.C + 63) / 64, kWfWaves * 64, 0, st>>>(a.part, a.dw, a.C, p.blocks, 0);
  }
}

}  // namespace

ActPreluPlan act_prelu_plan(const ActArgs& a) {
  ActPreluPlan p{};
  if (a.inner > 1) {  // contiguous [N, C, HW]: slice each plane so the grid fills the chip
    const int64_t planes = a.n / a.inner;
    p.planes = true;
    p.slices = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((2048 + planes - 1) / planes,
                                                                       (a.inner + 4095) / 4096)));
    p.blocks = static_cast<int>(planes * p.slices);
  } else {  // [M, C] rows; 16-byte channel vectors when C allows (channels-last, C > 1)
    const int64_t M = a.n / a.C;
    const int v = a.dtype == kF32 ? 4 : 8;
    p.vec = (a.C > 1 && a.C % v == 0) ? v : 1;
    const int groups = a.C / p.vec;
    p.tx = groups >= 64 ? 64 : groups;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(2048, (M + 63) / 64));
    p.rows_per_block = (M + blocks - 1) / blocks;
    p.blocks = static_cast<int>((M + p.rows_per_block - 1) / p.rows_per_block);
  }
  return p;
}

void launch_act(const ActArgs& a, hipStream_t st) {
  if (a.n == 0) return;
  switch (a.dtype) {
    case kF32: launch_typed<float>(a, st); break;
    case kBF16: launch_typed<uint16_t>(a, st); break;
    default: launch_typed<_Float16>(a, st); break;
  }
}

}  // namespace rtseg
