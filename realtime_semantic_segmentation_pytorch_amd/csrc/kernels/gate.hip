// Attention gating (K10): out = x * s, x * (1 + s) or x * s + y * (1 - s), with the gate s
// broadcast per channel ([N, C]: squeeze-excite / ARM / FFM / CGNet / CANet), per pixel
// ([N, H*W]: PP-LiteSeg spatial UAFM, AGLNet) or full-size (BiSeNetV2 BGA), optionally
// s = sigmoid(logits) computed in-kernel.  Channels-last activations, one pass each way.
//
// Reference sites: bisenetv1.py:76-114 (ARM, FFM), regseg.py:109-127 (SE), cgnet.py:105-108,
// canet.py:107-117, pp_liteseg.py:120-141, aglnet.py:95-111, bisenetv2.py:140-162 -- each a
// chain of 2-4 stock PyTorch ops (expand / sigmoid / mul / add) over the full activation.
//
// Backward: dx (and dy) elementwise, and the gate gradient reduced over what it was broadcast
// over -- per (n, c) over the image (two-level, deterministic: per-block partial rows + a
// finalize), per pixel over the channels (lanes of one pixel reduce by DPP-free shuffles inside
// the wave), or elementwise.
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {
namespace {

template <typename T, int V> struct Vec;
template <int V> struct Vec<float, V> {
  __device__ __forceinline__ static void ld(const float* p, float* f) {
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = p[j];
  }
  __device__ __forceinline__ static void st(float* p, const float* f) {
#pragma unroll
    for (int j = 0; j < V; ++j) p[j] = f[j];
  }
};
template <int V> struct Vec<uint16_t, V> {
  __device__ __forceinline__ static void ld(const uint16_t* p, float* f) {
    uint16_t e[V];
    __builtin_memcpy(e, p, sizeof(e));
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = bf16_to_f32(e[j]);
  }
  __device__ __forceinline__ static void st(uint16_t* p, const float* f) {
    uint16_t e[V];
#pragma unroll
    for (int j = 0; j < V; ++j) e[j] = f32_to_bf16(f[j]);
    __builtin_memcpy(p, e, sizeof(e));
  }
};
template <int V> struct Vec<_Float16, V> {
  __device__ __forceinline__ static void ld(const _Float16* p, float* f) {
    _Float16 e[V];
    __builtin_memcpy(e, p, sizeof(e));
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = static_cast<float>(e[j]);
  }
  __device__ __forceinline__ static void st(_Float16* p, const float* f) {
    _Float16 e[V];
#pragma unroll
    for (int j = 0; j < V; ++j) e[j] = static_cast<_Float16>(f[j]);
    __builtin_memcpy(p, e, sizeof(e));
  }
};

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + __expf(-v)); }

// gate values of one channel vector: s[j] (post-sigmoid)
template <typename T, int V, int BC, bool SIG>
__device__ __forceinline__ void load_gate(const void* att, int64_t pix, int64_t n, int c0, int C, int64_t off,
                                          float* s) {
  if constexpr (BC == kGateChannel) {
    const float* a = static_cast<const float*>(att) + n * C + c0;
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = a[j];
  } else if constexpr (BC == kGateSpatial) {
    const float v = static_cast<const float*>(att)[pix];
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = v;
  } else {
    Vec<T, V>::ld(static_cast<const T*>(att) + off, s);
  }
  if constexpr (SIG) {
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = sigm(s[j]);
  }
}

template <typename T, int V, int MODE, int BC, bool SIG>
__global__ void __launch_bounds__(256) gate_fwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                       const void* __restrict__ att, T* __restrict__ out,
                                                       int64_t M, int HW, int C) {
  const int cv = C / V;
  const int64_t total = M * cv;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t pix = i / cv;
    const int c0 = static_cast<int>(i - pix * cv) * V;
    const int64_t off = pix * C + c0;
    float xv[V], s[V], o[V];
    Vec<T, V>::ld(x + off, xv);
    load_gate<T, V, BC, SIG>(att, pix, pix / HW, c0, C, off, s);
    if constexpr (MODE == kGateBlend) {
      float yv[V];
      Vec<T, V>::ld(y + off, yv);
#pragma unroll
      for (int j = 0; j < V; ++j) o[j] = fmaf(xv[j] - yv[j], s[j], yv[j]);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) o[j] = MODE == kGateResidual ? fmaf(xv[j], s[j], xv[j]) : xv[j] * s[j];
    }
    Vec<T, V>::st(out + off, o);
  }
}

// elementwise part of the backward; returns the gate-gradient terms (w.r.t. the logits when SIG)
template <typename T, int V, int MODE, int BC, bool SIG>
__device__ __forceinline__ void bwd_one(const T* go, const T* x, const T* y, const void* att, T* gx, T* gy,
                                        int64_t pix, int64_t n, int c0, int C, float* ga) {
  const int64_t off = pix * C + c0;
  float g[V], xv[V], s[V], d[V];
  Vec<T, V>::ld(go + off, g);
  Vec<T, V>::ld(x + off, xv);
  load_gate<T, V, BC, SIG>(att, pix, n, c0, C, off, s);
  if constexpr (MODE == kGateBlend) {
    float yv[V], dy[V];
    Vec<T, V>::ld(y + off, yv);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      d[j] = g[j] * s[j];
      dy[j] = g[j] - d[j];
      ga[j] = g[j] * (xv[j] - yv[j]);
    }
    Vec<T, V>::st(gy + off, dy);
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      d[j] = MODE == kGateResidual ? fmaf(g[j], s[j], g[j]) : g[j] * s[j];
      ga[j] = g[j] * xv[j];
    }
  }
  Vec<T, V>::st(gx + off, d);
  if constexpr (SIG) {
#pragma unroll
    for (int j = 0; j < V; ++j) ga[j] *= s[j] * (1.f - s[j]);
  }
}

// full-size or per-pixel gate: one pass; a pixel's cv = C / V threads are consecutive lanes
// of one wave (cv a power of two <= 64) and reduce their gate terms with xor shuffles
template <typename T, int V, int MODE, int BC, bool SIG>
__global__ void __launch_bounds__(256) gate_bwd_kernel(const T* __restrict__ go, const T* __restrict__ x,
                                                       const T* __restrict__ y, const void* __restrict__ att,
                                                       T* __restrict__ gx, T* __restrict__ gy,
                                                       void* __restrict__ gatt, int64_t M, int HW, int C) {
  const int cv = C / V;
  const int64_t total = M * cv;
  const int64_t step = static_cast<int64_t>(gridDim.x) * blockDim.x;
  // every lane of a wave runs the same number of iterations (shuffles need the whole wave)
  const int64_t base = blockIdx.x * static_cast<int64_t>(blockDim.x) + (threadIdx.x & ~63);
  for (int64_t wbase = base; wbase < total; wbase += step) {
    const int64_t i = wbase + (threadIdx.x & 63);
    const bool live = i < total;
    const int64_t pix = live ? i / cv : 0;
    const int c0 = live ? static_cast<int>(i - pix * cv) * V : 0;
    float ga[V];
    if (live) {
      bwd_one<T, V, MODE, BC, SIG>(go, x, y, att, gx, gy, pix, pix / HW, c0, C, ga);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) ga[j] = 0.f;
    }
    if constexpr (BC == kGateFull) {
      if (live) Vec<T, V>::st(static_cast<T*>(gatt) + pix * C + c0, ga);
    } else {  // kGateSpatial
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) t += ga[j];
      for (int m = 1; m < cv; m <<= 1) t += __shfl_xor(t, m, 64);
      if (live && c0 == 0) static_cast<float*>(gatt)[pix] = t;
    }
  }
}

// per-channel gate: dx / dy elementwise + per-block partial sums over the block's pixels of one
// image -> part[n][blk][C]; rows of rpi = 256 / cv pixels per iteration
template <typename T, int V, int MODE, bool SIG>
__global__ void __launch_bounds__(256) gate_bwd_channel_kernel(const T* __restrict__ go, const T* __restrict__ x,
                                                               const T* __restrict__ y, const float* __restrict__ att,
                                                               T* __restrict__ gx, T* __restrict__ gy,
                                                               float* __restrict__ part, int HW, int C,
                                                               int per_blk) {
  __shared__ float red[256 * V];
  const int cv = C / V, rpi = 256 / cv;
  const int my_cv = threadIdx.x % cv, my_r = threadIdx.x / cv;
  const int n = blockIdx.y, blk = blockIdx.x;
  const int c0 = my_cv * V;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  if (my_r < rpi) {
    const int p0 = blk * per_blk, p1 = min(p0 + per_blk, HW);
    for (int p = p0 + my_r; p < p1; p += rpi) {
      float ga[V];
      bwd_one<T, V, MODE, kGateChannel, SIG>(go, x, y, att, gx, gy, static_cast<int64_t>(n) * HW + p, n, c0, C, ga);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += ga[j];
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[threadIdx.x * V + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < cv) {
    float s[V];
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = 0.f;
    for (int r = 0; r < rpi; ++r)
#pragma unroll
      for (int j = 0; j < V; ++j) s[j] += red[(r * cv + threadIdx.x) * V + j];
    float* row = part + (static_cast<int64_t>(n) * gridDim.x + blk) * C + threadIdx.x * V;
#pragma unroll
    for (int j = 0; j < V; ++j) row[j] = s[j];
  }
}

__global__ void gate_channel_finalize(const float* __restrict__ part, int blocks, int C, float* __restrict__ gatt) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int b = 0; b < blocks; ++b) s += part[(static_cast<int64_t>(n) * blocks + b) * C + c];
  gatt[static_cast<int64_t>(n) * C + c] = s;
}

int grid_for(int64_t work) {
  int64_t g = (work + 255) / 256;
  return static_cast<int>(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

template <typename T, int V, typename F>
void with_mode(int mode, int bc, bool sig, F&& f) {
#define RT_GATE_CASE(MODE, BC)                          \
  if (sig) f.template operator()<T, V, MODE, BC, true>(); \
  else f.template operator()<T, V, MODE, BC, false>();
  auto by_bc = [&]<int MODE>() {
    if (bc == kGateChannel) { RT_GATE_CASE(MODE, kGateChannel) }
    else if (bc == kGateSpatial) { RT_GATE_CASE(MODE, kGateSpatial) }
    else { RT_GATE_CASE(MODE, kGateFull) }
  };
#undef RT_GATE_CASE
  if (mode == kGateMul) by_bc.template operator()<kGateMul>();
  else if (mode == kGateResidual) by_bc.template operator()<kGateResidual>();
  else by_bc.template operator()<kGateBlend>();
}

template <typename F>
void with_type(int dtype, int V, F&& f) {
  if (dtype == kF32) {
    if (V == 4) f.template operator()<float, 4>();
    else if (V == 2) f.template operator()<float, 2>();
    else f.template operator()<float, 1>();
  } else if (dtype == kBF16) {
    if (V == 8) f.template operator()<uint16_t, 8>();
    else if (V == 4) f.template operator()<uint16_t, 4>();
    else if (V == 2) f.template operator()<uint16_t, 2>();
    else f.template operator()<uint16_t, 1>();
  } else {
    if (V == 8) f.template operator()<_Float16, 8>();
    else if (V == 4) f.template operator()<_Float16, 4>();
    else if (V == 2) f.template operator()<_Float16, 2>();
    else f.template operator()<_Float16, 1>();
  }
}

}  // namespace

int gate_vec_width(int dtype, int C) {
  for (int v = dtype == kF32 ? 4 : 8; v > 1; v >>= 1)
    if (C % v == 0 && C / v <= 256) return v;
  return C <= 256 ? 1 : 0;
}

bool gate_bwd_supported(int dtype, int C, int bc) {
  const int V = gate_vec_width(dtype, C);
  if (V == 0) return false;
  if (bc != kGateSpatial) return true;
  const int cv = C / V;
  return cv <= 64 && (cv & (cv - 1)) == 0;
}

int gate_channel_blocks(int64_t HW, int N) {
  // ~1024 blocks in all, >= 64 pixels each
  int64_t b = (1024 + N - 1) / N;
  const int64_t cap = (HW + 63) / 64;
  if (b > cap) b = cap;
  return static_cast<int>(b < 1 ? 1 : b);
}

void launch_gate_fwd(const GateArgs& g, hipStream_t st) {
  const int V = gate_vec_width(g.dtype, g.C);
  with_type(g.dtype, V, [&]<typename T, int VV>() {
    with_mode<T, VV>(g.mode, g.bc, g.sigmoid, [&]<typename TT, int W, int MODE, int BC, bool SIG>() {
      gate_fwd_kernel<TT, W, MODE, BC, SIG><<<grid_for(g.M * (g.C / W)), 256, 0, st>>>(
          static_cast<const TT*>(g.x), static_cast<const TT*>(g.y), g.att, static_cast<TT*>(g.out), g.M, g.HW,
          g.C);
    });
  });
}

void launch_gate_bwd(const GateArgs& g, const void* go, void* gx, void* gy, void* gatt, float* part, hipStream_t st) {
  const int V = gate_vec_width(g.dtype, g.C);
  with_type(g.dtype, V, [&]<typename T, int VV>() {
    with_mode<T, VV>(g.mode, g.bc, g.sigmoid, [&]<typename TT, int W, int MODE, int BC, bool SIG>() {
      if constexpr (BC == kGateChannel) {
        const int N = static_cast<int>(g.M / g.HW);
        const int blocks = gate_channel_blocks(g.HW, N);
        const int per_blk = static_cast<int>((g.HW + blocks - 1) / blocks);
        gate_bwd_channel_kernel<TT, W, MODE, SIG><<<dim3(blocks, N), 256, 0, st>>>(
            static_cast<const TT*>(go), static_cast<const TT*>(g.x), static_cast<const TT*>(g.y),
            static_cast<const float*>(g.att), static_cast<TT*>(gx), static_cast<TT*>(gy), part, g.HW, g.C, per_blk);
        gate_channel_finalize<<<dim3((g.C + 255) / 256, N), 256, 0, st>>>(part, blocks, g.C,
                                                                           static_cast<float*>(gatt));
      } else {
        gate_bwd_kernel<TT, W, MODE, BC, SIG><<<grid_for(g.M * (g.C / W)), 256, 0, st>>>(
            static_cast<const TT*>(go), static_cast<const TT*>(g.x), static_cast<const TT*>(g.y), g.att,
            static_cast<TT*>(gx), static_cast<TT*>(gy), gatt, g.M, g.HW, g.C);
      }
    });
  });
}

}  // namespace rtseg
