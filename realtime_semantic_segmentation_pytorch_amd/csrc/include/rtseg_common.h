// Shared device helpers for the rtseg CDNA4 (gfx950) kernels.
//
// Kernel translation units include ONLY this header (plus hip_runtime) so they
// compile in seconds; tensor plumbing lives in csrc/binding.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtseg {

// Element type tags passed from the binding layer.
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };
// Fused activation codes (epilogue functors).
enum Act : int { kActNone = 0, kActReLU = 1, kActReLU6 = 2 };

constexpr int kWave = 64;  // CDNA wavefront width

// ---- bf16 / fp16 scalar conversions (bf16 kept as raw bits) ---------------
__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
// Round-to-nearest-even, NaN stays NaN: the plain conversion is gfx950's v_cvt_pk_bf16_f32
// (one instruction; the integer-arithmetic form costs a compare + select per value)
typedef __bf16 rtseg_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float rtseg_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
// two values -> one packed dword (lo | hi << 16) in a single v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t f32x2_to_bf16x2(float lo, float hi) {
  const rtseg_f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, rtseg_bf16x2_t));
}

template <typename T> struct Io;
template <> struct Io<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};
template <> struct Io<uint16_t> {  // bf16
  __device__ __forceinline__ static float ld(const uint16_t* p) { return bf16_to_f32(*p); }
  __device__ __forceinline__ static void st(uint16_t* p, float v) { *p = f32_to_bf16(v); }
};
template <> struct Io<_Float16> {
  __device__ __forceinline__ static float ld(const _Float16* p) { return static_cast<float>(*p); }
  __device__ __forceinline__ static void st(_Float16* p, float v) { *p = static_cast<_Float16>(v); }
};

template <int ACT>
__device__ __forceinline__ float act_fwd(float v) {
  if constexpr (ACT == kActReLU) return v > 0.f ? v : 0.f;
  else if constexpr (ACT == kActReLU6) return fminf(fmaxf(v, 0.f), 6.f);
  else return v;
}
// Gradient mask from the activation OUTPUT y (valid for relu / relu6).
template <int ACT>
__device__ __forceinline__ float act_bwd_from_out(float g, float y) {
  if constexpr (ACT == kActReLU) return y > 0.f ? g : 0.f;
  else if constexpr (ACT == kActReLU6) return (y > 0.f && y < 6.f) ? g : 0.f;
  else return g;
}

// ---- fast unsigned division by a loop-invariant divisor ---------------------
// q = (umulhi(n, m) + n) >> s  (Granlund-Montgomery, exact for all 32-bit n): a
// 64-bit `/` or `%` in an index decomposition costs ~100 VALU instructions on
// CDNA, this costs 3-4, which matters in kernels doing O(10) FMAs per element.
struct FastDiv {
  uint32_t d, m, s;
  __host__ static FastDiv make(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;  // l = ceil(log2 d)
    f.s = l;
    f.m = static_cast<uint32_t>(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    return f;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint64_t t = __umulhi(n, m);
    return static_cast<uint32_t>((t + n) >> s);
  }
  __device__ __forceinline__ uint32_t divmod(uint32_t n, uint32_t& r) const {
    const uint32_t q = div(n);
    r = n - q * d;
    return q;
  }
};

// ---- wave / block reductions (64-lane waves) ------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum; `smem` must hold blockDim.x/64 elements. Result valid in all threads.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* smem) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = (blockDim.x + kWave - 1) / kWave;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += smem[i];
  return r;
}

// Grid sizing for streaming kernels: enough waves to fill 256 CUs, grid-stride the rest.
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  const int64_t cap = 256 * 16;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

// Source-index computation shared by every bilinear kernel (matches ATen's
// area_pixel_compute_source_index for linear mode).
struct LinMap {
  float scale;
  int in_size;
  bool align;
  __host__ __device__ static LinMap make(int in_size, int out_size, bool align) {
    LinMap m;
    m.in_size = in_size;
    m.align = align;
    if (align) m.scale = out_size > 1 ? static_cast<float>(in_size - 1) / static_cast<float>(out_size - 1) : 0.f;
    else m.scale = static_cast<float>(in_size) / static_cast<float>(out_size);
    return m;
  }
  // -> i0, i1 (= i0 or i0+1), lambda for i1 (host too: the loss backward's tile classes)
  __host__ __device__ __forceinline__ void map(int o, int& i0, int& i1, float& l) const {
    float src = align ? scale * static_cast<float>(o)
                      : fmaxf(scale * (static_cast<float>(o) + 0.5f) - 0.5f, 0.f);
    int f = static_cast<int>(src);
    if (f > in_size - 1) f = in_size - 1;
    i0 = f;
    i1 = f + (f < in_size - 1 ? 1 : 0);
    l = src - static_cast<float>(f);
  }
  // Weight with which output index o reads input index i.
  __device__ __forceinline__ float weight(int o, int i) const {
    int i0, i1; float l;
    map(o, i0, i1, l);
    float w = 0.f;
    if (i0 == i) w += 1.f - l;
    if (i1 == i) w += l;
    return w;
  }
  // Conservative range of output indices that may read input index i.
  __device__ __forceinline__ void out_range(int i, int out_size, int& lo, int& hi) const {
    if (scale <= 0.f) { lo = 0; hi = out_size - 1; return; }
    float a, b;
    if (align) { a = (i - 1) / scale; b = (i + 1) / scale; }
    else { a = (i - 0.5f) / scale - 0.5f; b = (i + 1.5f) / scale - 0.5f; }
    lo = static_cast<int>(floorf(a)) - 1;
    hi = static_cast<int>(ceilf(b)) + 1;
    if (lo < 0) lo = 0;
    if (hi > out_size - 1) hi = out_size - 1;
  }
};

}  // namespace rtseg
