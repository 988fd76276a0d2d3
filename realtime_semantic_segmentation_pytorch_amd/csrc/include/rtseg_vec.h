// Vectorised channel loads/stores (VEC contiguous channels of one NHWC pixel) into
// fp32 registers: 16-byte accesses for bf16 x8, element loops otherwise.  Shared by
// the depth-wise conv and pooling kernels.
#pragma once

#include "rtseg_common.h"

namespace rtseg {

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
    for (int i = 0; i < 4; ++i) w[i] = f32x2_to_bf16x2(v[2 * i], v[2 * i + 1]);
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
    r.x = f32x2_to_bf16x2(v[0], v[1]);
    r.y = f32x2_to_bf16x2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = r;
  }
};
template <> struct Vec<uint16_t, 2> {
  __device__ __forceinline__ static void load(const uint16_t* p, float* v) {
    const unsigned r = *reinterpret_cast<const unsigned*>(p);
    v[0] = __uint_as_float(r << 16); v[1] = __uint_as_float(r & 0xffff0000u);
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float* v) {
    *reinterpret_cast<unsigned*>(p) = f32x2_to_bf16x2(v[0], v[1]);
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

}  // namespace rtseg
