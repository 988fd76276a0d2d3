// Fused BatchNorm (train/eval) + optional residual add + activation for
// channels-last activations, forward and backward, SyncBN-ready.
//
// Replaces the reference's ConvBNAct tail (models/modules.py:73-85: BatchNorm2d
// -> Activation) and the residual epilogues of models/ddrnet.py:168-219
// (`out += identity; out = relu(out)`), which in stock PyTorch are 3-4 kernel
// families per layer (MIOpen BN fwd = 3 kernels, bwd = 3 kernels, add, relu,
// relu-backward).
//
// Layout: x is [M, C] row-major (M = N*H*W, i.e. NHWC / channels_last). One
// thread owns a 16-byte channel vector (8 bf16/fp16 or 4 fp32) and walks rows;
// per-channel partial sums are reduced in LDS and added to fp64 accumulators
// with one atomic per channel per block, so the cross-rank SyncBN reduction is
// a single all-reduce of [2, C] doubles (done by the caller on RCCL).
//
// Backward "mask modes": the activation derivative is recomputed instead of
// stored -- from the pre-activation x*scale+shift when there is no residual
// (so the forward output need not be kept), or from the saved output y.
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

enum MaskMode : int { kMaskNone = 0, kMaskFromY = 1, kMaskFromX = 2 };

template <typename T> struct Vec;
template <> struct Vec<uint16_t> {  // bf16
  static constexpr int N = 8;
  typedef short raw __attribute__((ext_vector_type(8)));
  __device__ __forceinline__ static void load(const uint16_t* p, float* f) {
    raw v = *reinterpret_cast<const raw*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = bf16_to_f32(static_cast<uint16_t>(v[j]));
  }
  __device__ __forceinline__ static void store(uint16_t* p, const float* f) {
    raw v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = static_cast<short>(f32_to_bf16(f[j]));
    *reinterpret_cast<raw*>(p) = v;
  }
};
template <> struct Vec<_Float16> {
  static constexpr int N = 8;
  typedef _Float16 raw __attribute__((ext_vector_type(8)));
  __device__ __forceinline__ static void load(const _Float16* p, float* f) {
    raw v = *reinterpret_cast<const raw*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = static_cast<float>(v[j]);
  }
  __device__ __forceinline__ static void store(_Float16* p, const float* f) {
    raw v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = static_cast<_Float16>(f[j]);
    *reinterpret_cast<raw*>(p) = v;
  }
};
template <> struct Vec<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float* f) {
    float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};

template <int ACT>
__device__ __forceinline__ float act_grad_pre(float g, float z) {  // from pre-activation z
  if constexpr (ACT == kActReLU) return z > 0.f ? g : 0.f;
  else if constexpr (ACT == kActReLU6) return (z > 0.f && z < 6.f) ? g : 0.f;
  else return g;
}

// --------------------------------------------------------------- stats ------
// sums[0:C] += sum x, sums[C:2C] += sum x^2
template <typename T>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ x, int64_t M, int C,
                                                       double* __restrict__ sums) {
  constexpr int V = Vec<T>::N;
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [rows_per_iter][C] x 2
  const int cv = C / V;
  const int rpi = blockDim.x / cv;  // rows per iteration
  const int t = threadIdx.x;
  const int my_cv = t % cv;
  const int my_r = t / cv;
  float s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (my_r < rpi) {
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * rpi + my_r; r < M;
         r += static_cast<int64_t>(gridDim.x) * rpi) {
      float f[V];
      Vec<T>::load(x + r * C + my_cv * V, f);
#pragma unroll
      for (int j = 0; j < V; ++j) { s[j] += f[j]; q[j] += f[j] * f[j]; }
    }
  }
  float* ss = sm;
  float* qq = sm + rpi * C;
  if (my_r < rpi) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      ss[my_r * C + my_cv * V + j] = s[j];
      qq[my_r * C + my_cv * V + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += blockDim.x) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < rpi; ++r) { a += ss[r * C + c]; b += qq[r * C + c]; }
    atomicAdd(sums + c, a);
    atomicAdd(sums + C + c, b);
  }
  if (blockIdx.x == 0 && t == 0) atomicAdd(sums + 2 * C, static_cast<double>(M));
}

// One thread per channel: batch mean/invstd, affine scale/shift, running stats.
__global__ void bn_finalize_kernel(const double* __restrict__ sums, int C,
                                   const float* __restrict__ w, const float* __restrict__ b,
                                   float* __restrict__ rmean, float* __restrict__ rvar,
                                   int64_t* __restrict__ nbt, float momentum, float eps,
                                   float* __restrict__ mean_invstd, float* __restrict__ scale_shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  const double count = sums[2 * C];
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  const float wc = w ? w[c] : 1.f;
  const float bc = b ? b[c] : 0.f;
  const float sc = wc * invstd;
  mean_invstd[c] = static_cast<float>(mean);
  mean_invstd[C + c] = invstd;
  scale_shift[c] = sc;
  scale_shift[C + c] = bc - static_cast<float>(mean) * sc;
  if (rmean) {
    const double unbiased = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * static_cast<float>(mean);
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * static_cast<float>(unbiased);
  }
}

// Eval mode: scale/shift from running statistics.
__global__ void bn_eval_coeffs_kernel(int C, const float* __restrict__ w, const float* __restrict__ b,
                                      const float* __restrict__ rmean, const float* __restrict__ rvar,
                                      float eps, float* __restrict__ mean_invstd,
                                      float* __restrict__ scale_shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rvar[c] + eps);
  const float sc = (w ? w[c] : 1.f) * invstd;
  mean_invstd[c] = rmean[c];
  mean_invstd[C + c] = invstd;
  scale_shift[c] = sc;
  scale_shift[C + c] = (b ? b[c] : 0.f) - rmean[c] * sc;
}

// --------------------------------------------------------------- apply ------
template <typename T, int ACT, bool RES>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ res,
                                                       const float* __restrict__ scale_shift,
                                                       T* __restrict__ y, int64_t M, int C) {
  constexpr int V = Vec<T>::N;
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [2][C]
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) coef[c] = scale_shift[c];
  __syncthreads();
  const int cv = C / V;
  const int64_t total = M * cv;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c0 = static_cast<int>(i % cv) * V;
    const int64_t off = (i / cv) * C + c0;
    float f[V], r[V];
    Vec<T>::load(x + off, f);
    if constexpr (RES) Vec<T>::load(res + off, r);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float z = f[j] * coef[c0 + j] + coef[C + c0 + j];
      if constexpr (RES) z += r[j];
      f[j] = act_fwd<ACT>(z);
    }
    Vec<T>::store(y + off, f);
  }
}

// ----------------------------------------------------------- backward -------
template <typename T, int ACT, int MASK>
__device__ __forceinline__ void load_g(const T* dy, const T* x, const T* y, const float* coef, int C,
                                       int64_t off, int c0, float* g, float* xv) {
  constexpr int V = Vec<T>::N;
  Vec<T>::load(dy + off, g);
  Vec<T>::load(x + off, xv);
  if constexpr (MASK == kMaskFromY) {
    float yv[V];
    Vec<T>::load(y + off, yv);
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = act_bwd_from_out<ACT>(g[j], yv[j]);
  } else if constexpr (MASK == kMaskFromX) {
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = act_grad_pre<ACT>(g[j], xv[j] * coef[c0 + j] + coef[C + c0 + j]);
  }
}

// sums[0:C] += sum g, sums[C:2C] += sum g * (x - mean)
template <typename T, int ACT, int MASK>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean_invstd, const float* __restrict__ scale_shift, int64_t M, int C,
    double* __restrict__ sums) {
  constexpr int V = Vec<T>::N;
  extern __shared__ __attribute__((aligned(16))) float sm[];  // coef[2C] | mean[C] | partials
  float* coef = sm;
  float* mu = sm + 2 * C;
  const int cv = C / V;
  const int rpi = blockDim.x / cv;
  float* ss = sm + 3 * C;
  float* qq = ss + rpi * C;
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) coef[c] = scale_shift[c];
  for (int c = threadIdx.x; c < C; c += blockDim.x) mu[c] = mean_invstd[c];
  __syncthreads();
  const int t = threadIdx.x;
  const int my_cv = t % cv, my_r = t / cv, c0 = my_cv * V;
  float s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (my_r < rpi) {
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * rpi + my_r; r < M;
         r += static_cast<int64_t>(gridDim.x) * rpi) {
      float g[V], xv[V];
      load_g<T, ACT, MASK>(dy, x, y, coef, C, r * C + c0, c0, g, xv);
#pragma unroll
      for (int j = 0; j < V; ++j) { s[j] += g[j]; q[j] += g[j] * (xv[j] - mu[c0 + j]); }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) { ss[my_r * C + c0 + j] = s[j]; qq[my_r * C + c0 + j] = q[j]; }
  }
  __syncthreads();
  for (int c = t; c < C; c += blockDim.x) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < rpi; ++r) { a += ss[r * C + c]; b += qq[r * C + c]; }
    atomicAdd(sums + c, a);
    atomicAdd(sums + C + c, b);
  }
}

// Per channel: dx coefficients (k1, k2, k3) and the parameter gradients.
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ sums,
                                       const double* __restrict__ count_ptr, int C,
                                       const float* __restrict__ w,
                                       const float* __restrict__ mean_invstd, int batch_stats,
                                       float* __restrict__ kcoef, float* __restrict__ dw,
                                       float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = mean_invstd[C + c];
  const double sg = sums[c], sgx = sums[C + c];
  const double count = count_ptr ? *count_ptr : 1.0;
  if (dw) dw[c] = static_cast<float>(sgx * invstd);
  if (db) db[c] = static_cast<float>(sg);
  const float wc = w ? w[c] : 1.f;
  kcoef[c] = wc * invstd;
  if (batch_stats) {
    kcoef[C + c] = static_cast<float>(sg / count);
    kcoef[2 * C + c] = static_cast<float>(sgx / count) * invstd * invstd;
  } else {
    kcoef[C + c] = 0.f;
    kcoef[2 * C + c] = 0.f;
  }
}

template <typename T, int ACT, int MASK, bool DRES>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean_invstd, const float* __restrict__ scale_shift,
    const float* __restrict__ kcoef, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C) {
  constexpr int V = Vec<T>::N;
  extern __shared__ __attribute__((aligned(16))) float sm[];  // coef[2C] | mu[C] | k[3C]
  float* coef = sm;
  float* mu = sm + 2 * C;
  float* k = sm + 3 * C;
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) coef[c] = scale_shift[c];
  for (int c = threadIdx.x; c < C; c += blockDim.x) mu[c] = mean_invstd[c];
  for (int c = threadIdx.x; c < 3 * C; c += blockDim.x) k[c] = kcoef[c];
  __syncthreads();
  const int cv = C / V;
  const int64_t total = M * cv;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c0 = static_cast<int>(i % cv) * V;
    const int64_t off = (i / cv) * C + c0;
    float g[V], xv[V], o[V];
    load_g<T, ACT, MASK>(dy, x, y, coef, C, off, c0, g, xv);
    if constexpr (DRES) Vec<T>::store(dres + off, g);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = c0 + j;
      o[j] = k[c] * (g[j] - k[C + c] - (xv[j] - mu[c]) * k[2 * C + c]);
    }
    Vec<T>::store(dx + off, o);
  }
}

// ------------------------------------------------------------ launchers -----
static int reduce_grid(int64_t M, int rpi) {
  int64_t g = (M + rpi * 64 - 1) / (rpi * 64);  // >= 64 rows per thread-row
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

template <typename T>
static void stats_t(const void* x, int64_t M, int C, double* sums, hipStream_t st) {
  const int cv = C / Vec<T>::N;
  const int rpi = 256 / cv;
  const size_t lds = sizeof(float) * 2 * rpi * C;
  bn_stats_kernel<T><<<reduce_grid(M, rpi), 256, lds, st>>>(static_cast<const T*>(x), M, C, sums);
}

void launch_bn_stats(const void* x, int dtype, int64_t M, int C, double* sums, hipStream_t st) {
  hipMemsetAsync(sums, 0, sizeof(double) * (2 * C + 1), st);
  if (dtype == kF32) stats_t<float>(x, M, C, sums, st);
  else if (dtype == kBF16) stats_t<uint16_t>(x, M, C, sums, st);
  else stats_t<_Float16>(x, M, C, sums, st);
}

void launch_bn_finalize(const double* sums, int C, const float* w, const float* b,
                        float* rmean, float* rvar, int64_t* nbt, float momentum, float eps,
                        float* mean_invstd, float* scale_shift, hipStream_t st) {
  bn_finalize_kernel<<<(C + 255) / 256, 256, 0, st>>>(sums, C, w, b, rmean, rvar, nbt,
                                                      momentum, eps, mean_invstd, scale_shift);
}

void launch_bn_eval_coeffs(int C, const float* w, const float* b, const float* rmean,
                           const float* rvar, float eps, float* mean_invstd, float* scale_shift,
                           hipStream_t st) {
  bn_eval_coeffs_kernel<<<(C + 255) / 256, 256, 0, st>>>(C, w, b, rmean, rvar, eps, mean_invstd,
                                                         scale_shift);
}

template <typename T, int ACT>
static void apply_t(const void* x, const void* res, const float* ss, void* y, int64_t M, int C,
                    hipStream_t st) {
  const int64_t work = M * (C / Vec<T>::N);
  const size_t lds = sizeof(float) * 2 * C;
  const int grid = stream_grid(work, 256);
  if (res)
    bn_apply_kernel<T, ACT, true><<<grid, 256, lds, st>>>(
        static_cast<const T*>(x), static_cast<const T*>(res), ss, static_cast<T*>(y), M, C);
  else
    bn_apply_kernel<T, ACT, false><<<grid, 256, lds, st>>>(
        static_cast<const T*>(x), nullptr, ss, static_cast<T*>(y), M, C);
}

template <typename T>
static void apply_act(const void* x, const void* res, const float* ss, void* y, int64_t M, int C,
                      int act, hipStream_t st) {
  if (act == kActReLU) apply_t<T, kActReLU>(x, res, ss, y, M, C, st);
  else if (act == kActReLU6) apply_t<T, kActReLU6>(x, res, ss, y, M, C, st);
  else apply_t<T, kActNone>(x, res, ss, y, M, C, st);
}

void launch_bn_apply(const void* x, const void* res, const float* scale_shift, void* y, int dtype,
                     int64_t M, int C, int act, hipStream_t st) {
  if (dtype == kF32) apply_act<float>(x, res, scale_shift, y, M, C, act, st);
  else if (dtype == kBF16) apply_act<uint16_t>(x, res, scale_shift, y, M, C, act, st);
  else apply_act<_Float16>(x, res, scale_shift, y, M, C, act, st);
}

template <typename T, int ACT, int MASK>
static void bwd_reduce_t(const void* dy, const void* x, const void* y, const float* mi,
                         const float* ss, int64_t M, int C, double* sums, hipStream_t st) {
  const int cv = C / Vec<T>::N;
  const int rpi = 256 / cv;
  const size_t lds = sizeof(float) * (3 * C + 2 * rpi * C);
  bn_bwd_reduce_kernel<T, ACT, MASK><<<reduce_grid(M, rpi), 256, lds, st>>>(
      static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mi, ss, M, C,
      sums);
}

template <typename T, int ACT, int MASK, bool DRES>
static void bwd_apply_t(const void* dy, const void* x, const void* y, const float* mi,
                        const float* ss, const float* k, void* dx, void* dres, int64_t M, int C,
                        hipStream_t st) {
  const int64_t work = M * (C / Vec<T>::N);
  const size_t lds = sizeof(float) * 6 * C;
  bn_bwd_apply_kernel<T, ACT, MASK, DRES><<<stream_grid(work, 256), 256, lds, st>>>(
      static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mi, ss, k,
      static_cast<T*>(dx), static_cast<T*>(dres), M, C);
}

#define RT_ACT_MASK_DISPATCH(FN, ...)                                                   \
  do {                                                                                  \
    if (act == kActNone) FN<T, kActNone, kMaskNone>(__VA_ARGS__);                       \
    else if (act == kActReLU) {                                                         \
      if (mask == kMaskFromY) FN<T, kActReLU, kMaskFromY>(__VA_ARGS__);                 \
      else FN<T, kActReLU, kMaskFromX>(__VA_ARGS__);                                    \
    } else {                                                                            \
      if (mask == kMaskFromY) FN<T, kActReLU6, kMaskFromY>(__VA_ARGS__);                \
      else FN<T, kActReLU6, kMaskFromX>(__VA_ARGS__);                                   \
    }                                                                                   \
  } while (0)

template <typename T>
static void bwd_reduce_dispatch(const void* dy, const void* x, const void* y, const float* mi,
                                const float* ss, int64_t M, int C, int act, int mask,
                                double* sums, hipStream_t st) {
  RT_ACT_MASK_DISPATCH(bwd_reduce_t, dy, x, y, mi, ss, M, C, sums, st);
}

void launch_bn_bwd_reduce(const void* dy, const void* x, const void* y, const float* mean_invstd,
                          const float* scale_shift, int dtype, int64_t M, int C, int act, int mask,
                          double* sums, hipStream_t st) {
  hipMemsetAsync(sums, 0, sizeof(double) * 2 * C, st);
  if (dtype == kF32) bwd_reduce_dispatch<float>(dy, x, y, mean_invstd, scale_shift, M, C, act, mask, sums, st);
  else if (dtype == kBF16) bwd_reduce_dispatch<uint16_t>(dy, x, y, mean_invstd, scale_shift, M, C, act, mask, sums, st);
  else bwd_reduce_dispatch<_Float16>(dy, x, y, mean_invstd, scale_shift, M, C, act, mask, sums, st);
}

void launch_bn_bwd_finalize(const double* sums, const double* count_ptr, int C, const float* w,
                            const float* mean_invstd, int batch_stats, float* kcoef, float* dw,
                            float* db, hipStream_t st) {
  bn_bwd_finalize_kernel<<<(C + 255) / 256, 256, 0, st>>>(sums, count_ptr, C, w, mean_invstd,
                                                          batch_stats, kcoef, dw, db);
}

template <typename T, int ACT, int MASK>
static void bwd_apply_res(const void* dy, const void* x, const void* y, const float* mi,
                          const float* ss, const float* k, void* dx, void* dres, int64_t M, int C,
                          hipStream_t st) {
  if (dres) bwd_apply_t<T, ACT, MASK, true>(dy, x, y, mi, ss, k, dx, dres, M, C, st);
  else bwd_apply_t<T, ACT, MASK, false>(dy, x, y, mi, ss, k, dx, dres, M, C, st);
}

template <typename T>
static void bwd_apply_dispatch(const void* dy, const void* x, const void* y, const float* mi,
                               const float* ss, const float* k, void* dx, void* dres, int64_t M,
                               int C, int act, int mask, hipStream_t st) {
  RT_ACT_MASK_DISPATCH(bwd_apply_res, dy, x, y, mi, ss, k, dx, dres, M, C, st);
}

void launch_bn_bwd_apply(const void* dy, const void* x, const void* y, const float* mean_invstd,
                         const float* scale_shift, const float* kcoef, void* dx, void* dres,
                         int dtype, int64_t M, int C, int act, int mask, hipStream_t st) {
  if (dtype == kF32) bwd_apply_dispatch<float>(dy, x, y, mean_invstd, scale_shift, kcoef, dx, dres, M, C, act, mask, st);
  else if (dtype == kBF16) bwd_apply_dispatch<uint16_t>(dy, x, y, mean_invstd, scale_shift, kcoef, dx, dres, M, C, act, mask, st);
  else bwd_apply_dispatch<_Float16>(dy, x, y, mean_invstd, scale_shift, kcoef, dx, dres, M, C, act, mask, st);
}

}  // namespace rtseg
