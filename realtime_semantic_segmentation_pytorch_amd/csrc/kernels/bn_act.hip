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
// thread owns a 16-byte channel vector (8 bf16/fp16 or 4 fp32) and walks a
// contiguous row range of its block with 4 independent loads in flight; each
// block writes its per-channel partial sums to a [G, 2C] fp32 slab (no atomics,
// no memset, deterministic), and a finalize kernel reduces the slab in fp64 and
// produces mean/invstd, the folded scale/shift and the running-stat update in
// the same launch.  For SyncBN the slab is reduced to [2C+1] fp64 sums that the
// caller all-reduces over RCCL before finalizing.
//
// Backward "mask modes": the activation derivative is recomputed instead of
// stored -- from the pre-activation x*scale+shift when there is no residual
// (so the forward output need not be kept), or from the saved output y, or -- with a
// residual -- from a bit mask the forward wrote next to y (kMaskBits: one byte per
// V-channel vector, bit j = activation derivative of channel c0+j is 1), which replaces
// the 2-byte-per-element re-read of y in both backward passes by 1/8 byte.
#include <cstdlib>
#include <type_traits>

#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

enum MaskMode : int { kMaskNone = 0, kMaskFromY = 1, kMaskFromX = 2, kMaskBits = 3 };

// V-element channel vector of T: 16-byte vectors on the fast path (8 bf16/fp16 or
// 4 fp32); narrower widths (down to one element) serve channel counts that are
// not multiples of the full width (e.g. 12, 19, 35 channels in the zoo).
template <int BYTES> struct RawT;
template <> struct RawT<2> { typedef uint16_t type; };
template <> struct RawT<4> { typedef uint32_t type; };
template <> struct RawT<8> { typedef uint2 type; };
template <> struct RawT<16> { typedef uint4 type; };

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<uint16_t>(uint16_t v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float to_f<_Float16>(_Float16 v) { return static_cast<float>(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t from_f<uint16_t>(float v) { return f32_to_bf16(v); }
template <> __device__ __forceinline__ _Float16 from_f<_Float16>(float v) { return static_cast<_Float16>(v); }

template <typename T, int V>
struct VecIO {
  typedef typename RawT<V * sizeof(T)>::type raw;
  __device__ __forceinline__ static void load(const T* p, float* f) {
    raw r = *reinterpret_cast<const raw*>(p);
    T e[V];
    __builtin_memcpy(e, &r, sizeof(raw));
#pragma unroll
    for (int j = 0; j < V; ++j) f[j] = to_f<T>(e[j]);
  }
  __device__ __forceinline__ static void store(T* p, const float* f) {
    T e[V];
#pragma unroll
    for (int j = 0; j < V; ++j) e[j] = from_f<T>(f[j]);
    raw r;
    __builtin_memcpy(&r, e, sizeof(raw));
    *reinterpret_cast<raw*>(p) = r;
  }
};

template <int ACT>
__device__ __forceinline__ float act_grad_pre(float g, float z) {  // from pre-activation z
  if constexpr (ACT == kActReLU) return z > 0.f ? g : 0.f;
  else if constexpr (ACT == kActReLU6) return (z > 0.f && z < 6.f) ? g : 0.f;
  else return g;
}

// ----------------------------------------------------------- geometry -------
// Channel-vector / row layout of a block of 256 threads.
struct RowGeo {
  int cv, rpi, my_cv, my_r;
  __device__ __forceinline__ RowGeo(int C, int V) {
    cv = C / V;
    rpi = 256 / cv;
    my_cv = threadIdx.x % cv;
    my_r = threadIdx.x / cv;
  }
};

// Block-contiguous row range, a multiple of rpi rows.
__device__ __forceinline__ void block_rows(int64_t M, int rpi, int64_t& r0, int64_t& r1) {
  int64_t per = (M + gridDim.x - 1) / gridDim.x;
  per = (per + rpi - 1) / rpi * rpi;
  r0 = static_cast<int64_t>(blockIdx.x) * per;
  r1 = r0 + per < M ? r0 + per : M;
}

// Write this thread's V partial pairs to LDS, reduce over the rpi row-slots and
// store one [2C] slab row per block.
template <int V>
__device__ __forceinline__ void block_partials_out(const float* s, const float* q, const RowGeo& g,
                                                   int C, float* sm, float* __restrict__ part) {
  float* ss = sm;
  float* qq = sm + g.rpi * C;
  if (g.my_r < g.rpi) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      ss[g.my_r * C + g.my_cv * V + j] = s[j];
      qq[g.my_r * C + g.my_cv * V + j] = q[j];
    }
  }
  __syncthreads();
  float* out = part + static_cast<int64_t>(blockIdx.x) * 2 * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double a = 0.0, b = 0.0;  // <= 256 slots per channel: fp64 costs nothing here
    for (int r = 0; r < g.rpi; ++r) { a += ss[r * C + c]; b += qq[r * C + c]; }
    out[c] = static_cast<float>(a);
    out[C + c] = static_cast<float>(b);
  }
}

// Error-free accumulation s + x = (s', e): s' = fl(s + x), e the exact rounding error (Knuth's
// TwoSum, branch-free; relies on IEEE add/sub without reassociation, which hipcc keeps).
__device__ __forceinline__ void two_sum_acc(float& s, float& comp, float x) {
  const float t = s + x;
  const float bp = t - s;
  comp += (s - (t - bp)) + (x - bp);
  s = t;
}

// Per-channel pivot of the shifted moments: the mean of 8 rows spread over the tensor
// ((2k + 1) M / 16), identical in every thread (same loads, same order).  A typical value, unlike
// the corner pixel row 0, which on zero-padded conv outputs is the atypical one: ESPNet's
// near-constant channels sat ~100 sigma from their row-0 value (round-5 zoo numerics).
template <typename T, int V>
__device__ __forceinline__ void sample_pivot(const T* __restrict__ x, int64_t M, int64_t C, int c0, float* pv) {
  float a[8][V];
#pragma unroll
  for (int k = 0; k < 8; ++k) VecIO<T, V>::load(x + ((2 * k + 1) * M / 16) * C + c0, a[k]);
#pragma unroll
  for (int j = 0; j < V; ++j)
    pv[j] = (((a[0][j] + a[1][j]) + (a[2][j] + a[3][j])) + ((a[4][j] + a[5][j]) + (a[6][j] + a[7][j]))) * 0.125f;
}

// --------------------------------------------------------------- stats ------
// Shifted, compensated one-pass moments: every partial accumulates d = x - p and d*d about a
// per-channel pivot p (``sample_pivot``; the finalize adds the shift back in fp64, ``unshift``),
// and the running sum of d carries its TwoSum rounding error.  Plain sum / sum-of-squares
// partials lose var = E[x^2] - mean^2 to cancellation when |mean| >> std (BatchNorms over a few
// pooled values per channel: DDRNet's DAPPM global branch, BiSeNetV2's context block, 2 values
// at batch 2), and a plain fp32 running sum loses a channel sum whose terms cancel (a
// classifier's bias gradient: ~+1/19 on most pixels, ~-1 on the class's own; DDRNet-23's head
// bias gradients were 3.5e-3 off fp64 that way in round 4).  The pivot row is stored after the
// G slab rows (slab [G + 1, 2C], row G = pivots) by block 0.  shift = 0: pivot 0 (raw moments).
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ x, int64_t M, int C,
                                                       float* __restrict__ part, int shift) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const RowGeo g(C, V);
  float s[V], q[V], pv[V], e[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s[j] = 0.f; q[j] = 0.f; e[j] = 0.f; }
  if (g.my_r < g.rpi) {
    if (shift) {
      sample_pivot<T, V>(x, M, C, g.my_cv * V, pv);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) pv[j] = 0.f;
    }
    if (blockIdx.x == 0 && g.my_r == 0) {
      float* prow = part + static_cast<int64_t>(gridDim.x) * 2 * C + g.my_cv * V;
#pragma unroll
      for (int j = 0; j < V; ++j) prow[j] = pv[j];
    }
    int64_t r0, r1;
    block_rows(M, g.rpi, r0, r1);
    const T* base = x + g.my_cv * V;
    int64_t r = r0 + g.my_r;
    const int64_t step = static_cast<int64_t>(g.rpi) * C;
    for (; r + 3 * g.rpi < r1; r += 4 * g.rpi) {  // 4 independent 16-B loads in flight
      float f0[V], f1[V], f2[V], f3[V];
      const T* p = base + r * C;
      VecIO<T, V>::load(p, f0); VecIO<T, V>::load(p + step, f1);
      VecIO<T, V>::load(p + 2 * step, f2); VecIO<T, V>::load(p + 3 * step, f3);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float d0 = f0[j] - pv[j], d1 = f1[j] - pv[j], d2 = f2[j] - pv[j], d3 = f3[j] - pv[j];
        two_sum_acc(s[j], e[j], (d0 + d1) + (d2 + d3));
        q[j] += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    }
    for (; r < r1; r += g.rpi) {
      float f[V];
      VecIO<T, V>::load(base + r * C, f);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float d = f[j] - pv[j];
        two_sum_acc(s[j], e[j], d);
        q[j] += d * d;
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] += e[j];
  }
  block_partials_out<V>(s, q, g, C, sm, part);
}

// Slab [G][2C] -> fp64 per-channel totals for 64 channels per block; kFinWaves
// waves split the slab rows (16 waves keep the serial load chain per lane at
// G/16 rows -- these kernels are latency-bound, one block per 64 channels).
// Result in red[0..63] (sum) / red[64..127] (second).
constexpr int kFinWaves = 16;
constexpr int kFinBlock = kFinWaves * 64;

template <typename P>
__device__ __forceinline__ void reduce_slab64(const P* __restrict__ part, int g0, int G, int C, int c,
                                              double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double a = 0.0, b = 0.0;
  if (c < C) {
    const int64_t rs = 2 * static_cast<int64_t>(C);
    const P* p = part + c;
    int gi = g0 + w;
    for (; gi + 7 * kFinWaves < G; gi += 8 * kFinWaves) {  // 8 rows (16 loads) in flight per lane
      P fa[8], fb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        fa[k] = p[(gi + kFinWaves * k) * rs];
        fb[k] = p[(gi + kFinWaves * k) * rs + C];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) { a += fa[k]; b += fb[k]; }
    }
    for (; gi < G; gi += kFinWaves) { a += p[gi * rs]; b += p[gi * rs + C]; }
  }
  red[w * 128 + lane] = a;
  red[w * 128 + 64 + lane] = b;
  __syncthreads();
  if (w == 0) {
    double ta = 0.0, tb = 0.0;
#pragma unroll
    for (int k = 0; k < kFinWaves; ++k) { ta += red[k * 128 + lane]; tb += red[k * 128 + 64 + lane]; }
    red[lane] = ta;
    red[64 + lane] = tb;
  }
  __syncthreads();
}

// Row-split pre-pass of a tall slab: block (x, y) reduces rows [y * per, (y + 1) * per) of 64
// channels into fp64 row y of out [S][2C].  One block per 64 channels reading a whole 2048-row
// slab (1 MiB at C = 64) is bound by one CU's load bandwidth (~13 us per backward BN); split over
// S = G / 128 blocks it is a few microseconds, and the finalize then reads S fp64 rows.  The
// summation order is fixed (deterministic).
__global__ void __launch_bounds__(kFinBlock) bn_slab_split_kernel(const float* __restrict__ part, int G, int C,
                                                                  int per, double* __restrict__ out) {
  __shared__ double red[kFinWaves * 128];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g0 = blockIdx.y * per;
  reduce_slab64<float>(part, g0, g0 + per < G ? g0 + per : G, C, c, red);
  if (threadIdx.x < 64 && c < C) {
    out[static_cast<int64_t>(blockIdx.y) * 2 * C + c] = red[threadIdx.x];
    out[static_cast<int64_t>(blockIdx.y) * 2 * C + C + c] = red[64 + threadIdx.x];
  }
}

__device__ __forceinline__ void finalize_channel(int c, int C, double sum, double sumsq,
                                                 double count, const float* w, const float* b,
                                                 float* rmean, float* rvar, float momentum,
                                                 float eps, float* mean_invstd, float* scale_shift) {
  const double mean = sum / count;
  double var = sumsq / count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  const float sc = (w ? w[c] : 1.f) * invstd;
  mean_invstd[c] = static_cast<float>(mean);
  mean_invstd[C + c] = invstd;
  scale_shift[c] = sc;
  scale_shift[C + c] = (b ? b[c] : 0.f) - static_cast<float>(mean) * sc;
  if (rmean) {
    const double unbiased = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * static_cast<float>(mean);
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * static_cast<float>(unbiased);
  }
}

// Shifted moments (S1 = sum d, S2 = sum d^2, d = x - p) -> raw (sum x, sum x^2) in fp64: exact
// up to fp64 rounding, so E[x^2] - mean^2 downstream cancels in fp64, not fp32.
__device__ __forceinline__ void unshift(const float* pivot, int c, double count, double& sum, double& sumsq) {
  if (pivot == nullptr) return;
  const double p = pivot[c], s1 = sum;
  sum = s1 + count * p;
  sumsq = sumsq + 2.0 * p * s1 + count * p * p;
}

// Fused: slab reduce + finalize (+ sums[2C+1] for the backward's count).  ``pivot``: the shift
// of a bn_stats slab (its row G), nullptr for a conv-epilogue slab (raw moments).
template <typename P>
__global__ void __launch_bounds__(kFinBlock) bn_finalize_partials_kernel(
    const P* __restrict__ part, int G, int C, double count, const float* __restrict__ w,
    const float* __restrict__ b, float* __restrict__ rmean, float* __restrict__ rvar,
    int64_t* __restrict__ nbt, float momentum, float eps, float* __restrict__ mean_invstd,
    float* __restrict__ scale_shift, double* __restrict__ sums_out, const float* __restrict__ pivot) {
  __shared__ double red[kFinWaves * 128];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  reduce_slab64<P>(part, 0, G, C, c, red);
  if (threadIdx.x < 64 && c < C) {
    double sum = red[threadIdx.x], sumsq = red[64 + threadIdx.x];
    unshift(pivot, c, count, sum, sumsq);
    if (sums_out) { sums_out[c] = sum; sums_out[C + c] = sumsq; }
    finalize_channel(c, C, sum, sumsq, count, w, b, rmean, rvar, momentum, eps, mean_invstd,
                     scale_shift);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (nbt) nbt[0] += 1;
    if (sums_out) sums_out[2 * C] = count;
  }
}

// SyncBN path, step 1: slab -> fp64 [2C+1] sums (all-reduced by the caller).
template <typename P>
__global__ void __launch_bounds__(kFinBlock) bn_slab_to_sums_kernel(const P* __restrict__ part, int G,
                                                              int C, double count,
                                                              double* __restrict__ sums,
                                                              const float* __restrict__ pivot) {
  __shared__ double red[kFinWaves * 128];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  reduce_slab64<P>(part, 0, G, C, c, red);
  if (threadIdx.x < 64 && c < C) {
    double sum = red[threadIdx.x], sumsq = red[64 + threadIdx.x];
    unshift(pivot, c, count, sum, sumsq);
    sums[c] = sum;
    sums[C + c] = sumsq;
  }
  if (count >= 0 && blockIdx.x == 0 && threadIdx.x == 0) sums[2 * C] = count;
}

// SyncBN path, step 2: finalize from the all-reduced sums.
__global__ void bn_finalize_kernel(const double* __restrict__ sums, int C,
                                   const float* __restrict__ w, const float* __restrict__ b,
                                   float* __restrict__ rmean, float* __restrict__ rvar,
                                   int64_t* __restrict__ nbt, float momentum, float eps,
                                   float* __restrict__ mean_invstd, float* __restrict__ scale_shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) nbt[0] += 1;
  if (c >= C) return;
  finalize_channel(c, C, sums[c], sums[C + c], sums[2 * C], w, b, rmean, rvar, momentum, eps,
                   mean_invstd, scale_shift);
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
template <typename T, int V, int ACT, bool RES, bool BITS = false>
__device__ __forceinline__ void apply_one(const T* __restrict__ x, const T* __restrict__ res,
                                          const float* coef, T* __restrict__ y, int64_t i, int cv,
                                          int C, uint8_t* __restrict__ bits, T* __restrict__ y2, int64_t ld2) {
  const int c0 = static_cast<int>(i % cv) * V;
  const int64_t off = (i / cv) * C + c0;
  float f[V], r[V];
  VecIO<T, V>::load(x + off, f);
  if constexpr (RES) VecIO<T, V>::load(res + off, r);
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    float z = f[j] * coef[c0 + j] + coef[C + c0 + j];
    if constexpr (RES) z += r[j];
    f[j] = act_fwd<ACT>(z);
    if constexpr (BITS) b |= (act_grad_pre<ACT>(1.f, z) != 0.f ? 1u : 0u) << j;
  }
  if (y != nullptr) VecIO<T, V>::store(y + off, f);  // null: the concat slice is the only output
  if (y2 != nullptr) VecIO<T, V>::store(y2 + (i / cv) * ld2 + c0, f);  // the concat-buffer copy
  if constexpr (BITS) bits[i] = static_cast<uint8_t>(b);  // vector i = byte i (off / V)
}

// Channel-stationary form (the channel-vector count cv divides the 256-thread block, i.e. C / V
// is a power of two <= 256, every DDRNet / ResNet width): the grid stride is a whole number of
// rows, so a thread keeps ONE channel vector for all its rows -- its per-channel coefficients
// live in registers (no per-element LDS reads: with 32 or 64 distinct channel vectors per wave
// those were 4-8-way bank-conflicted) and the row index advances by a constant (no 64-bit
// division per vector).
template <typename T, int V, int ACT, bool RES, bool BITS>
__device__ __forceinline__ void apply_rows(const T* __restrict__ x, const T* __restrict__ res,
                                           const float* __restrict__ scale_shift, T* __restrict__ y,
                                           int64_t M, int C, uint8_t* __restrict__ bits, T* __restrict__ y2,
                                           int64_t ld2, bool rev) {
  const int cv = C / V;
  const int cvi = threadIdx.x % cv;
  const int c0 = cvi * V;
  float sc[V], sh[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { sc[j] = scale_shift[c0 + j]; sh[j] = scale_shift[C + c0 + j]; }
  const int64_t rstep = static_cast<int64_t>(gridDim.x) * (blockDim.x / cv);
  auto one = [&](int64_t row) {
    if (rev) row = M - 1 - row;
    const int64_t off = row * C + c0;
    float f[V], r[V];
    VecIO<T, V>::load(x + off, f);
    if constexpr (RES) VecIO<T, V>::load(res + off, r);
    uint32_t b = 0;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float z = fmaf(f[j], sc[j], sh[j]);
      if constexpr (RES) z += r[j];
      f[j] = act_fwd<ACT>(z);
      if constexpr (BITS) b |= (act_grad_pre<ACT>(1.f, z) != 0.f ? 1u : 0u) << j;
    }
    if (y != nullptr) VecIO<T, V>::store(y + off, f);
    if (y2 != nullptr) VecIO<T, V>::store(y2 + row * ld2 + c0, f);
    if constexpr (BITS) bits[row * cv + cvi] = static_cast<uint8_t>(b);
  };
  int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x / cv) + threadIdx.x / cv;
  for (; row + rstep < M; row += 2 * rstep) {  // two rows in flight per thread
    one(row);
    one(row + rstep);
  }
  if (row < M) one(row);
}

template <typename T, int V, int ACT, bool RES, bool BITS = false>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ res,
                                                       const float* __restrict__ scale_shift,
                                                       T* __restrict__ y, int64_t M, int C,
                                                       uint8_t* __restrict__ bits = nullptr,
                                                       T* __restrict__ y2 = nullptr, int64_t ld2 = 0,
                                                       bool rev = false) {
  if (blockDim.x % (C / V) == 0) {  // block-uniform
    apply_rows<T, V, ACT, RES, BITS>(x, res, scale_shift, y, M, C, bits, y2, ld2, rev);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [2][C]
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) coef[c] = scale_shift[c];
  __syncthreads();
  const int cv = C / V;
  const int64_t total = M * cv;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  for (; i + stride < total; i += 2 * stride) {  // two vectors in flight per thread
    apply_one<T, V, ACT, RES, BITS>(x, res, coef, y, i, cv, C, bits, y2, ld2);
    apply_one<T, V, ACT, RES, BITS>(x, res, coef, y, i + stride, cv, C, bits, y2, ld2);
  }
  if (i < total) apply_one<T, V, ACT, RES, BITS>(x, res, coef, y, i, cv, C, bits, y2, ld2);
}

// ----------------------------------------------------------- backward -------
// g = dy (+ dy2: a channel slice of a wider channels-last gradient, row stride ld2 -- the concat
// buffer's gradient handed over by ops/concat.py; dy may then be null)
template <typename T, int V>
__device__ __forceinline__ void load_dy(const T* dy, const T* dy2, int64_t off, int64_t off2, float* g) {
  if (dy != nullptr) {
    VecIO<T, V>::load(dy + off, g);
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = 0.f;
  }
  if (dy2 != nullptr) {
    float h[V];
    VecIO<T, V>::load(dy2 + off2, h);
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] += h[j];
  }
}

template <typename T, int V, int ACT, int MASK>
__device__ __forceinline__ void load_g(const T* dy, const T* dy2, const T* x, const T* y, const float* coef, int C,
                                       int64_t off, int64_t off2, int c0, float* g, float* xv) {
  load_dy<T, V>(dy, dy2, off, off2, g);
  VecIO<T, V>::load(x + off, xv);
  if constexpr (MASK == kMaskFromY) {
    float yv[V];
    VecIO<T, V>::load(y + off, yv);
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = act_bwd_from_out<ACT>(g[j], yv[j]);
  } else if constexpr (MASK == kMaskFromX) {
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = act_grad_pre<ACT>(g[j], xv[j] * coef[c0 + j] + coef[C + c0 + j]);
  } else if constexpr (MASK == kMaskBits) {
    // off = row * C + c0 with V | C and V | c0: the vector index is off / V
    const uint32_t b = reinterpret_cast<const uint8_t*>(y)[off / V];
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = ((b >> j) & 1u) ? g[j] : 0.f;
  }
}

// slab[G][0:C] = sum g, slab[G][C:2C] = sum g * (x - mean)
template <typename T, int V, int ACT, int MASK>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean_invstd, const float* __restrict__ scale_shift, int64_t M, int C,
    float* __restrict__ part, const T* __restrict__ dy2, int64_t ld2, int order) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // coef[2C] | mean[C] | partials
  float* coef = sm;
  float* mu = sm + 2 * C;
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) coef[c] = scale_shift[c];
  for (int c = threadIdx.x; c < C; c += blockDim.x) mu[c] = mean_invstd[c];
  __syncthreads();
  const RowGeo g(C, V);
  const int c0 = g.my_cv * V;
  float s[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (g.my_r < g.rpi) {
    float m[V];
#pragma unroll
    for (int j = 0; j < V; ++j) m[j] = mu[c0 + j];
    auto acc4 = [&](int64_t ra, int64_t rb, int64_t rc, int64_t rd) {  // four rows (8-12 loads) in flight
      float ga[V], xa[V], gb[V], xb[V], gc[V], xc[V], gd[V], xd[V];
      load_g<T, V, ACT, MASK>(dy, dy2, x, y, coef, C, ra * C + c0, ra * ld2 + c0, c0, ga, xa);
      load_g<T, V, ACT, MASK>(dy, dy2, x, y, coef, C, rb * C + c0, rb * ld2 + c0, c0, gb, xb);
      load_g<T, V, ACT, MASK>(dy, dy2, x, y, coef, C, rc * C + c0, rc * ld2 + c0, c0, gc, xc);
      load_g<T, V, ACT, MASK>(dy, dy2, x, y, coef, C, rd * C + c0, rd * ld2 + c0, c0, gd, xd);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        s[j] += (ga[j] + gb[j]) + (gc[j] + gd[j]);
        q[j] += (ga[j] * (xa[j] - m[j]) + gb[j] * (xb[j] - m[j])) +
                (gc[j] * (xc[j] - m[j]) + gd[j] * (xd[j] - m[j]));
      }
    };
    auto acc1 = [&](int64_t r) {
      float ga[V], xa[V];
      load_g<T, V, ACT, MASK>(dy, dy2, x, y, coef, C, r * C + c0, r * ld2 + c0, c0, ga, xa);
#pragma unroll
      for (int j = 0; j < V; ++j) { s[j] += ga[j]; q[j] += ga[j] * (xa[j] - m[j]); }
    };
    if (order == 0) {  // block-contiguous row ranges
      int64_t r0, r1;
      block_rows(M, g.rpi, r0, r1);
      int64_t r = r0 + g.my_r;
      for (; r + 3 * g.rpi < r1; r += 4 * g.rpi) acc4(r, r + g.rpi, r + 2 * g.rpi, r + 3 * g.rpi);
      for (; r < r1; r += g.rpi) acc1(r);
    } else {  // grid-stride sweep over the whole tensor, from the last row down (order 1) or up (2)
      const int64_t S = static_cast<int64_t>(gridDim.x) * g.rpi;
      const int64_t e = order == 1 ? M - 1 : 0, d = order == 1 ? -1 : 1;
      int64_t v = static_cast<int64_t>(blockIdx.x) * g.rpi + g.my_r;
      for (; v + 3 * S < M; v += 4 * S) acc4(e + d * v, e + d * (v + S), e + d * (v + 2 * S), e + d * (v + 3 * S));
      for (; v < M; v += S) acc1(e + d * v);
    }
  }
  __syncthreads();  // coef/mu region is reused below only after every thread is done
  block_partials_out<V>(s, q, g, C, sm + 3 * C, part);
}

__device__ __forceinline__ void bwd_finalize_channel(int c, int C, double sg, double sgx,
                                                     double count, const float* w,
                                                     const float* mean_invstd, int batch_stats,
                                                     float* kcoef, float* dw, float* db) {
  const float invstd = mean_invstd[C + c];
  if (dw) dw[c] = static_cast<float>(sgx * invstd);
  if (db) db[c] = static_cast<float>(sg);
  kcoef[c] = (w ? w[c] : 1.f) * invstd;
  if (batch_stats) {
    kcoef[C + c] = static_cast<float>(sg / count);
    kcoef[2 * C + c] = static_cast<float>(sgx / count) * invstd * invstd;
  } else {
    kcoef[C + c] = 0.f;
    kcoef[2 * C + c] = 0.f;
  }
}

// Slab (or already-reduced sums, SyncBN) -> dx coefficients + parameter grads.
template <typename P>
__global__ void __launch_bounds__(kFinBlock) bn_bwd_finalize_kernel(
    const P* __restrict__ part, int G, const double* __restrict__ sums,
    const double* __restrict__ count_ptr, int C, const float* __restrict__ w,
    const float* __restrict__ mean_invstd, int batch_stats, float* __restrict__ kcoef,
    float* __restrict__ dw, float* __restrict__ db) {
  __shared__ double red[kFinWaves * 128];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (!sums) reduce_slab64<P>(part, 0, G, C, c, red);
  if (threadIdx.x < 64 && c < C) {
    const double sg = sums ? sums[c] : red[threadIdx.x];
    const double sgx = sums ? sums[C + c] : red[64 + threadIdx.x];
    const double count = count_ptr ? *count_ptr : 1.0;
    bwd_finalize_channel(c, C, sg, sgx, count, w, mean_invstd, batch_stats, kcoef, dw, db);
  }
}

template <typename T, int V, int ACT, int MASK, bool DRES>
__device__ __forceinline__ void bwd_apply_one(const T* dy, const T* x, const T* y, const float* coef,
                                              const float* mu, const float* k, T* dx, T* dres,
                                              int64_t i, int cv, int C, const T* dy2, int64_t ld2) {
  const int c0 = static_cast<int>(i % cv) * V;
  const int64_t off = (i / cv) * C + c0;
  float g[V], xv[V], o[V];
  load_g<T, V, ACT, MASK>(dy, dy2, x, y, coef, C, off, (i / cv) * ld2 + c0, c0, g, xv);
  if constexpr (DRES) VecIO<T, V>::store(dres + off, g);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = c0 + j;
    o[j] = k[c] * (g[j] - k[C + c] - (xv[j] - mu[c]) * k[2 * C + c]);
  }
  VecIO<T, V>::store(dx + off, o);
}

// Channel-stationary backward apply (see apply_rows): dx = k0 * (g - k1 - (x - mean) * k2) with
// the per-channel k0, k1, k2, mean held in registers (x - mean first, as in bwd_apply_one: no
// cancellation between separately rounded k2*x and k2*mean terms).
template <typename T, int V, int ACT, int MASK, bool DRES>
__device__ __forceinline__ void bwd_apply_rows(const T* __restrict__ dy, const T* __restrict__ x,
                                               const T* __restrict__ y, const float* __restrict__ mean_invstd,
                                               const float* __restrict__ scale_shift,
                                               const float* __restrict__ kcoef, T* __restrict__ dx,
                                               T* __restrict__ dres, int64_t M, int C,
                                               const T* __restrict__ dy2, int64_t ld2, bool rev) {
  const int cv = C / V;
  const int c0 = (threadIdx.x % cv) * V;
  float cf[2 * V], k0[V], k1[V], k2[V], mu[V];  // cf: scale | shift (pre-activation mask)
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = c0 + j;
    k0[j] = kcoef[c];
    k1[j] = kcoef[C + c];
    k2[j] = kcoef[2 * C + c];
    mu[j] = mean_invstd[c];
    cf[j] = scale_shift[c];
    cf[V + j] = scale_shift[C + c];
  }
  const int64_t rstep = static_cast<int64_t>(gridDim.x) * (blockDim.x / cv);
  auto one = [&](int64_t row) {
    if (rev) row = M - 1 - row;
    const int64_t off = row * C + c0;
    float g[V], xv[V], o[V];
    load_dy<T, V>(dy, dy2, off, row * ld2 + c0, g);
    VecIO<T, V>::load(x + off, xv);
    if constexpr (MASK == kMaskFromY) {
      float yv[V];
      VecIO<T, V>::load(y + off, yv);
#pragma unroll
      for (int j = 0; j < V; ++j) g[j] = act_bwd_from_out<ACT>(g[j], yv[j]);
    } else if constexpr (MASK == kMaskFromX) {
#pragma unroll
      for (int j = 0; j < V; ++j) g[j] = act_grad_pre<ACT>(g[j], fmaf(xv[j], cf[j], cf[V + j]));
    } else if constexpr (MASK == kMaskBits) {
      const uint32_t b = reinterpret_cast<const uint8_t*>(y)[off / V];
#pragma unroll
      for (int j = 0; j < V; ++j) g[j] = ((b >> j) & 1u) ? g[j] : 0.f;
    }
    if constexpr (DRES) VecIO<T, V>::store(dres + off, g);
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = k0[j] * (g[j] - k1[j] - (xv[j] - mu[j]) * k2[j]);
    VecIO<T, V>::store(dx + off, o);
  };
  int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x / cv) + threadIdx.x / cv;
  for (; row + rstep < M; row += 2 * rstep) {
    one(row);
    one(row + rstep);
  }
  if (row < M) one(row);
}

template <typename T, int V, int ACT, int MASK, bool DRES>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean_invstd, const float* __restrict__ scale_shift,
    const float* __restrict__ kcoef, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C,
    const T* __restrict__ dy2, int64_t ld2, bool rev) {
  if (blockDim.x % (C / V) == 0) {  // block-uniform
    bwd_apply_rows<T, V, ACT, MASK, DRES>(dy, x, y, mean_invstd, scale_shift, kcoef, dx, dres, M, C, dy2, ld2, rev);
    return;
  }
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
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  for (; i + stride < total; i += 2 * stride) {
    bwd_apply_one<T, V, ACT, MASK, DRES>(dy, x, y, coef, mu, k, dx, dres, i, cv, C, dy2, ld2);
    bwd_apply_one<T, V, ACT, MASK, DRES>(dy, x, y, coef, mu, k, dx, dres, i + stride, cv, C, dy2, ld2);
  }
  if (i < total) bwd_apply_one<T, V, ACT, MASK, DRES>(dy, x, y, coef, mu, k, dx, dres, i, cv, C, dy2, ld2);
}

// ------------------------------------------ odd channel counts: flat chunks ---
// An odd C (the 19-class heads of the 11 DeConvBNAct models, whose BN runs at full resolution)
// has channel vectors of ONE element: 2-byte loads, a quarter of the bandwidth of the 16-byte
// path.  Here the [M, C] tensor is walked as flat 16-byte chunks instead (E = 16 / sizeof(T)
// elements; element e has channel e % C).  The grid has a multiple of C threads, so a thread
// that starts at chunk t and strides by the thread count always sees the same E channels
// ((E * t + j) % C): its coefficients and partial sums stay in registers ("phase-stationary"),
// exactly like the channel-stationary kernels above.  Partial sums: one [2C] slab row per block,
// each channel summed over the block's (thread, element) slots in a fixed order (deterministic).
template <typename T>
struct Flat {
  static constexpr int E = 16 / static_cast<int>(sizeof(T));
  int64_t n_el, n_chunks, nthreads, t;
  int ch[E];
  __device__ __forceinline__ Flat(int64_t M, int C) {
    n_el = M * C;
    n_chunks = n_el / E;
    nthreads = static_cast<int64_t>(gridDim.x) * blockDim.x;
    t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int base = static_cast<int>((E * t) % C);
#pragma unroll
    for (int j = 0; j < E; ++j) ch[j] = (base + j) % C;
  }
  // the thread that owns the partial last chunk (n_el % E trailing elements), if any
  __device__ __forceinline__ bool owns_tail() const {
    return n_chunks * E < n_el && t == n_chunks % nthreads;
  }
};

// block partials of the phase-stationary layout -> one slab row: sum of slots f (= thread * E +
// element) with (E * blockIdx.x * blockDim.x + f) % C == c, in increasing f
template <int E>
__device__ __forceinline__ void flat_partials_out(const float* s, const float* q, int C, float* __restrict__ part) {
  __shared__ float red[2][256 * E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    red[0][threadIdx.x * E + j] = s[j];
    red[1][threadIdx.x * E + j] = q[j];
  }
  __syncthreads();
  const int b0 = static_cast<int>((static_cast<int64_t>(E) * blockIdx.x * blockDim.x) % C);
  const int nslot = blockDim.x * E;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double a = 0.0, b = 0.0;
    for (int f = ((c - b0) % C + C) % C; f < nslot; f += C) { a += red[0][f]; b += red[1][f]; }
    part[static_cast<int64_t>(blockIdx.x) * 2 * C + c] = static_cast<float>(a);
    part[static_cast<int64_t>(blockIdx.x) * 2 * C + C + c] = static_cast<float>(b);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_stats_flat_kernel(const T* __restrict__ x, int64_t M, int C,
                                                            float* __restrict__ part, int shift) {
  constexpr int E = Flat<T>::E;
  const Flat<T> fl(M, C);
  // shifted, compensated moments about the sampled pivot (see bn_stats_kernel)
  float s[E], q[E], pv[E], cmp[E];
  auto pivot = [&](int c) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = to_f<T>(x[((2 * k + 1) * M / 16) * C + c]);
    return (((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]))) * 0.125f;
  };
#pragma unroll
  for (int j = 0; j < E; ++j) { s[j] = 0.f; q[j] = 0.f; cmp[j] = 0.f; pv[j] = shift ? pivot(fl.ch[j]) : 0.f; }
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x)
      part[static_cast<int64_t>(gridDim.x) * 2 * C + c] = shift ? pivot(c) : 0.f;
  }
  auto acc = [&](const float* f) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float d = f[j] - pv[j];
      two_sum_acc(s[j], cmp[j], d);
      q[j] = fmaf(d, d, q[j]);
    }
  };
  int64_t i = fl.t;
  for (; i + fl.nthreads < fl.n_chunks; i += 2 * fl.nthreads) {
    float a[E], b[E];
    VecIO<T, E>::load(x + i * E, a);
    VecIO<T, E>::load(x + (i + fl.nthreads) * E, b);
    acc(a);
    acc(b);
  }
  if (i < fl.n_chunks) {
    float a[E];
    VecIO<T, E>::load(x + i * E, a);
    acc(a);
  }
  if (fl.owns_tail()) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int64_t e = fl.n_chunks * E + j;
      if (e < fl.n_el) {
        const float v = to_f<T>(x[e]) - pv[j];
        two_sum_acc(s[j], cmp[j], v);
        q[j] = fmaf(v, v, q[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < E; ++j) s[j] += cmp[j];
  flat_partials_out<E>(s, q, C, part);
}

template <typename T, int ACT, bool RES, bool BITS>
__global__ void __launch_bounds__(256) bn_apply_flat_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                            const float* __restrict__ scale_shift, T* __restrict__ y,
                                                            int64_t M, int C, uint8_t* __restrict__ bits) {
  constexpr int E = Flat<T>::E;
  const Flat<T> fl(M, C);
  float sc[E], sh[E];
#pragma unroll
  for (int j = 0; j < E; ++j) { sc[j] = scale_shift[fl.ch[j]]; sh[j] = scale_shift[C + fl.ch[j]]; }
  auto val = [&](int j, float f, float r, uint32_t& b) {
    float z = fmaf(f, sc[j], sh[j]);
    if constexpr (RES) z += r;
    if constexpr (BITS) b |= (act_grad_pre<ACT>(1.f, z) != 0.f ? 1u : 0u) << (8 * (j & 3));
    return act_fwd<ACT>(z);
  };
  auto one = [&](int64_t i) {
    float f[E], r[E];
    VecIO<T, E>::load(x + i * E, f);
    if constexpr (RES) VecIO<T, E>::load(res + i * E, r);
    uint32_t b[2] = {0u, 0u};  // one byte per element (channel vectors of one element)
#pragma unroll
    for (int j = 0; j < E; ++j) f[j] = val(j, f[j], RES ? r[j] : 0.f, b[j >> 2]);
    VecIO<T, E>::store(y + i * E, f);
    if constexpr (BITS) {
      if constexpr (E == 8) *reinterpret_cast<uint2*>(bits + i * E) = make_uint2(b[0], b[1]);
      else *reinterpret_cast<uint32_t*>(bits + i * E) = b[0];
    }
  };
  int64_t i = fl.t;
  for (; i + fl.nthreads < fl.n_chunks; i += 2 * fl.nthreads) {
    one(i);
    one(i + fl.nthreads);
  }
  if (i < fl.n_chunks) one(i);
  if (fl.owns_tail()) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int64_t e = fl.n_chunks * E + j;
      if (e < fl.n_el) {
        uint32_t b = 0u;
        y[e] = from_f<T>(val(j, to_f<T>(x[e]), RES ? to_f<T>(res[e]) : 0.f, b));
        if constexpr (BITS) bits[e] = static_cast<uint8_t>(b >> (8 * (j & 3)));
      }
    }
  }
}

// activation-masked gradient of element j (value g) given x (and y / the bit byte)
template <typename T, int ACT, int MASK>
__device__ __forceinline__ float flat_mask(float g, float xv, const T* y, int64_t e, float sc, float sh) {
  if constexpr (MASK == kMaskFromY) return act_bwd_from_out<ACT>(g, to_f<T>(y[e]));
  else if constexpr (MASK == kMaskFromX) return act_grad_pre<ACT>(g, fmaf(xv, sc, sh));
  else if constexpr (MASK == kMaskBits) return reinterpret_cast<const uint8_t*>(y)[e] ? g : 0.f;
  else return g;
}

template <typename T, int ACT, int MASK>
__global__ void __launch_bounds__(256) bn_bwd_reduce_flat_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean_invstd, const float* __restrict__ scale_shift, int64_t M, int C,
    float* __restrict__ part) {
  constexpr int E = Flat<T>::E;
  const Flat<T> fl(M, C);
  float m[E], sc[E], sh[E], s[E], q[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    m[j] = mean_invstd[fl.ch[j]];
    sc[j] = scale_shift[fl.ch[j]];
    sh[j] = scale_shift[C + fl.ch[j]];
    s[j] = 0.f;
    q[j] = 0.f;
  }
  auto one = [&](int64_t i) {
    float g[E], xv[E];
    VecIO<T, E>::load(dy + i * E, g);
    VecIO<T, E>::load(x + i * E, xv);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float gm = flat_mask<T, ACT, MASK>(g[j], xv[j], y, i * E + j, sc[j], sh[j]);
      s[j] += gm;
      q[j] = fmaf(gm, xv[j] - m[j], q[j]);
    }
  };
  int64_t i = fl.t;
  for (; i + fl.nthreads < fl.n_chunks; i += 2 * fl.nthreads) {
    one(i);
    one(i + fl.nthreads);
  }
  if (i < fl.n_chunks) one(i);
  if (fl.owns_tail()) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int64_t e = fl.n_chunks * E + j;
      if (e < fl.n_el) {
        const float xv = to_f<T>(x[e]);
        const float gm = flat_mask<T, ACT, MASK>(to_f<T>(dy[e]), xv, y, e, sc[j], sh[j]);
        s[j] += gm;
        q[j] = fmaf(gm, xv - m[j], q[j]);
      }
    }
  }
  flat_partials_out<E>(s, q, C, part);
}

template <typename T, int ACT, int MASK, bool DRES>
__global__ void __launch_bounds__(256) bn_bwd_apply_flat_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean_invstd, const float* __restrict__ scale_shift,
    const float* __restrict__ kcoef, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C) {
  constexpr int E = Flat<T>::E;
  const Flat<T> fl(M, C);
  float k0[E], k1[E], k2[E], mu[E], sc[E], sh[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int c = fl.ch[j];
    k0[j] = kcoef[c];
    k1[j] = kcoef[C + c];
    k2[j] = kcoef[2 * C + c];
    mu[j] = mean_invstd[c];
    sc[j] = scale_shift[c];
    sh[j] = scale_shift[C + c];
  }
  auto one = [&](int64_t i) {
    float g[E], xv[E], o[E];
    VecIO<T, E>::load(dy + i * E, g);
    VecIO<T, E>::load(x + i * E, xv);
#pragma unroll
    for (int j = 0; j < E; ++j) g[j] = flat_mask<T, ACT, MASK>(g[j], xv[j], y, i * E + j, sc[j], sh[j]);
    if constexpr (DRES) VecIO<T, E>::store(dres + i * E, g);
#pragma unroll
    for (int j = 0; j < E; ++j) o[j] = k0[j] * (g[j] - k1[j] - (xv[j] - mu[j]) * k2[j]);
    VecIO<T, E>::store(dx + i * E, o);
  };
  int64_t i = fl.t;
  for (; i + fl.nthreads < fl.n_chunks; i += 2 * fl.nthreads) {
    one(i);
    one(i + fl.nthreads);
  }
  if (i < fl.n_chunks) one(i);
  if (fl.owns_tail()) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int64_t e = fl.n_chunks * E + j;
      if (e < fl.n_el) {
        const float xv = to_f<T>(x[e]);
        const float g = flat_mask<T, ACT, MASK>(to_f<T>(dy[e]), xv, y, e, sc[j], sh[j]);
        if constexpr (DRES) dres[e] = from_f<T>(g);
        dx[e] = from_f<T>(k0[j] * (g - k1[j] - (xv - mu[j]) * k2[j]));
      }
    }
  }
}

// ------------------------------------------------------------ launchers -----
// Channel-vector width: the widest of {16 B, 8 B, 4 B, 1 element} that divides C
// with at most 256 vectors per row (fp16 keeps the 16-byte path only).
int bn_vec_width(int dtype, int C) {
  if (dtype == kF16) return (C % 8 == 0 && C / 8 <= 256) ? 8 : 0;
  for (int v = dtype == kF32 ? 4 : 8; v >= 1; v >>= 1)
    if (C % v == 0 && C / v <= 256) return v;
  return 0;
}

// odd channel counts take the flat, phase-stationary kernels (grids: multiples of C threads' blocks)
static bool bn_flat(int dtype, int C) { return dtype != kF16 && C >= 3 && (C & 1) && bn_vec_width(dtype, C) == 1; }

static int64_t round_up_to(int64_t g, int m) { return (g + m - 1) / m * m; }

// Grid caps of the streaming passes (RTSEG_BN_APPLY_CAP / RTSEG_BN_REDUCE_CAP: A/B of the
// block counts, tools/bench_bn_bw.py; read once)
static int64_t env_cap(const char* name, int64_t dflt) {
  const char* v = std::getenv(name);
  const long long x = v ? std::atoll(v) : 0;
  return x > 0 ? x : dflt;
}

int bn_partial_grid(int64_t M, int C, int dtype) {
  if (bn_flat(dtype, C)) {  // ~16 chunks per thread, <= ~1024 blocks, a multiple of C blocks
    const int64_t chunks = M * C / (dtype == kF32 ? 4 : 8);
    int64_t g = (chunks + 256 * 16 - 1) / (256 * 16);
    g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
    return static_cast<int>(round_up_to(g, C));
  }
  const int V = bn_vec_width(dtype, C);
  const int rpi = 256 / (C / V);
  int64_t g = (M + static_cast<int64_t>(rpi) * 32 - 1) / (static_cast<int64_t>(rpi) * 32);
  // 4 blocks (16 waves) per CU: with 4 rows (8 x 16-B loads) in flight per lane that keeps
  // ~64 KiB of reads outstanding per CU, what HBM3E latency x bandwidth needs
  // cap 2048 (8 blocks per CU): the backward reduce of the 537 MB / 268 MB / 134 MB DDRNet-23 layers
  // 925 -> 769 / 255 -> 233 / 135 -> 127 us vs 1024 (profiles/r5_bn_caps)
  static const int64_t cap = env_cap("RTSEG_BN_REDUCE_CAP", 2048);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

// Calls F.template operator()<T, V>() for the (dtype, width) of this layer.
template <typename F>
static void with_tv(int dtype, int C, F&& f) {
  const int v = bn_vec_width(dtype, C);
  if (dtype == kF32) {
    if (v == 4) f.template operator()<float, 4>();
    else if (v == 2) f.template operator()<float, 2>();
    else f.template operator()<float, 1>();
  } else if (dtype == kBF16) {
    if (v == 8) f.template operator()<uint16_t, 8>();
    else if (v == 4) f.template operator()<uint16_t, 4>();
    else if (v == 2) f.template operator()<uint16_t, 2>();
    else f.template operator()<uint16_t, 1>();
  } else {
    f.template operator()<_Float16, 8>();
  }
}

void launch_bn_stats(const void* x, int dtype, int64_t M, int C, float* part, int G,
                     hipStream_t st, bool shift) {
  const int sh = shift ? 1 : 0;
  if (bn_flat(dtype, C)) {  // G (bn_partial_grid) is a multiple of C
    if (dtype == kF32) bn_stats_flat_kernel<float><<<G, 256, 0, st>>>(static_cast<const float*>(x), M, C, part, sh);
    else bn_stats_flat_kernel<uint16_t><<<G, 256, 0, st>>>(static_cast<const uint16_t*>(x), M, C, part, sh);
    return;
  }
  with_tv(dtype, C, [&]<typename T, int V>() {
    const int rpi = 256 / (C / V);
    const size_t lds = sizeof(float) * 2 * rpi * C;
    bn_stats_kernel<T, V><<<G, 256, lds, st>>>(static_cast<const T*>(x), M, C, part, sh);
  });
}

constexpr int kSplitRows = 128;

// RTSEG_BN_SPLIT=0: off (A/B)
int bn_slab_splits(int G) {
  static const bool on = [] {
    const char* e = std::getenv("RTSEG_BN_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on && G >= 4 * kSplitRows ? (G + kSplitRows - 1) / kSplitRows : 1;
}

// scratch (bn_slab_splits(G) * 2C doubles, or nullptr): the row-split pre-pass, then F(fp64 rows, S);
// else F(the slab, G)
template <typename F>
static void with_split(const float* part, int G, int C, double* scratch, hipStream_t st, F&& f) {
  const int S = bn_slab_splits(G);
  if (scratch == nullptr || S <= 1 || part == nullptr) {
    f(part, G);
    return;
  }
  bn_slab_split_kernel<<<dim3((C + 63) / 64, S), kFinBlock, 0, st>>>(part, G, C, kSplitRows, scratch);
  f(static_cast<const double*>(scratch), S);
}

void launch_bn_finalize_partials(const float* part, int G, int C, double count, const float* w,
                                 const float* b, float* rmean, float* rvar, int64_t* nbt,
                                 float momentum, float eps, float* mean_invstd, float* scale_shift,
                                 double* sums_out, hipStream_t st, const float* pivot, double* scratch) {
  with_split(part, G, C, scratch, st, [&](const auto* p, int g) {
    using P = std::remove_cv_t<std::remove_pointer_t<decltype(p)>>;
    bn_finalize_partials_kernel<P><<<(C + 63) / 64, kFinBlock, 0, st>>>(p, g, C, count, w, b, rmean, rvar, nbt,
                                                                     momentum, eps, mean_invstd, scale_shift,
                                                                     sums_out, pivot);
  });
}

void launch_bn_slab_to_sums(const float* part, int G, int C, double count, double* sums,
                            hipStream_t st, const float* pivot, double* scratch) {
  with_split(part, G, C, scratch, st, [&](const auto* p, int g) {
    using P = std::remove_cv_t<std::remove_pointer_t<decltype(p)>>;
    bn_slab_to_sums_kernel<P><<<(C + 63) / 64, kFinBlock, 0, st>>>(p, g, C, count, sums, pivot);
  });
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

// Traversal order of the streaming passes, for reuse through the 256 MiB Infinity Cache: a pass
// that starts where the previous pass over the same tensors ended re-reads what that pass left
// resident.  RTSEG_BN_L3ORDER bits: 1 = backward reduce sweeps down from the last row, 2 = it sweeps
// up grid-stride (neither: block-contiguous ranges), 4 = backward apply from the last row,
// 8 = forward apply from the last row (its input's tail is what the producing conv wrote last).
// Default 14: the reduce ends at the tail of (dy, x), the backward apply starts there.  DDRNet-23
// b32 1024x2048: 537.2 (order 0) -> 543.0 images/s (profiles/r5_l3order).  Read once.
static int l3_order() {
  static const int v = [] {
    const char* e = std::getenv("RTSEG_BN_L3ORDER");
    return e ? std::atoi(e) : 14;
  }();
  return v;
}

static int apply_grid(int64_t work) {
  int64_t g = (work + 511) / 512;  // two vectors per thread
  // cap 1024 (4 blocks per CU): forward apply / backward apply of the 537 MB layer 906 -> 859 / 2209 ->
  // 2124 us, residual + bit-mask variants 3-7 % faster than at 2048 (profiles/r5_bn_caps)
  static const int64_t cap = env_cap("RTSEG_BN_APPLY_CAP", 1024);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

// flat kernels: a multiple of C blocks (so of C threads), ~2 chunks per thread up to 2048 blocks
static int flat_grid(int64_t M, int C, int dtype) {
  return static_cast<int>(round_up_to(apply_grid(M * C / (dtype == kF32 ? 4 : 8)), C));
}

template <typename T, int ACT>
static void apply_flat_t(const void* x, const void* res, const float* ss, void* y, uint8_t* bits, int64_t M,
                         int C, int dtype, hipStream_t st) {
  const int g = flat_grid(M, C, dtype);
  const T* xp = static_cast<const T*>(x);
  const T* rp = static_cast<const T*>(res);
  T* yp = static_cast<T*>(y);
  if (res != nullptr && bits != nullptr) bn_apply_flat_kernel<T, ACT, true, true><<<g, 256, 0, st>>>(xp, rp, ss, yp, M, C, bits);
  else if (res != nullptr) bn_apply_flat_kernel<T, ACT, true, false><<<g, 256, 0, st>>>(xp, rp, ss, yp, M, C, bits);
  else if (bits != nullptr) bn_apply_flat_kernel<T, ACT, false, true><<<g, 256, 0, st>>>(xp, rp, ss, yp, M, C, bits);
  else bn_apply_flat_kernel<T, ACT, false, false><<<g, 256, 0, st>>>(xp, rp, ss, yp, M, C, bits);
}

template <int ACT>
static void apply_flat(const void* x, const void* res, const float* ss, void* y, uint8_t* bits, int64_t M, int C,
                       int dtype, hipStream_t st) {
  if (dtype == kF32) apply_flat_t<float, ACT>(x, res, ss, y, bits, M, C, dtype, st);
  else apply_flat_t<uint16_t, ACT>(x, res, ss, y, bits, M, C, dtype, st);
}

template <typename T, int V, int ACT>
static void apply_t(const void* x, const void* res, const float* ss, void* y, int64_t M, int C,
                    hipStream_t st, void* y2, int64_t ld2) {
  const int64_t work = M * (C / V);
  const size_t lds = sizeof(float) * 2 * C;
  const int grid = apply_grid(work);
  if (res)
    bn_apply_kernel<T, V, ACT, true><<<grid, 256, lds, st>>>(
        static_cast<const T*>(x), static_cast<const T*>(res), ss, static_cast<T*>(y), M, C, nullptr,
        static_cast<T*>(y2), ld2, (l3_order() & 8) != 0);
  else
    bn_apply_kernel<T, V, ACT, false><<<grid, 256, lds, st>>>(
        static_cast<const T*>(x), nullptr, ss, static_cast<T*>(y), M, C, nullptr, static_cast<T*>(y2), ld2,
        (l3_order() & 8) != 0);
}

template <typename T, int V, int ACT>
static void apply_bits_t(const void* x, const void* res, const float* ss, void* y, uint8_t* bits,
                         int64_t M, int C, hipStream_t st, void* y2, int64_t ld2) {
  const int64_t work = M * (C / V);
  if (res != nullptr)
    bn_apply_kernel<T, V, ACT, true, true><<<apply_grid(work), 256, sizeof(float) * 2 * C, st>>>(
        static_cast<const T*>(x), static_cast<const T*>(res), ss, static_cast<T*>(y), M, C, bits,
        static_cast<T*>(y2), ld2, (l3_order() & 8) != 0);
  else
    bn_apply_kernel<T, V, ACT, false, true><<<apply_grid(work), 256, sizeof(float) * 2 * C, st>>>(
        static_cast<const T*>(x), nullptr, ss, static_cast<T*>(y), M, C, bits, static_cast<T*>(y2), ld2,
        (l3_order() & 8) != 0);
}

// (Residual +) activation forward that also writes the derivative bit mask (kMaskBits):
// bits holds M * C / V bytes, V = bn_vec_width(dtype, C).
void launch_bn_apply_bits(const void* x, const void* res, const float* scale_shift, void* y,
                          uint8_t* bits, int dtype, int64_t M, int C, int act, hipStream_t st, void* y2,
                          int64_t ld2) {
  if (bn_flat(dtype, C)) {
    if (act == kActReLU6) apply_flat<kActReLU6>(x, res, scale_shift, y, bits, M, C, dtype, st);
    else apply_flat<kActReLU>(x, res, scale_shift, y, bits, M, C, dtype, st);
    return;
  }
  with_tv(dtype, C, [&]<typename T, int V>() {
    if (act == kActReLU6) apply_bits_t<T, V, kActReLU6>(x, res, scale_shift, y, bits, M, C, st, y2, ld2);
    else apply_bits_t<T, V, kActReLU>(x, res, scale_shift, y, bits, M, C, st, y2, ld2);
  });
}

void launch_bn_apply(const void* x, const void* res, const float* scale_shift, void* y, int dtype,
                     int64_t M, int C, int act, hipStream_t st, void* y2, int64_t ld2) {
  if (bn_flat(dtype, C)) {
    if (act == kActReLU) apply_flat<kActReLU>(x, res, scale_shift, y, nullptr, M, C, dtype, st);
    else if (act == kActReLU6) apply_flat<kActReLU6>(x, res, scale_shift, y, nullptr, M, C, dtype, st);
    else apply_flat<kActNone>(x, res, scale_shift, y, nullptr, M, C, dtype, st);
    return;
  }
  with_tv(dtype, C, [&]<typename T, int V>() {
    if (act == kActReLU) apply_t<T, V, kActReLU>(x, res, scale_shift, y, M, C, st, y2, ld2);
    else if (act == kActReLU6) apply_t<T, V, kActReLU6>(x, res, scale_shift, y, M, C, st, y2, ld2);
    else apply_t<T, V, kActNone>(x, res, scale_shift, y, M, C, st, y2, ld2);
  });
}

template <typename T, int V, int ACT, int MASK>
static void bwd_reduce_t(const void* dy, const void* x, const void* y, const float* mi,
                         const float* ss, int64_t M, int C, float* part, int G, hipStream_t st,
                         const void* dy2, int64_t ld2) {
  const int rpi = 256 / (C / V);
  const size_t lds = sizeof(float) * (3 * C + 2 * rpi * C);
  bn_bwd_reduce_kernel<T, V, ACT, MASK><<<G, 256, lds, st>>>(
      static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mi, ss, M, C,
      part, static_cast<const T*>(dy2), ld2, (l3_order() & 1) ? 1 : (l3_order() & 2) ? 2 : 0);
}

template <typename T, int V, int ACT, int MASK, bool DRES>
static void bwd_apply_t(const void* dy, const void* x, const void* y, const float* mi,
                        const float* ss, const float* k, void* dx, void* dres, int64_t M, int C,
                        hipStream_t st, const void* dy2, int64_t ld2) {
  const int64_t work = M * (C / V);
  const size_t lds = sizeof(float) * 6 * C;
  bn_bwd_apply_kernel<T, V, ACT, MASK, DRES><<<apply_grid(work), 256, lds, st>>>(
      static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mi, ss, k,
      static_cast<T*>(dx), static_cast<T*>(dres), M, C, static_cast<const T*>(dy2), ld2,
      (l3_order() & 4) != 0);
}

#define RT_ACT_MASK_DISPATCH(FN, ...)                                                   \
  do {                                                                                  \
    if (act == kActNone || mask == kMaskNone) FN<T, V, kActNone, kMaskNone>(__VA_ARGS__); \
    else if (act == kActReLU) {                                                         \
      if (mask == kMaskFromY) FN<T, V, kActReLU, kMaskFromY>(__VA_ARGS__);              \
      else if (mask == kMaskBits) FN<T, V, kActReLU, kMaskBits>(__VA_ARGS__);           \
      else FN<T, V, kActReLU, kMaskFromX>(__VA_ARGS__);                                 \
    } else {                                                                            \
      if (mask == kMaskFromY) FN<T, V, kActReLU6, kMaskFromY>(__VA_ARGS__);             \
      else if (mask == kMaskBits) FN<T, V, kActReLU6, kMaskBits>(__VA_ARGS__);          \
      else FN<T, V, kActReLU6, kMaskFromX>(__VA_ARGS__);                                \
    }                                                                                   \
  } while (0)

// flat (odd C) backward dispatch: T = fp32 or bf16, (act, mask) as RT_ACT_MASK_DISPATCH
#define RT_FLAT_DISPATCH(...)                                                           \
  do {                                                                                  \
    auto run = [&]<typename T, int ACT, int MASK>() { __VA_ARGS__; };                   \
    auto by_mask = [&]<typename T>() {                                                  \
      if (act == kActNone || mask == kMaskNone) run.template operator()<T, kActNone, kMaskNone>(); \
      else if (act == kActReLU) {                                                       \
        if (mask == kMaskFromY) run.template operator()<T, kActReLU, kMaskFromY>();     \
        else if (mask == kMaskBits) run.template operator()<T, kActReLU, kMaskBits>();  \
        else run.template operator()<T, kActReLU, kMaskFromX>();                        \
      } else {                                                                          \
        if (mask == kMaskFromY) run.template operator()<T, kActReLU6, kMaskFromY>();    \
        else if (mask == kMaskBits) run.template operator()<T, kActReLU6, kMaskBits>(); \
        else run.template operator()<T, kActReLU6, kMaskFromX>();                       \
      }                                                                                 \
    };                                                                                  \
    if (dtype == kF32) by_mask.template operator()<float>();                            \
    else by_mask.template operator()<uint16_t>();                                       \
  } while (0)

void launch_bn_bwd_reduce(const void* dy, const void* x, const void* y, const float* mean_invstd,
                          const float* scale_shift, int dtype, int64_t M, int C, int act, int mask,
                          float* part, int G, hipStream_t st, const void* dy2, int64_t ld2) {
  if (bn_flat(dtype, C)) {  // G (bn_partial_grid) is a multiple of C
    RT_FLAT_DISPATCH((bn_bwd_reduce_flat_kernel<T, ACT, MASK><<<G, 256, 0, st>>>(
        static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mean_invstd, scale_shift,
        M, C, part)));
    return;
  }
  with_tv(dtype, C, [&]<typename T, int V>() {
    RT_ACT_MASK_DISPATCH(bwd_reduce_t, dy, x, y, mean_invstd, scale_shift, M, C, part, G, st, dy2, ld2);
  });
}

void launch_bn_bwd_finalize(const float* part, int G, const double* sums, const double* count_ptr,
                            int C, const float* w, const float* mean_invstd, int batch_stats,
                            float* kcoef, float* dw, float* db, hipStream_t st, double* scratch) {
  with_split(sums ? nullptr : part, G, C, scratch, st, [&](const auto* p, int g) {
    using P = std::remove_cv_t<std::remove_pointer_t<decltype(p)>>;
    bn_bwd_finalize_kernel<P><<<(C + 63) / 64, kFinBlock, 0, st>>>(p, g, sums, count_ptr, C, w, mean_invstd,
                                                                batch_stats, kcoef, dw, db);
  });
}

template <typename T, int V, int ACT, int MASK>
static void bwd_apply_res(const void* dy, const void* x, const void* y, const float* mi,
                          const float* ss, const float* k, void* dx, void* dres, int64_t M, int C,
                          hipStream_t st, const void* dy2, int64_t ld2) {
  if (dres) bwd_apply_t<T, V, ACT, MASK, true>(dy, x, y, mi, ss, k, dx, dres, M, C, st, dy2, ld2);
  else bwd_apply_t<T, V, ACT, MASK, false>(dy, x, y, mi, ss, k, dx, dres, M, C, st, dy2, ld2);
}

void launch_bn_bwd_apply(const void* dy, const void* x, const void* y, const float* mean_invstd,
                         const float* scale_shift, const float* kcoef, void* dx, void* dres,
                         int dtype, int64_t M, int C, int act, int mask, hipStream_t st,
                         const void* dy2, int64_t ld2) {
  if (bn_flat(dtype, C)) {
    const int g = flat_grid(M, C, dtype);
    RT_FLAT_DISPATCH({
      if (dres != nullptr)
        bn_bwd_apply_flat_kernel<T, ACT, MASK, true><<<g, 256, 0, st>>>(
            static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mean_invstd, scale_shift,
            kcoef, static_cast<T*>(dx), static_cast<T*>(dres), M, C);
      else
        bn_bwd_apply_flat_kernel<T, ACT, MASK, false><<<g, 256, 0, st>>>(
            static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(y), mean_invstd, scale_shift,
            kcoef, static_cast<T*>(dx), static_cast<T*>(dres), M, C);
    });
    return;
  }
  with_tv(dtype, C, [&]<typename T, int V>() {
    RT_ACT_MASK_DISPATCH(bwd_apply_res, dy, x, y, mean_invstd, scale_shift, kcoef, dx, dres, M, C,
                         st, dy2, ld2);
  });
}

}  // namespace rtseg
