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
#include "rtseg_vec.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace rtseg {

namespace {

constexpr int kDwBlock = 256;

// Divisors of the flattened (pixel, channel-vector) index: channel vectors, width, height.
struct DwDivs {
  FastDiv c, w, h;
};
constexpr int kMaxTaps = 9;  // taps accumulated per wgrad thread (tap groups cover larger kernels)

// MT: channel multiplier handled at compile time.  1 = plain depth-wise; 2/3/4/6 =
// multiplier path where a thread owns VEC *input* channels and the VEC*MT
// contiguous output channels they feed (BiSeNetV2's x6 gather-expansion: one
// input vector load + MT output vector stores per tap instead of per-element
// gathers); 0 = any other multiplier (per-element gather, correctness path).

// VEC consecutive fp32 weights (16-byte vectors when VEC % 4 == 0: the tap-major rows and
// the channel offsets are multiples of VEC, so those loads are aligned).
template <int VEC>
__device__ __forceinline__ void load_wvec(const float* p, float* w) {
  if constexpr (VEC % 4 == 0) {
#pragma unroll
    for (int q = 0; q < VEC / 4; ++q) {
      const float4 f = reinterpret_cast<const float4*>(p)[q];
      w[4 * q] = f.x; w[4 * q + 1] = f.y; w[4 * q + 2] = f.z; w[4 * q + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v) w[v] = p[v];
  }
}

// Out-of-image taps: every load is issued unconditionally from a clamped (valid)
// address and the LOADED VALUE is zeroed by a select -- never `ok ? fma(load) : acc`,
// which hipcc lowers to a branch + s_waitcnt around every single load.

// ---------------------------------------------------------------- forward
// STATS: also the per-channel (sum, sum of squares) of the fp32 outputs for a training BatchNorm
// (one [2 * Cout] row per block of `part`, reduced by bn_finalize_slab) -- the BN forward then
// never re-reads y.  Deterministic: the host makes gridDim.x * kDwBlock a multiple of the
// channel-vector count, so each thread keeps ONE channel vector for all its iterations and
// accumulates it in registers; the block then sums its threads in a fixed order through LDS.
// CSW (channel-stationary weights, MT == 1 and KS > 0 only): the host sizes the grid so every
// thread keeps ONE channel vector (gridDim.x * kDwBlock a multiple of the channel-vector count, as
// for STATS), and the thread's KS x KS x VEC weights are loaded into registers once instead of
// per output pixel -- the unrolled taps then issue only their input loads (KS^2 in flight).  Per
// output that removes 9 x 32 B of weight loads against 9 x 16 B of activations (the reason an
// unrolled 3 x 3 without it measured 4-5x slower: see launch_dw_fwd).
// QD (MT 1, 3 x 3, CSW, stride 1, column dilation 1): a thread computes 4 consecutive output pixels
// of its channel vector from 6 input columns per kernel row (18 loads instead of 36); fd.w then
// divides the 4-pixel segments of a row.
template <typename T, int VEC, int MT, int KS, bool STATS = false, bool CSW = false, bool QD = false>
__global__ void __launch_bounds__(kDwBlock) dw_fwd_kernel(DwGeom g, DwDivs fd, const T* __restrict__ x,
                                                          const float* __restrict__ wt,
                                                          const float* __restrict__ bias, T* __restrict__ y,
                                                          float* __restrict__ part = nullptr) {
  static_assert(!CSW || (MT >= 1 && KS > 0), "channel-stationary weights: compile-time taps");
  constexpr int OV = MT > 1 ? VEC * MT : VEC;  // output channels per thread
  // SV: the widest vector (<= 8) dividing OV -- output stores (co and Cout are multiples of OV)
  constexpr int SV = OV % 8 == 0 ? 8 : OV % 4 == 0 ? 4 : OV % 2 == 0 ? 2 : 1;
  const int cv_n = MT > 1 ? g.cin / VEC : g.cout / VEC;
  static_assert(!QD || (MT == 1 && KS == 3 && CSW), "row segments: plain 3 x 3 channel-stationary");
  const uint32_t total = static_cast<uint32_t>(g.n) * g.ho * (QD ? (g.wo + 3) / 4 : g.wo) * cv_n;  // < 2^31
  float wreg[CSW ? KS * KS : 1][CSW ? OV : 1];
  float breg[CSW ? OV : 1];
  if constexpr (CSW) {
    const int co = static_cast<int>((blockIdx.x * kDwBlock + threadIdx.x) % static_cast<uint32_t>(cv_n)) * OV;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) load_wvec<OV>(wt + t * g.cout + co, wreg[t]);
#pragma unroll
    for (int v = 0; v < OV; ++v) breg[v] = bias ? bias[co + v] : 0.f;
  }
  float ssum[STATS ? OV : 1], ssq[STATS ? OV : 1];
  if constexpr (STATS) {
#pragma unroll
    for (int e = 0; e < OV; ++e) ssum[e] = ssq[e] = 0.f;
  }
  for (uint32_t it = blockIdx.x * kDwBlock + threadIdx.x; it < total; it += gridDim.x * kDwBlock) {
    uint32_t cvu, wou, hou;
    const uint32_t pix = fd.c.divmod(it, cvu);
    const uint32_t r = fd.w.divmod(pix, wou);
    const int n = static_cast<int>(fd.h.divmod(r, hou));
    const int cv = static_cast<int>(cvu), wo = static_cast<int>(wou), ho = static_cast<int>(hou);
    const int co = MT > 1 ? cv * VEC * MT : cv * VEC;  // first output channel
    const int ci = cv * VEC;                             // first input channel (MT > 1)
    if constexpr (QD) {
      const int wo0 = wo * 4;
      float a4[4][VEC];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int v = 0; v < VEC; ++v) a4[q][v] = breg[v];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int hi = ho - g.ph + i * g.dh;
        const bool rok = hi >= 0 && hi < g.h;
        const T* xr = x + (static_cast<int64_t>(n) * g.h + min(max(hi, 0), g.h - 1)) * g.w * g.cin + co;
        float xv[6][VEC];
#pragma unroll
        for (int c = 0; c < 6; ++c) {  // output wo0 + q, tap j reads column wo0 + q + j - pw
          const int wi = wo0 - g.pw + c;
          const bool ok = rok && wi >= 0 && wi < g.w;
          Vec<T, VEC>::load(xr + static_cast<int64_t>(min(max(wi, 0), g.w - 1)) * g.cin, xv[c]);
#pragma unroll
          for (int v = 0; v < VEC; ++v) xv[c][v] = ok ? xv[c][v] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int v = 0; v < VEC; ++v) a4[q][v] = fmaf(xv[q + j][v], wreg[i * 3 + j][v], a4[q][v]);
      }
      T* yq = y + ((static_cast<int64_t>(n) * g.ho + ho) * g.wo + wo0) * g.cout + co;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (wo0 + q >= g.wo) break;
        if constexpr (!STATS) {
          if (g.act != 0) {
#pragma unroll
            for (int v = 0; v < VEC; ++v) a4[q][v] = g.act == 1 ? fmaxf(a4[q][v], 0.f) : fminf(fmaxf(a4[q][v], 0.f), 6.f);
          }
        }
        Vec<T, VEC>::store(yq + static_cast<int64_t>(q) * g.cout, a4[q]);
        if constexpr (STATS) {
#pragma unroll
          for (int v = 0; v < VEC; ++v) {
            ssum[v] += a4[q][v];
            ssq[v] = fmaf(a4[q][v], a4[q][v], ssq[v]);
          }
        }
      }
      continue;
    }
    float acc[OV];
#pragma unroll
    for (int v = 0; v < OV; ++v) {
      if constexpr (CSW) acc[v] = breg[v];
      else acc[v] = bias ? bias[co + v] : 0.f;
    }
    const int hb = ho * g.sh - g.ph, wb = wo * g.sw - g.pw;
    // branch-free tap: clamped (always valid) load, product selected away outside the image
    auto tap = [&](int i, int j) {
      const int hi = hb + i * g.dh, wi = wb + j * g.dw;
      const bool ok = hi >= 0 && hi < g.h && wi >= 0 && wi < g.w;
      const int hc = min(max(hi, 0), g.h - 1), wc = min(max(wi, 0), g.w - 1);
      const float* wp = wt + (i * g.kw + j) * g.cout + co;
      const T* xp = x + ((static_cast<int64_t>(n) * g.h + hc) * g.w + wc) * g.cin;
      float xv[VEC], wv[OV];
      if constexpr (CSW) {
#pragma unroll
        for (int v = 0; v < OV; ++v) wv[v] = wreg[KS > 0 ? i * KS + j : 0][v];
      } else {
        load_wvec<OV>(wp, wv);
      }
      if constexpr (MT == 1) {
        Vec<T, VEC>::load(xp + co, xv);
      } else if constexpr (MT > 1) {
        Vec<T, VEC>::load(xp + ci, xv);
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) xv[v] = Io<T>::ld(xp + (co + v) / g.mult);
      }
#pragma unroll
      for (int v = 0; v < VEC; ++v) xv[v] = ok ? xv[v] : 0.f;
#pragma unroll
      for (int e = 0; e < OV; ++e) acc[e] = fmaf(xv[MT > 1 ? e / MT : e], wv[e], acc[e]);
    };
    if constexpr (KS > 0) {
#pragma unroll
      for (int i = 0; i < KS; ++i)
#pragma unroll
        for (int j = 0; j < KS; ++j) tap(i, j);
    } else {
      for (int i = 0; i < g.kh; ++i)
        for (int j = 0; j < g.kw; ++j) tap(i, j);
    }
    T* yp = y + ((static_cast<int64_t>(n) * g.ho + ho) * g.wo + wo) * g.cout + co;
    if constexpr (!STATS) {
      if (g.act != 0) {  // an eval BN folded into weights / bias, then its ReLU / ReLU6 (uniform)
#pragma unroll
        for (int e = 0; e < OV; ++e) acc[e] = g.act == 1 ? fmaxf(acc[e], 0.f) : fminf(fmaxf(acc[e], 0.f), 6.f);
      }
    }
#pragma unroll
    for (int q = 0; q < OV / SV; ++q) Vec<T, SV>::store(yp + q * SV, acc + q * SV);
    if constexpr (STATS) {
#pragma unroll
      for (int e = 0; e < OV; ++e) {
        ssum[e] += acc[e];
        ssq[e] = fmaf(acc[e], acc[e], ssq[e]);
      }
    }
  }
  if constexpr (STATS) {
    // block reduction in 8-channel chunks: thread t owns channel vector (base + t) % cv_n
    __shared__ float red[2][8][kDwBlock];
    const int t = threadIdx.x;
    const int base = static_cast<int>((static_cast<uint64_t>(blockIdx.x) * kDwBlock) % cv_n);
    float* prow = part + static_cast<int64_t>(blockIdx.x) * 2 * g.cout;
#pragma unroll
    for (int k = 0; k < (OV + 7) / 8; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[0][e][t] = k * 8 + e < OV ? ssum[(k * 8 + e) % OV] : 0.f;
        red[1][e][t] = k * 8 + e < OV ? ssq[(k * 8 + e) % OV] : 0.f;
      }
      __syncthreads();
      // (channel vector cv, output e of this chunk): sum over the threads holding cv
      for (int r = t; r < cv_n * 8; r += kDwBlock) {
        const int cv = r >> 3, e = r & 7;
        if (k * 8 + e < OV) {
          int t0 = cv - base;
          t0 = ((t0 % cv_n) + cv_n) % cv_n;
          float a = 0.f, b = 0.f;
          for (int tt = t0; tt < kDwBlock; tt += cv_n) {
            a += red[0][e][tt];
            b += red[1][e][tt];
          }
          const int c = cv * OV + k * 8 + e;
          prow[c] = a;
          prow[g.cout + c] = b;
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- data grad
// CSW (MT > 1, KS > 0): channel-stationary grid (as the forward's), the thread's KS x KS x VEC*MT
// weights in registers and its VEC*MT contiguous dy values per tap in SV-wide loads -- instead of
// MT x (VEC dy + VEC fp32 weight) loads per tap
template <typename T, int VEC, int MT, int KS, bool CSW = false>
__global__ void __launch_bounds__(kDwBlock) dw_dgrad_kernel(DwGeom g, DwDivs fd, const T* __restrict__ dy,
                                                            const float* __restrict__ wt, T* __restrict__ dx) {
  static_assert(!CSW || (MT >= 1 && KS > 0), "channel-stationary dgrad: compile-time taps");
  constexpr int OV = MT > 1 ? VEC * MT : VEC;
  constexpr int SV = OV % 8 == 0 ? 8 : OV % 4 == 0 ? 4 : OV % 2 == 0 ? 2 : 1;
  const int cv_n = g.cin / VEC;
  const uint32_t total = static_cast<uint32_t>(g.n) * g.h * g.w * cv_n;  // < 2^31 (host splits)
  float wreg[CSW ? KS * KS : 1][CSW ? OV : 1];
  if constexpr (CSW) {
    const int c0 = static_cast<int>((blockIdx.x * kDwBlock + threadIdx.x) % static_cast<uint32_t>(cv_n)) * OV;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) load_wvec<OV>(wt + t * g.cout + c0, wreg[t]);
  }
  for (uint32_t it = blockIdx.x * kDwBlock + threadIdx.x; it < total; it += gridDim.x * kDwBlock) {
    uint32_t cvu, wiu, hiu;
    const uint32_t pix = fd.c.divmod(it, cvu);
    const uint32_t r = fd.w.divmod(pix, wiu);
    const int n = static_cast<int>(fd.h.divmod(r, hiu));
    const int cv = static_cast<int>(cvu), wi = static_cast<int>(wiu), hi = static_cast<int>(hiu);
    const int ci = cv * VEC;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    auto tap = [&](int i, int j) {
      const int hn = hi + g.ph - i * g.dh, wn = wi + g.pw - j * g.dw;
      const int ho = hn >= 0 ? hn / g.sh : 0, wo = wn >= 0 ? wn / g.sw : 0;
      const bool ok = hn >= 0 && wn >= 0 && ho * g.sh == hn && wo * g.sw == wn && ho < g.ho && wo < g.wo;
      const T* dp = dy + ((static_cast<int64_t>(n) * g.ho + min(ho, g.ho - 1)) * g.wo + min(wo, g.wo - 1)) * g.cout;
      const float* wp = wt + (i * g.kw + j) * g.cout;
      if constexpr (MT == 1) {
        float dv[VEC], wv[VEC];
        Vec<T, VEC>::load(dp + ci, dv);
        if constexpr (CSW) {
#pragma unroll
          for (int v = 0; v < VEC; ++v) wv[v] = wreg[i * KS + j][v];
        } else {
          load_wvec<VEC>(wp + ci, wv);
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = fmaf(ok ? dv[v] : 0.f, wv[v], acc[v]);
      } else if constexpr (CSW) {
        const int c0 = ci * MT;
        float dv[OV];
#pragma unroll
        for (int q = 0; q < OV / SV; ++q) Vec<T, SV>::load(dp + c0 + q * SV, dv + q * SV);
#pragma unroll
        for (int e = 0; e < OV; ++e) acc[e / MT] = fmaf(ok ? dv[e] : 0.f, wreg[i * KS + j][e], acc[e / MT]);
      } else if constexpr (MT > 1) {
        // the VEC*MT output channels fed by this input vector are contiguous
        const int c0 = ci * MT;
#pragma unroll
        for (int q = 0; q < MT; ++q) {
          float dv[VEC], wv[VEC];
          Vec<T, VEC>::load(dp + c0 + q * VEC, dv);
          load_wvec<VEC>(wp + c0 + q * VEC, wv);
#pragma unroll
          for (int r = 0; r < VEC; ++r) {
            const int e = q * VEC + r;
            acc[e / MT] = fmaf(ok ? dv[r] : 0.f, wv[r], acc[e / MT]);
          }
        }
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const int c0 = (ci + v) * g.mult;
          float sv = 0.f;
          for (int m = 0; m < g.mult; ++m) sv = fmaf(Io<T>::ld(dp + c0 + m), wp[c0 + m], sv);
          acc[v] = ok ? acc[v] + sv : acc[v];
        }
      }
    };
    if constexpr (KS > 0) {
#pragma unroll
      for (int i = 0; i < KS; ++i)
#pragma unroll
        for (int j = 0; j < KS; ++j) tap(i, j);
    } else {
      for (int i = 0; i < g.kh; ++i)
        for (int j = 0; j < g.kw; ++j) tap(i, j);
    }
    Vec<T, VEC>::store(dx + ((static_cast<int64_t>(n) * g.h + hi) * g.w + wi) * g.cin + ci, acc);
  }
}

// Stride-2 3 x 3 (pad 1, dilation 1) data gradient of a channel-multiplier conv, channel-stationary:
// a thread owns a 2 x 2 block of dx pixels (2a + p, 2b + q) of one input-channel vector.  Only
// taps on the stride grid contribute, so the block needs exactly the 2 x 2 dy pixels (a | a+1,
// b | b+1) -- 4 loads of the VEC*MT contiguous dy values instead of 4 x 9 clamped tap loads:
//   dx(2a,   2b  ) = dy(a,b) w11
//   dx(2a,   2b+1) = dy(a,b+1) w10 + dy(a,b) w12
//   dx(2a+1, 2b  ) = dy(a+1,b) w01 + dy(a,b) w21
//   dx(2a+1, 2b+1) = dy(a+1,b+1) w00 + dy(a+1,b) w02 + dy(a,b+1) w20 + dy(a,b) w22
// (hi = 2 ho - 1 + i: ho = (hi + 1 - i) / 2 on the grid).  fd: divisors (cv_n, ceil(W/2), ceil(H/2)).
template <typename T, int VEC, int MT>
__global__ void __launch_bounds__(kDwBlock) dw_dgrad_s2_kernel(DwGeom g, DwDivs fd, const T* __restrict__ dy,
                                                               const float* __restrict__ wt, T* __restrict__ dx) {
  constexpr int OV = VEC * MT;
  constexpr int SV = OV % 8 == 0 ? 8 : OV % 4 == 0 ? 4 : OV % 2 == 0 ? 2 : 1;
  const int cv_n = g.cin / VEC;
  const int A = (g.h + 1) / 2, B = (g.w + 1) / 2;
  const uint32_t total = static_cast<uint32_t>(g.n) * A * B * cv_n;  // < 2^31 (host splits)
  float wreg[9][OV];
  {
    const int c0 = static_cast<int>((blockIdx.x * kDwBlock + threadIdx.x) % static_cast<uint32_t>(cv_n)) * OV;
#pragma unroll
    for (int t = 0; t < 9; ++t) load_wvec<OV>(wt + t * g.cout + c0, wreg[t]);
  }
  for (uint32_t it = blockIdx.x * kDwBlock + threadIdx.x; it < total; it += gridDim.x * kDwBlock) {
    uint32_t cvu, bu, au;
    const uint32_t pix = fd.c.divmod(it, cvu);
    const uint32_t r = fd.w.divmod(pix, bu);
    const int n = static_cast<int>(fd.h.divmod(r, au));
    const int a = static_cast<int>(au), b = static_cast<int>(bu), ci = static_cast<int>(cvu) * VEC;
    const bool r1 = a + 1 < g.ho, c1 = b + 1 < g.wo;  // the second dy row / column exists
    const T* d00 = dy + ((static_cast<int64_t>(n) * g.ho + a) * g.wo + b) * g.cout + ci * MT;
    const int64_t rs = r1 ? static_cast<int64_t>(g.wo) * g.cout : 0, cs = c1 ? g.cout : 0;  // clamped steps
    float v00[OV], v01[OV], v10[OV], v11[OV];
#pragma unroll
    for (int q = 0; q < OV / SV; ++q) {
      Vec<T, SV>::load(d00 + q * SV, v00 + q * SV);
      Vec<T, SV>::load(d00 + cs + q * SV, v01 + q * SV);
      Vec<T, SV>::load(d00 + rs + q * SV, v10 + q * SV);
      Vec<T, SV>::load(d00 + rs + cs + q * SV, v11 + q * SV);
    }
#pragma unroll
    for (int e = 0; e < OV; ++e) {
      v01[e] = c1 ? v01[e] : 0.f;
      v10[e] = r1 ? v10[e] : 0.f;
      v11[e] = r1 && c1 ? v11[e] : 0.f;
    }
    float o00[VEC], o01[VEC], o10[VEC], o11[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) o00[v] = o01[v] = o10[v] = o11[v] = 0.f;
#pragma unroll
    for (int e = 0; e < OV; ++e) {
      const int v = e / MT;
      o00[v] = fmaf(v00[e], wreg[4][e], o00[v]);
      o01[v] = fmaf(v01[e], wreg[3][e], fmaf(v00[e], wreg[5][e], o01[v]));
      o10[v] = fmaf(v10[e], wreg[1][e], fmaf(v00[e], wreg[7][e], o10[v]));
      o11[v] = fmaf(v11[e], wreg[0][e], fmaf(v10[e], wreg[2][e], fmaf(v01[e], wreg[6][e], fmaf(v00[e], wreg[8][e], o11[v]))));
    }
    T* x00 = dx + ((static_cast<int64_t>(n) * g.h + 2 * a) * g.w + 2 * b) * g.cin + ci;
    const bool hr = 2 * a + 1 < g.h, hc = 2 * b + 1 < g.w;
    Vec<T, VEC>::store(x00, o00);
    if (hc) Vec<T, VEC>::store(x00 + g.cin, o01);
    if (hr) Vec<T, VEC>::store(x00 + static_cast<int64_t>(g.w) * g.cin, o10);
    if (hr && hc) Vec<T, VEC>::store(x00 + static_cast<int64_t>(g.w) * g.cin + g.cin, o11);
  }
}

// Plain (multiplier 1) 3 x 3 stride-1 data gradient (column dilation 1) over 4-pixel dx row
// segments, channel-stationary (9 x VEC weights in registers): per kernel row the segment needs 6
// dy columns -- 18 loads per 4 dx pixels instead of 36.  fd: divisors (cv_n, ceil(W/4), H).
template <typename T, int VEC>
__global__ void __launch_bounds__(kDwBlock) dw_dgrad_quad_kernel(DwGeom g, DwDivs fd, const T* __restrict__ dy,
                                                                 const float* __restrict__ wt, T* __restrict__ dx) {
  const int cv_n = g.cin / VEC;
  const int wq_n = (g.w + 3) / 4;
  const uint32_t total = static_cast<uint32_t>(g.n) * g.h * wq_n * cv_n;  // < 2^31 (host splits)
  float wreg[9][VEC];
  {
    const int c0 = static_cast<int>((blockIdx.x * kDwBlock + threadIdx.x) % static_cast<uint32_t>(cv_n)) * VEC;
#pragma unroll
    for (int t = 0; t < 9; ++t) load_wvec<VEC>(wt + t * g.cout + c0, wreg[t]);
  }
  for (uint32_t it = blockIdx.x * kDwBlock + threadIdx.x; it < total; it += gridDim.x * kDwBlock) {
    uint32_t cvu, wqu, hiu;
    const uint32_t pix = fd.c.divmod(it, cvu);
    const uint32_t r = fd.w.divmod(pix, wqu);
    const int n = static_cast<int>(fd.h.divmod(r, hiu));
    const int hi = static_cast<int>(hiu), wi0 = static_cast<int>(wqu) * 4, ci = static_cast<int>(cvu) * VEC;
    float acc[4][VEC];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[q][v] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int ho = hi + g.ph - i * g.dh;  // stride 1: always on the grid
      const bool rok = ho >= 0 && ho < g.ho;
      const T* dr = dy + (static_cast<int64_t>(n) * g.ho + min(max(ho, 0), g.ho - 1)) * g.wo * g.cout + ci;
      // dx column wi0 + q takes dy column wi0 + q + pw - j (j = 0..2): columns wi0 + pw - 2 + c, c = 0..5
      float dv[6][VEC];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int wo = wi0 + g.pw - 2 + c;
        const bool ok = rok && wo >= 0 && wo < g.wo;
        Vec<T, VEC>::load(dr + static_cast<int64_t>(min(max(wo, 0), g.wo - 1)) * g.cout, dv[c]);
#pragma unroll
        for (int v = 0; v < VEC; ++v) dv[c][v] = ok ? dv[c][v] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[q][v] = fmaf(dv[q + 2 - j][v], wreg[i * 3 + j][v], acc[q][v]);
    }
    T* xo = dx + ((static_cast<int64_t>(n) * g.h + hi) * g.w + wi0) * g.cin + ci;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (wi0 + q < g.w) Vec<T, VEC>::store(xo + static_cast<int64_t>(q) * g.cin, acc[q]);
  }
}

// ---------------------------------------------------------------- weight grad
// grid: x = pixel slices (G), y = channel chunks, z = tap groups.  Block = LANES
// channel-vector lanes x ROWS pixel rows; each thread accumulates <= kMaxTaps
// taps x VEC channels over its pixel stride, then the ROWS partials are reduced
// through LDS and one [taps x VEC] partial per (slice, channel vector) is stored.
template <typename T, int VEC, int MT, int NT>
__global__ void __launch_bounds__(kDwBlock) dw_wgrad_kernel(DwGeom g, DwDivs fd, const T* __restrict__ dy,
                                                            const T* __restrict__ x, float* __restrict__ part,
                                                            int lanes) {
  const int rows = kDwBlock / lanes;
  const int lane = threadIdx.x % lanes;
  const int row = threadIdx.x / lanes;
  const int cv = blockIdx.y * lanes + lane;
  const int cv_n = g.cout / VEC;
  const int taps = g.kh * g.kw;
  const int t0 = blockIdx.z * NT;
  const int nt = min(NT, taps - t0);
  const bool active = cv < cv_n;
  const int co = cv * VEC;
  // multiplier: the VEC output channels read input channels base + rel[v], rel in [0, 4)
  const int mult = MT > 0 ? MT : g.mult;
  const int base = co / mult;
  int rel[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) rel[v] = (co + v) / mult - base;
  float acc[NT][VEC];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[t][v] = 0.f;
  const uint32_t npix = static_cast<uint32_t>(g.n) * g.ho * g.wo;
  if (active) {
    for (uint32_t p = blockIdx.x * rows + row; p < npix; p += gridDim.x * rows) {
      uint32_t wou, hou;
      const uint32_t r = fd.w.divmod(p, wou);
      const int n = static_cast<int>(fd.h.divmod(r, hou));
      const int wo = static_cast<int>(wou), ho = static_cast<int>(hou);
      float dv[VEC];
      Vec<T, VEC>::load(dy + static_cast<int64_t>(p) * g.cout + co, dv);
      const int hb = ho * g.sh - g.ph, wb = wo * g.sw - g.pw;
      // Branch-free taps: every load goes to a clamped (valid) address and the product is
      // selected away for out-of-image / padding taps, so all NT taps' loads issue back to
      // back instead of one L2 round trip per tap behind a branch.
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int tap = t0 + min(t, nt - 1);
        const int i = tap / g.kw, j = tap - (tap / g.kw) * g.kw;
        const int hi = hb + i * g.dh, wi = wb + j * g.dw;
        const bool ok = t < nt && hi >= 0 && hi < g.h && wi >= 0 && wi < g.w;
        const int hc = min(max(hi, 0), g.h - 1), wc = min(max(wi, 0), g.w - 1);
        const T* xp = x + ((static_cast<int64_t>(n) * g.h + hc) * g.w + wc) * g.cin;
        float xv[VEC];
        if constexpr (MT == 1) {
          Vec<T, VEC>::load(xp + co, xv);
        } else {  // <= 4 distinct inputs (mult >= 2, VEC <= 8): scalar loads + selects; a
          // VEC-aligned group of 8 outputs spans only 2 inputs for mult 4 / 6 (BiSeNetV2's x6)
          constexpr int NIN = (MT == 4 || MT == 6) && VEC <= 8 ? 2 : 4;
          float xs[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) xs[k] = k < NIN ? Io<T>::ld(xp + min(base + k, g.cin - 1)) : 0.f;
#pragma unroll
          for (int v = 0; v < VEC; ++v)
            xv[v] = rel[v] == 0 ? xs[0] : rel[v] == 1 ? xs[1] : rel[v] == 2 ? xs[2] : xs[3];
        }
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[t][v] = fmaf(ok ? xv[v] : 0.f, dv[v], acc[t][v]);
      }
    }
  }
  // reduce the `rows` pixel rows of each lane through LDS, one tap at a time
  __shared__ float red[kDwBlock * 8];
  const int64_t slab = static_cast<int64_t>(blockIdx.x) * taps * g.cout;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
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

// Channel-multiplier weight gradient (bf16, MT = 2/3/4/6: BiSeNetV2's x6 gather-expansion):
// a thread owns one PAIR of input channels (ci, ci + 1) and the 2*MT contiguous output channels
// they feed.  Per pixel: the 2*MT dy values in 8-byte (even MT) or 4-byte loads, then per tap ONE
// 4-byte load of the input pair -- where dw_wgrad_kernel<VEC = 8> issues two 2-byte scalar loads
// + selects per tap for every 8 outputs and idles a quarter of its lanes (8-wide output vectors
// over a 6x channel count).  Lanes = input-channel pairs (a power of two for the zoo's 16..128
// channel inputs: no idle lanes); all KH*KW (<= 9) taps per thread, partials reduced through LDS
// into the same [G][taps][Cout] slab dw_wgrad_reduce_kernel sums (deterministic, no atomics).
template <int MT>
__global__ void __launch_bounds__(kDwBlock) dw_wgrad_pair_kernel(DwGeom g, DwDivs fd, const uint16_t* __restrict__ dy,
                                                                 const uint16_t* __restrict__ x,
                                                                 float* __restrict__ part, int lanes) {
  constexpr int OV = 2 * MT;  // outputs per thread
  const int rows = kDwBlock / lanes;
  const int lane = threadIdx.x % lanes;
  const int row = threadIdx.x / lanes;
  const int pv = blockIdx.y * lanes + lane;  // input-channel pair
  const bool active = pv < g.cin / 2;
  const int ci = pv * 2, co = ci * MT;
  const int taps = g.kh * g.kw;
  float acc[kMaxTaps][OV];
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t)
#pragma unroll
    for (int v = 0; v < OV; ++v) acc[t][v] = 0.f;
  const uint32_t npix = static_cast<uint32_t>(g.n) * g.ho * g.wo;
  if (active) {
    for (uint32_t p = blockIdx.x * rows + row; p < npix; p += gridDim.x * rows) {
      uint32_t wou, hou;
      const uint32_t r = fd.w.divmod(p, wou);
      const int n = static_cast<int>(fd.h.divmod(r, hou));
      const int wo = static_cast<int>(wou), ho = static_cast<int>(hou);
      uint32_t dw32[MT];  // OV bf16 = MT dwords
      const uint16_t* dp = dy + static_cast<int64_t>(p) * g.cout + co;
      if constexpr (MT % 2 == 0) {
#pragma unroll
        for (int q = 0; q < MT / 2; ++q) {
          const uint2 u = reinterpret_cast<const uint2*>(dp)[q];
          dw32[2 * q] = u.x;
          dw32[2 * q + 1] = u.y;
        }
      } else {
#pragma unroll
        for (int q = 0; q < MT; ++q) dw32[q] = reinterpret_cast<const uint32_t*>(dp)[q];
      }
      float dv[OV];
#pragma unroll
      for (int q = 0; q < MT; ++q) {
        dv[2 * q] = __uint_as_float(dw32[q] << 16);
        dv[2 * q + 1] = __uint_as_float(dw32[q] & 0xffff0000u);
      }
      const int hb = ho * g.sh - g.ph, wb = wo * g.sw - g.pw;
      const uint16_t* xn = x + static_cast<int64_t>(n) * g.h * g.w * g.cin + ci;
#pragma unroll
      for (int t = 0; t < kMaxTaps; ++t) {
        const int tap = min(t, taps - 1);
        const int i = tap / g.kw, j = tap - (tap / g.kw) * g.kw;
        const int hi = hb + i * g.dh, wi = wb + j * g.dw;
        const bool ok = t < taps && hi >= 0 && hi < g.h && wi >= 0 && wi < g.w;
        const int hc = min(max(hi, 0), g.h - 1), wc = min(max(wi, 0), g.w - 1);
        const uint32_t xu = *reinterpret_cast<const uint32_t*>(xn + (static_cast<int64_t>(hc) * g.w + wc) * g.cin);
        const float x0 = ok ? __uint_as_float(xu << 16) : 0.f;
        const float x1 = ok ? __uint_as_float(xu & 0xffff0000u) : 0.f;
#pragma unroll
        for (int v = 0; v < OV; ++v) acc[t][v] = fmaf(v < MT ? x0 : x1, dv[v], acc[t][v]);
      }
    }
  }
  __shared__ float red[kDwBlock * OV];
  const int64_t slab = static_cast<int64_t>(blockIdx.x) * taps * g.cout;
  const int c0 = blockIdx.y * lanes * OV;  // first output channel of this block
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t) {
    if (t < taps) {  // block-uniform
      __syncthreads();
#pragma unroll
      for (int v = 0; v < OV; ++v) red[(row * lanes + lane) * OV + v] = acc[t][v];
      __syncthreads();
      for (int k = threadIdx.x; k < lanes * OV; k += kDwBlock) {
        float s = 0.f;
        for (int rr = 0; rr < rows; ++rr) s += red[rr * lanes * OV + k];
        const int c = c0 + k;
        if (c < g.cout) part[slab + static_cast<int64_t>(t) * g.cout + c] = s;
      }
    }
  }
}

// Plain (multiplier 1) 3 x 3 stride-1 weight gradient (column dilation 1, any row dilation) over
// 4-pixel row segments: per kernel row the segment needs 6 input columns, so a thread loads 4 dy +
// 3 x 6 input vectors per 4 output pixels where dw_wgrad_kernel loads 4 x (1 + 9) -- the
// L1 / address traffic, not HBM, bounds that kernel (more slices do not help).  Same lanes /
// slab / column-reduce layout as dw_wgrad_kernel with NT = 9.
template <typename T, int VEC>
__global__ void __launch_bounds__(kDwBlock) dw_wgrad_quad_kernel(DwGeom g, DwDivs fd, const T* __restrict__ dy,
                                                                 const T* __restrict__ x, float* __restrict__ part,
                                                                 int lanes) {
  const int rows = kDwBlock / lanes;
  const int lane = threadIdx.x % lanes;
  const int row = threadIdx.x / lanes;
  const int cv = blockIdx.y * lanes + lane;
  const bool active = cv < g.cout / VEC;
  const int co = cv * VEC;
  float acc[9][VEC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[t][v] = 0.f;
  const int wq_n = (g.wo + 3) / 4;
  const uint32_t nq = static_cast<uint32_t>(g.n) * g.ho * wq_n;
  if (active) {
    for (uint32_t p = blockIdx.x * rows + row; p < nq; p += gridDim.x * rows) {
      uint32_t wqu, hou;
      const uint32_t r = fd.w.divmod(p, wqu);
      const int n = static_cast<int>(fd.h.divmod(r, hou));
      const int ho = static_cast<int>(hou), wo0 = static_cast<int>(wqu) * 4;
      float dv[4][VEC];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = wo0 + q < g.wo;
        Vec<T, VEC>::load(dy + ((static_cast<int64_t>(n) * g.ho + ho) * g.wo + min(wo0 + q, g.wo - 1)) * g.cout + co,
                          dv[q]);
#pragma unroll
        for (int v = 0; v < VEC; ++v) dv[q][v] = ok ? dv[q][v] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int hi = ho - g.ph + i * g.dh;
        const bool rok = hi >= 0 && hi < g.h;
        const T* xr = x + (static_cast<int64_t>(n) * g.h + min(max(hi, 0), g.h - 1)) * g.w * g.cin + co;
        float xv[6][VEC];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const int wi = wo0 - g.pw + c;
          const bool ok = rok && wi >= 0 && wi < g.w;
          Vec<T, VEC>::load(xr + static_cast<int64_t>(min(max(wi, 0), g.w - 1)) * g.cin, xv[c]);
#pragma unroll
          for (int v = 0; v < VEC; ++v) xv[c][v] = ok ? xv[c][v] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[i * 3 + j][v] = fmaf(xv[q + j][v], dv[q][v], acc[i * 3 + j][v]);
      }
    }
  }
  __shared__ float red[kDwBlock * 8];
  const int64_t slab = static_cast<int64_t>(blockIdx.x) * 9 * g.cout;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    __syncthreads();
#pragma unroll
    for (int v = 0; v < VEC; ++v) red[(row * lanes + lane) * VEC + v] = acc[t][v];
    __syncthreads();
    for (int k = threadIdx.x; k < lanes * VEC; k += kDwBlock) {
      float s = 0.f;
      for (int rr = 0; rr < rows; ++rr) s += red[rr * lanes * VEC + k];
      const int c = blockIdx.y * lanes * VEC + k;
      if (c < g.cout) part[slab + static_cast<int64_t>(t) * g.cout + c] = s;
    }
  }
}

// dw[co][tap] = sum_G part[G][tap][co]   (output in the [Cout, 1, KH, KW] layout).
// One block per 64 columns; 16 waves split the G rows (latency-bound reduction).
constexpr int kRedWaves = 16;
__global__ void __launch_bounds__(kRedWaves * 64) dw_wgrad_reduce_kernel(const float* __restrict__ part, int G,
                                                                         int taps, int cout, float* __restrict__ dw) {
  __shared__ float red[kRedWaves * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;  // k = tap * cout + co
  const int ncol = taps * cout;
  float s = 0.f;
  if (k < ncol) {
    const float* p = part + k;
    int gi = w;
    for (; gi + 7 * kRedWaves < G; gi += 8 * kRedWaves) {
      float f[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) f[u] = p[static_cast<int64_t>(gi + u * kRedWaves) * ncol];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += f[u];
    }
    for (; gi < G; gi += kRedWaves) s += p[static_cast<int64_t>(gi) * ncol];
  }
  red[w * 64 + lane] = s;
  __syncthreads();
  if (w == 0 && k < ncol) {
    float t = 0.f;
#pragma unroll
    for (int u = 0; u < kRedWaves; ++u) t += red[u * 64 + lane];
    const int tap = k / cout, co = k - (k / cout) * cout;
    dw[static_cast<int64_t>(co) * taps + tap] = t;
  }
}

template <typename F>
void dw_dispatch(int dtype, int vec, int mult, F&& f) {
  auto by_mt = [&](auto t, auto v) {
    switch (mult) {
      case 1: f(t, v, std::integral_constant<int, 1>{}); break;
      case 2: f(t, v, std::integral_constant<int, 2>{}); break;
      case 3: f(t, v, std::integral_constant<int, 3>{}); break;
      case 4: f(t, v, std::integral_constant<int, 4>{}); break;
      case 6: f(t, v, std::integral_constant<int, 6>{}); break;
      default: f(t, v, std::integral_constant<int, 0>{}); break;
    }
  };
  auto by_vec = [&](auto t) {
    if (vec == 8) by_mt(t, std::integral_constant<int, 8>{});
    else if (vec == 4) by_mt(t, std::integral_constant<int, 4>{});
    else if (vec == 2) by_mt(t, std::integral_constant<int, 2>{});
    else by_mt(t, std::integral_constant<int, 1>{});
  };
  if (dtype == kF32) by_vec(float{});
  else if (dtype == kBF16) by_vec(uint16_t{});
  else by_vec(_Float16{});
}

// Multiplier as the kernels treat it (see MT above).
int mt_of(int mult) { return (mult == 1 || mult == 2 || mult == 3 || mult == 4 || mult == 6) ? mult : 0; }

}  // namespace

int dw_vec(int dtype, int c) {
  const int maxv = dtype == kF32 ? 4 : 8;  // 16-byte vectors
  for (int v = maxv; v > 1; v >>= 1)
    if (c % v == 0) return v;
  return 1;
}

// The kernels index (pixel, channel-vector) pairs in 32 bits: split the batch so every
// launch stays below 2^31 items (sub-batches are plain pointer offsets in NHWC).
static int batch_chunk(int64_t per_image, int n) {
  const int64_t lim = (int64_t{1} << 31) - 1;
  int64_t c = per_image > 0 ? lim / per_image : n;
  if (c < 1) c = 1;
  return static_cast<int>(c < n ? c : n);
}

static int64_t elem_bytes(int dtype) { return dtype == kF32 ? 4 : 2; }

static int dw_stats_grid(int64_t items, int cv_n);

// RTSEG_DW_CS=0: the 3 x 3 channel-stationary register-weight forward off (A/B)
static bool dw_cs_enabled() {
  static const bool on = [] { const char* e = std::getenv("RTSEG_DW_CS"); return !(e && e[0] == '0'); }();
  return on;
}

// Multiplier convs (MT > 1) with a 3 x 3 kernel run channel-stationary on input-channel PAIRS:
// VEC = 2, so a thread's 9 x 2*MT weights fit in registers (108 for BiSeNetV2's x6) and it loads
// per tap one 4-byte input pair (forward) or 2*MT contiguous dy values (dgrad), where VEC = 8
// re-loaded 9 x 8*MT fp32 weights per output pixel.  RTSEG_DW_MT_CS=0: off (A/B)
static bool dw_mt_cs(const DwGeom& g) {
  static const bool on = [] { const char* e = std::getenv("RTSEG_DW_MT_CS"); return !(e && e[0] == '0'); }();
  return on && mt_of(g.mult) > 1 && g.kh == 3 && g.kw == 3 && g.cin % 2 == 0;
}

// Plain 3 x 3 stride-1 forwards (column dilation 1) on 4-pixel row segments (dw_fwd_kernel QD);
// RTSEG_DW_QD=0: one pixel per thread (A/B)
static bool dw_fwd_qd(const DwGeom& g) {
  static const bool on = [] { const char* e = std::getenv("RTSEG_DW_QD"); return !(e && e[0] == '0'); }();
  return on && mt_of(g.mult) == 1 && g.kh == 3 && g.kw == 3 && g.sh == 1 && g.sw == 1 && g.dw == 1 &&
         dw_cs_enabled();
}

void launch_dw_fwd(const DwGeom& g0, int dtype, const void* x, const float* wt, const float* bias, void* y,
                   hipStream_t st) {
  const int mt = mt_of(g0.mult);
  const bool mcs = dw_mt_cs(g0);
  // MT > 1: vectors over the INPUT channels (each feeds VEC*MT contiguous outputs)
  const int vec = mcs ? 2 : mt > 1 ? dw_vec(dtype, g0.cin) : dw_vec(dtype, g0.cout);
  const int cv_n = (mt > 1 ? g0.cin : g0.cout) / vec;
  const bool qd = dw_fwd_qd(g0);
  const int wq = qd ? (g0.wo + 3) / 4 : g0.wo;  // work items per output row
  const int64_t per_img = static_cast<int64_t>(g0.ho) * wq * cv_n;
  const int nb = batch_chunk(per_img, g0.n);
  const int64_t eb = elem_bytes(dtype);
  for (int n0 = 0; n0 < g0.n; n0 += nb) {
    DwGeom g = g0;
    g.n = n0 + nb <= g0.n ? nb : g0.n - n0;
    const char* xb = static_cast<const char*>(x) + static_cast<int64_t>(n0) * g.h * g.w * g.cin * eb;
    char* yb = static_cast<char*>(y) + static_cast<int64_t>(n0) * g.ho * g.wo * g.cout * eb;
    const DwDivs fd{FastDiv::make(cv_n), FastDiv::make(wq), FastDiv::make(g.ho)};
    const bool cs3 = (mt == 1 && g.kh == 3 && g.kw == 3 && dw_cs_enabled()) || mcs;
    const int grid = cs3 ? dw_stats_grid(per_img * g.n, cv_n) : stream_grid(per_img * g.n, kDwBlock);
    dw_dispatch(dtype, vec, g.mult, [&](auto t, auto v, auto m) {
      using T = decltype(t);
      constexpr int V = decltype(v)::value, M = decltype(m)::value;
      if constexpr (M == 1) {
        if (qd) {
          dw_fwd_kernel<T, V, 1, 3, false, true, true><<<grid, kDwBlock, 0, st>>>(
              g, fd, reinterpret_cast<const T*>(xb), wt, bias, reinterpret_cast<T*>(yb));
          return;
        }
      }
      if constexpr (M == 1 || (M > 1 && V == 2)) {
        if (cs3) {  // 3 x 3, channel-stationary: weights in registers, 9 loads in flight
          dw_fwd_kernel<T, V, M, 3, false, true><<<grid, kDwBlock, 0, st>>>(
              g, fd, reinterpret_cast<const T*>(xb), wt, bias, reinterpret_cast<T*>(yb));
          return;
        }
      }
      // KS = 0: runtime tap loop.  A fully unrolled 3x3 (KS = 3) WITHOUT register weights measured
      // 4-5x slower on BiSeNetV2 (it re-loads all 9 taps' weights per output with no latency to hide)
      dw_fwd_kernel<T, V, M, 0><<<grid, kDwBlock, 0, st>>>(g, fd, reinterpret_cast<const T*>(xb), wt, bias,
                                                             reinterpret_cast<T*>(yb));
    });
  }
}

// grid of one stats launch: a multiple of cv_n / gcd(cv_n, kDwBlock) blocks (every thread keeps
// one channel vector), never more blocks than the work needs rounded up to that multiple
static int dw_stats_grid(int64_t items, int cv_n) {
  int gg = kDwBlock, a = cv_n;
  while (a != 0) { const int r = gg % a; gg = a; a = r; }
  const int m = cv_n / gg;
  int grid = stream_grid(items, kDwBlock);
  grid = std::max(m, (grid + m - 1) / m * m);
  return grid;
}

static int dw_fwd_stats_vec(const DwGeom& g, int dtype) {
  const int mt = mt_of(g.mult);
  return dw_mt_cs(g) ? 2 : mt > 1 ? dw_vec(dtype, g.cin) : dw_vec(dtype, g.cout);
}

int dw_fwd_stats_rows(const DwGeom& g0, int dtype) {
  const int mt = mt_of(g0.mult);
  if (mt == 0) return 0;
  const int vec = dw_fwd_stats_vec(g0, dtype);
  const int cv_n = (mt > 1 ? g0.cin : g0.cout) / vec;
  const int64_t per_img = static_cast<int64_t>(g0.ho) * (dw_fwd_qd(g0) ? (g0.wo + 3) / 4 : g0.wo) * cv_n;
  const int nb = batch_chunk(per_img, g0.n);
  int rows = 0;
  for (int n0 = 0; n0 < g0.n; n0 += nb) rows += dw_stats_grid(per_img * std::min(nb, g0.n - n0), cv_n);
  return rows;
}

void launch_dw_fwd_stats(const DwGeom& g0, int dtype, const void* x, const float* wt, void* y, float* part,
                         hipStream_t st) {
  const int mt = mt_of(g0.mult);
  const int vec = dw_fwd_stats_vec(g0, dtype);
  const int cv_n = (mt > 1 ? g0.cin : g0.cout) / vec;
  const bool qd = dw_fwd_qd(g0);
  const int wq = qd ? (g0.wo + 3) / 4 : g0.wo;  // work items per output row (as dw_fwd_stats_rows)
  const int64_t per_img = static_cast<int64_t>(g0.ho) * wq * cv_n;
  const int nb = batch_chunk(per_img, g0.n);
  const int64_t eb = elem_bytes(dtype);
  for (int n0 = 0; n0 < g0.n; n0 += nb) {
    DwGeom g = g0;
    g.n = n0 + nb <= g0.n ? nb : g0.n - n0;
    const char* xb = static_cast<const char*>(x) + static_cast<int64_t>(n0) * g.h * g.w * g.cin * eb;
    char* yb = static_cast<char*>(y) + static_cast<int64_t>(n0) * g.ho * g.wo * g.cout * eb;
    const DwDivs fd{FastDiv::make(cv_n), FastDiv::make(wq), FastDiv::make(g.ho)};
    const int grid = dw_stats_grid(per_img * g.n, cv_n);
    dw_dispatch(dtype, vec, g.mult, [&](auto t, auto v, auto m) {
      using T = decltype(t);
      constexpr int V = decltype(v)::value, M = decltype(m)::value;
      if constexpr (M == 1) {
        if (qd) {
          dw_fwd_kernel<T, V, 1, 3, true, true, true><<<grid, kDwBlock, 0, st>>>(
              g, fd, reinterpret_cast<const T*>(xb), wt, nullptr, reinterpret_cast<T*>(yb), part);
          return;
        }
        if (g.kh == 3 && g.kw == 3 && dw_cs_enabled()) {  // the grid is channel-stationary already
          dw_fwd_kernel<T, V, 1, 3, true, true><<<grid, kDwBlock, 0, st>>>(
              g, fd, reinterpret_cast<const T*>(xb), wt, nullptr, reinterpret_cast<T*>(yb), part);
          return;
        }
      } else if constexpr (M > 1 && V == 2) {
        if (dw_mt_cs(g)) {
          dw_fwd_kernel<T, V, M, 3, true, true><<<grid, kDwBlock, 0, st>>>(
              g, fd, reinterpret_cast<const T*>(xb), wt, nullptr, reinterpret_cast<T*>(yb), part);
          return;
        }
      }
      if constexpr (M != 0) {
        dw_fwd_kernel<T, V, M, 0, true><<<grid, kDwBlock, 0, st>>>(g, fd, reinterpret_cast<const T*>(xb), wt, nullptr,
                                                                     reinterpret_cast<T*>(yb), part);
      }
    });
    part += static_cast<int64_t>(grid) * 2 * g.cout;
  }
}

void launch_dw_dgrad(const DwGeom& g0, int dtype, const void* dy, const float* wt, void* dx, hipStream_t st) {
  // channel-stationary 3 x 3: multiplier convs on input pairs (dw_mt_cs), plain ones (MT 1) on
  // their usual channel vectors with the 9 x VEC weights in registers (the forward's RTSEG_DW_CS)
  const bool mcs = dw_mt_cs(g0) || (mt_of(g0.mult) == 1 && g0.kh == 3 && g0.kw == 3 && dw_cs_enabled());
  // stride-2 3 x 3 pad-1 multiplier convs: the 2 x 2 dx-block kernel (dw_dgrad_s2_kernel)
  const bool s2 = mcs && g0.sh == 2 && g0.sw == 2 && g0.ph == 1 && g0.pw == 1 && g0.dh == 1 && g0.dw == 1;
  const int vec = dw_mt_cs(g0) ? 2 : dw_vec(dtype, g0.cin);
  const int cv_n = g0.cin / vec;
  // plain 3 x 3 stride-1 (column dilation 1): the 4-pixel row-segment kernel
  const bool q1 = mcs && mt_of(g0.mult) == 1 && g0.sh == 1 && g0.sw == 1 && g0.dw == 1;
  if (q1) {
    const int wq = (g0.w + 3) / 4;
    const int64_t per_img = static_cast<int64_t>(g0.h) * wq * cv_n;
    const int nb = batch_chunk(per_img, g0.n);
    const int64_t eb = elem_bytes(dtype);
    for (int n0 = 0; n0 < g0.n; n0 += nb) {
      DwGeom g = g0;
      g.n = n0 + nb <= g0.n ? nb : g0.n - n0;
      const char* dyb = static_cast<const char*>(dy) + static_cast<int64_t>(n0) * g.ho * g.wo * g.cout * eb;
      char* dxb = static_cast<char*>(dx) + static_cast<int64_t>(n0) * g.h * g.w * g.cin * eb;
      const DwDivs fd{FastDiv::make(cv_n), FastDiv::make(wq), FastDiv::make(g.h)};
      const int grid = dw_stats_grid(per_img * g.n, cv_n);
      dw_dispatch(dtype, vec, 1, [&](auto t, auto v, auto) {
        using T = decltype(t);
        constexpr int V = decltype(v)::value;
        dw_dgrad_quad_kernel<T, V><<<grid, kDwBlock, 0, st>>>(g, fd, reinterpret_cast<const T*>(dyb), wt,
                                                              reinterpret_cast<T*>(dxb));
      });
    }
    return;
  }
  if (s2) {
    const int A = (g0.h + 1) / 2, B = (g0.w + 1) / 2;
    const int64_t per_img = static_cast<int64_t>(A) * B * cv_n;
    const int nb = batch_chunk(per_img, g0.n);
    const int64_t eb = elem_bytes(dtype);
    for (int n0 = 0; n0 < g0.n; n0 += nb) {
      DwGeom g = g0;
      g.n = n0 + nb <= g0.n ? nb : g0.n - n0;
      const char* dyb = static_cast<const char*>(dy) + static_cast<int64_t>(n0) * g.ho * g.wo * g.cout * eb;
      char* dxb = static_cast<char*>(dx) + static_cast<int64_t>(n0) * g.h * g.w * g.cin * eb;
      const DwDivs fd{FastDiv::make(cv_n), FastDiv::make(B), FastDiv::make(A)};
      const int grid = dw_stats_grid(per_img * g.n, cv_n);
      dw_dispatch(dtype, vec, g.mult, [&](auto t, auto v, auto m) {
        using T = decltype(t);
        constexpr int V = decltype(v)::value, M = decltype(m)::value;
        if constexpr ((M > 1 && V == 2) || M == 1)
          dw_dgrad_s2_kernel<T, V, M><<<grid, kDwBlock, 0, st>>>(g, fd, reinterpret_cast<const T*>(dyb), wt,
                                                                 reinterpret_cast<T*>(dxb));
      });
    }
    return;
  }
  const int64_t per_img = static_cast<int64_t>(g0.h) * g0.w * cv_n;
  const int nb = batch_chunk(per_img, g0.n);
  const int64_t eb = elem_bytes(dtype);
  for (int n0 = 0; n0 < g0.n; n0 += nb) {
    DwGeom g = g0;
    g.n = n0 + nb <= g0.n ? nb : g0.n - n0;
    const char* dyb = static_cast<const char*>(dy) + static_cast<int64_t>(n0) * g.ho * g.wo * g.cout * eb;
    char* dxb = static_cast<char*>(dx) + static_cast<int64_t>(n0) * g.h * g.w * g.cin * eb;
    const DwDivs fd{FastDiv::make(cv_n), FastDiv::make(g.w), FastDiv::make(g.h)};
    const int grid = mcs ? dw_stats_grid(per_img * g.n, cv_n) : stream_grid(per_img * g.n, kDwBlock);
    dw_dispatch(dtype, vec, g.mult, [&](auto t, auto v, auto m) {
      using T = decltype(t);
      constexpr int V = decltype(v)::value, M = decltype(m)::value;
      if constexpr ((M > 1 && V == 2) || M == 1) {
        if (mcs) {  // channel-stationary 3 x 3
          dw_dgrad_kernel<T, V, M, 3, true><<<grid, kDwBlock, 0, st>>>(g, fd, reinterpret_cast<const T*>(dyb), wt,
                                                                        reinterpret_cast<T*>(dxb));
          return;
        }
      }
      dw_dgrad_kernel<T, V, M, 0><<<grid, kDwBlock, 0, st>>>(g, fd, reinterpret_cast<const T*>(dyb), wt,
                                                               reinterpret_cast<T*>(dxb));
    });
  }
}

// RTSEG_DW_WG_PAIR=0: the channel-multiplier wgrad on dw_wgrad_kernel (A/B)
static bool dw_wg_pair_enabled() {
  static const bool on = [] { const char* e = std::getenv("RTSEG_DW_WG_PAIR"); return !(e && e[0] == '0'); }();
  return on;
}

DwWgradPlan dw_wgrad_plan(const DwGeom& g, int dtype) {
  DwWgradPlan p;
  const int mt = mt_of(g.mult);
  if (dtype == kBF16 && mt > 1 && g.cin % 2 == 0 && g.kh * g.kw <= kMaxTaps && dw_wg_pair_enabled()) {
    p.pairs = 1;
    p.vec = 2 * mt;
    const int pv_n = g.cin / 2;
    p.lanes = 64;
    while (p.lanes > 1 && p.lanes / 2 >= pv_n) p.lanes /= 2;
    p.chunks = (pv_n + p.lanes - 1) / p.lanes;
    p.nt = kMaxTaps;
    p.tap_groups = 1;
    const int64_t npix = static_cast<int64_t>(g.n) * g.ho * g.wo;
    const int rows = kDwBlock / p.lanes;
    int64_t G = 1024 / p.chunks;
    if (const char* e = std::getenv("RTSEG_DW_WG_SLICES")) G = std::max(1, std::atoi(e)) / p.chunks;
    if (G > 1024) G = 1024;
    const int64_t gmax = (npix + static_cast<int64_t>(rows) * 16 - 1) / (static_cast<int64_t>(rows) * 16);
    if (G > gmax) G = gmax;
    if (G < 1) G = 1;
    p.slices = static_cast<int>(G);
    return p;
  }
  p.vec = dw_vec(dtype, g.cout);
  p.quad = mt == 1 && g.kh == 3 && g.kw == 3 && g.sh == 1 && g.sw == 1 && g.dw == 1 && dw_cs_enabled() ? 1 : 0;
  const int cv_n = g.cout / p.vec;
  p.lanes = 64;
  while (p.lanes > 1 && p.lanes / 2 >= cv_n) p.lanes /= 2;
  p.chunks = (cv_n + p.lanes - 1) / p.lanes;
  const int taps = g.kh * g.kw;
  p.nt = taps <= 3 ? 3 : taps <= 5 ? 5 : kMaxTaps;
  p.tap_groups = (taps + p.nt - 1) / p.nt;
  const int64_t npix = static_cast<int64_t>(g.n) * g.ho * (p.quad ? (g.wo + 3) / 4 : g.wo);  // work items
  const int rows = kDwBlock / p.lanes;
  // ~1024 blocks over 256 CUs, <= 512 slabs (the column reduce reads G rows), and
  // every block keeps >= 16 pixels per row
  int64_t G = 1024 / (static_cast<int64_t>(p.chunks) * p.tap_groups);
  int64_t gcap = 512;
  if (const char* e = std::getenv("RTSEG_DW_WG_SLICES1")) {  // (tuning experiments)
    gcap = std::max(1, std::atoi(e));
    G = gcap / (static_cast<int64_t>(p.chunks) * p.tap_groups);
  }
  if (G > gcap) G = gcap;
  const int64_t gmax = (npix + static_cast<int64_t>(rows) * 16 - 1) / (static_cast<int64_t>(rows) * 16);
  if (G > gmax) G = gmax;
  if (G < 1) G = 1;
  p.slices = static_cast<int>(G);
  return p;
}

void launch_dw_wgrad(const DwGeom& g, int dtype, const void* dy, const void* x, float* part, float* dw,
                     hipStream_t st) {
  // pixels are indexed in 32 bits; the binding rejects > 2^31 output pixels per call
  const DwWgradPlan p = dw_wgrad_plan(g, dtype);
  dim3 grid(p.slices, p.chunks, p.tap_groups);
  const DwDivs fd{FastDiv::make(1), FastDiv::make(g.wo), FastDiv::make(g.ho)};
  const int taps = g.kh * g.kw;
  const int rb = (taps * g.cout + 63) / 64;
  if (p.pairs) {
    const uint16_t* dyp = static_cast<const uint16_t*>(dy);
    const uint16_t* xp = static_cast<const uint16_t*>(x);
    switch (g.mult) {
      case 2: dw_wgrad_pair_kernel<2><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes); break;
      case 3: dw_wgrad_pair_kernel<3><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes); break;
      case 4: dw_wgrad_pair_kernel<4><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes); break;
      default: dw_wgrad_pair_kernel<6><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes); break;
    }
    dw_wgrad_reduce_kernel<<<rb, kRedWaves * 64, 0, st>>>(part, p.slices, taps, g.cout, dw);
    return;
  }
  if (p.quad) {
    const DwDivs fq{FastDiv::make(1), FastDiv::make((g.wo + 3) / 4), FastDiv::make(g.ho)};
    dw_dispatch(dtype, p.vec, 1, [&](auto t, auto v, auto) {
      using T = decltype(t);
      constexpr int V = decltype(v)::value;
      dw_wgrad_quad_kernel<T, V><<<grid, kDwBlock, 0, st>>>(g, fq, static_cast<const T*>(dy), static_cast<const T*>(x),
                                                           part, p.lanes);
    });
    dw_wgrad_reduce_kernel<<<rb, kRedWaves * 64, 0, st>>>(part, p.slices, taps, g.cout, dw);
    return;
  }
  dw_dispatch(dtype, p.vec, g.mult, [&](auto t, auto v, auto m) {
    using T = decltype(t);
    constexpr int V = decltype(v)::value, M = decltype(m)::value;
    const T* dyp = static_cast<const T*>(dy);
    const T* xp = static_cast<const T*>(x);
    if (p.nt == 3)
      dw_wgrad_kernel<T, V, M, 3><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes);
    else if (p.nt == 5)
      dw_wgrad_kernel<T, V, M, 5><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes);
    else
      dw_wgrad_kernel<T, V, M, kMaxTaps><<<grid, kDwBlock, 0, st>>>(g, fd, dyp, xp, part, p.lanes);
  });
  dw_wgrad_reduce_kernel<<<rb, kRedWaves * 64, 0, st>>>(part, p.slices, taps, g.cout, dw);
}

}  // namespace rtseg
