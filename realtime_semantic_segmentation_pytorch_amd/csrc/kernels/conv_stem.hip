// Stem convolution: the 3-channel 3x3 conv (pad 1, stride 1 or 2) that opens almost every model
// of the zoo -- DDRNet's conv1 (ddrnet.py:50; reference models/ddrnet.py:27-29), the STDC /
// BiSeNet / ResNet-style stems -- on bf16 MFMA, channels-last, gfx950.
//
// Why its own kernel: with Cin = 3 the implicit-GEMM K is 27, so the conv is pure streaming --
// DDRNet-23 at batch 32 reads a 0.4 GB image and writes a 2.1 GB output.  MIOpen/CK ran it at
// 0.95 ms and the BN statistics needed a second 2.1 GB pass (0.42 ms; profiles/r4_final/steady.txt);
// its weight gradient (igemm_wrw) another 0.87 ms.  Here:
//
//  * forward: K = 27 padded to 32 is ONE v_mfma_f32_16x16x32_bf16 per 16 pixels x 16 channels.
//    A = weights [cout][k] (registers, loaded once), B = im2col [k][pixel] gathered from an LDS
//    copy of the tile's input rows (dword loads; a pixel pair is 12 bytes, so every dword belongs
//    to one pair -- border pairs read as zeros).  C's lane holds 4 consecutive channels of one
//    pixel: 8-byte stores; BN statistics from the fp32 accumulators, one [2 x cout] slab row per
//    block (persistent grid).
//  * weight gradient: dW[k][cout] = sum_p im2col[p][k] dy[p][cout] with the pixels as the MFMA K
//    dimension (32 per MFMA); the dy tile is staged through LDS (16-byte global loads, 66-element
//    row pitch: conflict-free 16-bit column reads); per-block partials, then a column-sum kernel
//    (deterministic, no atomics).
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>
#include <type_traits>

namespace rtseg {

namespace {

using namespace mdev;
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

constexpr int kTW = 64;  // output tile width (4 MFMA pixel groups)

struct StemArgs {
  const uint16_t* x;   // [N][H][W][3] bf16
  const uint16_t* w;   // forward: [cout][3][3][3] bf16 (KRSC)
  const uint16_t* dy;  // weight gradient: [N][Ho][Wo][cout] bf16 (BN-fused: the BN OUTPUT's gradient)
  // BN-fused weight gradient (stem conv -> BN -> act): dy of the conv is the BN backward's dx,
  // k0 (g - k1 - (xb - mean) k2) with g = dy masked by the activation of xb * sc + sh
  const uint16_t* xb;  // the BN input (= this conv's output) [N][Ho][Wo][cout] bf16
  const float* kc;     // BN backward coefficients k0 | k1 | k2 [3 cout]
  const float* mi;     // mean | invstd [2 cout]
  const float* ss;     // scale | shift [2 cout]
  uint16_t* y;         // forward output [N][Ho][Wo][cout]
  float* part;         // forward: BN statistics slab [grid][2 * cout] or null; wgrad: [grid][32 * cout]
  int N, H, W, Ho, Wo, cout;
  int tilesW, tilesH, mtiles;
};

// per-lane LDS offsets of the 8 k entries 8h..8h+7 (k = ky * 9 + kx * 3 + ci) relative to the
// pixel's (row 0, tap 0) element; -1 for the zero padding k >= 27
template <int PX>
__device__ __forceinline__ void k_offsets(int h, int (&ko)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * h + j;
    const int ky = k / 9, r = k - 9 * ky;
    ko[j] = k < 27 ? ky * PX * 3 + r : -1;
  }
}

// input rows of an output tile [TH x kTW] into LDS: R rows x PX pixels (3 bf16 each) starting at
// input column ox0 * S - 2 (even, so dword-aligned); row r = input row oy0 * S - 1 + r
template <int S, int TH>
struct StemTile {
  static constexpr int R = (TH - 1) * S + 3;
  static constexpr int PX = (((kTW - 1) * S + 4) + 1) & ~1;
  static constexpr int DW = PX * 3 / 2;  // dwords per LDS row
};

template <int S, int TH>
__device__ __forceinline__ void stage_input(const StemArgs& a, uint32_t* l32, int n, int oy0, int ox0, int tid) {
  using T = StemTile<S, TH>;
  constexpr int kTotal = T::R * T::DW, kPer = (kTotal + 255) / 256;
  const int iw0 = ox0 * S - 2;
  const uint32_t* x32 = reinterpret_cast<const uint32_t*>(a.x);
  // all of this thread's loads in flight at once (compile-time count), then the LDS stores
  uint32_t v[kPer];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int d = tid + 256 * e;
    const int r = d / T::DW, dd = d - r * T::DW;
    const int ih = oy0 * S - 1 + r;
    const int iwp = iw0 + 2 * (dd / 3);
    v[e] = 0;
    if (d < kTotal && static_cast<unsigned>(ih) < static_cast<unsigned>(a.H) && iwp >= 0 && iwp < a.W)
      v[e] = x32[((static_cast<int64_t>(n) * a.H + ih) * a.W + iw0) * 3 / 2 + dd];
  }
#pragma unroll
  for (int e = 0; e < kPer; ++e)
    if (tid + 256 * e < kTotal) l32[tid + 256 * e] = v[e];
}

// input rows with every pixel padded to 4 channels (8 bytes, the 4th zero): pixel q of staged row r
// at uint2 index r * PX + q (the same rows / pixels as stage_input).  The forward's B fragment of
// lane half h -- taps 2h and 2h + 1, 4 channels each -- is then two 8-byte LDS reads instead of
// eight 2-byte gathers with their selects and packs (33 VALU per MFMA: profiles/r5_stempmc)
template <int S, int TH>
__device__ __forceinline__ void stage_input4(const StemArgs& a, uint2* l64, int n, int oy0, int ox0, int tid) {
  using T = StemTile<S, TH>;
  constexpr int PP = T::PX / 2;  // pixel pairs per row
  constexpr int kTotal = T::R * PP, kPer = (kTotal + 255) / 256;
  const int iw0 = ox0 * S - 2;
  const uint32_t* x32 = reinterpret_cast<const uint32_t*>(a.x);
  uint32_t d[kPer][3];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int pi = tid + 256 * e;
    const int r = pi / PP, pp = pi - r * PP;
    const int ih = oy0 * S - 1 + r, iwp = iw0 + 2 * pp;
    d[e][0] = d[e][1] = d[e][2] = 0u;
    if (pi < kTotal && static_cast<unsigned>(ih) < static_cast<unsigned>(a.H) && iwp >= 0 && iwp < a.W) {
      const uint32_t* src = x32 + ((static_cast<int64_t>(n) * a.H + ih) * a.W + iwp) * 3 / 2;
      d[e][0] = src[0]; d[e][1] = src[1]; d[e][2] = src[2];
    }
  }
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int pi = tid + 256 * e;
    if (pi >= kTotal) continue;
    const int r = pi / PP, pp = pi - r * PP;
    // two pixels (c0 c1 c2 | c0 c1 c2) -> (c0 c1 c2 0) (c0 c1 c2 0)
    *reinterpret_cast<uint4*>(l64 + r * T::PX + 2 * pp) =
        uint4{d[e][0], d[e][1] & 0xffffu, (d[e][1] >> 16) | (d[e][2] << 16), d[e][2] >> 16};
  }
}

// BNA: 0 = the raw conv output (+ STATS), else the training BN applied in the epilogue from the
// fp32 accumulators -- y = act(conv * scale + shift), act = BNA - 1 (none / ReLU / ReLU6): the
// stem BN's forward apply as a recompute of the (K = 27) conv from the 0.4 GB image instead of a
// pass over the 2.1 GB conv output (ops/bn.py; the conv output itself is still written by the
// statistics launch, for the BN backward)
// STATS 2: the stem BN's BACKWARD reduction with the conv recomputed -- per channel
// sum g' and sum g' (x - mean), g' = dy masked by act'(x * scale + shift) (act = BNA - 1), x = the
// bf16-rounded conv output exactly as the statistics launch stored it, read from the 0.4 GB image
// instead of the 2.1 GB stored x; no output stores.  Same [grid][2 cout] slab as the forward
// statistics (the BN backward finalize's input)
template <int S, int NT, int STATS, int BNA = 0>
__global__ void __launch_bounds__(256) stem_fwd_kernel(const StemArgs a) {
  static_assert(!(STATS == 1 && BNA), "statistics come from the raw conv output");
  static_assert(STATS != 2 || BNA != 0, "the backward reduction needs the activation");
  constexpr int TH = 8;  // 4 waves x 2 rows
  using T = StemTile<S, TH>;
  __shared__ __attribute__((aligned(16))) uint2 l64[T::R * T::PX];
  __shared__ float red[4][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 4, px = lane & 15;
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);

  // A fragments, K = tap * 4 + channel (the 4th channel zero): K block 0 = taps 0..7, block 1 =
  // tap 8 (lane half 0 only).  Row m of tile t is output channel cout_of(t, m) =
  // 4 NT (m >> 2) + 4 t + (m & 3), so the C rows 4h .. 4h + 3 of the NT tiles are the 4 NT
  // CONSECUTIVE channels 4 NT h .. of one pixel in a lane: 16-byte stores
  bf16x8_t wf[2][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int co = 4 * NT * (px >> 2) + 4 * t + (px & 3);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * h + j, tap = 8 * kb + (k >> 2), ch = k & 3;
        v[j] = (tap < 9 && ch < 3) ? static_cast<short>(a.w[co * 27 + tap * 3 + ch]) : short(0);
      }
      wf[kb][t] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  // this lane half's two taps (2h, 2h + 1): staged-pixel offsets from the output pixel's (row 0, tap 0)
  const int t0 = 2 * h, t1 = 2 * h + 1;
  const int off0 = (t0 / 3) * T::PX + t0 % 3 + 1, off1 = (t1 / 3) * T::PX + t1 % 3 + 1;
  const int off8 = 2 * T::PX + 2 + 1;  // tap 8 (lane half 0)

  float bsc[BNA ? NT : 1][4], bsh[BNA ? NT : 1][4];  // this lane's channels' BN scale / shift
  float bmu[STATS == 2 ? NT : 1][4];                   // ... and mean (backward reduction)
  if constexpr (BNA != 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 4 * NT * h + 4 * t + r;
        bsc[t][r] = a.ss[co];
        bsh[t][r] = a.ss[a.cout + co];
        if constexpr (STATS == 2) bmu[t][r] = a.mi[co];
      }
  }

  float ts[NT][4], tq[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) ts[t][r] = tq[t][r] = 0.f;

  for (int mt = lb; mt < a.mtiles; mt += G) {
    const int tx = mt % a.tilesW, t2 = mt / a.tilesW;
    const int n = t2 / a.tilesH, oy0 = (t2 % a.tilesH) * TH, ox0 = tx * kTW;
    __syncthreads();  // the previous tile's fragment reads are done
    stage_input4<S, TH>(a, l64, n, oy0, ox0, tid);
    __syncthreads();
#pragma unroll 2
    for (int g = 0; g < 8; ++g) {
      const int oyl = 2 * wid + (g >> 2), oxl = (g & 3) * 16 + px;
      const int pb = oyl * S * T::PX + oxl * S;
      const uint2 q0 = l64[pb + off0], q1 = l64[pb + off1], q8 = l64[pb + off8];
      const bf16x8_t bf = __builtin_bit_cast(bf16x8_t, uint4{q0.x, q0.y, q1.x, q1.y});
      const bf16x8_t bf8 = __builtin_bit_cast(bf16x8_t, h == 0 ? uint4{q8.x, q8.y, 0u, 0u} : uint4{0u, 0u, 0u, 0u});
      const int oy = oy0 + oyl, ox = ox0 + oxl;
      const bool ok = oy < a.Ho && ox < a.Wo;
      const int64_t poff = ((static_cast<int64_t>(n) * a.Ho + (ok ? oy : 0)) * a.Wo + (ok ? ox : 0)) * a.cout + 4 * NT * h;
      uint16_t* yp = a.y + poff;
      uint32_t gk[STATS == 2 ? 2 * NT : 1];  // the lane's 4 NT gradient values (STATS 2)
      if constexpr (STATS == 2) {
#pragma unroll
        for (int v = 0; v < 2 * NT; ++v) gk[v] = 0u;
        if (ok) {
          if constexpr (NT % 2 == 0) {
#pragma unroll
            for (int v = 0; v < NT / 2; ++v) {
              const uint4 q = reinterpret_cast<const uint4*>(a.dy + poff)[v];
              gk[4 * v] = q.x; gk[4 * v + 1] = q.y; gk[4 * v + 2] = q.z; gk[4 * v + 3] = q.w;
            }
          } else {
#pragma unroll
            for (int v = 0; v < NT; ++v) {
              const uint2 q = reinterpret_cast<const uint2*>(a.dy + poff)[v];
              gk[2 * v] = q.x; gk[2 * v + 1] = q.y;
            }
          }
        }
      }
      uint32_t pk[2 * NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4_t c = {0.f, 0.f, 0.f, 0.f};
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0][t], bf, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1][t], bf8, c, 0, 0, 0);
        if constexpr (STATS == 2) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t w2 = gk[2 * t + (r >> 1)];
            const float g = (r & 1) ? __uint_as_float(w2 & 0xffff0000u) : __uint_as_float(w2 << 16);
            const float xr = bf16_to_f32(f32_to_bf16(c[r]));  // the stored conv output's value
            const float z = fmaf(xr, bsc[t][r], bsh[t][r]);
            const bool live = BNA == 1 ? true : BNA == 2 ? z > 0.f : (z > 0.f && z < 6.f);
            const float gm = (ok && live) ? g : 0.f;
            ts[t][r] += gm;
            tq[t][r] = fmaf(gm, xr - bmu[t][r], tq[t][r]);
          }
          continue;
        }
        if constexpr (BNA != 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float z = fmaf(c[r], bsc[t][r], bsh[t][r]);
            c[r] = BNA == 2 ? fmaxf(z, 0.f) : BNA == 3 ? fminf(fmaxf(z, 0.f), 6.f) : z;
          }
        }
        pk[2 * t] = pack2(c[0], c[1]);
        pk[2 * t + 1] = pack2(c[2], c[3]);
        if constexpr (STATS == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float u = ok ? c[r] : 0.f;
            ts[t][r] += u;
            tq[t][r] = fmaf(u, u, tq[t][r]);
          }
        }
      }
      if (ok && STATS != 2 && a.y != nullptr) {  // null y: statistics only (the recompute path)
        if constexpr (NT % 2 == 0) {
#pragma unroll
          for (int v = 0; v < NT / 2; ++v)
            reinterpret_cast<uint4*>(yp)[v] = uint4{pk[4 * v], pk[4 * v + 1], pk[4 * v + 2], pk[4 * v + 3]};
        } else {
#pragma unroll
          for (int v = 0; v < NT; ++v) reinterpret_cast<uint2*>(yp)[v] = uint2{pk[2 * v], pk[2 * v + 1]};
        }
      }
    }
  }

  if constexpr (STATS) {
    // sum over the 16 pixel lanes of each row (DPP row_ror 8 / 4 / 2 / 1), then over the waves
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = ts[t][r], q = tq[t][r];
        s += dpp_f<0x128, 0xF>(s); q += dpp_f<0x128, 0xF>(q);
        s += dpp_f<0x124, 0xF>(s); q += dpp_f<0x124, 0xF>(q);
        s += dpp_f<0x122, 0xF>(s); q += dpp_f<0x122, 0xF>(q);
        s += dpp_f<0x121, 0xF>(s); q += dpp_f<0x121, 0xF>(q);
        if (px == 0) {
          red[wid][0][4 * NT * h + 4 * t + r] = s;
          red[wid][1][4 * NT * h + 4 * t + r] = q;
        }
      }
    __syncthreads();
    if (tid < 2 * a.cout) {
      const int sq = tid >= a.cout, c = sq ? tid - a.cout : tid;
      const float v = red[0][sq][c] + red[1][sq][c] + red[2][sq][c] + red[3][sq][c];
      a.part[static_cast<int64_t>(blockIdx.x) * 2 * a.cout + tid] = v;
    }
  }
}

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// BNF: 0 = plain dy; 1 / 2 / 3 = dy is the gradient of act(BN(conv output)) with act = none /
// ReLU / ReLU6, turned into the conv output's gradient while staged (the BN backward apply pass,
// fused: ops/bn.py hands its coefficients over instead of writing dx)
template <int BNF>
__device__ __forceinline__ float bn_dx(float g, float xv, int j, const float* k0, const float* k1, const float* k2,
                                       const float* mu, const float* sc, const float* sh) {
  if constexpr (BNF >= 2) {
    const float z = fmaf(xv, sc[j], sh[j]);
    if constexpr (BNF == 2) g = z > 0.f ? g : 0.f;
    else g = (z > 0.f && z < 6.f) ? g : 0.f;
  }
  return k0[j] * (g - k1[j] - (xv - mu[j]) * k2[j]);
}

// weight gradient partials: block b writes ws[b][k 32][cout] (k >= 27 rows are zero)
// RC (BN-fused only): the BN input x is not read back but recomputed from the staged image rows
// (one v_mfma_f32_16x16x32_bf16 per 16 pixels x 16 channels, the forward kernel's fragments) and
// rounded to bf16 exactly as the forward's statistics launch stored it
template <int S, int NT, int BNF = 0, int RC = 0>
__global__ void __launch_bounds__(256) stem_wgrad_kernel(const StemArgs a) {
  static_assert(RC == 0 || BNF != 0, "the recompute feeds the fused BN backward");
  constexpr int TH = 4;  // 4 waves x 1 row of 64 pixels (2 MFMA K-steps of 32 pixels)
  constexpr int CP = 16 * NT + 2;  // dy row pitch (elements)
  constexpr int XP = 16 * NT + 8;  // recomputed-x row pitch (elements; 16-byte rows)
  using T = StemTile<S, TH>;
  __shared__ uint32_t l32[T::R * T::DW];
  __shared__ uint16_t dyl[TH * kTW * CP];
  __shared__ __attribute__((aligned(16))) uint16_t xl[RC ? TH * kTW * XP : 8];
  const uint16_t* l16 = reinterpret_cast<const uint16_t*>(l32);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 4, c16 = lane & 15;
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);
  constexpr int C = 16 * NT;

  // A rows: k = 16 mt + c16 -> LDS offset of (ky, kx, ci) relative to the pixel's element
  int ka[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int k = 16 * m + c16;
    const int ky = k / 9, r = k - 9 * ky;
    ka[m] = k < 27 ? ky * T::PX * 3 + r : -1;
  }
  f32x4_t acc[2][NT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[m][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  constexpr int V = C / 8;  // 16-byte vectors per pixel
  // BN-fused: a thread always stages the same channel vector (V divides 256): its coefficients
  // stay in registers
  static_assert(BNF == 0 || 256 % V == 0, "BN-fused stem wgrad needs V | 256");
  bf16x8_t wf[RC ? NT : 1];  // RC: forward A fragments (see stem_fwd_kernel)
  int kof[8];
  if constexpr (RC != 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      s16x8_t v;
      const int co = 4 * NT * (c16 >> 2) + 4 * t + (c16 & 3);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * h + j;
        v[j] = k < 27 ? static_cast<short>(a.w[co * 27 + k]) : short(0);
      }
      wf[t] = __builtin_bit_cast(bf16x8_t, v);
    }
    k_offsets<T::PX>(h, kof);
  }
  float k0[8], k1[8], k2[8], mu[8], sc[8], sh[8];
  if constexpr (BNF != 0) {
    const int c0 = 8 * (tid % V);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k0[j] = a.kc[c0 + j]; k1[j] = a.kc[C + c0 + j]; k2[j] = a.kc[2 * C + c0 + j];
      mu[j] = a.mi[c0 + j]; sc[j] = a.ss[c0 + j]; sh[j] = a.ss[C + c0 + j];
    }
  }

  for (int mt = lb; mt < a.mtiles; mt += G) {
    const int tx = mt % a.tilesW, t2 = mt / a.tilesW;
    const int n = t2 / a.tilesH, oy0 = (t2 % a.tilesH) * TH, ox0 = tx * kTW;
    __syncthreads();
    stage_input<S, TH>(a, l32, n, oy0, ox0, tid);
    // dy tile [TH * 64 pixels][C] (pixels past the image read as zeros), loads all in flight
    constexpr int kPer = TH * kTW * V / 256;
    static_assert(kPer * 256 == TH * kTW * V, "dy staging");
    uint4 q[kPer];
    uint4 xq[BNF != 0 ? kPer : 1];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      const int p = e / V, v = e - p * V;
      const int oy = oy0 + p / kTW, ox = ox0 + (p % kTW);
      q[i] = uint4{0u, 0u, 0u, 0u};
      if constexpr (BNF != 0) xq[i] = uint4{0u, 0u, 0u, 0u};
      if (oy < a.Ho && ox < a.Wo) {
        const int64_t off = ((static_cast<int64_t>(n) * a.Ho + oy) * a.Wo + ox) * C + 8 * v;
        q[i] = *reinterpret_cast<const uint4*>(a.dy + off);
        if constexpr (BNF != 0 && RC == 0) xq[i] = *reinterpret_cast<const uint4*>(a.xb + off);
      }
    }
    if constexpr (RC != 0) {
      // the tile's conv output, recomputed while the dy loads are in flight: wave wid = tile row
      __syncthreads();  // every wave's image rows are staged
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        const int oxl = gi * 16 + c16;
        const int base = wid * S * T::PX * 3 + (oxl * S + 1) * 3;
        s16x8_t b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = kof[j] >= 0 ? static_cast<short>(l16[base + kof[j]]) : short(0);
        const bf16x8_t bf = __builtin_bit_cast(bf16x8_t, b);
        uint16_t* xp = xl + (wid * kTW + oxl) * XP + 4 * NT * h;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x4_t c = {0.f, 0.f, 0.f, 0.f};
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t], bf, c, 0, 0, 0);
          *reinterpret_cast<uint2*>(xp + 4 * t) = uint2{pack2(c[0], c[1]), pack2(c[2], c[3])};
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int e = tid + 256 * i;
        const int p = e / V, v = e - p * V;
        xq[i] = *reinterpret_cast<const uint4*>(xl + p * XP + 8 * v);
      }
    }
    if constexpr (BNF != 0) {
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int e = tid + 256 * i;
        const int p = e / V;
        const int oy = oy0 + p / kTW, ox = ox0 + (p % kTW);
        if (!(oy < a.Ho && ox < a.Wo)) continue;  // outside the tensor: stays 0
        const uint32_t gw[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
        const uint32_t xw[4] = {xq[i].x, xq[i].y, xq[i].z, xq[i].w};
        uint32_t ow[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float lo = bn_dx<BNF>(bf_lo(gw[u]), bf_lo(xw[u]), 2 * u, k0, k1, k2, mu, sc, sh);
          const float hi = bn_dx<BNF>(bf_hi(gw[u]), bf_hi(xw[u]), 2 * u + 1, k0, k1, k2, mu, sc, sh);
          ow[u] = pack2(lo, hi);
        }
        q[i] = uint4{ow[0], ow[1], ow[2], ow[3]};
      }
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      const int p = e / V, v = e - p * V;
      uint32_t* d = reinterpret_cast<uint32_t*>(dyl + p * CP + 8 * v);
      d[0] = q[i].x; d[1] = q[i].y; d[2] = q[i].z; d[3] = q[i].w;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // K = 32 pixels: lane half h holds pixels 8h .. 8h + 7 of this step
      const int p0 = wid * kTW + ks * 32 + 8 * h;  // tile pixel index
      const int oxl0 = ks * 32 + 8 * h;
      bf16x8_t af[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        s16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int base = wid * S * T::PX * 3 + ((oxl0 + j) * S + 1) * 3;
          v[j] = ka[m] >= 0 ? static_cast<short>(l16[base + ka[m]]) : short(0);
        }
        af[m] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        s16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = static_cast<short>(dyl[(p0 + j) * CP + 16 * t + c16]);
        const bf16x8_t bfr = __builtin_bit_cast(bf16x8_t, v);
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr, acc[m][t], 0, 0, 0);
      }
    }
  }

  // block partial: C[k = 16 m + 4 h + r][cout = 16 t + c16], summed over the 4 waves through LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(dyl);  // [4 waves][32][C] fp32 <= 32 KiB
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wid * 32 + 16 * m + 4 * h + r) * C + 16 * t + c16] = acc[m][t][r];
  __syncthreads();
  for (int e = tid; e < 32 * C; e += 256) {
    const float v = red[e] + red[32 * C + e] + red[64 * C + e] + red[96 * C + e];
    a.part[static_cast<int64_t>(blockIdx.x) * 32 * C + e] = v;
  }
}

// dw[cout][ci][ky][kx] (or KRSC when channels_last) = sum over blocks of ws[b][k][cout]; block =
// 16 row slices x 64 entries, the slices summed through LDS in a fixed order (deterministic)
__global__ void __launch_bounds__(1024) stem_wgrad_reduce(const float* __restrict__ ws, int rows, int cout,
                                                          float* __restrict__ dw, int krsc) {
  __shared__ float red[16][64];
  const int ei = threadIdx.x & 63, rs = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + ei;  // e = k * cout + co
  const int n = 27 * cout;
  float s = 0.f;
  if (e < n)
    for (int b = rs; b < rows; b += 16) s += ws[static_cast<int64_t>(b) * 32 * cout + e];
  red[rs][ei] = s;
  __syncthreads();
  if (rs != 0 || e >= n) return;
#pragma unroll
  for (int r = 1; r < 16; ++r) s += red[r][ei];
  const int k = e / cout, co = e - k * cout;
  const int ky = k / 9, kx = (k / 3) % 3, ci = k % 3;
  dw[krsc ? co * 27 + k : co * 27 + ci * 9 + ky * 3 + kx] = s;
}

bool stem_fill(StemArgs& k, const ConvGeom& g, int th) {
  if (g.cin != 3 || g.kh != 3 || g.kw != 3 || g.ph != 1 || g.pw != 1 || g.dh != 1 || g.dw != 1) return false;
  if (g.sh != g.sw || (g.sh != 1 && g.sh != 2)) return false;
  if (g.cout % 16 != 0 || g.cout > 64 || g.w_in % 2 != 0) return false;
  k.N = g.n; k.H = g.h; k.W = g.w_in; k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  k.tilesW = (g.wo + kTW - 1) / kTW;
  k.tilesH = (g.ho + th - 1) / th;
  k.mtiles = g.n * k.tilesW * k.tilesH;
  return true;
}

int stem_grid(int mtiles) { return std::max(1, std::min(mtiles, 2048)); }

template <int S, int NT>
void fwd_launch(const StemArgs& k, int grid, hipStream_t st, int bna) {
  if (k.part != nullptr) stem_fwd_kernel<S, NT, 1><<<grid, 256, 0, st>>>(k);
  else if (bna == 1) stem_fwd_kernel<S, NT, 0, 1><<<grid, 256, 0, st>>>(k);
  else if (bna == 2) stem_fwd_kernel<S, NT, 0, 2><<<grid, 256, 0, st>>>(k);
  else if (bna == 3) stem_fwd_kernel<S, NT, 0, 3><<<grid, 256, 0, st>>>(k);
  else stem_fwd_kernel<S, NT, 0><<<grid, 256, 0, st>>>(k);
}

template <int S>
void fwd_dispatch(const StemArgs& k, int grid, hipStream_t st, int bna) {
  switch (k.cout / 16) {
    case 1: fwd_launch<S, 1>(k, grid, st, bna); break;
    case 2: fwd_launch<S, 2>(k, grid, st, bna); break;
    case 3: fwd_launch<S, 3>(k, grid, st, bna); break;
    default: fwd_launch<S, 4>(k, grid, st, bna); break;
  }
}

template <int S, int BNF, int RC>
void wgrad_dispatch(const StemArgs& k, int grid, hipStream_t st) {
  switch (k.cout / 16) {
    case 1: stem_wgrad_kernel<S, 1, BNF, RC><<<grid, 256, 0, st>>>(k); break;
    case 2: stem_wgrad_kernel<S, 2, BNF, RC><<<grid, 256, 0, st>>>(k); break;
    case 3:
      if constexpr (BNF == 0) stem_wgrad_kernel<S, 3, 0><<<grid, 256, 0, st>>>(k);  // (BN-fused: V = 6 does not divide 256)
      break;
    default: stem_wgrad_kernel<S, 4, BNF, RC><<<grid, 256, 0, st>>>(k); break;
  }
}

template <int BNF>
void wgrad_dispatch_s(const StemArgs& k, int grid, int s, hipStream_t st, bool rc = false) {
  if constexpr (BNF == 0) {
    if (s == 2) wgrad_dispatch<2, 0, 0>(k, grid, st);
    else wgrad_dispatch<1, 0, 0>(k, grid, st);
  } else if (rc) {
    if (s == 2) wgrad_dispatch<2, BNF, 1>(k, grid, st);
    else wgrad_dispatch<1, BNF, 1>(k, grid, st);
  } else {
    if (s == 2) wgrad_dispatch<2, BNF, 0>(k, grid, st);
    else wgrad_dispatch<1, BNF, 0>(k, grid, st);
  }
}

}  // namespace

bool conv_stem_supported(const ConvGeom& g) {
  StemArgs k{};
  return stem_fill(k, g, 8);
}

int conv_stem_slabs(const ConvGeom& g) {
  StemArgs k{};
  if (!stem_fill(k, g, 8)) return 0;
  return stem_grid(k.mtiles);
}

void launch_conv_stem_fwd(const ConvGeom& g, hipStream_t st) {
  StemArgs k{};
  if (!stem_fill(k, g, 8)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = g.part;
  k.ss = g.scale_shift;  // the BN epilogue (no statistics then)
  const int bna = g.scale_shift != nullptr ? g.act + 1 : 0;
  const int grid = stem_grid(k.mtiles);
  if (g.sh == 2) fwd_dispatch<2>(k, grid, st, bna);
  else fwd_dispatch<1>(k, grid, st, bna);
}

// stem BN backward reduction with the conv recomputed (STATS 2): g.x = image, g.w = KRSC weights,
// g.y = dy (the BN output's gradient), part [conv_stem_slabs(g)][2 cout]
void launch_conv_stem_bn_sums(const ConvGeom& g, const float* mean_invstd, const float* scale_shift, int act,
                              float* part, hipStream_t st) {
  StemArgs k{};
  if (!stem_fill(k, g, 8)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.dy = static_cast<const uint16_t*>(g.y);
  k.mi = mean_invstd;
  k.ss = scale_shift;
  k.part = part;
  const int grid = stem_grid(k.mtiles);
  auto go = [&](auto s_tag) {
    constexpr int S = decltype(s_tag)::value;
    auto nt = [&](auto nt_tag) {
      constexpr int NT = decltype(nt_tag)::value;
      if (act == 1) stem_fwd_kernel<S, NT, 2, 2><<<grid, 256, 0, st>>>(k);
      else if (act == 2) stem_fwd_kernel<S, NT, 2, 3><<<grid, 256, 0, st>>>(k);
      else stem_fwd_kernel<S, NT, 2, 1><<<grid, 256, 0, st>>>(k);
    };
    switch (k.cout / 16) {
      case 1: nt(std::integral_constant<int, 1>{}); break;
      case 2: nt(std::integral_constant<int, 2>{}); break;
      case 3: nt(std::integral_constant<int, 3>{}); break;
      default: nt(std::integral_constant<int, 4>{}); break;
    }
  };
  if (g.sh == 2) go(std::integral_constant<int, 2>{});
  else go(std::integral_constant<int, 1>{});
}

int64_t conv_stem_wgrad_ws_elems(const ConvGeom& g) {
  StemArgs k{};
  if (!stem_fill(k, g, 4)) return 0;
  return static_cast<int64_t>(stem_grid(k.mtiles)) * 32 * g.cout;
}

// g.x = x [N,H,W,3], g.y = dy [N,Ho,Wo,Cout]; ws of conv_stem_wgrad_ws_elems(g) floats
void launch_conv_stem_wgrad(const ConvGeom& g, float* ws, float* dw, bool krsc, hipStream_t st,
                            const StemBnBwd* bn) {
  StemArgs k{};
  if (!stem_fill(k, g, 4)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.dy = static_cast<const uint16_t*>(g.y);
  k.part = ws;
  const int grid = stem_grid(k.mtiles);
  if (bn == nullptr) {
    wgrad_dispatch_s<0>(k, grid, g.sh, st);
  } else {
    k.xb = static_cast<const uint16_t*>(bn->xb);
    k.w = static_cast<const uint16_t*>(bn->w);  // non-null: recompute x instead of reading xb
    k.kc = bn->kcoef; k.mi = bn->mean_invstd; k.ss = bn->scale_shift;
    const bool rc = bn->w != nullptr;
    if (bn->act == 0) wgrad_dispatch_s<1>(k, grid, g.sh, st, rc);
    else if (bn->act == 1) wgrad_dispatch_s<2>(k, grid, g.sh, st, rc);
    else wgrad_dispatch_s<3>(k, grid, g.sh, st, rc);
  }
  const int n = 27 * g.cout;
  stem_wgrad_reduce<<<(n + 63) / 64, 1024, 0, st>>>(ws, grid, g.cout, dw, krsc ? 1 : 0);
}

}  // namespace rtseg
