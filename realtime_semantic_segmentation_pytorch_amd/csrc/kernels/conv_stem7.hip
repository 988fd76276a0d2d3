// The 7 x 7 / stride-2 / pad-3 ResNet stem (3 -> 64 channels: torchvision-style encoders -- the KD
// teacher's ResNet-101 in BASELINE config 5, reference models/__init__.py:102-122, SMP encoders,
// ICNet / SwiftNet / ShelfNet backbones) forward on bf16 MFMA, channels-last, gfx950, with an
// optional inference BN (+ ReLU / ReLU6) epilogue on the fp32 accumulators.
//
// MIOpen runs it channels-last at ~143 TFLOP/s (1.1 ms per batch-16 1024 x 2048 call; NCHW 1.7 ms,
// tools/bench_stem7.py) and the BN + ReLU is another pass over the 1 GB output.  The conv is pure
// streaming: 0.2 GB of image in, 1 GB out.  Same scheme as the 3 x 3 stem (conv_stem.hip):
//  * implicit GEMM with K = tap * 4 + channel (the 4th channel zero): 49 taps = 7 K-blocks of 32, one
//    v_mfma_f32_16x16x32_bf16 each per 16 pixels x 16 output channels; lane half h of K-block kb holds
//    taps 8 kb + 2h and 8 kb + 2h + 1 (taps >= 49 read as zeros);
//  * A = weights in registers (loaded once per block: 7 x NT fragments);
//  * B = the tile's input rows staged once in LDS with every pixel padded to 4 channels (8 bytes),
//    so a lane's 8 K values are two 8-byte LDS reads;
//  * C: a lane ends with 4 NT consecutive channels of one pixel -> 16-byte stores.
// Tile: 8 output rows x 64 pixels per 256-thread block (4 waves x 2 rows), persistent grid.
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>

namespace rtseg {

namespace {

using namespace mdev;
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));

constexpr int kKS = 7, kPad = 3, kTaps = kKS * kKS, kKB = (kTaps + 7) / 8;  // 7 K-blocks
constexpr int kTW = 64, kTH = 8;

struct Stem7Args {
  const uint16_t* x;   // [N][H][W][3] bf16
  const uint16_t* w;   // [cout][7][7][3] bf16 (KRSC)
  const float* ss;     // scale | shift [2 cout] (inference BN epilogue) or null
  uint16_t* y;         // [N][Ho][Wo][cout]
  int N, H, W, Ho, Wo, cout;
  int tilesW, tilesH, mtiles;
};

// staged geometry: R rows of PX pixels; row r = input row oy0 * S - 3 + r, pixel q = input column
// ox0 * S - 4 + q (even start: 12-byte pixel pairs are dword-aligned), so input column
// ox * S - 3 + tx is staged pixel (ox - ox0) * S + tx + 1
template <int S>
struct Stem7Tile {
  static constexpr int R = (kTH - 1) * S + kKS;
  static constexpr int PX = (((kTW - 1) * S + kKS + 1) + 1) & ~1;
};

template <int S>
__device__ __forceinline__ void stage7(const Stem7Args& a, uint2* l64, int n, int oy0, int ox0, int tid) {
  using T = Stem7Tile<S>;
  constexpr int PP = T::PX / 2;
  constexpr int kTotal = T::R * PP, kPer = (kTotal + 255) / 256;
  const int iw0 = ox0 * S - (kPad + 1);
  const uint32_t* x32 = reinterpret_cast<const uint32_t*>(a.x);
  uint32_t d[kPer][3];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int pi = tid + 256 * e;
    const int r = pi / PP, pp = pi - r * PP;
    const int ih = oy0 * S - kPad + r, iwp = iw0 + 2 * pp;
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

// BNA: 0 = the raw conv, else act(conv * scale + shift) with act = BNA - 1 (none / ReLU / ReLU6)
template <int S, int NT, int BNA>
__global__ void __launch_bounds__(256) stem7_fwd_kernel(const Stem7Args a) {
  using T = Stem7Tile<S>;
  __shared__ __attribute__((aligned(16))) uint2 l64[T::R * T::PX];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 4, px = lane & 15;
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);

  // A fragments: row m = px of tile t is output channel 4 NT (px >> 2) + 4 t + (px & 3); lane half
  // h of K-block kb holds K = 8h .. 8h + 7 = taps 8 kb + 2h (+ 1), 4 channels each
  bf16x8_t wf[kKB][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int co = 4 * NT * (px >> 2) + 4 * t + (px & 3);
#pragma unroll
    for (int kb = 0; kb < kKB; ++kb) {
      s16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * kb + 2 * h + (j >> 2), ch = j & 3;
        v[j] = (tap < kTaps && ch < 3) ? static_cast<short>(a.w[co * kTaps * 3 + tap * 3 + ch]) : short(0);
      }
      wf[kb][t] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  // staged-pixel offsets of this lane half's two taps per K-block (relative to the output pixel's
  // (row 0, column 0) staged pixel); -1: a tap past 48 (zero)
  int off[kKB][2];
#pragma unroll
  for (int kb = 0; kb < kKB; ++kb)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tap = 8 * kb + 2 * h + j;
      off[kb][j] = tap < kTaps ? (tap / kKS) * T::PX + tap % kKS + 1 : -1;
    }

  float bsc[BNA ? NT : 1][4], bsh[BNA ? NT : 1][4];
  if constexpr (BNA != 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 4 * NT * h + 4 * t + r;
        bsc[t][r] = a.ss[co];
        bsh[t][r] = a.ss[a.cout + co];
      }
  }

  for (int mt = lb; mt < a.mtiles; mt += G) {
    const int tx = mt % a.tilesW, t2 = mt / a.tilesW;
    const int n = t2 / a.tilesH, oy0 = (t2 % a.tilesH) * kTH, ox0 = tx * kTW;
    __syncthreads();  // the previous tile's fragment reads are done
    stage7<S>(a, l64, n, oy0, ox0, tid);
    __syncthreads();
#pragma unroll 2
    for (int g = 0; g < 8; ++g) {
      const int oyl = 2 * wid + (g >> 2), oxl = (g & 3) * 16 + px;
      const int pb = oyl * S * T::PX + oxl * S;
      f32x4_t c[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) c[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < kKB; ++kb) {
        uint2 q0 = make_uint2(0u, 0u), q1 = make_uint2(0u, 0u);
        if (off[kb][0] >= 0) q0 = l64[pb + off[kb][0]];
        if (off[kb][1] >= 0) q1 = l64[pb + off[kb][1]];
        const bf16x8_t bf = __builtin_bit_cast(bf16x8_t, uint4{q0.x, q0.y, q1.x, q1.y});
#pragma unroll
        for (int t = 0; t < NT; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kb][t], bf, c[t], 0, 0, 0);
      }
      const int oy = oy0 + oyl, ox = ox0 + oxl;
      if (oy >= a.Ho || ox >= a.Wo) continue;
      uint32_t pk[2 * NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = c[t][r];
          if constexpr (BNA != 0) {
            const float z = fmaf(v[r], bsc[t][r], bsh[t][r]);
            v[r] = BNA == 2 ? fmaxf(z, 0.f) : BNA == 3 ? fminf(fmaxf(z, 0.f), 6.f) : z;
          }
        }
        pk[2 * t] = pack2(v[0], v[1]);
        pk[2 * t + 1] = pack2(v[2], v[3]);
      }
      uint16_t* yp = a.y + ((static_cast<int64_t>(n) * a.Ho + oy) * a.Wo + ox) * a.cout + 4 * NT * h;
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

bool stem7_fill(Stem7Args& k, const ConvGeom& g) {
  if (g.cin != 3 || g.kh != kKS || g.kw != kKS || g.ph != kPad || g.pw != kPad || g.dh != 1 || g.dw != 1) return false;
  if (g.sh != g.sw || (g.sh != 1 && g.sh != 2)) return false;
  if (g.cout % 16 != 0 || g.cout > 64 || g.w_in % 2 != 0) return false;
  k.N = g.n; k.H = g.h; k.W = g.w_in; k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  k.tilesW = (g.wo + kTW - 1) / kTW;
  k.tilesH = (g.ho + kTH - 1) / kTH;
  k.mtiles = g.n * k.tilesW * k.tilesH;
  return true;
}

template <int S, int NT>
void stem7_launch(const Stem7Args& k, int grid, hipStream_t st, int bna) {
  if (bna == 1) stem7_fwd_kernel<S, NT, 1><<<grid, 256, 0, st>>>(k);
  else if (bna == 2) stem7_fwd_kernel<S, NT, 2><<<grid, 256, 0, st>>>(k);
  else if (bna == 3) stem7_fwd_kernel<S, NT, 3><<<grid, 256, 0, st>>>(k);
  else stem7_fwd_kernel<S, NT, 0><<<grid, 256, 0, st>>>(k);
}

template <int S>
void stem7_dispatch(const Stem7Args& k, int grid, hipStream_t st, int bna) {
  switch (k.cout / 16) {
    case 1: stem7_launch<S, 1>(k, grid, st, bna); break;
    case 2: stem7_launch<S, 2>(k, grid, st, bna); break;
    case 3: stem7_launch<S, 3>(k, grid, st, bna); break;
    default: stem7_launch<S, 4>(k, grid, st, bna); break;
  }
}

}  // namespace

bool conv_stem7_supported(const ConvGeom& g) {
  Stem7Args k{};
  return stem7_fill(k, g);
}

void launch_conv_stem7_fwd(const ConvGeom& g, hipStream_t st) {
  Stem7Args k{};
  if (!stem7_fill(k, g)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.ss = g.scale_shift;
  const int bna = g.scale_shift != nullptr ? g.act + 1 : 0;
  const int grid = std::max(1, std::min(k.mtiles, 2048));
  if (g.sh == 2) stem7_dispatch<2>(k, grid, st, bna);
  else stem7_dispatch<1>(k, grid, st, bna);
}

}  // namespace rtseg
