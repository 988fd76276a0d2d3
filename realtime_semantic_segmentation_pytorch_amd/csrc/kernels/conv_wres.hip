// Weights-resident halo convolution for 3x3 stride-1 convs that reduce over 64 channels: the
// forward of a Cin = 64 conv and the data gradient of a Cout = 64 conv -- DDRNet-23's layer1
// RB blocks at 256 x 512 (ddrnet.py:168-191), the ResNet-18/34 layer1 BasicBlocks of the
// backbone models (models/backbone.py), SwiftNet / ShelfNet / LinkNet decoders.
//
// Why a third conv kernel (profiles/r4_conv): on these layers the gather kernel (conv_igemm.hip)
// runs at 20 % of MFMA peak -- every K-step moves the (tap, 64-channel) slice of 512 gathered
// pixels + the weight slice through LDS-DMA (73 KiB per 4.2 MFLOP) with one step of prefetch,
// and waits on it; the halo kernel (conv_halo.hip) cuts the pixel traffic 9x but still streams a
// weight slice per K-step.  With 64 reduction channels the whole weight slice of a 64-channel
// output tile is 9 x 64 x 64 bf16 = 72 KiB: it is loaded into LDS ONCE per block and stays, and
// the only traffic left is the input halo, double-buffered a whole tile ahead.  A block needs one
// barrier per 256-pixel tile (not per K-step); inside a tile the 8 waves only read LDS.
//
//  * block = 8 waves, persistent over pixel tiles of TH x TW = 8 x 32 outputs for one 64-channel
//    output slice; wave w owns output row w of the tile (32 pixels = one MFMA column block) x all
//    64 channels: per (tap, 16-deep K sub-step) one B fragment (halo) + two A fragments (weights)
//    feed two v_mfma_f32_32x32x16_bf16;
//  * LDS: weights [tap][co 64][64 ch] (576 rows of 128 B) + two halo buffers of (TH+2) x (TW+2)
//    rows (344 with the DMA round-up); chunk c of row r lives at c ^ ((r >> 1) & 7) (source-side
//    swizzle), so both fragment reads are bank-conflict free for any tap shift;
//  * halo rows come in by LDS-DMA through a range-checked buffer resource: padding rows get an
//    out-of-range offset and read zeros -- no zero page, no per-lane select of a source;
//  * epilogue of tile t runs after tile t+1's barrier, before its halo DMA issue (stores and the
//    next halo retire under tile t+1's MFMAs); optional residual-gradient addend (dgrad) or BN
//    statistics (training forward: one [2 x Cout] slab row per block, deterministic).
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>
#include <cstdlib>

namespace rtseg {

namespace {

using namespace mdev;

constexpr int kTH = 8, kTW = 32;                      // output tile
constexpr int kHH = kTH + 2, kHW = kTW + 2;           // halo tile (3 x 3 footprint)
constexpr int kHRows = kHH * kHW;                     // 340
constexpr int kHInstr = (kHRows + 7) / 8;             // 43 DMA instructions (8 rows each)
constexpr int kHStage = kHInstr * 8 * 8;              // 16-byte chunks per halo buffer (344 rows)
constexpr int kWRows = 9 * 64;                        // weight rows [tap][co]
constexpr int kWStage = kWRows * 8;                   // 16-byte chunks of the weight slice
static_assert((kWStage + 2 * kHStage) * 16 <= 160 * 1024, "LDS budget");

struct WresArgs {
  const uint16_t* x;       // gathered operand [N][H][W][64] (forward: x, dgrad: dy)
  const uint16_t* w;       // [cout][3][3][64] bf16 (forward: KRSC weights; dgrad: [Cin][KH][KW][Cout])
  uint16_t* y;             // [N][Ho][Wo][cout]
  float* part;             // BN statistics slab [grid / ntiles][2 * cout], or null
  const uint16_t* addend;  // bf16 tensor of y's layout added to the result, or null
  const uint8_t* amask;    // bit mask of the addend (mask_addend4), or null
  const float* ss;         // STATS 2 (inference): BN scale [cout] | shift [cout]; the addend is the residual
  int act;                 // STATS 2: activation after the residual
  int H, W;                // gathered operand
  int Ho, Wo, cout;        // output
  int dh0, dw0;            // halo origin: input row of output row oy (tap-relative offset 0)
  int tilesW, tilesH, mtiles, ntiles;
  uint32_t xbytes;         // bytes of the gathered operand (< 2^31: buffer-resource range)
};

// one LDS-DMA through a buffer resource: 64 lanes x 16 B at M0 + 16 * lane; a voffset past the
// resource's range reads zeros (the image border)
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t lds_dst) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_dst);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(dst)
      : "memory");
}

// STATS: 0 = plain, 1 = BN statistics slab (training forward), 2 = inference BN epilogue
// act(y * scale + shift + residual) (forward only)
// NW waves; wave w owns TJ = kTH / NW consecutive output rows of the tile (32 pixels each) x all
// 64 channels (TI = 2 channel tiles); PD = fragment prefetch distance in (tap, K sub-step) steps
template <int STATS, int FLIP, int NW, int PD>
__global__ void __launch_bounds__(NW * 64) wres_conv_kernel(const WresArgs a) {
  constexpr int TJ = kTH / NW;
  static_assert(TJ * NW == kTH && PD >= 1 && PD <= 4, "wave tiling / prefetch");
  constexpr int NSTEP = 36;  // 9 taps x 4 sixteen-channel sub-steps
  __shared__ uint4 lds[kWStage + 2 * kHStage];
  uint4* const wl = lds;
  uint4* const hl = lds + kWStage;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);
  const int ntile = lb % a.ntiles;
  const int co0 = ntile * 64;
  const int mstep = G / a.ntiles;
  const int mfirst = lb / a.ntiles;
  const int my_tiles = mfirst < a.mtiles ? (a.mtiles - mfirst + mstep - 1) / mstep : 0;
  const int lr8 = lane >> 3, lch = lane & 7;

  // ---- weights of this block's 64 output channels, once: LDS row tap * 64 + co
  for (int e = wid; e < kWRows / 8; e += NW) {
    const int row = e * 8 + lr8;
    const int tap = row >> 6, co = row & 63;
    const int lc = lch ^ ((row >> 1) & 7);
    const uint16_t* src = a.w + (static_cast<int64_t>(co0 + co) * 9 + tap) * 64 + lc * 8;
    dma16(src, lds_addr(wl) + e * 1024);
  }

  // ---- halo DMA of tile mt into buffer hb
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, static_cast<int>(a.xbytes), 0x00020000);
  auto tile_xyz = [&](int mt, int& n, int& oy0, int& ox0) {
    const int tx = mt % a.tilesW;
    const int t2 = mt / a.tilesW;
    n = t2 / a.tilesH;
    oy0 = (t2 % a.tilesH) * kTH;
    ox0 = tx * kTW;
  };
  auto halo_dma = [&](int mt, int hb) {
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    const uint32_t base = lds_addr(hl + hb * kHStage);
    for (int e = wid; e < kHInstr; e += NW) {
      const int r = e * 8 + lr8;
      const int hy = r / kHW, hx = r - hy * kHW;
      const int ih = oy0 + a.dh0 + hy, iw = ox0 + a.dw0 + hx;
      const bool ok = r < kHRows && static_cast<unsigned>(ih) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(a.W);
      const int lc = lch ^ ((r >> 1) & 7);
      const uint32_t voff =
          ok ? static_cast<uint32_t>(((n * a.H + ih) * a.W + iw) * 64 + lc * 8) * 2u : 0x80000000u;
      bdma16(xr, voff, base + e * 1024);
    }
  };

  // ---- fragment geometry: lane -> pixel frow of each of the wave's tile rows, K half fhi
  const int frow = lane & 31, fhi = lane >> 5;
  int hrow0[TJ];  // halo row of this lane's pixel (row tj) at tap offset (0, 0)
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) hrow0[tj] = (wid * TJ + tj) * kHW + frow;

  f32x16_t acc[2][TJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float pst[STATS == 1 ? 32 : 1];
#pragma unroll
  for (int k = 0; k < (STATS == 1 ? 32 : 1); ++k) pst[k] = 0.f;

  const int co_lane = co0 + 4 * fhi;  // + ti * 32 + 8 g
  auto epilogue = [&](int mt) __attribute__((always_inline)) {
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    float ts[STATS == 1 ? 2 : 1][16], tq[STATS == 1 ? 2 : 1][16];
    if constexpr (STATS == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          ts[i][r] = 0.f;
          tq[i][r] = 0.f;
        }
    }
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      const int oy = oy0 + wid * TJ + tj, ox = ox0 + frow;
      const bool ok = oy < a.Ho && ox < a.Wo;
      const int64_t off = ((static_cast<int64_t>(n) * a.Ho + (ok ? oy : 0)) * a.Wo + (ok ? ox : 0)) * a.cout;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        uint2 pkp[2], adp[2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = co_lane + ti * 32 + 8 * g;
          if ((g & 1) == 0 && (FLIP == 1 || STATS == 2) && a.addend != nullptr && a.amask == nullptr) {  // uniform: 16-byte addend load
            uint4 raw = make_uint4(0u, 0u, 0u, 0u);
            if (ok) raw = *reinterpret_cast<const uint4*>(a.addend + off + co + 4 * fhi);
            pair_unswap16(raw, adp[0], adp[1]);
          }
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[ti][tj][4 * g + q];
          if constexpr (STATS == 2) {  // inference BN: scale / shift per channel, residual (addend) below
            const float4 sc = *reinterpret_cast<const float4*>(a.ss + co);
            const float4 sf = *reinterpret_cast<const float4*>(a.ss + a.cout + co);
            v[0] = fmaf(v[0], sc.x, sf.x); v[1] = fmaf(v[1], sc.y, sf.y);
            v[2] = fmaf(v[2], sc.z, sf.z); v[3] = fmaf(v[3], sc.w, sf.w);
          }
          if ((FLIP == 1 || STATS == 2) && a.addend != nullptr && ok) {
            float r[4];
            if (a.amask == nullptr) {
              bf16x4_unpack(adp[g & 1], r);
            } else {
              bf16x4_unpack(*reinterpret_cast<const uint2*>(a.addend + off + co), r);
              mask_addend4(a.amask, off + co, r);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] += r[q];
          }
          if constexpr (STATS == 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = epi_act(v[q], a.act);
          }
          uint2 pk;
          pk.x = pack2(v[0], v[1]);
          pk.y = pack2(v[2], v[3]);
          pkp[g & 1] = pk;
          if (g & 1) {  // 16-byte store of the group pair (g - 1, g): pair_swap16
            const uint4 w = pair_swap16(pkp[0], pkp[1]);
            if (ok) *reinterpret_cast<uint4*>(a.y + off + co - 8 + 4 * fhi) = w;
          }
          if constexpr (STATS == 1) {  // statistics of the fp32 outputs; pixels past the image do not count
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float u = ok ? v[q] : 0.f;
              ts[ti][4 * g + q] += u;
              tq[ti][4 * g + q] = fmaf(u, u, tq[ti][4 * g + q]);
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[ti][tj][r] = 0.f;
      }
    }
    if constexpr (STATS == 1) {
      float y1[32];
      stats_stage1<2>(ts, tq, y1);
#pragma unroll
      for (int k = 0; k < 32; ++k) pst[k] += y1[k];
    }
  };

  if (my_tiles > 0) halo_dma(mfirst, 0);
  for (int t = 0; t < my_tiles; ++t) {
    // this wave's DMAs (halo t; weights at t = 0) landed and its stores of two tiles ago retired;
    // the barrier publishes every wave's and frees the other halo buffer (read by tile t - 1)
    vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t > 0) epilogue(mfirst + (t - 1) * mstep);
    if (t + 1 < my_tiles) halo_dma(mfirst + (t + 1) * mstep, (t + 1) & 1);

    const uint4* hb = hl + (t & 1) * kHStage;
    // fragment reads PD steps ahead of the MFMAs (PD + 1 register slots)
    bf16x8_t af[PD + 1][2], bfg[PD + 1][TJ];
    auto load = [&](int s, int slot) {
      const int tap = s >> 2, ks = s & 3;
      const int i = tap / 3, j = tap - 3 * (tap / 3);
      const int sh = FLIP ? (2 - i) * kHW + (2 - j) : i * kHW + j;
      const int ch = 2 * ks + fhi;
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        const int hr = hrow0[tj] + sh;
        bfg[slot][tj] = as_frag(hb[hr * 8 + (ch ^ ((hr >> 1) & 7))]);
      }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        const int wr = tap * 64 + ti * 32 + frow;
        af[slot][ti] = as_frag(wl[wr * 8 + (ch ^ ((wr >> 1) & 7))]);
      }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p) load(p, p);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      if (s + PD < NSTEP) load(s + PD, (s + PD) % (PD + 1));
      const int sl = s % (PD + 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][ti], bfg[sl][tj], acc[ti][tj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  if (my_tiles > 0) epilogue(mfirst + (my_tiles - 1) * mstep);

  if constexpr (STATS == 1) {
    // one slab row per block: the pixel waves' per-channel sums through LDS in a fixed order
    __syncthreads();  // all fragment reads done, no DMA in flight
    float* red = reinterpret_cast<float*>(lds);  // [NW][2][64]
    stats_stage2<2>(pst, lane, [&](int, int sq, int dc, float v) { red[(wid * 2 + sq) * 64 + 4 * fhi + dc] = v; });
    __syncthreads();
    for (int e = tid; e < 128; e += NW * 64) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += red[w * 128 + e];
      const int sq = e >= 64, c = co0 + (sq ? e - 64 : e);
      a.part[static_cast<int64_t>(mfirst) * 2 * a.cout + (sq ? a.cout : 0) + c] = s;
    }
  }
}

int wres_grid(int mtiles, int ntiles) {
  const int64_t tiles = static_cast<int64_t>(mtiles) * ntiles;
  const int cap = std::max(ntiles, (256 / ntiles) * ntiles);  // one block per CU (LDS-bound)
  return static_cast<int>(tiles < cap ? tiles : cap);
}

// operand geometry of a pass: gathered H x W (64 channels) -> output Ho x Wo x outc
bool wres_fill(WresArgs& k, const ConvGeom& g, bool dgrad) {
  const int red = dgrad ? g.cout : g.cin, outc = dgrad ? g.cin : g.cout;
  if (red != 64 || outc % 64 != 0) return false;
  if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1 || g.ph != 1 || g.pw != 1)
    return false;
  k.H = dgrad ? g.ho : g.h;
  k.W = dgrad ? g.wo : g.w_in;
  k.Ho = dgrad ? g.h : g.ho;
  k.Wo = dgrad ? g.w_in : g.wo;
  k.cout = outc;
  const int64_t xb = static_cast<int64_t>(g.n) * k.H * k.W * 64 * 2;
  if (xb >= (int64_t{1} << 31)) return false;
  k.xbytes = static_cast<uint32_t>(xb);
  // forward: input row oy - 1 + i; data gradient (stride 1, pad 1): dy row y + 1 - i, lowest at
  // i = 2 -> origin -1 as well, tap (i, j) at halo offset (2 - i, 2 - j)
  k.dh0 = -1;
  k.dw0 = -1;
  k.tilesW = (k.Wo + kTW - 1) / kTW;
  k.tilesH = (k.Ho + kTH - 1) / kTH;
  k.mtiles = g.n * k.tilesW * k.tilesH;
  k.ntiles = outc / 64;
  return true;
}

// RTSEG_WRES_CFG=<n> (A/B sweeps): 0 = 8 waves x 1 row, prefetch 1 (default: fastest measured,
// profiles/r4_conv/bench_wres_cfg*.txt); 1 = 8 x 1, prefetch 2; 2 = 4 waves x 2 rows, prefetch 2;
// 3 = 4 x 2, prefetch 3
int wres_cfg() {
  static const int c = std::getenv("RTSEG_WRES_CFG") ? std::atoi(std::getenv("RTSEG_WRES_CFG")) : 0;
  return c;
}

template <int STATS, int FLIP>
void wres_launch(const WresArgs& k, int grid, hipStream_t st) {
  switch (wres_cfg()) {
    case 1: wres_conv_kernel<STATS, FLIP, 8, 2><<<grid, 512, 0, st>>>(k); break;
    case 3: wres_conv_kernel<STATS, FLIP, 4, 3><<<grid, 256, 0, st>>>(k); break;
    case 2: wres_conv_kernel<STATS, FLIP, 4, 2><<<grid, 256, 0, st>>>(k); break;
    default: wres_conv_kernel<STATS, FLIP, 8, 1><<<grid, 512, 0, st>>>(k); break;
  }
}

}  // namespace

bool conv_wres_supported(const ConvGeom& g, int mode) {
  WresArgs k{};
  return wres_fill(k, g, mode == 1);
}

int conv_wres_slabs(const ConvGeom& g) {
  WresArgs k{};
  if (!wres_fill(k, g, false)) return 0;
  return wres_grid(k.mtiles, k.ntiles) / k.ntiles;
}

// forward: g.x = x, g.w = wk [Cout][3][3][64], g.y = y, g.part = BN statistics slab or null
void launch_conv_wres_fwd(const ConvGeom& g, hipStream_t st) {
  WresArgs k{};
  if (!wres_fill(k, g, false)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = g.part;
  k.addend = nullptr;
  k.amask = nullptr;
  k.ss = g.scale_shift;
  k.act = g.act;
  if (k.ss != nullptr) k.addend = static_cast<const uint16_t*>(g.res);  // the residual
  const int grid = wres_grid(k.mtiles, k.ntiles);
  if (grid <= 0) return;
  if (k.ss != nullptr) wres_launch<2, 0>(k, grid, st);
  else if (k.part != nullptr) wres_launch<1, 0>(k, grid, st);
  else wres_launch<0, 0>(k, grid, st);
}

// data gradient: g = forward geometry; g.x = dy, g.w = wt [Cin][3][3][64], g.y = dx, g.res = addend
void launch_conv_wres_dgrad(const ConvGeom& g, hipStream_t st) {
  WresArgs k{};
  if (!wres_fill(k, g, true)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = nullptr;
  k.addend = static_cast<const uint16_t*>(g.res);
  k.amask = g.amask;
  const int grid = wres_grid(k.mtiles, k.ntiles);
  if (grid <= 0) return;
  wres_launch<0, 1>(k, grid, st);
}

}  // namespace rtseg
