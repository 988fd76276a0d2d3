// Halo-tiled implicit-GEMM convolution for small-footprint stride-1 convs (3x3 'same', 3x1,
// 1x3, and their data gradients) on bf16 MFMA (v_mfma_f32_32x32x16_bf16), channels-last, gfx950.
//
// Reference sites: the 3x3 stride-1 convs that carry most of the zoo's FLOPs -- DDRNet's RB / RBB
// blocks (ddrnet.py:168-219), ConvBNAct (models/modules.py:73-85), ResNet BasicBlocks.
//
// Why a second kernel next to conv_igemm.hip's gather kernel: the gather kernel streams one
// (tap, 64-channel) slice of BM gathered pixels per K-step, so every input pixel crosses the
// L2 -> LDS path once per tap (9x for a 3x3).  On the 64- and 128-channel layers that re-read,
// not the MFMA, sets the time: 512 x 64 tiles move 72 KiB per K-step for 4.2 MFLOP
// (~57 FLOP/B, profiles/r2_conv_igemm), above what an L2-served LDS-DMA gather sustains per CU.
// Here a block owns a TH x TW output tile and stages the (TH+2) x (TW+2) input halo of one
// 64-channel chunk ONCE; the taps read shifted windows of it from LDS, so the per-K-step
// traffic is the [BN][64] weight slice plus 1/9 of the halo (~13-22 KiB per K-step).
//
//  * LDS: two halo buffers (chunk parity) + an NST-stage weight ring; 128-byte rows (64 bf16
//    channels of one pixel / one output channel), chunk c of row r stored at c ^ ((r >> 1) & 7)
//    (source-side swizzle of the DMA).  A fragment of 32 consecutive pixels starting at ANY row
//    is conflict-free under this swizzle (the 16 lanes of a ds_read_b128 group hit 16 distinct
//    (row & 15) values), so shifted tap windows cost the same as aligned ones;
//  * one flat DMA stream across the block's persistent tile walk: group g carries the weights
//    of K-step g and -- for taps >= NST-1 -- one piece of the NEXT chunk's halo (the other
//    halo buffer, whose last reader finished before the chunk's first barrier), so the halo
//    load of chunk c+1 / the next tile hides under chunk c's MFMAs;
//  * epilogue as conv_igemm's: bf16 stores straight from the accumulators, optional per-channel
//    BN statistics (DPP half-wave sums, one slab row per (M tile, pixel wave)), optional
//    residual-gradient addend, or the inference BN scale/shift + residual + ReLU(6).
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>
#include <cstdlib>

namespace rtseg {

namespace {

using namespace mdev;

// zero page: the DMA source of padding rows / columns, at any chunk offset (C <= 8192)
__device__ uint4 g_halo_zero[1024];

constexpr int kHaloMaxTaps = 9;

struct HaloArgs {
  const uint16_t* x;       // gathered operand [N][H][W][C] (forward: x, dgrad: dy)
  const uint16_t* w;       // [cout][KT][C] bf16
  uint16_t* y;             // [N][Ho][Wo][cout]
  float* part;             // BN statistics slab, or null
  const float* ss;         // EPI 1: inference BN [scale | shift] fp32 [2*cout]
  const uint16_t* res;     // EPI 1: residual, y's layout, or null
  const uint16_t* addend;  // EPI 0: bf16 tensor of y's layout added to the result, or null
  const uint8_t* amask;    // EPI 0: bit mask of the addend (mask_addend4), or null
  int act;
  int H, W, C;             // gathered operand
  int Ho, Wo, cout;        // output
  int dh0, dw0;            // halo origin offset: input pixel of output (oy, ox), relative tap 0
  int wrow;                // KT * C
  int ntap, cch;           // taps, 64-channel chunks
  int tilesW, tilesH, mtiles, ntiles;
  // taps: the KH x KW grid, tap t = i * kw + j reads weight tap t at halo offset
  // (i * tdh, j * tdw) -- or ((kh-1-i) * tdh, (kw-1-j) * tdw) when flip (data gradient)
  int kh, kw, tdh, tdw, flip;
  const uint4* zero;       // g_halo_zero: the DMA source of padding rows
  int dbg;                 // RTSEG_HALO_DBG experiment bits (0 in production): 1 = no output stores
};

template <int TH, int TW, int BN, int WM, int WN, int NST, int EPI, int STATS>
__global__ void __launch_bounds__(WM* WN * 64) halo_conv_kernel(const HaloArgs a) {
  constexpr int NW = WM * WN;
  static_assert(NW == 8, "8 waves");
  constexpr int BM = TH * TW;
  constexpr int HW = TW + 2, HH = TH + 2;
  constexpr int HROWS = HH * HW;
  constexpr int HI = (HROWS + 7) / 8;       // 8-row DMA instructions per halo
  constexpr int HPW = (HI + NW - 1) / NW;   // ... per wave (at most)
  constexpr int HSTAGE = HI * 64;           // 16-byte chunks per halo buffer
  constexpr int WSTAGE = BN * 8;            // 16-byte chunks per weight stage
  constexpr int TI = BN / WN / 32, TJ = BM / WM / 32;
  constexpr int WI = BN / 8 / NW;           // weight DMA instructions per wave per stage
  static_assert(TW % 32 == 0 && (TW & (TW - 1)) == 0, "pixel fragments stay inside one output row");
  static_assert(TI >= 1 && TJ >= 1 && TI * WN * 32 == BN && TJ * WM * 32 == BM, "wave tiling");
  static_assert(WI >= 1 && WI * NW * 8 == BN, "weight DMA tiling");
  static_assert(NST >= 2 && NST <= 8, "ring depth");
  __shared__ uint4 lds[2 * HSTAGE + NST * WSTAGE];
  uint4* const wring = lds + 2 * HSTAGE;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid % WN, wm = wid / WN;
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);
  const int ntile = lb % a.ntiles;
  const int co0 = ntile * BN;
  const int mstep = G / a.ntiles;
  const int mfirst = lb / a.ntiles;
  const int my_tiles = mfirst < a.mtiles ? (a.mtiles - mfirst + mstep - 1) / mstep : 0;
  const int cch = a.cch, ntap = a.ntap;
  const int nk = ntap * cch;

  // taps are walked as (i, j) counters in SGPRs: no table lookup (a runtime-indexed array
  // becomes a scratch or scalar load whose wait would drain the DMA ring every K-step)
  const int kw = a.kw, kh1 = a.kh - 1, kw1 = a.kw - 1;
  auto tap_shift = [&](int i, int j) {  // halo row offset of tap (i, j)
    return (a.flip ? kh1 - i : i) * a.tdh * HW + (a.flip ? kw1 - j : j) * a.tdw;
  };
  const void* const zero = a.zero;

  const int lr8 = lane >> 3, lch = lane & 7;
  // ---- weight DMA geometry (as conv_igemm): instruction e fills rows (wid*WI + e)*8 + lane/8
  const uint16_t* wsrc[WI];
  bool wok[WI];
#pragma unroll
  for (int e = 0; e < WI; ++e) {
    const int row = (wid * WI + e) * 8 + lr8;
    const int lc = lch ^ ((row >> 1) & 7);
    const int co = co0 + row;
    wok[e] = co < a.cout;
    wsrc[e] = a.w + static_cast<int64_t>(min(co, a.cout - 1)) * a.wrow + lc * 8;
  }

  // tile ordinal -> (image, first output row, first output column)
  auto tile_xyz = [&](int mt, int& n, int& oy0, int& ox0) {
    const int tx = mt % a.tilesW;
    const int t2 = mt / a.tilesW;
    const int ty = t2 % a.tilesH;
    n = t2 / a.tilesH;
    oy0 = ty * TH;
    ox0 = tx * TW;
  };

  // Halo sources of the current halo TARGET tile, one 64-bit pointer per (wave, DMA instruction
  // jj), computed once per tile; padding rows point into the zero page (big enough for any
  // chunk offset), so a K-step's halo piece is one add + one DMA.  Piece jj of a chunk rides on
  // tap NST-1+jj (host check: ntap - (NST-1) >= HPW).
  const uint16_t* hsrc[HPW];
  auto set_halo = [&](int mt) {
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
#pragma unroll
    for (int jj = 0; jj < HPW; ++jj) {
      const int r = (wid + NW * jj) * 8 + lr8;
      const int hy = r / HW, hx = r % HW;  // constant divisors
      const int ih = oy0 + a.dh0 + hy, iw = ox0 + a.dw0 + hx;
      const bool ok = r < HROWS && static_cast<unsigned>(ih) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(a.W);
      const int lc = (lch ^ ((r >> 1) & 7)) * 8;
      hsrc[jj] = ok ? a.x + ((static_cast<int64_t>(n) * a.H + ih) * a.W + iw) * a.C + lc
                    : reinterpret_cast<const uint16_t*>(zero) + lc;
    }
  };
  auto halo_piece = [&](int jj, int c0, int hb) {
#pragma unroll
    for (int q = 0; q < HPW; ++q)
      if (q == jj && wid + NW * q < HI)
        dma16(hsrc[q] + c0, lds_addr(lds + hb * HSTAGE) + (wid + NW * q) * 1024);
  };

  // ---- staging cursor of the flat stream (wave-uniform): tile ordinal, chunk, tap, ring slot
  int st_ord = 0, st_c = 0, st_t = 0, st_buf = 0;
  bool halo_live = true;  // the halo target (next chunk) exists
  auto stage = [&]() {
    // halo piece of the next chunk, in the other halo buffer (free: its last reader finished
    // before this chunk's first barrier)
    const int jj = st_t - (NST - 1);
    if (jj >= 0 && jj < HPW) {
      int hord = st_ord, hc = st_c + 1;
      if (hc == cch) {
        hc = 0;
        ++hord;
      }
      if (jj == 0) {
        halo_live = hord < my_tiles;
        if (halo_live && hc == 0) set_halo(mfirst + hord * mstep);
      }
      if (halo_live) halo_piece(jj, hc * 64, (hord * cch + hc) & 1);
    }
    const int woff = st_t * a.C + st_c * 64;
    const uint32_t base = lds_addr(wring + st_buf * WSTAGE);
#pragma unroll
    for (int e = 0; e < WI; ++e) {
      const void* src = wok[e] ? static_cast<const void*>(wsrc[e] + woff) : zero;
      dma16(src, base + (wid * WI + e) * 1024);
    }
    if (++st_buf == NST) st_buf = 0;
    if (++st_t == ntap) {
      st_t = 0;
      if (++st_c == cch) {
        st_c = 0;
        ++st_ord;
      }
    }
  };

  // ---- fragment geometry
  const int frow = lane & 31, fhi = lane >> 5, fx = (frow >> 1) & 7;
  int hbase[TJ];  // halo row of this lane's pixel for relative tap (0, 0)
  int lpix[TJ];   // pixel index inside the tile
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int p = wm * (BM / WM) + tj * 32 + frow;
    lpix[tj] = p;
    hbase[tj] = (p / TW) * HW + (p % TW);
  }

  f32x16_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int64_t pend_off[TJ];
  const int co_lane = co0 + wn * (BN / WN) + 4 * fhi;  // + ti*32 + 8g
  // STATS: the lane's first-stage-reduced BN statistics summed over the block's tiles (they
  // share the channel tile); the rest of the reduction runs once, at the end (as conv_igemm)
  float pst[STATS ? TI * 16 : 1];
#pragma unroll
  for (int k = 0; k < (STATS ? TI * 16 : 1); ++k) pst[k] = 0.f;

  auto pack_tile = [&](int mt) __attribute__((always_inline)) {
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    float ts[STATS ? TI : 1][16], tq[STATS ? TI : 1][16];
    if constexpr (STATS) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          ts[i][r] = 0.f;
          tq[i][r] = 0.f;
        }
    }
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      const int oy = oy0 + lpix[tj] / TW, ox = ox0 + lpix[tj] % TW;
      const bool ok = oy < a.Ho && ox < a.Wo;
      pend_off[tj] = ((static_cast<int64_t>(n) * a.Ho + (ok ? oy : 0)) * a.Wo + (ok ? ox : 0)) * a.cout;
#pragma unroll
      for (int ti = 0; ti < TI; ++ti) {
        uint2 pkp[2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = co_lane + ti * 32 + 8 * g;
          const bool sok = ok && co < a.cout;
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[ti][tj][4 * g + q];
          if (a.addend != nullptr && sok) {
            float r[4];
            bf16x4_unpack(*reinterpret_cast<const uint2*>(a.addend + pend_off[tj] + co), r);
            if (a.amask != nullptr) mask_addend4(a.amask, pend_off[tj] + co, r);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] += r[q];
          }
          if constexpr (EPI == 1) {
            const int cc = min(co, a.cout - 4);
            const float4 sc = *reinterpret_cast<const float4*>(a.ss + cc);
            const float4 sf = *reinterpret_cast<const float4*>(a.ss + a.cout + cc);
            v[0] = fmaf(v[0], sc.x, sf.x);
            v[1] = fmaf(v[1], sc.y, sf.y);
            v[2] = fmaf(v[2], sc.z, sf.z);
            v[3] = fmaf(v[3], sc.w, sf.w);
            if (a.res != nullptr && sok) {
              float r[4];
              bf16x4_unpack(*reinterpret_cast<const uint2*>(a.res + pend_off[tj] + co), r);
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] += r[q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = epi_act(v[q], a.act);
          }
          uint2 pk;
          pk.x = pack2(v[0], v[1]);
          pk.y = pack2(v[2], v[3]);
          pkp[g & 1] = pk;
          if (g & 1) {  // 16-byte store of the group pair (g - 1, g): pair_swap16
            const uint4 w = pair_swap16(pkp[0], pkp[1]);
            const int c16 = co - 8 + 4 * fhi;
            if (ok && c16 < a.cout && !(a.dbg & 1)) *reinterpret_cast<uint4*>(a.y + pend_off[tj] + c16) = w;
          }
          if constexpr (STATS) {  // statistics of the fp32 outputs (the accumulators)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float u = sok ? v[e] : 0.f;  // halo rows past the image are not zero
              ts[ti][4 * g + e] += u;
              tq[ti][4 * g + e] = fmaf(u, u, tq[ti][4 * g + e]);
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[ti][tj][r] = 0.f;
      }
    }
    if constexpr (STATS) {
      float y1[TI * 16];
      stats_stage1<TI>(ts, tq, y1);
#pragma unroll
      for (int k = 0; k < TI * 16; ++k) pst[k] += y1[k];
    }
  };

  const int total = my_tiles * nk;
  if (total == 0) return;

  // prologue: the whole halo of the first chunk, then weight groups 0 .. NST-2 (taps < NST-1:
  // no halo pieces)
  set_halo(mfirst);
#pragma unroll
  for (int q = 0; q < HPW; ++q)
    if (wid + NW * q < HI) dma16(hsrc[q], lds_addr(lds) + (wid + NW * q) * 1024);
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < total) stage();

  int kt = 0, ki = 0, kj = 0, kc = 0, ord = 0, buf = 0, fc = 0, pend_mt = -1;
  for (int gs = 0; gs < total; ++gs) {
    // group gs (and every halo piece of the current chunk, all in older groups) has landed:
    // at most the newest (NST-2) groups' weight DMAs may still be in flight
    if (NST >= 3 && gs + 1 < total) {
      vm_wait<(NST - 2) * WI>();
    } else {
      vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (pend_mt >= 0) {
      pack_tile(pend_mt);
      pend_mt = -1;
    }
    if (gs + NST - 1 < total) stage();

    const int tshift = tap_shift(ki, kj);
    const uint4* Wt = wring + buf * WSTAGE + (wn * (BN / WN) + frow) * 8;
    const uint4* Hb = lds + (fc & 1) * HSTAGE;
    int hrow[TJ], hsw[TJ];
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      hrow[tj] = (hbase[tj] + tshift) * 8;
      hsw[tj] = ((hbase[tj] + tshift) >> 1) & 7;
    }
    constexpr int FB = TI + TJ <= 4 ? 2 : 1;
    bf16x8_t af[FB][TI], bfg[FB][TJ];
    auto load_frags = [&](int s, int slot) {
      const int k = 2 * s + fhi;
#pragma unroll
      for (int ti = 0; ti < TI; ++ti) af[slot][ti] = as_frag(Wt[ti * 256 + (k ^ fx)]);
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) bfg[slot][tj] = as_frag(Hb[hrow[tj] + (k ^ hsw[tj])]);
    };
    if constexpr (FB == 2) load_frags(0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if constexpr (FB == 2) {
        if (s < 3) load_frags(s + 1, (s + 1) & 1);
      } else {
        load_frags(s, 0);
      }
      const int sl = FB == 2 ? (s & 1) : 0;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ti = 0; ti < TI; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][ti], bfg[sl][tj], acc[ti][tj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (++buf == NST) buf = 0;
    if (++kj == kw) {
      kj = 0;
      ++ki;
    }
    if (++kt == ntap) {
      kt = 0;
      ki = 0;
      kj = 0;
      ++fc;
      if (++kc == cch) {
        kc = 0;
        pend_mt = mfirst + ord * mstep;
        ++ord;
      }
    }
  }
  if (pend_mt >= 0) pack_tile(pend_mt);

  if constexpr (STATS) {
    // one slab row per block: DPP stages per wave, the WM pixel waves summed in a fixed order
    // through LDS (deterministic; every block has >= 1 tile, so no early return skips this)
    __syncthreads();  // every wave is past its last fragment read; no DMA is in flight
    float* red = reinterpret_cast<float*>(lds);  // [WM][2][BN]
    const int cl = wn * (BN / WN) + 4 * fhi;
    stats_stage2<TI>(pst, lane, [&](int, int sq, int dc, float v) { red[(wm * 2 + sq) * BN + cl + dc] = v; });
    __syncthreads();
    for (int e = tid; e < 2 * BN; e += NW * 64) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) s += red[w * 2 * BN + e];
      const int sq = e >= BN, c = co0 + (sq ? e - BN : e);
      if (c < a.cout) a.part[static_cast<int64_t>(mfirst) * 2 * a.cout + (sq ? a.cout : 0) + c] = s;
    }
  }
}

// ------------------------------------------------------------------------------- host side
// Configurations (TH x TW output pixels, BN output channels, WM x WN waves, NST weight stages):
//   0: 4 x 64 px x  64 ch, 8 x 1 waves (64 x 32 wave tiles), 3 stages, 124 KiB LDS
//   1: 2 x 64 px x 128 ch, 4 x 2 waves (64 x 32),            5 stages, 148 KiB
//   2: 4 x 64 px x 128 ch, 4 x 2 waves (64 x 64),            3 stages, 148 KiB
// A chunk's halo is loaded as HPW one-instruction pieces per wave riding on taps NST-1 ..
// NST-2+HPW, so a config needs ntap - (NST-1) >= HPW (3x3 convs: 9 taps).
// RTSEG_HALO_CFG=<n> forces one (A/B sweeps).
struct HaloCfg {
  int id, th, bn, wm, nst, hpw;
};
constexpr int kHaloTW = 64;
constexpr int halo_hpw(int th) { return (((th + 2) * (kHaloTW + 2) + 7) / 8 + 7) / 8; }
constexpr HaloCfg kHaloCfgs[] = {{0, 4, 64, 8, 3, halo_hpw(4)},
                                 {1, 2, 128, 4, 5, halo_hpw(2)},
                                 {2, 4, 128, 4, 3, halo_hpw(4)}};

bool cfg_fits(const HaloCfg& c, int cout, int ntap) {
  return (c.bn == 64) == (cout <= 64) && ntap - (c.nst - 1) >= c.hpw;
}

// the configuration for (cout, ntap), or id -1 when none fits
HaloCfg halo_cfg(int cout, int ntap) {
  const char* e = std::getenv("RTSEG_HALO_CFG");
  if (e != nullptr && *e != '\0') {
    const int i = std::atoi(e);
    if (i >= 0 && i < 3 && cfg_fits(kHaloCfgs[i], cout, ntap)) return kHaloCfgs[i];
  }
  for (int i : {0, 2, 1})
    if (cfg_fits(kHaloCfgs[i], cout, ntap)) return kHaloCfgs[i];
  return HaloCfg{-1, 1, 64, 1, 2, 1};
}

template <int EPI, int STATS>
void launch_halo_cfg(const HaloArgs& k, const HaloCfg& c, int grid, hipStream_t st) {
  switch (c.id) {
    case 0: halo_conv_kernel<4, kHaloTW, 64, 8, 1, 3, EPI, STATS><<<grid, 512, 0, st>>>(k); break;
    case 1: halo_conv_kernel<2, kHaloTW, 128, 4, 2, 5, EPI, STATS><<<grid, 512, 0, st>>>(k); break;
    case 2: halo_conv_kernel<4, kHaloTW, 128, 4, 2, 3, EPI, STATS><<<grid, 512, 0, st>>>(k); break;
    default: break;
  }
}

// The KH x KW tap grid of a stride-1 conv (flip: its data gradient) -> halo origin and tap
// walk; false when the footprint is wider than the 3 x 3 the halo holds
bool halo_taps(HaloArgs& k, const ConvGeom& g, bool flip) {
  const int n = g.kh * g.kw;
  if (n < 3 || n > kHaloMaxTaps || g.cin > 8192 || g.cout > 8192) return false;
  const int eh = (g.kh - 1) * g.dh, ew = (g.kw - 1) * g.dw;
  if (eh > 2 || ew > 2) return false;
  // forward: input row = oy - ph + i*dh (origin -ph); data gradient: dy row = y + ph - i*dh,
  // lowest at i = kh-1 (origin ph - eh), relative offset (kh-1-i)*dh
  k.dh0 = flip ? g.ph - eh : -g.ph;
  k.dw0 = flip ? g.pw - ew : -g.pw;
  k.kh = g.kh; k.kw = g.kw; k.tdh = g.dh; k.tdw = g.dw; k.flip = flip ? 1 : 0;
  k.ntap = n;
  return halo_cfg(flip ? g.cin : g.cout, n).id >= 0;
}

// device address of g_halo_zero on the current device (cached per device)
const uint4* zero_page() {
  static const uint4* cache[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == nullptr) {
    void* d = nullptr;
    (void)hipGetSymbolAddress(&d, HIP_SYMBOL(g_halo_zero));
    cache[dev] = static_cast<const uint4*>(d);
  }
  return cache[dev];
}

void fill_tiles(HaloArgs& k, int n) {
  const HaloCfg c = halo_cfg(k.cout, k.ntap);
  k.tilesW = (k.Wo + kHaloTW - 1) / kHaloTW;
  k.tilesH = (k.Ho + c.th - 1) / c.th;
  k.mtiles = n * k.tilesW * k.tilesH;
  k.ntiles = (k.cout + c.bn - 1) / c.bn;
}

void launch_halo(HaloArgs& k, hipStream_t st) {
  k.zero = zero_page();
  static const int dbg = std::getenv("RTSEG_HALO_DBG") ? std::atoi(std::getenv("RTSEG_HALO_DBG")) : 0;
  k.dbg = dbg;
  const HaloCfg c = halo_cfg(k.cout, k.ntap);
  const int64_t tiles = static_cast<int64_t>(k.mtiles) * k.ntiles;
  const int cap = std::max(k.ntiles, (256 / k.ntiles) * k.ntiles);  // one block per CU (LDS-bound)
  const int grid = static_cast<int>(tiles < cap ? tiles : cap);
  if (grid <= 0) return;
  if (k.ss != nullptr) launch_halo_cfg<1, 0>(k, c, grid, st);
  else if (k.part != nullptr) launch_halo_cfg<0, 1>(k, c, grid, st);
  else launch_halo_cfg<0, 0>(k, c, grid, st);
}

bool fwd_taps(const ConvGeom& g, HaloArgs& k) { return halo_taps(k, g, false); }
bool dgrad_taps(const ConvGeom& g, HaloArgs& k) { return halo_taps(k, g, true); }


}  // namespace

bool conv_halo_supported(const ConvGeom& g, int mode) {
  if (g.sh != 1 || g.sw != 1) return false;
  const int red = mode == 1 ? g.cout : g.cin, outc = mode == 1 ? g.cin : g.cout;
  if (red % 64 != 0 || outc % 64 != 0) return false;
  HaloArgs k{};
  return mode == 1 ? dgrad_taps(g, k) : fwd_taps(g, k);
}

int conv_halo_slabs(const ConvGeom& g) {
  HaloArgs k{};
  k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  if (!fwd_taps(g, k)) return 0;
  fill_tiles(k, g.n);
  // one row per block of a channel tile (see the end of halo_conv_kernel)
  const int64_t tiles = static_cast<int64_t>(k.mtiles) * k.ntiles;
  const int cap = std::max(k.ntiles, (256 / k.ntiles) * k.ntiles);
  return static_cast<int>(tiles < cap ? tiles : cap) / k.ntiles;
}

void launch_conv_halo_fwd(const ConvGeom& g, hipStream_t st) {
  HaloArgs k{};
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = g.part;
  k.ss = g.scale_shift;
  k.res = static_cast<const uint16_t*>(g.res);
  k.act = g.act;
  k.H = g.h; k.W = g.w_in; k.C = g.cin;
  k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  k.wrow = g.kh * g.kw * g.cin;
  k.cch = g.cin / 64;
  if (!fwd_taps(g, k)) return;
  fill_tiles(k, g.n);
  launch_halo(k, st);
}

// g: forward geometry; g.x = dy [N,Ho,Wo,Cout], g.w = wt [Cin][KH][KW][Cout], g.y = dx [N,H,W,Cin],
// g.res = optional addend of dx's layout
void launch_conv_halo_dgrad(const ConvGeom& g, hipStream_t st) {
  HaloArgs k{};
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.addend = static_cast<const uint16_t*>(g.res);
  k.amask = g.amask;
  k.H = g.ho; k.W = g.wo; k.C = g.cout;
  k.Ho = g.h; k.Wo = g.w_in; k.cout = g.cin;
  k.wrow = g.kh * g.kw * g.cout;
  k.cch = g.cout / 64;
  if (!dgrad_taps(g, k)) return;
  fill_tiles(k, g.n);
  launch_halo(k, st);
}

}  // namespace rtseg
