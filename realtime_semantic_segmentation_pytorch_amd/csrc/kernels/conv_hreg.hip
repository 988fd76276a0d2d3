// Halo-tiled 3x3 stride-1 convolution with the weights streamed straight into registers, for the
// wide layers (reduction channels % 64 == 0, output channels % 128 == 0): DDRNet-23's 128-channel
// high-resolution branch and its 256 / 512-channel low-resolution branch (ddrnet.py:168-219,
// 241-291), ResNet layer2-4 BasicBlocks (models/backbone.py), forward and data gradient.
//
// The gather kernel (conv_igemm.hip) stages, per (tap, 64-channel) K-step, 512 gathered pixel rows
// + 128 weight rows through LDS with one step of prefetch and a block barrier per K-step: 29 % of
// MFMA peak on the 128-channel layers (profiles/r4_conv/pmc_table.txt).  Here:
//  * a block owns a 4 x 64-pixel output tile x 128 output channels and stages the (4+2) x (64+2)
//    input halo of one 64-channel chunk ONCE per chunk (double-buffered a whole chunk ahead); all
//    9 taps read shifted windows of it -- one block barrier per chunk (every 36 MFMA sub-steps),
//    not per K-step;
//  * the weights never touch LDS: they are pre-packed in MFMA A-fragment order
//    ([co/32][Cin/64][tap][16-deep sub-step][64 lanes][8]) so each wave loads its fragments with
//    fully coalesced 1 KiB reads (L2 / L1 resident: every block reads the same few hundred KiB),
//    two taps ahead of their MFMAs;
//  * 8 waves = 4 pixel rows (64 pixels) x 2 channel halves (64 channels): per 16-deep sub-step two
//    B fragments from LDS and two A fragments from registers feed four v_mfma_f32_32x32x16_bf16;
//  * halo rows by LDS-DMA through a range-checked buffer resource (zero padding for free); chunk c
//    of a 128-byte row r at c ^ ((r >> 1) & 7): B fragment reads conflict-free for any tap shift;
//  * epilogue of tile t after the first chunk barrier of tile t + 1: bf16 stores, optional BN
//    statistics slab (training forward) or residual-gradient addend (data gradient).
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace rtseg {

namespace {

using namespace mdev;

constexpr int kTH = 4, kTW = 64;                       // output tile: 256 pixels
constexpr int kHH = kTH + 2, kHW = kTW + 2;            // halo of one 64-channel chunk
constexpr int kHRows = kHH * kHW;                      // 396
constexpr int kHInstr = (kHRows + 7) / 8;              // 50 LDS-DMA instructions of 8 rows
constexpr int kHStage = kHInstr * 64;                  // 16-byte chunks per halo buffer (400 rows)
constexpr int kBN = 128;                               // output channels per block
constexpr int kRed = 4 * 2 * kBN;                      // BN statistics accumulator (floats)
static_assert(2 * kHStage * 16 + kRed * 4 <= 160 * 1024, "LDS budget");

struct HrArgs {
  const uint16_t* x;       // gathered operand [N][H][W][C] (forward: x; data gradient: dy)
  const uint4* wp;         // packed weights: [cout / 32][C / 64][9][4][64] x 16 bytes
  uint16_t* y;             // output [N][Ho][Wo][cout]
  float* part;             // BN statistics slab [grid / ntiles][2 * cout], or null
  const uint16_t* addend;  // bf16 tensor of y's layout added to the result, or null
  const uint8_t* amask;    // bit mask of the addend (mask_addend4), or null
  int H, W, C;             // gathered operand
  int Ho, Wo, cout;
  int cch;                 // 64-channel chunks of C
  int tilesW, tilesH, mtiles, ntiles;
  uint32_t xbytes;
  int dbg;                 // RTSEG_HREG_DBG (A/B only): 1 = no epilogue, 2 = no statistics, 4 = no stores
};

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

// Wave layouts (WL): NRG row groups x NCG channel groups of the 4 x 64-pixel x 128-channel tile;
// each wave owns RPW = 4 / NRG tile rows (TJ = 2 RPW 32-pixel tiles) x TI = 4 / NCG 32-channel tiles.
//  WL 1: 4 x 2 -> 8 waves of 2 x 2 tiles (2 per SIMD);
//  WL 2: 2 x 2 -> 4 waves of 2 x 4 tiles (1 per SIMD, 512-register file): half the weight stream;
//  WL 4: 2 x 4 -> 8 waves of 1 x 4 tiles: WL 2's weight stream (every A fragment feeds 4 MFMAs;
//        the per-CU stream of WL 1 is ~64 B/clk, above the L2's ~56 B/clk/CU share) with WL 1's
//        two waves per SIMD, for twice WL 1's B-fragment LDS reads (128 B/clk/CU of 256).
template <int WL> struct HrLayout;
template <> struct HrLayout<1> { static constexpr int NRG = 4, NCG = 2; };
template <> struct HrLayout<2> { static constexpr int NRG = 2, NCG = 2; };
template <> struct HrLayout<4> { static constexpr int NRG = 2, NCG = 4; };

template <int STATS, int FLIP, int WL>
__global__ void __launch_bounds__(HrLayout<WL>::NRG * HrLayout<WL>::NCG * 64) hreg_conv_kernel(const HrArgs a) {
  constexpr int NRG = HrLayout<WL>::NRG, NCG = HrLayout<WL>::NCG;
  constexpr int kNW = NRG * NCG, RPW = kTH / NRG, TJ = 2 * RPW, TI = 4 / NCG;
  __shared__ uint4 lds[2 * kHStage + kRed / 4];
  float* const red = reinterpret_cast<float*>(lds + 2 * kHStage);  // [row group][sum, sumsq][128]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NCG, wn = wid % NCG;  // row group of the tile, channel group
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);
  const int ntile = lb % a.ntiles;
  const int co0 = ntile * kBN;
  const int mstep = G / a.ntiles;
  const int mfirst = lb / a.ntiles;
  const int my_tiles = mfirst < a.mtiles ? (a.mtiles - mfirst + mstep - 1) / mstep : 0;
  const int cch = a.cch;
  const int nsteps = my_tiles * cch;  // chunk-steps of this block
  const int lr8 = lane >> 3, lch = lane & 7;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, static_cast<int>(a.xbytes), 0x00020000);
  auto tile_xyz = [&](int mt, int& n, int& oy0, int& ox0) {
    const int tx = mt % a.tilesW;
    const int t2 = mt / a.tilesW;
    n = t2 / a.tilesH;
    oy0 = (t2 % a.tilesH) * kTH;
    ox0 = tx * kTW;
  };
  // halo of chunk-step q (tile q / cch, chunk q % cch) into buffer q & 1
  auto halo_dma = [&](int q) {
    const int mt = mfirst + (q / cch) * mstep, c0 = (q % cch) * 64;
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    const uint32_t base = lds_addr(lds + (q & 1) * kHStage);
    for (int e = wid; e < kHInstr; e += kNW) {
      const int r = e * 8 + lr8;
      const int hy = r / kHW, hx = r - hy * kHW;
      const int ih = oy0 - 1 + hy, iw = ox0 - 1 + hx;
      const bool ok = r < kHRows && static_cast<unsigned>(ih) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(a.W);
      const int lc = lch ^ ((r >> 1) & 7);
      const uint32_t v =
          ok ? static_cast<uint32_t>(((n * a.H + ih) * a.W + iw) * a.C + c0 + lc * 8) * 2u : 0x80000000u;
      bdma16(xr, v, base + e * 1024);
    }
  };

  const uint4* wbase = a.wp + (static_cast<int64_t>(co0 / 32 + wn * TI) * cch * 9 * 4) * 64 + lane;
  const int64_t ti_stride = static_cast<int64_t>(cch) * 9 * 4 * 64;
  auto wload = [&](int g, bf16x8_t (&dst)[TI][4]) {  // g = chunk * 9 + tap
#pragma unroll
    for (int ti = 0; ti < TI; ++ti)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) dst[ti][ks] = as_frag(wbase[ti * ti_stride + (g * 4 + ks) * 64]);
  };

  // B fragment geometry: lane -> pixel frow of 32-pixel half tj of the wave's tile row
  const int frow = lane & 31, fhi = lane >> 5;
  const int hrow0 = wm * RPW * kHW + frow;  // + (tj / 2) * kHW + (tj % 2) * 32 + tap shift

  f32x16_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if constexpr (STATS) {  // this block's per-channel statistics accumulate in LDS (no registers)
    for (int e = tid; e < kRed; e += kNW * 64) red[e] = 0.f;
  }

  const int co_lane = co0 + wn * (TI * 32) + 4 * fhi;  // + ti * 32 + 8 g
  auto epilogue = [&](int mt) __attribute__((always_inline)) {
    if (a.dbg & 1) {
#pragma unroll
      for (int ti = 0; ti < TI; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[ti][tj][r] = 0.f;
      return;
    }
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    // the wave's values (+ addend) -> packed 16-byte groups -> memory; statistics; acc = 0
    auto produce = [&]() __attribute__((always_inline)) {
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
        const int oy = oy0 + wm * RPW + (tj >> 1), ox = ox0 + (tj & 1) * 32 + frow;
        const bool ok = oy < a.Ho && ox < a.Wo;
        const int64_t off = ((static_cast<int64_t>(n) * a.Ho + (ok ? oy : 0)) * a.Wo + (ok ? ox : 0)) * a.cout;
#pragma unroll
        for (int ti = 0; ti < TI; ++ti) {
          uint2 pkp[2], adp[2];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = co_lane + ti * 32 + 8 * g;
            if ((g & 1) == 0 && FLIP == 1 && a.addend != nullptr && a.amask == nullptr) {  // uniform: 16-byte addend load
              uint4 raw = make_uint4(0u, 0u, 0u, 0u);
              if (ok) raw = *reinterpret_cast<const uint4*>(a.addend + off + co + 4 * fhi);
              pair_unswap16(raw, adp[0], adp[1]);
            }
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[ti][tj][4 * g + q];
            if (FLIP == 1 && a.addend != nullptr && ok) {
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
            uint2 pk;
            pk.x = pack2(v[0], v[1]);
            pk.y = pack2(v[2], v[3]);
            pkp[g & 1] = pk;
            if (g & 1) {  // 16-byte group pair (g - 1, g): pair_swap16
              const uint4 w = pair_swap16(pkp[0], pkp[1]);
              if (ok && !(a.dbg & 4)) {
                *reinterpret_cast<uint4*>(a.y + off + co - 8 + 4 * fhi) = w;
              }
            }
            if constexpr (STATS) {
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
      if constexpr (STATS) {
        if (a.dbg & 2) return;
        // full per-tile wave reduction; every (row, channel) slot of red has one owning lane
        float y1[TI * 16];
        stats_stage1<TI>(ts, tq, y1);
        stats_stage2<TI>(y1, lane, [&](int, int sq, int dc, float v) {
          red[(wm * 2 + sq) * kBN + wn * (TI * 32) + 4 * fhi + dc] += v;
        });
      }
    };
    produce();
  };

  // weights two taps ahead of their MFMAs: three register slots, K-steps g walked in threes
  bf16x8_t wr[3][TI][4];
  const int gtot = cch * 9;
  if (nsteps > 0) {
    halo_dma(0);
    wload(0, wr[0]);
    if (gtot > 1) wload(1, wr[1]);
  }
  for (int q = 0; q < nsteps; ++q) {
    const int c = q % cch;
    // this wave's halo DMA for chunk-step q landed (it is older than the weight loads of the
    // two K-steps in flight: at most those 2 x TI x 4 loads may still be outstanding -- with TI = 1
    // a wait for 16 would let the prologue's DMA still be in flight); the barrier publishes every
    // wave's halo and frees the other buffer (read by chunk-step q - 1)
    vm_wait<8 * TI>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c == 0 && q > 0) epilogue(mfirst + (q / cch - 1) * mstep);
    if (q + 1 < nsteps) halo_dma(q + 1);
    const uint4* hb = lds + (q & 1) * kHStage;
    // one tap: K-step g = c * 9 + 3 i + j, whose weights are in slot j (9 % 3 == 0)
    auto tap_step = [&](int i, auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int tap = 3 * i + j;
      const int g = c * 9 + tap;
      // prefetch the weights of K-step g + 2 (the next chunk's first taps, or the next tile's)
      const int gn = g + 2 < gtot ? g + 2 : g + 2 - gtot;
      if (q * 9 + tap + 2 < nsteps * 9) wload(gn, wr[(j + 2) % 3]);
      const int sh = FLIP ? (2 - i) * kHW + (2 - j) : i * kHW + j;
      bf16x8_t bfg[2][TJ];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = 2 * ks + fhi;
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj) {
          const int hr = hrow0 + (tj >> 1) * kHW + (tj & 1) * 32 + sh;
          bfg[ks & 1][tj] = as_frag(hb[hr * 8 + (ch ^ ((hr >> 1) & 7))]);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ti = 0; ti < TI; ++ti)
#pragma unroll
          for (int tj = 0; tj < TJ; ++tj)
            acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[j][ti][ks], bfg[ks & 1][tj], acc[ti][tj], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    };
    if constexpr (WL == 4) {
      // tap rows rolled: with 4 pixel tiles per wave, hoisting the 9 x 4 x 4 swizzled B-fragment
      // addresses of a fully unrolled chunk out of the loop spilled
#pragma unroll 1
      for (int i = 0; i < 3; ++i) {
        tap_step(i, std::integral_constant<int, 0>{});
        tap_step(i, std::integral_constant<int, 1>{});
        tap_step(i, std::integral_constant<int, 2>{});
      }
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        tap_step(i, std::integral_constant<int, 0>{});
        tap_step(i, std::integral_constant<int, 1>{});
        tap_step(i, std::integral_constant<int, 2>{});
      }
    }
  }
  if (nsteps > 0) epilogue(mfirst + (my_tiles - 1) * mstep);

  if constexpr (STATS) {
    // one slab row per block: the row groups' sums of each channel in a fixed order
    __syncthreads();
    for (int e = tid; e < 2 * kBN; e += kNW * 64) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NRG; ++w) s += red[w * 2 * kBN + e];
      const int sq = e >= kBN, cc = co0 + (sq ? e - kBN : e);
      a.part[static_cast<int64_t>(mfirst) * 2 * a.cout + (sq ? a.cout : 0) + cc] = s;
    }
  }
}

// WL 4's layout (8 waves: 2 row groups x 4 channel quarters, 1 x 4 accumulator tiles per wave)
// with DOUBLE-BUFFERED accumulators: tile t accumulates into one set while the epilogue of tile
// t - 1 drains the other set in four pieces (one 32-pixel tile each) placed between the MFMA taps
// of tile t's first chunk.  The plain kernel runs its epilogue with every wave between two chunk
// barriers, MFMA pipes idle: on the 128-channel layers (2 chunks per tile) that epilogue is 20 % of
// the kernel (RTSEG_HREG_DBG=1 A/B, profiles/r6_hreg).  Drained pieces overlap the other wave's
// MFMAs on the same SIMD.  BN statistics are reduced per piece (per 32-pixel tile: the VALU work of
// four reductions instead of one, issued beside MFMAs) into the same LDS slots; the residual-gradient
// addend of a piece is loaded before its tap's weight prefetch, so waiting for it never waits on
// that prefetch.
#ifndef RTSEG_HREG_DB_BFG
#define RTSEG_HREG_DB_BFG 2
#endif
template <int STATS, int FLIP>
__global__ void __launch_bounds__(512) hreg_db_kernel(const HrArgs a) {
  constexpr int NRG = 2, NCG = 4, kNW = 8, RPW = 2, TJ = 4, kBfgBuf = RTSEG_HREG_DB_BFG;
  __shared__ uint4 lds[2 * kHStage + kRed / 4];
  float* const red = reinterpret_cast<float*>(lds + 2 * kHStage);  // [row group][sum, sumsq][128]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NCG, wn = wid % NCG;
  const int G = gridDim.x;
  const int lb = xcd_logical(blockIdx.x, G);
  const int ntile = lb % a.ntiles;
  const int co0 = ntile * kBN;
  const int mstep = G / a.ntiles;
  const int mfirst = lb / a.ntiles;
  const int my_tiles = mfirst < a.mtiles ? (a.mtiles - mfirst + mstep - 1) / mstep : 0;
  const int cch = a.cch;
  const int nsteps = my_tiles * cch;
  const int lr8 = lane >> 3, lch = lane & 7;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, static_cast<int>(a.xbytes), 0x00020000);
  auto tile_xyz = [&](int mt, int& n, int& oy0, int& ox0) {
    const int tx = mt % a.tilesW;
    const int t2 = mt / a.tilesW;
    n = t2 / a.tilesH;
    oy0 = (t2 % a.tilesH) * kTH;
    ox0 = tx * kTW;
  };
  auto halo_dma = [&](int q) {
    const int mt = mfirst + (q / cch) * mstep, c0 = (q % cch) * 64;
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    const uint32_t base = lds_addr(lds + (q & 1) * kHStage);
    for (int e = wid; e < kHInstr; e += kNW) {
      const int r = e * 8 + lr8;
      const int hy = r / kHW, hx = r - hy * kHW;
      const int ih = oy0 - 1 + hy, iw = ox0 - 1 + hx;
      const bool ok = r < kHRows && static_cast<unsigned>(ih) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(a.W);
      const int lc = lch ^ ((r >> 1) & 7);
      const uint32_t v =
          ok ? static_cast<uint32_t>(((n * a.H + ih) * a.W + iw) * a.C + c0 + lc * 8) * 2u : 0x80000000u;
      bdma16(xr, v, base + e * 1024);
    }
  };

  const uint4* wbase = a.wp + (static_cast<int64_t>(co0 / 32 + wn) * cch * 9 * 4) * 64 + lane;
  auto wload = [&](int g, bf16x8_t (&dst)[4]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) dst[ks] = as_frag(wbase[(g * 4 + ks) * 64]);
  };
  const int frow = lane & 31, fhi = lane >> 5;
  const int hrow0 = wm * RPW * kHW + frow;

  f32x16_t acc0[TJ], acc1[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[j][r] = 0.f;
      acc1[j][r] = 0.f;
    }
  if constexpr (STATS) {
    for (int e = tid; e < kRed; e += kNW * 64) red[e] = 0.f;
  }
  const int co_lane = co0 + wn * 32 + 4 * fhi;
  const bool has_add = FLIP == 1 && a.addend != nullptr;
  const bool add16 = has_add && a.amask == nullptr;

  // output geometry of piece tj of tile mt (lane's pixel)
  auto piece_off = [&](int mt, int tj, bool& ok) -> int64_t {
    int n, oy0, ox0;
    tile_xyz(mt, n, oy0, ox0);
    const int oy = oy0 + wm * RPW + (tj >> 1), ox = ox0 + (tj & 1) * 32 + frow;
    ok = oy < a.Ho && ox < a.Wo;
    return ((static_cast<int64_t>(n) * a.Ho + (ok ? oy : 0)) * a.Wo + (ok ? ox : 0)) * a.cout;
  };
  // addend of piece tj (two 16-byte loads: channel groups (0, 1) and (2, 3))
  auto piece_load = [&](int mt, int tj, uint4 (&raw)[2]) {
    bool ok;
    const int64_t off = piece_off(mt, tj, ok);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      raw[h] = make_uint4(0u, 0u, 0u, 0u);
      if (ok) raw[h] = *reinterpret_cast<const uint4*>(a.addend + off + co_lane + 16 * h + 4 * fhi);
    }
  };
  // store (+ addend, + statistics) piece tj of tile mt from accumulator tile D, then zero D
  auto piece_drain = [&](f32x16_t& D, int mt, int tj, const uint4 (&raw)[2]) __attribute__((always_inline)) {
    if (a.dbg & 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) D[r] = 0.f;
      return;
    }
    bool ok;
    const int64_t off = piece_off(mt, tj, ok);
    float ts[1][16], tq[1][16];
    uint2 pkp[2], adp[2];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int co = co_lane + 8 * g;
      if ((g & 1) == 0 && add16) pair_unswap16(raw[g >> 1], adp[0], adp[1]);
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = D[4 * g + q];
      if (has_add && ok) {
        float r[4];
        if (add16) {
          bf16x4_unpack(adp[g & 1], r);
        } else {
          bf16x4_unpack(*reinterpret_cast<const uint2*>(a.addend + off + co), r);
          mask_addend4(a.amask, off + co, r);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += r[q];
      }
      uint2 pk;
      pk.x = pack2(v[0], v[1]);
      pk.y = pack2(v[2], v[3]);
      pkp[g & 1] = pk;
      if (g & 1) {
        const uint4 w = pair_swap16(pkp[0], pkp[1]);
        if (ok) *reinterpret_cast<uint4*>(a.y + off + co - 8 + 4 * fhi) = w;
      }
      if constexpr (STATS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float u = ok ? v[q] : 0.f;
          ts[0][4 * g + q] = u;
          tq[0][4 * g + q] = u * u;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) D[r] = 0.f;
    if constexpr (STATS) {
      float y1[16];
      stats_stage1<1>(ts, tq, y1);
      stats_stage2<1>(y1, lane, [&](int, int sq, int dc, float v) {
        red[(wm * 2 + sq) * kBN + wn * 32 + 4 * fhi + dc] += v;
      });
    }
  };

  bf16x8_t wr[3][4];
  const int gtot = cch * 9;
  if (nsteps > 0) {
    halo_dma(0);
    wload(0, wr[0]);
    if (gtot > 1) wload(1, wr[1]);
  }
  // one chunk-step q accumulating into A; at a tile's first chunk (q > 0) it drains D = the
  // previous tile's accumulators piece by piece between its taps
  auto run_chunk = [&](f32x16_t (&A)[TJ], f32x16_t (&D)[TJ], int q) __attribute__((always_inline)) {
    const int c = q % cch;
    vm_wait<8>();  // (the two K-steps of weight loads in flight, 4 each)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (q + 1 < nsteps) halo_dma(q + 1);
    const uint4* hb = lds + (q & 1) * kHStage;
    const bool drain = c == 0 && q > 0;
    const int mtD = mfirst + (q / cch - 1) * mstep;
    auto tap_step = [&](int i, auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int tap = 3 * i + j;
      const int g = c * 9 + tap;
      const int gn = g + 2 < gtot ? g + 2 : g + 2 - gtot;
      if (q * 9 + tap + 2 < nsteps * 9) wload(gn, wr[(j + 2) % 3]);
      const int sh = FLIP ? (2 - i) * kHW + (2 - j) : i * kHW + j;
      // the swizzled B-fragment addresses are recomputed per tap from an opaque copy of the lane's
      // row: hoisted out of the loop (4 tiles x 4 K-slices x 9 taps) they spilled
      int h0 = hrow0;
      asm volatile("" : "+v"(h0));
      bf16x8_t bfg[kBfgBuf][TJ];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = 2 * ks + fhi;
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj) {
          const int hr = h0 + (tj >> 1) * kHW + (tj & 1) * 32 + sh;
          bfg[ks % kBfgBuf][tj] = as_frag(hb[hr * 8 + (ch ^ ((hr >> 1) & 7))]);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          A[tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[j][ks], bfg[ks % kBfgBuf][tj], A[tj], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    };
    // taps 0..2 (row i = 0) peeled: piece tj drains after tap tj (pieces 2 and 3 after tap 2);
    // a piece's addend is loaded before its tap issues the weight prefetch
    uint4 raw[2] = {make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
    auto drain_piece = [&](auto tjc) __attribute__((always_inline)) {
      constexpr int tj = decltype(tjc)::value;
      if (drain) {
        if (add16) piece_load(mtD, tj, raw);
        piece_drain(D[tj], mtD, tj, raw);
      }
    };
    if (drain && add16) piece_load(mtD, 0, raw);
    tap_step(0, std::integral_constant<int, 0>{});
    if (drain) piece_drain(D[0], mtD, 0, raw);
    if (drain && add16) piece_load(mtD, 1, raw);
    tap_step(0, std::integral_constant<int, 1>{});
    if (drain) piece_drain(D[1], mtD, 1, raw);
    if (drain && add16) piece_load(mtD, 2, raw);
    tap_step(0, std::integral_constant<int, 2>{});
    if (drain) piece_drain(D[2], mtD, 2, raw);
    drain_piece(std::integral_constant<int, 3>{});
#pragma unroll 1
    for (int i = 1; i < 3; ++i) {
      tap_step(i, std::integral_constant<int, 0>{});
      tap_step(i, std::integral_constant<int, 1>{});
      tap_step(i, std::integral_constant<int, 2>{});
    }
  };
  int q = 0;
  for (int t = 0; t < my_tiles; t += 2) {
    for (int c = 0; c < cch; ++c, ++q) run_chunk(acc0, acc1, q);
    if (t + 1 < my_tiles)
      for (int c = 0; c < cch; ++c, ++q) run_chunk(acc1, acc0, q);
  }
  if (nsteps > 0) {  // the last tile's accumulators
    const int mt = mfirst + (my_tiles - 1) * mstep;
    auto drain_all = [&](f32x16_t (&D)[TJ]) {
      uint4 raw[2] = {make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        if (add16) piece_load(mt, tj, raw);
        piece_drain(D[tj], mt, tj, raw);
      }
    };
    if ((my_tiles - 1) & 1) drain_all(acc1);
    else drain_all(acc0);
  }
  if constexpr (STATS) {
    __syncthreads();
    for (int e = tid; e < 2 * kBN; e += kNW * 64) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NRG; ++w) s += red[w * 2 * kBN + e];
      const int sq = e >= kBN, cc = co0 + (sq ? e - kBN : e);
      a.part[static_cast<int64_t>(mfirst) * 2 * a.cout + (sq ? a.cout : 0) + cc] = s;
    }
  }
}

// weight packing: w [cout][3][3][C] (forward KRSC; data gradient [Cin][KH][KW][Cout]) ->
// [cout / 32][C / 64][9][4][64 lanes][8]: lane l of fragment (ti, chunk, tap, ks) holds
// w[ti * 32 + (l & 31)][tap][chunk * 64 + ks * 16 + (l >> 5) * 8 .. + 8]
__global__ void hreg_pack_kernel(const uint4* __restrict__ w, uint4* __restrict__ wp, int cout, int C) {
  const int cch = C / 64;
  const int64_t total = static_cast<int64_t>(cout / 32) * cch * 9 * 4 * 64;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int lane = static_cast<int>(e & 63);
    int64_t r = e >> 6;
    const int ks = static_cast<int>(r & 3); r >>= 2;
    const int tap = static_cast<int>(r % 9); r /= 9;
    const int c = static_cast<int>(r % cch);
    const int ti = static_cast<int>(r / cch);
    const int co = ti * 32 + (lane & 31);
    const int k = c * 64 + ks * 16 + (lane >> 5) * 8;
    wp[e] = w[((static_cast<int64_t>(co) * 9 + tap) * C + k) / 8];
  }
}

bool hreg_fill(HrArgs& k, const ConvGeom& g, bool dgrad) {
  const int red = dgrad ? g.cout : g.cin, outc = dgrad ? g.cin : g.cout;
  if (red % 64 != 0 || outc % kBN != 0) return false;
  if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1 || g.ph != 1 || g.pw != 1)
    return false;
  k.H = dgrad ? g.ho : g.h;
  k.W = dgrad ? g.wo : g.w_in;
  k.C = red;
  k.Ho = dgrad ? g.h : g.ho;
  k.Wo = dgrad ? g.w_in : g.wo;
  k.cout = outc;
  k.cch = red / 64;
  const int64_t xb = static_cast<int64_t>(g.n) * k.H * k.W * red * 2;
  if (xb >= (int64_t{1} << 31)) return false;
  k.xbytes = static_cast<uint32_t>(xb);
  k.tilesW = (k.Wo + kTW - 1) / kTW;
  k.tilesH = (k.Ho + kTH - 1) / kTH;
  k.mtiles = g.n * k.tilesW * k.tilesH;
  k.ntiles = outc / kBN;
  return true;
}

int hreg_grid(const HrArgs& k) {
  const int64_t tiles = static_cast<int64_t>(k.mtiles) * k.ntiles;
  const int cap = std::max(k.ntiles, (256 / k.ntiles) * k.ntiles);  // one block per CU (LDS-bound)
  return static_cast<int>(tiles < cap ? tiles : cap);
}

}  // namespace

bool conv_hreg_supported(const ConvGeom& g, int mode) {
  HrArgs k{};
  return hreg_fill(k, g, mode == 1);
}

int conv_hreg_slabs(const ConvGeom& g) {
  HrArgs k{};
  if (!hreg_fill(k, g, false)) return 0;
  return hreg_grid(k) / k.ntiles;
}

int64_t conv_hreg_pack_elems(const ConvGeom& g, int mode) {  // bf16 elements of the packed weights
  const int red = mode == 1 ? g.cout : g.cin, outc = mode == 1 ? g.cin : g.cout;
  return static_cast<int64_t>(outc) * 9 * red;
}

// forward (mode 0: g.x = x, g.w = wk [Cout][3][3][Cin]) or data gradient (mode 1: g.x = dy,
// g.w = wt [Cin][3][3][Cout], g.res = addend); wpack: conv_hreg_pack_elems bf16 of scratch
void launch_conv_hreg(const ConvGeom& g, int mode, void* wpack, hipStream_t st, int layout) {
  HrArgs k{};
  const bool dgrad = mode == 1;
  if (!hreg_fill(k, g, dgrad)) return;
  {
    const int64_t total = static_cast<int64_t>(k.cout / 32) * k.cch * 9 * 4 * 64;
    const int blocks = static_cast<int>(std::min<int64_t>((total + 255) / 256, 4096));
    hreg_pack_kernel<<<blocks, 256, 0, st>>>(static_cast<const uint4*>(g.w), static_cast<uint4*>(wpack), k.cout, k.C);
  }
  static const int dbg = [] { const char* e = std::getenv("RTSEG_HREG_DBG"); return e ? std::atoi(e) : 0; }();
  k.dbg = dbg;
  k.x = static_cast<const uint16_t*>(g.x);
  k.wp = static_cast<const uint4*>(wpack);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = dgrad ? nullptr : g.part;
  k.addend = dgrad ? static_cast<const uint16_t*>(g.res) : nullptr;
  k.amask = dgrad ? g.amask : nullptr;
  const int grid = hreg_grid(k);
  if (grid <= 0) return;
  auto go = [&](auto wl) {
    constexpr int WL = decltype(wl)::value;
    constexpr int T = HrLayout<WL>::NRG * HrLayout<WL>::NCG * 64;
    if (dgrad) hreg_conv_kernel<0, 1, WL><<<grid, T, 0, st>>>(k);
    else if (k.part != nullptr) hreg_conv_kernel<1, 0, WL><<<grid, T, 0, st>>>(k);
    else hreg_conv_kernel<0, 0, WL><<<grid, T, 0, st>>>(k);
  };
  if (layout == 5) {
    if (dgrad) hreg_db_kernel<0, 1><<<grid, 512, 0, st>>>(k);
    else if (k.part != nullptr) hreg_db_kernel<1, 0><<<grid, 512, 0, st>>>(k);
    else hreg_db_kernel<0, 0><<<grid, 512, 0, st>>>(k);
    return;
  }
  if (layout == 2) go(std::integral_constant<int, 2>{});
  else if (layout == 4) go(std::integral_constant<int, 4>{});
  else go(std::integral_constant<int, 1>{});
}

}  // namespace rtseg
