// Implicit-GEMM convolution family on bf16 MFMA (v_mfma_f32_32x32x16_bf16) for channels-last
// activations on gfx950: forward, data gradient and weight gradient of every dense conv.
//
// Reference sites: every dense conv of the zoo -- ConvBNAct (models/modules.py:73-85), DDRNet's
// RB / RBB residual blocks (ddrnet.py:168-219), SegHead (modules.py:161-166), DeConvBNAct's
// ConvTranspose2d (modules.py:89-108) -- which the reference leaves to cuDNN (fwd / bwd-data /
// bwd-filter) followed by separate BatchNorm passes.
//
// ---- igemm_gather_kernel: forward conv, dgrad and transposed conv ---------------------------
// D[co, m] = sum_{t, c} W[co, wtap[t], c] * X[pix(m, t), c]
//   m    : a pixel of a "virtual" output grid (N x Hv x Wv); it is written to
//          y[n, hv*osh + oph, wv*osw + opw, co] (osh = 1, oph = 0 for a plain conv; the
//          dgrad of a strided conv runs one launch per output phase, sub-pixel style),
//   t    : an entry of a tap table (dh[t], dw[t], wtap[t]); X's pixel is
//          (hv*sh + dh[t], wv*sw + dw[t]) -- zero outside the image.
// A forward conv is tap table {(-p + i*d, wtap = i*KW+j)}; the data gradient of a stride-s
// conv is, per phase (a, b), the taps with (a + p - i*d) % s == 0 at dh = (a + p - i*d) / s
// over dy, with weights re-laid-out [Cin][KH][KW][Cout] -- the same kernel, no col2im.
//
//  * block tile: BN output channels (MFMA A operand = weights) x BM pixels (B operand = gathered
//    activations) x BK = 64 (one tap, 64 channels) per K-step; 8 waves (WN x WM), each a
//    (BN/WN) x (BM/WM) sub-tile of 32 x 32 MFMA tiles (the 32-row shape halves the LDS fragment
//    reads per FLOP against 16x16x32);
//  * operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, per-lane source address =
//    the gather), 128-byte LDS rows with chunk c of row r at c ^ ((r >> 1) & 7) (source-side
//    swizzle), which makes every ds_read_b128 fragment read conflict-free;
//  * a persistent, XCD-contiguous tile walk with ONE flat DMA stream across tiles: the NST-stage
//    ring keeps NST-1 K-steps in flight across tile boundaries, published by a counted vmcnt +
//    raw s_barrier (never vmcnt(0) inside the stream);
//  * epilogue straight from the accumulators (D rows = channels: each lane owns 4 consecutive
//    channels of one pixel per register quad -> 8-byte stores), run after the NEXT K-step's
//    barrier and before its DMA issue, so the stores retire under that step's MFMAs and never
//    hold up a ring wait;
//    optional per-channel (sum, sum of squares) of the bf16 outputs for training BatchNorm
//    (one [2*Cout] slab row per block), or the inference BN scale/shift + residual + ReLU(6).
//
// ---- igemm_wgrad_kernel: weight gradient ----------------------------------------------------
// D[co, (t, ci)] = sum_m dy[m, co] * x[pix(m, t), ci]: K = pixels.  Both operands are staged as
// [64 pixels][64 channels] sub-tiles (one DMA stream, the x side gathered per tap) and read
// with ds_read_b64_tr_b16 (the hardware transpose delivers 4 consecutive pixels per lane),
// chunk swizzle c ^ (((r >> 1) & 1) << 2) makes those reads conflict-free.  The pixel range is
// split over blocks (split-K); fp32 partial tiles go to a slab that igemm_wgrad_reduce sums
// (deterministic, no atomics) into the [Cout][Cin][KH][KW] fp32 weight gradient.
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>
#include <cstdlib>

namespace rtseg {

namespace {

using namespace mdev;

constexpr int kMaxTaps = kIgemmMaxTaps;
constexpr int kMaxPhases = 16;
constexpr int kNullTap = 0xff;  // tap_wt of a padding tap (fused phases): zero weights, no gather

// 64 zero bytes: the DMA source of padding taps / rows past the edge
__device__ uint4 g_igemm_zero[4];

struct IgArgs {
  const uint16_t* x;
  const uint16_t* w;
  uint16_t* y;
  float* part;
  const float* ss;
  const uint16_t* res;
  const float* bias;      // [cout] added to the accumulators first (transposed conv), or null
  const uint16_t* addend; // bf16 tensor of the output's layout added in the epilogue, or null
  const uint8_t* amask;   // bit mask of the addend (mask_addend4), or null
  const uint16_t* vaddend; // addend indexed by the virtual pixel m ([M][cout]), or null
  int act;
  int H, W, C;            // gathered operand [N][H][W][C]
  int Hv, Wv;             // virtual output grid
  int Ho, Wo, cout;       // output tensor [N][Ho][Wo][cout]
  int osh, osw, oph, opw; // output pixel = (hv*osh + oph, wv*osw + opw)
  int sh, sw;             // input pixel = (hv*sh + dh[t], wv*sw + dw[t])
  int wrow;               // weight row stride (elements) = KT * C
  int ntap, cch, nk;      // taps, 64-channel chunks per tap, K-steps per tile
  int ksplit, nkp;        // EPI 2 (split K): K parts per output tile, K-steps per part (nk = ksplit * nkp)
  float* ws;              // EPI 2: fp32 partial sums [ksplit][M][cout]
  int nph;                // output phases per launch (fused dgrad of a strided conv), else 1
  int wide;               // 16-byte epilogue stores (channel-group pairs swapped across half-waves)
  int phase_off[kMaxPhases];  // phase q: oph | opw << 8 (nph > 1; taps of phase q at q * ntap)
  int M, mtiles, ntiles;
  FastDiv fwv, fhv;
  uint32_t xbytes;        // bytes of the gathered operand (<= 2^31: buffer range, GB kernels)
  uint32_t ybytes;        // bytes of the output (<= 2^31 for GB kernels: range-checked stores)
  int taps[kMaxTaps];     // packed tap: see pack_tap (32-bit so the scalar unit can load it)
};

// Two LDS-DMA gathers through a buffer resource (range-checked: a voffset past the buffer's
// size returns zeros -- the image border / padding needs no per-lane select of a zero source):
// 64 lanes x 16 B land at M0 + 16 * lane.  Inline asm (opaque to hipcc's waitcnt pass, see dma16);
// M0 is compiler-reserved, so it is saved and restored around the pair.
__device__ __forceinline__ void bdma16x2(__amdgpu_buffer_rsrc_t r, uint32_t v0, uint32_t d0, uint32_t v1,
                                         uint32_t d1) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "s"(r), "s"(d0), "s"(d1)
      : "memory");
}


// EPI: 0 = plain / statistics / data-gradient epilogues, 1 = inference BN (+ residual + act),
// 2 = split K: tile t of the walk is output tile t / ksplit over K part t % ksplit, whose fp32
// partial sums go to a.ws; splitk_bn_kernel sums the parts in order and applies the BN epilogue
// (batch-1 inference layers with too few output tiles to fill the CUs)
// STATS: 0 = none, 1 = forward BN statistics of the output
// GB: gather the activation rows through a buffer resource (range-checked voffsets, the
// border handled by the range check) instead of 64-bit flat addresses with a zero source, and
// store / load the output-layout tensors (y, residual, addend) through range-checked buffer
// resources too: a pixel past M or a channel past Cout gets an out-of-range offset (the store is
// dropped, the load returns 0) instead of an exec-mask branch around every 8-byte access.
// PH: fused output phases (launch_conv_igemm_dgrad_fused; a.nph > 1), a separate instantiation so
// that the phase bookkeeping costs the other launches no registers
template <int BM, int BN, int WM, int WN, int NST, int EPI, int STATS, int GB, int PH = 0>
__global__ void __launch_bounds__(WM* WN * 64) igemm_gather_kernel(const IgArgs a) {
  constexpr int NW = WM * WN;
  constexpr int TI = BN / WN / 32;  // 32-channel MFMA tiles per wave
  constexpr int TJ = BM / WM / 32;  // 32-pixel MFMA tiles per wave
  constexpr int STAGE = (BN + BM) * 8;  // 16-byte chunks per ring stage
  constexpr int WI = BN / 8 / NW, PI = BM / 8 / NW;  // DMA instructions per wave per stage
  static_assert(TI >= 1 && TJ >= 1 && TI * WN * 32 == BN && TJ * WM * 32 == BM, "wave tiling");
  static_assert(WI >= 1 && PI >= 1 && WI * NW * 8 == BN && PI * NW * 8 == BM, "DMA tiling");
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  static_assert(PI % 2 == 0, "gather DMAs are issued in pairs");
  constexpr int PER = WI + PI;
  __shared__ uint4 lds[NST * STAGE];

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
  const int nk = EPI == 2 ? a.nkp : a.nk;

  // ---- DMA geometry: instruction I fills 8 rows (I*8 + lane/8) x 8 chunks of one operand
  const int lr8 = lane >> 3, lch = lane & 7;
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
  int plc[PI];
#pragma unroll
  for (int e = 0; e < PI; ++e) {
    const int row = (wid * PI + e) * 8 + lr8;
    plc[e] = lch ^ ((row >> 1) & 7);
  }
  // gathered rows.  GB: byte offset of the row's (n, hv*sh, wv*sw) pixel + chunk (u32 voffset
  // of a buffer resource over x) and the pixel's (h, w); else a 64-bit base pointer
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.x), 0, static_cast<int>(a.xbytes), 0x00020000);
  uint32_t roff[GB ? PI : 1];
  const uint16_t* pbase[GB ? 1 : PI];
  int phb[PI], pwb[PI];
  // fused phases: tile t = spatial tile t / nph of phase t % nph (the phases of one spatial tile
  // are neighbouring tiles of the walk: adjacent blocks of one XCD share its dy rows in L2 and
  // fill complementary pixels of the same dx lines)
  const int P = PH ? a.nph : 1;
  int st_phase = 0;
  auto set_rows = [&](int tile) {
    int mt = tile;
    if (PH) { mt = tile / P; st_phase = tile - mt * P; }
    if constexpr (EPI == 2) mt = tile / a.ksplit;
#pragma unroll
    for (int e = 0; e < PI; ++e) {
      const int m = mt * BM + (wid * PI + e) * 8 + lr8;
      const bool ok = m < a.M;
      uint32_t wv, hv;
      const uint32_t t = a.fwv.divmod(static_cast<uint32_t>(ok ? m : 0), wv);
      const uint32_t n = a.fhv.divmod(t, hv);
      phb[e] = ok ? static_cast<int>(hv) * a.sh : -(1 << 28);
      pwb[e] = static_cast<int>(wv) * a.sw;
      if constexpr (GB) {
        roff[e] = static_cast<uint32_t>(((static_cast<int>(n) * a.H + phb[e]) * a.W + pwb[e]) * a.C + plc[e] * 8) * 2u;
      } else {
        pbase[e] = a.x + static_cast<int64_t>(n) * a.H * a.W * a.C + plc[e] * 8;
      }
    }
  };

  // staging cursor (wave-uniform): tile ordinal, tap, channel chunk
  int st_ord = 0, st_t = 0, st_c = 0, st_buf = 0, st_k = 0;
  auto split_cursor = [&](int tile) {  // EPI 2: the first K-step (tap, chunk) of the tile's part
    const int k0 = (tile % a.ksplit) * a.nkp;
    st_t = k0 / a.cch;
    st_c = k0 - st_t * a.cch;
  };
  auto stage = [&]() {
    // uniform indices -> scalar (SMEM) tap-table loads: a VGPR-indexed kernarg load is a VMEM
    // load whose s_waitcnt vmcnt(0) would drain the whole DMA ring every K-step
    const int tv = a.taps[__builtin_amdgcn_readfirstlane(st_phase * a.ntap + st_t)];
    const bool null_tap = PH && tap_wt(tv) == kNullTap;  // uniform
    const int dh = tap_dh(tv), dw = tap_dw(tv);
    const int c0 = __builtin_amdgcn_readfirstlane(st_c) * 64;
    const int woff = tap_wt(tv) * a.C + c0;
    const uint32_t base = lds_addr(lds + st_buf * STAGE);
#pragma unroll
    for (int e = 0; e < WI; ++e) {
      const void* src = wok[e] && !null_tap ? static_cast<const void*>(wsrc[e] + woff)
                                            : static_cast<const void*>(g_igemm_zero);
      dma16(src, base + (wid * WI + e) * 1024);
    }
    if constexpr (GB) {
      // uniform tap delta; an out-of-image tap moves the voffset past the buffer (zeros)
      const uint32_t delta = static_cast<uint32_t>((dh * a.W + dw) * a.C + c0) * 2u;
      const uint32_t pb = base + BN * 128 + wid * PI * 1024;
#pragma unroll
      for (int e = 0; e < PI; e += 2) {
        uint32_t v[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bool ok = !null_tap && static_cast<unsigned>(phb[e + q] + dh) < static_cast<unsigned>(a.H) &&
                          static_cast<unsigned>(pwb[e + q] + dw) < static_cast<unsigned>(a.W);
          v[q] = ok ? roff[e + q] + delta : 0x80000000u;
        }
        bdma16x2(xr, v[0], __builtin_amdgcn_readfirstlane(pb + e * 1024), v[1],
                 __builtin_amdgcn_readfirstlane(pb + (e + 1) * 1024));
      }
    } else {
#pragma unroll
      for (int e = 0; e < PI; ++e) {
        const int hi = phb[e] + dh, wi = pwb[e] + dw;
        const bool ok = !null_tap && static_cast<unsigned>(hi) < static_cast<unsigned>(a.H) &&
                        static_cast<unsigned>(wi) < static_cast<unsigned>(a.W);
        const uint16_t* src = pbase[e] + static_cast<int64_t>(hi * a.W + wi) * a.C + c0;
        dma16(ok ? static_cast<const void*>(src) : static_cast<const void*>(g_igemm_zero),
              base + BN * 128 + (wid * PI + e) * 1024);
      }
    }
    if (++st_buf == NST) st_buf = 0;
    if constexpr (EPI == 2) {
      if (++st_k == a.nkp) {  // this K part is staged: the next tile's part
        st_k = 0;
        if (++st_ord < my_tiles) {
          set_rows(mfirst + st_ord * mstep);
          split_cursor(mfirst + st_ord * mstep);
        }
      } else if (++st_c == a.cch) {
        st_c = 0;
        ++st_t;
      }
    } else {
      if (++st_c == a.cch) {
        st_c = 0;
        if (++st_t == a.ntap) {
          st_t = 0;
          if (++st_ord < my_tiles) set_rows(mfirst + st_ord * mstep);
        }
      }
    }
  };

  // ---- fragment read geometry (ds_read_b128, conflict-free by the chunk swizzle)
  const int frow = lane & 31, fhi = lane >> 5, fx = (lane >> 1) & 7;

  f32x16_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;


  // A finished tile is packed and stored at the start of the NEXT K-step, after its barrier and
  // before its DMA issue: the accumulators are the deferred buffer (no extra registers), and the
  // stores get a whole compute step to retire before any counted vmcnt waits behind them.
  int64_t pend_off[GB ? 1 : TJ];
  uint32_t poff[GB ? TJ : 1];  // GB: byte offset of the pixel's row in y, or out of range
  const int co_lane = co0 + wn * (BN / WN) + 4 * fhi;  // + ti*32 + 8g
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, static_cast<int>(a.ybytes), 0x00020000);
  const uint16_t* side = EPI == 1 ? a.res : a.addend;  // an output-layout tensor read in the epilogue
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(side), 0, side != nullptr ? static_cast<int>(a.ybytes) : 0, 0x00020000);
  // STATS: this lane's BN statistics summed over all of the block's tiles (they share the channel
  // tile).  SP1: kept after the first reduce-scatter stage (TI * 16 registers; per tile only the
  // cheap stage 1), else -- the 512 x 128 tiles, which would spill -- after the whole per-tile
  // reduction (2 * TI * 16 / 32 registers)
  constexpr bool SP1 = BM * BN < 512 * 128;
  constexpr int NPS = !STATS ? 1 : SP1 ? TI * 16 : TI;
  float pst[NPS];
#pragma unroll
  for (int k = 0; k < NPS; ++k) pst[k] = 0.f;

  auto pack_tile = [&](int tile) __attribute__((always_inline)) {
    if constexpr (EPI == 2) {  // fp32 partial sums of K part tile % ksplit, 16-byte stores
      const int mt = tile / a.ksplit, kp = tile - mt * a.ksplit;
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        const int m = mt * BM + wm * (BM / WM) + tj * 32 + frow;
#pragma unroll
        for (int ti = 0; ti < TI; ++ti) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = co_lane + ti * 32 + 8 * g;
            if (m < a.M && co < a.cout)
              *reinterpret_cast<float4*>(a.ws + (static_cast<int64_t>(kp) * a.M + m) * a.cout + co) =
                  make_float4(acc[ti][tj][4 * g], acc[ti][tj][4 * g + 1], acc[ti][tj][4 * g + 2], acc[ti][tj][4 * g + 3]);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[ti][tj][r] = 0.f;
        }
      }
      return;
    }
    int mt = tile, oph = a.oph, opw = a.opw;
    bool phase0 = true;
    if (PH) {
      mt = tile / P;
      const int q = tile - mt * P;
      oph = a.phase_off[q] & 0xff;
      opw = a.phase_off[q] >> 8;
      phase0 = q == 0;
    }
    {
      // BN statistics of this tile: per-lane partial sums over the lane's TJ pixels
      float ts[STATS ? TI : 1][16], tq[STATS ? TI : 1][16];
      if constexpr (STATS) {
        #pragma unroll
        for (int i = 0; i < TI; ++i)
          #pragma unroll
          for (int r = 0; r < 16; ++r) { ts[i][r] = 0.f; tq[i][r] = 0.f; }
      }
      #pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        const int m = mt * BM + wm * (BM / WM) + tj * 32 + frow;
        const bool ok = m < a.M;
        uint32_t wv, hv;
        const uint32_t t = a.fwv.divmod(static_cast<uint32_t>(ok ? m : 0), wv);
        const uint32_t n = a.fhv.divmod(t, hv);
        const int ho = static_cast<int>(hv) * a.osh + oph, wo = static_cast<int>(wv) * a.osw + opw;
        if constexpr (GB) {
          poff[tj] = ok ? ((n * static_cast<uint32_t>(a.Ho) + ho) * static_cast<uint32_t>(a.Wo) + wo) *
                              static_cast<uint32_t>(a.cout) * 2u
                        : 0x80000000u;
        } else {
          pend_off[tj] = ((static_cast<int64_t>(n) * a.Ho + ho) * a.Wo + wo) * a.cout;
        }
        #pragma unroll
        for (int ti = 0; ti < TI; ++ti) {
          // channel groups in pairs (g2, g2 + 1): lane l < 32 holds channels 8g + 0..3 of pixel l,
          // lane l + 32 channels 8g + 4..7 of the same pixel; one v_permlane32_swap per dword
          // gives lanes < 32 channels 8 g2 .. 8 g2 + 7 and lanes >= 32 the next 8 -> one 16-byte
          // store per pair instead of two 8-byte ones (WIDE: RTSEG_IGEMM_WIDE_STORE=0 off, A/B)
          #pragma unroll
          for (int g2 = 0; g2 < 4; g2 += 2) {
          uint2 pkp[2];
          #pragma unroll
          for (int g = g2; g < g2 + 2; ++g) {
            const int co = co_lane + ti * 32 + 8 * g;
            float v[4];
            #pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[ti][tj][4 * g + q];
            // GB: the byte offset of these 4 channels, out of range past M or Cout
            uint32_t voff = 0;
            if constexpr (GB) voff = co < a.cout ? poff[tj] + static_cast<uint32_t>(co) * 2u : 0x80000000u;
            float sv[4] = {0.f, 0.f, 0.f, 0.f};  // residual (EPI 1) / addend (EPI 0) values
            if (side != nullptr && (EPI == 1 || STATS == 0)) {
              if constexpr (GB) {
                const auto r = __builtin_amdgcn_raw_buffer_load_b64(sr, voff, 0, 0);
                bf16x4_unpack(make_uint2(r[0], r[1]), sv);
                if (EPI == 0 && a.amask != nullptr && voff < a.ybytes) mask_addend4(a.amask, voff >> 1, sv);
              } else if (ok && co < a.cout) {
                bf16x4_unpack(*reinterpret_cast<const uint2*>(side + pend_off[tj] + co), sv);
                if (EPI == 0 && a.amask != nullptr) mask_addend4(a.amask, pend_off[tj] + co, sv);
              }
            }
            if constexpr (EPI == 0 && STATS == 0) {
              if (a.bias != nullptr) {  // transposed conv
                const float4 bb = *reinterpret_cast<const float4*>(a.bias + min(co, a.cout - 4));
                v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
              }
              if (side != nullptr) {  // e.g. a residual branch's gradient
                #pragma unroll
                for (int q = 0; q < 4; ++q) v[q] += sv[q];
              }
              if (a.vaddend != nullptr && phase0 && ok && co < a.cout) {  // e.g. a strided 1 x 1 shortcut's dx
                float pv[4];
                bf16x4_unpack(*reinterpret_cast<const uint2*>(a.vaddend + static_cast<int64_t>(m) * a.cout + co), pv);
                #pragma unroll
                for (int q = 0; q < 4; ++q) v[q] += pv[q];
              }
            }
            if constexpr (EPI == 1) {
              const int cc = min(co, a.cout - 4);
              const float4 sc = *reinterpret_cast<const float4*>(a.ss + cc);
              const float4 sf = *reinterpret_cast<const float4*>(a.ss + a.cout + cc);
              v[0] = fmaf(v[0], sc.x, sf.x); v[1] = fmaf(v[1], sc.y, sf.y);
              v[2] = fmaf(v[2], sc.z, sf.z); v[3] = fmaf(v[3], sc.w, sf.w);
              if (side != nullptr) {
                #pragma unroll
                for (int q = 0; q < 4; ++q) v[q] += sv[q];
              }
              #pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = epi_act(v[q], a.act);
            }
            uint2 pk;
            pk.x = pack2(v[0], v[1]);
            pk.y = pack2(v[2], v[3]);
            pkp[g - g2] = pk;
            if (!a.wide) {
              if constexpr (GB) {
                typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk.x, pk.y}, yr, voff, 0, 0);
              } else if (ok && co < a.cout) {
                *reinterpret_cast<uint2*>(a.y + pend_off[tj] + co) = pk;
              }
            }
            if constexpr (STATS) {
              // statistics of the fp32 conv outputs, straight from the accumulators: STATS == 1
              // launches (training forward) carry no bias / addend, and rows past M or channels
              // past Cout accumulated exactly zero (zero DMA sources), so nothing needs masking --
              // 2 VALU per value instead of a bf16 round trip + select
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                ts[ti][4 * g + q] += v[q];
                tq[ti][4 * g + q] = fmaf(v[q], v[q], tq[ti][4 * g + q]);
              }
            }
          }
          if (a.wide) {
            {
              const auto rx = __builtin_amdgcn_permlane32_swap(pkp[0].x, pkp[1].x, false, false);
              const auto ry = __builtin_amdgcn_permlane32_swap(pkp[0].y, pkp[1].y, false, false);
              pkp[0].x = rx[0]; pkp[1].x = rx[1];
              pkp[0].y = ry[0]; pkp[1].y = ry[1];
            }
            const int co = co_lane + ti * 32 + 8 * g2 + 4 * fhi;  // lanes >= 32: the next group
            if constexpr (GB) {
              typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
              const uint32_t voff = co < a.cout ? poff[tj] + static_cast<uint32_t>(co) * 2u : 0x80000000u;
              __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{pkp[0].x, pkp[0].y, pkp[1].x, pkp[1].y}, yr, voff, 0, 0);
            } else {
              if (ok && co < a.cout)
                *reinterpret_cast<uint4*>(a.y + pend_off[tj] + co) = make_uint4(pkp[0].x, pkp[0].y, pkp[1].x, pkp[1].y);
            }
          }
          }
          #pragma unroll
          for (int r = 0; r < 16; ++r) acc[ti][tj][r] = 0.f;
        }
      }
      if constexpr (STATS) {
        // first reduce-scatter stage only (rtseg_mfma_dev.h), summed over the block's tiles (all
        // of them share the channel tile); the rest of the reduction runs once, at the end
        float y1[TI * 16];
        stats_stage1<TI>(ts, tq, y1);
        if constexpr (SP1) {
#pragma unroll
          for (int k = 0; k < TI * 16; ++k) pst[k] += y1[k];
        } else {
          stats_stage2<TI>(y1, lane, [&](int k, int, int, float v) { pst[k] += v; });
        }
      }
    }
  };
  const int total = my_tiles * nk;
  if (nk == 0) {  // empty tap set (a dgrad phase no tap reaches): the outputs are zero
    for (int i = 0; i < my_tiles; ++i) pack_tile(mfirst + i * mstep);
  } else {
    if (my_tiles > 0) {
      set_rows(mfirst);
      if constexpr (EPI == 2) split_cursor(mfirst);
    }
#pragma unroll
    for (int p = 0; p < NST - 1; ++p)
      if (p < total) stage();

    int kk = 0, ord = 0, buf = 0, pend_mt = -1;
    for (int gs = 0; gs < total; ++gs) {
      if (NST >= 3 && gs + 1 < total) {
        vm_wait<(NST - 2) * PER>();
      } else {
        vm_wait<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // step gs landed for every wave; step gs-1's buffer is free
      if (pend_mt >= 0) {  // previous tile: epilogue + stores, ahead of this step's DMA issue
        pack_tile(pend_mt);
        pend_mt = -1;
      }
      if (gs + NST - 1 < total) stage();

      const uint4* Wt = lds + buf * STAGE + (wn * (BN / WN) + frow) * 8;
      const uint4* Pt = lds + buf * STAGE + BN * 8 + (wm * (BM / WM) + frow) * 8;
      // fragments of sub-step s+1 are read while the MFMAs of sub-step s run (double-buffered
      // registers for the 64 x 64 wave tiles; the 64 x 128 ones have no room and rely on the
      // partner wave of the SIMD to cover the read latency)
      constexpr int FB = TI + TJ <= 4 ? 2 : 1;
      bf16x8_t af[FB][TI], bfg[FB][TJ];
      auto load_frags = [&](int s, int slot) {
        const int ch = ((2 * s + fhi) ^ fx);
#pragma unroll
        for (int ti = 0; ti < TI; ++ti) af[slot][ti] = as_frag(Wt[ti * 256 + ch]);
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj) bfg[slot][tj] = as_frag(Pt[tj * 256 + ch]);
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
      if (++kk == nk) {
        kk = 0;
        pend_mt = mfirst + ord * mstep;
        ++ord;
      }
    }
    if (pend_mt >= 0) pack_tile(pend_mt);
  }

  if constexpr (STATS) {
    // finish the reduction once per block: DPP stages per wave, then the WM pixel waves of each
    // channel range summed in a fixed order through LDS -> ONE slab row per block (row = the
    // block's M-walk start, every (row, channel) written exactly once: deterministic, <= 256 rows)
    __syncthreads();  // every wave is past its last fragment read; no DMA is in flight
    float* red = reinterpret_cast<float*>(lds);  // [WM][2][BN]
    const int cl = wn * (BN / WN) + 4 * fhi;
    if constexpr (SP1) {
      stats_stage2<TI>(pst, lane, [&](int, int sq, int dc, float v) { red[(wm * 2 + sq) * BN + cl + dc] = v; });
    } else {
#pragma unroll
      for (int k = 0; k < NPS; ++k) {
        int sq, dc;
        stats_slot<TI>(k, lane, sq, dc);
        red[(wm * 2 + sq) * BN + cl + dc] = pst[k];
      }
    }
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

// ------------------------------------------------------------------------------- wgrad
struct WgArgs {
  const uint16_t* x;
  const uint16_t* dy;
  float* ws;
  int H, W, C, Ho, Wo, cout, sh, sw;
  int kp;          // KT * C (GEMM N)
  int M, ksteps, steps_per_split;
  int ntiles, tiles;
  FastDiv fwo, fho;
  int taps[kMaxTaps];  // pack_tap(dh, dw, tap)
};

// transposed 4 x bf16 read: lane (within its 16-lane group) 4q+p supplies row q, columns 4p..4p+3
__device__ __forceinline__ i16x4_t tr_read(const uint4* base, int byte_off) {
  auto p = (__attribute__((address_space(3))) i16x4_t*)(
      (__attribute__((address_space(3))) char*)((__attribute__((address_space(3))) void*)base) + byte_off);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
}

template <int MS, int NS, int WM, int WN, int NST>
__global__ void __launch_bounds__(WM* WN * 64) igemm_wgrad_kernel(const WgArgs a) {
  constexpr int NW = WM * WN;
  static_assert(NW == 8, "one DMA row group per wave");
  constexpr int SUB = 512;  // 16-byte chunks per [64][64] bf16 sub-tile
  constexpr int STAGE = (MS + NS) * SUB;
  constexpr int BMc = MS * 64, BNk = NS * 64;
  constexpr int TI = BMc / WM / 32, TJ = BNk / WN / 32;
  static_assert(TI >= 1 && TJ >= 1 && TI * WM * 32 == BMc && TJ * WN * 32 == BNk, "wave tiling");
  constexpr int PER = MS + NS;  // DMA instructions per wave per stage
  __shared__ uint4 lds[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lb = xcd_logical(blockIdx.x, gridDim.x);
  const int split = lb / a.tiles, tile = lb % a.tiles;
  const int co0 = (tile / a.ntiles) * BMc, kp0 = (tile % a.ntiles) * BNk;
  const int s0 = split * a.steps_per_split;
  const int s1 = min(s0 + a.steps_per_split, a.ksteps);
  const int nsteps = max(s1 - s0, 0);

  // DMA: wave w fills row group w (rows 8w .. 8w+7) of every sub-tile; lane -> row, chunk
  const int row = wid * 8 + (lane >> 3);
  const int lc = (lane & 7) ^ (((row >> 1) & 1) << 2);
  int aoff[MS];
  bool aok[MS];  // sub-tiles past Cout (a tile wider than the layer) read the zero page
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    aok[s] = co0 + s * 64 < a.cout;
    aoff[s] = co0 + s * 64 + lc * 8;
  }
  int bdh[NS], bdw[NS], boff[NS];
  bool bok[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int kb = kp0 + s * 64;
    bok[s] = kb < a.kp;
    const int t = __builtin_amdgcn_readfirstlane(bok[s] ? kb / a.C : 0);  // scalar table loads
    const int tv = a.taps[t];
    bdh[s] = tap_dh(tv);
    bdw[s] = tap_dw(tv);
    boff[s] = (bok[s] ? kb - t * a.C : 0) + lc * 8;
  }
  auto stage = [&](int step, int buf) {
    const int m = step * 64 + row;
    const bool mok = m < a.M;
    uint32_t wo, ho;
    const uint32_t t = a.fwo.divmod(static_cast<uint32_t>(mok ? m : 0), wo);
    const uint32_t n = a.fho.divmod(t, ho);
    const uint16_t* ximg = a.x + static_cast<int64_t>(n) * a.H * a.W * a.C;
    const uint32_t base = lds_addr(lds + buf * STAGE) + wid * 1024;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      const void* src = (mok && aok[s]) ? static_cast<const void*>(a.dy + static_cast<int64_t>(m) * a.cout + aoff[s])
                                        : static_cast<const void*>(g_igemm_zero);
      dma16(src, base + s * SUB * 16);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int hi = static_cast<int>(ho) * a.sh + bdh[s], wi = static_cast<int>(wo) * a.sw + bdw[s];
      const bool ok = mok && bok[s] && static_cast<unsigned>(hi) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(wi) < static_cast<unsigned>(a.W);
      const uint16_t* src = ximg + static_cast<int64_t>(hi * a.W + wi) * a.C + boff[s];
      dma16(ok ? static_cast<const void*>(src) : static_cast<const void*>(g_igemm_zero),
            base + (MS + s) * SUB * 16);
    }
  };

  // transposed fragment reads: lane -> (row q within the 4-row block, column 4p), group g16
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = (lane >> 4) & 1, hh = lane >> 5;
  const int swz = ((q >> 1) & 1) << 2;
  auto frag = [&](const uint4* sub, int col0, int k0) -> bf16x8_t {
    // col0: first of the 32 columns of this MFMA operand tile within the [64][64] sub-tile
    const int col = col0 + g16 * 16 + p4;
    const int ch = ((col >> 3) ^ swz);
    const int half = (col >> 2) & 1;
    const int r0 = k0 + hh * 8 + q;
    const i16x4_t lo = tr_read(sub, r0 * 128 + ch * 16 + half * 8);
    const i16x4_t hi = tr_read(sub, (r0 + 4) * 128 + ch * 16 + half * 8);
    return __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, lo), __builtin_bit_cast(bf16x4_t, hi), 0, 1, 2,
                                   3, 4, 5, 6, 7);
  };

  f32x16_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int pp = 0; pp < NST - 1; ++pp)
    if (pp < nsteps) stage(s0 + pp, pp);
  int buf = 0;
  for (int k = 0; k < nsteps; ++k) {
    if (NST >= 3 && k + 1 < nsteps) {
      vm_wait<(NST - 2) * PER>();
    } else {
      vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (k + NST - 1 < nsteps) {
      int nb = buf + NST - 1;
      if (nb >= NST) nb -= NST;
      stage(s0 + k + NST - 1, nb);
    }
    const uint4* A = lds + buf * STAGE;
    const uint4* B = A + MS * SUB;
    bf16x8_t af[2][TI], bfg[2][TJ];
    auto load_frags = [&](int s, int slot) {
#pragma unroll
      for (int ti = 0; ti < TI; ++ti) {
        const int c = wm * (BMc / WM) + ti * 32;
        af[slot][ti] = frag(A + (c >> 6) * SUB, c & 63, s * 16);
      }
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) {
        const int c = wn * (BNk / WN) + tj * 32;
        bfg[slot][tj] = frag(B + (c >> 6) * SUB, c & 63, s * 16);
      }
    };
    load_frags(0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s < 3) load_frags(s + 1, (s + 1) & 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ti = 0; ti < TI; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s & 1][ti], bfg[s & 1][tj], acc[ti][tj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (++buf == NST) buf = 0;
  }

  // fp32 partial tile -> slab [split][cout][kp]
  float* slab = a.ws + static_cast<int64_t>(split) * a.cout * a.kp;
#pragma unroll
  for (int ti = 0; ti < TI; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      const int kcol = kp0 + wn * (BNk / WN) + tj * 32 + (lane & 31);
      if (kcol >= a.kp) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * (BMc / WM) + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (co < a.cout) slab[static_cast<int64_t>(co) * a.kp + kcol] = acc[ti][tj][r];
      }
    }
}

// Split-K reduction, deterministic.  Stage 1 (only when there are > 16 splits): groups of 16
// slab rows -> one partial row each, float4 per thread, 16 loads in flight.  Stage 2: sum the
// (<= 16) remaining rows and write dw[co][ci][tap] from slab column co * KT*C + tap*C + ci.
__global__ void igemm_wgrad_reduce16(const float4* __restrict__ ws, float4* __restrict__ out, int splits,
                                     int64_t plane4) {
  const int64_t c = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (c >= plane4) return;
  const int s0 = blockIdx.y * 16, s1 = min(s0 + 16, splits);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 16
  for (int sp = s0; sp < s1; ++sp) {
    const float4 v = ws[sp * plane4 + c];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  out[blockIdx.y * plane4 + c] = acc;
}

// KRSC: dw in the slab's own [Cout][KH][KW][Cin] order -- the memory order of a channels-last
// [Cout, Cin, KH, KW] parameter, so the gradient already has the parameter's strides (what the
// fused optimizer and DDP's bucket views need); otherwise the NCHW order [Cout][Cin][KH][KW].
template <bool KRSC>
__global__ void igemm_wgrad_reduce(const float* __restrict__ ws, float* __restrict__ dw, int rows, int cout,
                                   int C, int kt) {
  const int64_t kp = static_cast<int64_t>(kt) * C;
  const int64_t plane = static_cast<int64_t>(cout) * kp;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < plane;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float s = 0.f;
#pragma unroll 16
    for (int sp = 0; sp < rows; ++sp) s += ws[sp * plane + e];
    if constexpr (KRSC) {
      dw[e] = s;
    } else {
      const int64_t co = e / kp;
      const int64_t r = e - co * kp;
      const int64_t t = r / C, ci = r - t * C;
      dw[(co * C + ci) * kt + t] = s;
    }
  }
}

// ------------------------------------------------------------------------------- host side
// Block-tile configurations (BM pixels x BN channels, WM x WN waves, NST ring stages):
//   0: 256 x  64, 4 x 2 waves (32 x 64 wave tiles), 3 stages, 120 KiB
//   1: 256 x 128, 4 x 2 waves (64 x 64),            3 stages, 144 KiB
//   2: 512 x  64, 8 x 1 waves (64 x 64),            2 stages, 144 KiB  -- Cout <= 64
//   3: 256 x 256, 2 x 4 waves (64 x 128),           2 stages, 128 KiB  -- Cout >= 256
//   4: 512 x 128, 4 x 2 waves (64 x 128),           2 stages, 160 KiB  -- Cout 65..128 (..255)
//   5: 128 x  64, 2 x 2 waves (64 x 32),            3 stages,  72 KiB, 2 blocks per CU -- the
//      inference BN epilogue only, on request (conv_igemm_small): batch-1 layers whose 256-pixel
//      tiles leave most of the 256 CUs idle (DDRNet-23's 1/16 and 1/32 branches: 32-64 blocks)
// The big wave tiles halve the LDS fragment reads per MFMA (profiles/r2_conv_igemm: 64 x 128
// tiles beat MIOpen's forward and its backward-data by 1.1-1.5x at batch 32); problems with
// fewer than one tile per CU fall back to the smaller tiles.
// RTSEG_IGEMM_CFG=<n> forces one (A/B sweeps, tools/bench_conv.py --cfgs).
struct Cfg {
  int id, bm, bn, wm;
};
constexpr Cfg kCfgs[] = {{0, 256, 64, 4}, {1, 256, 128, 4}, {2, 512, 64, 8}, {3, 256, 256, 2}, {4, 512, 128, 4},
                         {5, 128, 64, 2}};
constexpr int kShapeCfgs = 5;  // 0..4 are picked by shape / RTSEG_IGEMM_CFG; 5 only on request

int64_t cfg_tiles(const Cfg& c, int64_t M, int cout) { return ((M + c.bm - 1) / c.bm) * ((cout + c.bn - 1) / c.bn); }

Cfg pick_cfg(int cout, int64_t M) {
  const char* e = std::getenv("RTSEG_IGEMM_CFG");
  if (e != nullptr && *e != '\0') {
    const int i = std::atoi(e);
    if (i >= 0 && i < kShapeCfgs) return kCfgs[i];
  }
  const Cfg big = cout <= 64 ? kCfgs[2] : cout <= 128 ? kCfgs[4] : kCfgs[3];
  const Cfg small = cout <= 64 ? kCfgs[0] : kCfgs[1];
  return cfg_tiles(big, M, cout) >= 256 ? big : small;
}

int persistent_grid(int mtiles, int ntiles, int per_cu = 1) {
  const int64_t tiles = static_cast<int64_t>(mtiles) * ntiles;
  const int cap = std::max(ntiles, (256 * per_cu / ntiles) * ntiles);  // per_cu blocks per CU (LDS-bound)
  return static_cast<int>(tiles < cap ? tiles : cap);
}

void fill_common(IgArgs& k, const Cfg& c, int n) {
  if (k.nph < 1) k.nph = 1;
  const char* we = std::getenv("RTSEG_IGEMM_WIDE_STORE");  // read per launch (A/B in one process)
  k.wide = (we != nullptr && we[0] == '0') ? 0 : 1;
  k.M = n * k.Hv * k.Wv;
  k.mtiles = (k.M + c.bm - 1) / c.bm * k.nph;  // nph > 1: every phase walks the same pixel tiles
  k.ntiles = (k.cout + c.bn - 1) / c.bn;
  k.nk = k.ntap * k.cch;
  k.fwv = FastDiv::make(static_cast<uint32_t>(k.Wv));
  k.fhv = FastDiv::make(static_cast<uint32_t>(k.Hv));
}

template <int EPI, int STATS, int GB, int PH = 0>
void launch_cfg(const IgArgs& k, const Cfg& c, int grid, hipStream_t st) {
  switch (c.id) {
    case 0: igemm_gather_kernel<256, 64, 4, 2, 3, EPI, STATS, GB, PH><<<grid, 512, 0, st>>>(k); break;
    case 2: igemm_gather_kernel<512, 64, 8, 1, 2, EPI, STATS, GB, PH><<<grid, 512, 0, st>>>(k); break;
    case 3:
      if constexpr (EPI == 0) igemm_gather_kernel<256, 256, 2, 4, 2, 0, STATS, GB, PH><<<grid, 512, 0, st>>>(k);
      break;
    case 4:
      if constexpr (EPI == 0) igemm_gather_kernel<512, 128, 4, 2, 2, 0, STATS, GB, PH><<<grid, 512, 0, st>>>(k);
      break;
    case 5:
      if constexpr ((EPI == 1 || EPI == 2) && STATS == 0 && PH == 0)
        igemm_gather_kernel<128, 64, 2, 2, 3, EPI, 0, GB, 0><<<grid, 256, 0, st>>>(k);
      break;
    default: igemm_gather_kernel<256, 128, 4, 2, 3, EPI, STATS, GB, PH><<<grid, 512, 0, st>>>(k); break;
  }
}

// the buffer gather needs the gathered operand within a 2^31-byte range; RTSEG_IGEMM_GATHER=0
// forces the flat-address gather (A/B)
bool use_buffer_gather(const IgArgs& k) {
  static const int mode = std::getenv("RTSEG_IGEMM_GATHER") ? std::atoi(std::getenv("RTSEG_IGEMM_GATHER")) : 1;
  return mode != 0 && k.xbytes != 0 && k.xbytes <= 0x80000000u && k.ybytes != 0 && k.ybytes <= 0x80000000u;
}

template <int EPI, int STATS>
void launch_cfg(const IgArgs& k, const Cfg& c, int grid, hipStream_t st) {
  if (use_buffer_gather(k)) launch_cfg<EPI, STATS, 1>(k, c, grid, st);
  else launch_cfg<EPI, STATS, 0>(k, c, grid, st);
}

// out[r][c] = sum_{i < chunk} in[r * chunk + i][c] (rows past `rows` count as zero).
__global__ void slab_compact_kernel(const float* __restrict__ in, int rows, int width, int chunk,
                                    float* __restrict__ out) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= width) return;
  const int r0 = blockIdx.x * chunk, r1 = min(r0 + chunk, rows);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += in[static_cast<int64_t>(r) * width + c];
  out[static_cast<int64_t>(blockIdx.x) * width + c] = s;
}

void launch_gather(const IgArgs& k, const Cfg& c, hipStream_t st) {
  const int grid = persistent_grid(k.mtiles, k.ntiles, c.id == 5 ? 2 : 1);
  if (grid <= 0) return;
  if (k.nph > 1) {  // fused dgrad phases: data-gradient epilogue only
    if (use_buffer_gather(k)) launch_cfg<0, 0, 1, 1>(k, c, grid, st);
    else launch_cfg<0, 0, 0, 1>(k, c, grid, st);
    return;
  }
  if (k.ws != nullptr) launch_cfg<2, 0>(k, c, grid, st);
  else if (k.ss != nullptr) launch_cfg<1, 0>(k, c, grid, st);
  else if (k.part != nullptr) launch_cfg<0, 1>(k, c, grid, st);
  else launch_cfg<0, 0>(k, c, grid, st);
}

}  // namespace

bool conv_igemm_supported(const ConvGeom& g, int mode) {
  const int red = mode == 1 ? g.cout : g.cin;  // reduction channels (dgrad: forward Cout)
  const int outc = mode == 1 ? g.cin : g.cout;
  if (red % 64 != 0 || outc % 8 != 0) return false;
  if (g.kh * g.kw > kMaxTaps) return false;
  // tap offsets are packed as 8-bit signed values (pack_tap)
  if ((g.kh - 1) * g.dh + g.ph > 127 || (g.kw - 1) * g.dw + g.pw > 127) return false;
  if (mode == 2 && (g.cout % 64 != 0)) return false;
  return true;
}

// BN-statistics slab rows of a forward launch: one per block of a channel tile (the blocks of a
// persistent grid that walk the same channel tile), see the end of igemm_gather_kernel
int conv_igemm_slabs(const ConvGeom& g) {
  const int64_t M = static_cast<int64_t>(g.n) * g.ho * g.wo;
  const Cfg c = pick_cfg(g.cout, M);
  const int mtiles = static_cast<int>((M + c.bm - 1) / c.bm), ntiles = (g.cout + c.bn - 1) / c.bn;
  return persistent_grid(mtiles, ntiles) / ntiles;
}

// the BN-backward epilogue does not fit the registers of the 64 x 128 wave tiles (it spills):
// those layers take the 64 x 64 wave tiles of config 1 instead
static Cfg dgrad_cfg(const ConvGeom& g) {
  return pick_cfg(g.cin, static_cast<int64_t>(g.n) * g.h * g.w_in / (g.sh * g.sw));
}

void launch_slab_compact(const float* in, int rows, int width, int chunk, float* out, hipStream_t st) {
  const dim3 grid((rows + chunk - 1) / chunk, (width + 255) / 256);
  slab_compact_kernel<<<grid, 256, 0, st>>>(in, rows, width, chunk, out);
}

void launch_conv_igemm_fwd(const ConvGeom& g, hipStream_t st) {
  IgArgs k{};
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = g.part;
  k.ss = g.scale_shift;
  k.res = static_cast<const uint16_t*>(g.res);
  k.act = g.act;
  k.H = g.h; k.W = g.w_in; k.C = g.cin;
  k.Hv = g.ho; k.Wv = g.wo; k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  k.osh = 1; k.osw = 1; k.oph = 0; k.opw = 0; k.sh = g.sh; k.sw = g.sw;
  k.wrow = g.kh * g.kw * g.cin;
  k.cch = g.cin / 64;
  k.ntap = 0;
  const int64_t xb = static_cast<int64_t>(g.n) * g.h * g.w_in * g.cin * 2;
  k.xbytes = xb <= (int64_t{1} << 31) ? static_cast<uint32_t>(xb) : 0u;  // 0: flat gather
  const int64_t yb = static_cast<int64_t>(g.n) * g.ho * g.wo * g.cout * 2;
  k.ybytes = yb <= (int64_t{1} << 31) ? static_cast<uint32_t>(yb) : 0u;
  for (int i = 0; i < g.kh; ++i)
    for (int j = 0; j < g.kw; ++j) {
      k.taps[k.ntap++] = pack_tap(i * g.dh - g.ph, j * g.dw - g.pw, i * g.kw + j, i, j);
    }
  Cfg c = pick_cfg(g.cout, static_cast<int64_t>(g.n) * g.ho * g.wo);
  // the inference BN epilogue (scale/shift/residual loads) spills on the 64 x 128 wave tiles
  if (g.scale_shift != nullptr && (c.id == 3 || c.id == 4)) c = kCfgs[1];
  if (g.cfg == 5 && g.scale_shift != nullptr && g.part == nullptr) c = kCfgs[5];
  fill_common(k, c, g.n);
  launch_gather(k, c, st);
}

// split-K epilogue: y[m][c] = act(sum_kp ws[kp][m][c] * scale[c] + shift[c] (+ res[m][c])), the
// parts summed in order (deterministic); 8 channels per thread, 16-byte stores
__global__ void __launch_bounds__(256) splitk_bn_kernel(const float* __restrict__ ws, int ksplit, int64_t M, int cout,
                                                        const float* __restrict__ ss, const uint16_t* __restrict__ res,
                                                        int act, uint16_t* __restrict__ y) {
  const int cv = cout / 8;
  const int64_t total = M * cv;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t m = i / cv;
    const int c0 = static_cast<int>(i - m * cv) * 8;
    float v[8];
    const float4* p = reinterpret_cast<const float4*>(ws + m * cout + c0);
    float4 lo = p[0], hi = p[1];
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    for (int kp = 1; kp < ksplit; ++kp) {
      const float4* q = reinterpret_cast<const float4*>(ws + (static_cast<int64_t>(kp) * M + m) * cout + c0);
      lo = q[0]; hi = q[1];
      v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w; v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
    }
    float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (res != nullptr) {
      const uint4 rv = *reinterpret_cast<const uint4*>(res + m * cout + c0);
      bf16x4_unpack(make_uint2(rv.x, rv.y), r);
      bf16x4_unpack(make_uint2(rv.z, rv.w), r + 4);
    }
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const float a0 = epi_act(fmaf(v[j], ss[c0 + j], ss[cout + c0 + j]) + r[j], act);
      const float a1 = epi_act(fmaf(v[j + 1], ss[c0 + j + 1], ss[cout + c0 + j + 1]) + r[j + 1], act);
      o[j / 2] = pack2(a0, a1);
    }
    *reinterpret_cast<uint4*>(y + m * cout + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// K parts for the batch-1 split-K forward (128 x 64 tiles): enough blocks for two per CU, each
// part >= 4 K-steps, nk divisible by the part count; 1 = no split
int conv_igemm_splitk(const ConvGeom& g) {
  if (g.cout % 8 != 0 || g.cin % 64 != 0) return 1;
  const int64_t M = static_cast<int64_t>(g.n) * g.ho * g.wo;
  const int64_t tiles = cfg_tiles(kCfgs[5], M, g.cout);
  const int nk = g.kh * g.kw * (g.cin / 64);
  if (tiles >= 256) return 1;
  int best = 1;
  for (int s = 2; s <= 16; ++s)
    if (nk % s == 0 && nk / s >= 4 && tiles * best < 512) best = s;
  return best;
}

void launch_conv_igemm_fwd_splitk(const ConvGeom& g, float* ws, int ksplit, hipStream_t st) {
  IgArgs k{};
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.H = g.h; k.W = g.w_in; k.C = g.cin;
  k.Hv = g.ho; k.Wv = g.wo; k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  k.osh = 1; k.osw = 1; k.oph = 0; k.opw = 0; k.sh = g.sh; k.sw = g.sw;
  k.wrow = g.kh * g.kw * g.cin;
  k.cch = g.cin / 64;
  k.ntap = 0;
  const int64_t xb = static_cast<int64_t>(g.n) * g.h * g.w_in * g.cin * 2;
  k.xbytes = xb <= (int64_t{1} << 31) ? static_cast<uint32_t>(xb) : 0u;
  const int64_t yb = static_cast<int64_t>(g.n) * g.ho * g.wo * g.cout * 2;
  k.ybytes = yb <= (int64_t{1} << 31) ? static_cast<uint32_t>(yb) : 0u;
  for (int i = 0; i < g.kh; ++i)
    for (int j = 0; j < g.kw; ++j) k.taps[k.ntap++] = pack_tap(i * g.dh - g.ph, j * g.dw - g.pw, i * g.kw + j, i, j);
  const Cfg c = kCfgs[5];
  fill_common(k, c, g.n);
  k.ksplit = ksplit;
  k.nkp = k.nk / ksplit;
  k.mtiles *= ksplit;  // the walk's tiles: (output tile, K part) pairs
  k.ws = ws;
  launch_gather(k, c, st);
  const int64_t M = static_cast<int64_t>(g.n) * g.ho * g.wo;
  splitk_bn_kernel<<<stream_grid(M * (g.cout / 8), 256), 256, 0, st>>>(
      ws, ksplit, M, g.cout, g.scale_shift, static_cast<const uint16_t*>(g.res), g.act, static_cast<uint16_t*>(g.y));
}

// g: forward geometry; g.x = dy [N,Ho,Wo,Cout], g.w = wt [Cin][KH][KW][Cout], g.y = dx [N,H,W,Cin]
void launch_conv_igemm_dgrad(const ConvGeom& g, hipStream_t st) {
  const Cfg c = dgrad_cfg(g);
  for (int a = 0; a < g.sh; ++a)
    for (int b = 0; b < g.sw; ++b) {
      IgArgs k{};
      k.x = static_cast<const uint16_t*>(g.x);
      k.w = static_cast<const uint16_t*>(g.w);
      k.y = static_cast<uint16_t*>(g.y);
      k.bias = g.scale_shift;  // dgrad launches reuse the field as an optional bias (transposed conv)
      k.addend = static_cast<const uint16_t*>(g.res);  // ... and res as an optional addend
      k.amask = g.amask;
      k.vaddend = (a == 0 && b == 0) ? static_cast<const uint16_t*>(g.res_phase0) : nullptr;
      k.H = g.ho; k.W = g.wo; k.C = g.cout;
      k.Hv = (g.h - a + g.sh - 1) / g.sh;
      k.Wv = (g.w_in - b + g.sw - 1) / g.sw;
      if (k.Hv <= 0 || k.Wv <= 0) continue;
      k.Ho = g.h; k.Wo = g.w_in; k.cout = g.cin;
      k.osh = g.sh; k.osw = g.sw; k.oph = a; k.opw = b; k.sh = 1; k.sw = 1;
      k.wrow = g.kh * g.kw * g.cout;
      k.cch = g.cout / 64;
      k.ntap = 0;
      const int64_t xb = static_cast<int64_t>(g.n) * g.ho * g.wo * g.cout * 2;
      k.xbytes = xb <= (int64_t{1} << 31) ? static_cast<uint32_t>(xb) : 0u;  // 0: flat gather
      const int64_t yb = static_cast<int64_t>(g.n) * g.h * g.w_in * g.cin * 2;
      k.ybytes = yb <= (int64_t{1} << 31) ? static_cast<uint32_t>(yb) : 0u;
      for (int i = 0; i < g.kh; ++i) {
        const int vh = a + g.ph - i * g.dh;
        if (((vh % g.sh) + g.sh) % g.sh != 0) continue;
        for (int j = 0; j < g.kw; ++j) {
          const int vw = b + g.pw - j * g.dw;
          if (((vw % g.sw) + g.sw) % g.sw != 0) continue;
          k.taps[k.ntap++] = pack_tap(vh / g.sh, vw / g.sw, i * g.kw + j, i, j);
        }
      }
      fill_common(k, c, g.n);
      launch_gather(k, c, st);
    }
}

// Fused phases: the sh x sw output phases of a strided conv's data gradient in ONE launch.  The
// per-phase launches above each re-read all of dy for a quarter (stride 2) of dx and write dx in
// 1-pixel-wide strips; here tile t is spatial tile t / nph of phase t % nph, so the phases of one
// spatial tile run on neighbouring blocks of one XCD: dy is read from HBM about once and each dx
// line is completed in L2 before it is written back.  Phases have 1..4 taps (3 x 3, stride 2):
// shorter ones are padded with null taps (zero weights, no gather) to one K length, which costs
// MFMA work -- the autotuner weighs it against the per-phase form per shape.
bool conv_igemm_dgrad_fused_ok(const ConvGeom& g) {
  if (g.sh * g.sw <= 1 || g.sh * g.sw > kMaxPhases) return false;
  if (g.h % g.sh != 0 || g.w_in % g.sw != 0) return false;
  if (!conv_igemm_supported(g, 1)) return false;
  int maxt = 0;
  for (int a = 0; a < g.sh; ++a)
    for (int b = 0; b < g.sw; ++b) {
      int n = 0;
      for (int i = 0; i < g.kh; ++i)
        for (int j = 0; j < g.kw; ++j)
          n += (((a + g.ph - i * g.dh) % g.sh + g.sh) % g.sh == 0) && (((b + g.pw - j * g.dw) % g.sw + g.sw) % g.sw == 0);
      maxt = std::max(maxt, n);
    }
  return maxt >= 1 && maxt * g.sh * g.sw <= kMaxTaps;
}

void launch_conv_igemm_dgrad_fused(const ConvGeom& g, hipStream_t st) {
  if (!conv_igemm_dgrad_fused_ok(g)) return;
  const Cfg c = dgrad_cfg(g);
  IgArgs k{};
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.bias = g.scale_shift;
  k.addend = static_cast<const uint16_t*>(g.res);
  k.amask = g.amask;
  k.vaddend = static_cast<const uint16_t*>(g.res_phase0);  // phase 0 is (0, 0)
  k.H = g.ho; k.W = g.wo; k.C = g.cout;
  k.Hv = g.h / g.sh;
  k.Wv = g.w_in / g.sw;
  k.Ho = g.h; k.Wo = g.w_in; k.cout = g.cin;
  k.osh = g.sh; k.osw = g.sw; k.oph = 0; k.opw = 0; k.sh = 1; k.sw = 1;
  k.wrow = g.kh * g.kw * g.cout;
  k.cch = g.cout / 64;
  const int64_t xb = static_cast<int64_t>(g.n) * g.ho * g.wo * g.cout * 2;
  k.xbytes = xb <= (int64_t{1} << 31) ? static_cast<uint32_t>(xb) : 0u;
  const int64_t yb = static_cast<int64_t>(g.n) * g.h * g.w_in * g.cin * 2;
  k.ybytes = yb <= (int64_t{1} << 31) ? static_cast<uint32_t>(yb) : 0u;
  int cnt[kMaxPhases] = {};
  int tp[kMaxPhases][kMaxTaps];
  int maxt = 0;
  k.nph = g.sh * g.sw;
  for (int a = 0; a < g.sh; ++a)
    for (int b = 0; b < g.sw; ++b) {
      const int q = a * g.sw + b;
      k.phase_off[q] = a | (b << 8);
      for (int i = 0; i < g.kh; ++i) {
        const int vh = a + g.ph - i * g.dh;
        if (((vh % g.sh) + g.sh) % g.sh != 0) continue;
        for (int j = 0; j < g.kw; ++j) {
          const int vw = b + g.pw - j * g.dw;
          if (((vw % g.sw) + g.sw) % g.sw != 0) continue;
          tp[q][cnt[q]++] = pack_tap(vh / g.sh, vw / g.sw, i * g.kw + j, i, j);
        }
      }
      maxt = std::max(maxt, cnt[q]);
    }
  k.ntap = maxt;
  for (int q = 0; q < k.nph; ++q)
    for (int t = 0; t < maxt; ++t) k.taps[q * maxt + t] = t < cnt[q] ? tp[q][t] : pack_tap(0, 0, kNullTap);
  fill_common(k, c, g.n);
  launch_gather(k, c, st);
}

namespace {
// Weight-gradient tile configurations (MS x 64 output channels, NS x 64 (tap, ci) columns,
// WM x WN waves, NST stages):
//   0: 128 x 256, 2 x 4 waves (64 x 64),  3 stages, 144 KiB
//   1:  64 x 256, 1 x 8 waves (64 x 32),  3 stages, 120 KiB
//   2: 128 x 512, 2 x 4 waves (64 x 128), 2 stages, 160 KiB
//   3: 256 x 256, 2 x 4 waves (128 x 64), 2 stages, 128 KiB
//   4:  64 x 512, 1 x 8 waves (64 x 64),  2 stages, 144 KiB
//   5: 128 x 384, 2 x 4 waves (64 x 96),  2 stages, 128 KiB
// RTSEG_WGRAD_CFG=<n> forces one.
struct WgCfg {
  int id, ms, ns;
};
constexpr WgCfg kWgCfgs[] = {{0, 2, 4}, {1, 1, 4}, {2, 2, 8}, {3, 4, 4}, {4, 1, 8}, {5, 2, 6}};

struct WgPlan {
  WgCfg c;
  int ntiles, mtiles, tiles, ksteps, splits, steps_per_split;
};
WgPlan wgrad_plan(const ConvGeom& g) {
  WgPlan p{};
  const char* e = std::getenv("RTSEG_WGRAD_CFG");
  const int kp = g.kh * g.kw * g.cin;
  // measured at batch 32 (profiles/r2_conv_igemm/sweep): 256 x 256 for Cout >= 256 (up to 1.9x
  // MIOpen), 128 x 384 for 128-channel layers, 64 x 256 for 64-channel ones
  int id = g.cout % 256 == 0 ? 3 : g.cout % 128 == 0 ? 5 : 1;
  if (e != nullptr && *e != '\0') {
    const int i = std::atoi(e);
    if (i >= 0 && i < static_cast<int>(sizeof(kWgCfgs) / sizeof(kWgCfgs[0]))) id = i;
  }
  // never a channel tile wider than the layer (the kernel masks it, but it is wasted work)
  if (kWgCfgs[id].ms * 64 > g.cout) id = g.cout % 128 == 0 ? 0 : 1;
  p.c = kWgCfgs[id];
  p.mtiles = (g.cout + 64 * p.c.ms - 1) / (64 * p.c.ms);
  p.ntiles = (kp + 64 * p.c.ns - 1) / (64 * p.c.ns);
  p.tiles = p.mtiles * p.ntiles;
  const int64_t M = static_cast<int64_t>(g.n) * g.ho * g.wo;
  p.ksteps = static_cast<int>((M + 63) / 64);
  int splits = std::max(1, (256 + p.tiles / 2) / p.tiles);
  splits = std::min(splits, std::max(1, p.ksteps / 16));  // >= 16 K-steps per split
  p.steps_per_split = (p.ksteps + splits - 1) / splits;
  p.splits = (p.ksteps + p.steps_per_split - 1) / p.steps_per_split;
  return p;
}
}  // namespace

int64_t conv_igemm_wgrad_ws_elems(const ConvGeom& g) {
  const WgPlan p = wgrad_plan(g);
  const int64_t plane = static_cast<int64_t>(g.cout) * g.kh * g.kw * g.cin;
  return plane * (p.splits + (p.splits > 16 ? (p.splits + 15) / 16 : 0));
}

// g.x = x [N,H,W,Cin], g.y = dy [N,Ho,Wo,Cout] (bf16); dw fp32 [Cout][Cin][KH][KW], or
// [Cout][KH][KW][Cin] (krsc: a channels-last weight's memory order)
void launch_conv_igemm_wgrad(const ConvGeom& g, float* ws, float* dw, bool krsc, hipStream_t st) {
  const WgPlan p = wgrad_plan(g);
  WgArgs k{};
  k.x = static_cast<const uint16_t*>(g.x);
  k.dy = static_cast<const uint16_t*>(g.y);
  k.ws = ws;
  k.H = g.h; k.W = g.w_in; k.C = g.cin; k.Ho = g.ho; k.Wo = g.wo; k.cout = g.cout;
  k.sh = g.sh; k.sw = g.sw;
  k.kp = g.kh * g.kw * g.cin;
  k.M = g.n * g.ho * g.wo;
  k.ksteps = p.ksteps;
  k.steps_per_split = p.steps_per_split;
  k.ntiles = p.ntiles;
  k.tiles = p.tiles;
  k.fwo = FastDiv::make(static_cast<uint32_t>(g.wo));
  k.fho = FastDiv::make(static_cast<uint32_t>(g.ho));
  int t = 0;
  for (int i = 0; i < g.kh; ++i)
    for (int j = 0; j < g.kw; ++j, ++t) k.taps[t] = pack_tap(i * g.dh - g.ph, j * g.dw - g.pw, t);
  const int grid = p.tiles * p.splits;
  switch (p.c.id) {
    case 1: igemm_wgrad_kernel<1, 4, 1, 8, 3><<<grid, 512, 0, st>>>(k); break;
    case 2: igemm_wgrad_kernel<2, 8, 2, 4, 2><<<grid, 512, 0, st>>>(k); break;
    case 3: igemm_wgrad_kernel<4, 4, 2, 4, 2><<<grid, 512, 0, st>>>(k); break;
    case 4: igemm_wgrad_kernel<1, 8, 1, 8, 2><<<grid, 512, 0, st>>>(k); break;
    case 5: igemm_wgrad_kernel<2, 6, 2, 4, 2><<<grid, 512, 0, st>>>(k); break;
    default: igemm_wgrad_kernel<2, 4, 2, 4, 3><<<grid, 512, 0, st>>>(k); break;
  }
  launch_wgrad_slab_reduce(ws, p.splits, g.cout, g.cin, g.kh * g.kw, dw, krsc, st);
}

// ws [splits][cout][kt * cin] fp32 partial weight gradients (+ ceil(splits / 16) planes of room
// after them when splits > 16) -> dw, deterministic
void launch_wgrad_slab_reduce(float* ws, int splits, int cout, int cin, int kt, float* dw, bool krsc,
                              hipStream_t st) {
  const int64_t plane = static_cast<int64_t>(cout) * kt * cin;
  const float* src = ws;
  int rows = splits;
  if (rows > 16) {  // plane % 4 == 0: Cout % 64 == 0
    float* mid = ws + plane * splits;
    const int64_t plane4 = plane / 4;
    const dim3 g1(static_cast<unsigned>((plane4 + 255) / 256), static_cast<unsigned>((rows + 15) / 16));
    igemm_wgrad_reduce16<<<g1, 256, 0, st>>>(reinterpret_cast<const float4*>(ws), reinterpret_cast<float4*>(mid),
                                             rows, plane4);
    src = mid;
    rows = (rows + 15) / 16;
  }
  const int rg = static_cast<int>(std::min<int64_t>((plane + 255) / 256, 4096));
  if (krsc) igemm_wgrad_reduce<true><<<rg, 256, 0, st>>>(src, dw, rows, cout, cin, kt);
  else igemm_wgrad_reduce<false><<<rg, 256, 0, st>>>(src, dw, rows, cout, cin, kt);
}

}  // namespace rtseg
