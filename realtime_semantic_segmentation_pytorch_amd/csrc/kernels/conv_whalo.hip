// Halo-tiled weight gradient of 3x3 / stride-1 / pad-1 convs (Cin, Cout multiples of 64) on bf16
// MFMA (v_mfma_f32_32x32x16_bf16) for channels-last activations, gfx950.
//
// Reference layers: the 3x3 stride-1 convs of DDRNet's RB / RBB blocks (ddrnet.py:168-219),
// ConvBNAct (models/modules.py:73-85), ResNet BasicBlocks -- their backward-filter pass, which the
// reference leaves to cuDNN.
//
// dW[co][tap][ci] = sum_p dy[p][co] * x[p + off(tap)][ci].  The split-K gather kernel
// (conv_igemm.hip igemm_wgrad_kernel) stages, per 64-pixel K-step, the dy rows and the x rows of
// one tap (every x pixel crosses L2 -> LDS nine times) and runs at 24-40 % of MFMA peak
// (profiles/r4_conv/pmc_table.txt).  Here a block owns one (64 output, 64 input) channel pair and
// ALL 9 taps (36 accumulator tiles of 32 x 32): per 8 x 32-pixel tile it stages the dy tile
// (256 rows) and the input halo (10 x 34 rows) ONCE, double-buffered a whole tile ahead, and every
// tap reads a shifted window of the halo -- one barrier per tile, no per-K-step synchronisation.
//
//  * 12 waves (3 per SIMD): wave w owns output-channel tile w & 1 and the three (tap, 32-input-
//    channel) tiles 3 (w >> 1) .. 3 (w >> 1) + 2 -- per 16-pixel K sub-step one dy^T fragment
//    and three shifted x fragments feed three MFMAs;
//  * both operands are read K-major with ds_read_b64_tr_b16 (the hardware transpose gives each
//    lane 4 consecutive pixels of one channel); rows of 128 B, chunk c of row r stored at
//    c ^ (((r >> 1) & 1) << 2): conflict-free for any 4 consecutive rows, i.e. for every tap shift;
//  * LDS-DMA through range-checked buffer resources: rows past the image read zeros, so partial
//    tiles and the zero padding need no masking (a zero dy row contributes nothing);
//  * split-K over pixel tiles: each block writes its fp32 partial [64][9][64] into a slab that
//    launch_wgrad_slab_reduce sums deterministically (conv_igemm.hip).
#include "rtseg_common.h"
#include "rtseg_launch.h"
#include "rtseg_mfma_dev.h"

#include <algorithm>

namespace rtseg {

namespace {

using namespace mdev;

constexpr int kTH = 8, kTW = 32, kTP = kTH * kTW;     // dy tile: 256 pixels
constexpr int kHH = kTH + 2, kHW = kTW + 2;           // input halo (3 x 3 footprint)
constexpr int kHRows = kHH * kHW;                     // 340
constexpr int kHInstr = (kHRows + 7) / 8;             // 43 LDS-DMA instructions of 8 rows
constexpr int kDInstr = kTP / 8;                      // 32
constexpr int kDStage = kTP * 8;                      // 16-byte chunks of the dy tile
constexpr int kHStage = kHInstr * 64;                 // ... of the halo (344 rows)
constexpr int kStage = kDStage + kHStage;
constexpr int kNW = 12;
static_assert(2 * kStage * 16 <= 160 * 1024, "LDS budget");

struct WhArgs {
  const uint16_t* x;   // [N][H][W][Cin] bf16
  const uint16_t* dy;  // [N][H][W][Cout] bf16 (stride 1, pad 1: same spatial size)
  float* ws;           // slab [splits][Cout][9 * Cin]
  int H, W, cin, cout;
  int tilesW, tilesH, mtiles;
  int cich, pairs, splits;
  uint32_t xbytes, dybytes;
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

// transposed 4 x bf16 read (lane 4q + p of its 16-lane group supplies row q, columns 4p .. 4p+3)
__device__ __forceinline__ i16x4_t tr4(const uint4* lds_base, uint32_t byte_off) {
  auto p = (__attribute__((address_space(3))) i16x4_t*)(
      (__attribute__((address_space(3))) char*)((__attribute__((address_space(3))) void*)lds_base) + byte_off);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
}

__device__ __forceinline__ uint32_t swz_off(int row, int col) {  // byte offset of (row, col 4-aligned)
  const int ch = (col >> 3) ^ (((row >> 1) & 1) << 2);
  return static_cast<uint32_t>(row * 128 + ch * 16 + ((col >> 2) & 1) * 8);
}

// KS = 1: wave w owns output tile w & 1 and three (tap, input half) tiles, all 16 K sub-steps of a
//         pixel tile (round 4): 4 fragment reads (1 dy^T + 3 x) per 3 MFMAs.
// KS = 2: wave w owns BOTH output tiles and three (tap, input half) tiles, for half of the K
//         sub-steps (pixel rows 0-3 or 4-7 of the tile): 5 fragment reads per 6 MFMAs -- 37.5 %
//         fewer LDS transposed reads per MFMA (the K loop was LDS-read bound: 48 KiB of
//         ds_read_tr per CU per sub-step against 36 MFMAs); the two K halves are summed through
//         LDS once, after the last tile.
template <int KS>
__global__ void __launch_bounds__(kNW * 64) whalo_wgrad_kernel(const WhArgs a) {
  __shared__ uint4 lds[2 * kStage];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lb = xcd_logical(blockIdx.x, gridDim.x);
  const int pair = lb % a.pairs, split = lb / a.pairs;
  const int co0 = (pair / a.cich) * 64, ci0 = (pair % a.cich) * 64;
  const int lr8 = lane >> 3, lch = lane & 7;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, static_cast<int>(a.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t dr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.dy), 0, static_cast<int>(a.dybytes), 0x00020000);

  // ---- one tile's dy rows + input halo into buffer b (75 DMA instructions over the 12 waves)
  auto stage = [&](int mt, int b) {
    const int tx = mt % a.tilesW;
    const int t2 = mt / a.tilesW;
    const int n = t2 / a.tilesH;
    const int oy0 = (t2 % a.tilesH) * kTH, ox0 = tx * kTW;
    const uint32_t base = lds_addr(lds + b * kStage);
    for (int e = wid; e < kDInstr + kHInstr; e += kNW) {
      if (e < kDInstr) {
        const int r = e * 8 + lr8;
        const int oy = oy0 + (r >> 5), ox = ox0 + (r & 31);
        const int lc = lch ^ (((r >> 1) & 1) << 2);
        const bool ok = oy < a.H && ox < a.W;
        const uint32_t v = ok ? static_cast<uint32_t>(((n * a.H + oy) * a.W + ox) * a.cout + co0 + lc * 8) * 2u
                              : 0x80000000u;
        bdma16(dr, v, base + e * 1024);
      } else {
        const int h = e - kDInstr;
        const int r = h * 8 + lr8;
        const int hy = r / kHW, hx = r - hy * kHW;
        const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
        const int lc = lch ^ (((r >> 1) & 1) << 2);
        const bool ok = r < kHRows && static_cast<unsigned>(iy) < static_cast<unsigned>(a.H) &&
                        static_cast<unsigned>(ix) < static_cast<unsigned>(a.W);
        const uint32_t v = ok ? static_cast<uint32_t>(((n * a.H + iy) * a.W + ix) * a.cin + ci0 + lc * 8) * 2u
                              : 0x80000000u;
        bdma16(xr, v, base + kDStage * 16 + h * 1024);
      }
    }
  };

  // ---- wave tiles: output-channel tile(s) m (32 rows), three (tap, input-channel half) tiles
  constexpr int NM = KS == 2 ? 2 : 1;           // output tiles per wave
  const int m0 = KS == 2 ? 0 : (wid & 1);
  const int nb = KS == 2 ? 3 * (wid % 6) : 3 * (wid >> 1);
  const int kh = KS == 2 ? wid / 6 : 0;         // K half (KS = 2)
  int tap_i[3], tap_j[3], cit[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int nn = nb + u, tap = nn >> 1;
    tap_i[u] = tap / 3;
    tap_j[u] = tap - 3 * (tap / 3);
    cit[u] = nn & 1;
  }
  // transposed-read geometry: row q of the 4-row block, columns 4p.., 16-column group g16, K half hh
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = (lane >> 4) & 1, hh = lane >> 5;
  int bcol[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) bcol[u] = cit[u] * 32 + g16 * 16 + p4;

  f32x16_t acc[NM][3];
#pragma unroll
  for (int mm = 0; mm < NM; ++mm)
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mm][u][r] = 0.f;

  // Per-lane LDS byte offsets, so that every fragment read of the fully unrolled K loop is
  // base + compile-time immediate (round-4 PMC: 9.4 VALU per MFMA with per-read address math):
  //  * dy^T: rows kk * 16 + hh * 8 + q (+ 4): adding 16 or 4 rows keeps the swizzle bit
  //    ((row >> 1) & 1), so one base + (kk * 16 [+ 4]) * 128;
  //  * halo: rows (py + i) * 34 + px0 + hh * 8 + q + j: adding px0 (0 / 16) or 4 keeps the bit,
  //    adding 34 flips it -- one base for even and one for odd py, each + (py * 34 + px0) * 128
  uint32_t offA[NM];
#pragma unroll
  for (int mm = 0; mm < NM; ++mm) offA[mm] = swz_off(hh * 8 + q, (m0 + mm) * 32 + g16 * 16 + p4);  // dy^T column
  uint32_t offB[2][3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int r0 = tap_i[u] * kHW + hh * 8 + q + tap_j[u];
    offB[0][u] = swz_off(r0, bcol[u]) + kDStage * 16;
    offB[1][u] = swz_off(r0 + kHW, bcol[u]) - kHW * 128 + kDStage * 16;
  }

  const int my_tiles = split < a.mtiles ? (a.mtiles - split + a.splits - 1) / a.splits : 0;
  if (my_tiles > 0) stage(split, 0);
  for (int t = 0; t < my_tiles; ++t) {
    vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t landed for every wave; the other buffer is free
    if (t + 1 < my_tiles) stage(split + (t + 1) * a.splits, (t + 1) & 1);
    const uint4* dbase = lds + (t & 1) * kStage;
    constexpr int KSTEPS = kTP / 16 / KS;
#pragma unroll
    for (int k2 = 0; k2 < KSTEPS; ++k2) {
      const int kk = KS == 2 ? kh * KSTEPS + k2 : k2;  // (kh is wave-uniform: immediates per wave half)
      // KSTEPS is even: the parity of the pixel row py is a compile-time function of k2
      const int py = kk >> 1, px0 = (k2 & 1) * 16, par = (k2 >> 1) & 1;
      // dy^T fragment(s): rows = pixels kk*16 + hh*8 + q (+4), column of output tile m0 + mm
      bf16x8_t af[NM];
#pragma unroll
      for (int mm = 0; mm < NM; ++mm) {
        const i16x4_t alo = tr4(dbase, offA[mm] + kk * 16 * 128);
        const i16x4_t ahi = tr4(dbase, offA[mm] + (kk * 16 + 4) * 128);
        af[mm] = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, alo), __builtin_bit_cast(bf16x4_t, ahi), 0, 1,
                                         2, 3, 4, 5, 6, 7);
      }
      bf16x8_t bf[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const uint32_t o = offB[par][u] + (py * kHW + px0) * 128;
        const i16x4_t blo = tr4(dbase, o);
        const i16x4_t bhi = tr4(dbase, o + 4 * 128);
        bf[u] = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, blo), __builtin_bit_cast(bf16x4_t, bhi), 0, 1,
                                        2, 3, 4, 5, 6, 7);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mm = 0; mm < NM; ++mm)
#pragma unroll
        for (int u = 0; u < 3; ++u)
          acc[mm][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mm], bf[u], acc[mm][u], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  if constexpr (KS == 2) {
    // sum the two K halves: waves 6..11 park their accumulators in the (now idle) stage buffers
    float* red = reinterpret_cast<float*>(lds);  // [6 wave groups][NM * 3 * 16][64 lanes]
    const int wg = wid % 6;
    __syncthreads();
    if (kh == 1) {
#pragma unroll
      for (int mm = 0; mm < NM; ++mm)
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[((wg * NM + mm) * 3 + u) * 16 * 64 + r * 64 + lane] = acc[mm][u][r];
    }
    __syncthreads();
    if (kh == 1) return;
#pragma unroll
    for (int mm = 0; mm < NM; ++mm)
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mm][u][r] += red[((wg * NM + mm) * 3 + u) * 16 * 64 + r * 64 + lane];
  }

  // fp32 partial tile -> slab [split][cout][tap * cin + ci] (every element written by one block)
  const int64_t kp = 9 * static_cast<int64_t>(a.cin);
  float* slab = a.ws + static_cast<int64_t>(split) * a.cout * kp;
#pragma unroll
  for (int mm = 0; mm < NM; ++mm)
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int tap = (nb + u) >> 1;
      const int64_t col = tap * static_cast<int64_t>(a.cin) + ci0 + cit[u] * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + (m0 + mm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        slab[co * kp + col] = acc[mm][u][r];
      }
    }
}

bool whalo_fill(WhArgs& k, const ConvGeom& g) {
  if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1 || g.ph != 1 || g.pw != 1)
    return false;
  if (g.cin % 64 != 0 || g.cout % 64 != 0 || g.ho != g.h || g.wo != g.w_in) return false;
  const int64_t xb = static_cast<int64_t>(g.n) * g.h * g.w_in * g.cin * 2;
  const int64_t db = static_cast<int64_t>(g.n) * g.h * g.w_in * g.cout * 2;
  if (xb >= (int64_t{1} << 31) || db >= (int64_t{1} << 31)) return false;
  k.H = g.h; k.W = g.w_in; k.cin = g.cin; k.cout = g.cout;
  k.xbytes = static_cast<uint32_t>(xb);
  k.dybytes = static_cast<uint32_t>(db);
  k.tilesW = (g.w_in + kTW - 1) / kTW;
  k.tilesH = (g.h + kTH - 1) / kTH;
  k.mtiles = g.n * k.tilesW * k.tilesH;
  k.cich = g.cin / 64;
  k.pairs = k.cich * (g.cout / 64);
  // about one block per CU (LDS-bound), at least one pixel tile per block
  k.splits = std::max(1, std::min(256 / k.pairs, k.mtiles));
  return true;
}

}  // namespace

bool conv_whalo_supported(const ConvGeom& g) {
  WhArgs k{};
  return whalo_fill(k, g);
}

int64_t conv_whalo_ws_elems(const ConvGeom& g) {
  WhArgs k{};
  if (!whalo_fill(k, g)) return 0;
  const int64_t plane = static_cast<int64_t>(g.cout) * 9 * g.cin;
  return plane * (k.splits + (k.splits > 16 ? (k.splits + 15) / 16 : 0));
}

void launch_conv_whalo_wgrad(const ConvGeom& g, float* ws, float* dw, bool krsc, hipStream_t st, int variant) {
  WhArgs k{};
  if (!whalo_fill(k, g)) return;
  k.x = static_cast<const uint16_t*>(g.x);
  k.dy = static_cast<const uint16_t*>(g.y);
  k.ws = ws;
  if (variant == 2) whalo_wgrad_kernel<2><<<k.pairs * k.splits, kNW * 64, 0, st>>>(k);
  else whalo_wgrad_kernel<1><<<k.pairs * k.splits, kNW * 64, 0, st>>>(k);
  launch_wgrad_slab_reduce(ws, k.splits, g.cout, g.cin, 9, dw, krsc, st);
}

}  // namespace rtseg
