// Device helpers shared by the MFMA conv kernels (conv_igemm.hip, conv_halo.hip): LDS-DMA issue,
// counted vmcnt waits, packed tap tables, bf16 packing, DPP half-wave sums and the XCD-aware
// block -> tile map.  gfx950 only.
#pragma once

#include "rtseg_common.h"

namespace rtseg {
namespace mdev {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}

// LDS-DMA from inline asm (opaque to hipcc's waitcnt pass, which would otherwise drain vmcnt(0)
// before every later ds_read): 64 lanes x 16 B land at M0 + 16 * lane.
// M0 is compiler-reserved, so the statement saves and restores it around the DMA.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_dst) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_dst);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}

// Tap table entry: dh (8-bit signed) | dw (8-bit signed) << 8 | weight tap (8-bit) << 16 |
// tap-row index ri << 24 | tap-column index ci << 28.  The taps of every conv pass form a product
// set (rows x columns, possibly filtered by a dgrad phase); ri / ci index its distinct rows /
// columns so a gathered row's per-tap validity is two bits of a per-row mask.
// int32 (not short[]) because SMEM loads are dword-only on gfx950: a 16-bit table entry read
// with a uniform index becomes a VMEM load whose s_waitcnt would also drain the DMA ring.
__host__ __device__ inline int pack_tap(int dh, int dw, int wt, int ri = 0, int ci = 0) {
  return (dh & 0xff) | ((dw & 0xff) << 8) | ((wt & 0xff) << 16) | ((ri & 0xf) << 24) | (ci << 28);
}
__device__ __forceinline__ int tap_dh(int v) { return (v << 24) >> 24; }
__device__ __forceinline__ int tap_dw(int v) { return (v << 16) >> 24; }
__device__ __forceinline__ int tap_wt(int v) { return (v >> 16) & 0xff; }
__device__ __forceinline__ int tap_ri(int v) { return (v >> 24) & 0xf; }
__device__ __forceinline__ int tap_ci(int v) { return static_cast<int>(static_cast<unsigned>(v) >> 28); }

__device__ __forceinline__ bf16x8_t as_frag(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

// 16-byte epilogue stores from 32 x 32 MFMA accumulators whose rows are channels (T21 of the
// CDNA guide): lane l < 32 holds channels 8g + 0..3 of pixel l, lane l + 32 channels 8g + 4..7 of
// the same pixel.  For the channel-group pair (g, g + 1) -- pk0 / pk1 this lane's packed bf16 x 4
// of groups g / g + 1 -- one v_permlane32_swap per dword leaves lanes < 32 holding channels
// 8g .. 8g + 7 and lanes >= 32 channels 8g + 8 .. 8g + 15: one 16-byte store per lane at channel
// 8g + 8 * (lane >= 32) (= the lane's group-g channel + 4 * (lane >= 32)) instead of two 8-byte ones.
// The inverse for loads: a 16-byte load at the same per-lane channel (8g + 8 * (lane >= 32)),
// swapped back, gives this lane's words of groups g and g + 1 (lo[0] / lo[1]) -- one 16-byte load
// instead of two 8-byte ones.  Every lane must execute it (a cross-lane exchange).
__device__ __forceinline__ void pair_unswap16(uint4 raw, uint2& g0, uint2& g1) {
  const auto rx = __builtin_amdgcn_permlane32_swap(raw.x, raw.z, false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(raw.y, raw.w, false, false);
  g0 = make_uint2(rx[0], ry[0]);
  g1 = make_uint2(rx[1], ry[1]);
}

__device__ __forceinline__ uint4 pair_swap16(uint2 pk0, uint2 pk1) {
  const auto rx = __builtin_amdgcn_permlane32_swap(pk0.x, pk1.x, false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(pk0.y, pk1.y, false, false);
  return make_uint4(rx[0], ry[0], rx[1], ry[1]);
}

__device__ __forceinline__ float epi_act(float v, int act) {
  if (act == kActReLU) return fmaxf(v, 0.f);
  if (act == kActReLU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) { return f32x2_to_bf16x2(lo, hi); }

template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xF, false));
}
// Sum over each 32-lane half of the wave; valid in lanes 16..31 and 48..63 (DPP only, no LDS):
// quad swaps, half-row and row mirrors, then row 0 -> 1 / row 2 -> 3 broadcast of lane 15.
__device__ __forceinline__ float half_wave_sum(float v) {
  v += dpp_f<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xF>(v);  // row_half_mirror
  v += dpp_f<0x140, 0xF>(v);  // row_mirror
  v += dpp_f<0x142, 0xA>(v);  // row_bcast15 into rows 1 and 3
  return v;
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// One reduce-scatter butterfly step over lane pairs that differ in lane bit `hi`: of the pair
// (a, b) a lane keeps a (hi clear) or b (hi set) and adds its partner's copy of the same entry.
template <int CTRL>
__device__ __forceinline__ float rs_step(float a, float b, bool hi) {
  return (hi ? b : a) + dpp_mov<CTRL>(hi ? a : b);
}

// Sums of the BN-statistics epilogue: ts / tq [TI][16] per lane -> per-channel sums over the 32
// pixel lanes of each half-wave, stored to one slab row (prow[co] = sum, prow[cout + co] = sum of
// squares; lane channel of entry (ti, r): co_lane + ti * 32 + 8 * (r >> 2) + (r & 3)).
// A reduce-scatter instead of 2 * TI * 16 independent 5-step all-reduces: v_permlane16_swap
// (lane bit 4), then DPP row_ror:8 / row_half_mirror / quad_perm xor 2 / xor 1 (bits 3, 2, 1, 0),
// halving the live entries at every step -- about 3 * 2 * TI * 16 VALU instead of 15 per entry.
// Lane l ends with entries 32 k + bitrev5(l & 31) of the flat list [ts..., tq...].
// Stage 1 of the reduce-scatter (lane bit 4, v_permlane16_swap): the 2 * TI * 16 entries of
// [ts..., tq...] -> TI * 16 half-reduced values.  Linear, so stage-1 outputs of several tiles may
// be summed before stage 2 (the conv kernels keep that sum in registers across their tiles).
template <int TI>
__device__ __forceinline__ void stats_stage1(const float (&ts)[TI][16], const float (&tq)[TI][16], float (&y)[TI * 16]) {
  constexpr int V = 2 * TI * 16;
  float x[V];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      x[i * 16 + r] = ts[i][r];
      x[TI * 16 + i * 16 + r] = tq[i][r];
    }
#pragma unroll
  for (int k = 0; k < V / 2; ++k) {  // lane bit 4: rows 0 <-> 1 and 2 <-> 3
    const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x[2 * k]),
                                                     __builtin_bit_cast(unsigned, x[2 * k + 1]), false, false);
    y[k] = __builtin_bit_cast(float, static_cast<unsigned>(sw[0])) + __builtin_bit_cast(float, static_cast<unsigned>(sw[1]));
  }
}

// Which entry value k (0 <= k < 2 * TI * 16 / 32) of stats_stage2 a lane ends with: sq (0 = sum,
// 1 = sum of squares) and the channel offset from co_lane (ti * 32 + 8 * (r >> 2) + (r & 3)).
template <int TI>
__device__ __forceinline__ void stats_slot(int k, int lane, int& sq, int& dc) {
  const int j = static_cast<int>(__builtin_bitreverse32(static_cast<unsigned>(lane & 31)) >> 27);
  const int e = 32 * k + j;  // flat entry: [ts (TI*16) | tq (TI*16)]
  sq = e >= TI * 16;
  const int slot = sq ? e - TI * 16 : e;
  const int r = slot & 15;
  dc = (slot >> 4) * 32 + 8 * (r >> 2) + (r & 3);
}

// Stage 2 (lane bits 3..0, DPP) and the scatter: put(k, sq, dc, value) for the lane's entries
// k = 0 .. 2 * TI * 16 / 32 - 1 (stats_slot gives sq / dc).
template <int TI, class Put>
__device__ __forceinline__ void stats_stage2(const float (&y)[TI * 16], int lane, Put put) {
  constexpr int V = 2 * TI * 16;
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  float z[V / 4];
#pragma unroll
  for (int k = 0; k < V / 4; ++k) z[k] = rs_step<0x128>(y[2 * k], y[2 * k + 1], b3);  // row_ror:8
  float u[V / 8];
#pragma unroll
  for (int k = 0; k < V / 8; ++k) u[k] = rs_step<0x141>(z[2 * k], z[2 * k + 1], b2);  // row_half_mirror
  float w[V / 16];
#pragma unroll
  for (int k = 0; k < V / 16; ++k) w[k] = rs_step<0x4E>(u[2 * k], u[2 * k + 1], b1);  // quad_perm xor 2
#pragma unroll
  for (int k = 0; k < V / 32; ++k) {
    const float v = rs_step<0xB1>(w[2 * k], w[2 * k + 1], b0);  // quad_perm xor 1
    int sq, dc;
    stats_slot<TI>(k, lane, sq, dc);
    put(k, sq, dc, v);
  }
}

template <int TI>
__device__ __forceinline__ void stats_reduce_store(const float (&ts)[TI][16], const float (&tq)[TI][16], float* prow,
                                                   int co_lane, int cout, int lane) {
  float y[TI * 16];
  stats_stage1<TI>(ts, tq, y);
  stats_stage2<TI>(y, lane, [&](int, int sq, int dc, float v) {
    const int co = co_lane + dc;
    if (co < cout) prow[(sq ? cout : 0) + co] = v;
  });
}

// Bijective block -> logical id map that gives each XCD (blockIdx % 8 under round-robin
// dispatch) a contiguous range of logical ids: neighbouring tiles share L2.  Speed only.
__device__ __forceinline__ int xcd_logical(int b, int G) {
  const int q = G / 8, r = G % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ void bf16x4_unpack(uint2 r, float* f) {
  f[0] = bf16_to_f32(static_cast<uint16_t>(r.x & 0xffff));
  f[1] = bf16_to_f32(static_cast<uint16_t>(r.x >> 16));
  f[2] = bf16_to_f32(static_cast<uint16_t>(r.y & 0xffff));
  f[3] = bf16_to_f32(static_cast<uint16_t>(r.y >> 16));
}

// A residual-gradient addend handed over with its BN's activation mask (ops/bn.py, kMaskBits:
// one bit per element, element e in bit e % 8 of byte e / 8): the 4 addend values of elements
// e .. e + 3 (e % 4 == 0) where the mask is 0 become 0 -- the masked gradient g * relu'(z) is
// never written out by the BN backward.
__device__ __forceinline__ void mask_addend4(const uint8_t* __restrict__ m, int64_t e, float* r) {
  const uint32_t b = static_cast<uint32_t>(m[e >> 3]) >> (e & 7);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (!((b >> q) & 1u)) r[q] = 0.f;
}

}  // namespace mdev
}  // namespace rtseg
