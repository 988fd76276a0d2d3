// Implicit-GEMM 2-D convolution on bf16 MFMA for channels-last activations (gfx950).
//
// Reference sites: every dense conv of the zoo -- ConvBNAct (models/modules.py:73-85),
// DDRNet's RB/RBB residual blocks (ddrnet.py:168-219), SegHead 3x3 (modules.py:161-166)
// -- which the reference runs through cuDNN followed by a separate BatchNorm pass.
//
// GEMM view: M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin (tap-major, then
// channel).  A[m, k] = x[n, ho*s - p + i*d, wo*s - p + j*d, c] (zero outside the
// image), B[k, co] = w[co, i, j, c] (weights pre-laid-out [Cout][KH][KW][Cin]).
//
//  * block tile BM (pixels: 128; 256 selectable, see conv_bm) x BN (Cout: 128, or 64
//    for narrow layers) x BK (K: 64 when Cin % 64 == 0, else 32); BM/64 x 2 waves (4 or 8),
//    each wave a 64 x BN/2 sub-tile of v_mfma_f32_16x16x32_bf16 (BK/32 MFMA K-steps per
//    stage).  The 256-row tile halves the B-operand DMA per MFMA and runs 8 waves (two per
//    SIMD) in one block, so a CU's waves share one 144 KiB 3-stage ring;
//  * a K-step is one tap and BK consecutive input channels, so every A row is one
//    contiguous 64/128-byte read;
//  * operands go global -> LDS by DMA (global_load_lds_dwordx4, no staging registers)
//    into a 3-stage ring: steps k+1 and k+2 are in flight while step k's MFMAs run; one
//    counted vmcnt + raw barrier per K-step; padding taps DMA from a 16-byte zero page;
//  * LDS holds each 32-wide K sub-tile as rows of 64 B (four 16-byte chunks); chunk q of row r at
//    q ^ h[(r >> 2) & 3], h = {0, 2, 3, 1}, which makes the ds_read_b128 fragment
//    reads of the 16x16x32 layout conflict-free (each 16-lane LDS group hits 16
//    distinct 16-byte slots of the 256-byte bank window);
//  * epilogue: the output tile is staged through LDS and written with coalesced
//    16-byte stores; optionally
//      STATS -- per-channel (sum, sum of squares) of the bf16 outputs, accumulated
//               over the M tiles a block visits and written as one row of a [G, 2C]
//               slab that the fused BatchNorm finalize consumes (the separate BN
//               statistics pass over the conv output disappears);
//      EPI=1 -- inference BatchNorm (scale/shift) + optional residual + activation,
//               i.e. the whole ConvBNAct / RB tail in one kernel.
#include "rtseg_common.h"
#include "rtseg_launch.h"

#include <cstdlib>
#include <type_traits>

namespace rtseg {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kMaxSlabs = 512;                  // G of the BN statistics slab

struct ConvK {
  const uint16_t* x;
  const uint16_t* w;
  uint16_t* y;
  float* part;
  const float* ss;
  const uint16_t* res;
  int act;
  int ih, iw, cin, ho, wo, cout, kh, kw, sh, sw, ph, pw, dh, dw;
  int m, mtiles;
  FastDiv fwo, fho;
};

__device__ __forceinline__ int swz(int r, int q) {
  return r * 4 + (q ^ ((0x1320 >> (((r >> 2) & 3) * 4)) & 0xF));
}

__device__ __forceinline__ bf16x8_t as_frag(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

// 16 zero bytes in global memory: the DMA source of padding taps / rows past the edge.
__device__ uint4 g_zero16[1];

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 16, "vmcnt immediate");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // other counts: drain (correct, slower)
}

// LDS-DMA issued from inline asm: hipcc's waitcnt pass cannot tell which LDS bytes a
// __builtin_amdgcn_global_load_lds writes, so it drains vmcnt(0) before every later ds_read
// (it did, in this kernel) -- which serialises the ring.  Opaque to the compiler, the DMA is
// ordered by the kernel's own counted vmcnt + barrier instead.  M0 = LDS byte address of the
// wave's 1 KiB destination (wave-uniform); one wait state between the M0 write and its use.
__device__ __forceinline__ void glds16(const void* src, uint4* lds_dst) {
  const uint32_t lds_addr = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)lds_dst)));
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(src), "s"(lds_addr)
      : "memory", "m0");
}

__device__ __forceinline__ uint4 mask4(uint4 v, bool ok) {
  const unsigned m = ok ? 0xffffffffu : 0u;
  v.x &= m; v.y &= m; v.z &= m; v.w &= m;
  return v;
}

__device__ __forceinline__ float epi_act(float v, int act) {
  if (act == kActReLU) return fmaxf(v, 0.f);
  if (act == kActReLU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

template <int EPI, bool STATS, int BM, int BN, int BK>
__global__ void __launch_bounds__(BM * 2, 256 / BM) conv_mfma_kernel(ConvK a) {
  constexpr int kCBM = BM;
  constexpr int WAVES = BM / 32;               // (BM / 64) x 2 waves
  constexpr int QR = BK / 8;                   // 16-byte chunks per tile row
  constexpr int A_SUB = kCBM * 4;               // chunks of one 32-wide K sub-tile of A
  constexpr int B_SUB = BN * 4;
  constexpr int STAGE = (kCBM + BN) * QR;       // chunks per pipeline stage
  constexpr int WNT = BN / 32;                  // 16-wide N tiles per wave (waves are 2 wide in N)
  // pipeline stages: 3 keeps two K-steps of DMA in flight across each barrier; the 128 x 128 x 64
  // tile (32 KiB per stage) uses 2 so that two blocks still fit a CU's LDS (the 256-row tile
  // runs one block per CU: 3 x 48 KiB)
  constexpr int NST = (BM == 128 && BN == 128 && BK == 64) ? 2 : 3;
  constexpr int EPI_CHUNKS = WAVES * 64 * (BN / 2) / 8;  // bf16 epilogue staging, 16-byte chunks
  __shared__ uint4 lds[NST * STAGE > EPI_CHUNKS ? NST * STAGE : EPI_CHUNKS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.y * BN;
  const int cch = a.cin / BK;  // K-steps per tap
  const int nk = a.kh * a.kw * cch;
  // LDS-DMA staging: one global_load_lds_dwordx4 moves 64 lanes x 16 B = 16 rows of one 32-wide
  // K sub-tile into 1 KiB of LDS at (wave-uniform base + 16 B * lane).  The bank swizzle is
  // applied on the SOURCE side: lane L fills physical chunk L & 3 of row L >> 2, i.e. it loads
  // logical K chunk (L & 3) ^ h[(L >> 4) & 3] of that row (h = {0, 2, 3, 1}, see swz()).
  constexpr int A_INST = (BK / 32) * (kCBM / 16), B_INST = (BK / 32) * (BN / 16);
  constexpr int A_IW = A_INST / WAVES, B_IW = B_INST / WAVES;  // DMA instructions per wave per stage
  static_assert(A_IW >= 1 && B_IW >= 1 && A_IW * WAVES == A_INST && B_IW * WAVES == B_INST,
                "tile/wave mismatch");
  const int lrow = lane >> 2;
  const int lkc = (lane & 3) ^ ((0x1320 >> (((lane >> 4) & 3) * 4)) & 0xF);
  const int64_t wstride = static_cast<int64_t>(a.kh) * a.kw * a.cin;

  const uint16_t* wrow[B_IW];
  bool wok[B_IW];
#pragma unroll
  for (int e = 0; e < B_IW; ++e) {
    const int I = wid * B_IW + e;
    const int h = I / (BN / 16), rg = I % (BN / 16);
    const int co = n0 + 16 * rg + lrow;
    wok[e] = co < a.cout;
    wrow[e] = a.w + static_cast<int64_t>(min(co, a.cout - 1)) * wstride + (4 * h + lkc) * 8;
  }
  float csum[WNT], csq[WNT];
#pragma unroll
  for (int ni = 0; ni < WNT; ++ni) { csum[ni] = 0.f; csq[ni] = 0.f; }

  for (int mt = blockIdx.x; mt < a.mtiles; mt += gridDim.x) {
    const int m0 = mt * kCBM;
    const uint16_t* xbase[A_IW];
    int hb[A_IW], wb[A_IW];
    bool rok[A_IW];
#pragma unroll
    for (int e = 0; e < A_IW; ++e) {
      const int I = wid * A_IW + e;
      const int h = I / (kCBM / 16), rg = I % (kCBM / 16);
      const int m = m0 + 16 * rg + lrow;
      rok[e] = m < a.m;
      uint32_t wo_, ho_;
      const uint32_t t = a.fwo.divmod(static_cast<uint32_t>(rok[e] ? m : a.m - 1), wo_);
      const uint32_t n_ = a.fho.divmod(t, ho_);
      hb[e] = static_cast<int>(ho_) * a.sh - a.ph;
      wb[e] = static_cast<int>(wo_) * a.sw - a.pw;
      xbase[e] = a.x + static_cast<int64_t>(n_) * a.ih * a.iw * a.cin + (4 * h + lkc) * 8;
    }
    f32x4_t acc[4][WNT];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // issue the DMA of K-step kk into stage buffer `buf` (padding taps read the zero page)
    auto stage = [&](int kk, int buf) {
      const int tap = kk / cch;
      const int c0 = (kk - tap * cch) * BK;
      const int i = tap / a.kw, j = tap - (tap / a.kw) * a.kw;
      uint4* A = lds + buf * STAGE;
      uint4* B = A + kCBM * QR;
#pragma unroll
      for (int e = 0; e < A_IW; ++e) {
        const int I = wid * A_IW + e;
        const int hi = hb[e] + i * a.dh, wi = wb[e] + j * a.dw;
        const bool ok = rok[e] && hi >= 0 && hi < a.ih && wi >= 0 && wi < a.iw;
        const uint16_t* src = xbase[e] + (static_cast<int64_t>(hi) * a.iw + wi) * a.cin + c0;
        glds16(ok ? static_cast<const void*>(src) : static_cast<const void*>(g_zero16),
               A + (I / (kCBM / 16)) * A_SUB + (I % (kCBM / 16)) * 64);
      }
#pragma unroll
      for (int e = 0; e < B_IW; ++e) {
        const int I = wid * B_IW + e;
        const uint16_t* src = wrow[e] + tap * a.cin + c0;
        glds16(wok[e] ? static_cast<const void*>(src) : static_cast<const void*>(g_zero16),
               B + (I / (BN / 16)) * B_SUB + (I % (BN / 16)) * 64);
      }
    };

    // NST-stage ring: DMA of K-steps kk+1 .. kk+NST-1 is in flight while kk computes.  Step kk's
    // data is published by a COUNTED vmcnt (this wave's DMAs of the younger step may stay
    // outstanding) + a raw s_barrier -- __syncthreads() would drain every DMA (vmcnt(0)).
    constexpr int PER = A_IW + B_IW;  // DMA instructions per wave per stage
#pragma unroll
    for (int p = 0; p < NST - 1; ++p)
      if (p < nk) stage(p, p);
    for (int kk = 0; kk < nk; ++kk) {
      if (NST == 3 && kk + 1 < nk) wait_vmcnt<(NST - 2) * PER>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // all waves: step kk landed, step kk-1's buffer is free
      if (kk + NST - 1 < nk) stage(kk + NST - 1, (kk + NST - 1) % NST);
      const uint4* A = lds + (kk % NST) * STAGE;
      const uint4* B = A + kCBM * QR;
#pragma unroll
      for (int hs = 0; hs < BK / 32; ++hs) {
        bf16x8_t fa[4], fb[WNT];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          fa[mi] = as_frag(A[hs * A_SUB + swz(wm * 64 + mi * 16 + (lane & 15), lane >> 4)]);
#pragma unroll
        for (int ni = 0; ni < WNT; ++ni)
          fb[ni] = as_frag(B[hs * B_SUB + swz(wn * (BN / 2) + ni * 16 + (lane & 15), lane >> 4)]);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < WNT; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    __syncthreads();  // every wave's last MFMA operands are read before the LDS is reused

    // ---- epilogue: stage this wave's 64 x (BN/2) tile as bf16 rows, then 16-byte stores
    constexpr int WC = BN / 2;  // columns per wave
    uint16_t* stg = reinterpret_cast<uint16_t*>(lds) + wid * 64 * WC;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) {
        const int c = ni * 16 + (lane & 15);
        const int co = n0 + wn * WC + c;
        const int coc = min(co, a.cout - 1);
        float sc = 1.f, sh = 0.f;
        if constexpr (EPI == 1) { sc = a.ss[coc]; sh = a.ss[a.cout + coc]; }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = mi * 16 + (lane >> 4) * 4 + i;
          const int m = m0 + wm * 64 + r;
          float v = acc[mi][ni][i];
          if constexpr (EPI == 1) {
            v = fmaf(v, sc, sh);
            if (a.res) v += bf16_to_f32(a.res[static_cast<int64_t>(min(m, a.m - 1)) * a.cout + coc]);
            v = epi_act(v, a.act);
          }
          const uint16_t hv = f32_to_bf16(v);
          if constexpr (STATS) {
            const float q = (m < a.m && co < a.cout) ? bf16_to_f32(hv) : 0.f;
            csum[ni] += q;
            csq[ni] += q * q;
          }
          stg[r * WC + c] = hv;
        }
      }
    }
    __syncthreads();
    constexpr int RC = WC / 8;  // 16-byte chunks per staged row
#pragma unroll
    for (int t = 0; t < 64 * RC / 64; ++t) {
      const int idx = lane + 64 * t;
      const int r = idx / RC, q = idx % RC;
      const int m = m0 + wm * 64 + r, co = n0 + wn * WC + q * 8;
      const uint4 v = reinterpret_cast<const uint4*>(stg)[r * RC + q];
      if (m < a.m && co < a.cout) *reinterpret_cast<uint4*>(a.y + static_cast<int64_t>(m) * a.cout + co) = v;
    }
    __syncthreads();  // the next tile's staging overwrites the LDS
  }

  if constexpr (STATS) {
#pragma unroll
    for (int ni = 0; ni < WNT; ++ni) {
      csum[ni] += __shfl_xor(csum[ni], 16, kWave);
      csum[ni] += __shfl_xor(csum[ni], 32, kWave);
      csq[ni] += __shfl_xor(csq[ni], 16, kWave);
      csq[ni] += __shfl_xor(csq[ni], 32, kWave);
    }
    float* red = reinterpret_cast<float*>(lds);  // [BM/64 M-waves][BN][2]
    if (lane < 16) {
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) {
        const int col = wn * (BN / 2) + ni * 16 + lane;
        red[(wm * BN + col) * 2] = csum[ni];
        red[(wm * BN + col) * 2 + 1] = csq[ni];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
      float* prow = a.part + static_cast<int64_t>(blockIdx.x) * 2 * a.cout;
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) {
        const int col = wn * (BN / 2) + ni * 16 + lane;
        const int co = n0 + col;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int w = 0; w < kCBM / 64; ++w) {
          s1 += red[(w * BN + col) * 2];
          s2 += red[(w * BN + col) * 2 + 1];
        }
        if (co < a.cout) {
          prow[co] = s1;
          prow[a.cout + co] = s2;
        }
      }
    }
  }
}

}  // namespace

// Pixel-tile height.  128 (two blocks per CU) by default: measured on the DDRNet-23 shapes at
// batch 32 the 256-row / 8-wave tile is 0-5 % slower on 3x3 layers and up to 25 % slower on
// 1x1 ones -- both waves of a SIMD then belong to one block and stall on the same per-K-step
// barrier, which two independent blocks hide (profiles/r1_conv_mfma).  RTSEG_CONV_BM=256
// selects it for wide (Cout > 64, Cin % 64 == 0) layers, for A/B work on the schedule.
static int conv_bm(const ConvGeom& g) {
  const char* e = std::getenv("RTSEG_CONV_BM");
  const bool can = g.cout > 64 && g.cin % 64 == 0;
  return (can && e != nullptr && std::atoi(e) == 256) ? 256 : 128;
}

int conv_mfma_slabs(const ConvGeom& g) {
  const int64_t m = static_cast<int64_t>(g.n) * g.ho * g.wo;
  const int bm = conv_bm(g);
  const int64_t mtiles = (m + bm - 1) / bm;
  return static_cast<int>(mtiles < kMaxSlabs ? mtiles : kMaxSlabs);
}

void launch_conv_mfma(const ConvGeom& g, hipStream_t st) {
  ConvK k;
  k.x = static_cast<const uint16_t*>(g.x);
  k.w = static_cast<const uint16_t*>(g.w);
  k.y = static_cast<uint16_t*>(g.y);
  k.part = g.part;
  k.ss = g.scale_shift;
  k.res = static_cast<const uint16_t*>(g.res);
  k.act = g.act;
  k.ih = g.h; k.iw = g.w_in; k.cin = g.cin; k.ho = g.ho; k.wo = g.wo; k.cout = g.cout;
  k.kh = g.kh; k.kw = g.kw; k.sh = g.sh; k.sw = g.sw; k.ph = g.ph; k.pw = g.pw; k.dh = g.dh; k.dw = g.dw;
  k.m = g.n * g.ho * g.wo;
  const int bm = conv_bm(g);
  k.mtiles = (k.m + bm - 1) / bm;
  k.fwo = FastDiv::make(g.wo);
  k.fho = FastDiv::make(g.ho);
  const bool stats = g.part != nullptr;
  const bool bn64 = g.cout <= 64;  // narrow layers: a 128-wide N tile would be half padding
  const bool bk64 = g.cin % 64 == 0;
  const int bn = bn64 ? 64 : 128;
  dim3 grid(conv_mfma_slabs(g), (g.cout + bn - 1) / bn);
  auto go = [&](auto bmc, auto bnc, auto bkc) {
    constexpr int BM = decltype(bmc)::value, BN = decltype(bnc)::value, BK = decltype(bkc)::value;
    if (g.scale_shift != nullptr) conv_mfma_kernel<1, false, BM, BN, BK><<<grid, BM * 2, 0, st>>>(k);
    else if (stats) conv_mfma_kernel<0, true, BM, BN, BK><<<grid, BM * 2, 0, st>>>(k);
    else conv_mfma_kernel<0, false, BM, BN, BK><<<grid, BM * 2, 0, st>>>(k);
  };
  using I64 = std::integral_constant<int, 64>;
  using I128 = std::integral_constant<int, 128>;
  using I256 = std::integral_constant<int, 256>;
  using I32 = std::integral_constant<int, 32>;
  if (bm == 256) {
    go(I256{}, I128{}, I64{});
  } else if (bn64) {
    if (bk64) go(I128{}, I64{}, I64{});
    else go(I128{}, I64{}, I32{});
  } else {
    if (bk64) go(I128{}, I128{}, I64{});
    else go(I128{}, I128{}, I32{});
  }
}

}  // namespace rtseg
