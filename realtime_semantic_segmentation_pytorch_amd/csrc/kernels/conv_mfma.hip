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
//  * block tile 128 (pixels) x BN (Cout: 128, or 64 for narrow layers) x BK (K: 64 when
//    Cin % 64 == 0, else 32); 256 threads = 4 waves in 2x2, each wave a 64 x BN/2
//    sub-tile of v_mfma_f32_16x16x32_bf16 (BK/32 MFMA K-steps per stage);
//  * a K-step is one tap and BK consecutive input channels, so every A row is one
//    contiguous 64/128-byte read (padding taps: the load is still issued from a clamped
//    address and the VALUE is masked to zero -- no branch around the load);
//  * register-staged double-buffered LDS: the global loads of step k+1 are in flight
//    while step k's MFMAs run; one barrier per K-step;
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

#include <type_traits>

namespace rtseg {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kCBM = 128;  // pixels per block tile (N tile: 64 or 128, K step: 32 or 64)
constexpr int kCThreads = 256;
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

template <int EPI, bool STATS, int BN, int BK>
__global__ void __launch_bounds__(kCThreads, 2) conv_mfma_kernel(ConvK a) {
  constexpr int QR = BK / 8;                   // 16-byte chunks per tile row
  constexpr int A_PER = kCBM * QR / kCThreads;  // A chunks staged per thread per K-step
  constexpr int B_PER = BN * QR / kCThreads;    // B chunks staged per thread per K-step
  constexpr int A_SUB = kCBM * 4;               // chunks of one 32-wide K sub-tile of A
  constexpr int B_SUB = BN * 4;
  constexpr int STAGE = (kCBM + BN) * QR;       // chunks per pipeline stage
  constexpr int WNT = BN / 32;                  // 16-wide N tiles per wave (2x2 waves)
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small for 256 threads");
  __shared__ uint4 lds[2 * STAGE > 2048 ? 2 * STAGE : 2048];  // 2 stages; >= 32 KiB for the epilogue
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.y * BN;
  const int cch = a.cin / BK;  // K-steps per tap
  const int nk = a.kh * a.kw * cch;
  const int lq = tid % QR;     // this thread's 16-byte chunk within a row
  const int lr = tid / QR;     // first row; rows lr + e * (256 / QR)
  constexpr int RSTEP = kCThreads / QR;
  const int64_t wstride = static_cast<int64_t>(a.kh) * a.kw * a.cin;

  const uint16_t* wrow[B_PER];
  bool wok[B_PER];
#pragma unroll
  for (int e = 0; e < B_PER; ++e) {
    const int co = n0 + lr + RSTEP * e;
    wok[e] = co < a.cout;
    wrow[e] = a.w + static_cast<int64_t>(min(co, a.cout - 1)) * wstride + lq * 8;
  }
  float csum[WNT], csq[WNT];
#pragma unroll
  for (int ni = 0; ni < WNT; ++ni) { csum[ni] = 0.f; csq[ni] = 0.f; }

  for (int mt = blockIdx.x; mt < a.mtiles; mt += gridDim.x) {
    const int m0 = mt * kCBM;
    const uint16_t* xbase[A_PER];
    int hb[A_PER], wb[A_PER];
    bool rok[A_PER];
#pragma unroll
    for (int e = 0; e < A_PER; ++e) {
      const int m = m0 + lr + RSTEP * e;
      rok[e] = m < a.m;
      uint32_t wo_, ho_;
      const uint32_t t = a.fwo.divmod(static_cast<uint32_t>(rok[e] ? m : a.m - 1), wo_);
      const uint32_t n_ = a.fho.divmod(t, ho_);
      hb[e] = static_cast<int>(ho_) * a.sh - a.ph;
      wb[e] = static_cast<int>(wo_) * a.sw - a.pw;
      xbase[e] = a.x + static_cast<int64_t>(n_) * a.ih * a.iw * a.cin + lq * 8;
    }
    f32x4_t acc[4][WNT];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    uint4 ra[A_PER], rb[B_PER];
    auto gload = [&](int kk) {
      const int tap = kk / cch;
      const int c0 = (kk - tap * cch) * BK;
      const int i = tap / a.kw, j = tap - (tap / a.kw) * a.kw;
#pragma unroll
      for (int e = 0; e < A_PER; ++e) {
        const int hi = hb[e] + i * a.dh, wi = wb[e] + j * a.dw;
        const bool ok = rok[e] && hi >= 0 && hi < a.ih && wi >= 0 && wi < a.iw;
        const int hc = min(max(hi, 0), a.ih - 1), wc = min(max(wi, 0), a.iw - 1);
        const uint4 v = *reinterpret_cast<const uint4*>(xbase[e] + (static_cast<int64_t>(hc) * a.iw + wc) * a.cin + c0);
        ra[e] = mask4(v, ok);
      }
#pragma unroll
      for (int e = 0; e < B_PER; ++e) {
        const uint4 v = *reinterpret_cast<const uint4*>(wrow[e] + tap * a.cin + c0);
        rb[e] = mask4(v, wok[e]);
      }
    };
    // chunk lq of a row: K sub-tile lq / 4, chunk lq % 4 inside it
    auto sstore = [&](int buf) {
      uint4* A = lds + buf * STAGE;
      uint4* B = A + kCBM * QR;
#pragma unroll
      for (int e = 0; e < A_PER; ++e) A[(lq >> 2) * A_SUB + swz(lr + RSTEP * e, lq & 3)] = ra[e];
#pragma unroll
      for (int e = 0; e < B_PER; ++e) B[(lq >> 2) * B_SUB + swz(lr + RSTEP * e, lq & 3)] = rb[e];
    };

    gload(0);
    sstore(0);
    __syncthreads();
    for (int kk = 0; kk < nk; ++kk) {
      const int cur = kk & 1;
      if (kk + 1 < nk) gload(kk + 1);
      const uint4* A = lds + cur * STAGE;
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
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < WNT; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
      }
      if (kk + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
    }

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
    float* red = reinterpret_cast<float*>(lds);
    if (wm == 1 && lane < 16) {
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) {
        const int col = wn * (BN / 2) + ni * 16 + lane;
        red[2 * col] = csum[ni];
        red[2 * col + 1] = csq[ni];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < 16) {
      float* prow = a.part + static_cast<int64_t>(blockIdx.x) * 2 * a.cout;
#pragma unroll
      for (int ni = 0; ni < WNT; ++ni) {
        const int col = wn * (BN / 2) + ni * 16 + lane;
        const int co = n0 + col;
        if (co < a.cout) {
          prow[co] = csum[ni] + red[2 * col];
          prow[a.cout + co] = csq[ni] + red[2 * col + 1];
        }
      }
    }
  }
}

}  // namespace

int conv_mfma_slabs(const ConvGeom& g) {
  const int64_t m = static_cast<int64_t>(g.n) * g.ho * g.wo;
  const int64_t mtiles = (m + kCBM - 1) / kCBM;
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
  k.mtiles = (k.m + kCBM - 1) / kCBM;
  k.fwo = FastDiv::make(g.wo);
  k.fho = FastDiv::make(g.ho);
  const bool stats = g.part != nullptr;
  const bool bn64 = g.cout <= 64;  // narrow layers: a 128-wide N tile would be half padding
  const bool bk64 = g.cin % 64 == 0;
  const int bn = bn64 ? 64 : 128;
  dim3 grid(conv_mfma_slabs(g), (g.cout + bn - 1) / bn);
  auto go = [&](auto bnc, auto bkc) {
    constexpr int BN = decltype(bnc)::value, BK = decltype(bkc)::value;
    if (g.scale_shift != nullptr) conv_mfma_kernel<1, false, BN, BK><<<grid, kCThreads, 0, st>>>(k);
    else if (stats) conv_mfma_kernel<0, true, BN, BK><<<grid, kCThreads, 0, st>>>(k);
    else conv_mfma_kernel<0, false, BN, BK><<<grid, kCThreads, 0, st>>>(k);
  };
  using I64 = std::integral_constant<int, 64>;
  using I128 = std::integral_constant<int, 128>;
  using I32 = std::integral_constant<int, 32>;
  if (bn64) {
    if (bk64) go(I64{}, I64{});
    else go(I64{}, I32{});
  } else {
    if (bk64) go(I128{}, I64{});
    else go(I128{}, I32{});
  }
}

}  // namespace rtseg
