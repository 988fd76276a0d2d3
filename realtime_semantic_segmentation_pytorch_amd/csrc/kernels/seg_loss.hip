// Fused segmentation cross-entropy: bilinear logit upsample + log-softmax +
// NLL + OHEM hard-pixel selection, forward and backward, with no host syncs.
//
// Reference semantics (core/loss.py:6-20, OhemCELoss):
//   n_min = #(labels != ignore) // 16
//   loss  = per-pixel CE (0 at ignored pixels), flattened
//   hard  = loss[loss > thresh];  if hard.numel() < n_min: hard = loss.topk(n_min)
//   return hard.mean()
// and core/loss.py:61-63 (nn.CrossEntropyLoss, optional class weights, mean/sum).
//
// MI355X design:
//  * The model's final F.interpolate(logits, full_res, bilinear) (e.g. reference
//    models/ddrnet.py:52) is folded into the loss: logits stay at 1/8 resolution
//    and each full-resolution pixel interpolates its 4 taps on the fly, so the
//    [N, C, H, W] fp32 full-resolution logit tensor and its gradient are never
//    materialised in HBM.
//  * Auxiliary heads (nearest-downsampled masks, reference core/seg_trainer.py:57-62)
//    use the same kernel: the label map is read through a nearest-neighbour
//    index remap instead of being resized.
//  * The top-k fallback is a 3-pass radix select on the float bits of the
//    per-pixel loss (11/11/10 bits, LDS-private histograms); every pass reads a
//    device flag and exits immediately when the threshold branch was taken, so
//    the whole loss is one stream of launches with zero host synchronisation
//    (the reference performs 3 host syncs per call).
//  * Backward recomputes the softmax per pixel, weights it by the device-side
//    selection rule, and reduces the transpose of the bilinear map through LDS
//    (row pass, then column pass); only block-border cells use global atomics.
//  * Deterministic: the backward's tiles are launched in classes (tile row mod Py, tile column
//    mod Px) whose low-resolution bounding boxes are pairwise disjoint, so every gradient cell
//    takes at most one atomic add per launch and the launches run in a fixed stream order; every
//    sum inside a block has one writer per cell and phase; the loss sums are per-block slabs
//    reduced in a fixed order.  Same inputs -> the same bits, run to run and process to process.
#include <algorithm>
#include <cstdlib>

#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

// stats[] slots (double so counts stay exact)
enum : int {
  S_VALID = 0, S_HARD_CNT, S_HARD_SUM, S_WLOSS, S_WSUM, S_FLAG_TOPK, S_K, S_KREM, S_PREFIX,
  S_CNT_EQ, S_SUM_GT, S_SEL_T, S_SEL_A, S_SEL_B, S_LOSS, S_NSTATS = 32
};
enum : int { MODE_OHEM = 0, MODE_MEAN = 1, MODE_SUM = 2 };

struct LossGeo {
  int n, c, h, w;  // logits
  int64_t sn, sc, sh, sw;
  int lh, lw, oh, ow;
  LinMap mh, mw;
  float lab_sy, lab_sx;  // nearest label remap scales (label = floor(o * s))
  const int64_t* lab64;  // labels: int64 (torch.long) ...
  const uint8_t* lab8;   // ... or uint8 (8x less label traffic); exactly one is set
};

__device__ __forceinline__ int64_t label_at(const LossGeo& g, int n, int oy, int ox) {
  int ly = (g.lh == g.oh) ? oy : min(static_cast<int>(floorf(oy * g.lab_sy)), g.lh - 1);
  int lx = (g.lw == g.ow) ? ox : min(static_cast<int>(floorf(ox * g.lab_sx)), g.lw - 1);
  const int64_t i = (static_cast<int64_t>(n) * g.lh + ly) * g.lw + lx;
  return g.lab8 ? static_cast<int64_t>(g.lab8[i]) : g.lab64[i];
}

// ------------------------------- tiles -------------------------------------
// A block owns a TH x TW tile of output pixels.  The low-resolution logits
// under the tile's bounding box are staged once into LDS as fp32 [BH][BW][CP]
// (CP = C rounded up to odd -> conflict-free strided reads), then vertically
// interpolated to the tile's TH rows, V[TH][BW][CP]; every pixel then needs
// only 2 LDS reads per class.  Identity geometry (aux heads) reads L directly.
struct TileGeo {
  int n, oy0, ox0, oy1, ox1, by0, bx0, BH, BW, CP;
  bool ident_h, ident_w;
};

// A launch over the tiles with tile row = py (mod Py) and tile column = px (mod Px); {0, 1, 0, 1}:
// every tile
struct TileClass {
  int py, Py, px, Px;
};

template <int TH, int TW>
__device__ __forceinline__ TileGeo tile_geo(const LossGeo& g, TileClass k = {0, 1, 0, 1}) {
  TileGeo t;
  const int tiles_x = (g.ow + TW - 1) / TW;
  const int tiles_y = (g.oh + TH - 1) / TH;
  const int cx = (tiles_x - k.px + k.Px - 1) / k.Px, cy = (tiles_y - k.py + k.Py - 1) / k.Py;
  const int bid = blockIdx.x;
  const int tx = k.px + k.Px * (bid % cx);
  const int ty = k.py + k.Py * ((bid / cx) % cy);
  t.n = bid / (cx * cy);
  t.oy0 = ty * TH; t.ox0 = tx * TW;
  t.oy1 = min(t.oy0 + TH, g.oh) - 1; t.ox1 = min(t.ox0 + TW, g.ow) - 1;
  int a0, a1; float l;
  g.mh.map(t.oy0, a0, a1, l); t.by0 = a0;
  g.mh.map(t.oy1, a0, a1, l); const int by1 = a1;
  g.mw.map(t.ox0, a0, a1, l); t.bx0 = a0;
  g.mw.map(t.ox1, a0, a1, l); const int bx1 = a1;
  t.BH = by1 - t.by0 + 1; t.BW = bx1 - t.bx0 + 1;
  t.CP = g.c | 1;
  t.ident_h = g.oh == g.h; t.ident_w = g.ow == g.w;
  return t;
}

template <typename T, int TH, int NC>
__device__ __forceinline__ const float* stage_logits(const T* __restrict__ x, const LossGeo& g,
                                                     const TileGeo& t, float* L, float* V,
                                                     bool want_v = true) {
  const int C = NC > 0 ? NC : g.c;
  const T* base = x + t.n * g.sn + t.by0 * g.sh + t.bx0 * g.sw;
  // one thread per bounding-box pixel, classes innermost (contiguous in NHWC)
  for (int e = threadIdx.x; e < t.BH * t.BW; e += blockDim.x) {
    const int i = e / t.BW, j = e - (e / t.BW) * t.BW;
    const T* src = base + i * g.sh + j * g.sw;
    float* dst = L + e * t.CP;
    if constexpr (NC > 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) dst[c] = Io<T>::ld(src + c * g.sc);
    } else {
      for (int c = 0; c < C; ++c) dst[c] = Io<T>::ld(src + c * g.sc);
    }
  }
  __syncthreads();
  if (t.ident_h || !want_v) return L;  // rows already at output resolution / caller uses L taps
  // vertical interpolation to the tile's TH output rows: one thread per (row, column)
  for (int e = threadIdx.x; e < TH * t.BW; e += blockDim.x) {
    const int r = e / t.BW, j = e - (e / t.BW) * t.BW;
    int y0, y1; float ly;
    g.mh.map(min(t.oy0 + r, t.oy1), y0, y1, ly);
    const float* a0 = L + ((y0 - t.by0) * t.BW + j) * t.CP;
    const float* a1 = L + ((y1 - t.by0) * t.BW + j) * t.CP;
    float* dst = V + e * t.CP;
    if constexpr (NC > 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) dst[c] = a0[c] + ly * (a1[c] - a0[c]);
    } else {
      for (int c = 0; c < C; ++c) dst[c] = a0[c] + ly * (a1[c] - a0[c]);
    }
  }
  __syncthreads();
  return V;
}

// pointers to the two horizontal taps of output pixel (r, ox) inside the staged rows
__device__ __forceinline__ void pixel_taps(const LossGeo& g, const TileGeo& t, const float* rows,
                                           int r, int ox, const float*& pa, const float*& pb,
                                           float& lx) {
  const int rr = t.ident_h ? (t.oy0 + r - t.by0) : r;
  int x0, x1;
  g.mw.map(ox, x0, x1, lx);
  pa = rows + (rr * t.BW + (x0 - t.bx0)) * t.CP;
  pb = rows + (rr * t.BW + (x1 - t.bx0)) * t.CP;
}

// ------------------------------- forward -----------------------------------
enum : int { SL_VALID = 0, SL_HCNT, SL_HSUM, SL_WLOSS, SL_WSUM, SL_N };

// Log-sum-exp of the interpolated logits of one pixel. NC > 0: class count known
// at compile time -> logits held in registers, max then sum (no divergence);
// NC == 0: runtime class count, online (single pass) formulation.
template <int NC>
__device__ __forceinline__ float pixel_lse(const float* pa, const float* pb, float lx, int C,
                                           int64_t y, float& zy) {
  if constexpr (NC > 0) {
    float z[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) z[c] = pa[c] + lx * (pb[c] - pa[c]);
    float m = z[0];
#pragma unroll
    for (int c = 1; c < NC; ++c) m = fmaxf(m, z[c]);
    float s = 0.f;
    zy = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      s += __expf(z[c] - m);
      zy = (c == y) ? z[c] : zy;
    }
    return m + __logf(s);
  } else {
    float m = -INFINITY, s = 0.f;
    zy = 0.f;
    for (int c = 0; c < C; ++c) {
      const float z = pa[c] + lx * (pb[c] - pa[c]);
      if (c == y) zy = z;
      if (z > m) { s = s * __expf(m - z) + 1.f; m = z; }
      else s += __expf(z - m);
    }
    return m + __logf(s);
  }
}

template <typename T, int TH, int TW, int NC>
__global__ void __launch_bounds__(256) seg_ce_fwd_tile(
    const T* __restrict__ x, LossGeo g, int ignore,
    const float* __restrict__ cw, float thresh, float* __restrict__ pix_loss,
    float* __restrict__ pix_lse, double* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ double red[4];
  const TileGeo t = tile_geo<TH, TW>(g);
  float* L = sm;
  float* V = sm + t.BH * t.BW * t.CP;
  const float* rows = stage_logits<T, TH, NC>(x, g, t, L, V);
  float acc[SL_N] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = threadIdx.x; p < TH * TW; p += blockDim.x) {
    const int r = p / TW, oy = t.oy0 + r, ox = t.ox0 + p % TW;
    if (oy > t.oy1 || ox > t.ox1) continue;
    const float *pa, *pb; float lx;
    pixel_taps(g, t, rows, r, ox, pa, pb, lx);
    const int64_t y = label_at(g, t.n, oy, ox);
    float zy;
    const float lse = pixel_lse<NC>(pa, pb, lx, g.c, y, zy);
    float l = 0.f;
    if (y != ignore && y >= 0 && y < g.c) {
      l = fmaxf(lse - zy, 0.f);
      const float w = cw ? cw[y] : 1.f;
      acc[SL_VALID] += 1.f;
      acc[SL_WLOSS] += w * l;
      acc[SL_WSUM] += w;
    }
    if (l > thresh) { acc[SL_HCNT] += 1.f; acc[SL_HSUM] += l; }
    const int64_t pi = (static_cast<int64_t>(t.n) * g.oh + oy) * g.ow + ox;
    pix_loss[pi] = l;
    pix_lse[pi] = lse;
  }
#pragma unroll
  for (int k = 0; k < SL_N; ++k) {
    const double v = block_sum(static_cast<double>(acc[k]), red);
    if (threadIdx.x == 0) slab[static_cast<int64_t>(blockIdx.x) * SL_N + k] = v;
  }
}

// One block: reduce the per-tile slab, then decide threshold vs top-k on device.
__global__ void __launch_bounds__(1024) seg_finalize1(const double* __restrict__ slab, int nblk,
                                                      double* stats, int mode, float thresh,
                                                      float* out_loss) {
  __shared__ double red[16];
  double tot[SL_N];
#pragma unroll
  for (int k = 0; k < SL_N; ++k) {
    double v = 0.0;
    for (int i = threadIdx.x; i < nblk; i += blockDim.x) v += slab[static_cast<int64_t>(i) * SL_N + k];
    tot[k] = block_sum(v, red);
  }
  if (threadIdx.x != 0) return;
  for (int k = S_VALID; k < S_NSTATS; ++k) stats[k] = 0.0;
  stats[S_VALID] = tot[SL_VALID];
  stats[S_HARD_CNT] = tot[SL_HCNT];
  stats[S_HARD_SUM] = tot[SL_HSUM];
  stats[S_WLOSS] = tot[SL_WLOSS];
  stats[S_WSUM] = tot[SL_WSUM];
  if (mode == MODE_OHEM) {
    const double n_min = floor(stats[S_VALID] / 16.0);
    const double hc = stats[S_HARD_CNT];
    if (hc >= n_min) {
      const double v = hc > 0 ? stats[S_HARD_SUM] / hc : 0.0;
      stats[S_LOSS] = v;
      stats[S_SEL_T] = thresh;
      stats[S_SEL_A] = hc > 0 ? 1.0 / hc : 0.0;
      stats[S_SEL_B] = 0.0;
      stats[S_FLAG_TOPK] = 0.0;
      *out_loss = static_cast<float>(v);
    } else {
      stats[S_FLAG_TOPK] = 1.0;
      stats[S_K] = n_min;
      stats[S_KREM] = n_min;
      stats[S_PREFIX] = 0.0;
    }
  } else {
    const double ws = stats[S_WSUM];
    const double v = (mode == MODE_MEAN) ? (ws > 0 ? stats[S_WLOSS] / ws : 0.0) : stats[S_WLOSS];
    stats[S_LOSS] = v;
    stats[S_SEL_A] = (mode == MODE_MEAN) ? (ws > 0 ? 1.0 / ws : 0.0) : 1.0;
    stats[S_FLAG_TOPK] = 0.0;
    *out_loss = static_cast<float>(v);
  }
}

// Radix-select pass: histogram of `bits` bits at `shift` among keys whose
// higher bits equal the current prefix.
__global__ void __launch_bounds__(256) radix_hist_kernel(const float* __restrict__ loss,
                                                         int64_t total, const double* stats,
                                                         unsigned* __restrict__ hist, int shift,
                                                         int bits, int pass) {
  if (stats[S_FLAG_TOPK] != 1.0) return;
  __shared__ unsigned h[2048];
  const int nb = 1 << bits;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const unsigned prefix = static_cast<unsigned>(stats[S_PREFIX]);
  const int hi_shift = shift + bits;  // bits above this pass
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    unsigned u = __float_as_uint(loss[i]);
    if (pass > 0 && (u >> hi_shift) != prefix) continue;
    atomicAdd(&h[(u >> shift) & (nb - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += blockDim.x)
    if (h[i]) atomicAdd(hist + i, h[i]);
}

// Single block: find the bin holding the k_rem-th largest candidate.
__global__ void __launch_bounds__(256) radix_scan_kernel(double* stats,
                                                         const unsigned* __restrict__ hist,
                                                         int bits, int last, float* out_loss) {
  if (stats[S_FLAG_TOPK] != 1.0) return;
  __shared__ unsigned part[256];
  const int nb = 1 << bits;
  const int per = nb / 256;
  unsigned s = 0;
  for (int j = 0; j < per; ++j) s += hist[threadIdx.x * per + j];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  double krem = stats[S_KREM];
  if (krem <= 0) {  // n_min == 0: nothing selected
    stats[S_FLAG_TOPK] = 2.0;  // resolved, empty selection
    stats[S_SEL_T] = INFINITY; stats[S_SEL_A] = 0; stats[S_SEL_B] = 0; stats[S_LOSS] = 0;
    *out_loss = 0.f;
    return;
  }
  double above = 0;
  int p = 255;
  for (; p > 0; --p) {
    if (above + part[p] >= krem) break;
    above += part[p];
  }
  int b = p * per + per - 1;
  for (; b > p * per; --b) {
    if (above + hist[b] >= krem) break;
    above += hist[b];
  }
  unsigned prefix = static_cast<unsigned>(stats[S_PREFIX]);
  stats[S_PREFIX] = static_cast<double>((prefix << bits) | static_cast<unsigned>(b));
  stats[S_KREM] = krem - above;
  if (last) stats[S_CNT_EQ] = hist[b];
}

__global__ void __launch_bounds__(256) sum_gt_kernel(const float* __restrict__ loss, int64_t total,
                                                     const double* stats, double* __restrict__ slab) {
  if (stats[S_FLAG_TOPK] != 1.0) return;
  __shared__ double red[4];
  const float vk = __uint_as_float(static_cast<unsigned>(stats[S_PREFIX]));
  double s = 0;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float l = loss[i];
    if (l > vk) s += l;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) slab[blockIdx.x] = s;  // summed in block order by seg_finalize2
}

__global__ void seg_finalize2(double* stats, const double* __restrict__ slab, int nblk, float* out_loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (stats[S_FLAG_TOPK] != 1.0) return;
  double sgt = 0.0;
  for (int i = 0; i < nblk; ++i) sgt += slab[i];
  stats[S_SUM_GT] = sgt;
  const double k = stats[S_K];
  const double krem = stats[S_KREM];
  const float vk = __uint_as_float(static_cast<unsigned>(stats[S_PREFIX]));
  double v = (stats[S_SUM_GT] + krem * static_cast<double>(vk)) / k;
  stats[S_LOSS] = v;
  stats[S_SEL_T] = vk;
  stats[S_SEL_A] = 1.0 / k;
  stats[S_SEL_B] = stats[S_CNT_EQ] > 0 ? krem / (stats[S_CNT_EQ] * k) : 0.0;
  *out_loss = static_cast<float>(v);
}

// ------------------------------- backward ----------------------------------
struct SelRule {
  int mode;
  float T, a, b;
};

__device__ __forceinline__ SelRule load_rule(const double* stats, int mode) {
  SelRule r;
  r.mode = mode;
  r.T = static_cast<float>(stats[S_SEL_T]);
  r.a = static_cast<float>(stats[S_SEL_A]);
  r.b = static_cast<float>(stats[S_SEL_B]);
  return r;
}

// d loss / d z_c at one pixel = w * (softmax_c - [c == y]); returns w.
__device__ __forceinline__ float pixel_weight(const SelRule& r, float l, int64_t y, int ignore,
                                              int C, const float* cw) {
  bool ok = (y != ignore) && y >= 0 && y < C;
  if (!ok) return 0.f;  // ignored pixels carry a constant 0 loss: no gradient
  if (r.mode == MODE_OHEM) {
    if (l > r.T) return r.a;
    if (l == r.T) return r.b;
    return 0.f;
  }
  return r.a * (cw ? cw[y] : 1.f);
}

// Identity geometry (loss grid == logit grid): gradient written per pixel.
template <typename T, typename G>
__global__ void __launch_bounds__(256) seg_ce_bwd_identity(
    const T* __restrict__ x, LossGeo g, int ignore,
    const float* __restrict__ cw, const float* __restrict__ pix_loss,
    const float* __restrict__ pix_lse, const double* __restrict__ stats, int mode,
    const float* __restrict__ grad_out, G* __restrict__ gx, int64_t gsn, int64_t gsc,
    int64_t gsh, int64_t gsw) {
  const SelRule r = load_rule(stats, mode);
  const float go = *grad_out;
  const int64_t total = static_cast<int64_t>(g.n) * g.oh * g.ow;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int ox = static_cast<int>(i % g.ow);
    int64_t t = i / g.ow;
    int oy = static_cast<int>(t % g.oh);
    int n = static_cast<int>(t / g.oh);
    int64_t y = label_at(g, n, oy, ox);
    float w = pixel_weight(r, pix_loss[i], y, ignore, g.c, cw) * go;
    G* o = gx + n * gsn + oy * gsh + ox * gsw;
    if (w == 0.f) {
      for (int c = 0; c < g.c; ++c) Io<G>::st(o + c * gsc, 0.f);
      continue;
    }
    const T* p = x + n * g.sn + oy * g.sh + ox * g.sw;
    const float lse = pix_lse[i];
    for (int c = 0; c < g.c; ++c) {
      float z = Io<T>::ld(p + c * g.sc);
      float v = __expf(z - lse) - (c == y ? 1.f : 0.f);
      Io<G>::st(o + c * gsc, w * v);
    }
  }
}

// Upsampled geometry.  The gradient w.r.t. low-res logit (c, i, j) is
//   sum_{oy, ox} wy(oy, i) * wx(ox, j) * G_c(oy, ox),
//   G_c = w_pixel * (softmax_c - [c == label]).
// Pass 1: one thread per (output row r, low-res column j) walks the ~1/scale
// output pixels whose horizontal taps include j, recomputes G for each (every
// pixel is visited by its two columns) and accumulates wx * G in registers ->
// R[c][r][j] in LDS.  Pass 2: one thread per (class, low-res column) folds the
// rows with wy and issues fp32 atomics only for the tile's bounding-box cells
// (shared with neighbouring tiles).  No [C, TH, TW] gradient tile, so LDS stays
// small and occupancy high.
template <typename T, int TH, int TW, int NC>
__global__ void __launch_bounds__(256) seg_ce_bwd_tile(
    const T* __restrict__ x, LossGeo g, int ignore,
    const float* __restrict__ cw, const float* __restrict__ pix_loss,
    const float* __restrict__ pix_lse, const double* __restrict__ stats, int mode,
    const float* __restrict__ grad_out, float* __restrict__ gacc, int64_t asn, int64_t asc,
    int64_t ash, int64_t asw, TileClass cls) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ int tx0[TW], tx1[TW], ty0[TH], ty1[TH], jlo[TW + 4], jhi[TW + 4];  // BW <= TW + 2
  __shared__ float tlx[TW], tly[TH];
  const TileGeo t = tile_geo<TH, TW>(g, cls);
  const int C = NC > 0 ? NC : g.c;
  const int BW = t.BW, RS = BW | 1;
  const int nx = t.ox1 - t.ox0 + 1, ny = t.oy1 - t.oy0 + 1;
  float* L = sm;                          // [BH][BW][CP]
  float* R = L + t.BH * t.BW * t.CP;      // [C][TH][RS]
  for (int k = threadIdx.x; k < TW; k += blockDim.x) {
    int a0, a1; float l;
    g.mw.map(min(t.ox0 + k, t.ox1), a0, a1, l);
    tx0[k] = a0 - t.bx0; tx1[k] = a1 - t.bx0; tlx[k] = l;
  }
  for (int k = threadIdx.x; k < TH; k += blockDim.x) {
    int a0, a1; float l;
    g.mh.map(min(t.oy0 + k, t.oy1), a0, a1, l);
    ty0[k] = a0 - t.by0; ty1[k] = a1 - t.by0; tly[k] = l;
  }
  stage_logits<T, TH, NC>(x, g, t, L, nullptr, false);  // syncs: tables visible too
  // ox range of each low-res column (taps are monotone in ox)
  for (int j = threadIdx.x; j < BW; j += blockDim.x) {
    int lo = nx, hi = -1;
    for (int k = 0; k < nx; ++k)
      if (tx0[k] == j || tx1[k] == j) { lo = min(lo, k); hi = k; }
    jlo[j] = lo; jhi[j] = hi;
  }
  __syncthreads();
  const SelRule rule = load_rule(stats, mode);
  const float go = *grad_out;
  for (int rj = threadIdx.x; rj < TH * BW; rj += blockDim.x) {
    const int r = rj / BW, j = rj - (rj / BW) * BW;
    float* Rc = R + r * RS + j;
    float acc[NC > 0 ? NC : 1];
    if constexpr (NC > 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = 0.f;
    } else {
      for (int c = 0; c < C; ++c) Rc[c * TH * RS] = 0.f;
    }
    if (r < ny) {
      const int oy = t.oy0 + r;
      const float ly = tly[r];
      const float* row0 = L + ty0[r] * t.BW * t.CP;
      const float* row1 = L + ty1[r] * t.BW * t.CP;
      const int64_t prow = (static_cast<int64_t>(t.n) * g.oh + oy) * g.ow + t.ox0;
      for (int k = jlo[j]; k <= jhi[j]; ++k) {
        const float lx = tlx[k];
        const float wx = (tx0[k] == j ? 1.f - lx : 0.f) + (tx1[k] == j ? lx : 0.f);
        const int64_t y = label_at(g, t.n, oy, t.ox0 + k);
        const float w = wx * pixel_weight(rule, pix_loss[prow + k], y, ignore, C, cw) * go;
        if (w == 0.f) continue;
        const float lse = pix_lse[prow + k];
        const float* p00 = row0 + tx0[k] * t.CP;
        const float* p01 = row0 + tx1[k] * t.CP;
        const float* p10 = row1 + tx0[k] * t.CP;
        const float* p11 = row1 + tx1[k] * t.CP;
        const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx;
        const float w10 = ly * (1.f - lx), w11 = ly * lx;
        if constexpr (NC > 0) {
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const float z = w00 * p00[c] + w01 * p01[c] + w10 * p10[c] + w11 * p11[c];
            acc[c] += w * (__expf(z - lse) - (c == y ? 1.f : 0.f));
          }
        } else {
          for (int c = 0; c < C; ++c) {
            const float z = w00 * p00[c] + w01 * p01[c] + w10 * p10[c] + w11 * p11[c];
            Rc[c * TH * RS] += w * (__expf(z - lse) - (c == y ? 1.f : 0.f));
          }
        }
      }
    }
    if constexpr (NC > 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) Rc[c * TH * RS] = acc[c];
    }
  }
  __syncthreads();
  // column pass: fold output rows onto low-res rows, accumulate globally
  for (int cj = threadIdx.x; cj < C * BW; cj += blockDim.x) {
    const int c = cj / BW, j = cj - (cj / BW) * BW;
    float* dst = gacc + t.n * asn + c * asc + t.by0 * ash + (t.bx0 + j) * asw;
    int ic = ty0[0];
    float a = 0.f, b = 0.f;
    for (int r = 0; r < ny; ++r) {
      const int i0 = ty0[r];
      while (ic < i0) {
        if (a != 0.f) atomicAdd(dst + static_cast<int64_t>(ic) * ash, a);
        a = b; b = 0.f; ++ic;
      }
      const float v = R[(c * TH + r) * RS + j];
      if (ty1[r] == i0) a += v;
      else { const float l = tly[r]; a += (1.f - l) * v; b += l * v; }
    }
    if (a != 0.f) atomicAdd(dst + static_cast<int64_t>(ic) * ash, a);
    if (b != 0.f && ic + 1 < t.BH) atomicAdd(dst + static_cast<int64_t>(ic + 1) * ash, b);
  }
}

// Upsampled geometry, class count known at compile time (Cityscapes' 19): the "run" form.
// Every output pixel has ONE left horizontal tap x0; the ~1/scale pixels of an output row
// that share x0 = j (a run) also share their right tap x1 and the row's two vertical taps.
// One thread per (output row r, run j) -- the tile is sized so that TH x BW <= 256 threads:
//   * the tile's per-pixel (weight, lse, label) are staged to LDS first, coalesced, so the
//     run loop below issues no global loads;
//   * the thread reads the run's 4 x C tap logits from LDS once and folds them vertically into
//     u_c = lerp_y(L[y0][j], L[y1][j]) and d_c = lerp_y(L[y0][x1], L[y1][x1]) - u_c (registers);
//   * per pixel of the run: z_c = u_c + lx * d_c (one FMA), G_c = w (exp(z_c - lse) - [c == y]),
//     A0_c += (1 - lx) G_c, A1_c += lx G_c -- every pixel's softmax is computed exactly once;
//   * stores A0 to R[c][r][j]; after a barrier adds A1 (still in registers) to R[c][r][x1]:
//     runs of one row have distinct x1, so no two threads write one cell in either phase;
//   * the column pass folds R onto low-res rows (global atomics only for tile-border cells).
// The round-4 form above visits every pixel from both of its columns (2 softmaxes per pixel),
// re-interpolates 4 taps per class per visit from LDS and loads each pixel's loss / lse /
// label inside its serial loop: 2.05 ms per DDRNet-23 step (profiles/r5_start_prof).
template <typename T, int TH, int TW, int NC>
__global__ void __launch_bounds__(256) seg_ce_bwd_run(
    const T* __restrict__ x, LossGeo g, int ignore,
    const float* __restrict__ cw, const float* __restrict__ pix_loss,
    const float* __restrict__ pix_lse, const double* __restrict__ stats, int mode,
    const float* __restrict__ grad_out, float* __restrict__ gacc, int64_t asn, int64_t asc,
    int64_t ash, int64_t asw, TileClass cls) {
  static_assert(NC > 0, "run form needs the class count at compile time");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ int tx0[TW], tx1[TW], ty0[TH], ty1[TH], jlo[TW + 4], jhi[TW + 4];  // BW <= TW + 2
  __shared__ float tlx[TW], tly[TH];
  __shared__ float2 pwl[TH * TW];  // per tile pixel: (gradient weight, lse)
  __shared__ uint8_t plab[TH * TW];
  const TileGeo t = tile_geo<TH, TW>(g, cls);
  const int BW = t.BW, RS = BW | 1;
  const int nx = t.ox1 - t.ox0 + 1, ny = t.oy1 - t.oy0 + 1;
  float* L = sm;                          // [BH][BW][CP]
  float* R = L + t.BH * t.BW * t.CP;      // [TH][BW][NC]: classes innermost (conflict-free)
  for (int k = threadIdx.x; k < TW; k += blockDim.x) {
    int a0, a1; float l;
    g.mw.map(min(t.ox0 + k, t.ox1), a0, a1, l);
    tx0[k] = a0 - t.bx0; tx1[k] = a1 - t.bx0; tlx[k] = l;
  }
  for (int k = threadIdx.x; k < TH; k += blockDim.x) {
    int a0, a1; float l;
    g.mh.map(min(t.oy0 + k, t.oy1), a0, a1, l);
    ty0[k] = a0 - t.by0; ty1[k] = a1 - t.by0; tly[k] = l;
  }
  {
    const SelRule rule = load_rule(stats, mode);
    const float go = *grad_out;
    for (int p = threadIdx.x; p < TH * TW; p += blockDim.x) {
      const int r = p / TW, k = p - (p / TW) * TW;
      float w = 0.f, lse = 0.f;
      int64_t y = 0;
      if (r < ny && k < nx) {
        const int oy = t.oy0 + r, ox = t.ox0 + k;
        const int64_t pi = (static_cast<int64_t>(t.n) * g.oh + oy) * g.ow + ox;
        y = label_at(g, t.n, oy, ox);
        w = pixel_weight(rule, pix_loss[pi], y, ignore, NC, cw) * go;
        lse = pix_lse[pi];
      }
      pwl[p] = make_float2(w, lse);
      plab[p] = static_cast<uint8_t>(w != 0.f ? y : 0);  // w != 0 implies 0 <= y < NC <= 255
    }
  }
  for (int j = threadIdx.x; j < TW + 4; j += blockDim.x) { jlo[j] = nx; jhi[j] = -1; }
  stage_logits<T, TH, NC>(x, g, t, L, nullptr, false);  // syncs: tables and pixels visible too
  // the run of each low-res column: tile columns k with x0(k) == j (x0 is monotone in k), from
  // the run boundaries -- one thread per tile column
  for (int k = threadIdx.x; k < nx; k += blockDim.x) {
    const int j = tx0[k];
    if (k == 0 || tx0[k - 1] != j) jlo[j] = k;
    if (k == nx - 1 || tx0[k + 1] != j) jhi[j] = k;
  }
  __syncthreads();
  // one item per thread (launcher: TH * BW <= blockDim)
  const int rj = threadIdx.x;
  const bool item = rj < TH * BW;
  const int r = item ? rj / BW : 0, j = item ? rj - (rj / BW) * BW : 0;
  float a0[NC], a1[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) { a0[c] = 0.f; a1[c] = 0.f; }
  int j1 = j;
  if (item && r < ny && jlo[j] <= jhi[j]) {
    j1 = tx1[jlo[j]];
    const float ly = tly[r];
    const float* q00 = L + (ty0[r] * t.BW + j) * t.CP;
    const float* q10 = L + (ty1[r] * t.BW + j) * t.CP;
    const float* q01 = L + (ty0[r] * t.BW + j1) * t.CP;
    const float* q11 = L + (ty1[r] * t.BW + j1) * t.CP;
    float u[NC], d[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float left = q00[c] + ly * (q10[c] - q00[c]);
      const float right = q01[c] + ly * (q11[c] - q01[c]);
      u[c] = left;
      d[c] = right - left;
    }
    for (int k = jlo[j]; k <= jhi[j]; ++k) {
      const float2 wl = pwl[r * TW + k];
      if (wl.x == 0.f) continue;
      const int y = plab[r * TW + k];
      const float lx = tlx[k];
      const float wa = wl.x * (1.f - lx), wb = wl.x * lx;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float gc = __expf(fmaf(lx, d[c], u[c]) - wl.y) - (c == y ? 1.f : 0.f);
        a0[c] = fmaf(wa, gc, a0[c]);
        a1[c] = fmaf(wb, gc, a1[c]);
      }
    }
  }
  if (j1 == j) {  // no right column (empty run, or the clamped last low-res column)
#pragma unroll
    for (int c = 0; c < NC; ++c) { a0[c] += a1[c]; a1[c] = 0.f; }
  }
  if (item) {
#pragma unroll
    for (int c = 0; c < NC; ++c) R[(r * RS + j) * NC + c] = a0[c];
  }
  __syncthreads();
  if (item && j1 != j) {
#pragma unroll
    for (int c = 0; c < NC; ++c) R[(r * RS + j1) * NC + c] += a1[c];
  }
  __syncthreads();
  // column pass: fold output rows onto low-res rows, accumulate globally.  Classes fastest
  // across lanes: a wave's atomics then cover contiguous channels-last cells (64 x 4 B runs)
  // instead of one 4-B add per 76-B pixel row
  for (int cj = threadIdx.x; cj < NC * BW; cj += blockDim.x) {
    const int jj = cj / NC, c = cj - (cj / NC) * NC;
    float* dst = gacc + t.n * asn + c * asc + t.by0 * ash + (t.bx0 + jj) * asw;
    int ic = ty0[0];
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < ny; ++rr) {
      const int i0 = ty0[rr];
      while (ic < i0) {
        if (a != 0.f) atomicAdd(dst + static_cast<int64_t>(ic) * ash, a);
        a = b; b = 0.f; ++ic;
      }
      const float v = R[(rr * RS + jj) * NC + c];
      if (ty1[rr] == i0) a += v;
      else { const float l = tly[rr]; a += (1.f - l) * v; b += l * v; }
    }
    if (a != 0.f) atomicAdd(dst + static_cast<int64_t>(ic) * ash, a);
    if (b != 0.f && ic + 1 < t.BH) atomicAdd(dst + static_cast<int64_t>(ic + 1) * ash, b);
  }
}

// Round-5 form of the run kernel (the default; RTSEG_LOSS_BWD_RUN=1 selects the form above).
// Same (output row, run) work split and the same LDS row buffer R, three changes:
//  * per-pixel metadata packed into 6 bytes (lse pre-scaled by log2 e, and a 16-bit word holding
//    the label and the selection code -- the weight is a function of (code, label), evaluated per
//    pixel in the run loop): 44 -> 37 KB of LDS per block, 4 blocks per CU instead of 3; the
//    tile's metadata loads are issued together (unrolled) before any of them is used;
//  * logits pre-scaled by log2 e and shifted by the run's largest lse, the shift undone in the
//    per-pixel weight: per pixel and class one FMA, one v_exp_f32 and two FMAs (the round-5
//    form above: 7 VALU + exp).  A run whose lse spans more than 2^60 falls back to a per-pixel
//    shift;
//  * the one-hot term -w [c == y] leaves the class loop: after the row buffer is complete each
//    thread subtracts its pixels' weights from R[r][j][y] / R[r][j1][y] with LDS float atomics
//    (no two lanes of one instruction address one cell).
template <typename T, int TH, int TW, int NC>
__global__ void __launch_bounds__(256) seg_ce_bwd_run2(
    const T* __restrict__ x, LossGeo g, int ignore,
    const float* __restrict__ cw, const float* __restrict__ pix_loss,
    const float* __restrict__ pix_lse, const double* __restrict__ stats, int mode,
    const float* __restrict__ grad_out, float* __restrict__ gacc, int64_t asn, int64_t asc,
    int64_t ash, int64_t asw, TileClass cls) {
  static_assert(NC > 0 && NC < 255, "run form needs the class count at compile time");
  constexpr float kL2E = 1.4426950408889634f;
  constexpr int PIT = (TH * TW + 255) / 256;  // metadata items per thread (launch: 256 threads)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ int tx0[TW], tx1[TW], ty0[TH], ty1[TH], jlo[TW + 4], jhi[TW + 4];  // BW <= TW + 2
  __shared__ float tlx[TW], tly[TH];
  __shared__ float plse[TH * TW];      // lse * log2 e
  __shared__ uint16_t pcode[TH * TW];  // label | selection code << 8 (code 0: no gradient)
  const TileGeo t = tile_geo<TH, TW>(g, cls);
  const int BW = t.BW, RS = BW | 1;
  const int nx = t.ox1 - t.ox0 + 1, ny = t.oy1 - t.oy0 + 1;
  float* L = sm;                          // [BH][BW][CP]
  float* R = L + t.BH * t.BW * t.CP;      // [TH][RS][NC]: classes innermost
  for (int k = threadIdx.x; k < TW; k += blockDim.x) {
    int a0, a1; float l;
    g.mw.map(min(t.ox0 + k, t.ox1), a0, a1, l);
    tx0[k] = a0 - t.bx0; tx1[k] = a1 - t.bx0; tlx[k] = l;
  }
  for (int k = threadIdx.x; k < TH; k += blockDim.x) {
    int a0, a1; float l;
    g.mh.map(min(t.oy0 + k, t.oy1), a0, a1, l);
    ty0[k] = a0 - t.by0; ty1[k] = a1 - t.by0; tly[k] = l;
  }
  const SelRule rule = load_rule(stats, mode);
  const float go = *grad_out;
  {
    float pl[PIT], ls[PIT];
    int yy[PIT];
#pragma unroll
    for (int it = 0; it < PIT; ++it) {  // all loads first
      const int p = threadIdx.x + it * 256;
      const int r = p / TW, k = p - (p / TW) * TW;
      pl[it] = 0.f; ls[it] = 0.f; yy[it] = -1;
      if (p < TH * TW && r < ny && k < nx) {
        const int oy = t.oy0 + r, ox = t.ox0 + k;
        const int64_t pi = (static_cast<int64_t>(t.n) * g.oh + oy) * g.ow + ox;
        const int64_t y = label_at(g, t.n, oy, ox);
        yy[it] = (y == ignore || y < 0 || y >= NC) ? -1 : static_cast<int>(y);
        pl[it] = pix_loss[pi];
        ls[it] = pix_lse[pi];
      }
    }
#pragma unroll
    for (int it = 0; it < PIT; ++it) {
      const int p = threadIdx.x + it * 256;
      if (p >= TH * TW) break;
      int code = 0;
      if (yy[it] >= 0) {
        if (rule.mode != MODE_OHEM) code = 3;
        else if (pl[it] > rule.T) code = 1;
        else if (pl[it] == rule.T) code = 2;
      }
      plse[p] = ls[it] * kL2E;
      pcode[p] = static_cast<uint16_t>(code == 0 ? 0 : (yy[it] | (code << 8)));
    }
  }
  for (int j = threadIdx.x; j < TW + 4; j += blockDim.x) { jlo[j] = nx; jhi[j] = -1; }
  stage_logits<T, TH, NC>(x, g, t, L, nullptr, false);  // syncs: tables and pixels visible too
  for (int k = threadIdx.x; k < nx; k += blockDim.x) {
    const int j = tx0[k];
    if (k == 0 || tx0[k - 1] != j) jlo[j] = k;
    if (k == nx - 1 || tx0[k + 1] != j) jhi[j] = k;
  }
  __syncthreads();
  // gradient weight of a pixel from its code word (0 when it carries no gradient)
  auto weight = [&](int cw16) -> float {
    const int code = cw16 >> 8;
    const float w = code == 1 ? rule.a : code == 2 ? rule.b : code == 3 ? rule.a * (cw ? cw[cw16 & 255] : 1.f) : 0.f;
    return w * go;
  };
  const int rj = threadIdx.x;
  const bool item = rj < TH * BW;
  const int r = item ? rj / BW : 0, j = item ? rj - (rj / BW) * BW : 0;
  const bool run = item && r < ny && jlo[j] <= jhi[j];
  const int k0 = run ? jlo[j] : 0, k1 = run ? jhi[j] : -1;
  const int j1 = run ? tx1[k0] : j;  // == j: no right column (the clamped last low-res column)
  float a0[NC], a1[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) { a0[c] = 0.f; a1[c] = 0.f; }
  if (run) {
    float m = -INFINITY, mn = INFINITY;
    for (int k = k0; k <= k1; ++k) {
      if (pcode[r * TW + k] == 0) continue;
      const float v = plse[r * TW + k];
      m = fmaxf(m, v); mn = fminf(mn, v);
    }
    if (m != -INFINITY) {
      const bool wide = m - mn > 60.f;
      const float sh = wide ? 0.f : m;
      const float ly = tly[r];
      const float* q00 = L + (ty0[r] * t.BW + j) * t.CP;
      const float* q10 = L + (ty1[r] * t.BW + j) * t.CP;
      const float* q01 = L + (ty0[r] * t.BW + j1) * t.CP;
      const float* q11 = L + (ty1[r] * t.BW + j1) * t.CP;
      float u[NC], d[NC];  // log2-scaled left tap (shifted) and right-minus-left
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float left = q00[c] + ly * (q10[c] - q00[c]);
        const float right = q01[c] + ly * (q11[c] - q01[c]);
        u[c] = fmaf(left, kL2E, -sh);
        d[c] = (right - left) * kL2E;
      }
      if (!wide) {
        for (int k = k0; k <= k1; ++k) {
          const int cwd = pcode[r * TW + k];
          if (cwd == 0) continue;
          const float lx = tlx[k];
          const float s = weight(cwd) * __builtin_amdgcn_exp2f(m - plse[r * TW + k]);
          const float wa = s * (1.f - lx), wb = s * lx;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const float e = __builtin_amdgcn_exp2f(fmaf(lx, d[c], u[c]));
            a0[c] = fmaf(wa, e, a0[c]);
            a1[c] = fmaf(wb, e, a1[c]);
          }
        }
      } else {
        for (int k = k0; k <= k1; ++k) {
          const int cwd = pcode[r * TW + k];
          if (cwd == 0) continue;
          const float lx = tlx[k];
          const float s = weight(cwd), ls = plse[r * TW + k];
          const float wa = s * (1.f - lx), wb = s * lx;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const float e = __builtin_amdgcn_exp2f(fmaf(lx, d[c], u[c]) - ls);
            a0[c] = fmaf(wa, e, a0[c]);
            a1[c] = fmaf(wb, e, a1[c]);
          }
        }
      }
    }
  }
  if (j1 == j) {
#pragma unroll
    for (int c = 0; c < NC; ++c) { a0[c] += a1[c]; a1[c] = 0.f; }
  }
  if (item) {
#pragma unroll
    for (int c = 0; c < NC; ++c) R[(r * RS + j) * NC + c] = a0[c];
  }
  __syncthreads();
  if (item && j1 != j) {
#pragma unroll
    for (int c = 0; c < NC; ++c) R[(r * RS + j1) * NC + c] += a1[c];
  }
  __syncthreads();
  // one-hot terms in two phases, left taps then right taps: in each phase a cell (r, j) has one
  // writing thread (j1 = j + 1 is injective), so the order of the adds is fixed
  if (run) {
    float* ra = R + (r * RS + j) * NC;
    for (int k = k0; k <= k1; ++k) {
      const int cwd = pcode[r * TW + k];
      if (cwd == 0) continue;
      const float w = weight(cwd);
      ra[cwd & 255] -= j1 == j ? w : w * (1.f - tlx[k]);
    }
  }
  __syncthreads();
  if (run && j1 != j) {
    float* rb = R + (r * RS + j1) * NC;
    for (int k = k0; k <= k1; ++k) {
      const int cwd = pcode[r * TW + k];
      if (cwd == 0) continue;
      rb[cwd & 255] -= weight(cwd) * tlx[k];
    }
  }
  __syncthreads();
  for (int cj = threadIdx.x; cj < NC * BW; cj += blockDim.x) {
    const int jj = cj / NC, c = cj - (cj / NC) * NC;
    float* dst = gacc + t.n * asn + c * asc + t.by0 * ash + (t.bx0 + jj) * asw;
    int ic = ty0[0];
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < ny; ++rr) {
      const int i0 = ty0[rr];
      while (ic < i0) {
        if (a != 0.f) atomicAdd(dst + static_cast<int64_t>(ic) * ash, a);
        a = b; b = 0.f; ++ic;
      }
      const float v = R[(rr * RS + jj) * NC + c];
      if (ty1[rr] == i0) a += v;
      else { const float l = tly[rr]; a += (1.f - l) * v; b += l * v; }
    }
    if (a != 0.f) atomicAdd(dst + static_cast<int64_t>(ic) * ash, a);
    if (b != 0.f && ic + 1 < t.BH) atomicAdd(dst + static_cast<int64_t>(ic + 1) * ash, b);
  }
}

// fp32 accumulator (same strides as the gradient tensor) -> gradient dtype
template <typename G>
__global__ void __launch_bounds__(256) cast_out_kernel(const float* __restrict__ acc,
                                                       G* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    Io<G>::st(out + i, acc[i]);
}

// ------------------------------- launchers ---------------------------------
static LossGeo make_geo(const SegLossArgs& a) {
  LossGeo g;
  g.n = a.logits.n; g.c = a.logits.c; g.h = a.logits.h; g.w = a.logits.w;
  g.sn = a.logits.sn; g.sc = a.logits.sc; g.sh = a.logits.sh; g.sw = a.logits.sw;
  g.lh = a.lh; g.lw = a.lw; g.oh = a.out_h; g.ow = a.out_w;
  g.mh = LinMap::make(g.h, g.oh, a.align_corners);
  g.mw = LinMap::make(g.w, g.ow, a.align_corners);
  g.lab_sy = static_cast<float>(a.lh) / static_cast<float>(a.out_h);
  g.lab_sx = static_cast<float>(a.lw) / static_cast<float>(a.out_w);
  g.lab64 = a.label_bytes == 1 ? nullptr : static_cast<const int64_t*>(a.labels);
  g.lab8 = a.label_bytes == 1 ? static_cast<const uint8_t*>(a.labels) : nullptr;
  return g;
}

// Tile shape: wide tiles for the usual <= 32 classes, smaller ones otherwise
// so the staged logits / gradient tile stay within LDS.
template <int TH, int TW>
static int tiles_of(const LossGeo& g) {
  return ((g.oh + TH - 1) / TH) * ((g.ow + TW - 1) / TW) * g.n;
}

template <int TH, int TW>
static size_t stage_floats(const LossGeo& g) {
  const int bh = static_cast<int>((TH - 1) * g.mh.scale) + 3;
  const int bw = static_cast<int>((TW - 1) * g.mw.scale) + 3;
  const int cp = g.c | 1;
  const size_t v = g.oh == g.h ? 0 : static_cast<size_t>(TH) * bw * cp;  // no V rows on identity
  return static_cast<size_t>(bh) * bw * cp + v;
}

// Tile shape per geometry: 16x64 for upsampled main heads, 8x64 for identity
// (aux heads: the staged logits cover the whole tile), 4x32 beyond 32 classes.
enum TileKind { kTile16x64 = 0, kTile8x64 = 1, kTile4x32 = 2 };
static TileKind tile_kind(const LossGeo& g) {
  if (g.c > 32) return kTile4x32;
  return (g.oh == g.h) ? kTile8x64 : kTile16x64;
}

template <typename K>
static void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
}

int seg_loss_fwd_blocks(const SegLossArgs& a) {
  LossGeo g = make_geo(a);
  switch (tile_kind(g)) {
    case kTile16x64: return tiles_of<16, 64>(g);
    case kTile8x64: return tiles_of<8, 64>(g);
    default: return tiles_of<4, 32>(g);
  }
}

template <typename T, int TH, int TW, int NC>
static void fwd_tile(const SegLossArgs& a, const LossGeo& g, hipStream_t st) {
  const size_t lds = sizeof(float) * stage_floats<TH, TW>(g);
  auto k = seg_ce_fwd_tile<T, TH, TW, NC>;
  allow_lds(k, lds);
  const int nblk = tiles_of<TH, TW>(g);
  k<<<nblk, 256, lds, st>>>(static_cast<const T*>(a.logits.data), g, a.ignore_index,
                            a.class_weight, a.ohem_thresh, a.pix_loss, a.pix_lse, a.slab);
  seg_finalize1<<<1, 1024, 0, st>>>(a.slab, nblk, a.stats, a.mode, a.ohem_thresh, a.out_loss);
}

template <typename T>
static void fwd_t(const SegLossArgs& a, const LossGeo& g, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(g.n) * g.oh * g.ow;
  const TileKind tk = tile_kind(g);
  if (tk == kTile16x64) {
    if (g.c == 19) fwd_tile<T, 16, 64, 19>(a, g, st);  // Cityscapes: classes in registers
    else fwd_tile<T, 16, 64, 0>(a, g, st);
  } else if (tk == kTile8x64) {
    if (g.c == 19) fwd_tile<T, 8, 64, 19>(a, g, st);
    else fwd_tile<T, 8, 64, 0>(a, g, st);
  } else {
    fwd_tile<T, 4, 32, 0>(a, g, st);
  }
  if (a.mode != MODE_OHEM) return;
  // top-k fallback (every kernel exits at once when the threshold branch was taken)
  hipMemsetAsync(a.hist, 0, sizeof(unsigned) * 3 * 2048, st);
  const int shifts[3] = {21, 10, 0};
  const int bits[3] = {11, 11, 10};
  int grid = static_cast<int>((total + 4095) / 4096);
  grid = grid < 1 ? 1 : (grid > 512 ? 512 : grid);
  for (int p = 0; p < 3; ++p) {
    radix_hist_kernel<<<grid, 256, 0, st>>>(a.pix_loss, total, a.stats, a.hist + p * 2048,
                                            shifts[p], bits[p], p);
    radix_scan_kernel<<<1, 256, 0, st>>>(a.stats, a.hist + p * 2048, bits[p], p == 2, a.out_loss);
  }
  // a.slab (one row per forward tile, >= grid doubles) is free again after seg_finalize1
  sum_gt_kernel<<<grid, 256, 0, st>>>(a.pix_loss, total, a.stats, a.slab);
  seg_finalize2<<<1, 64, 0, st>>>(a.stats, a.slab, grid, a.out_loss);
}

void launch_seg_loss_fwd(const SegLossArgs& a, hipStream_t st) {
  LossGeo g = make_geo(a);
  switch (a.logits.dtype) {
    case kF32: fwd_t<float>(a, g, st); break;
    case kBF16: fwd_t<uint16_t>(a, g, st); break;
    default: fwd_t<_Float16>(a, g, st); break;
  }
}

// Tile classes for the backward: the smallest strides (Py, Px) such that two tiles of one class
// never share a low-resolution bounding-box cell (with one cell of margin, so a host/device
// rounding difference in the map cannot matter)
static int class_stride(const LinMap& m, int out, int T) {
  const int tiles = (out + T - 1) / T;
  auto lo = [&](int t) { int a0, a1; float l; m.map(t * T, a0, a1, l); return a0; };
  auto hi = [&](int t) { int a0, a1; float l; m.map(std::min((t + 1) * T, out) - 1, a0, a1, l); return a1; };
  for (int P = 1; P < tiles; ++P) {
    bool ok = true;
    for (int t = 0; t + P < tiles && ok; ++t) ok = hi(t) + 1 < lo(t + P);
    if (ok) return P;
  }
  return std::max(tiles, 1);
}

// launch(cls, grid) once per tile class, in a fixed order
template <int TH, int TW, typename F>
static void for_tile_classes(const LossGeo& g, F&& launch) {
  static const bool one = [] { const char* e = std::getenv("RTSEG_LOSS_ONE_CLASS"); return e && e[0] == '1'; }();
  const int Py = one ? 1 : class_stride(g.mh, g.oh, TH), Px = one ? 1 : class_stride(g.mw, g.ow, TW);
  const int tiles_y = (g.oh + TH - 1) / TH, tiles_x = (g.ow + TW - 1) / TW;
  for (int py = 0; py < Py; ++py)
    for (int px = 0; px < Px; ++px) {
      const int cy = (tiles_y - py + Py - 1) / Py, cx = (tiles_x - px + Px - 1) / Px;
      if (cy > 0 && cx > 0) launch(TileClass{py, Py, px, Px}, cy * cx * g.n);
    }
}

template <typename T, int TH, int TW, int NC>
static void bwd_run(const SegLossArgs& a, const LossGeo& g, const float* grad_out, hipStream_t st) {
  const int bh = static_cast<int>((TH - 1) * g.mh.scale) + 3;
  const int bw = static_cast<int>((TW - 1) * g.mw.scale) + 3;
  const size_t lds = sizeof(float) * (static_cast<size_t>(bh) * bw * (g.c | 1) +
                                      static_cast<size_t>(g.c) * TH * (bw | 1));
  auto k = seg_ce_bwd_run<T, TH, TW, NC>;
  allow_lds(k, lds);
  for_tile_classes<TH, TW>(g, [&](TileClass cls, int grid) {
    k<<<grid, 256, lds, st>>>(static_cast<const T*>(a.logits.data), g, a.ignore_index, a.class_weight,
                              a.pix_loss, a.pix_lse, a.stats, a.mode, grad_out, a.acc, a.acc_sn, a.acc_sc,
                              a.acc_sh, a.acc_sw, cls);
  });
}

template <typename T, int TH, int TW, int NC>
static void bwd_run2(const SegLossArgs& a, const LossGeo& g, const float* grad_out, hipStream_t st) {
  const int bh = static_cast<int>((TH - 1) * g.mh.scale) + 3;
  const int bw = static_cast<int>((TW - 1) * g.mw.scale) + 3;
  const size_t lds = sizeof(float) * (static_cast<size_t>(bh) * bw * (g.c | 1) +
                                      static_cast<size_t>(g.c) * TH * (bw | 1));
  auto k = seg_ce_bwd_run2<T, TH, TW, NC>;
  allow_lds(k, lds);
  for_tile_classes<TH, TW>(g, [&](TileClass cls, int grid) {
    k<<<grid, 256, lds, st>>>(static_cast<const T*>(a.logits.data), g, a.ignore_index, a.class_weight,
                              a.pix_loss, a.pix_lse, a.stats, a.mode, grad_out, a.acc, a.acc_sn, a.acc_sc,
                              a.acc_sh, a.acc_sw, cls);
  });
}

template <typename T, int TH, int TW, int NC>
static void bwd_tile(const SegLossArgs& a, const LossGeo& g, const float* grad_out,
                     hipStream_t st) {
  const int bh = static_cast<int>((TH - 1) * g.mh.scale) + 3;
  const int bw = static_cast<int>((TW - 1) * g.mw.scale) + 3;
  const size_t lds = sizeof(float) * (static_cast<size_t>(bh) * bw * (g.c | 1) +
                                      static_cast<size_t>(g.c) * TH * (bw | 1));
  auto k = seg_ce_bwd_tile<T, TH, TW, NC>;
  allow_lds(k, lds);
  for_tile_classes<TH, TW>(g, [&](TileClass cls, int grid) {
    k<<<grid, 256, lds, st>>>(static_cast<const T*>(a.logits.data), g, a.ignore_index, a.class_weight,
                              a.pix_loss, a.pix_lse, a.stats, a.mode, grad_out, a.acc, a.acc_sn, a.acc_sc,
                              a.acc_sh, a.acc_sw, cls);
  });
}

template <typename T, typename G>
static void bwd_t(const SegLossArgs& a, const LossGeo& g, const float* grad_out,
                  const Tensor4& gl, hipStream_t st) {
  const T* x = static_cast<const T*>(a.logits.data);
  if (g.oh == g.h && g.ow == g.w) {
    const int64_t total = static_cast<int64_t>(g.n) * g.oh * g.ow;
    seg_ce_bwd_identity<T, G><<<stream_grid(total, 256), 256, 0, st>>>(
        x, g, a.ignore_index, a.class_weight, a.pix_loss, a.pix_lse, a.stats, a.mode,
        grad_out, static_cast<G*>(gl.data), gl.sn, gl.sc, gl.sh, gl.sw);
    return;
  }
  const int64_t nacc = static_cast<int64_t>(g.n) * g.c * g.h * g.w;
  hipMemsetAsync(a.acc, 0, sizeof(float) * nacc, st);
  // x2 / x4 upsampling (ContextNet's, and other half-resolution heads): a 16 x 128 tile stages
  // 10 x 66 logit cells + a 19 x 16 x 67 row buffer (131 KB of LDS, one block per CU: the x2
  // head's backward ran 10x slower per pixel than DDRNet's x8, profiles/r4_zoo_models); 8 x 64
  // tiles fit four blocks per CU
  const bool fine = (g.mh.scale > 0.2f || g.mw.scale > 0.2f) && g.mh.scale <= 1.f && g.mw.scale <= 1.f;
  const char* rf = std::getenv("RTSEG_LOSS_BWD_RUN");
  const char run_form = rf != nullptr && rf[0] != 0 ? rf[0] : '2';
  if (g.c == 19) {
    if (fine) bwd_tile<T, 8, 64, 19>(a, g, grad_out, st);
    else if ((static_cast<int>(127 * g.mw.scale) + 3) * 14 <= 256 && run_form != '0') {
      // one (row, run) item per thread; =1: the first run form, =0: round-4 form
      if (run_form == '1') bwd_run<T, 14, 128, 19>(a, g, grad_out, st);
      else bwd_run2<T, 14, 128, 19>(a, g, grad_out, st);
    } else bwd_tile<T, 16, 128, 19>(a, g, grad_out, st);
  } else if (g.c <= 32) {
    if (fine) bwd_tile<T, 8, 64, 0>(a, g, grad_out, st);
    else bwd_tile<T, 16, 128, 0>(a, g, grad_out, st);
  } else {
    bwd_tile<T, 4, 32, 0>(a, g, grad_out, st);
  }
  cast_out_kernel<G><<<stream_grid(nacc, 256), 256, 0, st>>>(a.acc, static_cast<G*>(gl.data), nacc);
}

void launch_seg_loss_bwd(const SegLossArgs& a, const float* grad_out, const Tensor4& gl,
                         hipStream_t st) {
  LossGeo g = make_geo(a);
#define RT_BWD_G(T)                                                     \
  switch (gl.dtype) {                                                   \
    case kF32: bwd_t<T, float>(a, g, grad_out, gl, st); break;          \
    case kBF16: bwd_t<T, uint16_t>(a, g, grad_out, gl, st); break;      \
    default: bwd_t<T, _Float16>(a, g, grad_out, gl, st); break;         \
  }
  switch (a.logits.dtype) {
    case kF32: RT_BWD_G(float) break;
    case kBF16: RT_BWD_G(uint16_t) break;
    default: RT_BWD_G(_Float16) break;
  }
#undef RT_BWD_G
}

}  // namespace rtseg
