// Fused multi-tensor optimizer step + model-EMA update for CDNA4 (gfx950).
//
// Reference: utils/optimizer.py:4-20 (SGD momentum/wd, Adam, AdamW) and
// utils/model_ema.py:28-40 (EMA lerp of every parameter after the step).  The
// reference runs the optimizer (torch foreach kernels) and then walks the whole
// state dict again for the EMA; here ONE launch reads each parameter, its
// gradient and its optimizer state once, writes the updated parameter/state and
// the EMA copy in the same pass:
//
//   SGD : g' = g + wd*p ; buf = first ? g' : mom*buf + (1-damp)*g' ;
//         p -= lr * (nesterov ? g' + mom*buf : buf)
//   Adam: g' = g + wd*p (Adam) | p *= 1 - lr*wd (AdamW) ;
//         m = b1*m + (1-b1)*g' ; v = b2*v + (1-b2)*g'^2 ;
//         p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
//   EMA : e += ema_w * (p - e)      (ema_w = 1 - decay; 1 => plain copy)
//
// Work decomposition: the host packs a table of tensors (pointers + numel) and a
// block -> (tensor, chunk) map into one int64 device buffer; every block owns a
// kChunk-element slice of one tensor, so tiny BN vectors and 2M-element conv
// weights are load-balanced over the whole chip in a single launch.
#include "rtseg_common.h"
#include "rtseg_launch.h"

namespace rtseg {

namespace {

constexpr int kOptBlock = 256;
constexpr int kOptUnroll = 4;

// torch.lerp's two-sided formula (exact endpoint at w = 1).
__device__ __forceinline__ float lerp_like_torch(float a, float b, float w) {
  return w < 0.5f ? a + w * (b - a) : b - (b - a) * (1.f - w);
}

__global__ void __launch_bounds__(kOptBlock) fused_opt_kernel(const int64_t* meta, int ntensor,
                                                              OptHyper hp) {
  // meta layout: [ntensor x kOptMetaFields] then [nblocks x 2] (tensor, chunk start)
  const int64_t* bmap = meta + static_cast<int64_t>(ntensor) * kOptMetaFields;
  const int ti = static_cast<int>(bmap[2 * blockIdx.x]);
  const int64_t start = bmap[2 * blockIdx.x + 1];
  const int64_t* tm = meta + static_cast<int64_t>(ti) * kOptMetaFields;
  float* p = reinterpret_cast<float*>(tm[0]);
  const void* graw = reinterpret_cast<const void*>(tm[1]);
  float* m1 = reinterpret_cast<float*>(tm[2]);
  float* m2 = reinterpret_cast<float*>(tm[3]);
  float* ema = reinterpret_cast<float*>(tm[4]);
  const int64_t n = tm[5];
  const bool g_bf16 = tm[6] != 0;
  const bool first = tm[7] != 0;
  // bf16 conv-weight shadows: the layouts the MFMA conv kernels read (forward B operand, data-
  // gradient B operand), rewritten here with the parameter instead of a cast + a transpose
  // kernel per conv per step
  uint16_t* sh_krsc = reinterpret_cast<uint16_t*>(tm[8]);
  uint16_t* sh_crsk = reinterpret_cast<uint16_t*>(tm[9]);
  const int cout = static_cast<int>(tm[10]), cin = static_cast<int>(tm[11]);
  const int kh = static_cast<int>(tm[12] >> 8), kw = static_cast<int>(tm[12] & 255);
  const bool wcl = tm[13] != 0;
  int64_t end = start + kOptChunk;
  if (end > n) end = n;

  const bool sgd = hp.mode == kOptSGD;
  const bool use_m1 = !sgd || hp.momentum != 0.f;
  const bool read_m1 = use_m1 && !(sgd && first);
  for (int64_t base = start + threadIdx.x; base < end; base += kOptBlock * kOptUnroll) {
    // every operand of the kOptUnroll elements is loaded before any is used: one memory round
    // trip per iteration instead of three (parameter + gradient, then state, then the EMA copy)
    float pv[kOptUnroll], gv[kOptUnroll], av[kOptUnroll], bv[kOptUnroll], ev[kOptUnroll];
    bool ok[kOptUnroll];
#pragma unroll
    for (int u = 0; u < kOptUnroll; ++u) {
      const int64_t i = base + u * kOptBlock;
      ok[u] = i < end;
      const int64_t j = ok[u] ? i : start;  // in-range dummy address for the tail lanes
      pv[u] = p[j];
      gv[u] = g_bf16 ? bf16_to_f32(static_cast<const uint16_t*>(graw)[j]) : static_cast<const float*>(graw)[j];
      av[u] = read_m1 ? m1[j] : 0.f;
      bv[u] = sgd ? 0.f : m2[j];
      ev[u] = ema != nullptr ? ema[j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kOptUnroll; ++u) {
      if (!ok[u]) continue;
      const int64_t i = base + u * kOptBlock;
      float pp = pv[u];
      float g = gv[u] * hp.grad_scale;
      if (sgd) {
        if (hp.weight_decay != 0.f) g += hp.weight_decay * pp;
        float d = g;
        if (hp.momentum != 0.f) {
          const float b = first ? g : hp.momentum * av[u] + (1.f - hp.dampening) * g;
          m1[i] = b;
          d = hp.nesterov ? g + hp.momentum * b : b;
        }
        pp -= hp.lr * d;
      } else {
        if (hp.mode == kOptAdamW) pp *= 1.f - hp.lr * hp.weight_decay;
        else if (hp.weight_decay != 0.f) g += hp.weight_decay * pp;
        const float m = hp.beta1 * av[u] + (1.f - hp.beta1) * g;
        const float v = hp.beta2 * bv[u] + (1.f - hp.beta2) * g * g;
        m1[i] = m;
        m2[i] = v;
        const float denom = sqrtf(v) * hp.inv_sqrt_bc2 + hp.eps;
        pp -= hp.step_size * m / denom;
      }
      p[i] = pp;
      if (sh_krsc != nullptr) {
        const int ii = static_cast<int>(i);  // weights have < 2^31 elements
        int co, ci, r, q;
        if (wcl) {  // memory order [Cout][KH][KW][Cin]
          ci = ii % cin;
          int t = ii / cin;
          q = t % kw;
          t /= kw;
          r = t % kh;
          co = t / kh;
        } else {  // [Cout][Cin][KH][KW]
          q = ii % kw;
          int t = ii / kw;
          r = t % kh;
          t /= kh;
          ci = t % cin;
          co = t / cin;
        }
        const uint16_t b = f32_to_bf16(pp);
        sh_krsc[((co * kh + r) * kw + q) * cin + ci] = b;
        if (sh_crsk != nullptr) sh_crsk[((ci * kh + r) * kw + q) * cout + co] = b;
      }
      if (ema != nullptr) {
        ema[i] = lerp_like_torch(ev[u], pp, hp.ema_w);
      }
    }
  }
}

// Buffers-only EMA (BN running stats; integer counters are copied on the host side).
__global__ void __launch_bounds__(kOptBlock) ema_lerp_kernel(const int64_t* meta, int ntensor, float w) {
  const int64_t* bmap = meta + static_cast<int64_t>(ntensor) * kOptMetaFields;
  const int ti = static_cast<int>(bmap[2 * blockIdx.x]);
  const int64_t start = bmap[2 * blockIdx.x + 1];
  const int64_t* tm = meta + static_cast<int64_t>(ti) * kOptMetaFields;
  const float* src = reinterpret_cast<const float*>(tm[0]);
  float* ema = reinterpret_cast<float*>(tm[4]);
  const int64_t n = tm[5];
  int64_t end = start + kOptChunk;
  if (end > n) end = n;
  for (int64_t i = start + threadIdx.x; i < end; i += kOptBlock) {
    ema[i] = lerp_like_torch(ema[i], src[i], w);
  }
}

// Data-gradient weight shadows: crsk[ci][rq][co] = krsc[co][rq][ci] (bf16), one 64 x 64 (co, ci)
// tile of one tap per block through LDS, after the fused step wrote krsc.  Written from the
// step itself these were 2-byte stores scattered cout elements apart (0.77 ms of a 0.91 ms step
// on DDRNet-23, profiles/r4_stem); here both sides move whole 128-byte rows.
// tiles: [ntiles][6] = krsc, crsk, cout | cin << 32, taps | tap << 32, co0 | ci0 << 32, 0
__global__ void __launch_bounds__(256) shadow_crsk_kernel(const int64_t* __restrict__ tiles) {
  __shared__ uint16_t t[64][65];
  const int64_t* d = tiles + static_cast<int64_t>(blockIdx.x) * 6;
  const uint16_t* krsc = reinterpret_cast<const uint16_t*>(d[0]);
  uint16_t* crsk = reinterpret_cast<uint16_t*>(d[1]);
  const int cout = static_cast<int>(d[2] & 0xffffffff), cin = static_cast<int>(d[2] >> 32);
  const int rqn = static_cast<int>(d[3] & 0xffffffff), rq = static_cast<int>(d[3] >> 32);
  const int co0 = static_cast<int>(d[4] & 0xffffffff), ci0 = static_cast<int>(d[4] >> 32);
  const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
#pragma unroll 4
  for (int r = ly; r < 64; r += 4) {  // row r = output channel co0 + r, lanes along ci
    const int co = co0 + r, ci = ci0 + lx;
    if (co < cout && ci < cin) t[r][lx] = krsc[(static_cast<int64_t>(co) * rqn + rq) * cin + ci];
  }
  __syncthreads();
#pragma unroll 4
  for (int r = ly; r < 64; r += 4) {  // row r = input channel ci0 + r, lanes along co
    const int ci = ci0 + r, co = co0 + lx;
    if (co < cout && ci < cin) crsk[(static_cast<int64_t>(ci) * rqn + rq) * cout + co] = t[lx][r];
  }
}

}  // namespace

void launch_shadow_crsk(const int64_t* tiles, int ntiles, hipStream_t st) {
  if (ntiles <= 0) return;
  shadow_crsk_kernel<<<ntiles, 256, 0, st>>>(tiles);
}

void launch_fused_opt(const int64_t* meta, int ntensor, int nblocks, const OptHyper& hp, hipStream_t st) {
  if (nblocks <= 0) return;
  fused_opt_kernel<<<nblocks, kOptBlock, 0, st>>>(meta, ntensor, hp);
}

void launch_ema_lerp(const int64_t* meta, int ntensor, int nblocks, float w, hipStream_t st) {
  if (nblocks <= 0) return;
  ema_lerp_kernel<<<nblocks, kOptBlock, 0, st>>>(meta, ntensor, w);
}

}  // namespace rtseg
