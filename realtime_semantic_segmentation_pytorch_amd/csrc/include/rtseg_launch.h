// Host-side launcher interface between csrc/binding.cpp (torch tensors) and
// the kernel translation units (raw pointers). Kept free of torch headers.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <type_traits>

namespace rtseg {

// A strided 4-D view (N, C, H, W) with element strides.
struct Tensor4 {
  void* data;
  int dtype;  // rtseg::DType
  int n, c, h, w;
  int64_t sn, sc, sh, sw;
};

// ---- interp.hip -------------------------------------------------------------
void launch_interp_fwd(const Tensor4& x, const Tensor4* skip, const Tensor4& y, int act,
                       bool align_corners, hipStream_t st);
// ws: fp32 workspace of interp_bwd_ws_elems(g, gx) elements (separable path for large
// up-scaling), or nullptr when that returns 0
int64_t interp_bwd_ws_elems(const Tensor4& g, const Tensor4& gx);
void launch_interp_bwd(const Tensor4& g, const Tensor4& gx, bool align_corners, float* ws, hipStream_t st);
void launch_act_mask(const void* g, const void* y, void* out, int64_t n, int dtype, int act,
                     hipStream_t st);

// ---- seg_loss.hip -----------------------------------------------------------
// Per-pixel cross-entropy of (bilinearly resized) logits against (nearest
// resized) labels, plus OHEM / mean selection entirely on device.
struct SegLossArgs {
  Tensor4 logits;        // [N, C, h, w] (any strides)
  const void* labels;    // [N, LH, LW] contiguous, int64 or uint8
  int label_bytes;       // 8 or 1
  int lh, lw;
  int out_h, out_w;      // loss is evaluated on this grid (== label grid normally)
  bool align_corners;
  int ignore_index;
  const float* class_weight;  // [C] or nullptr
  float* pix_loss;       // [N, out_h, out_w] fp32 workspace
  float* pix_lse;        // [N, out_h, out_w] fp32 workspace (log-sum-exp per pixel)
  double* stats;         // kSegStats device scalars, see seg_loss.hip
  double* slab;          // [seg_loss_fwd_blocks, 5] per-tile partial statistics
  unsigned* hist;        // 3 x 2048 radix-select histogram workspace
  float* acc;            // fp32 backward accumulator (upsample path), strides of the gradient
  int64_t acc_sn, acc_sc, acc_sh, acc_sw;
  int mode;              // 0 = OHEM, 1 = weighted mean CE, 2 = sum CE
  float ohem_thresh;     // -log(p)
  float* out_loss;       // scalar
};
int seg_loss_fwd_blocks(const SegLossArgs& a);
void launch_seg_loss_fwd(const SegLossArgs& a, hipStream_t st);
// grad_logits (fp32, layout of grad tensor given) = grad_scale * d loss / d logits
void launch_seg_loss_bwd(const SegLossArgs& a, const float* grad_out, const Tensor4& grad_logits,
                         hipStream_t st);

// ---- bn_act.hip --------------------------------------------------------------
// x is [M, C] row-major (channels-last). Partial slabs are [G, 2C] fp32
// (G = bn_partial_grid); sums are [2C+1] fp64 (sum, second moment, count).
// launch_bn_stats writes a [G + 1, 2C] slab of moments shifted by a per-channel pivot
// (row G, first C floats); the reducers take that row as ``pivot`` (nullptr: raw moments,
// e.g. a conv-epilogue slab).
int bn_partial_grid(int64_t M, int C, int dtype);
// Channel-vector width used for (dtype, C); 0 = layer not supported by the fused kernels.
int bn_vec_width(int dtype, int C);
void launch_bn_stats(const void* x, int dtype, int64_t M, int C, float* part, int G, hipStream_t st,
                     bool shift = true);
void launch_bn_finalize_partials(const float* part, int G, int C, double count, const float* w,
                                 const float* b, float* rmean, float* rvar, int64_t* nbt,
                                 float momentum, float eps, float* mean_invstd, float* scale_shift,
                                 double* sums_out, hipStream_t st, const float* pivot = nullptr,
                                 double* scratch = nullptr);
void launch_bn_slab_to_sums(const float* part, int G, int C, double count, double* sums,
                            hipStream_t st, const float* pivot = nullptr, double* scratch = nullptr);
// Row splits of a G-row statistics slab the finalize launchers pre-reduce when given a scratch of
// bn_slab_splits(G) * 2C doubles (1: no pre-pass, no scratch needed).
int bn_slab_splits(int G);
void launch_bn_finalize(const double* sums, int C, const float* w, const float* b, float* rmean,
                        float* rvar, int64_t* nbt, float momentum, float eps, float* mean_invstd,
                        float* scale_shift, hipStream_t st);
void launch_bn_eval_coeffs(int C, const float* w, const float* b, const float* rmean,
                           const float* rvar, float eps, float* mean_invstd, float* scale_shift,
                           hipStream_t st);
// y2 / dy2 (channel-stationary path only, bn_flat(dtype, C) false): a channel slice of a wider
// channels-last tensor with row stride ld2 elements -- the concat buffer (ops/concat.py).  The
// apply kernels also store the output there; the backward kernels add it to dy (dy may be null).
void launch_bn_apply_bits(const void* x, const void* res, const float* scale_shift, void* y,
                          uint8_t* bits, int dtype, int64_t M, int C, int act, hipStream_t st,
                          void* y2 = nullptr, int64_t ld2 = 0);
void launch_bn_apply(const void* x, const void* res, const float* scale_shift, void* y, int dtype,
                     int64_t M, int C, int act, hipStream_t st, void* y2 = nullptr, int64_t ld2 = 0);
void launch_bn_bwd_reduce(const void* dy, const void* x, const void* y, const float* mean_invstd,
                          const float* scale_shift, int dtype, int64_t M, int C, int act, int mask,
                          float* part, int G, hipStream_t st, const void* dy2 = nullptr, int64_t ld2 = 0);
void launch_bn_bwd_finalize(const float* part, int G, const double* sums, const double* count_ptr,
                            int C, const float* w, const float* mean_invstd, int batch_stats,
                            float* kcoef, float* dw, float* db, hipStream_t st, double* scratch = nullptr);
void launch_bn_bwd_apply(const void* dy, const void* x, const void* y, const float* mean_invstd,
                         const float* scale_shift, const float* kcoef, void* dx, void* dres,
                         int dtype, int64_t M, int C, int act, int mask, hipStream_t st,
                         const void* dy2 = nullptr, int64_t ld2 = 0);


// ---- kd_metrics.hip ---------------------------------------------------------
int kd_partial_blocks(int64_t npix);
// lse: [2, N*H*W] fp32 (student, teacher log-sum-exp of z/T); part: [kd_partial_blocks] fp64
// KD with the student's final bilinear upsample folded in: s_lo [N][Hl][Wl][C] at head resolution,
// t (and gs) at full resolution, dense channels-last; kd_fold_ok(s_lo, t) first
bool kd_fold_ok(const Tensor4& s_lo, const Tensor4& t);
void launch_kd_fwd_fold(const Tensor4& s_lo, const Tensor4& t, bool align, float temperature, float* lse, double* part,
                        float* out, hipStream_t st);
void launch_kd_bwd_fold(const Tensor4& s_lo, const Tensor4& t, const Tensor4& gs, bool align, float temperature,
                        const float* lse, const float* gout, hipStream_t st);
void launch_kd_fwd(const Tensor4& s, const Tensor4& t, float temperature, float* lse, double* part,
                   float* out, hipStream_t st);
void launch_kd_bwd(const Tensor4& s, const Tensor4& t, const Tensor4& gs, float temperature,
                   const float* lse, const float* gout, hipStream_t st);
// cm: [C, C] uint64 (accumulated, caller zeroes), target: [N, H, W] int64 contiguous
void launch_confmat(const Tensor4& x, const int64_t* target, int ignore, unsigned long long* cm,
                    hipStream_t st);

// ---- optim.hip --------------------------------------------------------------
// Tensor table row: {param f32*, grad*, state1 f32*, state2 f32*, ema f32*, numel, grad_is_bf16,
// first_step}; followed by a [nblocks, 2] (tensor, chunk-start) map.
// per tensor: param, grad, state1, state2, ema, numel, grad_bf16, first_step, then the optional bf16
// conv-weight shadows written with the updated parameter (ops/conv.py weight_shadow): krsc
// [Cout][KH][KW][Cin], crsk [Cin][KH][KW][Cout], Cout, Cin, KH * 256 + KW, parameter channels-last
constexpr int kOptMetaFields = 14;
constexpr int64_t kOptChunk = 16384;
enum OptMode : int { kOptSGD = 0, kOptAdam = 1, kOptAdamW = 2 };
struct OptHyper {
  int mode;
  float lr, momentum, dampening, weight_decay;
  int nesterov;
  float beta1, beta2, eps, step_size, inv_sqrt_bc2;
  float grad_scale;
  float ema_w;  // 1 - decay (1 => copy)
};
void launch_fused_opt(const int64_t* meta, int ntensor, int nblocks, const OptHyper& hp, hipStream_t st);
void launch_ema_lerp(const int64_t* meta, int ntensor, int nblocks, float w, hipStream_t st);
// crsk[ci][rq][co] = krsc[co][rq][ci] for a table of 64 x 64 tiles (6 int64 each, optim.hip)
void launch_shadow_crsk(const int64_t* tiles, int ntiles, hipStream_t st);

// ---- dwconv.hip -------------------------------------------------------------
// Depth-wise conv geometry; activations channels-last, weights tap-major fp32 [KH*KW][Cout].
struct DwGeom {
  int n, h, w, cin, cout, mult;  // mult = cout / cin
  int ho, wo, kh, kw, sh, sw, ph, pw, dh, dw;
  int act = 0;  // forward: activation after the bias (0 none, 1 ReLU, 2 ReLU6; an eval BN folded in)
};
struct DwWgradPlan {
  int vec, lanes, chunks, nt, tap_groups, slices;  // nt = taps per wgrad thread
  int pairs = 0;  // 1: the channel-multiplier kernel (bf16, mult 2/3/4/6): threads own input-channel pairs
  int quad = 0;   // 1: plain 3 x 3 stride-1 kernel over 4-pixel row segments (dw_wgrad_quad_kernel)
};
int dw_vec(int dtype, int c);
DwWgradPlan dw_wgrad_plan(const DwGeom& g, int dtype);
// forward + BN statistics slab (fp32 [rows, 2*Cout]); rows = dw_fwd_stats_rows (0: unsupported
// channel multiplier -> use launch_dw_fwd + a statistics pass)
int dw_fwd_stats_rows(const DwGeom& g, int dtype);
void launch_dw_fwd_stats(const DwGeom& g, int dtype, const void* x, const float* wt, void* y, float* part,
                         hipStream_t st);
void launch_dw_fwd(const DwGeom& g, int dtype, const void* x, const float* wt, const float* bias, void* y,
                   hipStream_t st);
void launch_dw_dgrad(const DwGeom& g, int dtype, const void* dy, const float* wt, void* dx, hipStream_t st);
// part: [slices, KH*KW, Cout] fp32 workspace; dw: [Cout, KH*KW] fp32
void launch_dw_wgrad(const DwGeom& g, int dtype, const void* dy, const void* x, float* part, float* dw,
                     hipStream_t st);

// ---- conv_mfma.hip ------------------------------------------------------------
// Implicit-GEMM conv, bf16 NHWC: x [N,H,W,Cin], w [Cout,KH,KW,Cin], y [N,Ho,Wo,Cout].
// part != nullptr: BN statistics slab [conv_mfma_slabs(g), 2*Cout] fp32 (sum | sum of squares).
// scale_shift != nullptr: y = act(conv * scale + shift (+ res)) (inference BN epilogue).
struct ConvGeom {
  const void* x;
  const void* w;
  void* y;
  float* part;
  const float* scale_shift;
  const void* res;
  int act;
  int n, h, w_in, cin, ho, wo, cout, kh, kw, sh, sw, ph, pw, dh, dw;
  const uint8_t* amask = nullptr;  // data gradient: bit mask of the addend (res), see mask_addend4
  // igemm data gradient: a second addend indexed by the pixels of output phase (0, 0) (the even
  // rows / columns of a stride-2 dx, [N][ceil(H/2)][ceil(W/2)][Cin]): the data gradient of a
  // stride-2 1 x 1 shortcut on the same input, computed as a plain GEMM (ops/conv.py _TwinConvFn)
  const void* res_phase0 = nullptr;
  // igemm forward: a forced block-tile configuration (conv_igemm.hip kCfgs), -1 = by shape
  int cfg = -1;
};
// BN activation-derivative sources (= ops/bn.py MASK_*)
enum BnMaskMode : int { kBnMaskNone = 0, kBnMaskFromY = 1, kBnMaskFromX = 2, kBnMaskBits = 3 };
int conv_mfma_slabs(const ConvGeom& g);
void launch_conv_mfma(const ConvGeom& g, hipStream_t st);

// ---- conv_igemm.hip -----------------------------------------------------------
// 32x32x16-MFMA implicit-GEMM conv family (ConvGeom always describes the FORWARD conv).
// mode 0 = forward, 1 = data gradient, 2 = weight gradient.
constexpr int kIgemmMaxTaps = 49;
bool conv_igemm_supported(const ConvGeom& g, int mode);
// batch-1 inference forward split over K: parts (1 = no split) and the launch (fp32 workspace of
// parts * N * Ho * Wo * Cout floats; g.scale_shift required, g.res / g.act applied after the sum)
int conv_igemm_splitk(const ConvGeom& g);
void launch_conv_igemm_fwd_splitk(const ConvGeom& g, float* ws, int ksplit, hipStream_t st);
// rows of the BN statistics slab [rows, 2*Cout] written by the forward when g.part != nullptr
// (one per M tile and pixel wave); launch_slab_compact sums groups of `chunk` rows
int conv_igemm_slabs(const ConvGeom& g);
void launch_slab_compact(const float* in, int rows, int width, int chunk, float* out, hipStream_t st);
void launch_conv_igemm_fwd(const ConvGeom& g, hipStream_t st);
// g.x = dy [N,Ho,Wo,Cout], g.w = [Cin][KH][KW][Cout] bf16, g.y = dx [N,H,W,Cin];
// g.scale_shift, when set, is a [Cin] bias added to dx (the forward of a transposed conv);
// g.res, when set, is a bf16 tensor of dx's layout added to dx (a residual branch's gradient);
void launch_conv_igemm_dgrad(const ConvGeom& g, hipStream_t st);
// the same data gradient of a strided conv with every output phase in ONE launch (padding taps
// even out the phases' tap counts); needs H % sh == 0, W % sw == 0 -- conv_igemm_dgrad_fused_ok
bool conv_igemm_dgrad_fused_ok(const ConvGeom& g);
void launch_conv_igemm_dgrad_fused(const ConvGeom& g, hipStream_t st);
// g.x = x [N,H,W,Cin], g.y = dy [N,Ho,Wo,Cout]; ws fp32 of conv_igemm_wgrad_ws_elems(g);
// dw fp32 [Cout][Cin][KH][KW]
int64_t conv_igemm_wgrad_ws_elems(const ConvGeom& g);
void launch_conv_igemm_wgrad(const ConvGeom& g, float* ws, float* dw, bool krsc, hipStream_t st);
// split-K slab [splits][cout][kt * cin] -> dw (NCHW or, krsc, [Cout][KH][KW][Cin] order)
void launch_wgrad_slab_reduce(float* ws, int splits, int cout, int cin, int kt, float* dw, bool krsc,
                              hipStream_t st);

// ---- conv_halo.hip ------------------------------------------------------------
// Halo-tiled stride-1 conv (taps within a 3 x 3 footprint, Cin % 64 == 0, Cout % 64 == 0):
// forward (+ BN statistics slab of conv_halo_slabs(g) rows / inference BN epilogue) and data
// gradient (g as for launch_conv_igemm_dgrad; g.res = optional addend).  mode 0 fwd, 1 dgrad.
bool conv_halo_supported(const ConvGeom& g, int mode);
int conv_halo_slabs(const ConvGeom& g);
void launch_conv_halo_fwd(const ConvGeom& g, hipStream_t st);
void launch_conv_halo_dgrad(const ConvGeom& g, hipStream_t st);

// ---- conv_wres.hip ------------------------------------------------------------
// Weights-resident halo conv: 3 x 3, stride 1, pad 1, dilation 1, 64 reduction channels
// (forward: Cin == 64; data gradient: Cout == 64), output channels % 64 == 0; forward (+ BN
// statistics slab of conv_wres_slabs(g) rows) and data gradient (g.res = optional addend).
bool conv_wres_supported(const ConvGeom& g, int mode);
int conv_wres_slabs(const ConvGeom& g);
void launch_conv_wres_fwd(const ConvGeom& g, hipStream_t st);
void launch_conv_wres_dgrad(const ConvGeom& g, hipStream_t st);

// ---- conv_hreg.hip ------------------------------------------------------------
// Halo-tiled 3 x 3 / stride 1 / pad 1 conv with register-streamed weights: reduction channels
// % 64 == 0, output channels % 128 == 0.  mode 0 forward (+ BN statistics slab of
// conv_hreg_slabs(g) rows), 1 data gradient (g as for launch_conv_igemm_dgrad, g.res = addend);
// wpack: scratch of conv_hreg_pack_elems(g, mode) bf16.
bool conv_hreg_supported(const ConvGeom& g, int mode);
int conv_hreg_slabs(const ConvGeom& g);
int64_t conv_hreg_pack_elems(const ConvGeom& g, int mode);
// layout: 1 = 8 waves of 2 x 2 accumulator tiles, 2 = 4 waves of 2 x 4, 4 = 8 waves of 1 x 4
void launch_conv_hreg(const ConvGeom& g, int mode, void* wpack, hipStream_t st, int layout = 1);

// ---- conv_stem.hip ------------------------------------------------------------
// 3-channel 3 x 3 stem conv (pad 1, stride 1 / 2, Cout % 16 == 0 and <= 64, even W): forward
// (+ BN statistics slab of conv_stem_slabs(g) rows) and weight gradient (g.x = x, g.y = dy).
bool conv_stem_supported(const ConvGeom& g);
// 7 x 7 / pad 3 / stride 1 or 2 stem (conv_stem7.hip): Cin 3, Cout % 16 <= 64, even W; forward with
// an optional inference BN (+ act) epilogue (g.scale_shift, g.act)
bool conv_stem7_supported(const ConvGeom& g);
void launch_conv_stem7_fwd(const ConvGeom& g, hipStream_t st);
int conv_stem_slabs(const ConvGeom& g);
// stem BN backward reduction with the conv recomputed from the image (g.y = the BN output's gradient)
void launch_conv_stem_bn_sums(const ConvGeom& g, const float* mean_invstd, const float* scale_shift, int act,
                              float* part, hipStream_t st);
void launch_conv_stem_fwd(const ConvGeom& g, hipStream_t st);
int64_t conv_stem_wgrad_ws_elems(const ConvGeom& g);
// BN-fused weight gradient: g.y is the gradient of act(BN(conv output)); the BN backward's apply
// pass (dx = k0 (g - k1 - (xb - mean) k2), g masked by act'(xb * sc + sh)) runs in the dy staging.
// act: 0 none, 1 ReLU, 2 ReLU6.  Cout of 16, 32 or 64.
struct StemBnBwd {
  const void* xb;           // the BN input (the conv output), or null with w set
  const float* kcoef;
  const float* mean_invstd;
  const float* scale_shift;
  int act;
  const void* w = nullptr;  // KRSC stem weights: recompute the BN input from the image instead
};
void launch_conv_stem_wgrad(const ConvGeom& g, float* ws, float* dw, bool krsc, hipStream_t st,
                            const StemBnBwd* bn = nullptr);

// ---- conv_whalo.hip -----------------------------------------------------------
// Halo-tiled weight gradient of 3 x 3 / stride 1 / pad 1 / dilation 1 convs (Cin, Cout % 64 == 0):
// g.x = x, g.y = dy; ws of conv_whalo_ws_elems(g) floats; dw fp32 as launch_conv_igemm_wgrad.
bool conv_whalo_supported(const ConvGeom& g);
int64_t conv_whalo_ws_elems(const ConvGeom& g);
// variant 1: one output tile per wave; 2: both output tiles per wave, K split across wave halves
void launch_conv_whalo_wgrad(const ConvGeom& g, float* ws, float* dw, bool krsc, hipStream_t st, int variant = 1);

// ---- gate.hip -----------------------------------------------------------------
// out = x * s (mul), x * (1 + s) (residual), x * s + y * (1 - s) (blend); s = att or
// sigmoid(att), broadcast per (n, c) (att fp32 [N, C]), per pixel (fp32 [N, H*W]) or full (x's
// dtype and layout).  x / y / out channels-last [M = N*H*W][C].
enum GateMode : int { kGateMul = 0, kGateResidual = 1, kGateBlend = 2 };
enum GateBcast : int { kGateChannel = 0, kGateSpatial = 1, kGateFull = 2 };
struct GateArgs {
  const void* x;
  const void* y;
  const void* att;
  void* out;
  int dtype, mode, bc;
  bool sigmoid;
  int64_t M;
  int HW, C;
};
int gate_vec_width(int dtype, int C);  // 0: unsupported channel count
bool gate_bwd_supported(int dtype, int C, int bc);
int gate_channel_blocks(int64_t HW, int N);  // part: fp32 [N, blocks, C] for the channel gate
void launch_gate_fwd(const GateArgs& g, hipStream_t st);
void launch_gate_bwd(const GateArgs& g, const void* go, void* gx, void* gy, void* gatt, float* part, hipStream_t st);

// ---- pool.hip -----------------------------------------------------------------
enum PoolMode : int { kPoolAvg = 0, kPoolMax = 1 };
struct PoolParams {
  int kh, kw, sh, sw, ph, pw;
  int count_include_pad;  // avg: divisor over the padded window (ATen default)
  int mode;               // PoolMode
  int adaptive;           // avg only: ATen adaptive windows from the input/output sizes
};
// max pooling writes idx: dense NHWC uint8 [N, OH, OW, C] window offsets (kh*kw <= 256)
void launch_pool_fwd(const Tensor4& x, const Tensor4& y, const PoolParams& p, uint8_t* idx, hipStream_t st);
void launch_pool_bwd(const Tensor4& gy, const Tensor4& gx, const PoolParams& p, const uint8_t* idx, hipStream_t st);
struct GapPlan {
  int vec, cpb, cblocks, per_slice, slices;
};
GapPlan gap_plan(const Tensor4& x);
// indexed max pool / max unpool (int64 flat plane indices, PyTorch's convention); idx is a
// Tensor4 view of an int64 tensor (its dtype field is ignored)
void launch_unpool_gather(const Tensor4& x, const Tensor4& idx, const Tensor4& y, int kh, int kw, hipStream_t st);
void launch_unpool_bwd(const Tensor4& gy, const Tensor4& idx, const Tensor4& gx, hipStream_t st);
void launch_maxpool_flat_index(const uint8_t* win, const Tensor4& out, int in_w, const PoolParams& p,
                               hipStream_t st);
// global max pool (AdaptiveMaxPool2d(1)) with first-max int64 argmax: y dense [N, C], idx [N, C]
void launch_global_max(const Tensor4& x, void* y, int64_t* idx, hipStream_t st);
// global average pool; part: fp32 workspace of plan.slices * N * C
void launch_gap_fwd(const Tensor4& x, const Tensor4& y, const GapPlan& plan, float* part, hipStream_t st);

// ---- detail_loss.hip ----------------------------------------------------------
// STDC detail loss: d = low-resolution detail logits [N,1,h,w]; labels [N,H,W] uint8 or int64;
// wb = detail_conv (w0, w1, w2, bias) fp32 on device.  part: fp64 [N * detail_loss_blocks * 4],
// sums: fp64 [N, 4], yout: uint8 [N, H, W] binary target, out: fp32 scalar loss.
int detail_loss_blocks(int n, int h, int w);
void launch_detail_fwd(const Tensor4& d, const void* labels, bool labels_u8, int n, int h, int w, const float* wb,
                       float thrs, float dice_coef, float bce_coef, uint8_t* yout, double* part, double* sums,
                       float* out, hipStream_t st);
// gp: fp32 [N, H, W] = dL/d(upsampled logits)
void launch_detail_bwd(const Tensor4& d, int n, int h, int w, const uint8_t* yin, const double* sums,
                       const float* gout, float dice_coef, float bce_coef, float* gp, hipStream_t st);

// ---- colorize.hip -------------------------------------------------------------
// argmax over C of x [N,C,H,W] -> cls uint8 [N,H,W] (C <= 256), rgb = lut[cls] uint8 [N,H,W,3],
// blend = trunc(img + alpha * (rgb - img)) in fp32 (bit-identical to PIL Image.blend) with img uint8 [N,H,W,3]; null outputs are skipped.
void launch_colorize(const Tensor4& x, const uint8_t* lut, const uint8_t* img, float alpha, uint8_t* cls,
                     uint8_t* rgb, uint8_t* blend, hipStream_t st);

// ---- tapconv.hip --------------------------------------------------------------
// Same-padded stride-1 1-D conv with K <= kTapConvMaxTaps taps, dilation dil, along H (axis 0)
// or W (axis 1) of channels-last x [N, H, W, ci] -> y [N, H, W, co]; ci, co in {4, 8, 16};
// w fp32 [K, ci, co]; bias fp32 [co] or nullptr.  tap_stride: pixels between taps / dil.
constexpr int kTapConvMaxTaps = 7;
struct TapConvGeo {
  int n, h, w, k, dil, axis;
  int64_t tap_stride;
};
void launch_tapconv(const void* x, const float* w, const float* bias, void* y, const TapConvGeo& g, int ci, int co,
                    int dtype, hipStream_t st);

// ---- augment.hip --------------------------------------------------------------
// Per-sample parameter row (fp32 [N, kAugParams]): scaled size, centred-pad offsets, crop origin,
// flip, jitter op count + order code (2 bits per op: 0 brightness, 1 contrast, 2 saturation,
// 3 hue), jitter factors.  Drawn on the host by ops/augment.py.
enum AugParam : int {
  kAugNh = 0, kAugNw, kAugTop, kAugLeft, kAugCy, kAugCx, kAugFlip, kAugNops, kAugCode,
  kAugBright, kAugContrast, kAugSat, kAugHue, kAugParams
};
struct AugArgs {
  const uint8_t* img;     // [N, H, W, 3] uint8
  const uint8_t* msk;     // [N, H, W] uint8 raw labels, or null
  const float* params;    // [N, kAugParams]
  const uint8_t* lut;     // [256] raw label -> training label
  const float* norm;      // [6] mean[3], std[3] (on [0, 1] pixels)
  float* part;            // [N, augment_stat_blocks] contrast statistics workspace, or null
  Tensor4 out;            // [N, 3, ch, cw] fp32 / bf16 / fp16, any strides
  void* mout;             // [N, ch, cw] int64 or uint8, or null
  int mask_bytes;
  int n, h, w, ch, cw;
  float pad_value;
  int mask_pad;
};
int augment_stat_blocks(int ch, int cw);
void launch_augment(const AugArgs& a, hipStream_t st);

// ---- act.hip ------------------------------------------------------------------
enum ActKind : int {
  kActPReLU = 0, kActLeaky, kActELU, kActCELU, kActSELU, kActHardswish, kActHardtanh, kActSiLU,
  kActSigmoid, kActTanh, kActGELU, kActGELUTanh
};
// forward: out = f(x); backward (bwd): out = dx = dy * f'(x).  PReLU with a weight tensor w
// (C = 1 for a scalar slope): channel of element i = (i / inner) % C (inner = 1: channels-last
// or flat; inner = H*W: contiguous NCHW); its backward also writes dw [C] through `part`
// (act_prelu_plan(a).blocks * C floats, or blocks floats in planes mode).  Other kinds: slope /
// alpha / min in `a`, max in `b`.
struct ActArgs {
  const void* x;
  const void* dy;
  void* out;
  const float* w;
  float* part;
  float* dw;
  int dtype, kind;
  bool bwd;
  int64_t n;
  int C;
  int64_t inner;
  float a, b;
  // forward of a per-channel PReLU only: an eval BN's scale [C] | shift [C] applied first, so
  // BN + PReLU of inference is one pass (ops/bn.py bn_act), or null
  const float* ss = nullptr;
};
struct ActPreluPlan {
  bool planes;
  int blocks, slices, tx, vec;  // vec: channels per lane (16-byte vectors) in rows mode
  int64_t rows_per_block;
};
ActPreluPlan act_prelu_plan(const ActArgs& a);
void launch_act(const ActArgs& a, hipStream_t st);

// ---- shuffle.hip --------------------------------------------------------------
// out (contiguous NCHW, or channels-last when out_cl) <- remap of in (any strides):
// kShufPixel: PixelShuffle(r); kShufPixelInv: PixelUnshuffle(r); kShufChannel: channel shuffle
// with r groups.  fp32 / bf16 / fp16.
enum ShufMode : int { kShufPixel = 0, kShufPixelInv = 1, kShufChannel = 2 };
void launch_shuffle(const Tensor4& in, const Tensor4& out, int mode, int r, bool out_cl, hipStream_t st);

}  // namespace rtseg
