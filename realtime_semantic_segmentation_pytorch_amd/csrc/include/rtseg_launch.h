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
void launch_interp_bwd(const Tensor4& g, const Tensor4& gx, bool align_corners, hipStream_t st);
void launch_act_mask(const void* g, const void* y, void* out, int64_t n, int dtype, int act,
                     hipStream_t st);

// ---- seg_loss.hip -----------------------------------------------------------
// Per-pixel cross-entropy of (bilinearly resized) logits against (nearest
// resized) labels, plus OHEM / mean selection entirely on device.
struct SegLossArgs {
  Tensor4 logits;        // [N, C, h, w] (any strides)
  const int64_t* labels; // [N, LH, LW] contiguous
  int lh, lw;
  int out_h, out_w;      // loss is evaluated on this grid (== label grid normally)
  bool align_corners;
  int ignore_index;
  const float* class_weight;  // [C] or nullptr
  float* pix_loss;       // [N, out_h, out_w] fp32 workspace
  float* pix_lse;        // [N, out_h, out_w] fp32 workspace (log-sum-exp per pixel)
  double* stats;         // kSegStats device scalars, see seg_loss.hip
  unsigned* hist;        // 3 x 2048 radix-select histogram workspace
  float* acc;            // [N, C, h, w] fp32 backward accumulator (upsample path)
  int mode;              // 0 = OHEM, 1 = weighted mean CE, 2 = sum CE
  float ohem_thresh;     // -log(p)
  float* out_loss;       // scalar
};
void launch_seg_loss_fwd(const SegLossArgs& a, hipStream_t st);
// grad_logits (fp32, layout of grad tensor given) = grad_scale * d loss / d logits
void launch_seg_loss_bwd(const SegLossArgs& a, const float* grad_out, const Tensor4& grad_logits,
                         hipStream_t st);

}  // namespace rtseg
