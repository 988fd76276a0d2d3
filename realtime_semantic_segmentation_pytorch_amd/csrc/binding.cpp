// torch.library registration of the rtseg HIP operators (namespace `rtseg`).
//
// Only this translation unit sees torch headers; the kernels are called through
// the raw-pointer launchers of rtseg_launch.h. Every op is registered for the
// CUDA dispatch key (which is the HIP device on ROCm builds of PyTorch) and
// always runs on the caller's current HIP stream, so it composes with
// torch.cuda streams and graph capture.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <cmath>
#include <cstdlib>
#include <vector>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "rtseg: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

Tensor4 view4(const at::Tensor& t) {
  TORCH_CHECK(t.dim() == 4, "rtseg: expected a 4-D tensor, got ", t.dim(), "-D");
  TORCH_CHECK(t.is_cuda(), "rtseg: expected a GPU tensor");
  Tensor4 v;
  v.data = const_cast<void*>(t.data_ptr());
  v.dtype = dtype_code(t);
  v.n = static_cast<int>(t.size(0)); v.c = static_cast<int>(t.size(1));
  v.h = static_cast<int>(t.size(2)); v.w = static_cast<int>(t.size(3));
  v.sn = t.stride(0); v.sc = t.stride(1); v.sh = t.stride(2); v.sw = t.stride(3);
  return v;
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

static int act_code(int64_t a) {
  TORCH_CHECK(a >= 0 && a <= 2, "rtseg: bad activation code ", a);
  return static_cast<int>(a);
}

// ------------------------------ interp ---------------------------------------
static at::Tensor interp_fwd(const at::Tensor& x, int64_t out_h, int64_t out_w,
                             bool align_corners, const std::optional<at::Tensor>& skip,
                             int64_t act) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto fmt = x.suggest_memory_format();
  at::Tensor y = at::empty({x.size(0), x.size(1), out_h, out_w}, x.options().memory_format(fmt));
  Tensor4 xs = view4(x), ys = view4(y);
  Tensor4 ks;
  if (skip.has_value()) {
    TORCH_CHECK(skip->sizes() == y.sizes(), "rtseg.interp: skip shape mismatch");
    TORCH_CHECK(skip->scalar_type() == x.scalar_type(), "rtseg.interp: skip dtype mismatch");
    ks = view4(*skip);
  }
  launch_interp_fwd(xs, skip.has_value() ? &ks : nullptr, ys, act_code(act), align_corners,
                    cur_stream());
  return y;
}

static at::Tensor interp_bwd(const at::Tensor& g, int64_t in_h, int64_t in_w, bool align_corners,
                             bool channels_last) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  auto fmt = channels_last ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  at::Tensor gx = at::empty({g.size(0), g.size(1), in_h, in_w}, g.options().memory_format(fmt));
  const char* sep_env = std::getenv("RTSEG_INTERP_SEP");  // "0": gather-form kernels only (A/B)
  const int64_t wsn = (sep_env && sep_env[0] == '0') ? 0 : interp_bwd_ws_elems(view4(g), view4(gx));
  at::Tensor ws;
  if (wsn > 0) ws = at::empty({wsn}, g.options().dtype(at::kFloat));
  launch_interp_bwd(view4(g), view4(gx), align_corners, wsn > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  return gx;
}

static at::Tensor act_mask(const at::Tensor& g, const at::Tensor& y, int64_t act) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  TORCH_CHECK(g.sizes() == y.sizes() && g.scalar_type() == y.scalar_type(), "rtseg.act_mask: mismatch");
  // operate in y's memory order
  at::Tensor gg = g.contiguous(y.suggest_memory_format());
  TORCH_CHECK(y.is_non_overlapping_and_dense(), "rtseg.act_mask: y must be dense");
  at::Tensor out = at::empty_like(y);
  launch_act_mask(gg.data_ptr(), y.data_ptr(), out.data_ptr(), y.numel(), dtype_code(y),
                  act_code(act), cur_stream());
  return out;
}

// ------------------------------ seg loss -------------------------------------
static SegLossArgs loss_args(const at::Tensor& logits, const at::Tensor& labels, int64_t out_h,
                             int64_t out_w, bool align, int64_t ignore,
                             const std::optional<at::Tensor>& cw, int64_t mode, double thresh) {
  TORCH_CHECK(labels.dim() == 3 && labels.is_contiguous() &&
                  (labels.scalar_type() == at::kLong || labels.scalar_type() == at::kByte),
              "rtseg.seg_loss: labels must be contiguous int64 or uint8 [N,H,W]");
  TORCH_CHECK(labels.size(0) == logits.size(0), "rtseg.seg_loss: batch mismatch");
  SegLossArgs a{};
  a.logits = view4(logits);
  a.labels = labels.data_ptr();
  a.label_bytes = labels.scalar_type() == at::kByte ? 1 : 8;
  a.lh = static_cast<int>(labels.size(1));
  a.lw = static_cast<int>(labels.size(2));
  a.out_h = static_cast<int>(out_h);
  a.out_w = static_cast<int>(out_w);
  a.align_corners = align;
  a.ignore_index = static_cast<int>(ignore);
  if (cw.has_value()) {
    TORCH_CHECK(cw->scalar_type() == at::kFloat && cw->numel() == logits.size(1) && cw->is_contiguous(),
                "rtseg.seg_loss: class weights must be fp32 [C]");
    a.class_weight = cw->data_ptr<float>();
  }
  a.mode = static_cast<int>(mode);
  a.ohem_thresh = static_cast<float>(thresh);
  return a;
}

static std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> seg_loss_fwd(
    const at::Tensor& logits, const at::Tensor& labels, int64_t out_h, int64_t out_w, bool align,
    int64_t ignore, const std::optional<at::Tensor>& cw, int64_t mode, double thresh) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  SegLossArgs a = loss_args(logits, labels, out_h, out_w, align, ignore, cw, mode, thresh);
  auto f32 = logits.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({}, f32);
  at::Tensor pix_loss = at::empty({logits.size(0), out_h, out_w}, f32);
  at::Tensor pix_lse = at::empty({logits.size(0), out_h, out_w}, f32);
  at::Tensor stats = at::empty({32}, logits.options().dtype(at::kDouble));
  at::Tensor hist = at::empty({3 * 2048}, logits.options().dtype(at::kInt));
  at::Tensor slab = at::empty({static_cast<int64_t>(seg_loss_fwd_blocks(a)) * 5},
                              logits.options().dtype(at::kDouble));
  a.slab = slab.data_ptr<double>();
  a.pix_loss = pix_loss.data_ptr<float>();
  a.pix_lse = pix_lse.data_ptr<float>();
  a.stats = stats.data_ptr<double>();
  a.hist = reinterpret_cast<unsigned*>(hist.data_ptr<int>());
  a.out_loss = loss.data_ptr<float>();
  launch_seg_loss_fwd(a, cur_stream());
  return {loss, pix_loss, pix_lse, stats};
}

static at::Tensor seg_loss_bwd(const at::Tensor& grad, const at::Tensor& logits,
                               const at::Tensor& labels, const at::Tensor& pix_loss,
                               const at::Tensor& pix_lse, const at::Tensor& stats, int64_t out_h,
                               int64_t out_w, bool align, int64_t ignore,
                               const std::optional<at::Tensor>& cw, int64_t mode) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  SegLossArgs a = loss_args(logits, labels, out_h, out_w, align, ignore, cw, mode, 0.0);
  a.pix_loss = const_cast<float*>(pix_loss.data_ptr<float>());
  a.pix_lse = const_cast<float*>(pix_lse.data_ptr<float>());
  a.stats = const_cast<double*>(stats.data_ptr<double>());
  at::Tensor g32 = grad.to(at::kFloat).contiguous();
  at::Tensor gl = at::empty(logits.sizes(), logits.options().memory_format(logits.suggest_memory_format()));
  at::Tensor acc;
  if (!(out_h == logits.size(2) && out_w == logits.size(3))) {
    acc = at::empty_like(gl, gl.options().dtype(at::kFloat));
    TORCH_CHECK(acc.strides() == gl.strides() && gl.is_non_overlapping_and_dense(),
                "rtseg.seg_loss_bwd: accumulator layout mismatch");
    a.acc = acc.data_ptr<float>();
    a.acc_sn = acc.stride(0); a.acc_sc = acc.stride(1);
    a.acc_sh = acc.stride(2); a.acc_sw = acc.stride(3);
  }
  launch_seg_loss_bwd(a, g32.data_ptr<float>(), view4(gl), cur_stream());
  return gl;
}

}  // namespace rtseg

TORCH_LIBRARY(rtseg, m) {
  m.def("interp(Tensor x, int out_h, int out_w, bool align_corners, Tensor? skip, int act) -> Tensor");
  m.def("interp_backward(Tensor grad, int in_h, int in_w, bool align_corners, bool channels_last) -> Tensor");
  m.def("act_mask(Tensor grad, Tensor y, int act) -> Tensor");
  m.def("seg_loss_fwd(Tensor logits, Tensor labels, int out_h, int out_w, bool align_corners, "
        "int ignore_index, Tensor? class_weight, int mode, float thresh) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("seg_loss_bwd(Tensor grad, Tensor logits, Tensor labels, Tensor pix_loss, Tensor pix_lse, "
        "Tensor stats, int out_h, int out_w, bool align_corners, int ignore_index, Tensor? class_weight, "
        "int mode) -> Tensor");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("interp", &rtseg::interp_fwd);
  m.impl("interp_backward", &rtseg::interp_bwd);
  m.impl("act_mask", &rtseg::act_mask);
  m.impl("seg_loss_fwd", &rtseg::seg_loss_fwd);
  m.impl("seg_loss_bwd", &rtseg::seg_loss_bwd);
}
