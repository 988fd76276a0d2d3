// torch.library registration of the KD-loss, confusion-matrix and fused
// optimizer/EMA operators (kernels: kd_metrics.hip, optim.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

static void check_pair(const at::Tensor& s, const at::Tensor& t) {
  TORCH_CHECK(s.dim() == 4 && t.dim() == 4 && s.sizes() == t.sizes(),
              "rtseg.kd: student/teacher logits must both be [N,C,H,W] of equal shape");
  TORCH_CHECK(s.scalar_type() == t.scalar_type(), "rtseg.kd: student/teacher dtype mismatch");
  TORCH_CHECK(s.is_cuda() && t.is_cuda() && s.device() == t.device(), "rtseg.kd: tensors on different devices");
}

// -> (loss scalar fp32, lse [2, N*H*W] fp32)
static std::tuple<at::Tensor, at::Tensor> kd_kl_fwd(const at::Tensor& s, const at::Tensor& t, double temperature) {
  check_pair(s, t);
  TORCH_CHECK(temperature > 0.0, "rtseg.kd: temperature must be > 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(s.device());
  const int64_t npix = s.size(0) * s.size(2) * s.size(3);
  auto f32 = s.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({}, f32);
  at::Tensor lse = at::empty({2, npix}, f32);
  at::Tensor part = at::empty({kd_partial_blocks(npix)}, s.options().dtype(at::kDouble));
  launch_kd_fwd(view4(s), view4(t), static_cast<float>(temperature), lse.data_ptr<float>(),
                part.data_ptr<double>(), loss.data_ptr<float>(), cur_stream());
  return {loss, lse};
}

static at::Tensor kd_kl_bwd(const at::Tensor& grad, const at::Tensor& s, const at::Tensor& t,
                            const at::Tensor& lse, double temperature) {
  check_pair(s, t);
  c10::hip::HIPGuardMasqueradingAsCUDA g(s.device());
  const int64_t npix = s.size(0) * s.size(2) * s.size(3);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == 2 * npix,
              "rtseg.kd_bwd: bad lse workspace");
  at::Tensor g32 = grad.to(at::kFloat).contiguous();
  at::Tensor gs = at::empty(s.sizes(), s.options().memory_format(s.suggest_memory_format()));
  launch_kd_bwd(view4(s), view4(t), view4(gs), static_cast<float>(temperature), lse.data_ptr<float>(),
                g32.data_ptr<float>(), cur_stream());
  return gs;
}

// KD with the student's final upsample folded in: s_lo at head resolution, t at full resolution
static std::tuple<at::Tensor, at::Tensor> kd_kl_fwd_fold(const at::Tensor& s_lo, const at::Tensor& t,
                                                         double temperature, bool align_corners) {
  TORCH_CHECK(s_lo.is_cuda() && t.is_cuda() && s_lo.dim() == 4 && t.dim() == 4, "rtseg.kd_fold: 4-D GPU tensors");
  TORCH_CHECK(temperature > 0.0, "rtseg.kd: temperature must be > 0");
  TORCH_CHECK(kd_fold_ok(view4(s_lo), view4(t)), "rtseg.kd_fold: needs dense channels-last, 16-byte aligned "
              "tensors of one dtype with the same batch and channels");
  c10::hip::HIPGuardMasqueradingAsCUDA g(t.device());
  const int64_t npix = t.size(0) * t.size(2) * t.size(3);
  auto f32 = t.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({}, f32);
  at::Tensor lse = at::empty({2, npix}, f32);
  at::Tensor part = at::empty({kd_partial_blocks(npix)}, t.options().dtype(at::kDouble));
  launch_kd_fwd_fold(view4(s_lo), view4(t), align_corners, static_cast<float>(temperature), lse.data_ptr<float>(),
                     part.data_ptr<double>(), loss.data_ptr<float>(), cur_stream());
  return {loss, lse};
}

// -> the gradient of the FULL-resolution student logits (the upsample's backward maps it down)
static at::Tensor kd_kl_bwd_fold(const at::Tensor& grad, const at::Tensor& s_lo, const at::Tensor& t,
                                 const at::Tensor& lse, double temperature, bool align_corners) {
  TORCH_CHECK(kd_fold_ok(view4(s_lo), view4(t)), "rtseg.kd_fold: bad tensors");
  c10::hip::HIPGuardMasqueradingAsCUDA g(t.device());
  const int64_t npix = t.size(0) * t.size(2) * t.size(3);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == 2 * npix,
              "rtseg.kd_bwd: bad lse workspace");
  at::Tensor g32 = grad.to(at::kFloat).contiguous();
  at::Tensor gs = at::empty(t.sizes(), t.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_kd_bwd_fold(view4(s_lo), view4(t), view4(gs), align_corners, static_cast<float>(temperature),
                     lse.data_ptr<float>(), g32.data_ptr<float>(), cur_stream());
  return gs;
}

// cm[target, argmax_c x] as int64 [C, C]
static at::Tensor confmat(const at::Tensor& x, const at::Tensor& target, int64_t num_class, int64_t ignore) {
  TORCH_CHECK(x.dim() == 4 && x.size(1) == num_class, "rtseg.confmat: logits must be [N, num_class, H, W]");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.dim() == 3 &&
                  target.size(0) == x.size(0) && target.size(1) == x.size(2) && target.size(2) == x.size(3),
              "rtseg.confmat: target must be contiguous int64 [N, H, W] matching the logits");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor cm = at::zeros({num_class, num_class}, x.options().dtype(at::kLong));
  launch_confmat(view4(x), target.data_ptr<int64_t>(), static_cast<int>(ignore),
                 reinterpret_cast<unsigned long long*>(cm.data_ptr<int64_t>()), cur_stream());
  return cm;
}

static OptHyper hyper(int64_t mode, double lr, double momentum, double dampening, double weight_decay,
                      bool nesterov, double beta1, double beta2, double eps, double step_size,
                      double inv_sqrt_bc2, double grad_scale, double ema_w) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "rtseg.fused_opt: bad mode");
  OptHyper h;
  h.mode = static_cast<int>(mode);
  h.lr = static_cast<float>(lr);
  h.momentum = static_cast<float>(momentum);
  h.dampening = static_cast<float>(dampening);
  h.weight_decay = static_cast<float>(weight_decay);
  h.nesterov = nesterov ? 1 : 0;
  h.beta1 = static_cast<float>(beta1);
  h.beta2 = static_cast<float>(beta2);
  h.eps = static_cast<float>(eps);
  h.step_size = static_cast<float>(step_size);
  h.inv_sqrt_bc2 = static_cast<float>(inv_sqrt_bc2);
  h.grad_scale = static_cast<float>(grad_scale);
  h.ema_w = static_cast<float>(ema_w);
  return h;
}

static void check_meta(const at::Tensor& meta, int64_t ntensor, int64_t nblocks) {
  TORCH_CHECK(meta.is_cuda() && meta.scalar_type() == at::kLong && meta.is_contiguous() &&
                  meta.numel() == ntensor * kOptMetaFields + 2 * nblocks,
              "rtseg.fused_opt: malformed tensor table");
}

static void fused_opt_step(const at::Tensor& meta, int64_t ntensor, int64_t nblocks, int64_t mode, double lr,
                           double momentum, double dampening, double weight_decay, bool nesterov, double beta1,
                           double beta2, double eps, double step_size, double inv_sqrt_bc2, double grad_scale,
                           double ema_w) {
  check_meta(meta, ntensor, nblocks);
  c10::hip::HIPGuardMasqueradingAsCUDA g(meta.device());
  launch_fused_opt(meta.data_ptr<int64_t>(), static_cast<int>(ntensor), static_cast<int>(nblocks),
                   hyper(mode, lr, momentum, dampening, weight_decay, nesterov, beta1, beta2, eps, step_size,
                         inv_sqrt_bc2, grad_scale, ema_w),
                   cur_stream());
}

static void ema_lerp(const at::Tensor& meta, int64_t ntensor, int64_t nblocks, double w) {
  check_meta(meta, ntensor, nblocks);
  c10::hip::HIPGuardMasqueradingAsCUDA g(meta.device());
  launch_ema_lerp(meta.data_ptr<int64_t>(), static_cast<int>(ntensor), static_cast<int>(nblocks),
                  static_cast<float>(w), cur_stream());
}

static void shadow_crsk(const at::Tensor& tiles, int64_t ntiles) {
  TORCH_CHECK(tiles.is_cuda() && tiles.scalar_type() == at::kLong && tiles.is_contiguous() &&
                  tiles.numel() == 6 * ntiles,
              "rtseg.shadow_crsk: malformed tile table");
  c10::hip::HIPGuardMasqueradingAsCUDA g(tiles.device());
  launch_shadow_crsk(tiles.data_ptr<int64_t>(), static_cast<int>(ntiles), cur_stream());
}

// ---- STDC detail loss (detail_loss.hip) ------------------------------------------
static void check_detail(const at::Tensor& d) {
  TORCH_CHECK(d.is_cuda() && d.dim() == 4 && d.size(1) == 1, "rtseg.detail_loss: logits must be [N, 1, h, w] on GPU");
  TORCH_CHECK(d.scalar_type() == at::kFloat || d.scalar_type() == at::kBFloat16 || d.scalar_type() == at::kHalf,
              "rtseg.detail_loss: logits dtype must be fp32, bf16 or fp16");
}

// -> (loss fp32 scalar, binary target uint8 [N, H, W], per-sample sums fp64 [N, 4])
static std::tuple<at::Tensor, at::Tensor, at::Tensor> detail_loss_fwd(const at::Tensor& d, const at::Tensor& labels,
                                                                      const at::Tensor& wb, double thrs,
                                                                      double dice_coef, double bce_coef) {
  check_detail(d);
  TORCH_CHECK(labels.dim() == 3 && labels.is_contiguous() && labels.size(0) == d.size(0) &&
                  (labels.scalar_type() == at::kByte || labels.scalar_type() == at::kLong) &&
                  labels.device() == d.device(),
              "rtseg.detail_loss: labels must be contiguous uint8/int64 [N, H, W] on the logits' device");
  TORCH_CHECK(wb.scalar_type() == at::kFloat && wb.is_contiguous() && wb.numel() == 4 && wb.device() == d.device(),
              "rtseg.detail_loss: wb must be fp32 (w0, w1, w2, bias) on the logits' device");
  const int n = static_cast<int>(labels.size(0)), h = static_cast<int>(labels.size(1)),
            w = static_cast<int>(labels.size(2));
  TORCH_CHECK(static_cast<int64_t>(h) * w < (int64_t{1} << 31), "rtseg.detail_loss: image too large");
  c10::hip::HIPGuardMasqueradingAsCUDA g(d.device());
  auto opt = d.options();
  at::Tensor loss = at::empty({}, opt.dtype(at::kFloat));
  at::Tensor y = at::empty({n, h, w}, opt.dtype(at::kByte));
  at::Tensor sums = at::empty({n, 4}, opt.dtype(at::kDouble));
  at::Tensor part = at::empty({static_cast<int64_t>(n) * detail_loss_blocks(n, h, w) * 4}, opt.dtype(at::kDouble));
  launch_detail_fwd(view4(d), labels.data_ptr(), labels.scalar_type() == at::kByte, n, h, w, wb.data_ptr<float>(),
                    static_cast<float>(thrs), static_cast<float>(dice_coef), static_cast<float>(bce_coef),
                    y.data_ptr<uint8_t>(), part.data_ptr<double>(), sums.data_ptr<double>(), loss.data_ptr<float>(),
                    cur_stream());
  return {loss, y, sums};
}

static at::Tensor detail_loss_bwd(const at::Tensor& grad, const at::Tensor& d, const at::Tensor& y,
                                  const at::Tensor& sums, double dice_coef, double bce_coef) {
  check_detail(d);
  TORCH_CHECK(y.scalar_type() == at::kByte && y.is_contiguous() && y.dim() == 3 && y.size(0) == d.size(0),
              "rtseg.detail_loss_bwd: bad target");
  TORCH_CHECK(sums.scalar_type() == at::kDouble && sums.is_contiguous() && sums.numel() == 4 * d.size(0),
              "rtseg.detail_loss_bwd: bad sums");
  const int n = static_cast<int>(y.size(0)), h = static_cast<int>(y.size(1)), w = static_cast<int>(y.size(2));
  c10::hip::HIPGuardMasqueradingAsCUDA g(d.device());
  at::Tensor g32 = grad.to(at::kFloat).contiguous();
  auto f32 = d.options().dtype(at::kFloat);
  at::Tensor gp = at::empty({n, 1, h, w}, f32);
  launch_detail_bwd(view4(d), n, h, w, y.data_ptr<uint8_t>(), sums.data_ptr<double>(), g32.data_ptr<float>(),
                    static_cast<float>(dice_coef), static_cast<float>(bce_coef), gp.data_ptr<float>(), cur_stream());
  at::Tensor gd = at::empty({d.size(0), 1, d.size(2), d.size(3)}, f32);
  const int64_t wsn = interp_bwd_ws_elems(view4(gp), view4(gd));
  at::Tensor ws;
  if (wsn > 0) ws = at::empty({wsn}, f32);
  launch_interp_bwd(view4(gp), view4(gd), true, wsn > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  return gd.to(d.scalar_type());
}

// ---- prediction colouring (colorize.hip) ------------------------------------------
// -> (class map uint8 [N,H,W], colour uint8 [N,H,W,3], blend uint8 [N,H,W,3] or empty)
static std::tuple<at::Tensor, at::Tensor, at::Tensor> colorize(const at::Tensor& x, const at::Tensor& lut,
                                                               const std::optional<at::Tensor>& image, double alpha) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) >= 1 && x.size(1) <= 256,
              "rtseg.colorize: logits must be [N, C <= 256, H, W] on GPU");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf,
              "rtseg.colorize: logits dtype must be fp32, bf16 or fp16");
  TORCH_CHECK(lut.scalar_type() == at::kByte && lut.is_contiguous() && lut.dim() == 2 && lut.size(1) == 3 &&
                  lut.size(0) >= x.size(1) && lut.device() == x.device(),
              "rtseg.colorize: colormap must be contiguous uint8 [>= C, 3] on the logits' device");
  const int64_t n = x.size(0), h = x.size(2), w = x.size(3);
  TORCH_CHECK(n * h * w < (int64_t{1} << 31), "rtseg.colorize: too many pixels");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto u8 = x.options().dtype(at::kByte);
  at::Tensor cls = at::empty({n, h, w}, u8);
  at::Tensor rgb = at::empty({n, h, w, 3}, u8);
  at::Tensor blend = at::empty({0}, u8);
  const uint8_t* img = nullptr;
  if (image.has_value()) {
    TORCH_CHECK(image->scalar_type() == at::kByte && image->is_contiguous() && image->dim() == 4 &&
                    image->size(0) == n && image->size(1) == h && image->size(2) == w && image->size(3) == 3 &&
                    image->device() == x.device(),
                "rtseg.colorize: image must be contiguous uint8 [N, H, W, 3] matching the logits");
    blend = at::empty({n, h, w, 3}, u8);
    img = image->data_ptr<uint8_t>();
  }
  launch_colorize(view4(x), lut.data_ptr<uint8_t>(), img, static_cast<float>(alpha), cls.data_ptr<uint8_t>(),
                  rgb.data_ptr<uint8_t>(), img != nullptr ? blend.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {cls, rgb, blend};
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("kd_kl_fwd(Tensor s, Tensor t, float temperature) -> (Tensor, Tensor)");
  m.def("kd_kl_bwd(Tensor grad, Tensor s, Tensor t, Tensor lse, float temperature) -> Tensor");
  m.def("kd_kl_fwd_fold(Tensor s_lo, Tensor t, float temperature, bool align_corners) -> (Tensor, Tensor)");
  m.def("kd_kl_bwd_fold(Tensor grad, Tensor s_lo, Tensor t, Tensor lse, float temperature, bool align_corners) "
        "-> Tensor");
  m.def("detail_loss_fwd(Tensor d, Tensor labels, Tensor wb, float thrs, float dice_coef, float bce_coef) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("detail_loss_bwd(Tensor grad, Tensor d, Tensor y, Tensor sums, float dice_coef, float bce_coef) -> Tensor");
  m.def("colorize(Tensor x, Tensor lut, Tensor? image, float alpha) -> (Tensor, Tensor, Tensor)");
  m.def("confmat(Tensor x, Tensor target, int num_class, int ignore_index) -> Tensor");
  m.def("fused_opt_step(Tensor meta, int ntensor, int nblocks, int mode, float lr, float momentum, "
        "float dampening, float weight_decay, bool nesterov, float beta1, float beta2, float eps, "
        "float step_size, float inv_sqrt_bc2, float grad_scale, float ema_w) -> ()");
  m.def("ema_lerp(Tensor meta, int ntensor, int nblocks, float w) -> ()");
  m.def("shadow_crsk(Tensor tiles, int ntiles) -> ()");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("kd_kl_fwd", &rtseg::kd_kl_fwd);
  m.impl("kd_kl_bwd", &rtseg::kd_kl_bwd);
  m.impl("kd_kl_fwd_fold", &rtseg::kd_kl_fwd_fold);
  m.impl("kd_kl_bwd_fold", &rtseg::kd_kl_bwd_fold);
  m.impl("detail_loss_fwd", &rtseg::detail_loss_fwd);
  m.impl("detail_loss_bwd", &rtseg::detail_loss_bwd);
  m.impl("colorize", &rtseg::colorize);
  m.impl("confmat", &rtseg::confmat);
  m.impl("fused_opt_step", &rtseg::fused_opt_step);
  m.impl("ema_lerp", &rtseg::ema_lerp);
  m.impl("shadow_crsk", &rtseg::shadow_crsk);
}

// ------------------------------ depth-wise conv (dwconv.hip) -------------------------
namespace rtseg {

static void check_cl(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast),
              "rtseg.dwconv: ", what, " must be a channels-last contiguous 4-D GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "rtseg.dwconv: ", what,
              " must be 16-byte aligned");
}

static DwGeom dw_geom(int64_t n, int64_t cin, int64_t h, int64_t w, int64_t cout, int64_t kh, int64_t kw,
                      int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  TORCH_CHECK(cin > 0 && cout % cin == 0, "rtseg.dwconv: out_channels must be a multiple of in_channels");
  TORCH_CHECK(kh > 0 && kw > 0 && sh > 0 && sw > 0 && dh > 0 && dw > 0 && ph >= 0 && pw >= 0,
              "rtseg.dwconv: bad geometry");
  DwGeom g;
  g.n = static_cast<int>(n); g.cin = static_cast<int>(cin); g.h = static_cast<int>(h); g.w = static_cast<int>(w);
  g.cout = static_cast<int>(cout); g.mult = static_cast<int>(cout / cin);
  g.kh = static_cast<int>(kh); g.kw = static_cast<int>(kw); g.sh = static_cast<int>(sh); g.sw = static_cast<int>(sw);
  g.ph = static_cast<int>(ph); g.pw = static_cast<int>(pw); g.dh = static_cast<int>(dh); g.dw = static_cast<int>(dw);
  g.ho = static_cast<int>((h + 2 * ph - dh * (kh - 1) - 1) / sh + 1);
  g.wo = static_cast<int>((w + 2 * pw - dw * (kw - 1) - 1) / sw + 1);
  TORCH_CHECK(g.ho > 0 && g.wo > 0, "rtseg.dwconv: empty output");
  return g;
}

static void check_wt(const at::Tensor& wt, int64_t taps, int64_t cout) {
  TORCH_CHECK(wt.is_cuda() && wt.scalar_type() == at::kFloat && wt.is_contiguous() && wt.dim() == 2 &&
                  wt.size(0) == taps && wt.size(1) == cout,
              "rtseg.dwconv: weights must be tap-major fp32 [KH*KW, Cout]");
}

static at::Tensor dw_conv_fwd(const at::Tensor& x, const at::Tensor& wt, const std::optional<at::Tensor>& bias,
                              int64_t cout, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                              int64_t dh, int64_t dw, int64_t act) {
  check_cl(x, "input");
  TORCH_CHECK(act >= 0 && act <= 2, "rtseg.dw_conv_fwd: act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  DwGeom g = dw_geom(x.size(0), x.size(1), x.size(2), x.size(3), cout, kh, kw, sh, sw, ph, pw, dh, dw);
  g.act = static_cast<int>(act);
  check_wt(wt, kh * kw, cout);
  const float* b = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == cout,
                "rtseg.dwconv: bias must be fp32 [Cout]");
    b = bias->data_ptr<float>();
  }
  at::Tensor y = at::empty({x.size(0), cout, g.ho, g.wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_dw_fwd(g, dtype_code(x), x.data_ptr(), wt.data_ptr<float>(), b, y.data_ptr(), cur_stream());
  return y;
}

// forward + per-block BN statistics slab [rows, 2*Cout] (empty slab: unsupported multiplier)
static std::tuple<at::Tensor, at::Tensor> dw_conv_fwd_stats(const at::Tensor& x, const at::Tensor& wt, int64_t cout,
                                                            int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                                                            int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  check_cl(x, "input");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  DwGeom g = dw_geom(x.size(0), x.size(1), x.size(2), x.size(3), cout, kh, kw, sh, sw, ph, pw, dh, dw);
  check_wt(wt, kh * kw, cout);
  at::Tensor y = at::empty({x.size(0), cout, g.ho, g.wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rows = dw_fwd_stats_rows(g, dtype_code(x));
  at::Tensor part = at::empty({rows, 2 * cout}, x.options().dtype(at::kFloat));
  if (rows == 0) {
    launch_dw_fwd(g, dtype_code(x), x.data_ptr(), wt.data_ptr<float>(), nullptr, y.data_ptr(), cur_stream());
  } else {
    launch_dw_fwd_stats(g, dtype_code(x), x.data_ptr(), wt.data_ptr<float>(), y.data_ptr(), part.data_ptr<float>(),
                        cur_stream());
  }
  return {y, part};
}

static at::Tensor dw_conv_dgrad(const at::Tensor& dy, const at::Tensor& wt, int64_t cin, int64_t h, int64_t w,
                                int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                                int64_t dw) {
  check_cl(dy, "grad_output");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  DwGeom g = dw_geom(dy.size(0), cin, h, w, dy.size(1), kh, kw, sh, sw, ph, pw, dh, dw);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3), "rtseg.dwconv: grad_output shape mismatch");
  check_wt(wt, kh * kw, dy.size(1));
  at::Tensor dx = at::empty({dy.size(0), cin, h, w}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_dw_dgrad(g, dtype_code(dy), dy.data_ptr(), wt.data_ptr<float>(), dx.data_ptr(), cur_stream());
  return dx;
}

static at::Tensor dw_conv_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t kh, int64_t kw, int64_t sh,
                                int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  check_cl(dy, "grad_output");
  check_cl(x, "input");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "rtseg.dwconv: dtype mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  DwGeom g = dw_geom(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(1), kh, kw, sh, sw, ph, pw, dh, dw);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3) && dy.size(0) == x.size(0),
              "rtseg.dwconv: grad_output shape mismatch");
  TORCH_CHECK(static_cast<int64_t>(g.n) * g.ho * g.wo < (int64_t{1} << 31),
              "rtseg.dwconv: weight gradient over more than 2^31 output pixels per call");
  const DwWgradPlan p = dw_wgrad_plan(g, dtype_code(x));
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor part = at::empty({static_cast<int64_t>(p.slices) * kh * kw * g.cout}, f32);
  at::Tensor dwt = at::empty({g.cout, 1, kh, kw}, f32);
  launch_dw_wgrad(g, dtype_code(x), dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), dwt.data_ptr<float>(),
                  cur_stream());
  return dwt;
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("dw_conv_fwd(Tensor x, Tensor wt, Tensor? bias, int cout, int kh, int kw, int sh, int sw, int ph, int pw, "
        "int dh, int dw, int act=0) -> Tensor");
  m.def("dw_conv_fwd_stats(Tensor x, Tensor wt, int cout, int kh, int kw, int sh, int sw, int ph, int pw, "
        "int dh, int dw) -> (Tensor, Tensor)");
  m.def("dw_conv_dgrad(Tensor dy, Tensor wt, int cin, int h, int w, int kh, int kw, int sh, int sw, int ph, "
        "int pw, int dh, int dw) -> Tensor");
  m.def("dw_conv_wgrad(Tensor dy, Tensor x, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw) -> Tensor");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("dw_conv_fwd", &rtseg::dw_conv_fwd);
  m.impl("dw_conv_fwd_stats", &rtseg::dw_conv_fwd_stats);
  m.impl("dw_conv_dgrad", &rtseg::dw_conv_dgrad);
  m.impl("dw_conv_wgrad", &rtseg::dw_conv_wgrad);
}
