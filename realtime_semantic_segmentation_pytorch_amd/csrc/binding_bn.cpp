// torch.library registration of the fused BatchNorm(+residual)+activation ops.
//
// Non-synchronised BN runs as three launches forward (stats slab, fused
// finalize, apply) and three backward (reduce slab, finalize, apply), each op
// below issuing its kernels back to back on the current stream.  The SyncBN
// variants stop after producing fp64 sums so the caller can all-reduce them.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {
namespace {

int64_t rows_of(const at::Tensor& x) { return x.numel() / x.size(1); }

void check_cl(const at::Tensor& x, const char* what) {
  TORCH_CHECK(x.is_cuda(), "rtseg.bn: ", what, " must be on the GPU");
  TORCH_CHECK(x.dim() == 4 || x.dim() == 2, "rtseg.bn: ", what, " must be 4-D (or [M,C])");
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "rtseg.bn: ", what, " must be channels_last contiguous");
  } else {
    TORCH_CHECK(x.is_contiguous(), "rtseg.bn: ", what, " must be contiguous");
  }
  const int64_t C = x.size(1);
  TORCH_CHECK(C <= (1 << 20) && bn_vec_width(dtype_code(x), static_cast<int>(C)) > 0,
              "rtseg.bn: channel count ", C, " unsupported for ", x.scalar_type());
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "rtseg.bn: ", what,
              " must be 16-byte aligned");
}

// A channel slice [N, C, H, W] of a wider channels-last tensor (row stride ld elements): the
// concat buffer of ops/concat.py, which the apply kernels also write and whose gradient the
// backward kernels read in place of / on top of dy.  Full 16-byte channel vectors only.
struct Slice {
  void* p = nullptr;
  int64_t ld = 0;
};
Slice slice_of(const std::optional<at::Tensor>& t, const at::Tensor& like, const char* what) {
  if (!t.has_value() || !t->defined()) return {};
  TORCH_CHECK(t->is_cuda() && t->dim() == 4 && like.dim() == 4 && t->scalar_type() == like.scalar_type(),
              "rtseg.bn: ", what, " must be a 4-D GPU tensor of the activation's dtype");
  TORCH_CHECK(t->sizes() == like.sizes(), "rtseg.bn: ", what, " must have the activation's shape");
  const int64_t ld = t->stride(3), H = t->size(2), W = t->size(3);
  TORCH_CHECK(t->stride(1) == 1 && ld >= t->size(1) && (H == 1 || t->stride(2) == ld * W) &&
                  (t->size(0) == 1 || t->stride(0) == ld * W * H),
              "rtseg.bn: ", what, " must be a channel slice of a channels-last tensor");
  const int C = static_cast<int>(like.size(1));
  const int V = bn_vec_width(dtype_code(like), C);
  TORCH_CHECK(V * static_cast<int>(like.element_size()) == 16 && ld % V == 0 &&
                  reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
              "rtseg.bn: ", what, " needs 16-byte channel vectors and a 16-byte aligned slice");
  return {t->data_ptr(), ld};
}

const float* fptr(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}
float* fptr_mut(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? const_cast<float*>(t->data_ptr<float>()) : nullptr;
}
int64_t* nbt_ptr(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<int64_t>() : nullptr;
}

at::Tensor stats_slab(const at::Tensor& x, int& G, bool shift = true) {
  const int C = static_cast<int>(x.size(1));
  const int64_t M = rows_of(x);
  G = bn_partial_grid(M, C, dtype_code(x));
  at::Tensor part = at::empty({G + 1, 2 * C}, x.options().dtype(at::kFloat));  // row G: pivots
  launch_bn_stats(x.data_ptr(), dtype_code(x), M, C, part.data_ptr<float>(), G, cur_stream(), shift);
  return part;
}

// forward, single device: -> (mean_invstd[2C], scale_shift[2C], sums[2C+1])
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_stats_finalize(
    const at::Tensor& x, const std::optional<at::Tensor>& w, const std::optional<at::Tensor>& b,
    const std::optional<at::Tensor>& rmean, const std::optional<at::Tensor>& rvar,
    const std::optional<at::Tensor>& nbt, double momentum, double eps) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  const int C = static_cast<int>(x.size(1));
  int G = 0;
  at::Tensor part = stats_slab(x, G);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor mi = at::empty({2 * C}, f32), ss = at::empty({2 * C}, f32);
  at::Tensor sums = at::empty({2 * C + 1}, x.options().dtype(at::kDouble));
  launch_bn_finalize_partials(part.data_ptr<float>(), G, C, static_cast<double>(rows_of(x)),
                              fptr(w), fptr(b), fptr_mut(rmean), fptr_mut(rvar), nbt_ptr(nbt),
                              static_cast<float>(momentum), static_cast<float>(eps),
                              mi.data_ptr<float>(), ss.data_ptr<float>(), sums.data_ptr<double>(),
                              cur_stream(), part.data_ptr<float>() + static_cast<int64_t>(G) * 2 * C,
                              SlabScratch(G, C, part).ptr());
  return {mi, ss, sums};
}

// forward, SyncBN step 1 (and ops.channel_sum): -> sums[2C+1] (to be all-reduced).
// shift=false: raw moments about 0 instead of the sampled pivot (bn_act.hip)
at::Tensor bn_stats_sums(const at::Tensor& x, bool shift) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  const int C = static_cast<int>(x.size(1));
  int G = 0;
  at::Tensor part = stats_slab(x, G, shift);
  at::Tensor sums = at::empty({2 * C + 1}, x.options().dtype(at::kDouble));
  launch_bn_slab_to_sums(part.data_ptr<float>(), G, C, static_cast<double>(rows_of(x)),
                         sums.data_ptr<double>(), cur_stream(),
                         part.data_ptr<float>() + static_cast<int64_t>(G) * 2 * C, SlabScratch(G, C, part).ptr());
  return sums;
}

// forward, SyncBN step 2
std::tuple<at::Tensor, at::Tensor> bn_finalize(const at::Tensor& sums,
                                               const std::optional<at::Tensor>& w,
                                               const std::optional<at::Tensor>& b,
                                               const std::optional<at::Tensor>& rmean,
                                               const std::optional<at::Tensor>& rvar,
                                               const std::optional<at::Tensor>& nbt,
                                               double momentum, double eps) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(sums.device());
  const int C = static_cast<int>((sums.numel() - 1) / 2);
  auto f32 = sums.options().dtype(at::kFloat);
  at::Tensor mi = at::empty({2 * C}, f32), ss = at::empty({2 * C}, f32);
  launch_bn_finalize(sums.data_ptr<double>(), C, fptr(w), fptr(b), fptr_mut(rmean), fptr_mut(rvar),
                     nbt_ptr(nbt), static_cast<float>(momentum), static_cast<float>(eps),
                     mi.data_ptr<float>(), ss.data_ptr<float>(), cur_stream());
  return {mi, ss};
}

std::tuple<at::Tensor, at::Tensor> bn_eval_coeffs(const std::optional<at::Tensor>& w,
                                                  const std::optional<at::Tensor>& b,
                                                  const at::Tensor& rmean, const at::Tensor& rvar,
                                                  double eps) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(rmean.device());
  const int C = static_cast<int>(rmean.numel());
  auto f32 = rmean.options().dtype(at::kFloat);
  at::Tensor mi = at::empty({2 * C}, f32), ss = at::empty({2 * C}, f32);
  launch_bn_eval_coeffs(C, fptr(w), fptr(b), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                        static_cast<float>(eps), mi.data_ptr<float>(), ss.data_ptr<float>(),
                        cur_stream());
  return {mi, ss};
}

// slice_only: out2 (a channel slice of a wider channels-last buffer) is the only output -- the
// concat-then-BN sites (ops.cat_bn_act) write each part's normalised channels straight into the
// concatenated output; returns out2
at::Tensor bn_apply(const at::Tensor& x, const at::Tensor& scale_shift,
                    const std::optional<at::Tensor>& res, int64_t act, const std::optional<at::Tensor>& out2,
                    bool slice_only) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_cl(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(),
                "rtseg.bn_apply: residual mismatch");
    rp = res->data_ptr();
  }
  const Slice o2 = slice_of(out2, x, "out2");
  TORCH_CHECK(!slice_only || o2.p != nullptr, "rtseg.bn_apply: slice_only needs out2");
  at::Tensor y = slice_only ? *out2 : at::empty_like(x);
  launch_bn_apply(x.data_ptr(), rp, scale_shift.data_ptr<float>(), slice_only ? nullptr : y.data_ptr(),
                  dtype_code(x), rows_of(x), static_cast<int>(x.size(1)), static_cast<int>(act), cur_stream(), o2.p,
                  o2.ld);
  return y;
}

// Residual + activation forward that also returns the activation-derivative bit mask
// (one byte per channel vector; mask mode 3 of bn_bwd_sums / bn_backward).
std::tuple<at::Tensor, at::Tensor> bn_apply_bits(const at::Tensor& x, const at::Tensor& scale_shift,
                                                 const std::optional<at::Tensor>& res, int64_t act,
                                                 const std::optional<at::Tensor>& out2) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_cl(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(),
                "rtseg.bn_apply_bits: residual mismatch");
    rp = res->data_ptr();
  }
  TORCH_CHECK(act == 1 || act == 2, "rtseg.bn_apply_bits: relu / relu6 only");
  const int C = static_cast<int>(x.size(1));
  const int V = bn_vec_width(dtype_code(x), C);
  TORCH_CHECK(V > 0, "rtseg.bn_apply_bits: unsupported channel count");
  at::Tensor y = at::empty_like(x);
  at::Tensor bits = at::empty({rows_of(x) * (C / V)}, x.options().dtype(at::kByte));
  const Slice o2 = slice_of(out2, x, "out2");
  launch_bn_apply_bits(x.data_ptr(), rp, scale_shift.data_ptr<float>(), y.data_ptr(),
                       bits.data_ptr<uint8_t>(), dtype_code(x), rows_of(x), C, static_cast<int>(act),
                       cur_stream(), o2.p, o2.ld);
  return {y, bits};
}

const void* opt_y(const std::optional<at::Tensor>& y, int64_t mask) {
  const void* yp = nullptr;
  if (y.has_value() && y->defined()) {
    if (mask == 3) {
      TORCH_CHECK(y->scalar_type() == at::kByte && y->is_contiguous(), "rtseg.bn_bwd: bad bit mask");
    } else {
      check_cl(*y, "y");
    }
    yp = y->data_ptr();
  }
  TORCH_CHECK((mask != 1 && mask != 3) || yp, "rtseg.bn_bwd: mask-from-y / bit mask needs y");
  return yp;
}

// dy (null: the gradient is g2's alone) + g2 (a concat-buffer slice, or null)
const void* opt_dy(const std::optional<at::Tensor>& dy, const Slice& g2) {
  if (dy.has_value() && dy->defined()) {
    check_cl(*dy, "grad");
    return dy->data_ptr();
  }
  TORCH_CHECK(g2.p != nullptr, "rtseg.bn_bwd: needs grad or grad2");
  return nullptr;
}

at::Tensor bwd_slab(const void* dyp, const Slice& g2, const at::Tensor& x, const void* yp, const at::Tensor& mi,
                    const at::Tensor& ss, int64_t act, int64_t mask, int& G) {
  const int C = static_cast<int>(x.size(1));
  const int64_t M = rows_of(x);
  G = bn_partial_grid(M, C, dtype_code(x));
  at::Tensor part = at::empty({G, 2 * C}, x.options().dtype(at::kFloat));
  launch_bn_bwd_reduce(dyp, x.data_ptr(), yp, mi.data_ptr<float>(), ss.data_ptr<float>(),
                       dtype_code(x), M, C, static_cast<int>(act), static_cast<int>(mask),
                       part.data_ptr<float>(), G, cur_stream(), g2.p, g2.ld);
  return part;
}

// backward, SyncBN step 1: -> bsums[2C] (to be all-reduced)
at::Tensor bn_bwd_sums(const std::optional<at::Tensor>& dy, const at::Tensor& x, const std::optional<at::Tensor>& y,
                       const at::Tensor& mi, const at::Tensor& ss, int64_t act, int64_t mask,
                       const std::optional<at::Tensor>& grad2) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  const Slice g2 = slice_of(grad2, x, "grad2");
  const void* dyp = opt_dy(dy, g2);
  int G = 0;
  at::Tensor part = bwd_slab(dyp, g2, x, opt_y(y, mask), mi, ss, act, mask, G);
  const int C = static_cast<int>(x.size(1));
  at::Tensor bsums = at::empty({2 * C}, x.options().dtype(at::kDouble));
  launch_bn_slab_to_sums(part.data_ptr<float>(), G, C, -1.0, bsums.data_ptr<double>(), cur_stream(), nullptr,
                         SlabScratch(G, C, part).ptr());
  return bsums;
}

// backward, first half: reduce (unless bsums / slab given) + finalize -> (kcoef[3C], dw, db)
std::tuple<at::Tensor, at::Tensor, at::Tensor> bwd_coeffs_impl(
    const void* dyp, const Slice& g2, const at::Tensor& x, const void* yp,
    const std::optional<at::Tensor>& bsums, const std::optional<at::Tensor>& fwd_sums,
    const at::Tensor& mi, const at::Tensor& ss, const std::optional<at::Tensor>& w, int64_t act,
    int64_t mask, bool batch_stats, bool want_dw, const std::optional<at::Tensor>& slab) {
  const int C = static_cast<int>(x.size(1));
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor part;
  int G = 0;
  const double* sums_p = nullptr;
  if (bsums.has_value() && bsums->defined()) {
    sums_p = bsums->data_ptr<double>();
  } else if (slab.has_value() && slab->defined()) {  // reduction already done by the producer of dy
    TORCH_CHECK(slab->is_cuda() && slab->scalar_type() == at::kFloat && slab->dim() == 2 &&
                    slab->is_contiguous() && slab->size(1) == 2 * C,
                "rtseg.bn_backward: slab must be contiguous fp32 [G, 2C]");
    part = *slab;
    G = static_cast<int>(part.size(0));
  } else {
    part = bwd_slab(dyp, g2, x, yp, mi, ss, act, mask, G);
  }
  at::Tensor k = at::empty({3 * C}, f32);
  at::Tensor dw, db;
  if (want_dw) { dw = at::empty({C}, f32); db = at::empty({C}, f32); }
  const double* cnt = nullptr;
  if (fwd_sums.has_value() && fwd_sums->defined()) cnt = fwd_sums->data_ptr<double>() + 2 * C;
  TORCH_CHECK(!batch_stats || cnt, "rtseg.bn_bwd: batch statistics need the forward count");
  launch_bn_bwd_finalize(part.defined() ? part.data_ptr<float>() : nullptr, G, sums_p, cnt, C,
                         fptr(w), mi.data_ptr<float>(), batch_stats ? 1 : 0, k.data_ptr<float>(),
                         want_dw ? dw.data_ptr<float>() : nullptr,
                         want_dw ? db.data_ptr<float>() : nullptr, cur_stream(),
                         part.defined() && !sums_p ? SlabScratch(G, C, part).ptr() : nullptr);
  return {k, dw, db};
}

// backward: reduce (unless bsums given) + finalize + apply -> (dx, dres, dw, db)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_backward(
    const std::optional<at::Tensor>& dy, const at::Tensor& x, const std::optional<at::Tensor>& y,
    const std::optional<at::Tensor>& bsums, const std::optional<at::Tensor>& fwd_sums,
    const at::Tensor& mi, const at::Tensor& ss, const std::optional<at::Tensor>& w, int64_t act,
    int64_t mask, bool want_dres, bool batch_stats, bool want_dw, const std::optional<at::Tensor>& slab,
    const std::optional<at::Tensor>& grad2) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  const Slice g2 = slice_of(grad2, x, "grad2");
  const void* dyp = opt_dy(dy, g2);
  const void* yp = opt_y(y, mask);
  const int C = static_cast<int>(x.size(1));
  auto [k, dw, db] = bwd_coeffs_impl(dyp, g2, x, yp, bsums, fwd_sums, mi, ss, w, act, mask, batch_stats,
                                     want_dw, slab);
  at::Tensor dx = at::empty_like(x);
  at::Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  launch_bn_bwd_apply(dyp, x.data_ptr(), yp, mi.data_ptr<float>(), ss.data_ptr<float>(),
                      k.data_ptr<float>(), dx.data_ptr(), want_dres ? dres.data_ptr() : nullptr,
                      dtype_code(x), rows_of(x), C, static_cast<int>(act), static_cast<int>(mask),
                      cur_stream(), g2.p, g2.ld);
  return {dx, dres, dw, db};
}

// backward without the apply pass -> (kcoef[3C], dw, db): the dx pass is done by the consumer of
// dx instead (the stem conv's weight gradient, conv_stem_wgrad_bn)
std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_bwd_coeffs(
    const at::Tensor& dy, const at::Tensor& x, const std::optional<at::Tensor>& y,
    const std::optional<at::Tensor>& bsums, const std::optional<at::Tensor>& fwd_sums,
    const at::Tensor& mi, const at::Tensor& ss, const std::optional<at::Tensor>& w, int64_t act,
    int64_t mask, bool batch_stats, bool want_dw) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_cl(x, "x");
  check_cl(dy, "grad");
  const Slice g2{nullptr, 0};
  return bwd_coeffs_impl(dy.data_ptr(), g2, x, opt_y(y, mask), bsums, fwd_sums, mi, ss, w, act, mask,
                         batch_stats, want_dw, std::nullopt);
}

}  // namespace
}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("bn_stats_finalize(Tensor x, Tensor? weight, Tensor? bias, Tensor(a!)? running_mean, "
        "Tensor(b!)? running_var, Tensor(c!)? num_batches_tracked, float momentum, float eps) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("bn_stats_sums(Tensor x, bool shift=True) -> Tensor");
  m.def("bn_finalize(Tensor sums, Tensor? weight, Tensor? bias, Tensor(a!)? running_mean, "
        "Tensor(b!)? running_var, Tensor(c!)? num_batches_tracked, float momentum, float eps) -> (Tensor, Tensor)");
  m.def("bn_eval_coeffs(Tensor? weight, Tensor? bias, Tensor running_mean, Tensor running_var, "
        "float eps) -> (Tensor, Tensor)");
  m.def("bn_apply(Tensor x, Tensor scale_shift, Tensor? residual, int act, Tensor(a!)? out2=None, "
        "bool slice_only=False) -> Tensor");
  m.def("bn_apply_bits(Tensor x, Tensor scale_shift, Tensor? residual, int act, Tensor(a!)? out2=None) "
        "-> (Tensor, Tensor)");
  m.def("bn_bwd_sums(Tensor? grad, Tensor x, Tensor? y, Tensor mean_invstd, Tensor scale_shift, "
        "int act, int mask, Tensor? grad2=None) -> Tensor");
  m.def("bn_backward(Tensor? grad, Tensor x, Tensor? y, Tensor? bsums, Tensor? fwd_sums, "
        "Tensor mean_invstd, Tensor scale_shift, Tensor? weight, int act, int mask, bool want_dres, "
        "bool batch_stats, bool want_dw, Tensor? slab=None, Tensor? grad2=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("bn_bwd_coeffs(Tensor grad, Tensor x, Tensor? y, Tensor? bsums, Tensor? fwd_sums, "
        "Tensor mean_invstd, Tensor scale_shift, Tensor? weight, int act, int mask, bool batch_stats, "
        "bool want_dw) -> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("bn_stats_finalize", &rtseg::bn_stats_finalize);
  m.impl("bn_stats_sums", &rtseg::bn_stats_sums);
  m.impl("bn_finalize", &rtseg::bn_finalize);
  m.impl("bn_eval_coeffs", &rtseg::bn_eval_coeffs);
  m.impl("bn_apply", &rtseg::bn_apply);
  m.impl("bn_apply_bits", &rtseg::bn_apply_bits);
  m.impl("bn_bwd_sums", &rtseg::bn_bwd_sums);
  m.impl("bn_backward", &rtseg::bn_backward);
  m.impl("bn_bwd_coeffs", &rtseg::bn_bwd_coeffs);
}
