// torch.library registration of the 32x32x16-MFMA implicit-GEMM conv family (conv_igemm.hip):
// forward (+ BN statistics / inference BN epilogue), data gradient and weight gradient.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {
namespace {

void check_act(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.scalar_type() == at::kBFloat16 &&
                  t.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "rtseg.conv_igemm: ", what, " must be a 16-byte aligned channels-last bf16 GPU tensor");
}

ConvGeom geom(int64_t N, int64_t Cin, int64_t H, int64_t W, int64_t Cout, int64_t KH, int64_t KW,
              at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation) {
  TORCH_CHECK(stride.size() == 2 && padding.size() == 2 && dilation.size() == 2, "rtseg.conv_igemm: 2-D geometry");
  ConvGeom g{};
  g.n = static_cast<int>(N); g.cin = static_cast<int>(Cin); g.h = static_cast<int>(H); g.w_in = static_cast<int>(W);
  g.cout = static_cast<int>(Cout); g.kh = static_cast<int>(KH); g.kw = static_cast<int>(KW);
  g.sh = static_cast<int>(stride[0]); g.sw = static_cast<int>(stride[1]);
  g.ph = static_cast<int>(padding[0]); g.pw = static_cast<int>(padding[1]);
  g.dh = static_cast<int>(dilation[0]); g.dw = static_cast<int>(dilation[1]);
  TORCH_CHECK(g.sh >= 1 && g.sw >= 1 && g.dh >= 1 && g.dw >= 1 && g.ph >= 0 && g.pw >= 0,
              "rtseg.conv_igemm: bad geometry");
  g.ho = static_cast<int>((H + 2 * padding[0] - dilation[0] * (KH - 1) - 1) / stride[0] + 1);
  g.wo = static_cast<int>((W + 2 * padding[1] - dilation[1] * (KW - 1) - 1) / stride[1] + 1);
  TORCH_CHECK(g.ho > 0 && g.wo > 0, "rtseg.conv_igemm: empty output");
  TORCH_CHECK(N * H * W < (int64_t{1} << 31) && N * g.ho * g.wo < (int64_t{1} << 31) &&
                  H * W * std::max(Cin, Cout) < (int64_t{1} << 31),
              "rtseg.conv_igemm: problem too large for 32-bit pixel indexing");
  return g;
}

// x [N,Cin,H,W] CL bf16, wk [Cout,KH,KW,Cin] bf16 -> (y CL bf16, BN statistics slab or empty)
std::tuple<at::Tensor, at::Tensor> conv_fwd_impl(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                                 at::IntArrayRef padding, at::IntArrayRef dilation, bool stats,
                                                 const std::optional<at::Tensor>& scale_shift,
                                                 const std::optional<at::Tensor>& residual, int64_t act, int kind) {
  // kind 7: the stem kernel's statistics without the output stores
  const bool halo = kind == 1, wres = kind == 2, hreg = kind == 3 || kind == 4 || kind == 8 || kind == 9, stem = kind == 5 || kind == 7;
  check_act(x, "input");
  TORCH_CHECK(wk.is_cuda() && wk.dim() == 4 && wk.scalar_type() == at::kBFloat16 && wk.is_contiguous() &&
                  wk.size(3) == x.size(1),
              "rtseg.conv_igemm: weights must be contiguous bf16 [Cout, KH, KW, Cin]");
  TORCH_CHECK(act >= 0 && act <= 2, "rtseg.conv_igemm: bad activation");
  ConvGeom g = geom(x.size(0), x.size(1), x.size(2), x.size(3), wk.size(0), wk.size(1), wk.size(2), stride, padding,
                    dilation);
  if (stem) {
    TORCH_CHECK(conv_stem_supported(g),
                "rtseg.conv_stem: needs Cin == 3, 3 x 3 / pad 1 / stride 1 or 2, Cout % 16 == 0 and <= 64, even W");
    TORCH_CHECK(!(residual.has_value() && residual->defined()), "rtseg.conv_stem: no residual epilogue");
  } else if (halo) {
    TORCH_CHECK(conv_halo_supported(g, 0),
                "rtseg.conv_halo: needs stride 1, taps within 3 x 3, Cin % 64 == 0, Cout % 64 == 0");
  } else if (wres) {
    TORCH_CHECK(conv_wres_supported(g, 0), "rtseg.conv_wres: needs 3 x 3 / stride 1 / pad 1, Cin == 64, Cout % 64 == 0");
  } else if (hreg) {
    TORCH_CHECK(conv_hreg_supported(g, 0),
                "rtseg.conv_hreg: needs 3 x 3 / stride 1 / pad 1, Cin % 64 == 0, Cout % 128 == 0");
    TORCH_CHECK(!(scale_shift.has_value() && scale_shift->defined()), "rtseg.conv_hreg: no inference BN epilogue");
  } else {
    TORCH_CHECK(conv_igemm_supported(g, 0), "rtseg.conv_igemm: needs Cin % 64 == 0, Cout % 8 == 0, <= 49 taps");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({g.n, g.cout, g.ho, g.wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  g.x = x.data_ptr(); g.w = wk.data_ptr(); g.y = kind == 7 ? nullptr : y.data_ptr();
  g.part = nullptr; g.scale_shift = nullptr; g.res = nullptr; g.act = static_cast<int>(act);
  at::Tensor part;
  if (stats) {
    part = at::empty({stem ? conv_stem_slabs(g) : halo ? conv_halo_slabs(g) : wres ? conv_wres_slabs(g) : hreg ? conv_hreg_slabs(g)
                                                                                 : conv_igemm_slabs(g),
                      2 * g.cout},
                     x.options().dtype(at::kFloat));
    g.part = part.data_ptr<float>();
  }
  if (scale_shift.has_value() && scale_shift->defined()) {
    TORCH_CHECK(!stats, "rtseg.conv_igemm: statistics and the inference BN epilogue are exclusive");
    TORCH_CHECK(scale_shift->scalar_type() == at::kFloat && scale_shift->is_contiguous() &&
                    scale_shift->numel() == 2 * g.cout && scale_shift->is_cuda(),
                "rtseg.conv_igemm: scale_shift must be fp32 [2*Cout]");
    g.scale_shift = scale_shift->data_ptr<float>();
    if (residual.has_value() && residual->defined()) {
      check_act(*residual, "residual");
      TORCH_CHECK(residual->sizes() == y.sizes(), "rtseg.conv_igemm: residual must match the output");
      g.res = residual->data_ptr();
    }
  } else {
    TORCH_CHECK(!(residual.has_value() && residual->defined()) && act == 0,
                "rtseg.conv_igemm: residual / activation need the BN epilogue (scale_shift)");
  }
  if (stem) launch_conv_stem_fwd(g, cur_stream());
  else if (halo) launch_conv_halo_fwd(g, cur_stream());
  else if (wres) launch_conv_wres_fwd(g, cur_stream());
  else if (hreg) {
    at::Tensor wpack = at::empty({conv_hreg_pack_elems(g, 0)}, wk.options());
    launch_conv_hreg(g, 0, wpack.data_ptr(), cur_stream(), kind == 4 ? 2 : kind == 8 ? 4 : kind == 9 ? 5 : 1);
  } else {
    if (kind == 11 || kind == 12) {
      TORCH_CHECK(g.scale_shift != nullptr && !stats, "rtseg.conv_igemm_small: the inference BN epilogue only");
      g.cfg = 5;
    }
    const int ks = kind == 12 ? conv_igemm_splitk(g) : 1;
    if (ks > 1) {
      at::Tensor ws = at::empty({static_cast<int64_t>(ks) * g.n * g.ho * g.wo * g.cout}, x.options().dtype(at::kFloat));
      launch_conv_igemm_fwd_splitk(g, ws.data_ptr<float>(), ks, cur_stream());
    } else {
      launch_conv_igemm_fwd(g, cur_stream());
    }
  }
  if (stats && part.size(0) > 256) {  // fold the per-tile rows so the BN finalize stays cheap
    const int rows = static_cast<int>(part.size(0));
    const int chunk = (rows + 255) / 256;
    at::Tensor small = at::empty({(rows + chunk - 1) / chunk, 2 * g.cout}, part.options());
    launch_slab_compact(part.data_ptr<float>(), rows, 2 * g.cout, chunk, small.data_ptr<float>(), cur_stream());
    part = small;
  }
  return {y, part};
}

std::tuple<at::Tensor, at::Tensor> conv_igemm(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                              at::IntArrayRef padding, at::IntArrayRef dilation, bool stats,
                                              const std::optional<at::Tensor>& scale_shift,
                                              const std::optional<at::Tensor>& residual, int64_t act) {
  return conv_fwd_impl(x, wk, stride, padding, dilation, stats, scale_shift, residual, act, 0);
}

// conv_wres with the inference BN epilogue act(conv * scale + shift (+ residual)): 64-channel
// 3 x 3 layers at batch-1 inference (DDRNet-23's 1/4-resolution stage)
at::Tensor conv_wres_eval(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride, at::IntArrayRef padding,
                          at::IntArrayRef dilation, const at::Tensor& scale_shift,
                          const std::optional<at::Tensor>& residual, int64_t act) {
  return std::get<0>(conv_fwd_impl(x, wk, stride, padding, dilation, false, scale_shift, residual, act, 2));
}

// the gather kernel on 128 x 64 block tiles, 2 blocks per CU (inference BN epilogue only): small
// batch-1 layers, timed against the shape-picked tiles and MIOpen (ops/conv.py conv_bn_act_eval)
at::Tensor conv_igemm_small(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride, at::IntArrayRef padding,
                            at::IntArrayRef dilation, const at::Tensor& scale_shift,
                            const std::optional<at::Tensor>& residual, int64_t act, bool split_k) {
  return std::get<0>(conv_fwd_impl(x, wk, stride, padding, dilation, false, scale_shift, residual, act,
                                   split_k ? 12 : 11));
}

// the halo-tiled kernel (conv_halo.hip): stride-1 convs whose taps fit a 3 x 3 footprint
std::tuple<at::Tensor, at::Tensor> conv_halo(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                             at::IntArrayRef padding, at::IntArrayRef dilation, bool stats,
                                             const std::optional<at::Tensor>& scale_shift,
                                             const std::optional<at::Tensor>& residual, int64_t act) {
  return conv_fwd_impl(x, wk, stride, padding, dilation, stats, scale_shift, residual, act, 1);
}

// the register-weight halo kernel (conv_hreg.hip): 3 x 3 stride-1 convs, Cin % 64, Cout % 128
// (rows_per_wave = wave layout 1: 8 waves of 2 x 2 tiles; 2: 4 waves of 2 x 4; 4: 8 waves of 1 x 4;
// 5: layout 4 with double-buffered accumulators, the epilogue drained beside the next tile's MFMAs)
std::tuple<at::Tensor, at::Tensor> conv_hreg(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                             at::IntArrayRef padding, at::IntArrayRef dilation, bool stats,
                                             int64_t rows_per_wave) {
  TORCH_CHECK(rows_per_wave == 1 || rows_per_wave == 2 || rows_per_wave == 4 || rows_per_wave == 5,
              "rtseg.conv_hreg: rows_per_wave (wave layout) must be 1, 2, 4 or 5");
  return conv_fwd_impl(x, wk, stride, padding, dilation, stats, std::nullopt, std::nullopt, 0,
                       rows_per_wave == 2 ? 4 : rows_per_wave == 4 ? 8 : rows_per_wave == 5 ? 9 : 3);
}

// the weights-resident halo kernel (conv_wres.hip): 3 x 3 stride-1 convs with Cin == 64
std::tuple<at::Tensor, at::Tensor> conv_wres(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                             at::IntArrayRef padding, at::IntArrayRef dilation, bool stats) {
  return conv_fwd_impl(x, wk, stride, padding, dilation, stats, std::nullopt, std::nullopt, 0, 2);
}

// the 3-channel stem kernel (conv_stem.hip): 3 x 3 / pad 1 / stride 1 or 2, Cout % 16 <= 64
// store = false (with stats): the statistics only; y is returned allocated but never written -- the
// stem BN recomputes it wherever it is needed (ops/bn.py, conv_stem_bn_act / _bn_sums / _wgrad_bn)
std::tuple<at::Tensor, at::Tensor> conv_stem(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                                             at::IntArrayRef padding, at::IntArrayRef dilation, bool stats,
                                             bool store) {
  TORCH_CHECK(store || stats, "rtseg.conv_stem: store = false needs stats");
  return conv_fwd_impl(x, wk, stride, padding, dilation, stats, std::nullopt, std::nullopt, 0, store ? 5 : 7);
}

// the stem BN's backward reduction [slabs, 2 cout] (sum g', sum g' (x - mean)) with the conv
// output x recomputed from the image instead of read back (conv_stem.hip, STATS 2)
at::Tensor conv_stem_bn_sums(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                             at::IntArrayRef padding, at::IntArrayRef dilation, const at::Tensor& dy,
                             const at::Tensor& mean_invstd, const at::Tensor& scale_shift, int64_t act) {
  check_act(x, "input");
  check_act(dy, "grad_output");
  TORCH_CHECK(wk.is_cuda() && wk.dim() == 4 && wk.scalar_type() == at::kBFloat16 && wk.is_contiguous() &&
                  wk.size(3) == x.size(1),
              "rtseg.conv_stem_bn_sums: weights must be contiguous bf16 [Cout, KH, KW, Cin]");
  ConvGeom g = geom(x.size(0), x.size(1), x.size(2), x.size(3), wk.size(0), wk.size(1), wk.size(2), stride, padding,
                    dilation);
  TORCH_CHECK(conv_stem_supported(g), "rtseg.conv_stem_bn_sums: not a stem geometry");
  TORCH_CHECK(dy.size(0) == g.n && dy.size(1) == g.cout && dy.size(2) == g.ho && dy.size(3) == g.wo,
              "rtseg.conv_stem_bn_sums: grad_output does not match the geometry");
  TORCH_CHECK(mean_invstd.is_cuda() && mean_invstd.scalar_type() == at::kFloat && mean_invstd.numel() == 2 * g.cout &&
                  scale_shift.is_cuda() && scale_shift.scalar_type() == at::kFloat && scale_shift.numel() == 2 * g.cout,
              "rtseg.conv_stem_bn_sums: coefficients must be fp32 [2 cout]");
  TORCH_CHECK(act >= 0 && act <= 2, "rtseg.conv_stem_bn_sums: bad activation");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor part = at::empty({conv_stem_slabs(g), 2 * g.cout}, x.options().dtype(at::kFloat));
  g.x = x.data_ptr(); g.w = wk.data_ptr(); g.y = const_cast<void*>(dy.data_ptr());
  launch_conv_stem_bn_sums(g, mean_invstd.data_ptr<float>(), scale_shift.data_ptr<float>(), static_cast<int>(act),
                           part.data_ptr<float>(), cur_stream());
  return part;
}

// ... with a BN (+ activation) epilogue on the fp32 accumulators: act(conv(x) * scale + shift)
at::Tensor conv_stem_bn_act(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride, at::IntArrayRef padding,
                            at::IntArrayRef dilation, const at::Tensor& scale_shift, int64_t act) {
  return std::get<0>(conv_fwd_impl(x, wk, stride, padding, dilation, false, scale_shift, std::nullopt, act, 5));
}

// the 7 x 7 stem (conv_stem7.hip): x [N,3,H,W] CL bf16, wk [Cout,7,7,3] bf16 -> y [N,Cout,Ho,Wo] CL
// bf16, = act(conv * scale + shift) when scale_shift is given (inference BN epilogue)
at::Tensor conv_stem7(const at::Tensor& x, const at::Tensor& wk, at::IntArrayRef stride,
                      const std::optional<at::Tensor>& scale_shift, int64_t act) {
  check_act(x, "input");
  TORCH_CHECK(wk.is_cuda() && wk.dim() == 4 && wk.scalar_type() == at::kBFloat16 && wk.is_contiguous() &&
                  wk.size(1) == 7 && wk.size(2) == 7 && wk.size(3) == 3 && x.size(1) == 3,
              "rtseg.conv_stem7: weights must be contiguous bf16 [Cout, 7, 7, 3] on a 3-channel input");
  const int64_t pad[2] = {3, 3}, dil[2] = {1, 1};
  ConvGeom g = geom(x.size(0), 3, x.size(2), x.size(3), wk.size(0), 7, 7, stride, pad, dil);
  TORCH_CHECK(conv_stem7_supported(g), "rtseg.conv_stem7: needs stride 1 / 2, Cout % 16 <= 64, even W");
  if (scale_shift.has_value() && scale_shift->defined()) {
    TORCH_CHECK(scale_shift->is_cuda() && scale_shift->scalar_type() == at::kFloat &&
                    scale_shift->numel() == 2 * g.cout && scale_shift->is_contiguous(),
                "rtseg.conv_stem7: scale_shift must be fp32 [2 cout]");
    TORCH_CHECK(act >= 0 && act <= 2, "rtseg.conv_stem7: bad activation");
    g.scale_shift = scale_shift->data_ptr<float>();
    g.act = static_cast<int>(act);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor y = at::empty({g.n, g.cout, g.ho, g.wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  g.x = x.data_ptr(); g.w = wk.data_ptr(); g.y = y.data_ptr();
  launch_conv_stem7_fwd(g, cur_stream());
  return y;
}

// dy [N,Cout,Ho,Wo] CL bf16, wt [Cin,KH,KW,Cout] bf16 -> dx [N,Cin,H,W] CL bf16
at::Tensor conv_dgrad_impl(const at::Tensor& dy, const at::Tensor& wt, at::IntArrayRef x_size,
                           at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                           const std::optional<at::Tensor>& bias, const std::optional<at::Tensor>& addend, int kind,
                           const std::optional<at::Tensor>& addend_mask,
                           const std::optional<at::Tensor>& phase_addend, bool fused_phases = false) {
  const bool halo = kind == 1, wres = kind == 2, hreg = kind == 3 || kind == 4 || kind == 8 || kind == 9;
  check_act(dy, "grad_output");
  TORCH_CHECK(x_size.size() == 4, "rtseg.conv_igemm_dgrad: x_size must be [N, Cin, H, W]");
  TORCH_CHECK(wt.is_cuda() && wt.dim() == 4 && wt.scalar_type() == at::kBFloat16 && wt.is_contiguous() &&
                  wt.size(0) == x_size[1] && wt.size(3) == dy.size(1),
              "rtseg.conv_igemm_dgrad: weights must be contiguous bf16 [Cin, KH, KW, Cout]");
  ConvGeom g = geom(x_size[0], x_size[1], x_size[2], x_size[3], dy.size(1), wt.size(1), wt.size(2), stride, padding,
                    dilation);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3) && g.n == dy.size(0),
              "rtseg.conv_igemm_dgrad: grad_output does not match the geometry");
  if (halo) {
    TORCH_CHECK(conv_halo_supported(g, 1),
                "rtseg.conv_halo_dgrad: needs stride 1, taps within 3 x 3, Cin % 64 == 0, Cout % 64 == 0");
    TORCH_CHECK(!(bias.has_value() && bias->defined()), "rtseg.conv_halo_dgrad: no bias");
  } else if (wres) {
    TORCH_CHECK(conv_wres_supported(g, 1), "rtseg.conv_wres_dgrad: needs 3 x 3 / stride 1 / pad 1, Cout == 64, Cin % 64 == 0");
    TORCH_CHECK(!(bias.has_value() && bias->defined()), "rtseg.conv_wres_dgrad: no bias");
  } else if (hreg) {
    TORCH_CHECK(conv_hreg_supported(g, 1),
                "rtseg.conv_hreg_dgrad: needs 3 x 3 / stride 1 / pad 1, Cout % 64 == 0, Cin % 128 == 0");
    TORCH_CHECK(!(bias.has_value() && bias->defined()), "rtseg.conv_hreg_dgrad: no bias");
  } else {
    TORCH_CHECK(conv_igemm_supported(g, 1), "rtseg.conv_igemm_dgrad: needs Cout % 64 == 0, Cin % 8 == 0");
    TORCH_CHECK(!fused_phases || conv_igemm_dgrad_fused_ok(g),
                "rtseg.conv_igemm_dgrad: fused phases need a strided conv with H % sh == 0, W % sw == 0");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  at::Tensor dx = at::empty({g.n, g.cin, g.h, g.w_in}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  g.x = dy.data_ptr(); g.w = wt.data_ptr(); g.y = dx.data_ptr();
  g.scale_shift = nullptr;
  if (bias.has_value() && bias->defined()) {  // transposed-conv forward: y = convT(x) + b
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->is_contiguous() &&
                    bias->numel() == g.cin,
                "rtseg.conv_igemm_dgrad: bias must be fp32 [Cin]");
    g.scale_shift = bias->data_ptr<float>();
  }
  g.res = nullptr;
  if (addend.has_value() && addend->defined()) {  // dx = dgrad(dy) + addend, fused in the epilogue
    check_act(*addend, "addend");
    TORCH_CHECK(addend->sizes() == dx.sizes(), "rtseg.conv_igemm_dgrad: addend must match dx");
    g.res = addend->data_ptr();
    if (addend_mask.has_value() && addend_mask->defined()) {  // dx += addend * mask (ops/bn.py kMaskBits)
      TORCH_CHECK(addend_mask->is_cuda() && addend_mask->scalar_type() == at::kByte && addend_mask->is_contiguous() &&
                      addend_mask->numel() * 8 == dx.numel() && g.cin % 8 == 0,
                  "rtseg.conv_dgrad: addend_mask must be contiguous uint8 [numel(dx) / 8]");
      g.amask = addend_mask->data_ptr<uint8_t>();
    }
  } else {
    TORCH_CHECK(!(addend_mask.has_value() && addend_mask->defined()), "rtseg.conv_dgrad: addend_mask without addend");
  }
  if (phase_addend.has_value() && phase_addend->defined()) {  // added to output phase (0, 0) only
    TORCH_CHECK(kind == 0, "rtseg.conv_dgrad: phase_addend is an igemm dgrad option");
    check_act(*phase_addend, "phase_addend");
    TORCH_CHECK(phase_addend->size(0) == g.n && phase_addend->size(1) == g.cin &&
                    phase_addend->size(2) == (g.h + g.sh - 1) / g.sh && phase_addend->size(3) == (g.w_in + g.sw - 1) / g.sw,
                "rtseg.conv_igemm_dgrad: phase_addend must be [N, Cin, ceil(H / sh), ceil(W / sw)]");
    g.res_phase0 = phase_addend->data_ptr();
  }
  if (halo) launch_conv_halo_dgrad(g, cur_stream());
  else if (wres) launch_conv_wres_dgrad(g, cur_stream());
  else if (hreg) {
    at::Tensor wpack = at::empty({conv_hreg_pack_elems(g, 1)}, wt.options());
    launch_conv_hreg(g, 1, wpack.data_ptr(), cur_stream(), kind == 4 ? 2 : kind == 8 ? 4 : kind == 9 ? 5 : 1);
  } else if (fused_phases) {
    launch_conv_igemm_dgrad_fused(g, cur_stream());
  } else {
    launch_conv_igemm_dgrad(g, cur_stream());
  }
  return dx;
}

at::Tensor conv_igemm_dgrad(const at::Tensor& dy, const at::Tensor& wt, at::IntArrayRef x_size,
                            at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                            const std::optional<at::Tensor>& bias, const std::optional<at::Tensor>& addend,
                            const std::optional<at::Tensor>& addend_mask,
                            const std::optional<at::Tensor>& phase_addend, bool fused_phases) {
  return conv_dgrad_impl(dy, wt, x_size, stride, padding, dilation, bias, addend, 0, addend_mask, phase_addend,
                         fused_phases);
}

at::Tensor conv_halo_dgrad(const at::Tensor& dy, const at::Tensor& wt, at::IntArrayRef x_size,
                           at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                           const std::optional<at::Tensor>& addend, const std::optional<at::Tensor>& addend_mask) {
  return conv_dgrad_impl(dy, wt, x_size, stride, padding, dilation, std::nullopt, addend, 1, addend_mask,
                         std::nullopt);
}

at::Tensor conv_hreg_dgrad(const at::Tensor& dy, const at::Tensor& wt, at::IntArrayRef x_size,
                           at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                           const std::optional<at::Tensor>& addend, int64_t rows_per_wave,
                           const std::optional<at::Tensor>& addend_mask) {
  TORCH_CHECK(rows_per_wave == 1 || rows_per_wave == 2 || rows_per_wave == 4 || rows_per_wave == 5,
              "rtseg.conv_hreg_dgrad: rows_per_wave (wave layout) must be 1, 2, 4 or 5");
  return conv_dgrad_impl(dy, wt, x_size, stride, padding, dilation, std::nullopt, addend,
                         rows_per_wave == 2 ? 4 : rows_per_wave == 4 ? 8 : rows_per_wave == 5 ? 9 : 3, addend_mask,
                         std::nullopt);
}

at::Tensor conv_wres_dgrad(const at::Tensor& dy, const at::Tensor& wt, at::IntArrayRef x_size,
                           at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                           const std::optional<at::Tensor>& addend, const std::optional<at::Tensor>& addend_mask) {
  return conv_dgrad_impl(dy, wt, x_size, stride, padding, dilation, std::nullopt, addend, 2, addend_mask,
                         std::nullopt);
}

// x [N,Cin,H,W], dy [N,Cout,Ho,Wo] (CL bf16) -> dw fp32 [Cout,Cin,KH,KW]
at::Tensor conv_igemm_wgrad(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw,
                            at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                            bool channels_last) {
  check_act(x, "input");
  check_act(dy, "grad_output");
  ConvGeom g = geom(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(1), kh, kw, stride, padding, dilation);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3) && g.n == dy.size(0),
              "rtseg.conv_igemm_wgrad: grad_output does not match the geometry");
  TORCH_CHECK(conv_igemm_supported(g, 2), "rtseg.conv_igemm_wgrad: needs Cin % 64 == 0 and Cout % 64 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  g.x = x.data_ptr(); g.y = dy.data_ptr();
  at::Tensor ws = at::empty({conv_igemm_wgrad_ws_elems(g)}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({g.cout, g.cin, g.kh, g.kw},
                            x.options().dtype(at::kFloat).memory_format(channels_last ? at::MemoryFormat::ChannelsLast
                                                                                      : at::MemoryFormat::Contiguous));
  launch_conv_igemm_wgrad(g, ws.data_ptr<float>(), dw.data_ptr<float>(), channels_last, cur_stream());
  return dw;
}

// halo-tiled weight gradient (conv_whalo.hip): 3 x 3 / stride 1 / pad 1, Cin and Cout % 64 == 0
at::Tensor conv_whalo_wgrad(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw, at::IntArrayRef stride,
                            at::IntArrayRef padding, at::IntArrayRef dilation, bool channels_last, int64_t variant) {
  check_act(x, "input");
  check_act(dy, "grad_output");
  ConvGeom g = geom(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(1), kh, kw, stride, padding, dilation);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3) && g.n == dy.size(0),
              "rtseg.conv_whalo_wgrad: grad_output does not match the geometry");
  TORCH_CHECK(conv_whalo_supported(g), "rtseg.conv_whalo_wgrad: needs 3 x 3 / stride 1 / pad 1, Cin and Cout % 64 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  g.x = x.data_ptr(); g.y = dy.data_ptr();
  at::Tensor ws = at::empty({conv_whalo_ws_elems(g)}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({g.cout, g.cin, g.kh, g.kw},
                            x.options().dtype(at::kFloat).memory_format(channels_last ? at::MemoryFormat::ChannelsLast
                                                                                      : at::MemoryFormat::Contiguous));
  TORCH_CHECK(variant == 1 || variant == 2, "rtseg.conv_whalo_wgrad: variant must be 1 or 2");
  launch_conv_whalo_wgrad(g, ws.data_ptr<float>(), dw.data_ptr<float>(), channels_last, cur_stream(),
                          static_cast<int>(variant));
  return dw;
}

// stem weight gradient (conv_stem.hip): x [N,3,H,W], dy [N,Cout,Ho,Wo] CL bf16 -> dw fp32
at::Tensor conv_stem_wgrad(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw, at::IntArrayRef stride,
                           at::IntArrayRef padding, at::IntArrayRef dilation, bool channels_last) {
  check_act(x, "input");
  check_act(dy, "grad_output");
  ConvGeom g = geom(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(1), kh, kw, stride, padding, dilation);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3) && g.n == dy.size(0),
              "rtseg.conv_stem_wgrad: grad_output does not match the geometry");
  TORCH_CHECK(conv_stem_supported(g),
              "rtseg.conv_stem_wgrad: needs Cin == 3, 3 x 3 / pad 1 / stride 1 or 2, Cout % 16 == 0 and <= 64, even W");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  g.x = x.data_ptr(); g.y = dy.data_ptr();
  at::Tensor ws = at::empty({conv_stem_wgrad_ws_elems(g)}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({g.cout, g.cin, g.kh, g.kw},
                            x.options().dtype(at::kFloat).memory_format(channels_last ? at::MemoryFormat::ChannelsLast
                                                                                      : at::MemoryFormat::Contiguous));
  launch_conv_stem_wgrad(g, ws.data_ptr<float>(), dw.data_ptr<float>(), channels_last, cur_stream());
  return dw;
}

// stem weight gradient with the following BN's backward apply fused (conv_stem.hip, BNF):
// dy = gradient of act(BN(xb)), xb = this conv's output [N,Cout,Ho,Wo] CL bf16; kcoef [3 Cout],
// mean_invstd / scale_shift [2 Cout] fp32 from the BN (ops/bn.py); act 0 none / 1 ReLU / 2 ReLU6
at::Tensor conv_stem_wgrad_bn(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& xb,
                              const at::Tensor& kcoef, const at::Tensor& mean_invstd,
                              const at::Tensor& scale_shift, int64_t act, int64_t kh, int64_t kw,
                              at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation,
                              bool channels_last, const std::optional<at::Tensor>& wk) {
  check_act(x, "input");
  check_act(dy, "grad_output");
  const bool rc = wk.has_value() && wk->defined();  // recompute the BN input (xb may be a placeholder)
  if (!rc) check_act(xb, "bn_input");
  ConvGeom g = geom(x.size(0), x.size(1), x.size(2), x.size(3), dy.size(1), kh, kw, stride, padding, dilation);
  TORCH_CHECK(g.ho == dy.size(2) && g.wo == dy.size(3) && g.n == dy.size(0) && xb.sizes() == dy.sizes(),
              "rtseg.conv_stem_wgrad_bn: grad_output / bn_input do not match the geometry");
  TORCH_CHECK(conv_stem_supported(g) && g.cout % 16 == 0 && (g.cout / 16) != 3,
              "rtseg.conv_stem_wgrad_bn: needs the stem geometry and Cout of 16, 32 or 64");
  const int C = static_cast<int>(g.cout);
  auto fchk = [&](const at::Tensor& t, int64_t n, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n,
                "rtseg.conv_stem_wgrad_bn: ", what, " must be contiguous fp32 of ", n, " elements");
  };
  fchk(kcoef, 3 * C, "kcoef");
  fchk(mean_invstd, 2 * C, "mean_invstd");
  fchk(scale_shift, 2 * C, "scale_shift");
  TORCH_CHECK(act >= 0 && act <= 2, "rtseg.conv_stem_wgrad_bn: act must be 0, 1 or 2");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  g.x = x.data_ptr(); g.y = dy.data_ptr();
  at::Tensor ws = at::empty({conv_stem_wgrad_ws_elems(g)}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({g.cout, g.cin, g.kh, g.kw},
                            x.options().dtype(at::kFloat).memory_format(channels_last ? at::MemoryFormat::ChannelsLast
                                                                                      : at::MemoryFormat::Contiguous));
  if (rc)
    TORCH_CHECK(wk->is_cuda() && wk->scalar_type() == at::kBFloat16 && wk->is_contiguous() && wk->numel() == 27 * C,
                "rtseg.conv_stem_wgrad_bn: wk must be contiguous bf16 [Cout, 3, 3, 3]");
  StemBnBwd bn{rc ? nullptr : xb.data_ptr(), kcoef.data_ptr<float>(), mean_invstd.data_ptr<float>(),
               scale_shift.data_ptr<float>(), static_cast<int>(act)};
  if (rc) bn.w = wk->data_ptr();
  launch_conv_stem_wgrad(g, ws.data_ptr<float>(), dw.data_ptr<float>(), channels_last, cur_stream(), &bn);
  return dw;
}

}  // namespace
}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("conv_igemm(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, bool stats, "
        "Tensor? scale_shift, Tensor? residual, int act) -> (Tensor, Tensor)");
  m.def("conv_igemm_small(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, Tensor scale_shift, "
        "Tensor? residual, int act, bool split_k=False) -> Tensor");
  m.def("conv_igemm_dgrad(Tensor dy, Tensor wt, int[] x_size, int[] stride, int[] padding, int[] dilation, "
        "Tensor? bias=None, Tensor? addend=None, Tensor? addend_mask=None, Tensor? phase_addend=None, "
        "bool fused_phases=False) -> Tensor");
  m.def("conv_halo(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, bool stats, "
        "Tensor? scale_shift, Tensor? residual, int act) -> (Tensor, Tensor)");
  m.def("conv_halo_dgrad(Tensor dy, Tensor wt, int[] x_size, int[] stride, int[] padding, int[] dilation, "
        "Tensor? addend=None, Tensor? addend_mask=None) -> Tensor");
  m.def("conv_hreg(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, bool stats, "
        "int rows_per_wave=1) -> (Tensor, Tensor)");
  m.def("conv_hreg_dgrad(Tensor dy, Tensor wt, int[] x_size, int[] stride, int[] padding, int[] dilation, "
        "Tensor? addend=None, int rows_per_wave=1, Tensor? addend_mask=None) -> Tensor");
  m.def("conv_wres(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, bool stats) -> (Tensor, Tensor)");
  m.def("conv_wres_eval(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, Tensor scale_shift, "
        "Tensor? residual, int act) -> Tensor");
  m.def("conv_wres_dgrad(Tensor dy, Tensor wt, int[] x_size, int[] stride, int[] padding, int[] dilation, "
        "Tensor? addend=None, Tensor? addend_mask=None) -> Tensor");
  m.def("conv_stem(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, bool stats, bool store=True) "
        "-> (Tensor, Tensor)");
  m.def("conv_stem7(Tensor x, Tensor wk, int[] stride, Tensor? scale_shift, int act) -> Tensor");
  m.def("conv_stem_bn_act(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, Tensor scale_shift, "
        "int act) -> Tensor");
  m.def("conv_stem_bn_sums(Tensor x, Tensor wk, int[] stride, int[] padding, int[] dilation, Tensor dy, "
        "Tensor mean_invstd, Tensor scale_shift, int act) -> Tensor");
  m.def("conv_stem_wgrad_bn(Tensor x, Tensor dy, Tensor bn_input, Tensor kcoef, Tensor mean_invstd, "
        "Tensor scale_shift, int act, int kh, int kw, int[] stride, int[] padding, int[] dilation, "
        "bool channels_last, Tensor? wk=None) -> Tensor");
  m.def("conv_stem_wgrad(Tensor x, Tensor dy, int kh, int kw, int[] stride, int[] padding, int[] dilation, "
        "bool channels_last=False) -> Tensor");
  m.def("conv_whalo_wgrad(Tensor x, Tensor dy, int kh, int kw, int[] stride, int[] padding, int[] dilation, "
        "bool channels_last=False, int variant=1) -> Tensor");
  m.def("conv_igemm_wgrad(Tensor x, Tensor dy, int kh, int kw, int[] stride, int[] padding, int[] dilation, "
        "bool channels_last=False) -> Tensor");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("conv_igemm", &rtseg::conv_igemm);
  m.impl("conv_igemm_small", &rtseg::conv_igemm_small);
  m.impl("conv_wres_eval", &rtseg::conv_wres_eval);
  m.impl("conv_igemm_dgrad", &rtseg::conv_igemm_dgrad);
  m.impl("conv_halo", &rtseg::conv_halo);
  m.impl("conv_halo_dgrad", &rtseg::conv_halo_dgrad);
  m.impl("conv_hreg", &rtseg::conv_hreg);
  m.impl("conv_hreg_dgrad", &rtseg::conv_hreg_dgrad);
  m.impl("conv_wres", &rtseg::conv_wres);
  m.impl("conv_wres_dgrad", &rtseg::conv_wres_dgrad);
  m.impl("conv_igemm_wgrad", &rtseg::conv_igemm_wgrad);
  m.impl("conv_whalo_wgrad", &rtseg::conv_whalo_wgrad);
  m.impl("conv_stem", &rtseg::conv_stem);
  m.impl("conv_stem_bn_act", &rtseg::conv_stem_bn_act);
  m.impl("conv_stem7", &rtseg::conv_stem7);
  m.impl("conv_stem_bn_sums", &rtseg::conv_stem_bn_sums);
  m.impl("conv_stem_wgrad_bn", &rtseg::conv_stem_wgrad_bn);
  m.impl("conv_stem_wgrad", &rtseg::conv_stem_wgrad);
}
