// torch.library registration of the pooling operators (kernels: pool.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "rtseg_launch.h"
#include "rtseg_ops.h"

namespace rtseg {

static PoolParams pool_params(at::IntArrayRef k, at::IntArrayRef s, at::IntArrayRef p, int64_t mode,
                              bool count_include_pad, bool adaptive) {
  TORCH_CHECK(k.size() == 2 && s.size() == 2 && p.size() == 2, "rtseg.pool: kernel/stride/padding must have 2 entries");
  PoolParams pp{static_cast<int>(k[0]), static_cast<int>(k[1]), static_cast<int>(s[0]), static_cast<int>(s[1]),
                static_cast<int>(p[0]), static_cast<int>(p[1]), count_include_pad ? 1 : 0, static_cast<int>(mode),
                adaptive ? 1 : 0};
  if (!adaptive) {
    TORCH_CHECK(pp.kh > 0 && pp.kw > 0 && pp.sh > 0 && pp.sw > 0, "rtseg.pool: kernel and stride must be positive");
    TORCH_CHECK(pp.ph >= 0 && pp.pw >= 0 && 2 * pp.ph <= pp.kh && 2 * pp.pw <= pp.kw,
                "rtseg.pool: padding must be at most half the kernel");
  }
  TORCH_CHECK(mode == kPoolAvg || (mode == kPoolMax && !adaptive && pp.kh * pp.kw <= 256),
              "rtseg.pool: max pooling needs a fixed window of at most 256 taps");
  return pp;
}

static void check_x(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, "rtseg.pool: expected a 4-D GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf,
              "rtseg.pool: dtype must be fp32, bf16 or fp16");
  TORCH_CHECK(x.numel() < (int64_t{1} << 31), "rtseg.pool: tensor too large for 32-bit indexing");
}

// -> (y, idx); idx is a uint8 [N, OH, OW, C] argmax map for max pooling, empty otherwise
static std::tuple<at::Tensor, at::Tensor> pool2d_fwd(const at::Tensor& x, at::IntArrayRef kernel,
                                                     at::IntArrayRef stride, at::IntArrayRef padding, int64_t mode,
                                                     bool count_include_pad) {
  check_x(x);
  const PoolParams p = pool_params(kernel, stride, padding, mode, count_include_pad, false);
  const int64_t oh = (x.size(2) + 2 * p.ph - p.kh) / p.sh + 1;
  const int64_t ow = (x.size(3) + 2 * p.pw - p.kw) / p.sw + 1;
  TORCH_CHECK(oh > 0 && ow > 0, "rtseg.pool: output would be empty");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor y = at::empty({x.size(0), x.size(1), oh, ow}, x.options().memory_format(x.suggest_memory_format()));
  at::Tensor idx;
  if (mode == kPoolMax) idx = at::empty({x.size(0), oh, ow, x.size(1)}, x.options().dtype(at::kByte));
  else idx = at::empty({0}, x.options().dtype(at::kByte));
  launch_pool_fwd(view4(x), view4(y), p, mode == kPoolMax ? idx.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {y, idx};
}

// pool2d_fwd into a caller-owned output y (e.g. a channel slice of a concat buffer: the kernel
// indexes y by its strides, 16-byte vectors when the slice's offset and row stride allow) -> idx
static at::Tensor pool2d_fwd_out(const at::Tensor& x, const at::Tensor& y, at::IntArrayRef kernel,
                                 at::IntArrayRef stride, at::IntArrayRef padding, int64_t mode,
                                 bool count_include_pad) {
  check_x(x);
  check_x(y);
  const PoolParams p = pool_params(kernel, stride, padding, mode, count_include_pad, false);
  const int64_t oh = (x.size(2) + 2 * p.ph - p.kh) / p.sh + 1;
  const int64_t ow = (x.size(3) + 2 * p.pw - p.kw) / p.sw + 1;
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == x.size(1) && y.size(2) == oh && y.size(3) == ow,
              "rtseg.pool_fwd_out: output shape does not match the pooling geometry");
  TORCH_CHECK(y.scalar_type() == x.scalar_type() && y.device() == x.device(), "rtseg.pool_fwd_out: dtype/device");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor idx;
  if (mode == kPoolMax) idx = at::empty({x.size(0), oh, ow, x.size(1)}, x.options().dtype(at::kByte));
  else idx = at::empty({0}, x.options().dtype(at::kByte));
  launch_pool_fwd(view4(x), view4(y), p, mode == kPoolMax ? idx.data_ptr<uint8_t>() : nullptr, cur_stream());
  return idx;
}

static at::Tensor pool2d_bwd(const at::Tensor& gy, const at::Tensor& idx, int64_t in_h, int64_t in_w,
                             at::IntArrayRef kernel, at::IntArrayRef stride, at::IntArrayRef padding, int64_t mode,
                             bool count_include_pad) {
  check_x(gy);
  const PoolParams p = pool_params(kernel, stride, padding, mode, count_include_pad, false);
  TORCH_CHECK((in_h + 2 * p.ph - p.kh) / p.sh + 1 == gy.size(2) && (in_w + 2 * p.pw - p.kw) / p.sw + 1 == gy.size(3),
              "rtseg.pool_bwd: grad_output shape does not match the pooling geometry");
  if (mode == kPoolMax)
    TORCH_CHECK(idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.dim() == 4 &&
                    idx.size(0) == gy.size(0) && idx.size(1) == gy.size(2) && idx.size(2) == gy.size(3) &&
                    idx.size(3) == gy.size(1),
                "rtseg.pool_bwd: bad argmax map");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gy.device());
  at::Tensor gx =
      at::empty({gy.size(0), gy.size(1), in_h, in_w}, gy.options().memory_format(gy.suggest_memory_format()));
  launch_pool_bwd(view4(gy), view4(gx), p, mode == kPoolMax ? idx.data_ptr<uint8_t>() : nullptr, cur_stream());
  return gx;
}

static at::Tensor adaptive_avg_pool_fwd(const at::Tensor& x, int64_t out_h, int64_t out_w) {
  check_x(x);
  TORCH_CHECK(out_h > 0 && out_w > 0, "rtseg.adaptive_avg_pool: output size must be positive");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor y = at::empty({x.size(0), x.size(1), out_h, out_w}, x.options().memory_format(x.suggest_memory_format()));
  if (out_h == 1 && out_w == 1) {
    const Tensor4 xv = view4(x);
    const GapPlan pl = gap_plan(xv);
    at::Tensor part = at::empty({static_cast<int64_t>(pl.slices) * x.size(0) * x.size(1)}, x.options().dtype(at::kFloat));
    launch_gap_fwd(xv, view4(y), pl, part.data_ptr<float>(), cur_stream());
    return y;
  }
  const PoolParams p{1, 1, 1, 1, 0, 0, 1, kPoolAvg, 1};
  launch_pool_fwd(view4(x), view4(y), p, nullptr, cur_stream());
  return y;
}

static at::Tensor adaptive_avg_pool_bwd(const at::Tensor& gy, int64_t in_h, int64_t in_w, bool channels_last) {
  check_x(gy);
  c10::hip::HIPGuardMasqueradingAsCUDA g(gy.device());
  const auto fmt = channels_last ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  at::Tensor gx = at::empty({gy.size(0), gy.size(1), in_h, in_w}, gy.options().memory_format(fmt));
  const PoolParams p{1, 1, 1, 1, 0, 0, 1, kPoolAvg, 1};
  launch_pool_bwd(view4(gy), view4(gx), p, nullptr, cur_stream());
  return gx;
}

static Tensor4 idx_view(const at::Tensor& idx) {
  TORCH_CHECK(idx.is_cuda() && idx.dim() == 4 && idx.scalar_type() == at::kLong, "rtseg.unpool: indices must be int64 4-D");
  Tensor4 v{};
  v.data = idx.data_ptr();
  v.dtype = -1;
  v.n = static_cast<int>(idx.size(0)); v.c = static_cast<int>(idx.size(1));
  v.h = static_cast<int>(idx.size(2)); v.w = static_cast<int>(idx.size(3));
  v.sn = idx.stride(0); v.sc = idx.stride(1); v.sh = idx.stride(2); v.sw = idx.stride(3);
  return v;
}

// max pool with PyTorch-style int64 indices: (y, flat indices, uint8 window map for the backward)
static std::tuple<at::Tensor, at::Tensor, at::Tensor> max_pool_indices(const at::Tensor& x, at::IntArrayRef kernel,
                                                                       at::IntArrayRef stride, at::IntArrayRef padding) {
  auto [y, win] = pool2d_fwd(x, kernel, stride, padding, kPoolMax, true);
  const PoolParams p = pool_params(kernel, stride, padding, kPoolMax, true, false);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor idx = at::empty(y.sizes(), y.options().dtype(at::kLong).memory_format(y.suggest_memory_format()));
  launch_maxpool_flat_index(win.data_ptr<uint8_t>(), idx_view(idx), static_cast<int>(x.size(3)), p, cur_stream());
  return {y, idx, win};
}

// MaxUnpool2d with kernel == stride, no padding: y [N, C, out_h, out_w] gathered from x / idx
static at::Tensor max_unpool_fwd(const at::Tensor& x, const at::Tensor& idx, int64_t kh, int64_t kw, int64_t out_h,
                                 int64_t out_w) {
  check_x(x);
  TORCH_CHECK(idx.sizes() == x.sizes(), "rtseg.max_unpool: indices must match the input");
  TORCH_CHECK(kh > 0 && kw > 0 && out_h >= x.size(2) * kh - kh + 1 && out_w >= x.size(3) * kw - kw + 1,
              "rtseg.max_unpool: output too small for the windows");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor y = at::empty({x.size(0), x.size(1), out_h, out_w}, x.options().memory_format(x.suggest_memory_format()));
  launch_unpool_gather(view4(x), idx_view(idx), view4(y), static_cast<int>(kh), static_cast<int>(kw), cur_stream());
  return y;
}

// backward of max_unpool_fwd: gx[n, c, i, j] = gy at the plane position idx[n, c, i, j]
static at::Tensor max_unpool_bwd(const at::Tensor& gy, const at::Tensor& idx) {
  check_x(gy);
  c10::hip::HIPGuardMasqueradingAsCUDA g(gy.device());
  at::Tensor gx = at::empty(idx.sizes(), gy.options().memory_format(gy.suggest_memory_format()));
  launch_unpool_bwd(view4(gy), idx_view(idx), view4(gx), cur_stream());
  return gx;
}

// AdaptiveMaxPool2d(1): (y [N, C, 1, 1], idx int64 [N, C, 1, 1])
static std::tuple<at::Tensor, at::Tensor> global_max_pool(const at::Tensor& x) {
  check_x(x);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor y = at::empty({x.size(0), x.size(1), 1, 1}, x.options());
  at::Tensor idx = at::empty({x.size(0), x.size(1), 1, 1}, x.options().dtype(at::kLong));
  launch_global_max(view4(x), y.data_ptr(), idx.data_ptr<int64_t>(), cur_stream());
  return {y, idx};
}

}  // namespace rtseg

TORCH_LIBRARY_FRAGMENT(rtseg, m) {
  m.def("global_max_pool(Tensor x) -> (Tensor, Tensor)");
  m.def("max_pool_indices(Tensor x, int[] kernel, int[] stride, int[] padding) -> (Tensor, Tensor, Tensor)");
  m.def("max_unpool_fwd(Tensor x, Tensor idx, int kh, int kw, int out_h, int out_w) -> Tensor");
  m.def("max_unpool_bwd(Tensor gy, Tensor idx) -> Tensor");
  m.def("pool2d_fwd(Tensor x, int[] kernel, int[] stride, int[] padding, int mode, bool count_include_pad) "
        "-> (Tensor, Tensor)");
  m.def("pool2d_fwd_out(Tensor x, Tensor(a!) y, int[] kernel, int[] stride, int[] padding, int mode, "
        "bool count_include_pad) -> Tensor");
  m.def("pool2d_bwd(Tensor gy, Tensor idx, int in_h, int in_w, int[] kernel, int[] stride, int[] padding, int mode, "
        "bool count_include_pad) -> Tensor");
  m.def("adaptive_avg_pool_fwd(Tensor x, int out_h, int out_w) -> Tensor");
  m.def("adaptive_avg_pool_bwd(Tensor gy, int in_h, int in_w, bool channels_last) -> Tensor");
}

TORCH_LIBRARY_IMPL(rtseg, CUDA, m) {
  m.impl("pool2d_fwd", &rtseg::pool2d_fwd);
  m.impl("pool2d_fwd_out", &rtseg::pool2d_fwd_out);
  m.impl("pool2d_bwd", &rtseg::pool2d_bwd);
  m.impl("adaptive_avg_pool_fwd", &rtseg::adaptive_avg_pool_fwd);
  m.impl("adaptive_avg_pool_bwd", &rtseg::adaptive_avg_pool_bwd);
  m.impl("max_pool_indices", &rtseg::max_pool_indices);
  m.impl("max_unpool_fwd", &rtseg::max_unpool_fwd);
  m.impl("max_unpool_bwd", &rtseg::max_unpool_bwd);
  m.impl("global_max_pool", &rtseg::global_max_pool);
}
