// Helpers shared by the torch-facing binding translation units (binding*.cpp).
// Additional op groups register through TORCH_LIBRARY_FRAGMENT(rtseg, m).
#pragma once

#include <ATen/ATen.h>
#include <hip/hip_runtime_api.h>

#include "rtseg_launch.h"

namespace rtseg {
int dtype_code(const at::Tensor& t);
Tensor4 view4(const at::Tensor& t);
hipStream_t cur_stream();

// Scratch of the BN finalize row-split pre-pass (bn_slab_splits): nullptr when the slab is short.
struct SlabScratch {
  at::Tensor t;
  SlabScratch(int G, int C, const at::Tensor& like) {
    const int S = bn_slab_splits(G);
    if (S > 1) t = at::empty({static_cast<int64_t>(S) * 2 * C}, like.options().dtype(at::kDouble));
  }
  double* ptr() const { return t.defined() ? t.data_ptr<double>() : nullptr; }
};
}  // namespace rtseg
