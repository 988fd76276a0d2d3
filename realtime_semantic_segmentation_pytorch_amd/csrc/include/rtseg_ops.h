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
}  // namespace rtseg
