// Normalization kernels (BatchNorm NHWC, LayerNorm, RMSNorm) for gfx950.
#pragma once

#include <pybind11/pybind11.h>

namespace xddp {
namespace kernels {

void bind_norm_kernels(pybind11::module_& m);

}  // namespace kernels
}  // namespace xddp
