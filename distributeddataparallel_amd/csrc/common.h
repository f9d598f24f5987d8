// Shared helpers for the xddp native layer (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <torch/extension.h>

#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string>

#define XDDP_HIP_CHECK(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ", __FILE__, \
                ":", __LINE__, " (" #expr ")");                                       \
  } while (0)

namespace xddp {

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Reduction ops, numbered like c10d::ReduceOp::RedOpType so Python enums line up.
enum class RedOp : int { SUM = 0, AVG = 1, PRODUCT = 2, MIN = 3, MAX = 4, BAND = 5, BOR = 6, BXOR = 7, PREMUL_SUM = 8 };

}  // namespace xddp
