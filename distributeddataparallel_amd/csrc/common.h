// Shared helpers for the xddp native layer (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <torch/extension.h>

#include <chrono>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>

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

// Opt a kernel in to `lds` bytes (> 64 KiB) of dynamic LDS, once per kernel: the attribute is a
// property of the function, so the cache is keyed by the kernel pointer (one static per launch
// site would skip the call for a second kernel launched from the same site with less LDS).
inline void ensure_dyn_lds(const void* kern, size_t lds) {
  if (lds <= 65536) return;
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> done;
  std::lock_guard<std::mutex> g(mu);
  size_t& cur = done[kern];
  if (lds <= cur) return;
  XDDP_HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  cur = lds;
}

// Reduction ops, numbered like c10d::ReduceOp::RedOpType so Python enums line up.
enum class RedOp : int { SUM = 0, AVG = 1, PRODUCT = 2, MIN = 3, MAX = 4, BAND = 5, BOR = 6, BXOR = 7, PREMUL_SUM = 8 };

}  // namespace xddp
