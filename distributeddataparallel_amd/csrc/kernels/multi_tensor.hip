// Multi-tensor HIP kernels for the DDP hot path on gfx950 (CDNA4).
//
// One launch walks a list of up to kMaxSeg tensors described in the kernel-argument
// segment table (no H2D upload, so the launch is graph-capturable). Every block owns a
// fixed 8192-element chunk of one segment; each lane moves 8 elements per iteration with
// 16-byte loads/stores (Guideline 13) and converts dtypes in registers (bf16 through
// v_cvt_pk_bf16_f32). Grids are thousands of blocks for MB-sized buckets, well past the
// 256 CUs.
#include "kernels/multi_tensor.h"

#include <ATen/hip/HIPContext.h>

#include <algorithm>
#include <type_traits>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

using dev::bf16_t;
using dev::f16_t;
using dev::Elem;
using dev::Vec8;

constexpr int kThreads = 256;
constexpr int kIters = 4;
constexpr int64_t kChunk = (int64_t)kThreads * 8 * kIters;  // elements per block
constexpr int kMaxSeg = 40;

template <int NPTR>
struct SegTable {
  void* ptr[NPTR][kMaxSeg];
  int64_t numel[kMaxSeg];
  int32_t blk_end[kMaxSeg];  // inclusive prefix sum of blocks per segment
  int32_t nseg;
};

template <int NPTR>
__device__ __forceinline__ int find_seg(const SegTable<NPTR>& t, int b) {
  // wave-uniform binary search over the (kernarg-resident) prefix array
  int lo = 0, hi = t.nseg - 1;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (b < t.blk_end[mid]) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// Builds segment tables and launches `launch(table, nblocks)` whenever one fills.
template <int NPTR, typename F>
static void for_each_table(const std::vector<std::array<void*, NPTR>>& ptrs, const std::vector<int64_t>& numels,
                           F&& launch) {
  SegTable<NPTR> t;
  t.nseg = 0;
  int32_t blocks = 0;
  for (size_t i = 0; i < ptrs.size(); ++i) {
    const int64_t n = numels[i];
    if (n == 0) continue;
    int64_t nb = (n + kChunk - 1) / kChunk;
    TORCH_CHECK(nb < (int64_t)(1 << 30), "tensor too large for multi-tensor launch");
    if (t.nseg == kMaxSeg || (int64_t)blocks + nb > (int64_t)(1 << 30)) {
      launch(t, blocks);
      t.nseg = 0;
      blocks = 0;
    }
    for (int p = 0; p < NPTR; ++p) t.ptr[p][t.nseg] = ptrs[i][p];
    t.numel[t.nseg] = n;
    blocks += (int32_t)nb;
    t.blk_end[t.nseg] = blocks;
    t.nseg++;
  }
  if (t.nseg) launch(t, blocks);
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ------------------------------------------------------------------------------------
// scale-copy: dst = cast(src * scale * (*sp))
// ------------------------------------------------------------------------------------
template <typename Ti, typename To, bool VEC>
__global__ __launch_bounds__(kThreads) void scale_copy_kernel(SegTable<2> t, float scale, const float* sp) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  const Ti* __restrict__ src = reinterpret_cast<const Ti*>(t.ptr[0][s]);
  To* __restrict__ dst = reinterpret_cast<To*>(t.ptr[1][s]);
  const int64_t n = t.numel[s];
  const float sc = sp ? scale * (*sp) : scale;
  const int64_t base = blk * kChunk;
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
    if (VEC && i + 8 <= n) {
      float v[8];
      Vec8<Ti>::ld(src + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= sc;
      Vec8<To>::st(dst + i, v);
    } else {
      for (int64_t k = i; k < i + 8 && k < n; ++k)
        Elem<To, float>::st(dst, k, Elem<Ti, float>::ld(src, k) * sc);
    }
  }
}

template <typename Ti, typename To>
__global__ __launch_bounds__(kThreads) void scale_copy_kernel_f64(SegTable<2> t, double scale, const float* sp) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  const Ti* src = reinterpret_cast<const Ti*>(t.ptr[0][s]);
  To* dst = reinterpret_cast<To*>(t.ptr[1][s]);
  const int64_t n = t.numel[s];
  const double sc = sp ? scale * (double)(*sp) : scale;
  for (int64_t k = blk * kChunk + threadIdx.x; k < std::min(n, (blk + 1) * kChunk); k += kThreads)
    Elem<To, double>::st(dst, k, Elem<Ti, double>::ld(src, k) * sc);
}

template <typename T>
struct DevType {
  using type = T;
};
template <>
struct DevType<at::BFloat16> {
  using type = bf16_t;
};
template <>
struct DevType<at::Half> {
  using type = f16_t;
};

#define XDDP_DISPATCH_FLOAT(st, NAME, ...)                                     \
  switch (st) {                                                                \
    case at::kFloat: { using NAME = float; __VA_ARGS__; break; }               \
    case at::kBFloat16: { using NAME = bf16_t; __VA_ARGS__; break; }           \
    case at::kHalf: { using NAME = f16_t; __VA_ARGS__; break; }                \
    case at::kDouble: { using NAME = double; __VA_ARGS__; break; }             \
    default: TORCH_CHECK(false, "xddp multi-tensor: unsupported dtype ", st);  \
  }

// ------------------------------------------------------------------------------------
// byte-exact copy (any dtype, bit patterns preserved): "numel" is bytes; a block owns
// kChunk bytes, 16 B per lane per iteration when both ends of the segment are aligned.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void copy_bytes_kernel(SegTable<2> t) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  const char* __restrict__ src = reinterpret_cast<const char*>(t.ptr[0][s]);
  char* __restrict__ dst = reinterpret_cast<char*>(t.ptr[1][s]);
  const int64_t n = t.numel[s];
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  constexpr int kIt = kChunk / (kThreads * 16);
  const int64_t base = blk * kChunk;
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 16;
    if (vec && i + 16 <= n) {
      *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
      for (int64_t k = i; k < i + 16 && k < n; ++k) dst[k] = src[k];
    }
  }
}

void mt_copy_bytes(const std::vector<const void*>& src, const std::vector<void*>& dst,
                   const std::vector<int64_t>& nbytes, hipStream_t stream) {
  TORCH_CHECK(src.size() == dst.size() && src.size() == nbytes.size(), "copy_bytes: list length mismatch");
  std::vector<std::array<void*, 2>> ptrs;
  for (size_t i = 0; i < src.size(); ++i) ptrs.push_back({const_cast<void*>(src[i]), dst[i]});
  for_each_table<2>(ptrs, nbytes, [&](const SegTable<2>& t, int32_t nb) {
    hipLaunchKernelGGL(copy_bytes_kernel, dim3(nb), dim3(kThreads), 0, stream, t);
    XDDP_HIP_CHECK(hipGetLastError());
  });
}

static void check_dense_pair(const at::Tensor& a, const at::Tensor& b) {
  TORCH_CHECK(a.numel() == b.numel(), "numel mismatch ", a.numel(), " vs ", b.numel());
  TORCH_CHECK(a.is_non_overlapping_and_dense() && b.is_non_overlapping_and_dense(),
              "multi-tensor copy needs dense tensors");
  if (a.dim() > 0 && a.numel() > 1) TORCH_CHECK(a.strides() == b.strides() || (a.is_contiguous() && b.is_contiguous()),
              "multi-tensor copy needs identical memory order");
}

static void launch_scale_copy(const std::vector<std::array<void*, 2>>& ptrs, const std::vector<int64_t>& numels,
                              at::ScalarType ti, at::ScalarType to, double scale, const float* sp,
                              hipStream_t stream) {
  bool vec = true;
  for (auto& p : ptrs) vec = vec && aligned16(p[0]) && aligned16(p[1]);
  const bool f64 = (ti == at::kDouble || to == at::kDouble);
  XDDP_DISPATCH_FLOAT(ti, Ti, XDDP_DISPATCH_FLOAT(to, To, {
    for_each_table<2>(ptrs, numels, [&](const SegTable<2>& t, int32_t nb) {
      if (f64)
        hipLaunchKernelGGL((scale_copy_kernel_f64<Ti, To>), dim3(nb), dim3(kThreads), 0, stream, t, scale, sp);
      else if (vec)
        hipLaunchKernelGGL((scale_copy_kernel<Ti, To, true>), dim3(nb), dim3(kThreads), 0, stream, t, (float)scale, sp);
      else
        hipLaunchKernelGGL((scale_copy_kernel<Ti, To, false>), dim3(nb), dim3(kThreads), 0, stream, t, (float)scale, sp);
      XDDP_HIP_CHECK(hipGetLastError());
    });
  }));
}

static const float* scale_ptr(const c10::optional<at::Tensor>& st) {
  if (!st.has_value() || !st->defined()) return nullptr;
  TORCH_CHECK(st->scalar_type() == at::kFloat && st->is_cuda(), "scale tensor must be a float32 device tensor");
  return st->data_ptr<float>();
}

void mt_scale_copy(const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst, double scale,
                   const c10::optional<at::Tensor>& scale_tensor, hipStream_t stream) {
  TORCH_CHECK(src.size() == dst.size(), "src/dst list length mismatch");
  if (src.empty()) return;
  std::vector<std::array<void*, 2>> ptrs;
  std::vector<int64_t> numels;
  ptrs.reserve(src.size());
  numels.reserve(src.size());
  const auto ti = src[0].scalar_type(), to = dst[0].scalar_type();
  for (size_t i = 0; i < src.size(); ++i) {
    TORCH_CHECK(src[i].scalar_type() == ti && dst[i].scalar_type() == to, "mixed dtypes in tensor list");
    TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda(), "mt_scale_copy expects device tensors");
    check_dense_pair(src[i], dst[i]);
    ptrs.push_back({const_cast<void*>(src[i].data_ptr()), dst[i].data_ptr()});
    numels.push_back(src[i].numel());
  }
  launch_scale_copy(ptrs, numels, ti, to, scale, scale_ptr(scale_tensor), stream);
}

void mt_pack(const std::vector<at::Tensor>& src, const at::Tensor& flat, const std::vector<int64_t>& offsets,
             double scale, hipStream_t stream) {
  TORCH_CHECK(src.size() == offsets.size(), "pack: offsets length mismatch");
  if (src.empty()) return;
  TORCH_CHECK(flat.is_contiguous(), "pack target must be contiguous");
  const auto ti = src[0].scalar_type(), to = flat.scalar_type();
  const int64_t es = flat.element_size();
  std::vector<std::array<void*, 2>> ptrs;
  std::vector<int64_t> numels;
  for (size_t i = 0; i < src.size(); ++i) {
    TORCH_CHECK(src[i].scalar_type() == ti, "mixed dtypes in pack list");
    TORCH_CHECK(src[i].is_non_overlapping_and_dense(), "pack source must be dense");
    TORCH_CHECK(offsets[i] + src[i].numel() <= flat.numel(), "pack overflows target");
    ptrs.push_back({const_cast<void*>(src[i].data_ptr()), static_cast<char*>(flat.data_ptr()) + offsets[i] * es});
    numels.push_back(src[i].numel());
  }
  launch_scale_copy(ptrs, numels, ti, to, scale, nullptr, stream);
}

void mt_unpack(const at::Tensor& flat, const std::vector<int64_t>& offsets, const std::vector<at::Tensor>& dst,
               double scale, hipStream_t stream) {
  TORCH_CHECK(dst.size() == offsets.size(), "unpack: offsets length mismatch");
  if (dst.empty()) return;
  TORCH_CHECK(flat.is_contiguous(), "unpack source must be contiguous");
  const auto ti = flat.scalar_type(), to = dst[0].scalar_type();
  const int64_t es = flat.element_size();
  std::vector<std::array<void*, 2>> ptrs;
  std::vector<int64_t> numels;
  for (size_t i = 0; i < dst.size(); ++i) {
    TORCH_CHECK(dst[i].scalar_type() == to, "mixed dtypes in unpack list");
    TORCH_CHECK(dst[i].is_non_overlapping_and_dense(), "unpack target must be dense");
    TORCH_CHECK(offsets[i] + dst[i].numel() <= flat.numel(), "unpack overflows source");
    ptrs.push_back({static_cast<char*>(flat.data_ptr()) + offsets[i] * es, dst[i].data_ptr()});
    numels.push_back(dst[i].numel());
  }
  launch_scale_copy(ptrs, numels, ti, to, scale, nullptr, stream);
}

// ------------------------------------------------------------------------------------
// L2 norm (deterministic two-pass: per-block partials, then one block folds them)
// ------------------------------------------------------------------------------------
template <typename T, bool VEC>
__global__ __launch_bounds__(kThreads) void sumsq_kernel(SegTable<1> t, float* partials, int32_t part_off) {
  __shared__ float scratch[kThreads / 64];
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  const T* x = reinterpret_cast<const T*>(t.ptr[0][s]);
  const int64_t n = t.numel[s];
  const int64_t base = blk * kChunk;
  float acc = 0.f;
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
    if (VEC && i + 8 <= n) {
      float v[8];
      Vec8<T>::ld(x + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(v[j], v[j], acc);
    } else {
      for (int64_t k = i; k < i + 8 && k < n; ++k) {
        float v = Elem<T, float>::ld(x, k);
        acc = fmaf(v, v, acc);
      }
    }
  }
  acc = dev::block_sum(acc, scratch);
  if (threadIdx.x == 0) partials[part_off + blockIdx.x] = acc;
}

__global__ __launch_bounds__(1024) void norm_finalize_kernel(const float* partials, int64_t n, float* out,
                                                             float max_norm) {
  __shared__ float scratch[1024 / 64];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  acc = dev::block_sum(acc, scratch);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(acc);
    out[0] = norm;
    if (max_norm > 0.f) out[1] = fminf(1.f, max_norm / (norm + 1e-6f));
  }
}

void mt_l2norm(const std::vector<at::Tensor>& tensors, const at::Tensor& out, double max_norm, hipStream_t stream) {
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 2 && out.is_cuda(), "out must be float32[>=2] on device");
  if (tensors.empty()) {
    out.zero_();
    if (max_norm > 0) out.narrow(0, 1, 1).fill_(1.0);
    return;
  }
  const auto st = tensors[0].scalar_type();
  std::vector<std::array<void*, 1>> ptrs;
  std::vector<int64_t> numels;
  int64_t total_blocks = 0;
  bool vec = true;
  for (auto& x : tensors) {
    TORCH_CHECK(x.scalar_type() == st, "mixed dtypes in norm list");
    TORCH_CHECK(x.is_non_overlapping_and_dense(), "norm needs dense tensors");
    ptrs.push_back({const_cast<void*>(x.data_ptr())});
    numels.push_back(x.numel());
    total_blocks += (x.numel() + kChunk - 1) / kChunk;
    vec = vec && aligned16(x.data_ptr());
  }
  auto partials = at::empty({std::max<int64_t>(total_blocks, 1)}, out.options());
  int32_t off = 0;
  XDDP_DISPATCH_FLOAT(st, T, {
    for_each_table<1>(ptrs, numels, [&](const SegTable<1>& t, int32_t nb) {
      if (vec)
        hipLaunchKernelGGL((sumsq_kernel<T, true>), dim3(nb), dim3(kThreads), 0, stream, t, partials.data_ptr<float>(), off);
      else
        hipLaunchKernelGGL((sumsq_kernel<T, false>), dim3(nb), dim3(kThreads), 0, stream, t, partials.data_ptr<float>(), off);
      XDDP_HIP_CHECK(hipGetLastError());
      off += nb;
    });
  });
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(1024), 0, stream, partials.data_ptr<float>(), (int64_t)off,
                     out.data_ptr<float>(), (float)max_norm);
  XDDP_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------
// non-finite check (TORCH_NCCL_NAN_CHECK analogue)
// ------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads) void nonfinite_kernel(SegTable<1> t, int* flag) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  const T* x = reinterpret_cast<const T*>(t.ptr[0][s]);
  const int64_t n = t.numel[s];
  bool bad = false;
  for (int64_t k = blk * kChunk + threadIdx.x; k < std::min(n, (blk + 1) * kChunk); k += kThreads) {
    float v = Elem<T, float>::ld(x, k);
    bad |= !isfinite(v);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

void mt_nonfinite(const std::vector<at::Tensor>& tensors, const at::Tensor& out, hipStream_t stream) {
  TORCH_CHECK(out.scalar_type() == at::kInt && out.is_cuda(), "flag must be int32 device tensor");
  XDDP_HIP_CHECK(hipMemsetAsync(out.data_ptr(), 0, sizeof(int), stream));
  if (tensors.empty()) return;
  const auto st = tensors[0].scalar_type();
  std::vector<std::array<void*, 1>> ptrs;
  std::vector<int64_t> numels;
  for (auto& x : tensors) {
    TORCH_CHECK(x.scalar_type() == st && x.is_non_overlapping_and_dense(), "nonfinite: dense, single dtype");
    ptrs.push_back({const_cast<void*>(x.data_ptr())});
    numels.push_back(x.numel());
  }
  XDDP_DISPATCH_FLOAT(st, T, {
    for_each_table<1>(ptrs, numels, [&](const SegTable<1>& t, int32_t nb) {
      hipLaunchKernelGGL((nonfinite_kernel<T>), dim3(nb), dim3(kThreads), 0, stream, t, out.data_ptr<int>());
      XDDP_HIP_CHECK(hipGetLastError());
    });
  });
}

// ------------------------------------------------------------------------------------
// replica checksum: fp64 sum of the values + XOR of a 64-bit mix of every element's raw bits with
// its (tensor, index) position, over a list of tensors of any dtypes. Per-block partials are
// written at fixed slots and merged by one block in a fixed order, so equal bytes on two ranks
// give bit-equal checksums (the DDP replica check compares them across ranks).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {  // splitmix64 finalizer
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
template <typename T>
__device__ __forceinline__ unsigned long long raw_bits(const T* x, int64_t k) {
  if constexpr (sizeof(T) == 8) return reinterpret_cast<const unsigned long long*>(x)[k];
  else if constexpr (sizeof(T) == 4) return reinterpret_cast<const uint32_t*>(x)[k];
  else if constexpr (sizeof(T) == 2) return reinterpret_cast<const uint16_t*>(x)[k];
  else return reinterpret_cast<const uint8_t*>(x)[k];
}
template <typename T>
__device__ __forceinline__ double as_double(const T* x, int64_t k) {
  if constexpr (std::is_same<T, bf16_t>::value || std::is_same<T, f16_t>::value) return (double)Elem<T, float>::ld(x, k);
  else return (double)x[k];
}

template <typename T>
__global__ __launch_bounds__(kThreads) void checksum_kernel(SegTable<2> t, double* psum, unsigned long long* phash,
                                                            int32_t off) {
  __shared__ double ssum[kThreads / 64];
  __shared__ unsigned long long shash[kThreads / 64];
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  const T* x = reinterpret_cast<const T*>(t.ptr[0][s]);
  const unsigned long long seed = mix64(reinterpret_cast<uintptr_t>(t.ptr[1][s]) + 0x9e3779b97f4a7c15ull);
  const int64_t n = t.numel[s];
  double acc = 0.0;
  unsigned long long h = 0ull;
  const int64_t end = std::min(n, (blk + 1) * kChunk);
  for (int64_t k = blk * kChunk + threadIdx.x; k < end; k += kThreads) {
    acc += as_double(x, k);
    h ^= mix64(raw_bits(x, k) ^ mix64(seed + (unsigned long long)k));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    acc += __shfl_xor(acc, o, 64);
    h ^= __shfl_xor(h, o, 64);
  }
  if (lane == 0) {
    ssum[wid] = acc;
    shash[wid] = h;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    unsigned long long hh = 0ull;
    for (int w = 0; w < kThreads / 64; ++w) {
      a += ssum[w];
      hh ^= shash[w];
    }
    psum[off + blockIdx.x] = a;
    phash[off + blockIdx.x] = hh;
  }
}

// one block, fixed order: out = [sum, hash low 32 bits, hash high 32 bits] as float64 (exact)
__global__ __launch_bounds__(kThreads) void checksum_finalize_kernel(const double* psum, const unsigned long long* phash,
                                                                     int64_t n, double* out) {
  __shared__ double ssum[kThreads];
  __shared__ unsigned long long shash[kThreads];
  double a = 0.0;
  unsigned long long h = 0ull;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) {
    a += psum[i];
    h ^= phash[i];
  }
  ssum[threadIdx.x] = a;
  shash[threadIdx.x] = h;
  __syncthreads();
  for (int st = kThreads / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      ssum[threadIdx.x] += ssum[threadIdx.x + st];
      shash[threadIdx.x] ^= shash[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = ssum[0];
    out[1] = (double)(shash[0] & 0xffffffffull);
    out[2] = (double)(shash[0] >> 32);
  }
}

at::Tensor mt_checksum(const std::vector<at::Tensor>& tensors, hipStream_t stream) {
  TORCH_CHECK(!tensors.empty(), "checksum of an empty tensor list");
  const auto dev = tensors[0].device();
  auto out = at::zeros({3}, at::TensorOptions().dtype(at::kDouble).device(dev));
  int64_t total_blocks = 0;
  for (auto& x : tensors) {
    TORCH_CHECK(x.device() == dev && x.is_non_overlapping_and_dense(), "checksum: dense tensors on one device");
    total_blocks += (x.numel() + kChunk - 1) / kChunk;
  }
  auto psum = at::empty({std::max<int64_t>(total_blocks, 1)}, out.options());
  auto phash = at::empty({std::max<int64_t>(total_blocks, 1)}, out.options().dtype(at::kLong));
  int32_t off = 0;
  // one table per dtype; the tensor's position in the list seeds its mix (order-sensitive)
  std::vector<at::ScalarType> seen;
  for (auto& x0 : tensors)
    if (std::find(seen.begin(), seen.end(), x0.scalar_type()) == seen.end()) seen.push_back(x0.scalar_type());
  for (auto st : seen) {
    std::vector<std::array<void*, 2>> ptrs;
    std::vector<int64_t> numels;
    for (size_t i = 0; i < tensors.size(); ++i) {
      if (tensors[i].scalar_type() != st) continue;
      ptrs.push_back({const_cast<void*>(tensors[i].data_ptr()), reinterpret_cast<void*>((uintptr_t)(i + 1))});
      numels.push_back(tensors[i].numel());
    }
    auto launch = [&](auto tag) {
      using T = decltype(tag);
      for_each_table<2>(ptrs, numels, [&](const SegTable<2>& t, int32_t nb) {
        hipLaunchKernelGGL((checksum_kernel<T>), dim3(nb), dim3(kThreads), 0, stream, t, psum.data_ptr<double>(),
                           reinterpret_cast<unsigned long long*>(phash.data_ptr<int64_t>()), off);
        XDDP_HIP_CHECK(hipGetLastError());
        off += nb;
      });
    };
    switch (st) {
      case at::kFloat: launch(float{}); break;
      case at::kBFloat16: launch(bf16_t{}); break;
      case at::kHalf: launch(f16_t{}); break;
      case at::kDouble: launch(double{}); break;
      case at::kLong: launch(int64_t{}); break;
      case at::kInt: launch(int32_t{}); break;
      case at::kShort: launch(int16_t{}); break;
      case at::kByte: launch(uint8_t{}); break;
      case at::kChar: launch(int8_t{}); break;
      case at::kBool: launch(uint8_t{}); break;
      default: TORCH_CHECK(false, "checksum: unsupported dtype ", st);
    }
  }
  hipLaunchKernelGGL(checksum_finalize_kernel, dim3(1), dim3(kThreads), 0, stream, psum.data_ptr<double>(),
                     reinterpret_cast<const unsigned long long*>(phash.data_ptr<int64_t>()), (int64_t)off,
                     out.data_ptr<double>());
  XDDP_HIP_CHECK(hipGetLastError());
  return out;
}

// ------------------------------------------------------------------------------------
// Fused SGD: slots {param, grad, momentum_buf}
// ------------------------------------------------------------------------------------
template <typename P, typename G, bool VEC, bool MOM>
__global__ __launch_bounds__(kThreads) void sgd_kernel(SegTable<3> t, float lr, float momentum, float dampening,
                                                       float wd, bool nesterov, bool maximize, bool first,
                                                       const float* gs) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  P* p = reinterpret_cast<P*>(t.ptr[0][s]);
  const G* g = reinterpret_cast<const G*>(t.ptr[1][s]);
  float* buf = reinterpret_cast<float*>(t.ptr[2][s]);
  const int64_t n = t.numel[s];
  const float gscale = (gs ? *gs : 1.f) * (maximize ? -1.f : 1.f);
  const int64_t base = blk * kChunk;
  auto upd = [&](float& pv, float gv, float& bv) {
    float d = gv * gscale;
    if (wd != 0.f) d = fmaf(wd, pv, d);
    if (MOM) {
      bv = first ? d : fmaf(momentum, bv, (1.f - dampening) * d);
      d = nesterov ? fmaf(momentum, bv, d) : bv;
    }
    pv = fmaf(-lr, d, pv);
  };
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
    if (VEC && i + 8 <= n) {
      float pv[8], gv[8], bv[8];
      Vec8<P>::ld(p + i, pv);
      Vec8<G>::ld(g + i, gv);
      if (MOM && !first) Vec8<float>::ld(buf + i, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) upd(pv[j], gv[j], bv[j]);
      Vec8<P>::st(p + i, pv);
      if (MOM) Vec8<float>::st(buf + i, bv);
    } else {
      for (int64_t k = i; k < i + 8 && k < n; ++k) {
        float pv = Elem<P, float>::ld(p, k), gv = Elem<G, float>::ld(g, k), bv = 0.f;
        if (MOM && !first) bv = buf[k];
        upd(pv, gv, bv);
        Elem<P, float>::st(p, k, pv);
        if (MOM) buf[k] = bv;
      }
    }
  }
}

// Master-weight SGD: slots {fp32 master, grad, fp32 momentum, low-precision model param}. The
// updated master is rounded into the model's param in the same pass (no second launch that
// re-reads the masters).
template <typename G, typename Mdl, bool VEC, bool MOM>
__global__ __launch_bounds__(kThreads) void sgd_master_kernel(SegTable<4> t, float lr, float momentum,
                                                              float dampening, float wd, bool nesterov,
                                                              bool maximize, bool first, const float* gs) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  float* p = reinterpret_cast<float*>(t.ptr[0][s]);
  const G* g = reinterpret_cast<const G*>(t.ptr[1][s]);
  float* buf = reinterpret_cast<float*>(t.ptr[2][s]);
  Mdl* q = reinterpret_cast<Mdl*>(t.ptr[3][s]);
  const int64_t n = t.numel[s];
  const float gscale = (gs ? *gs : 1.f) * (maximize ? -1.f : 1.f);
  const int64_t base = blk * kChunk;
  auto upd = [&](float& pv, float gv, float& bv) {
    float d = gv * gscale;
    if (wd != 0.f) d = fmaf(wd, pv, d);
    if (MOM) {
      bv = first ? d : fmaf(momentum, bv, (1.f - dampening) * d);
      d = nesterov ? fmaf(momentum, bv, d) : bv;
    }
    pv = fmaf(-lr, d, pv);
  };
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
    if (VEC && i + 8 <= n) {
      float pv[8], gv[8], bv[8];
      Vec8<float>::ld(p + i, pv);
      Vec8<G>::ld(g + i, gv);
      if (MOM && !first) Vec8<float>::ld(buf + i, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) upd(pv[j], gv[j], bv[j]);
      Vec8<float>::st(p + i, pv);
      if (MOM) Vec8<float>::st(buf + i, bv);
      Vec8<Mdl>::st(q + i, pv);
    } else {
      for (int64_t k = i; k < i + 8 && k < n; ++k) {
        float pv = p[k], gv = Elem<G, float>::ld(g, k), bv = 0.f;
        if (MOM && !first) bv = buf[k];
        upd(pv, gv, bv);
        p[k] = pv;
        if (MOM) buf[k] = bv;
        Elem<Mdl, float>::st(q, k, pv);
      }
    }
  }
}

void fused_sgd_master(const std::vector<at::Tensor>& masters, const std::vector<at::Tensor>& grads,
                      const std::vector<at::Tensor>& momentum_bufs, const std::vector<at::Tensor>& model_params,
                      double lr, double momentum, double dampening, double weight_decay, bool nesterov, bool maximize,
                      bool first_step, const c10::optional<at::Tensor>& grad_scale, hipStream_t stream) {
  TORCH_CHECK(masters.size() == grads.size() && masters.size() == model_params.size(), "SGD list length mismatch");
  const bool mom = momentum != 0.0;
  TORCH_CHECK(!mom || momentum_bufs.size() == masters.size(), "momentum buffers missing");
  if (masters.empty()) return;
  const auto gt = grads[0].scalar_type(), mt = model_params[0].scalar_type();
  std::vector<std::array<void*, 4>> ptrs;
  std::vector<int64_t> numels;
  bool vec = true;
  for (size_t i = 0; i < masters.size(); ++i) {
    TORCH_CHECK(masters[i].scalar_type() == at::kFloat, "master weights must be fp32");
    TORCH_CHECK(grads[i].scalar_type() == gt && model_params[i].scalar_type() == mt, "mixed dtypes in SGD list");
    check_dense_pair(masters[i], grads[i]);
    check_dense_pair(masters[i], model_params[i]);
    void* b = nullptr;
    if (mom) {
      TORCH_CHECK(momentum_bufs[i].scalar_type() == at::kFloat, "momentum buffers must be fp32");
      check_dense_pair(masters[i], momentum_bufs[i]);
      b = momentum_bufs[i].data_ptr();
    }
    vec = vec && aligned16(masters[i].data_ptr()) && aligned16(grads[i].data_ptr()) && (!mom || aligned16(b)) &&
          aligned16(model_params[i].data_ptr());
    ptrs.push_back({masters[i].data_ptr(), const_cast<void*>(grads[i].data_ptr()), b, model_params[i].data_ptr()});
    numels.push_back(masters[i].numel());
  }
  const float* gs = scale_ptr(grad_scale);
  TORCH_CHECK(mt == at::kBFloat16 || mt == at::kHalf, "master-weight SGD: model params must be bf16/fp16");
  XDDP_DISPATCH_FLOAT(gt, G, {
    auto go = [&](auto tag) {
      using Mdl = decltype(tag);
      for_each_table<4>(ptrs, numels, [&](const SegTable<4>& t, int32_t nb) {
        auto k = vec ? (mom ? sgd_master_kernel<G, Mdl, true, true> : sgd_master_kernel<G, Mdl, true, false>)
                     : (mom ? sgd_master_kernel<G, Mdl, false, true> : sgd_master_kernel<G, Mdl, false, false>);
        hipLaunchKernelGGL(k, dim3(nb), dim3(kThreads), 0, stream, t, (float)lr, (float)momentum, (float)dampening,
                           (float)weight_decay, nesterov, maximize, first_step, gs);
        XDDP_HIP_CHECK(hipGetLastError());
      });
    };
    if (mt == at::kBFloat16) go(bf16_t{}); else go(f16_t{});
  });
}

void fused_sgd(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
               const std::vector<at::Tensor>& momentum_bufs, double lr, double momentum, double dampening,
               double weight_decay, bool nesterov, bool maximize, bool first_step,
               const c10::optional<at::Tensor>& grad_scale, hipStream_t stream) {
  TORCH_CHECK(params.size() == grads.size(), "params/grads length mismatch");
  const bool mom = momentum != 0.0;
  TORCH_CHECK(!mom || momentum_bufs.size() == params.size(), "momentum buffers missing");
  if (params.empty()) return;
  const auto pt = params[0].scalar_type(), gt = grads[0].scalar_type();
  std::vector<std::array<void*, 3>> ptrs;
  std::vector<int64_t> numels;
  bool vec = true;
  for (size_t i = 0; i < params.size(); ++i) {
    TORCH_CHECK(params[i].scalar_type() == pt && grads[i].scalar_type() == gt, "mixed dtypes in SGD list");
    check_dense_pair(params[i], grads[i]);
    void* b = nullptr;
    if (mom) {
      TORCH_CHECK(momentum_bufs[i].scalar_type() == at::kFloat, "momentum buffers must be fp32");
      check_dense_pair(params[i], momentum_bufs[i]);
      b = momentum_bufs[i].data_ptr();
    }
    ptrs.push_back({params[i].data_ptr(), const_cast<void*>(grads[i].data_ptr()), b});
    numels.push_back(params[i].numel());
    vec = vec && aligned16(params[i].data_ptr()) && aligned16(grads[i].data_ptr()) && (!mom || aligned16(b));
  }
  const float* gs = scale_ptr(grad_scale);
  TORCH_CHECK(pt != at::kDouble && gt != at::kDouble, "fused SGD: fp64 unsupported");
  XDDP_DISPATCH_FLOAT(pt, P, XDDP_DISPATCH_FLOAT(gt, G, {
    for_each_table<3>(ptrs, numels, [&](const SegTable<3>& t, int32_t nb) {
      auto k = vec ? (mom ? sgd_kernel<P, G, true, true> : sgd_kernel<P, G, true, false>)
                   : (mom ? sgd_kernel<P, G, false, true> : sgd_kernel<P, G, false, false>);
      hipLaunchKernelGGL(k, dim3(nb), dim3(kThreads), 0, stream, t, (float)lr, (float)momentum, (float)dampening,
                         (float)weight_decay, nesterov, maximize, first_step, gs);
      XDDP_HIP_CHECK(hipGetLastError());
    });
  }));
}

// ------------------------------------------------------------------------------------
// Fused Adam / AdamW: slots {param, grad, exp_avg, exp_avg_sq, master}
// ------------------------------------------------------------------------------------
template <typename P, typename G, bool VEC, bool MASTER>
__global__ __launch_bounds__(kThreads) void adam_kernel(SegTable<5> t, float lr, float b1, float b2, float eps,
                                                        float wd, float bc1, float bc2_sqrt, bool decoupled,
                                                        bool maximize, const float* gs) {
  const int s = find_seg(t, blockIdx.x);
  const int64_t blk = blockIdx.x - (s ? t.blk_end[s - 1] : 0);
  P* p = reinterpret_cast<P*>(t.ptr[0][s]);
  const G* g = reinterpret_cast<const G*>(t.ptr[1][s]);
  float* m = reinterpret_cast<float*>(t.ptr[2][s]);
  float* v = reinterpret_cast<float*>(t.ptr[3][s]);
  float* mp = reinterpret_cast<float*>(t.ptr[4][s]);
  const int64_t n = t.numel[s];
  const float gscale = (gs ? *gs : 1.f) * (maximize ? -1.f : 1.f);
  const float step_size = lr / bc1;
  const int64_t base = blk * kChunk;
  auto upd = [&](float& pv, float gv, float& mv, float& vv) {
    float gg = gv * gscale;
    if (wd != 0.f) {
      if (decoupled) pv *= (1.f - lr * wd);
      else gg = fmaf(wd, pv, gg);
    }
    mv = fmaf(b1, mv, (1.f - b1) * gg);
    vv = fmaf(b2, vv, (1.f - b2) * gg * gg);
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    pv = pv - step_size * mv / denom;
  };
  if (VEC && base + kChunk <= n) {
    // whole chunk: every iteration's loads first, then the updates and stores. (Interleaved, the
    // stores of iteration it may alias the loads of it + 1 for the compiler, so each iteration's 7
    // loads waited alone: 112 B in flight per thread instead of 448 B.)
    float pv[kIters][8], gv[kIters][8], mv[kIters][8], vv[kIters][8];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
      if (MASTER) Vec8<float>::ld(mp + i, pv[it]); else Vec8<P>::ld(p + i, pv[it]);
      Vec8<G>::ld(g + i, gv[it]);
      Vec8<float>::ld(m + i, mv[it]);
      Vec8<float>::ld(v + i, vv[it]);
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) upd(pv[it][j], gv[it][j], mv[it][j], vv[it][j]);
      Vec8<P>::st(p + i, pv[it]);
      if (MASTER) Vec8<float>::st(mp + i, pv[it]);
      Vec8<float>::st(m + i, mv[it]);
      Vec8<float>::st(v + i, vv[it]);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int64_t i = base + ((int64_t)it * kThreads + threadIdx.x) * 8;
    if (VEC && i + 8 <= n) {
      float pv[8], gv[8], mv[8], vv[8];
      if (MASTER) Vec8<float>::ld(mp + i, pv); else Vec8<P>::ld(p + i, pv);
      Vec8<G>::ld(g + i, gv);
      Vec8<float>::ld(m + i, mv);
      Vec8<float>::ld(v + i, vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) upd(pv[j], gv[j], mv[j], vv[j]);
      Vec8<P>::st(p + i, pv);
      if (MASTER) Vec8<float>::st(mp + i, pv);
      Vec8<float>::st(m + i, mv);
      Vec8<float>::st(v + i, vv);
    } else {
      for (int64_t k = i; k < i + 8 && k < n; ++k) {
        float pv = MASTER ? mp[k] : Elem<P, float>::ld(p, k);
        float gv = Elem<G, float>::ld(g, k), mv = m[k], vv = v[k];
        upd(pv, gv, mv, vv);
        Elem<P, float>::st(p, k, pv);
        if (MASTER) mp[k] = pv;
        m[k] = mv;
        v[k] = vv;
      }
    }
  }
}

void fused_adam(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
                const std::vector<at::Tensor>& exp_avgs, const std::vector<at::Tensor>& exp_avg_sqs,
                const std::vector<at::Tensor>& masters, double lr, double beta1, double beta2, double eps,
                double weight_decay, int64_t step, bool decoupled, bool maximize,
                const c10::optional<at::Tensor>& grad_scale, hipStream_t stream) {
  const size_t N = params.size();
  TORCH_CHECK(grads.size() == N && exp_avgs.size() == N && exp_avg_sqs.size() == N, "adam: list length mismatch");
  const bool has_master = !masters.empty();
  TORCH_CHECK(!has_master || masters.size() == N, "adam: masters length mismatch");
  if (N == 0) return;
  TORCH_CHECK(step >= 1, "adam: step must be >= 1");
  const auto pt = params[0].scalar_type(), gt = grads[0].scalar_type();
  TORCH_CHECK(pt != at::kDouble && gt != at::kDouble, "fused Adam: fp64 unsupported");
  std::vector<std::array<void*, 5>> ptrs;
  std::vector<int64_t> numels;
  bool vec = true;
  for (size_t i = 0; i < N; ++i) {
    TORCH_CHECK(params[i].scalar_type() == pt && grads[i].scalar_type() == gt, "mixed dtypes in Adam list");
    TORCH_CHECK(exp_avgs[i].scalar_type() == at::kFloat && exp_avg_sqs[i].scalar_type() == at::kFloat,
                "Adam states must be fp32");
    check_dense_pair(params[i], grads[i]);
    check_dense_pair(params[i], exp_avgs[i]);
    check_dense_pair(params[i], exp_avg_sqs[i]);
    void* mp = nullptr;
    if (has_master) {
      TORCH_CHECK(masters[i].scalar_type() == at::kFloat, "master weights must be fp32");
      check_dense_pair(params[i], masters[i]);
      mp = masters[i].data_ptr();
    }
    ptrs.push_back({params[i].data_ptr(), const_cast<void*>(grads[i].data_ptr()), exp_avgs[i].data_ptr(),
                    exp_avg_sqs[i].data_ptr(), mp});
    numels.push_back(params[i].numel());
    for (auto* q : ptrs.back()) vec = vec && (q == nullptr || aligned16(q));
  }
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float* gs = scale_ptr(grad_scale);
  XDDP_DISPATCH_FLOAT(pt, P, XDDP_DISPATCH_FLOAT(gt, G, {
    for_each_table<5>(ptrs, numels, [&](const SegTable<5>& t, int32_t nb) {
      auto k = vec ? (has_master ? adam_kernel<P, G, true, true> : adam_kernel<P, G, true, false>)
                   : (has_master ? adam_kernel<P, G, false, true> : adam_kernel<P, G, false, false>);
      hipLaunchKernelGGL(k, dim3(nb), dim3(kThreads), 0, stream, t, (float)lr, (float)beta1, (float)beta2,
                         (float)eps, (float)weight_decay, (float)bc1, (float)std::sqrt(bc2), decoupled, maximize, gs);
      XDDP_HIP_CHECK(hipGetLastError());
    });
  }));
}

}  // namespace kernels
}  // namespace xddp
