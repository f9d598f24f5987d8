// Softmax cross-entropy over a large vocabulary (the Llama-3-8B LM head: 4096 rows x 128,256
// classes per step), bf16 logits, fp32 math, without materialising the fp32 logits.
//
// The eager form (F.cross_entropy(logits.float(), t)) writes a 2.1 GB fp32 copy of the logits,
// reads / writes it again for log_softmax, zero-fills an fp32 gradient, runs the log_softmax
// backward over it and casts the result back to bf16: ~4.4 ms per Llama step on MI355X (rocprofv3).
// Here the forward reads the bf16 logits once (one online max / sum-exp pass per row, the
// row's log-sum-exp kept in fp32) and the backward reads them once more and writes the bf16
// gradient (softmax - onehot) · g / count directly: 3 x 1.05 GB of traffic.
//
// One 256-thread block per row, 16-B (8 x bf16) loads; per thread an online (max, sum) pair,
// merged across the block (shuffles, then LDS). Rows whose target is ignore_index contribute 0
// and no gradient. A target outside [0, V) that is not ignore_index is an error, as in torch: the
// row's loss is NaN (the step's loss shows it at once), it gets no gradient, and the kernel sets a
// device-side flag that the Python wrapper turns into an IndexError without a per-step host sync
// (ops/cross_entropy.py). Same math as torch's fp32 cross entropy on the upcast logits (the sums
// in a different order).
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cmath>

#include "common.h"
#include "kernels/dev_utils.h"

namespace xddp {
namespace kernels {

namespace {

constexpr int kXT = 256;

__device__ __forceinline__ void merge(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;  // both empty
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

__global__ __launch_bounds__(kXT) void xent_fwd_kernel(const dev::bf16_t* __restrict__ logits,
                                                       const int64_t* __restrict__ target, float* __restrict__ loss,
                                                       float* __restrict__ lse, int* __restrict__ bad, int64_t V,
                                                       int64_t ignore_index) {
  const int64_t r = blockIdx.x;
  const dev::bf16_t* row = logits + r * V;
  float m = -INFINITY, s = 0.f;
  for (int64_t i = (int64_t)threadIdx.x * 8; i < V; i += (int64_t)kXT * 8) {
    float v[8];
    dev::Vec8<dev::bf16_t>::ld(row + i, v);
    float vm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) vm = fmaxf(vm, v[j]);
    const float M = fmaxf(m, vm);
    float acc = s * __expf(m - M);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(v[j] - M);
    m = M;
    s = acc;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  __shared__ float sm[kXT / 64], ss[kXT / 64];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int w = 1; w < kXT / 64; ++w) merge(M, S, sm[w], ss[w]);
    const float l = M + logf(S);
    lse[r] = l;
    const int64_t t = target[r];
    const bool invalid = t != ignore_index && (t < 0 || t >= V);
    if (invalid) atomicOr(bad, 1);
    loss[r] = t == ignore_index ? 0.f : invalid ? NAN : l - dev::bf16_to_f32(row[t].x);
  }
}

__global__ __launch_bounds__(kXT) void xent_bwd_kernel(const dev::bf16_t* __restrict__ logits,
                                                       const int64_t* __restrict__ target,
                                                       const float* __restrict__ lse, const float* __restrict__ gscale,
                                                       dev::bf16_t* __restrict__ dlogits, int64_t V,
                                                       int64_t ignore_index) {
  const int64_t r = blockIdx.x;
  const dev::bf16_t* row = logits + r * V;
  dev::bf16_t* drow = dlogits + r * V;
  const int64_t t = target[r];
  const bool skip = t == ignore_index || t < 0 || t >= V;
  const float l = lse[r], g = skip ? 0.f : gscale[0];
  for (int64_t i = (int64_t)threadIdx.x * 8; i < V; i += (int64_t)kXT * 8) {
    float v[8], d[8];
    dev::Vec8<dev::bf16_t>::ld(row + i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = (__expf(v[j] - l) - (i + j == t ? 1.f : 0.f)) * g;
    dev::st8_stream(drow + i, d);
  }
}

void check_xent(const at::Tensor& logits, const at::Tensor& target) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.is_contiguous(),
              "cross_entropy: logits must be a contiguous 2-D bf16 CUDA tensor");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.dim() == 1 &&
                  target.size(0) == logits.size(0) && target.is_contiguous(),
              "cross_entropy: target must be int64 [rows] on the logits' device");
  TORCH_CHECK(logits.size(1) % 8 == 0 && (reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16) == 0,
              "cross_entropy: the class count must be a multiple of 8 (16-B rows)");
  TORCH_CHECK(logits.size(0) < (int64_t(1) << 31), "cross_entropy: too many rows");
}

}  // namespace

// -> (loss per row fp32 [R], lse per row fp32 [R]); rows with target == ignore_index give 0,
// rows with a target outside [0, V) give NaN and set bad[0] (int32 on the device, never cleared)
std::vector<at::Tensor> cross_entropy_forward(const at::Tensor& logits, const at::Tensor& target, int64_t ignore_index,
                                              const at::Tensor& bad) {
  check_xent(logits, target);
  TORCH_CHECK(bad.is_cuda() && bad.scalar_type() == at::kInt && bad.numel() >= 1 && bad.device() == logits.device(),
              "cross_entropy: bad-target flag must be an int32 tensor on the logits' device");
  const int64_t R = logits.size(0), V = logits.size(1);
  auto loss = at::empty({R}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({R}, logits.options().dtype(at::kFloat));
  if (R == 0) return {loss, lse};
  auto stream = c10::hip::getCurrentHIPStream(logits.device().index()).stream();
  hipLaunchKernelGGL(xent_fwd_kernel, dim3((unsigned)R), dim3(kXT), 0, stream,
                     reinterpret_cast<const dev::bf16_t*>(logits.data_ptr()), target.data_ptr<int64_t>(),
                     loss.data_ptr<float>(), lse.data_ptr<float>(), bad.data_ptr<int>(), V, ignore_index);
  XDDP_HIP_CHECK(hipGetLastError());
  return {loss, lse};
}

// dlogits (bf16, like logits) = (softmax - onehot(target)) · gscale[0] per non-ignored row
at::Tensor cross_entropy_backward(const at::Tensor& logits, const at::Tensor& target, const at::Tensor& lse,
                                  const at::Tensor& gscale, int64_t ignore_index) {
  check_xent(logits, target);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == logits.size(0) && gscale.scalar_type() == at::kFloat &&
                  gscale.numel() == 1 && gscale.is_cuda(),
              "cross_entropy_backward: lse [rows] and gscale [1] must be fp32 on the device");
  const int64_t R = logits.size(0), V = logits.size(1);
  auto d = at::empty_like(logits);
  if (R == 0) return d;
  auto stream = c10::hip::getCurrentHIPStream(logits.device().index()).stream();
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((unsigned)R), dim3(kXT), 0, stream,
                     reinterpret_cast<const dev::bf16_t*>(logits.data_ptr()), target.data_ptr<int64_t>(),
                     lse.data_ptr<float>(), gscale.data_ptr<float>(), reinterpret_cast<dev::bf16_t*>(d.data_ptr()), V,
                     ignore_index);
  XDDP_HIP_CHECK(hipGetLastError());
  return d;
}

}  // namespace kernels
}  // namespace xddp
