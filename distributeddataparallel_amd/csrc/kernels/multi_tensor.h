// Host-side API of the multi-tensor HIP kernels (gfx950).
//
// These replace the per-parameter ATen launches of the reference stack's DDP hot path
// (SURVEY.md §2.6 K12 `reducer::mul_out`, K13 `copy_bucket_to_grad`, K14 buffer
// pack/unpack, K15 `_foreach_add_`, K19 NaN check) with one launch per tensor list.
#pragma once

#include <ATen/ATen.h>
#include <c10/util/Optional.h>
#include <hip/hip_runtime.h>

#include <vector>

namespace xddp {
namespace kernels {

// dst[i] = cast(src[i] * scale * (*scale_ptr if given)). src[i]/dst[i] must have equal numel and
// be dense in the same memory order (checked). All srcs share one dtype, all dsts share one.
void mt_scale_copy(const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst, double scale,
                   const c10::optional<at::Tensor>& scale_tensor, hipStream_t stream);

// Pack a list of dense tensors into consecutive slices of `flat` at `offsets` (elements) and back.
// Raw byte copies (dtype-agnostic, bit-exact) of up to any number of (src, dst, nbytes) regions.
void mt_copy_bytes(const std::vector<const void*>& src, const std::vector<void*>& dst,
                   const std::vector<int64_t>& nbytes, hipStream_t stream);
void mt_pack(const std::vector<at::Tensor>& src, const at::Tensor& flat, const std::vector<int64_t>& offsets,
             double scale, hipStream_t stream);
void mt_unpack(const at::Tensor& flat, const std::vector<int64_t>& offsets, const std::vector<at::Tensor>& dst,
               double scale, hipStream_t stream);

// Sum of squares of all elements of all tensors, in fp32, written to out[0] (device scalar).
// If max_norm > 0, out[1] = min(1, max_norm / (sqrt(out[0]) + 1e-6)) (clip coefficient), and
// out[0] holds the total L2 norm. `out` must be a float32 tensor with >= 2 elements.
void mt_l2norm(const std::vector<at::Tensor>& tensors, const at::Tensor& out, double max_norm, hipStream_t stream);

// out[0] (int32) becomes 1 if any element of any tensor is NaN/Inf; 0 otherwise (zeroed here).
void mt_nonfinite(const std::vector<at::Tensor>& tensors, const at::Tensor& out, hipStream_t stream);

// Replica checksum of a list of dense device tensors (any dtypes): float64 [3] = (fp64 sum of the
// values, low / high 32 bits of an XOR of per-element position-mixed raw-bit hashes). Bit-equal
// inputs give bit-equal outputs (fixed-order merge); the DDP replica check compares it across ranks.
at::Tensor mt_checksum(const std::vector<at::Tensor>& tensors, hipStream_t stream);

// Fused SGD over a tensor list (torch.optim.SGD semantics).
void fused_sgd_master(const std::vector<at::Tensor>& masters, const std::vector<at::Tensor>& grads,
                      const std::vector<at::Tensor>& momentum_bufs, const std::vector<at::Tensor>& model_params,
                      double lr, double momentum, double dampening, double weight_decay, bool nesterov, bool maximize,
                      bool first_step, const c10::optional<at::Tensor>& grad_scale, hipStream_t stream);
void fused_sgd(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
               const std::vector<at::Tensor>& momentum_bufs, double lr, double momentum, double dampening,
               double weight_decay, bool nesterov, bool maximize, bool first_step,
               const c10::optional<at::Tensor>& grad_scale, hipStream_t stream);

// Fused Adam/AdamW over a tensor list (torch.optim.AdamW / Adam semantics, no amsgrad).
// If `masters` is non-empty, fp32 master weights are updated and params receive the cast.
void fused_adam(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
                const std::vector<at::Tensor>& exp_avgs, const std::vector<at::Tensor>& exp_avg_sqs,
                const std::vector<at::Tensor>& masters, double lr, double beta1, double beta2, double eps,
                double weight_decay, int64_t step, bool decoupled, bool maximize,
                const c10::optional<at::Tensor>& grad_scale, hipStream_t stream);

}  // namespace kernels
}  // namespace xddp
