// Normalization kernels (BatchNorm NHWC with fused residual/ReLU, LayerNorm, RMSNorm) for gfx950.
#pragma once

#include <ATen/ATen.h>
#include <pybind11/pybind11.h>

#include <vector>

namespace xddp {
namespace kernels {

std::vector<at::Tensor> bn_forward(const at::Tensor& x, const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& running_mean,
                                   const c10::optional<at::Tensor>& running_var,
                                   const c10::optional<at::Tensor>& num_batches_tracked, bool training,
                                   double momentum, bool cumulative, double eps,
                                   const c10::optional<at::Tensor>& residual, bool relu, bool save_mask);
std::vector<at::Tensor> bn_backward(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& y,
                                    const c10::optional<at::Tensor>& weight, const at::Tensor& mean,
                                    const at::Tensor& invstd, const c10::optional<at::Tensor>& ss, bool relu,
                                    bool need_dres, bool need_dweight, const c10::optional<at::Tensor>& dy2,
                                    const c10::optional<at::Tensor>& mask_bits, bool coef_only);
// SyncBatchNorm halves: one rank's (count, mean, M2) [3, C]; one rank's backward sums [blocks, C, 2]
at::Tensor bn_moments(const at::Tensor& x);
at::Tensor bn_grad_partials(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& mean);
std::vector<at::Tensor> bn_apply(const at::Tensor& x, const at::Tensor& ss, const c10::optional<at::Tensor>& residual,
                                 bool relu, bool save_mask, const c10::optional<at::Tensor>& num_batches_tracked,
                                 const c10::optional<at::Tensor>& residual_ss,
                                 const c10::optional<at::Tensor>& residual_nbt, const c10::optional<at::Tensor>& out,
                                 const c10::optional<at::Tensor>& out_bits);
// 1x1 conv as an MFMA GEMM with BN prologue (previous BN's apply+ReLU) / epilogue (stats partials)
std::vector<at::Tensor> conv1x1_gemm(const at::Tensor& x, const at::Tensor& w, int64_t stride,
                                     const c10::optional<at::Tensor>& prologue_ss, bool stats,
                                     const c10::optional<at::Tensor>& prologue_y, bool w_t,
                                     const c10::optional<at::Tensor>& epi_add, const c10::optional<at::Tensor>& epi_y,
                                     const c10::optional<at::Tensor>& epi_bits, const c10::optional<at::Tensor>& epi_mean,
                                     const c10::optional<at::Tensor>& epi_ss, int64_t epi_add_stride,
                                     const c10::optional<at::Tensor>& pro_out, const c10::optional<at::Tensor>& pro_bits,
                                     const c10::optional<at::Tensor>& pro_res, const c10::optional<at::Tensor>& pro_res_ss,
                                     const c10::optional<at::Tensor>& pro_nbt, const c10::optional<at::Tensor>& pro_res_nbt);
// BN backward from external (sum g, sum g·(x - mean)) partials [groups, C, 2]: (coef [3, C] with the
// mean folded in, dweight, dbias)
std::vector<at::Tensor> bn_backward_from_partials(const at::Tensor& part, int64_t M,
                                                  const c10::optional<at::Tensor>& weight, const at::Tensor& mean,
                                                  const at::Tensor& invstd, bool need_dweight, bool fold_mean);
// dx = k1·g + k2·(x - mean) + k3 per channel (coef [3, C] unfolded): the BN-backward elementwise
// pass on an already-masked gradient g
bool bn_tail_timeouts(int64_t device);
at::Tensor bn_backward_elem(const at::Tensor& g, const at::Tensor& x, const at::Tensor& mean, const at::Tensor& coef);
// 3x3 pad-1 conv (stride 1/2) as an implicit MFMA GEMM (csrc/kernels/conv3x3.hip)
// Transformer linear layers (gemm.hip): y = a · wᵀ with epilogue 0 none | 1 + bias |
// 2 + bias -> GELU (returns {pre-activation, activation}) | 3 + residual (in place with out) |
// 4 GELU backward: residual = h, returns {(a·wᵀ)·gelu'(h), its column sums}.
std::vector<at::Tensor> gemm_nt(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                                int64_t epi, const c10::optional<at::Tensor>& residual,
                                const c10::optional<at::Tensor>& out);
std::vector<at::Tensor> conv3x3_forward(const at::Tensor& x, const at::Tensor& w, int64_t stride, bool stats);
// the same on the dense GEMM pipeline (gemm.hip; N % 128 == 0, input < 2^31 elements); zeros: a
// 256-B zero line on the device
std::vector<at::Tensor> conv3x3_gemm(const at::Tensor& x, const at::Tensor& w, int64_t stride, bool stats,
                                     const uint16_t* zeros);
// stride-1 3x3 conv on row bands that may span images (conv3x3_band.hip); rows = output rows per
// band (0: the measured choice, conv3x3_band_rows; 0 returned there = shape not covered)
std::vector<at::Tensor> conv3x3_band(const at::Tensor& x, const at::Tensor& w, bool stats, int64_t rows,
                                     const uint16_t* zeros, int64_t cfg = -1);
int conv3x3_band_rows(int64_t W, int64_t H, int64_t bm);
std::vector<at::Tensor> conv3x3_band_forward(const at::Tensor& x, const at::Tensor& w, bool stats, int64_t rows,
                                             int64_t cfg);
at::Tensor conv3x3_rot_weight(const at::Tensor& w);
std::vector<at::Tensor> conv3x3_rot_weights(const std::vector<at::Tensor>& ws);
at::Tensor conv3x3_dgrad_s2(const at::Tensor& dy, const at::Tensor& w_rot, int64_t H, int64_t W);
at::Tensor conv3x3_dgrad_s2_gemm(const at::Tensor& dy, const at::Tensor& wr, int64_t XH, int64_t XW,
                                 const uint16_t* zeros);
// 3x3 weight gradient over 8x8 output patches with a shared X halo (csrc/kernels/conv3x3_wgrad.hip)
at::Tensor conv3x3_wgrad_patch(const at::Tensor& dy, const at::Tensor& x, int64_t stride, const at::Tensor& w_like,
                               int64_t splits = -1);
at::Tensor conv1x1_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t stride, const at::Tensor& w_like,
                         const c10::optional<at::Tensor>& prologue_y, const c10::optional<at::Tensor>& coef);
// stride-1 1x1 input + weight gradient from one staging of dY = k1·g + k2·y2 + k3' (conv_gemm.hip)
bool conv1x1_bwd_fused_supported(int64_t N, int64_t K);
std::vector<at::Tensor> conv1x1_bwd_fused(const at::Tensor& g, const at::Tensor& y2, const at::Tensor& coef,
                                          const at::Tensor& x, const at::Tensor& w);
std::vector<at::Tensor> bn_stats_from_partials(const at::Tensor& part, int64_t M,
                                               const c10::optional<at::Tensor>& weight,
                                               const c10::optional<at::Tensor>& bias,
                                               const c10::optional<at::Tensor>& running_mean,
                                               const c10::optional<at::Tensor>& running_var,
                                               const c10::optional<at::Tensor>& num_batches_tracked, double momentum,
                                               bool cumulative, double eps, bool group_minor);
std::vector<at::Tensor> ln_forward(const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
                                   const c10::optional<at::Tensor>& beta, double eps, bool rms,
                                   const c10::optional<at::Tensor>& add_bias);
std::vector<at::Tensor> ln_backward(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
                                    const c10::optional<at::Tensor>& mean, const at::Tensor& rstd, bool rms,
                                    bool need_dgamma, bool need_dbeta, const c10::optional<at::Tensor>& res);
void colsum_partials(const at::Tensor& part, at::Tensor& out);

std::vector<at::Tensor> maxpool_forward(const at::Tensor& x, int64_t k, int64_t stride, int64_t pad);
at::Tensor global_avg_pool_backward(const at::Tensor& g, const at::Tensor& x_like);
// ResNet stem 7x7/s2 conv (3 -> 64) with BN-statistics partials, and its weight gradient
// (csrc/kernels/stem_conv.hip)
std::vector<at::Tensor> stem_conv_forward(const at::Tensor& x, const at::Tensor& w);
at::Tensor stem_conv_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w_like);
// ResNet stem bn1 -> ReLU -> maxpool(3, 2, 1) without the normalized activation (csrc/kernels/pool.hip)
std::vector<at::Tensor> stem_pool_forward(const at::Tensor& x, const at::Tensor& ss);
at::Tensor stem_pool_bn_backward(const at::Tensor& dy, const c10::optional<at::Tensor>& dy2, const at::Tensor& idx,
                                 const at::Tensor& x, const at::Tensor& ss, const at::Tensor& mean,
                                 const c10::optional<at::Tensor>& coef);
at::Tensor maxpool_backward(const at::Tensor& dy, const at::Tensor& idx, const at::Tensor& x_like, int64_t k,
                            int64_t stride, int64_t pad, const c10::optional<at::Tensor>& dy2);

// transformer elementwise kernels (csrc/kernels/transformer.hip)
at::Tensor rope(const at::Tensor& x, const at::Tensor& cosv, const at::Tensor& sinv, bool backward);
at::Tensor swiglu_forward(const at::Tensor& a, const at::Tensor& b);
std::vector<at::Tensor> swiglu_backward(const at::Tensor& g, const at::Tensor& a, const at::Tensor& b);
at::Tensor gelu_forward(const at::Tensor& h);
at::Tensor transpose16(const at::Tensor& x);
std::vector<at::Tensor> bias_grad(const at::Tensor& g, const c10::optional<at::Tensor>& gelu_input,
                                  const at::Tensor& bias_like);

// flash attention, [B, S, H, D] bf16 (csrc/kernels/flash_attn.hip)
std::vector<at::Tensor> flash_attn_forward(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal,
                                           double scale);
std::vector<at::Tensor> flash_attn_backward(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                                            const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
                                            bool causal, double scale, const c10::optional<at::Tensor>& dq_out,
                                            const c10::optional<at::Tensor>& dk_out,
                                            const c10::optional<at::Tensor>& dv_out,
                                            const c10::optional<at::Tensor>& bias_like);

void bind_norm_kernels(pybind11::module_& m);

// cross_entropy.hip: softmax cross-entropy over bf16 logits [R, V] (fp32 math, no fp32 copy)
std::vector<at::Tensor> cross_entropy_forward(const at::Tensor& logits, const at::Tensor& target, int64_t ignore_index,
                                              const at::Tensor& bad);
at::Tensor cross_entropy_backward(const at::Tensor& logits, const at::Tensor& target, const at::Tensor& lse,
                                  const at::Tensor& gscale, int64_t ignore_index);

}  // namespace kernels
}  // namespace xddp
