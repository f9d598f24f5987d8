#include <torch/extension.h>

#include "kernels/norm.h"

namespace py = pybind11;

namespace xddp {
namespace kernels {

void bind_norm_kernels(py::module_& m) {
  m.def("bn_forward", &bn_forward, py::arg("x"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("num_batches_tracked"), py::arg("training"), py::arg("momentum"),
        py::arg("cumulative"), py::arg("eps"), py::arg("residual"), py::arg("relu"), py::arg("save_mask") = false);
  m.def("bn_backward", &bn_backward, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("weight"), py::arg("mean"),
        py::arg("invstd"), py::arg("scale_shift"), py::arg("relu"), py::arg("need_dres"), py::arg("need_dweight"),
        py::arg("dy2") = py::none(), py::arg("mask_bits") = py::none(), py::arg("coef_only") = false);
  m.def("bn_apply", &bn_apply, py::arg("x"), py::arg("scale_shift"), py::arg("residual"), py::arg("relu"),
        py::arg("save_mask"), py::arg("num_batches_tracked"), py::arg("residual_ss") = py::none(),
        py::arg("residual_nbt") = py::none(), py::arg("out") = py::none(), py::arg("out_bits") = py::none());
  m.def("conv1x1_gemm", &conv1x1_gemm, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("prologue_ss"),
        py::arg("stats"), py::arg("prologue_y") = py::none(), py::arg("w_t") = false, py::arg("epi_add") = py::none(),
        py::arg("epi_y") = py::none(), py::arg("epi_bits") = py::none(), py::arg("epi_mean") = py::none(),
        py::arg("epi_ss") = py::none(), py::arg("epi_add_stride") = 1, py::arg("pro_out") = py::none(),
        py::arg("pro_bits") = py::none(), py::arg("pro_res") = py::none(), py::arg("pro_res_ss") = py::none(),
        py::arg("pro_nbt") = py::none(), py::arg("pro_res_nbt") = py::none());
  m.def("bn_backward_from_partials", &bn_backward_from_partials, py::arg("partials"), py::arg("M"), py::arg("weight"),
        py::arg("mean"), py::arg("invstd"), py::arg("need_dweight"), py::arg("fold_mean") = true);
  m.def("bn_tail_timeouts", &bn_tail_timeouts, py::arg("device"),
        "whether a folded BN finalize hit its spin bound since the last call (clears the flag; synchronizes)");
  m.def("bn_backward_elem", &bn_backward_elem, py::arg("g"), py::arg("x"), py::arg("mean"), py::arg("coef"));
  m.def("bn_moments", &bn_moments, py::arg("x"));
  m.def("cross_entropy_forward", &cross_entropy_forward, py::arg("logits"), py::arg("target"),
        py::arg("ignore_index"), py::arg("bad"));
  m.def("cross_entropy_backward", &cross_entropy_backward, py::arg("logits"), py::arg("target"), py::arg("lse"),
        py::arg("gscale"), py::arg("ignore_index") = -100);
  m.def("bn_grad_partials", &bn_grad_partials, py::arg("dy"), py::arg("x"), py::arg("mean"));
  m.def("conv3x3_forward", &conv3x3_forward, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("stats"));
  m.def("conv3x3_rot_weight", &conv3x3_rot_weight, py::arg("w"));
  m.def("conv3x3_rot_weights", &conv3x3_rot_weights, py::arg("ws"));
  m.def("conv3x3_band_forward", &conv3x3_band_forward, py::arg("x"), py::arg("w"), py::arg("stats"),
        py::arg("rows") = 0, py::arg("cfg") = -1);
  m.def("conv3x3_dgrad_s2", &conv3x3_dgrad_s2, py::arg("dy"), py::arg("w_rot"), py::arg("H"), py::arg("W"));
  m.def("conv3x3_wgrad_patch", &conv3x3_wgrad_patch, py::arg("dy"), py::arg("x"), py::arg("stride"), py::arg("w_like"),
        py::arg("splits") = -1);
  m.def("conv1x1_bwd_fused_supported", &conv1x1_bwd_fused_supported, py::arg("N"), py::arg("K"));
  m.def("conv1x1_bwd_fused", &conv1x1_bwd_fused, py::arg("g"), py::arg("y2"), py::arg("coef"), py::arg("x"),
        py::arg("w"));
  m.def("conv1x1_wgrad", &conv1x1_wgrad, py::arg("dy"), py::arg("x"), py::arg("stride"), py::arg("w_like"),
        py::arg("prologue_y") = py::none(), py::arg("coef") = py::none());
  m.def("bn_stats_from_partials", &bn_stats_from_partials, py::arg("partials"), py::arg("M"), py::arg("weight"),
        py::arg("bias"), py::arg("running_mean"), py::arg("running_var"), py::arg("num_batches_tracked"),
        py::arg("momentum"), py::arg("cumulative"), py::arg("eps"), py::arg("group_minor") = false);
  m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("w"), py::arg("bias") = py::none(), py::arg("epi") = 0,
        py::arg("residual") = py::none(), py::arg("out") = py::none(),
        "y = a @ w.T (bf16, MFMA LDS-DMA GEMM) with epilogue 0 none | 1 +bias | 2 +bias->GELU | 3 +residual | "
        "4 GELU backward (residual = h): {(a @ w.T) * gelu'(h), column sums} | 5 BatchNorm statistics: "
        "{y, partials [3, N, mtiles] group-minor}");
  m.def("flash_attn_forward", &flash_attn_forward, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"),
        py::arg("scale"));
  m.def("flash_attn_backward", &flash_attn_backward, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"),
        py::arg("o"), py::arg("lse"), py::arg("causal"), py::arg("scale"), py::arg("dq_out") = py::none(),
        py::arg("dk_out") = py::none(), py::arg("dv_out") = py::none(), py::arg("bias_like") = py::none());
  m.def("rope", &rope, py::arg("x"), py::arg("cos"), py::arg("sin"), py::arg("backward") = false);
  m.def("swiglu_forward", &swiglu_forward, py::arg("a"), py::arg("b"));
  m.def("swiglu_backward", &swiglu_backward, py::arg("grad"), py::arg("a"), py::arg("b"));
  m.def("stem_conv_forward", &stem_conv_forward, py::arg("x"), py::arg("w"));
  m.def("stem_conv_wgrad", &stem_conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("w_like"));
  m.def("stem_pool_forward", &stem_pool_forward, py::arg("x"), py::arg("scale_shift"));
  m.def("stem_pool_bn_backward", &stem_pool_bn_backward, py::arg("dy"), py::arg("dy2"), py::arg("idx"), py::arg("x"),
        py::arg("scale_shift"), py::arg("mean"), py::arg("coef") = py::none());
  m.def("maxpool_forward", &maxpool_forward, py::arg("x"), py::arg("kernel"), py::arg("stride"), py::arg("pad"));
  m.def("global_avg_pool_backward", &global_avg_pool_backward, py::arg("g"), py::arg("x_like"));
  m.def("maxpool_backward", &maxpool_backward, py::arg("dy"), py::arg("idx"), py::arg("x_like"), py::arg("kernel"),
        py::arg("stride"), py::arg("pad"), py::arg("dy2") = py::none());
  m.def("ln_forward", &ln_forward, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("rms"),
        py::arg("add_bias") = py::none());
  m.def("ln_backward", &ln_backward, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("rms"), py::arg("need_dgamma"), py::arg("need_dbeta"), py::arg("res") = py::none());
  m.def("gelu_forward", &gelu_forward, py::arg("h"));
  m.def("transpose16", &transpose16, py::arg("x"));
  m.def("bias_grad", &bias_grad, py::arg("grad"), py::arg("gelu_input") = py::none(), py::arg("bias_like"));
}

}  // namespace kernels
}  // namespace xddp
