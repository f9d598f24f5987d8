"""Hand-written HIP ops (gfx950) with autograd: fused BatchNorm(+add+ReLU), 1x1-conv MFMA GEMM with
BatchNorm statistics in its epilogue, LayerNorm, RMSNorm, NHWC max-pool."""
from .batch_norm import FusedBatchNorm2d, batch_norm_act  # noqa: F401
from .layer_norm import FusedLayerNorm, FusedRMSNorm, layer_norm, rms_norm  # noqa: F401
from .pool import FusedMaxPool2d  # noqa: F401
from .conv_bn import conv1x1_bn_act, conv3x3_bn_relu  # noqa: F401
