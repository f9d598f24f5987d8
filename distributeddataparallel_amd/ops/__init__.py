"""Hand-written HIP ops (gfx950) with autograd: fused BatchNorm(+add+ReLU), LayerNorm, RMSNorm."""
from .batch_norm import FusedBatchNorm2d, batch_norm_act  # noqa: F401
from .layer_norm import FusedLayerNorm, FusedRMSNorm, layer_norm, rms_norm  # noqa: F401
from .pool import FusedMaxPool2d  # noqa: F401
