from .fused import FusedAdam, FusedAdamW, FusedSGD, clip_grad_norm_, grad_norm  # noqa: F401
