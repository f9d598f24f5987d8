"""Model zoo: the reference's ResNet-18/CIFAR head plus the BASELINE.json north-star configs."""
from .llama import Llama, LlamaConfig, llama3_8b, llama_tiny  # noqa: F401
from .mlp import MLP  # noqa: F401
from .resnet import (  # noqa: F401
    BasicBlock, Bottleneck, ResNet, SimpleCNN, resnet18, resnet34, resnet50, resnet101, resnet152,
)
from .vit import VisionTransformer, vit_b_16, vit_l_16, vit_tiny  # noqa: F401
