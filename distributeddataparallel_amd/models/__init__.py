"""Model zoo: the reference's ResNet-18/CIFAR head plus the BASELINE.json north-star configs."""
from .mlp import MLP  # noqa: F401
from .resnet import (  # noqa: F401
    BasicBlock, Bottleneck, ResNet, SimpleCNN, resnet18, resnet34, resnet50, resnet101, resnet152,
)
