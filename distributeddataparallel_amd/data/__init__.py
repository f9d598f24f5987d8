from .datasets import CIFAR10Binary, SyntheticImages  # noqa: F401
from .sampler import DistributedSampler  # noqa: F401
