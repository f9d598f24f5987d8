"""2-layer MLP for MNIST-shaped data (BASELINE.json config 1: DDP plumbing on the CPU backend)."""
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self, in_features: int = 784, hidden: int = 256, num_classes: int = 10):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden)
        self.act = nn.ReLU()
        self.fc2 = nn.Linear(hidden, num_classes)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x.flatten(1))))
