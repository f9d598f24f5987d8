"""Short workload for rocprofv3 --pmc passes: the 1x1-conv MFMA GEMM (+BN-stats epilogue) on
three ResNet-50 bs256 shapes, 5 calls each (see profiles/README.md)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
for cin, hw, cout in ((64, 56, 256), (256, 56, 64), (1024, 14, 256)):
    x = torch.randn(256, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
    for _ in range(5):
        C.conv1x1_gemm(x, w, 1, None, True)
torch.cuda.synchronize()
print("pmc workload done")
