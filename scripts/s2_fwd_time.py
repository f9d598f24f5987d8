import os, sys, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from distributeddataparallel_amd._native import load
C = load()
def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3): fn()
    torch.cuda.synchronize(); best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(iters): fn()
        e.record(); torch.cuda.synchronize(); best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best
cl = torch.channels_last
for cin, hw, n in ((128, 56, 128), (256, 28, 256), (512, 14, 512)):
    x = torch.randn(256, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(n, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    t = timed(lambda: C.conv3x3_forward(x, w, 2, True))
    fl = 2.0 * 256 * (hw // 2) ** 2 * n * 9 * cin
    print(json.dumps({"shape": f"s2 C{cin} {hw}x{hw} N{n}", "us": round(t, 1), "tflops": round(fl / t / 1e6, 1)}))
