"""Replica check on the GPU (utils/replicas.py + multi_tensor.hip mt_checksum):
the device checksum is bit-stable and bit-sensitive, and bench.py with two ranks sharing one GPU
over the peer-memory backend (device-side one-shot / two-shot all-reduce, calibrated) reports
``replicas_identical: true`` when clean, and exits 3 naming rank 1 when a bucket is corrupted on
rank 1 after its all-reduce (XDDP_FAULT_CORRUPT, inside the Reducer)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_device_checksum_stable_and_bit_sensitive():
    from distributeddataparallel_amd.utils.replicas import checksum

    torch.manual_seed(0)
    ts = [torch.randn(1_000_003, device="cuda").to(torch.bfloat16), torch.randn(4097, device="cuda"),
          torch.arange(5, device="cuda"), torch.randn(3, 3, device="cuda", dtype=torch.float16)]
    c0 = checksum(ts)
    assert c0.dtype == torch.float64 and c0.numel() == 3 and c0.is_cuda
    for _ in range(3):
        assert torch.equal(checksum([t.clone() for t in ts]), c0)
    ref_sum = sum(float(t.double().sum()) for t in ts)
    assert abs(float(c0[0]) - ref_sum) <= 1e-9 * max(1.0, abs(ref_sum)) + 1e-6
    b = [t.clone() for t in ts]
    b[0].view(torch.int16)[123_456] ^= 1  # one bit of one bf16 element
    assert not torch.equal(checksum(b)[1:], c0[1:])
    assert not torch.equal(checksum(ts[::-1])[1:], c0[1:])


def _bench(extra_env):
    env = dict(os.environ, XDDP_NO_AUTOBUILD="1")
    env.pop("XDDP_FAULT_CORRUPT", None)
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "peer",
                           "--model", "simplecnn", "--batch-size", "32", "--image-size", "32", "--steps", "4",
                           "--warmup", "2", "--diag-steps", "0", "--launch-timeout", "200"],
                          capture_output=True, text=True, env=env, timeout=240, cwd=REPO)


@pytest.mark.parametrize("corrupt", [False, True])
def test_bench_peer_backend_replica_check(corrupt):
    r = _bench({"XDDP_FAULT_CORRUPT": "rank=1,iter=4"} if corrupt else {})
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["backend"] == "peer"
    if corrupt:
        assert r.returncode == 3, (r.returncode, r.stderr[-4000:])
        assert out["replicas_identical"] is False and out["replica_mismatch_ranks"] == [1], out
        assert out["replica_max_abs_diff"] > 0
    else:
        assert r.returncode == 0, r.stderr[-4000:]
        assert out["replicas_identical"] is True and out["replica_max_abs_diff"] == 0.0, out
