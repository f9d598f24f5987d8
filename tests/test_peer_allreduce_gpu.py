"""Peer-memory collectives (csrc/comm/peer_allreduce.hip) across processes that share cuda:0 on
a 1-GPU box (IPC handles opened by the other processes of the same device), IPC handles exchanged
through the process group's store. Oracle: the exact sum / mean / root copy computed locally from
every rank's deterministic input; every rank must also hold bitwise the same result.

Covers: the one-shot lane (all dtypes, broadcast, HIP-graph replay), the two-shot lane (fp32 /
bf16 / fp16, SUM / AVG, ragged sizes, chunking through a small staging buffer, 2 and 4 ranks,
graph replay), back-to-back calls of alternating sizes with no host sync in between (the slot
parity is per call, not per workgroup), and the failure path: a rank that skips a collective
makes its peers raise within XDDP_PEER_TIMEOUT_MS, with a flight dump naming the collective."""
import json
import os

import pytest
import torch

from _dist_utils import run_ranks

pytestmark = pytest.mark.gpu

SUM, AVG = 0, 1
TOL = {torch.float32: 1e-5, torch.bfloat16: 1e-2, torch.float16: 2e-3}


def _input(rank, n, dtype, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    if dtype.is_floating_point:
        return torch.randn(n, generator=g).to(dtype)
    return torch.randint(-1000, 1000, (n,), generator=g).to(dtype)


def _exact(ins, op, world):
    e = sum(x.double() for x in ins)
    return e / world if op == AVG else e


def _check(t, exact, dtype):
    if dtype.is_floating_point:
        torch.testing.assert_close(t.cpu().double(), exact, rtol=TOL[dtype], atol=TOL[dtype])
    else:
        assert torch.equal(t.cpu(), exact.to(dtype)), dtype


def _same_on_all_ranks(t, world):
    from distributeddataparallel_amd import distributed as xdist

    flat = t.detach().cpu().contiguous().view(torch.uint8).view(-1)
    allv = torch.zeros(world * flat.numel(), dtype=torch.uint8)
    xdist.all_gather_into_tensor(allv, flat)
    for r in range(world):
        assert torch.equal(allv[r * flat.numel():(r + 1) * flat.numel()], flat), "ranks disagree bitwise"


def _make(rank, world, two_cap, tag):
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd._native import load

    C = load()
    torch.cuda.set_device(0)
    pg = xdist.get_default_group()
    return C.PeerAllReduce(C.PrefixStore(tag, pg.store), rank, world, 0, 1 << 20, two_cap, 120.0)


def _graph_replay(world, rank, run):
    x = torch.full((1 << 16,), float(rank + 1), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        run(x)  # warm (outside the capture)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=s):
            run(x)
    torch.cuda.synchronize()
    total = float(sum(range(1, world + 1)))
    x.fill_(float(rank + 1))
    for _ in range(3):  # each replay advances the device-side call counters
        graph.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(x.cpu(), torch.full((1 << 16,), total))
        x.div_(total).mul_(rank + 1)


def _w_one_shot(rank, world):
    from distributeddataparallel_amd import distributed as xdist

    peer = _make(rank, world, 0, "peer_one")
    salt = 0
    for dtype in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64):
        for n in (1, 7, 1000, 4096 + 3, (1 << 20) // torch.empty(0, dtype=dtype).element_size()):
            for op in ((SUM, AVG) if dtype.is_floating_point else (SUM,)):
                salt += 1
                ins = [_input(r, n, dtype, salt) for r in range(world)]
                t = ins[rank].cuda()
                assert peer.supports(t, op)
                peer.allreduce(t, op)
                torch.cuda.synchronize()
                _check(t, _exact(ins, op, world), dtype)
                _same_on_all_ranks(t, world)
    # broadcast of raw bytes from either root (odd sizes take the byte path)
    for root in range(world):
        for n in (3, 64, 100001):
            salt += 1
            src = _input(root, n, torch.int32, salt).to(torch.uint8)
            t = (src if rank == root else torch.zeros(n, dtype=torch.uint8)).cuda()
            peer.broadcast(t, root)
            torch.cuda.synchronize()
            assert torch.equal(t.cpu(), src)
    _graph_replay(world, rank, lambda x: peer.allreduce(x, SUM))
    assert peer.status() == 0
    xdist.barrier()
    peer.close()


def _w_two_shot(rank, world):
    from distributeddataparallel_amd import distributed as xdist

    # a 256 KiB staging slot: messages above it are walked in chunks (one launch each)
    peer = _make(rank, world, 256 << 10, "peer_two")
    salt = 0
    for dtype in (torch.float32, torch.bfloat16, torch.float16):
        esz = torch.empty(0, dtype=dtype).element_size()
        for n in (1, 7, 4095, 100003, (256 << 10) // esz, 3 * (256 << 10) // esz + 5):
            for op in (SUM, AVG):
                salt += 1
                ins = [_input(r, n, dtype, salt) for r in range(world)]
                t = ins[rank].cuda()
                assert peer.supports_two_shot(t, op)
                peer.allreduce_two_shot(t, op)
                torch.cuda.synchronize()
                _check(t, _exact(ins, op, world), dtype)
                _same_on_all_ranks(t, world)
    _graph_replay(world, rank, lambda x: peer.allreduce_two_shot(x, SUM))
    assert peer.status() == 0
    xdist.barrier()
    peer.close()


def _w_alternating(rank, world):
    """Many calls of changing sizes on both lanes, enqueued back to back without a host sync: a
    fast rank's next call must never overwrite staging a slower rank is still reading."""
    from distributeddataparallel_amd import distributed as xdist

    peer = _make(rank, world, 256 << 10, "peer_alt")
    sizes = [1 << 10, 40 << 10, 20 << 10, 1 << 20, 600 << 10, (256 << 10) * 3 + 4096, 4 << 10, 1 << 20]
    outs = []
    salt = 7000
    for rep in range(4):
        for k, nb in enumerate(sizes):
            salt += 1
            n = nb // 4
            ins = [_input(r, n, torch.float32, salt) for r in range(world)]
            t = ins[rank].cuda()
            if nb <= (1 << 20) and (k + rep) % 2 == 0:
                peer.allreduce(t, SUM)
            else:
                peer.allreduce_two_shot(t, SUM)
            outs.append((t, _exact(ins, SUM, world)))
            if rank == 1 and k % 3 == 0:  # let the ranks drift apart
                torch.cuda._sleep(200000)
    torch.cuda.synchronize()
    for t, e in outs:
        _check(t, e, torch.float32)
    assert peer.status() == 0
    xdist.barrier()
    peer.close()


def test_peer_one_shot_two_processes_one_gpu():
    run_ranks(_w_one_shot, world=2)


def test_peer_two_shot_two_processes_one_gpu():
    run_ranks(_w_two_shot, world=2)


def test_peer_two_shot_four_processes_one_gpu():
    run_ranks(_w_two_shot, world=4)


def test_peer_alternating_sizes_no_host_sync():
    run_ranks(_w_alternating, world=2)


def _w_peer_backend_timeout(rank, world, prefix):
    """Backend "peer": rank 1 skips one all-reduce; rank 0 must raise (not return stale data)."""
    import time

    from distributeddataparallel_amd import distributed as xdist

    pg = xdist.get_default_group()
    x = torch.ones(1 << 12, device="cuda")
    xdist.all_reduce(x)  # healthy collective first
    torch.cuda.synchronize()
    assert torch.all(x == world)
    if rank == 0:
        t0 = time.monotonic()
        w = xdist.all_reduce(torch.ones(1 << 12, device="cuda"), async_op=True)
        with pytest.raises(RuntimeError, match="error state"):
            w.synchronize()
        assert time.monotonic() - t0 < 30
        for _ in range(100):  # the watchdog has dumped the flight record naming the collective
            if os.path.exists(f"{prefix}0.json"):
                break
            time.sleep(0.05)
        rec = json.load(open(f"{prefix}0.json"))
        assert any(e["op"].startswith("allreduce") and e["state"] == "failed" for e in rec["entries"]), rec
        with pytest.raises(RuntimeError, match="error state"):  # the communicator stays poisoned
            xdist.all_reduce(torch.ones(4, device="cuda"))
        pg.store.set("test/rank0_done", "1")
    else:
        pg.store.wait(["test/rank0_done"], 120.0)  # stay alive (IPC buffers mapped) until rank 0 is done


def test_peer_backend_missing_rank_fails_loudly(tmp_path):
    prefix = str(tmp_path / "flight_rank_")
    run_ranks(_w_peer_backend_timeout, world=2, backend="peer", args=(prefix,),
              env={"XDDP_PEER_TIMEOUT_MS": "2000", "XDDP_FLIGHT_DUMP_PREFIX": prefix})
