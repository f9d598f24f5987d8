"""One-shot peer-memory all-reduce / broadcast (csrc/comm/peer_allreduce.hip) across two
processes: both ranks share cuda:0 on a 1-GPU box (IPC handles opened by the other process of
the same device), exchanging IPC handles through the process group's store. Oracle: the exact
sum / mean / root copy computed locally from every rank's deterministic input."""
import pytest
import torch

from _dist_utils import run_ranks

pytestmark = pytest.mark.gpu

SUM, AVG = 0, 1


def _input(rank, n, dtype, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    if dtype.is_floating_point:
        return torch.randn(n, generator=g).to(dtype)
    return torch.randint(-1000, 1000, (n,), generator=g).to(dtype)


def _w_peer(rank, world):
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd._native import load

    C = load()
    torch.cuda.set_device(0)
    pg = xdist.get_default_group()
    peer = C.PeerAllReduce(C.PrefixStore("peer_test", pg.store), rank, world, 0, 1 << 20)
    salt = 0
    for dtype in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64):
        for n in (1, 7, 1000, 4096 + 3, (1 << 20) // torch.empty(0, dtype=dtype).element_size()):
            for op in ((SUM, AVG) if dtype.is_floating_point else (SUM,)):
                salt += 1
                ins = [_input(r, n, dtype, salt) for r in range(world)]
                t = ins[rank].cuda()
                assert peer.supports(t, op)
                peer.allreduce(t, op)
                exact = sum(x.double() for x in ins)
                if op == AVG:
                    exact = exact / world
                torch.cuda.synchronize()
                if dtype.is_floating_point:
                    tol = {torch.float32: 1e-6, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dtype]
                    torch.testing.assert_close(t.cpu().double(), exact, rtol=tol, atol=tol)
                else:
                    assert torch.equal(t.cpu(), exact.to(dtype)), (dtype, n)
    # broadcast of raw bytes from either root (odd sizes take the byte path)
    for root in range(world):
        for n in (3, 64, 100001):
            salt += 1
            src = _input(root, n, torch.int32, salt).to(torch.uint8)
            t = (src if rank == root else torch.zeros(n, dtype=torch.uint8)).cuda()
            peer.broadcast(t, root)
            torch.cuda.synchronize()
            assert torch.equal(t.cpu(), src)
    # the same kernel replayed from a HIP graph keeps advancing its generation counter
    x = torch.full((4096,), float(rank + 1), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        peer.allreduce(x, SUM)  # warm (outside the capture)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=s):
            peer.allreduce(x, SUM)
    torch.cuda.synchronize()
    total = float(sum(range(1, world + 1)))
    x.fill_(float(rank + 1))
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        x.div_(total).mul_(rank + 1)  # back to the rank's own value for the next replay
        torch.testing.assert_close(x.cpu(), torch.full((4096,), float(rank + 1)))
    assert peer.status() == 0
    xdist.barrier()
    peer.close()


def test_peer_allreduce_two_processes_one_gpu():
    run_ranks(_w_peer, world=2)
