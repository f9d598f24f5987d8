"""Native TCP store."""
import threading
import time

import pytest

from distributeddataparallel_amd._native import load


def test_tcp_store_basic():
    C = load()
    s = C.TCPStore("127.0.0.1", 0, True, 1, 10.0, False)
    c = C.TCPStore("127.0.0.1", s.port, False, 1, 10.0, False)
    s.set("k", "v")
    assert c.get("k") == b"v"
    assert c.add("n", 3) == 3 and s.add("n", 4) == 7
    assert c.check(["k", "n"]) and not c.check(["missing"])
    assert c.compare_set("k", "v", "w") == b"w"
    assert c.compare_set("k", "zzz", "q") == b"w"
    assert c.compare_set("fresh", "", "x") == b"x"
    c.append("k", "!")
    assert s.get("k") == b"w!"
    assert c.delete_key("k") and not c.check(["k"])
    assert c.num_keys() >= 2


def test_tcp_store_blocking_get_and_timeout():
    C = load()
    s = C.TCPStore("127.0.0.1", 0, True, 1, 10.0, False)
    c = C.TCPStore("127.0.0.1", s.port, False, 1, 10.0, False)
    threading.Timer(0.2, lambda: s.set("late", "1")).start()
    t0 = time.time()
    assert c.get("late") == b"1"
    assert time.time() - t0 >= 0.15
    c.timeout_s = 0.3
    with pytest.raises(TimeoutError):
        c.get("never")
    with pytest.raises(TimeoutError):
        c.wait(["never2"], 0.2)


def test_prefix_and_hash_store():
    C = load()
    h = C.HashStore()
    p = C.PrefixStore("pg0", h)
    p.set("a", "1")
    assert h.get("pg0/a") == b"1"
    assert p.add("cnt", 2) == 2
    q = C.PrefixStore("pg1", h)
    assert not q.check(["a"])


def test_many_clients_concurrent_add():
    C = load()
    s = C.TCPStore("127.0.0.1", 0, True, 1, 10.0, False)
    clients = [C.TCPStore("127.0.0.1", s.port, False, 1, 10.0, False) for _ in range(8)]

    def work(c):
        for _ in range(50):
            c.add("ctr", 1)

    ts = [threading.Thread(target=work, args=(c,)) for c in clients]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert s.add("ctr", 0) == 400


def test_file_store_semantics_and_cleanup(tmp_path):
    C = load()
    path = str(tmp_path / "fs")
    a = C.FileStore(path, 2, 10.0)
    b = C.FileStore(path, 2, 10.0)  # second handle = another process on the shared file
    a.set("k", "v")
    assert b.get("k") == b"v"
    assert a.add("n", 3) == 3 and b.add("n", 4) == 7
    assert b.compare_set("k", "v", "w") == b"w" and a.compare_set("k", "zz", "q") == b"w"
    b.append("k", "!")
    assert a.get("k") == b"w!"
    assert a.delete_key("k") and not b.check(["k"])
    assert a.num_keys() == 1
    threading.Timer(0.2, lambda: a.set("late", "1")).start()
    assert b.get("late") == b"1"
    b.timeout_s = 0.2
    with pytest.raises(TimeoutError):
        b.get("never")
    del a
    import os

    assert os.path.exists(path)
    del b  # last handle removes the file
    assert not os.path.exists(path)


def _file_rdzv_worker(rank, world, path):
    import torch

    from distributeddataparallel_amd import distributed as xdist

    xdist.init_process_group("cpu", init_method=f"file://{path}", rank=rank, world_size=world)
    t = torch.full((4,), float(rank + 1))
    xdist.all_reduce(t)
    assert torch.equal(t, torch.full((4,), float(sum(range(1, world + 1)))))
    xdist.destroy_process_group()


def test_file_rendezvous_multiprocess(tmp_path):
    from distributeddataparallel_amd.utils.spawn import spawn

    spawn(_file_rdzv_worker, args=(3, str(tmp_path / "rdzv")), nprocs=3, env={"OMP_NUM_THREADS": "1"})
