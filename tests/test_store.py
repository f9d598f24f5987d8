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
