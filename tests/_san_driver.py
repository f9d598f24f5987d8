"""Entry point of one sanitizer run (tests/test_sanitizers_cpu.py): runs the named scenarios of
``_san_scenarios`` with W=2 ranks on the package found at ``$XDDP_PKG_ROOT`` (the instrumented
build), each rank asserting that it loaded that build's extension (``_dist_utils._entry``)."""
import os
import sys

if __name__ == "__main__":
    sys.path.insert(0, os.environ["XDDP_PKG_ROOT"])
    sys.path.insert(1, os.path.dirname(os.path.abspath(__file__)))
    import _dist_utils
    import _san_scenarios as S

    for name in sys.argv[1:]:
        _dist_utils.run_ranks(getattr(S, name), world=2)
        print("ok", name, flush=True)
    print("sanitizer scenarios OK", flush=True)
