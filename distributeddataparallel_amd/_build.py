"""In-tree native build of ``distributeddataparallel_amd._C`` for gfx950.

No hipify, no ``torch.utils.cpp_extension`` JIT cache: we generate a ninja file that
drives ``hipcc --offload-arch=gfx950`` for the HIP kernels and the host C++ (store,
communicators, Reducer, bindings) and links one shared object next to this file, so
the ``.so`` travels with the repo snapshot to the GPU box.

Usage::

    python -m distributeddataparallel_amd._build          # incremental
    python -m distributeddataparallel_amd._build --clean  # full rebuild
    python -m distributeddataparallel_amd._build --sanitize address,undefined --out DIR

``--sanitize`` builds the host C++ (store, communicators, Reducer, bindings)
with the given clang sanitizers (``address,undefined`` or ``thread``) into ``build_san_<kind>/``
and links it with the regular build's device objects (the HIP kernels are not instrumented: GPU
sanitizers are not available on this pool) into ``DIR/distributeddataparallel_amd/_C*.so``, next
to a copy of the Python package: a process that puts ``DIR`` first on ``sys.path`` and preloads
the clang sanitizer runtime (:func:`sanitizer_runtime`) runs the package on the instrumented
host code (``tests/test_sanitizers_cpu.py``).
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR / "build"
OUT_SO = PKG_DIR / ("_C" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
ROCM = Path(os.environ.get("ROCM_HOME", "/opt/rocm"))
ARCH = os.environ.get("XDDP_OFFLOAD_ARCH", "gfx950")


def _torch_paths():
    import torch  # noqa: F401  (import only to locate headers/libs)

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return tdir, inc, tdir / "lib", bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def _sources():
    # csrc/tests holds standalone host programs (sanitizer stress drivers), not extension code
    keep = lambda p: "tests" not in p.relative_to(CSRC).parts  # noqa: E731
    hip = sorted(p for p in CSRC.rglob("*.hip") if keep(p))
    cpp = sorted(p for p in CSRC.rglob("*.cpp") if keep(p))
    return hip, cpp


def _ninja_escape(p: str) -> str:
    return p.replace("$", "$$").replace(" ", "$ ").replace(":", "$:")


def sanitizer_runtime(kind: str) -> Path:
    """The clang sanitizer runtime to LD_PRELOAD into an uninstrumented python for ``kind``."""
    name = "tsan" if kind == "thread" else "asan"
    libs = sorted((ROCM / "lib" / "llvm" / "lib" / "clang").glob(f"*/lib/linux/libclang_rt.{name}-x86_64.so"))
    if not libs:
        raise FileNotFoundError(f"no clang {name} runtime under {ROCM}/lib/llvm/lib/clang")
    return libs[-1]


def write_ninja(debug: bool = False, sanitize: str | None = None, out_so: Path | None = None) -> Path:
    tdir, incs, tlib, abi = _torch_paths()
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    inc_flags = " ".join(
        f"-isystem {p}" for p in [*map(str, incs), py_inc, pybind11.get_include(), str(ROCM / "include")]
    ) + f" -I{CSRC}"
    defs = (
        "-D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME=_C "
        "-DTORCH_API_INCLUDE_EXTENSION_H -D__HIP_NO_HALF_OPERATORS__=1 "
        "-D__HIP_NO_HALF_CONVERSIONS__=1 "
        f"-D_GLIBCXX_USE_CXX11_ABI={int(abi)}"
    )
    opt = "-O0 -g" if debug else "-O3"
    if sanitize:
        opt = f"-O1 -g -fno-omit-frame-pointer -fsanitize={sanitize} -shared-libsan"
    common = f"-std=c++17 -fPIC {opt} -Wno-unused-result -Wno-deprecated-declarations {defs} {inc_flags}"
    hipcc = str(ROCM / "bin" / "hipcc")
    hip_flags = f"{common} -x hip --offload-arch={ARCH} -fno-gpu-rdc -munsafe-fp-atomics"
    # host-only translation units: same compiler (clang) but no device pass
    cpp_flags = f"{common} -x c++"
    libs = (
        f"-L{tlib} -Wl,-rpath,{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip "
        f"-ltorch_python -lamdhip64 -lrccl -lroctx64 -lpthread"
    )
    hip, cpp = _sources()
    BUILD_DIR.mkdir(exist_ok=True)
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"hipflags = {hip_flags}",
        f"cppflags = {cpp_flags}",
        f"ldflags = -shared --hip-link --offload-arch={ARCH} {libs}"
        + (f" -fsanitize={sanitize} -shared-libsan" if sanitize else ""),
        "rule hip",
        "  command = $hipcc -MMD -MF $out.d $hipflags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule cxx",
        "  command = $hipcc -MMD -MF $out.d $cppflags -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $hipcc $in $ldflags -o $out",
        "  description = LINK $out",
    ]
    bdir = _san_dir(sanitize) if sanitize else BUILD_DIR
    out_so = out_so or OUT_SO
    objs = []
    for src in hip + cpp:
        rel = src.relative_to(CSRC)
        name = str(rel).replace(os.sep, "__") + ".o"
        if sanitize and src.suffix == ".hip":  # the regular build's device objects, uninstrumented
            objs.append(_ninja_escape(str(BUILD_DIR / name)))
            continue
        obj = bdir / name
        rule = "hip" if src.suffix == ".hip" else "cxx"
        lines.append(f"build {_ninja_escape(str(obj))}: {rule} {_ninja_escape(str(src))}")
        objs.append(_ninja_escape(str(obj)))
    lines.append(f"build {_ninja_escape(str(out_so))}: link {' '.join(objs)}")
    lines.append(f"default {_ninja_escape(str(out_so))}")
    bdir.mkdir(exist_ok=True)
    nf = bdir / "build.ninja"
    content = "\n".join(lines) + "\n"
    if not nf.exists() or nf.read_text() != content:
        nf.write_text(content)
    return nf


def _ninja_bin() -> str:
    exe = shutil.which("ninja")
    if exe:
        return exe
    import ninja  # pip wheel ships the binary

    return str(Path(ninja.BIN_DIR) / "ninja")


def _san_dir(kind: str) -> Path:
    return PKG_DIR / ("build_san_" + kind.replace(",", "_"))


def build_sanitized(kind: str, out_dir: Path, jobs: int | None = None) -> Path:
    """Host code under ``kind`` sanitizers + the regular device objects -> a package copy in
    ``out_dir`` (module docstring). Builds the regular objects first if needed."""
    build(jobs=jobs)
    pkg = Path(out_dir) / PKG_DIR.name
    if pkg.exists():
        shutil.rmtree(pkg)
    shutil.copytree(PKG_DIR, pkg, ignore=shutil.ignore_patterns("build*", "_C*.so", "__pycache__", "csrc"))
    so = pkg / OUT_SO.name
    nf = write_ninja(sanitize=kind, out_so=so)
    jobs = jobs or min(16, os.cpu_count() or 4)
    subprocess.run([_ninja_bin(), "-f", str(nf), "-j", str(jobs)], check=True, cwd=str(nf.parent))
    return so


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False, debug: bool = False) -> Path:
    if clean and BUILD_DIR.exists():
        shutil.rmtree(BUILD_DIR)
    nf = write_ninja(debug=debug)
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = [_ninja_bin(), "-f", str(nf), "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True, cwd=str(BUILD_DIR))
    return OUT_SO


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", default=None, help="address,undefined | thread (host code only)")
    ap.add_argument("--out", default=None, help="with --sanitize: directory for the package copy")
    a = ap.parse_args(argv)
    if a.sanitize:
        out = build_sanitized(a.sanitize, Path(a.out or f"/tmp/xddp_san_{a.sanitize.replace(',', '_')}"), a.jobs)
    else:
        out = build(clean=a.clean, jobs=a.jobs, verbose=a.verbose, debug=a.debug)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
