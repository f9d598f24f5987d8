"""In-tree native build of ``distributeddataparallel_amd._C`` for gfx950.

No hipify, no ``torch.utils.cpp_extension`` JIT cache: we generate a ninja file that
drives ``hipcc --offload-arch=gfx950`` for the HIP kernels and the host C++ (store,
communicators, Reducer, bindings) and links one shared object next to this file, so
the ``.so`` travels with the repo snapshot to the GPU box.

Usage::

    python -m distributeddataparallel_amd._build          # incremental
    python -m distributeddataparallel_amd._build --clean  # full rebuild
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


def write_ninja(debug: bool = False) -> Path:
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
        f"ldflags = -shared --hip-link --offload-arch={ARCH} {libs}",
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
    objs = []
    for src in hip + cpp:
        rel = src.relative_to(CSRC)
        obj = BUILD_DIR / (str(rel).replace(os.sep, "__") + ".o")
        rule = "hip" if src.suffix == ".hip" else "cxx"
        lines.append(f"build {_ninja_escape(str(obj))}: {rule} {_ninja_escape(str(src))}")
        objs.append(_ninja_escape(str(obj)))
    lines.append(f"build {_ninja_escape(str(OUT_SO))}: link {' '.join(objs)}")
    lines.append(f"default {_ninja_escape(str(OUT_SO))}")
    nf = BUILD_DIR / "build.ninja"
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
    a = ap.parse_args(argv)
    out = build(clean=a.clean, jobs=a.jobs, verbose=a.verbose, debug=a.debug)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
